# two (and four) RCCL ranks sharing one GPU: V-cycle forms (tools/rehearse_vcycles.py) and the bench's N = 2 launch
set -o pipefail
tr() { port=$1; shift; echo "== $*"; timeout -k 10 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/rehearse_vcycles.py "$@" 2>&1 | grep -E "^\[rank|WARN|Error"; echo "rc=$?"; }
tr 29621 --sync
tr 29622
tr 29624 --options 4
echo "== bench rehearsal rccl"
MAD_BENCH_SHARED_GPU=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29625 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-precision-cycles --halo rccl 2>&1 | grep -E "bench rank|metric|WARN|Error"; echo "rc=$?"
echo "== bench rehearsal auto (the default: peer after the in-run bitwise check)"
MAD_BENCH_SHARED_GPU=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29626 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-precision-cycles 2>&1 | grep -E "bench rank|metric|WARN|Error"; echo "rc=$?"
echo "== bench rehearsal auto, 4 ranks"
MAD_BENCH_SHARED_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29627 bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline --no-precision-cycles 2>&1 | grep -E "bench rank 0|metric|WARN|Error"; echo "rc=$?"
echo "== bench rehearsal auto, 8 ranks (the driver's N = 8 launch, all ranks on the one GPU)"
MAD_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29628 bench.py --gpus 8 --steps 10 --warmup 3 --no-cpu-baseline --no-precision-cycles 2>&1 | grep -E "bench rank 0|metric|WARN|Error"; echo "rc=$?"
