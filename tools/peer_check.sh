# peer halo: parity tests (LOCAL / SOLO / RCCL-SOLO / two RCCL processes on one GPU, C4 slabs),
# the bench's N = 2 torchrun launch rehearsed on one GPU (both halo modes), then the SOLO /
# RCCL-SOLO per-rank timings with and without it, and a kernel trace of the RCCL-SOLO 8-rank
# cycle with it (no RCCL kernel in the level-0 sweeps)
set -o pipefail
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u tools/bench_local_split.py "$@"; }
tr() { MAD_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $1 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-precision-cycles --halo $2; }
MAD_MP_KEEP_LOGS=gpurun_out/mp_logs timeout -k 10 900 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_distributed.py tests/test_gpu_distributed_full.py -m gpu -x -v --timeout 400 --timeout-method thread && \
echo "== bench rehearsal peer" && tr 29611 peer && \
echo "== bench rehearsal rccl" && tr 29612 rccl && \
echo "== solo default" && run --solo 1 2 4 8 && \
echo "== solo peer" && run --options 4 --solo 2 4 8 && \
echo "== rccl-solo default" && run --rccl --solo 2 4 8 && \
echo "== rccl-solo peer" && run --rccl --options 4 --solo 2 4 8 && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_peer -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_local_split.py --rccl --options 4 --solo 8
