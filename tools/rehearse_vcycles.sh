set -o pipefail
tr() { port=$1; shift; echo "== $*"; timeout -k 10 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/rehearse_vcycles.py "$@" 2>&1 | grep -E "^\[rank|WARN|Error" ; echo "rc=$?"; }
tr 29621 --sync
tr 29622
tr 29623 --eager
tr 29624 --options 4
tr 29625 --size 256
