set -e
for cfg in "0 2 2048" "0 3 2048" "1 2 2048" "1 2 1024" "2 2 2048" "2 2 1024" "3 2 2048" "3 2 1024"; do
  set -- $cfg
  echo "cfg tile=$1 lead=$2 blocks=$3"
  MAD_FUSED_TILE=$1 MAD_FUSED_LEAD=$2 MAD_FUSED_BLOCKS=$3 timeout -k 10 120 python bench.py --gs-kernel 3 --no-cpu-baseline --vcycles 2 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms_mean'], d['vcycles_per_s'])"
done
