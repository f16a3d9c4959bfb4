#!/bin/bash
set -e
export TMPDIR=/tmp
for nb in 1024 4096 16384; do
  MAD_XFER_BLOCKS=$nb timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/xf_$nb -o x -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/xf_$nb.log 2>&1
  grep -h vcycles gpurun_out/xf_$nb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($nb, d['ms_per_vcycle'])"
done
