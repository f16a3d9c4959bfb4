#!/bin/bash
# V-cycle time at 512^3 with the one-pass residual + restriction (default) and without
set -e
for v in 1 0 1 0; do
  out=$(MAD_FUSED_RR=$v timeout -k 10 90 python bench.py --steps 5 --warmup 2 --vcycles 30 --no-cpu-baseline)
  echo "MAD_FUSED_RR=$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_vcycle"], d["vcycles_per_s"])')"
done
