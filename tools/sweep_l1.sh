#!/bin/bash
# fused-sweep launch shape at 256^3 (= level 1 of the 512^3 hierarchy): tile x target blocks
set -e
for t in 1 0 3; do
  for b in 128 256 512 1024; do
    out=$(MAD_FUSED_TILE=$t MAD_FUSED_BLOCKS=$b timeout -k 10 60 python bench.py --size 256 --steps 30 --warmup 3 --vcycles 2 --no-cpu-baseline)
    echo "tile=$t blocks=$b $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_ms_median"], r["kernel"])')"
  done
done
