#!/bin/bash
# V-cycle time at 512^3: one-pass residual + restriction with 1024-thread blocks (one
# per CU) vs 512-thread blocks (two per CU, barriers of one block overlap the other's
# loads), at two block-count targets
set -e
for rep in 1 2; do
  for nt in 1024 512; do
    for nb in 512 1024; do
      out=$(MAD_RR_NT=$nt MAD_RR_BLOCKS=$nb timeout -k 10 90 python bench.py --steps 5 --warmup 2 --vcycles 30 --no-cpu-baseline)
      echo "MAD_RR_NT=$nt blocks=$nb $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_vcycle"], d["vcycles_per_s"])')"
    done
  done
done
