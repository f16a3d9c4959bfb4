#!/bin/bash
# rank-slab sweep proxy (boundary + interior launches, no exchange) over tuning knobs:
#   tools/sweep_slab.sh NZ...
set -e
for nz in "${@:-64 128}"; do
for cfg in "8 256 1 256" "4 256 1 256" "8 384 1 256" "8 512 1 256" "4 512 1 256" "8 512 0 512" "8 1024 0 512" "4 1024 0 1024"; do
  set -- $cfg
  MAD_SPLIT_PROXY=1 MAD_BOUNDARY_PLANES=$1 MAD_INTERIOR_BLOCKS=$2 MAD_FUSED_TILE=$3 MAD_FUSED_BLOCKS=$4 \
    timeout -k 10 120 python tools/bench_slab.py $nz | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('nz=$nz bp=$1 iblocks=$2 tile=$3 blocks=$4 ms=%.4f gvox=%.1f' % (d['ms_per_sweep'], d['gvox_s']))"
done
done
