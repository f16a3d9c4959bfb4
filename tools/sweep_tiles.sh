#!/bin/bash
# fused-sweep tile / grid A/B on the bench workload (levels 0-2 per-sweep times + V-cycle)
set -e
for cfg in "1 256" "1 512" "0 512" "0 1024" "2 256" "2 512" "3 512" "1 256"; do
  set -- $cfg
  MAD_FUSED_TILE=$1 MAD_FUSED_BLOCKS=$2 timeout -k 10 120 python tools/bench_levels.py --gs-kernel 3 | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('tile=$1 blocks=$2', ' '.join('L%d %.4f' % (L['level'], L['ms_per_sweep']) for L in d['levels'][:3]), 'vc %.3f' % d['ms_per_vcycle'])"
done
