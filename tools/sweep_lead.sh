#!/bin/bash
# level-0 fused sweep: prefetch lead (stages) A/B, 3 runs each, interleaved
set -e
for rep in 1 2 3; do
for lead in 2 3 4; do
  MAD_FUSED_LEAD=$lead timeout -k 10 120 python bench.py --no-cpu-baseline --vcycles 3 --steps 30 | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('lead=$lead', d['value'], d['roofline']['kernel_ms_mean'], d['roofline']['kernel'], d['vcycles_per_s'])"
done
done
