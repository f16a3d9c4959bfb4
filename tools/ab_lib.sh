#!/bin/bash
# A/B of alternative library builds on the bench (kernel mean ms of the level-0 sweep,
# ms per V-cycle), alternating builds: tools/ab_lib.sh tools/build_probe/libmad_hip_X.so ...
set -e
b() { timeout -k 10 150 python bench.py --no-cpu-baseline --vcycles 20 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel'], d['roofline']['kernel_ms_mean'], d['ms_per_vcycle'])"; }
for r in 1 2; do
  echo "base"; b
  for lib in "$@"; do echo "$lib"; MAD_HIP_LIB=$lib b; done
done
