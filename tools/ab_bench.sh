#!/bin/bash
# A/B of library builds on the whole bench line (V-cycle, refine / fp64 cycle costs, sweep), alternated:
#   tools/ab_bench.sh REPS LIB ...   ("base" = the in-tree libmad_hip.so)
set -o pipefail
R=$1; shift
b() { timeout -k 10 200 python bench.py --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'sweep_ms': d['roofline']['kernel_ms_mean'], 'ms_per_vcycle': d['device_ms_per_vcycle'], 'vcycles_per_s': d['vcycles_per_s'], 'run_ms_per_cycle': d.get('run_ms_per_cycle')}))"; }
for r in $(seq "$R"); do
  for lib in "$@"; do
    echo -n "$lib "
    if [ "$lib" = base ]; then b || exit 1; else MAD_HIP_LIB=$lib b || exit 1; fi
  done
done
