#!/bin/bash
set -e
b() { timeout -k 10 120 python bench.py --no-cpu-baseline --vcycles 2 "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms_mean'], d['ms_per_vcycle'])"; }
for v in base REC_NT U_NT ST_NT base; do
  echo -n "$v "
  if [ $v = base ]; then b; else MAD_HIP_LIB=tools/build_probe/libmad_hip_$v.so b; fi
done
