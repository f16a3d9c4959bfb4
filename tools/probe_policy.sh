#!/bin/bash
# cache-policy A/B of the level-0 sweep (tools/probe_builds.sh REC_NT U_NT ST_NT first)
set -e
b() { timeout -k 10 120 python bench.py --no-cpu-baseline --vcycles 2 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms_mean'], d['ms_per_vcycle'])"; }
for rep in 1 2; do
  echo "base $(b)"
  for v in REC_NT U_NT ST_NT; do echo "$v $(MAD_HIP_LIB=tools/build_probe/libmad_hip_$v.so b)"; done
done
