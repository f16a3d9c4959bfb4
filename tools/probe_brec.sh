#!/bin/bash
# record-carried rhs (level 0) on / off: smoother bench, V-cycles and the VED filter
set -e
for rep in 1 2; do
for v in 1 0; do
  echo "MAD_BREC=$v bench: $(MAD_BREC=$v timeout -k 10 120 python bench.py --no-cpu-baseline --vcycles 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms_mean'], d['ms_per_vcycle'])")"
  echo "MAD_BREC=$v ved: $(MAD_BREC=$v timeout -k 10 200 python tools/bench_ved.py | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['diffusion_device_ms'], d['ved_wall_ms_incl_pcie'], d['cycles'])")"
done
done
