#!/bin/bash
# A/B of library builds on the VED bench (tensor device ms, one GPU), alternating:
#   tools/ab_ved.sh lib.so ...
set -e
b() { timeout -k 10 200 python tools/bench_ved.py --reps 2 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tensor_ms', d['tensor_device_ms'], 'diffusion_ms', d['diffusion_device_ms'])"; }
for r in 1 2; do
  echo "base"; b
  for lib in "$@"; do echo "$lib"; MAD_HIP_LIB=$lib b; done
done
