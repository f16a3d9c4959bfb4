#!/bin/bash
set -e
b() { timeout -k 10 120 python bench.py --no-cpu-baseline --vcycles 2 "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel'], d['roofline']['kernel_ms_mean'], d['ms_per_vcycle'])"; }
for sh in 0 4; do for bl in 256 512; do echo "shift=$sh blocks=$bl"; MAD_X_SHIFT=$sh MAD_FUSED_BLOCKS=$bl b; done; done
echo "t2 shift4 512"; MAD_X_SHIFT=4 MAD_FUSED_TILE=2 MAD_FUSED_BLOCKS=512 b
echo "t2 shift4 256"; MAD_X_SHIFT=4 MAD_FUSED_TILE=2 MAD_FUSED_BLOCKS=256 b
export TMPDIR=/tmp
MAD_X_SHIFT=4 timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/probe_s4 -o pmc -- python3 tools/profile_traffic.py > gpurun_out/probe_s4.log 2>&1
MAD_X_SHIFT=4 timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/probe_s4w -o pmc -- python3 tools/profile_traffic.py > gpurun_out/probe_s4w.log 2>&1
echo done
