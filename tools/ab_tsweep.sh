#!/bin/bash
# gs_tsweep_k kernel time (bench, gs_kernel 7) of the default build and of probe builds:
#   tools/ab_tsweep.sh tools/pglibs/libmad_hip_X.so ...
b() { timeout -k 10 150 python bench.py --no-cpu-baseline --gs-kernel 7 --vcycles 2 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel'], d['roofline']['kernel_ms_mean'])"; }
echo "base"; b
for lib in "$@"; do echo "$lib"; MAD_HIP_LIB=$lib b; done
