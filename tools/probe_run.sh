#!/bin/bash
# A/B timing of the fused sweep: stream-removed builds and launch configs
set -e
b() { timeout -k 10 120 python bench.py --no-cpu-baseline --vcycles 2 "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel'], d['roofline']['kernel_ms_mean'], d['ms_per_vcycle'])"; }
echo base; b
echo NO_B; MAD_HIP_LIB=tools/build_probe/libmad_hip_NO_B.so b
echo NO_U; MAD_HIP_LIB=tools/build_probe/libmad_hip_NO_U.so b
echo t1_512; MAD_FUSED_BLOCKS=512 b
echo t1_768; MAD_FUSED_BLOCKS=768 b
echo t2_512; MAD_FUSED_TILE=2 MAD_FUSED_BLOCKS=512 b
echo t3_512; MAD_FUSED_TILE=3 MAD_FUSED_BLOCKS=512 b
echo t0_1024; MAD_FUSED_TILE=0 MAD_FUSED_BLOCKS=1024 b
export TMPDIR=/tmp
for v in NO_B NO_U; do
  MAD_HIP_LIB=tools/build_probe/libmad_hip_$v.so timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/probe_$v -o pmc -- python3 tools/profile_traffic.py > gpurun_out/probe_$v.log 2>&1
done
MAD_FUSED_BLOCKS=512 timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/probe_t1_512 -o pmc -- python3 tools/profile_traffic.py > gpurun_out/probe_t1_512.log 2>&1
echo done
