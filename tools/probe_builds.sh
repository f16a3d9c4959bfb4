#!/bin/bash
# Measurement-only builds of libmad_hip.so (A/B of the fused sweep):
#   NO_B / NO_U   one input stream removed (results wrong by design), to price it
#   REC_NT etc.   cache-policy variants of the streams
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/build_probe
bld() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $2 \
    -o tools/build_probe/libmad_hip_$1.so multigridanisotropicdiffusion_amd/csrc/mad_solver.hip \
    -lrccl -lrocsolver -lrocblas 2>&1 | grep -v warning || true
}
for v in ${@:-NO_B NO_U REC_NT U_NT ST_NT}; do
  case $v in
    NO_B) bld $v -DMAD_PROBE_NO_B ;;
    NO_U) bld $v -DMAD_PROBE_NO_U ;;
    REC_NT) bld $v -DMAD_REC_AUX=2 ;;
    U_NT) bld $v -DMAD_U_AUX=2 ;;
    ST_NT) bld $v -DMAD_ST_AUX=2 ;;
  esac
done
ls tools/build_probe
