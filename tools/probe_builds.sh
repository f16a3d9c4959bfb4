#!/bin/bash
# Measurement-only builds of libmad_hip.so with one input stream of the fused sweep
# removed (results are wrong by design), to price each stream:  tools/probe_builds.sh
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/build_probe
for v in NO_B NO_U; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMAD_PROBE_$v \
    -o tools/build_probe/libmad_hip_$v.so multigridanisotropicdiffusion_amd/csrc/mad_solver.hip \
    -lrccl -lrocsolver -lrocblas 2>&1 | grep -v warning || true
done
ls -la tools/build_probe
