#!/bin/bash
# Measurement builds of gs_tsweep_k with parts of the loop removed (results wrong, timings
# only): tools/probe_tsweep.sh builds tools/pglibs/libmad_hip_<probe>.so for every probe macro
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/pglibs
build() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function \
    -D$1 -o tools/pglibs/libmad_hip_$2.so multigridanisotropicdiffusion_amd/csrc/mad_solver.hip \
    -lrccl -lrocsolver -lrocblas
}
build TSW_PROBE_NO_TLOAD notload &
build TSW_PROBE_NO_WAIT nowait &
build TSW_PROBE_NO_STAGE nostage &
build TSW_PROBE_NO_FORM noform &
build TSW_PROBE_NO_ULOAD noulooad &
wait
ls -la tools/pglibs
