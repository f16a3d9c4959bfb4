#!/bin/bash
# Measurement-only builds of gs_fusedg_k with one part removed (results wrong by design):
#   NO_STORE  output stores     NO_T   tensor / b stream     NO_STAGE  stage reads + arithmetic
#   NO_X      exchange-plane reads (in-plane differences from the thread's own block)
#   tools/probe_fusedg.sh [variants]   -> tools/pglibs/libmad_hip_PG_<v>.so (travels to the GPU box)
cd "$(dirname "$0")/.."
mkdir -p tools/pglibs
for v in ${@:-NO_STORE NO_T NO_STAGE NO_X}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMAD_PG_$v \
    -o tools/pglibs/libmad_hip_PG_$v.so multigridanisotropicdiffusion_amd/csrc/mad_solver.hip \
    -lrccl -lrocsolver -lrocblas > tools/pglibs/PG_$v.log 2>&1 &
done
wait
grep -l error tools/pglibs/PG_*.log || true
ls -la tools/pglibs/*.so
