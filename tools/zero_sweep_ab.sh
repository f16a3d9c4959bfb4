# zero-iterate first sweep of the refine correction cycle (gs_fused3_k ZU, no x = 0 fill): refine tests
# vs the oracle, bitwise equality of a whole mad_run with a -DMAD_NO_ZERO_SWEEP build
# (tools/pglibs/libmad_nozero.so), then the bench's per-cycle costs alternated.  Build that library first, here:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMAD_NO_ZERO_SWEEP -o tools/pglibs/libmad_nozero.so \
#     multigridanisotropicdiffusion_amd/csrc/mad_solver.hip -lrccl -lrocsolver -lrocblas
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_refine.py -m gpu -x -q --timeout 300 --timeout-method thread && \
timeout -k 10 120 python -u tools/refine_fold_ab.py /tmp/zu_new.npy && \
MAD_HIP_LIB=tools/pglibs/libmad_nozero.so timeout -k 10 120 python -u tools/refine_fold_ab.py /tmp/zu_old.npy && \
timeout -k 10 200 python -u tools/refine_fold_ab.py /tmp/zu_new512.npy 512 && \
MAD_HIP_LIB=tools/pglibs/libmad_nozero.so timeout -k 10 200 python -u tools/refine_fold_ab.py /tmp/zu_old512.npy 512 && \
python -c "import numpy as np
for s in ('', '512'):
    a=np.load(f'/tmp/zu_new{s}.npy'); b=np.load(f'/tmp/zu_old{s}.npy'); print(s or '256', 'bitwise equal:', np.array_equal(a, b), 'max diff', float(np.abs(a-b).max()))" && \
for r in 1 2 3; do
  echo "== zero sweep" && timeout -k 10 150 python bench.py --no-cpu-baseline --vcycles 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['run_ms_per_cycle'])" && \
  echo "== fill + load" && MAD_HIP_LIB=tools/pglibs/libmad_nozero.so timeout -k 10 150 python bench.py --no-cpu-baseline --vcycles 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['run_ms_per_cycle'])" || exit 1
done
