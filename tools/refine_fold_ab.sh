# folded defect-correction update: refine tests vs the oracle, bitwise equality of a whole mad_run with
# the pre-fold build, then the bench's per-cycle costs alternated
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_refine.py -m gpu -x -q --timeout 300 --timeout-method thread && \
timeout -k 10 120 python -u tools/refine_fold_ab.py /tmp/fold_new.npy && \
MAD_HIP_LIB=tools/pglibs/libmad_prefold.so timeout -k 10 120 python -u tools/refine_fold_ab.py /tmp/fold_old.npy && \
python -c "import numpy as np; a=np.load('/tmp/fold_new.npy'); b=np.load('/tmp/fold_old.npy'); print('bitwise equal:', np.array_equal(a, b), 'max diff', float(np.abs(a-b).max()))" && \
for r in 1 2 3; do
  echo "== fold" && timeout -k 10 150 python bench.py --no-cpu-baseline --vcycles 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['run_ms_per_cycle'])" && \
  echo "== pre-fold" && MAD_HIP_LIB=tools/pglibs/libmad_prefold.so timeout -k 10 150 python bench.py --no-cpu-baseline --vcycles 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['run_ms_per_cycle'])" || exit 1
done
