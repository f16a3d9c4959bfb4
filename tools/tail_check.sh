# V-cycle tail + LDS-staged dense b in the fused sweep: parity tests, then V-cycle timings on one GPU
# and the SOLO 8-rank proxy, alternated: default (tail 32^3, b via LDS), no tail, tail 16^3, tail 64^3,
# b read from global memory
set -o pipefail
run() { timeout -k 10 200 python -u tools/bench_local_split.py "$@"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_vtail.py tests/test_gpu_kernels.py tests/test_gpu_filter.py tests/test_gpu_coarse.py -m gpu -x -q --timeout 300 --timeout-method thread && \
for r in 1 2; do
  echo "== default" && run --solo 1 8 && \
  echo "== no tail" && run --options 8 --solo 1 8 && \
  echo "== tail 16^3" && MAD_HIP_LIB=tools/pglibs/libmad_tail4096.so run --solo 1 8 && \
  echo "== tail 64^3" && MAD_HIP_LIB=tools/pglibs/libmad_tail262144.so run --solo 1 8 && \
  echo "== b from global" && MAD_HIP_LIB=tools/pglibs/libmad_nobl.so run --solo 1 8 || exit 1
done
