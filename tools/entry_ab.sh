# graph entry without an eager level-0 exchange: parity tests, then RCCL-SOLO / SOLO 8-rank timings
set -o pipefail
run() { timeout -k 10 200 python -u tools/bench_local_split.py "$@"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread && \
for r in 1 2; do
  echo "== rccl-solo" && run --rccl --solo 2 8 && \
  echo "== solo" && run --solo 8 || exit 1
done
