# dense b through LDS (BL, default) vs from global memory (MAD_FUSED_B_LDS=0 probe): V-cycle time at
# 512^3 on one GPU and one rank of 8 (SOLO), alternated; then a kernel trace of each
set -o pipefail
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u tools/bench_local_split.py "$@"; }
for r in 1 2 3; do
  echo "== BL" && run --solo 1 8 && \
  echo "== b from global" && MAD_HIP_LIB=tools/pglibs/libmad_nobl.so run --solo 1 8 || exit 1
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bl -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_local_split.py --solo 1 && \
MAD_HIP_LIB=$GRAFT_REPO_ROOT/tools/pglibs/libmad_nobl.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_nobl -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_local_split.py --solo 1
