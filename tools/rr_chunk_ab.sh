# small-level descent chunking: kernel traces of one-GPU and 8-rank SOLO V-cycles, per grid size
set -o pipefail
export TMPDIR=/tmp
cd /tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rr_new -o t -- python3 $GRAFT_REPO_ROOT/tools/bench_local_split.py --solo 1 8 && \
MAD_HIP_LIB=$GRAFT_REPO_ROOT/tools/pglibs/libmad_rr4.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rr_old -o t -- python3 $GRAFT_REPO_ROOT/tools/bench_local_split.py --solo 1 8 && \
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_filter.py tests/test_gpu_distributed.py tests/test_gpu_c4_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread
