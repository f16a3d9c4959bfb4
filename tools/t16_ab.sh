# fp32 full-tensor sweeps below level 0 in 64x16 / 512-thread tiles (MAD_SMALL_TILE16 probe) vs 64x32 / 1024
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/t16_base -o vc -- python3 $R/tools/vcycle_trace.py && \
MAD_HIP_LIB=$R/tools/pglibs/libmad_t16.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/t16_new -o vc -- python3 $R/tools/vcycle_trace.py && \
cd $R && for r in 1 2; do
  echo "== base" && timeout -k 10 150 python tools/bench_local_split.py --solo 1 2 && \
  echo "== t16" && MAD_HIP_LIB=tools/pglibs/libmad_t16.so timeout -k 10 150 python tools/bench_local_split.py --solo 1 2 || exit 1
done
