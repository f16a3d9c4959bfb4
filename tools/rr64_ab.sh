# fp64 descent grid target (MAD_RR64_TARGET probe builds): FP64 V-cycle kernel traces
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/rr64_1024 -o vc -- python3 $R/tools/vcycle_trace_fp64.py || exit 1
for v in 256 512 2048; do
  MAD_HIP_LIB=$R/tools/pglibs/libmad_rr64t$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/rr64_$v -o vc -- python3 $R/tools/vcycle_trace_fp64.py || exit 1
done
