#!/bin/bash
# Kernel traces of the graph-replayed V-cycle with the one-launch tail and with the per-level launches
# (MAD_OPT_NO_VCYCLE_TAIL = 128): one GPU and one interior rank of 8 through RCCL (RCCL-SOLO).
#   -> gpurun_out/vt_{1,1n,8,8n}/
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vt_1 -o vc -- python3 $R/tools/vcycle_trace.py
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vt_1n -o vc -- python3 $R/tools/vcycle_trace.py --options 128
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vt_8 -o vc -- python3 $R/tools/vcycle_trace.py --ranks 8 --rccl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vt_8n -o vc -- python3 $R/tools/vcycle_trace.py --ranks 8 --rccl --options 128
echo "tail profiles done"
