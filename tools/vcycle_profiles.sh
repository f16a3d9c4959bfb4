#!/bin/bash
# Kernel traces of the graph-replayed V-cycle (tools/vcycle_trace.py): one GPU, and one interior rank of 8
# through RCCL (RCCL-SOLO) with the exchange and with the peer halo.  -> gpurun_out/vc_{1,8rccl,8peer}/
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vc_1 -o vc -- python3 $R/tools/vcycle_trace.py
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vc_8rccl -o vc -- python3 $R/tools/vcycle_trace.py --ranks 8 --rccl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vc_8peer -o vc -- python3 $R/tools/vcycle_trace.py --ranks 8 --rccl --options 4
echo "vcycle profiles done"
