#!/bin/bash
# PMC passes for the fused-GS variants and the streaming probe (one counter group per run)
set -e
export TMPDIR=/tmp
G="FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_32B_sum TCC_HIT_sum,TCC_MISS_sum"
MAD_FUSED_TILE=0 MAD_FUSED_BLOCKS=2048 bash tools/profile_counters.sh cnt_t0 "--gs-kernel 3" $G
MAD_FUSED_TILE=1 MAD_FUSED_BLOCKS=1024 bash tools/profile_counters.sh cnt_t1 "--gs-kernel 3" $G
mkdir -p gpurun_out/cnt_probe
i=0
for grp in $G; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv -d gpurun_out/cnt_probe/pmc$i -o pmc -- tools/stream_probe 3 > gpurun_out/cnt_probe/pmc$i.log 2>&1
done
echo done
