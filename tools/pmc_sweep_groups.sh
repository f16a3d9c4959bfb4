#!/bin/bash
# Counter passes on the bench kernel (tools/profile_traffic.py: 3 level-0 sweeps of the 512^3
# SMOOTHER-mode system), one rocprofv3 --pmc run per group, each under a hard kill limit.
#   tools/pmc_sweep_groups.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc_groups}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_TOTAL_CYCLES_sum" \
  "TD_TD_BUSY_sum TD_TC_STALL_sum" \
  "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
  "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum" \
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_avr" \
  "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
  "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc \
      -- python3 tools/profile_traffic.py > "$OUT/p$i.log" 2>&1
done
echo "pmc groups done: $OUT"
