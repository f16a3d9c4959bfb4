#!/bin/bash
# SQ counter passes over V-cycles of the bench workload (tools/vcycle_trace.py), each --pmc
# set in its own run; output dir prefix $1 (gpurun_out/<prefix>1, <prefix>2)
P=${1:-sqv}
W="python3 tools/vcycle_trace.py --cycles 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/${P}1 -o s -- $W &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/${P}2 -o s -- $W
