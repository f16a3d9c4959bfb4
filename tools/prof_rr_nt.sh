#!/bin/bash
# per-launch durations of the one-pass residual + restriction at 512^3 for each
# block shape (rocprofv3 kernel trace; the stats CSV holds the average per kernel)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFGS=${CFGS:-"1024 512|512 1024|512 512|1024 1024"}
IFS="|" read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  MAD_RR_NT=$1 MAD_RR_BLOCKS=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rr_$1_$2 -o run -- python3 bench.py --steps 3 --warmup 1 --vcycles 20 --no-cpu-baseline > /dev/null 2>&1
  f=$(find gpurun_out/prof_rr_$1_$2 -name "*kernel_stats.csv" | head -1)
  echo "NT=$1 blocks=$2"; grep resid_restrict "$f" | cut -c1-200
done
