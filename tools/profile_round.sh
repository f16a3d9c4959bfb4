#!/bin/bash
# rocprofv3 evidence for the bench kernel, three separate runs (never --pmc with trace domains):
#   1. --kernel-trace --stats of the bench command itself  -> per-kernel averages
#   2. --pmc FETCH_SIZE  on tools/profile_traffic.py        -> HBM reads (calibrated)
#   3. --pmc WRITE_SIZE  on tools/profile_traffic.py        -> HBM writes
#   tools/profile_round.sh TAG "BENCH ARGS" "TRAFFIC ARGS"
# Each step has its own time limit; the script stops at the first failure.
set -e
TAG=$1; BARGS=${2:-}; TARGS=${3:-}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
    -- python3 bench.py --no-cpu-baseline $BARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o fetch \
    -- python3 tools/profile_traffic.py $TARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o write \
    -- python3 tools/profile_traffic.py $TARGS > "$OUT/write.log" 2>&1
echo "profile $TAG done"
