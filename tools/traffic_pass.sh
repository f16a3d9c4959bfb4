#!/bin/bash
# HBM traffic of the level-0 sweep (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs)
#   tools/traffic_pass.sh OUTDIR [profile_traffic.py args]
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o fetch \
    -- python3 tools/profile_traffic.py "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o write \
    -- python3 tools/profile_traffic.py "$@" > "$OUT/write.log" 2>&1
python3 tools/traffic_table.py "$OUT"
