#!/bin/bash
# Extra PMC passes (one counter group per run, kernel-trace only) on the
# tools/profile_traffic.py workload:  tools/profile_counters.sh TAG "TRAFFIC ARGS" GROUP...
# GROUP is a space-free comma list of counters, e.g. TCC_HIT_sum,TCC_MISS_sum
set -e
TAG=$1; TARGS=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv -d "$OUT/pmc$i" -o pmc \
      -- python3 tools/profile_traffic.py $TARGS > "$OUT/pmc$i.log" 2>&1
done
echo "counters $TAG done"
