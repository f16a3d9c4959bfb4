#!/bin/bash
# PMC counters of the SMOOTHER-layout 512^3 level-0 sweep (tools/placement_probe.py --one) in a fast and a
# slow placement of level 0's arrays (MAD_LEVEL0_PLACE, csrc/mad_alloc.hpp), one --pmc pass per group,
# each in its own process under its own time limit.
#   tools/placement_pmc.sh OUT "PLACE_A" "PLACE_B" "CTR1 CTR2 ..." ["CTR ..." ...]
# ("sep" = separate allocations); CSVs under gpurun_out/OUT/<place>/<group>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$1; A=$2; B=$3; shift 3
g=0
for grp in "$@"; do
  g=$((g + 1))
  for place in "$A" "$B"; do
    tag=$(echo "$place" | tr ':,' '__')
    d=gpurun_out/$OUT/$tag/g$g
    mkdir -p "$d"
    if [ "$place" = "sep" ]; then
      timeout -s KILL 90 rocprofv3 --pmc $grp -d "$d" -o run --output-format csv -- python3 tools/placement_probe.py --one 0 > "$d/stdout.txt" 2>&1
    else
      MAD_LEVEL0_PLACE="$place" timeout -s KILL 90 rocprofv3 --pmc $grp -d "$d" -o run --output-format csv -- python3 tools/placement_probe.py --one 0 > "$d/stdout.txt" 2>&1
    fi
    rc=$?
    echo "[$place] group $g ($grp): rc $rc $(tail -1 "$d/stdout.txt")"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
