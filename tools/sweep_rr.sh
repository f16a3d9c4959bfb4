#!/bin/bash
# resid_restrict3_k launch shape at 512^3 (level 0 -> 1): coarse tile x grid target,
# kernel-trace mean per instantiation + V-cycle time
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in 0 1; do
  for b in 256 512 1024; do
    d=gpurun_out/rr_${t}_$b
    MAD_RR_TILE=$t MAD_RR_BLOCKS=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o rr -- python3 bench.py --steps 2 --warmup 1 --vcycles 20 --no-cpu-baseline > $d.log 2>&1
    python3 - "$d" "$t" "$b" <<'PY'
import csv, glob, json, sys
d, t, b = sys.argv[1:4]
f = glob.glob(d + "/*kernel_stats.csv")[0]
rows = [r for r in csv.DictReader(open(f)) if "resid_restrict3_k" in r["Name"]]
line = [l for l in open(d + ".log") if l.startswith("{")][-1]
print(f"tile={t} blocks={b} vcycle_ms={json.loads(line)['ms_per_vcycle']}",
      " ".join(f"{r['Name'].split('(')[0].split('<')[1][:-1]}:{float(r['AverageNs'])/1e3:.1f}us" for r in rows))
PY
  done
done
