"""Which counters tell a fast from a slow level-0 sweep?  The same SMOOTHER-layout 512^3 sweep runs in
1.13, 1.18 or 1.25 ms depending on the process (profiles/r06_place2.log): run fresh processes of
tools/placement_probe.py --one under `rocprofv3 --pmc GROUP` (one counter group per run, each run under its
own time limit), and print per process the probe's kernel mean and the mean of every counter over the
level-0 gs_fused3_k dispatches.
    python tools/placement_pmc.py OUTDIR REPS "CTR CTR ..." ["CTR ..." ...]   (fresh processes, default setup)"""
import csv
import glob
import json
import os
import subprocess
import sys


def counters(d):
    acc = {}
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "gs_fused3_k" in r["Kernel_Name"]]
    if not rows:
        return {}
    big = max(int(r.get("Grid_Size", 0) or 0) for r in rows)
    for r in rows:
        if int(r.get("Grid_Size", 0) or 0) != big:
            continue
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    out, reps, groups = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    probe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "placement_probe.py")
    for rep in range(reps):
        for g, grp in enumerate(groups):
            d = os.path.join(out, f"r{rep}_g{g}")
            os.makedirs(d, exist_ok=True)
            cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + grp.split() + \
                  ["-d", d, "-o", "run", "--output-format", "csv", "--", sys.executable, probe, "--one", "0"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not line:
                print(f"rep {rep} group {g}: rc {r.returncode}\n{r.stdout[-800:]}\n{r.stderr[-1500:]}", flush=True)
                return 1
            kern = json.loads(line[-1])["kernel_ms"]
            c = counters(d)
            print(json.dumps({"rep": rep, "group": g, "kernel_ms": kern,
                              "counters": {k: round(v, 1) for k, v in sorted(c.items())}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
