"""Host API calls that block inside the traced V-cycles: from a rocprofv3 run with
--kernel-trace --hip-runtime-trace (no PMC), list the HIP API calls longer than --min-us whose span
overlaps the last --cycles cycles (delimited by coarse_solve_k launches), grouped by name.
    python tools/api_stalls.py OUTDIR [--cycles 10] [--min-us 100]"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("root")
    p.add_argument("--cycles", type=int, default=10)
    p.add_argument("--min-us", type=float, default=100.0)
    a = p.parse_args()
    kt = glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True)[0]
    at = glob.glob(os.path.join(a.root, "**", "*hip_api_trace.csv"), recursive=True)[0]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(kt)))
    ends = [i for i, e in enumerate(ev) if "coarse_solve" in e[2]]
    t0, t1 = ev[ends[-a.cycles - 1]][1], ev[ends[-1]][1]
    print(f"window {(t1 - t0) / 1e3:.1f} us over {a.cycles} cycles ({(t1 - t0) / 1e3 / a.cycles:.1f} us per cycle)")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    rows = []
    for r in csv.DictReader(open(at)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 or s > t1:
            continue
        d = (e - s) / 1e3
        g = agg[r["Function"]]
        g[0] += 1
        g[1] += d
        g[2] = max(g[2], d)
        if d >= a.min_us:
            rows.append((s, d, r["Function"]))
    print("API calls in the window: name, count, total us, max us")
    for k, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {k:40s} {n:6d} {tot:10.1f} {mx:9.1f}")
    print(f"calls >= {a.min_us} us:")
    for s, d, f in sorted(rows)[:40]:
        print(f"  t+{(s - t0) / 1e3:10.1f} us  {d:9.1f} us  {f}")


if __name__ == "__main__":
    main()
