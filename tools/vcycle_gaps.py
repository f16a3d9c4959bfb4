"""Largest idle gaps between consecutive kernels of a rocprofv3 kernel trace, grouped by the
(previous kernel, next kernel) pair: where a graph-replayed cycle waits between launches.
    python tools/vcycle_gaps.py gpurun_out/vc8/vc_kernel_trace.csv [--cycles 10] [--top 15]"""
import argparse
import csv
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").split("(")[0]
    return n if len(n) < 60 else n[:57] + "..."


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--cycles", type=int, default=10)
    p.add_argument("--top", type=int, default=15)
    a = p.parse_args()
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(a.trace)))
    # the last `cycles` cycles: delimited by the coarse solve, as tools/vcycle_breakdown.py
    ends = [i for i, e in enumerate(ev) if "coarse_solve" in e[2]]
    if len(ends) > a.cycles:
        ev = ev[ends[-a.cycles - 1] + 1:ends[-1] + 1]
    gaps = defaultdict(lambda: [0, 0.0])
    for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
        g = max(0, s1 - e0) / 1e3
        k = (n0, n1)
        gaps[k][0] += 1
        gaps[k][1] += g
    tot = sum(v[1] for v in gaps.values())
    print(f"total gap {tot / a.cycles:.1f} us per cycle over {len(ev)} launches")
    print("| previous | next | per cycle | us per cycle |")
    print("|---|---|---|---|")
    for (n0, n1), (c, g) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{n0}` | `{n1}` | {c / a.cycles:.1f} | {g / a.cycles:.1f} |")


if __name__ == "__main__":
    main()
