"""Per-kernel totals of a rocprofv3 kernel trace: calls, mean and total time, sorted by total.
    python tools/kstats.py gpurun_out/X/x_kernel_trace.csv [--top 20] [--match SUBSTR]"""
import argparse
import csv
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--top", type=int, default=20)
    p.add_argument("--match", default="")
    a = p.parse_args()
    agg = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(a.trace)):
        n = r["Kernel_Name"].replace("void ", "").split("(")[0]
        if a.match and a.match not in n:
            continue
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print("| kernel | calls | mean ms | total ms |")
    print("|---|---|---|---|")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{n[:90]}` | {c} | {t / c:.4f} | {t:.3f} |")


if __name__ == "__main__":
    main()
