"""Per-kernel averages of every counter in rocprofv3 --pmc runs (one dir per pass).
   python tools/pmc_table.py gpurun_out/cnt_v2  [--kernel gs_fused]"""
import argparse
import csv
import glob
import os


def main():
    p = argparse.ArgumentParser()
    p.add_argument("root")
    p.add_argument("--kernel", default="")
    a = p.parse_args()
    acc = {}
    files = glob.glob(os.path.join(a.root, "*", "*counter_collection.csv")) + \
        glob.glob(os.path.join(a.root, "*counter_collection.csv"))
    for f in sorted(files):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if a.kernel not in k:
                continue
            key = (k, r["Counter_Name"])
            acc.setdefault(key, []).append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k[:60]:60s} {c:28s} n={len(v):3d} mean={sum(v)/len(v):.4e} max={max(v):.4e}")


if __name__ == "__main__":
    main()
