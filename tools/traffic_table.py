"""Calibrated per-launch HBM bytes of every kernel in a tools/traffic_pass.sh directory.
FETCH_SIZE / WRITE_SIZE (KiB) are scaled by the factors that make sumsq_k read and fill_k
write exactly 4 N bytes (tools/profile_traffic.py runs both on the 512^3 level 0 first);
MI355X_MICROARCH.md: FETCH_SIZE under-reports wide streaming reads on gfx950.
    python tools/traffic_table.py gpurun_out/tr7 [--n 134217728]"""
import argparse
import csv
import glob
import os


def load(root, name, counter):
    f = glob.glob(os.path.join(root, name, "*counter_collection.csv"))[0]
    d = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            d.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]) * 1024.0)
    return d


def main():
    p = argparse.ArgumentParser()
    p.add_argument("root")
    p.add_argument("--n", type=float, default=512.0 ** 3)
    a = p.parse_args()
    fe = load(a.root, "fetch", "FETCH_SIZE")
    wr = load(a.root, "write", "WRITE_SIZE")
    cf = 4 * a.n / [v for k, v in fe.items() if "sumsq_k" in k][0][0]
    cw = 4 * a.n / [v for k, v in wr.items() if "fill_k" in k][0][0]
    print(f"calibration: fetch x{cf:.3f}, write x{cw:.3f}")
    for k in fe:
        f = sum(fe[k]) / len(fe[k]) * cf
        w = sum(wr.get(k, [0.0])) / max(1, len(wr.get(k, [0.0]))) * cw
        print(f"{k[:70]:70s} n={len(fe[k]):2d} read {f/1e9:7.3f} GB ({f/a.n:6.2f} B/vox)  "
              f"write {w/1e9:7.3f} GB ({w/a.n:6.2f} B/vox)")


if __name__ == "__main__":
    main()
