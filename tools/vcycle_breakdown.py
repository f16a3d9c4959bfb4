"""Per-V-cycle breakdown of a rocprofv3 kernel trace (tools/vcycle_trace.py):
device-busy time vs span (launch gaps), and time per kernel family and grid size.
    python tools/vcycle_breakdown.py gpurun_out/vc/vc_kernel_trace.csv [--cycles 10]"""
import argparse
import csv
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--cycles", type=int, default=10)
    a = p.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = []
    for r in rows:
        name = r["Kernel_Name"]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        ev.append((t0, t1, name, grid))
    ev.sort()
    # the timed cycles are the last `cycles` repetitions; one coarse solve per V-cycle, so the
    # kernels after the (cycles+1)-th last coarse solve up to the last one are `cycles` whole
    # cycles' worth (second half of one, first half of the next)
    # (with the one-launch V-cycle tail, vtail_k stands in for the coarse solve)
    cs = [i for i, e in enumerate(ev) if "coarse_solve" in e[2] or "vtail_k" in e[2]]
    sel = ev[cs[-(a.cycles + 1)] + 1: cs[-1] + 1]
    span = (sel[-1][1] - sel[0][0]) / 1e6
    busy = sum(e[1] - e[0] for e in sel) / 1e6
    print(f"launches per cycle {len(sel) / a.cycles:.1f}; span {span / a.cycles:.3f} ms/cycle, "
          f"busy {busy / a.cycles:.3f} ms/cycle, gaps {(span - busy) / a.cycles:.3f} ms/cycle")
    fam = defaultdict(lambda: [0, 0.0])
    for e in sel:
        short = e[2].split("(")[0].replace("void ", "")
        k = (short[:90], e[3])
        fam[k][0] += 1
        fam[k][1] += (e[1] - e[0]) / 1e6
    print("| kernel | grid | launches/cycle | ms/cycle | us/launch |")
    print("|---|---|---|---|---|")
    for k, (n, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k[0]}` | {k[1]} | {n / a.cycles:.1f} | {t / a.cycles:.4f} | {t / n * 1e3:.1f} |")


if __name__ == "__main__":
    main()
