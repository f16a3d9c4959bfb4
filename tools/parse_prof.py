"""Summarise rocprofv3 CSV output into profiles/.

  python tools/parse_prof.py --trace gpurun_out/prof_trace/bench_kernel_stats.csv \
      --fetch gpurun_out/prof_fetch/fetch_counter_collection.csv \
      --write gpurun_out/prof_write/write_counter_collection.csv \
      --kernel gs_color_k --size 512 --tag r01_gs_512 [--traffic-json profiles/traffic_gs_512.json]

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are
in KiB; FETCH_SIZE under-reports reads on gfx950, so both are calibrated on
kernels of known traffic in the same process and access width: sumsq_k<float>
reads exactly 4*N bytes, fill_k<float> writes exactly 4*N bytes
(tools/profile_traffic.py).
"""
import argparse
import csv
import json
import os


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def find(d, sub):
    keys = [k for k in d if sub in k]
    if not keys:
        raise KeyError(sub)
    return keys[0], d[keys[0]]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--trace", required=True)
    p.add_argument("--ktrace", help="kernel_trace.csv of the same run (per-dispatch durations)")
    p.add_argument("--tail", type=int, default=0,
                   help="also average the last N level-0 dispatches (the bench's timed + sustained windows; "
                        "the earlier ones include setup's placement trials)")
    p.add_argument("--fetch")
    p.add_argument("--write")
    p.add_argument("--kernel", required=True)
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--tag", required=True)
    p.add_argument("--alg-bytes-per-launch", type=float, required=True)
    p.add_argument("--traffic-json")
    a = p.parse_args()
    lines = [f"# rocprofv3 summary: {a.tag}", ""]
    rows = list(csv.DictReader(open(a.trace)))
    lines.append("## kernel stats (rocprofv3 --kernel-trace --stats)")
    lines.append("")
    lines.append("| kernel | calls | avg us | total ms | % |")
    lines.append("|---|---|---|---|---|")
    for r in rows[:15]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                     f"{float(r['TotalDurationNs'])/1e6:.3f} | {r['Percentage']} |")
    target = [r for r in rows if a.kernel in r["Name"]][0]
    avg_ns = float(target["AverageNs"])
    lines += ["", f"target kernel `{target['Name']}`: average {avg_ns/1e3:.2f} us over "
              f"{target['Calls']} calls (includes coarse-level launches)"]
    res = {"kernel": target["Name"], "trace_avg_us_all_levels": avg_ns / 1e3}
    if a.ktrace:
        groups = {}
        for r in csv.DictReader(open(a.ktrace)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            groups.setdefault(g, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        gmax = max(groups)
        d = groups[gmax]
        # coarser levels can launch the same grid (z-chunks): keep the level-0 cluster
        # (durations within 40% of the longest dispatch of that grid)
        ref = sorted(d)[(len(d) * 9) // 10]  # (not the maximum: one stalled dispatch would set it)
        d = [v for v in d if v >= 0.6 * ref]
        lvl0 = sum(d) / len(d) / 1e3
        res["trace_avg_us_level0"] = lvl0
        res["trace_level0_calls"] = len(d)
        lines += [f"level-0 dispatches (grid {gmax} work-items): {len(d)} calls, average "
                  f"{lvl0:.2f} us, min {min(d)/1e3:.2f} us, max {max(d)/1e3:.2f} us "
                  f"(compare bench.py roofline.kernel_ms_mean)"]
        if a.tail and len(d) >= a.tail:
            t = d[-a.tail:]
            res["trace_avg_us_level0_tail"] = sum(t) / len(t) / 1e3
            lines += [f"the last {a.tail} of them (the bench's timed + sustained windows): average "
                      f"{sum(t) / len(t) / 1e3:.2f} us, median {sorted(t)[len(t) // 2] / 1e3:.2f} us"]
    if a.fetch and a.write:
        n = float(a.size) ** 3
        fe = per_kernel(a.fetch, "FETCH_SIZE")
        wr = per_kernel(a.write, "WRITE_SIZE")
        _, cal_r = find(fe, "sumsq_k<float>")
        _, cal_w = find(wr, "fill_k<float>")
        fr = 4.0 * n / cal_r[0]
        fw = 4.0 * n / cal_w[0]
        kname, kf = find(fe, a.kernel)
        _, kw = find(wr, a.kernel)
        # level-0 launches are the large ones
        big_f = sorted(kf)[len(kf) // 2:]
        big_w = sorted(kw)[len(kw) // 2:]
        rd = sum(big_f) / len(big_f) * fr
        wt = sum(big_w) / len(big_w) * fw
        tot = rd + wt
        lines += ["", "## HBM traffic (rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE passes)", "",
                  f"calibration: sumsq_k reads {4*n/1e6:.1f} MB, FETCH_SIZE said {cal_r[0]/1e6:.1f} MB "
                  f"-> read factor {fr:.3f}; fill_k writes {4*n/1e6:.1f} MB, WRITE_SIZE said "
                  f"{cal_w[0]/1e6:.1f} MB -> write factor {fw:.3f}",
                  "",
                  f"`{kname[:80]}` per level-0 launch: reads {rd/1e9:.3f} GB, writes {wt/1e9:.3f} GB, "
                  f"total {tot/1e9:.3f} GB vs algorithmic {a.alg_bytes_per_launch/1e9:.3f} GB "
                  f"(ratio {tot/a.alg_bytes_per_launch:.2f})"]
        res.update({"bytes_per_launch": tot, "read_bytes_per_launch": rd, "write_bytes_per_launch": wt,
                    "algorithmic_bytes_per_launch": a.alg_bytes_per_launch,
                    "read_factor": fr, "write_factor": fw,
                    "source": f"profiles/{a.tag}_summary.md (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, "
                              "calibrated on sumsq_k/fill_k)"})
        if a.traffic_json:
            json.dump(res, open(a.traffic_json, "w"), indent=1)
    os.makedirs("profiles", exist_ok=True)
    open(f"profiles/{a.tag}_summary.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
