"""Is the level-0 sweep's 1.13 / 1.18 / 1.25 ms spread the memory system's clocks?  Runs the SMOOTHER-layout
512^3 sweep back to back for ~SECONDS while a separate process samples the GPU's SMU metrics table
(amdsmi_get_gpu_metrics_info: current clocks, power, temperatures, throttle status) of the same device,
then prints both on one time line (50 ms windows: mean / min / max kernel ms beside the clocks sampled in
the window).  Raw data: OUT/sweeps.jsonl, OUT/metrics.jsonl.
    python tools/clock_probe.py OUT [SECONDS]"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def scalar(v):
    if isinstance(v, (list, tuple)):
        v = [x for x in v if isinstance(x, (int, float)) and x not in (65535, 0xFFFFFFFF, 2**64 - 1)]
        return v[0] if v else None
    return v if isinstance(v, (int, float)) else None


def sample(out, bdf, seconds):
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    h = None
    for q in hs:
        if amdsmi.amdsmi_get_gpu_device_bdf(q).lower().endswith(bdf.lower()[-7:]):
            h = q
    h = h or hs[0]
    t_end = time.time() + seconds
    with open(out, "w") as f:
        first = True
        while time.time() < t_end:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            rec = {k: scalar(v) for k, v in m.items()}
            rec = {k: v for k, v in rec.items() if v is not None}
            if first:  # every field once, lists as they are
                f.write(json.dumps({"t": time.time(), "full": {k: str(v)[:200] for k, v in m.items()}}) + "\n")
                first = False
            f.write(json.dumps({"t": time.time(), "m": rec}) + "\n")
            time.sleep(0.005)
    amdsmi.amdsmi_shut_down()


def main():
    if sys.argv[1] == "--sample":
        return sample(sys.argv[2], sys.argv[3], float(sys.argv[4]))
    out = sys.argv[1]
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
    os.makedirs(out, exist_ok=True)
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    hip.hipDeviceGetPCIBusId(buf, 64, 0)
    bdf = buf.value.decode()
    import multigridanisotropicdiffusion_amd as M
    s = M.Solver((512, 512, 512), (1.0, 1.0, 1.0), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    s.bench_smooth(0, 5)
    smp = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--sample",
                            os.path.join(out, "metrics.jsonl"), bdf, str(seconds + 1.0)])
    time.sleep(0.5)
    rows = []
    t_end = time.time() + seconds
    while time.time() < t_end:
        t0 = time.time()
        s.bench_smooth(0, 10)
        t1 = time.time()
        ms = s.bench_launch_times()
        rows.append({"t0": t0, "t1": t1, "ms": [round(v, 4) for v in ms]})
    smp.wait(timeout=30)
    with open(os.path.join(out, "sweeps.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    mets = [json.loads(ln) for ln in open(os.path.join(out, "metrics.jsonl"))]
    full = [m for m in mets if "full" in m]
    if full and os.environ.get("CLOCK_PROBE_TIMELINE") == "1":
        print("metrics fields:", json.dumps(full[0]["full"])[:3000])
    mets = [m for m in mets if "m" in m]
    keys = [k for k in ("current_gfxclk", "current_gfxclks", "current_uclk", "current_socclk", "current_socclks",
                        "current_fclk", "average_socket_power", "current_socket_power", "temperature_hotspot",
                        "temperature_mem", "throttle_status", "indep_throttle_status")
            if any(k in m["m"] for m in mets)]
    allk = sorted(v for r in rows for v in r["ms"])
    summ = {"launches": len(allk), "kern_mean": round(sum(allk) / len(allk), 4),
            "kern_median": allk[len(allk) // 2], "frac_over_1.2ms": round(sum(v > 1.2 for v in allk) / len(allk), 3)}
    for k in keys:
        vals = [m["m"][k] for m in mets if k in m["m"]]
        if vals:
            summ[k] = round(sum(vals) / len(vals), 1)
    print("SUMMARY " + json.dumps(summ), flush=True)
    if os.environ.get("CLOCK_PROBE_TIMELINE") != "1":
        s.close()
        return
    print("window_start  n  kern_mean kern_min kern_max | " + " ".join(keys))
    t = rows[0]["t0"] if rows else time.time()
    while rows and t < rows[-1]["t1"]:
        w = [v for r in rows if t <= r["t0"] < t + 0.05 for v in r["ms"]]
        mm = [m["m"] for m in mets if t <= m["t"] < t + 0.05]
        if w:
            cols = []
            for k in keys:
                vals = [m[k] for m in mm if k in m]
                cols.append(f"{min(vals)}-{max(vals)}" if vals else "-")
            print(f"{t - rows[0]['t0']:8.3f} {len(w):3d} {sum(w) / len(w):.4f} {min(w):.4f} {max(w):.4f} | " +
                  " ".join(cols), flush=True)
        t += 0.05
    s.close()


if __name__ == "__main__":
    main()
