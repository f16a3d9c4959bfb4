"""Does where the 512^3 sweep's arrays land in device memory change its speed?  (round 4 saw
the third-allocated solver of a process sweep ~20 % slower, profiles/r04_tile_order_ab.md)

Each configuration runs in a fresh process: hipMalloc a spacer of S MiB first (kept), then
build the bench's SMOOTHER-layout 512^3 solver and time its level-0 sweep (mean kernel ms of
40 launches after 5 warm-up sweeps); `--order N` builds N solvers one after another in the
same process (all kept alive) and times each.
    python tools/placement_probe.py [spacer_mib ...]
    python tools/placement_probe.py --order 3
Round 6: `--places REPS SPEC ...` alternates fresh processes of the specs: tune (the default setup, with
the level-0 placement tuning), notune (MAD_OPT_NO_PLACEMENT_TUNE), prefixed vcycle- (the V-cycle layout's
sweep) or flip- (gs_kernel 4); each line carries the setup's placement trials (mad_placement_trials).
The round-6 runs that carved the level's arrays from one block (MAD_LEVEL0_PLACE, profiles/r06_place*.log)
used a probe hook of commit 21c67c3, removed since."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sweep_ms(M):
    opt = M.capi.OPT_NO_PLACEMENT_TUNE if os.environ.get("MAD_PROBE_NOTUNE") == "1" else 0
    if os.environ.get("MAD_PROBE_NORECB") == "1":  # SMOOTHER without b in the records (split-b sweep)
        opt |= M.capi.OPT_NO_RECORD_B
    cyc = M.VCYCLE if os.environ.get("MAD_PROBE_LAYOUT") == "vcycle" else M.SMOOTHER
    # MAD_PROBE_GSK=4: the last z-chunk marched downward (mad_desc.gs_kernel 4)
    s = M.Solver((512, 512, 512), (1.0, 1.0, 1.0), time_step=0.1, precision=M.FP32, cycle=cyc,
                 options=opt, gs_kernel=int(os.environ.get("MAD_PROBE_GSK", "0")))
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    s.bench_smooth(0, 5)
    _, kern, _ = s.bench_smooth(0, 40)
    return s, kern


def one(spacer_mib):
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    if spacer_mib:
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(spacer_mib << 20)) == 0
    import multigridanisotropicdiffusion_amd as M
    s, kern = sweep_ms(M)
    print(json.dumps({"spacer_mib": spacer_mib, "spacer_ptr": hex(p.value or 0), "kernel_ms": round(kern, 4),
                      "placement_trials": [round(v, 4) for v in s.placement_trials()]}), flush=True)


def order(n, free=False, prealloc=0):
    import multigridanisotropicdiffusion_amd as M
    if prealloc:  # a buffer allocated and freed before the first solver
        hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(prealloc << 20)) == 0
        assert hip.hipFree(p) == 0
    keep = []
    for q in range(n):
        s, kern = sweep_ms(M)
        if free:
            s.close()
        else:
            keep.append(s)
        print(json.dumps({"solver": q, "freed": free, "prealloc_mib": prealloc, "kernel_ms": round(kern, 4)}),
              flush=True)


def places(specs, reps):
    """round 6: fresh process per spec, the specs alternated `reps` times (see the module doc)"""
    for rep in range(reps):
        for label in specs:
            spec = label
            env = dict(os.environ)
            env.pop("MAD_PROBE_NOTUNE", None)
            env.pop("MAD_PROBE_LAYOUT", None)
            env.pop("MAD_PROBE_GSK", None)
            env.pop("MAD_PROBE_NORECB", None)
            if spec.startswith("bs"):  # SMOOTHER layout, b from the split copy instead of the records
                env["MAD_PROBE_NORECB"] = "1"
                spec = spec[len("bs"):].lstrip("-") or "tune"
            if spec.startswith("flip"):  # gs_kernel 4: the second z-chunk marches downward
                env["MAD_PROBE_GSK"] = "4"
                spec = spec[len("flip"):].lstrip("-") or "tune"
            if spec.startswith("vcycle"):  # the V-cycle layout's level-0 sweep (36-B records, dense b)
                env["MAD_PROBE_LAYOUT"] = "vcycle"
                spec = spec[len("vcycle"):].lstrip("-") or "tune"
            if spec == "notune":  # the first allocation, as before round 6
                env["MAD_PROBE_NOTUNE"] = "1"
            elif spec not in ("sep", "tune"):
                raise SystemExit(f"unknown spec {label}")
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", "0"], capture_output=True,
                               text=True, timeout=120, env=env)
            out = r.stdout.strip()
            res = json.loads(out) if r.returncode == 0 and out else {}
            kern = res.get("kernel_ms")
            notes = [ln for ln in r.stderr.splitlines() if ln.startswith("[mad]")]
            print(json.dumps({"rep": rep, "place": label, "kernel_ms": kern, "trials": res.get("placement_trials"),
                              "notes": notes}) if kern else
                  f"{label}: rc {r.returncode} {r.stderr[-400:]}", flush=True)
            if r.returncode != 0:
                return 1
    return 0


def main():
    a = sys.argv[1:]
    if a and a[0] == "--places":
        return places(a[2:], int(a[1]))
    if a and a[0] == "--one":
        return one(int(a[1]))
    if a and a[0] == "--order":
        return order(int(a[1]))
    if a and a[0] == "--order-free":
        return order(int(a[1]), free=True)
    if a and a[0] == "--prealloc":
        return order(int(a[2]) if len(a) > 2 else 1, prealloc=int(a[1]))
    sizes = [int(v) for v in a] or [0, 2, 64, 512, 1024, 2048, 4096, 6144, 8192, 0]
    for mib in sizes:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", str(mib)], capture_output=True,
                           text=True, timeout=120)
        print(r.stdout.strip() or r.stderr[-500:], flush=True)


if __name__ == "__main__":
    main()
