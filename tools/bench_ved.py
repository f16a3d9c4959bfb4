"""VED pipeline timing (BASELINE config C4 "512^3 VED pipeline"):
tensor generation (5 scales: Hessian + eigen-analysis + vesselness + tensor) and the
whole filter (1 iteration, DiffusionIterations steps) on a synthetic tube phantom.

    python tools/bench_ved.py [--size 512] [--steps 5] [--reps 3]

Phantom: 64 axis-aligned bright tubes (radius 2..6 voxels, intensity 200 on 0,
seed 4) plus N(0, 10^2) noise, fp32.  Prints one JSON line; per-kernel durations
come from rocprofv3 runs of this script (tools/profile_ved.sh).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def phantom(S, seed=4):
    rng = np.random.default_rng(seed)
    img = rng.normal(0.0, 10.0, size=(S, S, S)).astype(np.float32)
    g = np.arange(S, dtype=np.float32)
    for axis in range(3):
        prof = np.zeros((S, S), np.float32)
        for _ in range(64 // 3 + (1 if axis < 64 % 3 else 0)):
            a, b = rng.uniform(8, S - 8, size=2)
            r = rng.uniform(2, 6)
            prof += 200.0 * np.exp(-((g[:, None] - a) ** 2 + (g[None, :] - b) ** 2) / (2 * r * r))
        if axis == 0:    # tube along z: profile over (y, x)
            img += prof[None, :, :]
        elif axis == 1:  # along y: profile over (z, x)
            img += prof[:, None, :]
        else:            # along x: profile over (z, y)
            img += prof[:, :, None]
    return img


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--fp64", action="store_true")
    ap.add_argument("--ranks", type=int, default=1,
                    help="> 1: one interior rank (ranks // 2) of that decomposition alone on the device "
                         "(mad_ved_comm_init_solo): its partitioned tensor generation and slab diffusion")
    ap.add_argument("--hessian", action="store_true",
                    help="also run one Hessian-only pass (profiling the FIR without the eigen stage)")
    a = ap.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    t0 = time.perf_counter()
    img = phantom(S)
    t_ph = time.perf_counter() - t0
    prec = M.FP64 if a.fp64 else M.FP32
    rk = dict(nranks=a.ranks, rank=a.ranks // 2) if a.ranks > 1 else {}
    v = M.VED((S, S, S), (1.0, 1.0, 1.0), omega=1.5, diffusion_iterations=a.steps,
              precision=prec, **rk)
    if a.ranks > 1:
        v.comm_init_solo()
    if a.hessian and a.ranks == 1:
        v.hessian(img, 2.0)
    # tensor generation only (device time from the run's stats is below; here wall)
    tw = [float("nan")]
    if a.ranks == 1:
        v.tensor(img)  # warm-up (allocations)
        tw = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            v.tensor(img)
            tw.append(time.perf_counter() - t0)
    runs = []
    if a.ranks > 1:
        v.run(img, out_dtype=np.float32)  # warm-up (allocations, first eager cycles)
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out, st = v.run(img, out_dtype=np.float32)
        st["wall_ms"] = (time.perf_counter() - t0) * 1e3
        runs.append(st)
    best = min(runs, key=lambda r: r["wall_ms"])
    N = float(S) ** 3
    print(json.dumps({
        "workload": f"VED {S}^3 tube phantom, 5 scales, 1 iteration, {a.steps} diffusion steps",
        "ranks": a.ranks, "rank": a.ranks // 2 if a.ranks > 1 else 0,
        "precision": "fp64" if a.fp64 else "fp32",
        "tensor_wall_ms_incl_pcie": round(min(tw) * 1e3, 2),
        "tensor_device_ms": round(best["tensor_ms"], 3),
        "diffusion_device_ms": round(best["diffusion_ms"], 3),
        "ved_wall_ms_incl_pcie": round(best["wall_ms"], 2),
        "cycles": best["total_cycles"], "last_relres": best["last_relres"],
        "tensor_Mvox_per_s": round(N / (best["tensor_ms"] * 1e-3) / 1e6, 1),
        "phantom_s": round(t_ph, 1),
    }), flush=True)


if __name__ == "__main__":
    main()
