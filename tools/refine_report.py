"""Cycle counts and final relres of the C1 (lena) and VED-test solves at the reference's
Tolerance 1e-10 in the three precision modes, beside the oracle's (lexicographic GS, fp64):
    python tools/refine_report.py > profiles/r02_refine_cycles.md"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import multigridanisotropicdiffusion_amd as M  # noqa: E402
import synth  # noqa: E402
from conftest import GOLDEN, load_golden  # noqa: E402

MODES = [("FP32", M.FP32), ("FP32_REFINE", M.FP32_REFINE), ("FP64", M.FP64)]


def relinf(a, ref):
    return float(np.abs(np.asarray(a, np.float64) - ref).max() / np.abs(ref).max())


print("# Reference tolerance 1e-10 by precision mode (tools/refine_report.py)\n")
print("cycles per time step / final relres / max |u - u_oracle| / max |u_oracle|; oracle = fp64"
      " lexicographic GS restating the reference (parity unpinned, DESIGN.md)\n")
print("| case | mode | cycles | oracle cycles | relres | stalled | rel. error vs oracle |")
print("|---|---|---|---|---|---|---|")
lena = np.load(os.path.join(GOLDEN, "lena_256_u8.npy")).astype(np.float64)
T2 = np.stack([np.full(lena.shape, 50.0), np.zeros(lena.shape), np.full(lena.shape, 30.0)], axis=-1)
g = load_golden("lena_c1_f64")
for sm, stag in ((M.GAUSS_SEIDEL, "gs"), (M.WEIGHTED_JACOBI, "wj")):
    for cy, ctag in ((M.VCYCLE, "v"), (M.FMG, "fmg")):
        for name, prec in MODES:
            s = M.Solver(lena.shape, (1.0, 1.0), time_step=0.1, smoother=sm, cycle=cy,
                         iterations_per_grid=2, max_cycles=100, tolerance=1e-10, precision=prec)
            s.set_tensor(T2)
            out, st = s.run(lena, out_dtype=np.float64)
            s.close()
            key = f"{stag}_{ctag}"
            print(f"| C1 lena {key} | {name} | {st['step_cycles']} | {g[key + '_cycles'].tolist()} | "
                  f"{st['last_relres']:.2e} | {st['stalled']} | {relinf(out, g[key]):.1e} |")
for fx, crop, sp in (("ved_mad", "ved_crop_i16.npy", (0.3125, 0.3125, 0.5)),
                     ("ved2_mad", "ved2_crop_i16.npy", (0.330017,) * 3)):
    v = np.load(os.path.join(GOLDEN, crop))
    g = load_golden(fx)
    for name, prec in MODES:
        s = M.Solver(v.shape, sp, time_step=0.1, iterations_per_grid=3, number_of_steps=4,
                     tolerance=1e-10, precision=prec)
        s.set_tensor(synth.ved_form(v.shape))
        out, st = s.run(v, out_dtype=np.float64)
        s.close()
        print(f"| {fx} {v.shape} | {name} | {st['step_cycles']} | {g['cycles'].tolist()} | "
              f"{st['last_relres']:.2e} | {st['stalled']} | {relinf(out, g['out']):.1e} |")
