"""Seconds per solver cycle in mad_run (the reference's while-loop: cycle, residual, host check) at
512^3 on the C4 VED-form tensor, by precision mode: MAD_FP32 (the bench's mode) and
MAD_FP32_REFINE (what the default descriptor resolves to at the reference's Tolerance 1e-10).
Per-cycle time = median difference of mad_get_cycle_trace's timestamps (host clock after the
per-cycle convergence check), cycles 2 .. K of one time step (Tolerance 1e-30: every run takes K cycles).
    python tools/bench_refine.py [--size 512] [--cycles 8]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--cycles", type=int, default=12)
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    rng = np.random.default_rng(5)
    img = (rng.random((S, S, S), dtype=np.float32) * 100.0).astype(np.float32)
    out = {"size": S}
    for name, prec in (("FP32", M.FP32), ("FP32_REFINE", M.FP32_REFINE)):
        s = M.Solver((S, S, S), time_step=0.1, precision=prec, cycle=M.VCYCLE, tolerance=1e-30,
                     max_cycles=a.cycles, stall_guard=0)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        s.run(img)  # warm-up (graph capture)
        s.run(img)
        t = [q[2] for q in s.cycle_trace()]
        d = np.diff(t)[1:]
        out[name] = {"ms_per_cycle": float(np.median(d) * 1e3), "cycles": len(t),
                     "relres": s.cycle_trace()[-1][1]}
        s.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
