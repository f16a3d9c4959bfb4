"""Workload for rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE are separate runs).

Runs, on the bench configuration (512^3 VED-form, fp32):
  1. calibration: sum of squares of b (reads exactly 4*N bytes, 4 B/lane) and a
     fill of r (writes exactly 4*N bytes), so the counters can be converted with
     a factor measured on our own access width (MI355X_MICROARCH.md, HBM section:
     FETCH_SIZE under-reports wide streaming reads on gfx950; calibrate per pattern);
  2. `--sweeps` smoother sweeps on level 0 (the bench kernel).
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -- \
        python tools/profile_traffic.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--sweeps", type=int, default=3)
    p.add_argument("--smoother", default="gs", choices=["gs", "wj"])
    p.add_argument("--gs-kernel", type=int, default=0)
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    sm = M.GAUSS_SEIDEL if a.smoother == "gs" else M.WEIGHTED_JACOBI
    s = M.Solver((S, S, S), time_step=0.1, smoother=sm, gs_kernel=a.gs_kernel,
                 cycle=M.SMOOTHER)  # the bench's configuration
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    s.synchronize()
    s.norm(0, M.capi.B)          # sumsq_k: 4*N bytes read
    s.fill(0, M.capi.R, 0.0)     # fill_k: 4*N bytes written
    s.synchronize()
    s.smooth(0, a.sweeps)
    s.synchronize()
    print("done", S, a.sweeps, a.smoother)


if __name__ == "__main__":
    main()
