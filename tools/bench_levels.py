"""Per-level smoother timing (kernel mean per launch and per sweep) on the bench
workload, for choosing the smoother kernel per level size.
    python tools/bench_levels.py [--gs-kernel K] [--size 512] [--sweeps 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gs-kernel", type=int, default=0)
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--sweeps", type=int, default=10)
    p.add_argument("--smoother", default="gs", choices=["gs", "wj"])
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    sm = M.GAUSS_SEIDEL if a.smoother == "gs" else M.WEIGHTED_JACOBI
    s = M.Solver((S, S, S), time_step=0.1, smoother=sm, gs_kernel=a.gs_kernel, cycle=M.SMOOTHER)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    out = []
    for l in range(s.num_levels):
        s.synth_level(l, M.capi.B, 3)
        s.synth_level(l, M.capi.X, 5)
        s.bench_smooth(l, 2)
        tot, kern, n = s.bench_smooth(l, a.sweeps)
        shape = s.shape_at(l)
        nv = shape[0] * shape[1] * shape[2]
        out.append({"level": l, "shape": shape, "kernel": s.smooth_kernel_name(l),
                    "ms_per_sweep": tot / a.sweeps, "kernel_ms_mean": kern, "launches": n,
                    "gvox_per_s": nv / (tot / a.sweeps * 1e-3) / 1e9})
    tot, = [s.bench_vcycle(5)]
    print(json.dumps({"gs_kernel": a.gs_kernel, "levels": out, "ms_per_vcycle_smoother_layout": tot / 5}))


if __name__ == "__main__":
    main()
