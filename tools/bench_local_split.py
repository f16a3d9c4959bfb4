"""Proxy for the per-rank cost of the z-slab split on a one-GPU box: N ranks of the
512^3 volume run as threads of one process on one device (in-process transport,
real boundary/interior split and plane exchange).  Their kernels mostly serialise on
the GPU (each fused launch fills every CU), so wall / N approximates one rank's
sweep time on its own GPU, and 1-GPU time / (wall / N) the strong-scaling factor
the sweep alone allows (xGMI transfer time not included: the device copies of the
in-process transport stand in for it).

    python tools/bench_local_split.py [N ...]
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    S, sweeps, vcyc = 512, 20, 3
    for n in [int(v) for v in (sys.argv[1:] or ["1", "2", "4", "8"])]:
        bar = threading.Barrier(n)
        res = {}

        def body(r, s):
            s.synth_tensor(kind=0, seed=4)
            s.setup()
            s.synth_level(0, M.capi.B, 3)
            s.synth_level(0, M.capi.X, 3)
            s.bench_smooth(0, 3)
            s.synchronize()
            bar.wait()
            t0 = time.perf_counter()
            _, kern, _ = s.bench_smooth(0, sweeps)
            s.synchronize()
            bar.wait()
            t1 = time.perf_counter()
            s.vcycle()
            s.synchronize()
            bar.wait()
            t2 = time.perf_counter()
            for _ in range(vcyc):
                s.vcycle()
            s.synchronize()
            bar.wait()
            t3 = time.perf_counter()
            res[r] = (t1 - t0, kern, t3 - t2, s.level_info(0)["shape"])
            return None

        if n == 1:
            body(0, M.Solver((S, S, S), time_step=0.1, cycle=M.SMOOTHER))
        else:
            D.run_local(n, body, (S, S, S), time_step=0.1, cycle=M.SMOOTHER)
        wall = max(v[0] for v in res.values())
        vwall = max(v[2] for v in res.values())
        print(json.dumps({"ranks": n, "slab": list(res[0][3]),
                          "wall_ms_per_sweep": wall / sweeps * 1e3,
                          "rank_equiv_ms_per_sweep": wall / sweeps * 1e3 / n,
                          "rank0_kernel_ms": res[0][1],
                          "wall_ms_per_vcycle": vwall / vcyc * 1e3,
                          "rank_equiv_ms_per_vcycle": vwall / vcyc * 1e3 / n}), flush=True)


if __name__ == "__main__":
    main()
