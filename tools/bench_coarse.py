"""Device time of the coarsest-level direct solve (mad_coarse_solve) and of whole V-cycles on
volumes whose coarsest level is large (csrc/mad_coarse.hpp block-plane LU) or small (dense
inverse), plus the setup time.
    python tools/bench_coarse.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    for shape in [(512, 512, 512), (64, 512, 512), (32, 512, 512), (40, 256, 256), (10, 130, 130),
                  (10, 256, 256)]:
        t0 = time.perf_counter()
        s = M.Solver(shape, time_step=0.1, precision=M.FP32)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        setup_s = time.perf_counter() - t0
        nl = s.num_levels
        cs = s.shape_at(nl - 1)
        s.synth_level(nl - 1, M.capi.B, 3)
        s.coarse_solve()
        s.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            s.coarse_solve()
        s.synchronize()
        cs_ms = (time.perf_counter() - t0) / n * 1e3
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        s.vcycle()
        vc = s.bench_vcycle(5) / 5
        print(json.dumps({"shape": shape, "levels": nl, "coarsest": cs, "unknowns": int(
            cs[0] * cs[1] * cs[2]), "setup_s": round(setup_s, 2), "coarse_solve_ms": round(cs_ms, 3),
            "vcycle_ms": round(vc, 3)}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
