"""Whole-grid direct solves of realistic CT slabs (any axis < 12 makes the whole grid the
coarsest level, GH.hxx:36-59): setup time, device memory of the block-plane LU, solve time
and the fp64 residual ||b - A x|| / ||b|| of x = A^-1 b (the oracle's band LU does not fit in
host memory at these sizes, so the check is by property).
    python tools/coarse_large.py [nz ...]       (default 8 10 11; volumes nz x 512 x 512)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    nzs = [int(a) for a in sys.argv[1:]] or [8, 10, 11]
    for nz in nzs:
        shape = (nz, 512, 512)
        t0 = time.perf_counter()
        s = M.Solver(shape, time_step=0.1, precision=M.FP64)
        s.synth_tensor(kind=0, seed=4)
        try:
            s.setup()
        except M.MadError as e:
            print(json.dumps({"shape": shape, "setup_error": str(e)}), flush=True)
            s.close()
            continue
        setup_s = time.perf_counter() - t0
        assert s.num_levels == 1
        s.synth_level(0, M.capi.B, 3)
        s.coarse_solve()
        s.synchronize()
        n = 5
        t0 = time.perf_counter()
        for _ in range(n):
            s.coarse_solve()
        s.synchronize()
        cs_ms = (time.perf_counter() - t0) / n * 1e3
        rel = s.residual(0) / s.norm(0, M.capi.B)
        print(json.dumps({"shape": shape, "unknowns": nz * 512 * 512, "plane_unknowns": nz * 512,
                          "setup_s": round(setup_s, 2), "coarse_solve_ms": round(cs_ms, 2),
                          "relres_fp64": rel}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
