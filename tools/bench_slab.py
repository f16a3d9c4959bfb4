"""Compute-only proxy for one rank of the z-slab split: fused sweeps and V-cycles on a
512 x 512 x nz slab on one GPU (no exchange), for nz = 512 / N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    out = []
    for nz in [int(v) for v in (sys.argv[1:] or ["512", "256", "128", "64"])]:
        # a middle rank of the 512^3 split (ghost planes on both sides, no transport:
        # halos are skipped, the ghost planes hold zeros -- timing only)
        nr = 512 // nz
        s = M.Solver((nz, 512, 512), (1.0, 1.0, 1.0), time_step=0.1, smoother=M.GAUSS_SEIDEL,
                     cycle=M.SMOOTHER,
                     nranks=nr, rank=min(1, nr - 1), global_shape=(512, 512, 512))
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        s.bench_smooth(0, 3)
        tot, kern, n = s.bench_smooth(0, 20)
        out.append({"nz": nz, "ms_per_sweep": tot / 20, "kernel_ms": kern,
                    "gvox_s": 512 * 512 * nz / (tot / 20 * 1e-3) / 1e9,
                    "kernel": s.smooth_kernel_name(0)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
