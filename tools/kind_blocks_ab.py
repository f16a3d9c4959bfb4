"""Fused GS sweep and V-cycle at 512^3 for a synthetic tensor kind (0 VED-form full, 1 isotropic) and
precision, for an A/B of library builds (MAD_HIP_LIB).
    python tools/kind_blocks_ab.py KIND fp32|fp64"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    kind, prec = int(sys.argv[1]), sys.argv[2]
    S = 512
    P = M.FP32 if prec == "fp32" else M.FP64
    out = {"lib": os.path.basename(os.environ.get("MAD_HIP_LIB", "in-tree")), "kind": kind, "prec": prec}
    for cyc, key in ((M.SMOOTHER, "sweep"), (M.VCYCLE, "vcycle")):
        s = M.Solver((S, S, S), time_step=0.1, cycle=cyc, precision=P)
        s.synth_tensor(kind=kind, seed=4)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        if key == "sweep":
            s.bench_smooth(0, 3)
            dev, kern, _ = s.bench_smooth(0, 10)
            out["ms_per_sweep"] = round(dev / 10, 4)
            out["kernel"] = s.smooth_kernel_name(0)
        else:
            s.vcycle()
            s.vcycle()
            out["ms_per_vcycle"] = round(s.bench_vcycle(5) / 5, 3)
        s.close()
    print(out, flush=True)


if __name__ == "__main__":
    main()
