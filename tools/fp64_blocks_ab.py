"""FP64 level-0 fused sweep and V-cycle at 512^3 (bench workload), for an A/B of library builds
(MAD_HIP_LIB): prints the device ms per sweep (SMOOTHER layout) and per V-cycle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    S = 512
    out = {"lib": os.path.basename(os.environ.get("MAD_HIP_LIB", "in-tree"))}
    for cyc, key in ((M.SMOOTHER, "sweep"), (M.VCYCLE, "vcycle")):
        s = M.Solver((S, S, S), time_step=0.1, cycle=cyc, precision=M.FP64)
        s.synth_tensor(kind=0, seed=4)
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
