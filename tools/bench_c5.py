"""BASELINE config C5 on ONE MI355X: 1024 x 1024 x 512 (x, y, z) VED-form full tensor,
fp32, GS smoother -- level-0 sweep throughput and V-cycles/s of the whole volume on
one GPU (the config is quoted for 8 GPUs; this is the single-GPU reference point,
537 M voxels, ~45 GB of HBM)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    shape = (512, 1024, 1024)  # (z, y, x)
    s = M.Solver(shape, (1.0, 1.0, 1.0), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER)
    t0 = time.perf_counter()
    s.synth_tensor(kind=0, seed=5)
    s.setup()
    s.synth_level(0, M.capi.B, 5)
    s.synth_level(0, M.capi.X, 5)
    s.synchronize()
    setup_s = time.perf_counter() - t0
    s.bench_smooth(0, 3)
    tot, kern, n = s.bench_smooth(0, 10)
    s.vcycle()
    s.synchronize()
    t0 = time.perf_counter()
    vms = s.bench_vcycle(5)
    s.synchronize()
    vwall = (time.perf_counter() - t0) / 5
    nvox = float(shape[0] * shape[1] * shape[2])
    print(json.dumps({
        "workload": "C5 1024x1024x512 VED-form full tensor, GS, 1 GPU",
        "levels": s.num_levels, "setup_s": round(setup_s, 2),
        "sweep_ms": round(tot / 10, 3), "kernel_ms": round(kern, 3),
        "Mvoxel_smooths_per_s": round(nvox / (tot / 10 * 1e-3) / 1e6, 1),
        "hbm_frac_algorithmic": round(36.0 * nvox / (kern * 1e-3) / 8e12, 4),
        "ms_per_vcycle": round(vwall * 1e3, 2), "vcycles_per_s": round(1.0 / vwall, 2),
        "kernel": s.smooth_kernel_name(0)}), flush=True)


if __name__ == "__main__":
    main()
