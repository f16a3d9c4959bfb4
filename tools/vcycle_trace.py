"""Run V-cycles of the bench workload for a kernel trace (per-level breakdown).
    rocprofv3 --kernel-trace --output-format csv -d OUT -o vc -- python3 tools/vcycle_trace.py
then   python tools/vcycle_breakdown.py OUT/vc_kernel_trace.csv"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--cycles", type=int, default=10)
    p.add_argument("--layout", default="vcycle", choices=["vcycle", "smoother"],
                   help="solver CycleType: vcycle (production layout, dense rhs; bench.py's "
                        "V-cycles/s) or smoother (level-0 records carrying b)")
    p.add_argument("--ranks", type=int, default=1,
                   help="> 1: one interior rank (ranks // 2) of that z-slab decomposition alone "
                        "on the device (mad_comm_init_solo; timings, not results)")
    p.add_argument("--options", type=int, default=0, help="mad_desc.options (MAD_OPT_* bits)")
    p.add_argument("--rccl", action="store_true",
                   help="with --ranks: exchanges through RCCL (mad_comm_init_rccl_solo)")
    p.add_argument("--sweeps", type=int, default=0,
                   help="> 0: time that many level-0 sweeps instead of V-cycles")
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    S = a.size
    cyc = M.VCYCLE if a.layout == "vcycle" else M.SMOOTHER
    if a.ranks > 1:
        r = a.ranks // 2
        z0, z1 = D.slabs((S, S, S), a.ranks)[r]
        s = M.Solver((z1 - z0, S, S), time_step=0.1, precision=M.FP32, cycle=cyc, nranks=a.ranks,
                     rank=r, global_shape=(S, S, S), options=a.options)
        if a.rccl:
            s.comm_init_rccl_solo()
        else:
            s.comm_init_solo()
    else:
        s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, cycle=cyc, options=a.options)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    if a.sweeps:
        s.bench_smooth(0, 3)
        dev, kern, nl = s.bench_smooth(0, a.sweeps)
        print(f"ms_per_sweep {dev / a.sweeps:.4f} kernel_ms {kern:.4f} launches {nl}", flush=True)
        return
    s.vcycle()
    s.vcycle()  # (a rank slab's first cycle runs eagerly, the second is captured)
    s.synchronize()
    ms = s.bench_vcycle(a.cycles)
    print(f"ms_per_vcycle {ms / a.cycles:.3f}", flush=True)


if __name__ == "__main__":
    main()
