"""Proxy for the per-rank cost of the z-slab split on a one-GPU box: N ranks of the
512^3 volume run as threads of one process on one device (in-process transport,
real boundary/interior split and plane exchange).  Their kernels mostly serialise on
the GPU (each fused launch fills every CU), so wall / N approximates one rank's
sweep time on its own GPU, and 1-GPU time / (wall / N) the strong-scaling factor
the sweep alone allows (xGMI transfer time not included: the device copies of the
in-process transport stand in for it).

    python tools/bench_local_split.py [N ...]
    python tools/bench_local_split.py --solo [N ...]

--solo: one interior rank (N // 2) of the N-rank decomposition alone on the device
(mad_comm_init_solo: every exchange a device copy of the same bytes), its sweeps and
V-cycles timed on the device -- the V-cycle graph-replayed as on an RCCL rank -- so the
per-rank cost is measured directly instead of as wall / N of serialised ranks.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def solo(ns, msp=0, gsk=0, opts=0, rccl=False, msv=0):
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    S, sweeps, vcyc = 512, 20, 10
    ref = {}
    for n in ns:
        r = n // 2
        z0, z1 = D.slabs((S, S, S), n)[r]
        out = {"ranks": n, "rank": r, "slab": [z1 - z0, S, S], "min_slab_planes": msp, "min_slab_voxels": msv, "gs_kernel": gsk, "options": opts,
               "transport": "rccl-solo" if rccl else "solo",
               "distributed_levels": sum(p["distributed"] for p in D.plan((S, S, S), n, r, msp, msv))}
        for cyc, key in ((M.SMOOTHER, "sweep"), (M.VCYCLE, "vcycle")):
            kw = dict(nranks=n, rank=r, global_shape=(S, S, S), min_slab_planes=msp,
                      min_slab_voxels=msv) if n > 1 else {}
            s = M.Solver((z1 - z0, S, S), time_step=0.1, cycle=cyc, gs_kernel=gsk, options=opts, **kw)
            if n > 1:
                if rccl:
                    s.comm_init_rccl_solo()
                else:
                    s.comm_init_solo()
            s.synth_tensor(kind=0, seed=4)
            s.setup()
            s.synth_level(0, M.capi.B, 3)
            s.synth_level(0, M.capi.X, 3)
            if key == "sweep":
                s.bench_smooth(0, 3)
                dev, kern, _ = s.bench_smooth(0, sweeps)
                out["ms_per_sweep"] = dev / sweeps
            else:
                s.vcycle()
                s.vcycle()
                out["ms_per_vcycle"] = s.bench_vcycle(vcyc) / vcyc
            s.close()
        if n == 1:
            ref = dict(out)
        elif ref:
            out["sweep_speedup_vs_1"] = ref["ms_per_sweep"] / out["ms_per_sweep"]
            out["vcycle_speedup_vs_1"] = ref["ms_per_vcycle"] / out["ms_per_vcycle"]
        print(json.dumps(out), flush=True)


def main():
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    args = sys.argv[1:]
    msp = 0
    if "--msp" in args:  # mad_desc.min_slab_planes
        i = args.index("--msp")
        msp = int(args[i + 1])
        del args[i:i + 2]
    gsk = 0
    if "--gs-kernel" in args:  # mad_desc.gs_kernel
        i = args.index("--gs-kernel")
        gsk = int(args[i + 1])
        del args[i:i + 2]
    opts = 0
    if "--options" in args:  # mad_desc.options (MAD_OPT_* bits)
        i = args.index("--options")
        opts = int(args[i + 1])
        del args[i:i + 2]
    msv = 0
    if "--msv" in args:  # mad_desc.min_slab_voxels
        i = args.index("--msv")
        msv = int(args[i + 1])
        del args[i:i + 2]
    rccl = "--rccl" in args  # --solo through RCCL (mad_comm_init_rccl_solo)
    if rccl:
        args.remove("--rccl")
    if args and args[0] == "--solo":
        return solo([int(v) for v in (args[1:] or ["1", "2", "4", "8"])], msp, gsk, opts, rccl, msv)
    S, sweeps, vcyc = 512, 20, 3
    for n in [int(v) for v in (args or ["1", "2", "4", "8"])]:
        bar = threading.Barrier(n)
        res = {}

        # sweeps on the SMOOTHER layout (bench.py's headline), V-cycles on the VCYCLE layout
        # (bench.py's vcycles_per_s, the production solve)
        def sweep_body(r, s):
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
            res.setdefault(r, {}).update(sweep=time.perf_counter() - t0, kern=kern,
                                         shape=s.level_info(0)["shape"])

        def vcycle_body(r, s):
            s.synth_tensor(kind=0, seed=4)
            s.setup()
            s.synth_level(0, M.capi.B, 3)
            s.synth_level(0, M.capi.X, 3)
            s.vcycle()
            s.synchronize()
            bar.wait()
            t0 = time.perf_counter()
            for _ in range(vcyc):
                s.vcycle()
            s.synchronize()
            bar.wait()
            res.setdefault(r, {}).update(vcycle=time.perf_counter() - t0)

        for g, (body, cyc) in enumerate(((sweep_body, M.SMOOTHER), (vcycle_body, M.VCYCLE))):
            if n == 1:
                s = M.Solver((S, S, S), time_step=0.1, cycle=cyc)
                body(0, s)
                s.close()
            else:
                D.run_local(n, body, (S, S, S), group=1000 * (g + 1) + n, time_step=0.1, cycle=cyc)
        wall = max(v["sweep"] for v in res.values())
        vwall = max(v["vcycle"] for v in res.values())
        print(json.dumps({"ranks": n, "slab": list(res[0]["shape"]),
                          "wall_ms_per_sweep": wall / sweeps * 1e3,
                          "rank_equiv_ms_per_sweep": wall / sweeps * 1e3 / n,
                          "rank0_kernel_ms": res[0]["kern"],
                          "wall_ms_per_vcycle": vwall / vcyc * 1e3,
                          "rank_equiv_ms_per_vcycle": vwall / vcyc * 1e3 / n}), flush=True)


if __name__ == "__main__":
    main()
