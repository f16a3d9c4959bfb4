"""A/B of the one-launch V-cycle tail (vtail_k) against the per-level launches (MAD_OPT_NO_VCYCLE_TAIL):
the bench workload's graph-replayed V-cycle (512^3 fp32 VED-form), alternated within one process, on one
GPU or as one interior rank of an N-rank z-slab decomposition alone on the device (the SOLO / RCCL-SOLO
proxy of tools/vcycle_trace.py).  One JSON line per configuration: per-rep ms per V-cycle for each form.
    python tools/tail_ab.py [--ranks 8 --rccl] [--reps 6] [--cycles 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--ranks", type=int, default=1)
    p.add_argument("--rccl", action="store_true")
    p.add_argument("--reps", type=int, default=6)
    p.add_argument("--cycles", type=int, default=20)
    p.add_argument("--nu", type=int, default=2)
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    S = a.size
    forms = {"tail": 0, "launches": M.capi.OPT_NO_VCYCLE_TAIL}
    sv = {}
    for name, opt in forms.items():
        if a.ranks > 1:
            r = a.ranks // 2
            z0, z1 = D.slabs((S, S, S), a.ranks)[r]
            s = M.Solver((z1 - z0, S, S), time_step=0.1, precision=M.FP32, nranks=a.ranks, rank=r,
                         global_shape=(S, S, S), options=opt, iterations_per_grid=a.nu)
            (s.comm_init_rccl_solo if a.rccl else s.comm_init_solo)()
        else:
            s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, options=opt, iterations_per_grid=a.nu)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        s.vcycle()
        s.vcycle()
        s.synchronize()
        tails = [s.vcycle_tail(l) for l in range(s.num_levels)]
        sv[name] = s
        print(json.dumps({"form": name, "tail_per_level": tails}), flush=True)
    for s in sv.values():
        s.bench_vcycle(40)  # settle the clocks
    res = {k: [] for k in forms}
    for _ in range(a.reps):
        for name, s in sv.items():
            res[name].append(round(s.bench_vcycle(a.cycles) / a.cycles, 4))
    best = {k: min(v) for k, v in res.items()}
    print(json.dumps({"size": S, "ranks": a.ranks, "rccl": a.rccl, "nu": a.nu, "ms_per_vcycle": res,
                      "best": best, "saved_ms": round(best["launches"] - best["tail"], 4)}), flush=True)


if __name__ == "__main__":
    main()
