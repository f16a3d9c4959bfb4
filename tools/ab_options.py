"""A/B of mad_desc.options bits on the bench sweep (512^3 SMOOTHER layout), the VCYCLE layout's
level-0 sweep and the V-cycle, alternated; per rep (sweep ms, VCYCLE-layout sweep ms, V-cycle ms): python tools/ab_options.py OPT_A OPT_B [--reps 4]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("a", type=int)
    p.add_argument("b", type=int)
    p.add_argument("--reps", type=int, default=4)
    p.add_argument("--size", type=int, default=512)
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    sv = {}
    for opt in (a.a, a.b):
        s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER, options=opt)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        v = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, cycle=M.VCYCLE, options=opt)
        v.synth_tensor(kind=0, seed=4)
        v.setup()
        v.synth_level(0, M.capi.B, 3)
        v.synth_level(0, M.capi.X, 3)
        v.vcycle()
        sv[opt] = (s, v)
    res = {a.a: [], a.b: []}
    for _ in range(a.reps):
        for opt in (a.a, a.b):
            s, v = sv[opt]
            s.bench_smooth(0, 3)
            _, k, _ = s.bench_smooth(0, 20)
            vc = v.bench_vcycle(10) / 10
            _, kv, _ = v.bench_smooth(0, 8)  # the production (VCYCLE) layout's level-0 sweep
            v.vcycle()
            res[opt].append((round(k, 4), round(kv, 4), round(vc, 3)))
    print(json.dumps({str(k): v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
