"""Per-launch durations of the bench sweep (mad_bench_launch_times): does the out-of-place
ping-pong (x -> t, t -> x) alternate fast and slow launches?
    python tools/launch_pattern.py [--sweeps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sweeps", type=int, default=20)
    p.add_argument("--size", type=int, default=512)
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    s.bench_smooth(0, 4)
    s.bench_smooth(0, a.sweeps)
    t = s.bench_launch_times()
    ev, od = t[0::2], t[1::2]
    print(json.dumps({"launch_ms": [round(v, 4) for v in t],
                      "even_mean": round(sum(ev) / len(ev), 4), "odd_mean": round(sum(od) / len(od), 4)}))


if __name__ == "__main__":
    main()
