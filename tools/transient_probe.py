"""Is the level-0 sweep's slow phase after start-up a device state or a property of fresh allocations?
Solver A (512^3 SMOOTHER, no placement tuning) sweeps in windows of 100 launches for ~3 s; then solver
B (fresh arrays) is set up and swept at once, then A again.  If B starts slow while A is fast, the slow
phase belongs to new allocations; if B is as fast as A, it was the device warming up.
    python tools/transient_probe.py [--seconds 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=3.0)
    p.add_argument("--size", type=int, default=512)
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    t_start = time.perf_counter()

    def make():
        s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER,
                     options=M.capi.OPT_NO_PLACEMENT_TUNE)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        return s

    def windows(s, tag, seconds):
        out = []
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            s.bench_smooth(0, 100)
            ser = s.bench_launch_times()
            out.append((round(time.perf_counter() - t_start, 2), round(sum(ser[0::2]) / len(ser[0::2]), 4),
                        round(sum(ser[1::2]) / len(ser[1::2]), 4)))
        print(json.dumps({"phase": tag, "t_even_odd": out}), flush=True)

    A = make()
    windows(A, "A", a.seconds)
    B = make()
    windows(B, "B fresh", a.seconds)
    windows(A, "A again", 1.0)
    B.close()
    C = make()
    windows(C, "C fresh (after B freed)", a.seconds)


if __name__ == "__main__":
    main()
