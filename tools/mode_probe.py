"""Does a level-0 allocation keep its sweep speed, and does the data matter?  One 512^3 SMOOTHER-layout
solver (placement tuning off): per-direction sweep ms (launches 0, 2, ... read x / write t; 1, 3, ... the
reverse) on the zero arrays setup leaves, after writing the bench's synthetic x and b, after zeroing them
again, and once more with data -- 8 launches per measurement after a 16-launch warm-up.
    python tools/mode_probe.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dirs(s):
    s.bench_smooth(0, 8)
    v = s.bench_launch_times()
    return round(sum(v[0::2]) / len(v[0::2]), 4), round(sum(v[1::2]) / len(v[1::2]), 4)


def main():
    import multigridanisotropicdiffusion_amd as M
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = M.Solver((512, 512, 512), (1.0, 1.0, 1.0), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER,
                 options=M.capi.OPT_NO_PLACEMENT_TUNE)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.bench_smooth(0, 16)
    out = []
    for _ in range(reps):
        out.append(("zero", dirs(s)))
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        out.append(("data", dirs(s)))
        s.fill(0, M.capi.X, 0.0)
        s.fill(0, M.capi.B, 0.0)
    print(json.dumps(out), flush=True)
    s.close()


if __name__ == "__main__":
    main()
