"""Per-launch device times of consecutive level-0 sweeps (bench workload, SMOOTHER layout), in
launch order: is the spread between launches systematic (e.g. the x / t ping-pong) or noise?
    python tools/launch_spread.py [--sweeps 60] [--size 512]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sweeps", type=int, default=60)
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--cycle", default="smoother", choices=["smoother", "vcycle"])
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    S = a.size
    s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32,
                 cycle=M.SMOOTHER if a.cycle == "smoother" else M.VCYCLE)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    s.bench_smooth(0, 4)
    s.bench_smooth(0, a.sweeps)
    t = s.bench_launch_times()
    print("kernel", s.smooth_kernel_name(0))
    print("order  " + " ".join(f"{v:.3f}" for v in t))
    ev, od = t[0::2], t[1::2]
    print(f"even launches mean {sum(ev) / len(ev):.4f}  odd launches mean {sum(od) / len(od):.4f}")
    st = sorted(t)
    print(f"min {st[0]:.4f} median {st[len(st) // 2]:.4f} max {st[-1]:.4f}")
    s.close()


if __name__ == "__main__":
    main()
