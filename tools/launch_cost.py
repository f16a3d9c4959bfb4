"""Host cost of submitting one graph-replayed V-cycle (hipGraphLaunch of the captured cycle) against
its device time, untraced: is a rank's cycle host-bound?  Times the host call of mad_vcycle on an
idle device (queue empty: the submission itself) and back-to-back (steady state), and the device
time per cycle (bench_vcycle's events).
    python tools/launch_cost.py [--ranks 8] [--rccl]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--ranks", type=int, default=1)
    p.add_argument("--rccl", action="store_true")
    a = p.parse_args()
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    S = a.size
    if a.ranks > 1:
        r = a.ranks // 2
        z0, z1 = D.slabs((S, S, S), a.ranks)[r]
        s = M.Solver((z1 - z0, S, S), time_step=0.1, precision=M.FP32, nranks=a.ranks, rank=r,
                     global_shape=(S, S, S))
        s.comm_init_rccl_solo() if a.rccl else s.comm_init_solo()
    else:
        s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    for _ in range(3):
        s.vcycle()  # eager cycle, capture, replay
    s.synchronize()
    idle = []
    for _ in range(5):
        t0 = time.perf_counter()
        s.vcycle()
        idle.append((time.perf_counter() - t0) * 1e3)
        s.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        s.vcycle()
    host_b2b = (time.perf_counter() - t0) * 1e3 / n
    s.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / n
    dev = s.bench_vcycle(n) / n
    print(json.dumps({"ranks": a.ranks, "rccl": a.rccl, "submit_ms_idle": sorted(idle),
                      "submit_ms_back_to_back": round(host_b2b, 3), "wall_ms_per_cycle": round(wall, 3),
                      "device_ms_per_cycle": round(dev, 3)}), flush=True)


if __name__ == "__main__":
    main()
