"""Two RCCL ranks sharing one GPU (distinct NCCL_HOSTID: RCCL's socket transport) run the bench's
512^3 V-cycle sequence in a chosen form, printing a line per step -- to localise a multi-rank
RCCL mismatch on a one-GPU box.
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port P tools/rehearse_vcycles.py [--options N] [--sync] [--eager] [--cycles K]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--options", type=int, default=0)
    p.add_argument("--sync", action="store_true", help="synchronise after every V-cycle")
    p.add_argument("--eager", action="store_true", help="MAD_OPT_EAGER_RANK_VCYCLE")
    p.add_argument("--cycles", type=int, default=4)
    p.add_argument("--size", type=int, default=512)
    a = p.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["NCCL_HOSTID"] = f"mad-rehearse-rank{rank}"
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    S = a.size
    z0, z1 = D.slabs((S, S, S), world)[rank]
    opts = a.options | (M.capi.OPT_EAGER_RANK_VCYCLE if a.eager else 0)
    s = M.Solver((z1 - z0, S, S), time_step=0.1, precision=M.FP32, cycle=M.VCYCLE, nranks=world,
                 rank=rank, global_shape=(S, S, S), device=0, options=opts)
    t0 = time.perf_counter()

    def say(m):
        print(f"[rank {rank} +{time.perf_counter() - t0:6.2f}] {m}", flush=True)
    D.bootstrap_node(s, rank, world, tag="rehearse")
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    say("setup done")
    for q in range(a.cycles):
        s.vcycle()
        if a.sync:
            s.synchronize()
        say(f"V-cycle {q + 1} issued{' and synchronised' if a.sync else ''}")
    s.synchronize()
    say("all done")
    s.close()


if __name__ == "__main__":
    main()
