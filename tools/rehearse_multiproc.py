"""Rehearse bench.py's multi-process start-up on a one-GPU box: two torchrun ranks,
the RCCL unique id broadcast over gloo, NCCL_SOCKET_IFNAME=lo bootstrap, then
mad_comm_init with both ranks on device 0.  RCCL refuses two ranks of one communicator
on one device ("Duplicate GPU"), so the expected outcome is that error from BOTH ranks
(the bootstrap reached the device check) -- anything else (a hang, a crash, a different
error) points at the start-up path the 8-GPU bench run relies on.
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29555 tools/rehearse_multiproc.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import multigridanisotropicdiffusion_amd as M
    S = 64
    s = M.Solver((S // world, S, S), (1.0, 1.0, 1.0), time_step=0.1, precision=M.FP32,
                 nranks=world, rank=rank, device=0, global_shape=(S, S, S))
    uid = M.comm_unique_id() if rank == 0 else bytes(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, src=0)
    out = {"rank": rank, "uid_nonzero": any(t.tolist())}
    try:
        s.comm_init(bytes(t.tolist()))
        out["comm_init"] = "ok"
    except Exception as e:  # noqa: BLE001 - reported
        out["comm_init"] = f"error: {e}"
    print(json.dumps(out), flush=True)
    dist.barrier()


if __name__ == "__main__":
    main()
