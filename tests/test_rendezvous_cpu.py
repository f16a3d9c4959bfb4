"""Torch-free rendezvous of bench.py's ranks (distributed.bootstrap_node), on CPU:
rank 0 publishes the RCCL unique id in a file keyed by the common launcher and
MASTER_PORT, the other ranks read the same 128 bytes, the file is removed."""
import multiprocessing as mp
import os

import pytest


def _rank(rank, world, q, bar):
    from multigridanisotropicdiffusion_amd import distributed as D

    class FakeSolver:
        def comm_init(self, uid):  # collective, like ncclCommInitRank
            q.put((rank, bytes(uid)))
            bar.wait(30)

    # the id is RCCL's on the GPU box; any 128 bytes exercise the file protocol here
    D.comm_unique_id = lambda: bytes((7 * i + 3) % 256 for i in range(128))
    D.bootstrap_node(FakeSolver(), rank, world, tag="cputest", timeout=30)


def test_bootstrap_node_file_rendezvous(monkeypatch):
    monkeypatch.setenv("MASTER_PORT", str(40000 + os.getpid() % 1000))
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    world = 3
    bar = ctx.Barrier(world)
    # non-zero ranks first: they must wait for rank 0's file
    ps = [ctx.Process(target=_rank, args=(r, world, q, bar)) for r in (2, 1, 0)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    got = dict(q.get(timeout=5) for _ in range(world))
    assert sorted(got) == [0, 1, 2]
    assert len(set(got.values())) == 1 and len(got[0]) == 128
    from multigridanisotropicdiffusion_amd import distributed as D
    assert not os.path.exists(D._rdzv_path("cputest").replace(str(os.getppid()), str(os.getpid())))
