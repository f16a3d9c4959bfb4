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


def test_rendezvous_key_carries_the_elastic_restart(monkeypatch):
    """A torchrun restart keeps the agent pid and MASTER_PORT; the run id and restart count
    make the restarted ranks meet in a fresh file (a dead rank 0's id is never read)."""
    from multigridanisotropicdiffusion_amd import distributed as D
    monkeypatch.setenv("MASTER_PORT", "29555")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job7")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    first = D._rdzv_path("sweep")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    second = D._rdzv_path("sweep")
    assert first != second and "job7" in first
    assert D._rdzv_path("vcycle") != second


def test_bootstrap_node_fails_fast_without_launcher_env(monkeypatch):
    from multigridanisotropicdiffusion_amd import distributed as D
    monkeypatch.delenv("MASTER_PORT", raising=False)

    class Never:
        def comm_init(self, uid):
            raise AssertionError("must not get here")
    with pytest.raises(RuntimeError, match="MASTER_PORT"):
        D.bootstrap_node(Never(), 1, 2, tag="x", timeout=0.1)
    with pytest.raises(ValueError):
        monkeypatch.setenv("MASTER_PORT", "1")
        D.bootstrap_node(Never(), 3, 2, tag="x", timeout=0.1)
