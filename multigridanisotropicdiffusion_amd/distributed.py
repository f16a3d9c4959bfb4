"""z-slab multi-GPU helpers (one rank per GPU, RCCL over xGMI).

The decomposition itself lives in the C++ library (plan_geometry in
csrc/mad_solver.hip, transports in csrc/mad_comm.hpp).  This module only
bootstraps it:

* ``bootstrap_node(solver, rank, world, tag)`` -- torch-free rendezvous on one
  node: rank 0 creates the RCCL unique id and publishes it in a file keyed by the
  launcher (the parent process shared by all ranks under torch.distributed.run)
  and MASTER_PORT; the other ranks read it, then every rank joins.  Importing
  torch is then unnecessary -- torch bundles its own librccl.so.1 / HIP runtime,
  and a process that loads it first binds libmad_hip.so to that RCCL
  (mad_comm_init refuses a major.minor other than the headers').
* ``bootstrap_rccl(solver, dist)`` -- the same over an initialised
  torch.distributed process group (gloo is enough: 128 bytes, once).
* ``run_local(nranks, body)`` -- runs ``nranks`` ranks as host threads of this
  process on one device with the in-process transport (tests / rehearsal).
* ``slabs(global_shape, nranks)`` -- the level-0 slab of every rank, from the
  host-only planner (mad_plan_level).
"""
import ctypes
import os
import tempfile
import threading
import time
import zlib

from . import _capi as C
from .solver import Solver, comm_unique_id


def plan(global_shape, nranks=1, rank=0, min_slab_planes=0, min_slab_voxels=0):
    """Per-level plan of one rank: list of dicts(size (x,y,z), z0, z1, distributed)."""
    d = C.default_desc()
    d.min_slab_planes = int(min_slab_planes)
    d.min_slab_voxels = int(min_slab_voxels)
    dim = len(global_shape)
    d.dim = dim
    size = list(reversed(global_shape)) + [1] * (3 - dim)
    for q in range(3):
        d.size[q] = size[q]
    d.nranks, d.rank = nranks, rank
    L = C.load()
    out, l, nl = [], 0, 1
    while l < nl:
        n = (ctypes.c_int64 * 3)()
        z0, z1, dist = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        r = L.mad_plan_level(ctypes.byref(d), l, n, None, None, ctypes.byref(z0),
                             ctypes.byref(z1), ctypes.byref(dist))
        if r < 0:
            raise C.MadError(-r, L.mad_last_error(None).decode())
        nl = r
        out.append(dict(size=tuple(n), z0=z0.value, z1=z1.value, distributed=bool(dist.value)))
        l += 1
    return out


def slabs(global_shape, nranks):
    return [(p[0]["z0"], p[0]["z1"]) for p in (plan(global_shape, nranks, r) for r in range(nranks))]


def _rdzv_path(tag):
    """The id file of one communicator: keyed by the launcher shared by all ranks (parent
    pid), MASTER_PORT and, under torchrun, the elastic run id and restart count (so a
    restarted job never reads the id a dead rank 0 left behind)."""
    parts = [str(os.getppid()), os.environ.get("MASTER_PORT", "0")]
    for k in ("TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT"):
        if os.environ.get(k):
            parts.append(os.environ[k])
    key = "-".join(parts + [str(tag)])
    return os.path.join(tempfile.gettempdir(), f"mad_rccl_uid_{key}")


def bootstrap_node(solver, rank, world, tag="0", timeout=120.0):
    """Join the RCCL communicator of `world` ranks on this node without torch.

    `tag` must differ between the communicators one job creates.  Rank 0 writes
    the 128-byte unique id atomically (tmp file + rename); the others poll for it.
    ncclCommInitRank is collective, so once it returns on rank 0 every rank has
    read the id and rank 0 removes the file."""
    if world > 1 and not os.environ.get("MASTER_PORT"):
        # every rank must derive the same key; without the launcher's MASTER_PORT two
        # concurrent jobs under one parent could meet in the same file
        raise RuntimeError("bootstrap_node: MASTER_PORT is not set; launch the ranks with "
                           "torch.distributed.run (or export MASTER_PORT, identical on every rank)")
    if not 0 <= rank < world:
        raise ValueError(f"bootstrap_node: rank {rank} outside world {world}")
    path = _rdzv_path(tag)
    if rank == 0:
        uid = comm_unique_id()
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
    else:
        t0 = time.monotonic()
        while True:
            try:
                with open(path, "rb") as f:
                    uid = f.read()
                if len(uid) == 128:
                    break
            except FileNotFoundError:
                pass
            if time.monotonic() - t0 > timeout:
                raise TimeoutError(f"rank {rank}: no RCCL unique id at {path} after {timeout} s")
            time.sleep(0.01)
    solver.comm_init(uid)
    if rank == 0:
        try:
            os.remove(path)
        except FileNotFoundError:
            pass


def bootstrap_rccl(solver, dist):
    """Join the RCCL communicator; `dist` is an initialised torch.distributed."""
    import torch
    uid = comm_unique_id() if dist.get_rank() == 0 else bytes(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, src=0)
    solver.comm_init(bytes(t.tolist()))


def run_local(nranks, body, global_shape, group=None, **solver_kw):
    """Run body(rank, solver) on `nranks` host threads sharing one process (and
    device), each with its z-slab context joined to an in-process group.
    Returns the list of body results (rank order); re-raises the first error."""
    sl = slabs(global_shape, nranks)
    key = group if group is not None else zlib.crc32(repr((global_shape, nranks)).encode())
    results = [None] * nranks
    errors = []

    def worker(r):
        try:
            z0, z1 = sl[r]
            shape = (z1 - z0,) + tuple(global_shape[1:])
            s = Solver(shape, nranks=nranks, rank=r, global_shape=global_shape, **solver_kw)
            s.comm_init_local(key)
            results[r] = body(r, s)
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append((r, e))

    th = [threading.Thread(target=worker, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0][1]
    return results
