"""One rank of the multi-process RCCL parity test (tests/test_gpu_multiproc.py).

Started by tests/conftest.py (pytest_sessionstart) before the test process makes any GPU
call, one process per GPU (RANK / WORLD_SIZE / MASTER_PORT in the environment, device =
RANK).  Torch-free: ranks meet through distributed.bootstrap_node and exchange over RCCL.
The C4 workload at 512^3 in the production V-cycle layout: two level-0 sweeps, then three
V-cycles (the first eager, the later ones replaying the captured multi-rank hipGraph); the
rank's level-0 x after each stage goes to <outdir>/rank<r>.npz.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GSHAPE = (512, 512, 512)
VCYCLES = 3


def drive(s, M):
    """The sequence both transports run (the test replays it on the LOCAL transport)."""
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 5)
    s.smooth(0, 2)
    out = {"sweeps": s.download(0, M.capi.X).astype(np.float32)}
    for q in range(VCYCLES):
        s.vcycle()
        out[f"vcycle{q + 1}"] = s.download(0, M.capi.X).astype(np.float32)
    # graph replays back to back (no host synchronisation between them), as bench.py runs them:
    # each replay's eager entry work must not overtake the previous replay's RCCL operations
    s.bench_vcycle(3)
    out["vcycles_back_to_back"] = s.download(0, M.capi.X).astype(np.float32)
    return out


def variants(M):
    """(name, mad_desc.options) of the sequences every rank runs: the default exchange after
    each sweep (RCCL grouped send / recv), and the peer halo (edge planes stored by the sweep
    into the neighbours' IPC-mapped mailboxes)."""
    return [("default", 0), ("peer", M.capi.OPT_PEER_HALO)]


def make_solver(M, world, rank, device=-1, options=0):
    from multigridanisotropicdiffusion_amd import distributed as D
    z0, z1 = D.slabs(GSHAPE, world)[rank]
    return M.Solver((z1 - z0,) + GSHAPE[1:], time_step=0.1, precision=M.FP32, cycle=M.VCYCLE,
                    nranks=world, rank=rank, global_shape=GSHAPE, device=device, options=options)


def main():
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    outdir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # MAD_MP_DEVICE: the shared-device mode of tests/conftest.py (both ranks on GPU 0)
    device = int(os.environ.get("MAD_MP_DEVICE", rank))
    for name, opts in variants(M):
        s = make_solver(M, world, rank, device=device, options=opts)
        D.bootstrap_node(s, rank, world, tag=f"mp_parity_{name}")
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        out = drive(s, M)
        out["kernel"] = np.array(s.smooth_kernel_name(0))
        s.close()
        np.savez(os.path.join(outdir, f"rank{rank}_{name}.npz"), **out)
        print(f"rank {rank}/{world} {name}: done", flush=True)


if __name__ == "__main__":
    main()
