"""z-slab decomposition at the full bench sizes (BASELINE.json C4 512^3 at 2 / 4 / 8
ranks, C5 1024 x 1024 x 512 at 8 ranks), rehearsed on one GPU with the in-process
transport (ranks as host threads; the RCCL path moves the same planes).

Two level-0 sweeps and one V-cycle on the rank slabs must equal the single-rank run
BIT for bit, with the default fused rank sweep (one launch, then the exchange) on the
64-plane slabs of the 8-rank C4 split, and with the split form (boundary + interior
launches, exchange overlapped: MAD_OPT_OVERLAP_RANK_SWEEP) on the 8-rank SMOOTHER case.  Inputs are generated on the device from
global coordinates (mad_bench_synth_tensor / mad_bench_synth_level), so every rank
builds the same operator the single-rank run builds.

Memory: a rank builds its operators from its own tensor slab (+ TENSOR_GHOST ghost planes
exchanged level by level; mad_setup is collective), so the ranks' setups run concurrently
and no global fp64 tensor (26 GB at C5) exists anywhere.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _drive(s, M):
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 5)
    s.smooth(0, 2)
    a = s.download(0, M.capi.X).astype(np.float32)
    s.vcycle()
    v = s.download(0, M.capi.X).astype(np.float32)
    return a, v


@pytest.mark.timeout(400)
@pytest.mark.parametrize("gshape,nranks,cycle,peer", [
    ((512, 512, 512), 2, 0, 0),
    ((512, 512, 512), 4, 0, 0),
    ((512, 512, 512), 8, 0, 0),
    ((512, 512, 512), 8, 2, 0),     # SMOOTHER layout (records carry b): the bench's sweep
    ((512, 1024, 1024), 8, 0, 0),   # C5
    # MAD_OPT_PEER_HALO: the fused sweeps store their edge planes into the neighbours' mailboxes
    ((512, 512, 512), 2, 0, 1),
    ((512, 512, 512), 4, 0, 1),
    ((512, 512, 512), 8, 0, 1),
    ((512, 512, 512), 8, 2, 1),
])
def test_full_size_slabs_bitwise(gshape, nranks, cycle, peer):
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    opts = M.capi.OPT_OVERLAP_RANK_SWEEP if cycle == 2 and not peer else 0
    if peer:
        opts |= M.capi.OPT_PEER_HALO
    kw = dict(time_step=0.1, precision=M.FP32, cycle=cycle, gs_kernel=0, options=opts)
    s = M.Solver(gshape, **kw)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    ref = _drive(s, M)
    nlev = s.num_levels
    s.close()

    def body(r, s):
        lo, hi = s.tensor_planes()
        z0, z1 = D.slabs(gshape, nranks)[r]
        assert (lo, hi) == (max(z0 - 8, 0), min(z1 + 8, gshape[0]))  # O(slab) tensor
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        assert s.num_levels == nlev
        return _drive(s, M), s.smooth_kernel_name(0)

    out = D.run_local(nranks, body, gshape, **kw)
    sl = D.slabs(gshape, nranks)
    for r, ((a, v), kname) in enumerate(out):
        assert ("peer halo" in kname) == bool(peer), kname
        z0, z1 = sl[r]
        assert z1 - z0 == gshape[0] // nranks
        np.testing.assert_array_equal(a, ref[0][z0:z1], err_msg=f"rank {r} sweeps ({kname})")
        np.testing.assert_array_equal(v, ref[1][z0:z1], err_msg=f"rank {r} V-cycle ({kname})")
