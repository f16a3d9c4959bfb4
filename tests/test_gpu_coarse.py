"""Large coarsest levels (DirectSolver, include/mad/itkDirectSolver.hxx:32-147).

The reference LU-factors the coarsest operator with vnl_sparse_lu whatever its size
(DS.hxx:44, 81-86).  Thin volumes stop coarsening early (512x512x64 -> 64x64x8 = 32768
unknowns, 256x256x40 -> 64x64x10) and any axis < 12 leaves the whole grid to the direct
solver (maxDepth 0, include/mad/itkGridsHierarchy.hxx:36-59).  Above
mad_desc.coarse_dense_max unknowns the library solves them with the block-plane LU
(csrc/mad_coarse.hpp); the oracle uses a banded partial-pivot LU of the same operator
(oracle/mad_oracle.c band_factor), an independent exact solver, so agreement is to fp64
rounding of two different factorisations.
"""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def relmax(a, ref):
    return np.abs(a - ref).max() / np.abs(ref).max()


# (shape, block target): partial last block, one plane per block (chain only), 2D, and a
# small grid forced onto the block path next to its dense inverse
CASES = [
    ((9, 40, 30), 0, ""),       # q = 270 (x, z inside y), 7 planes per block, last block 5 planes
    ((9, 40, 30), 1, ""),       # one plane per block: 2 x 39 chained q x q products
    ((10, 1500), 0, ""),        # 2D: planes of 10, 204 per block
    ((10, 26, 50), 3000, ""),   # q = 260 (x outermost), 11 planes per block, 5 blocks
]


@pytest.mark.parametrize("shape,target,opts", CASES + [((9, 40, 30), 1, "no_chain")])
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_block_coarse_solve_matches_oracle(oracle_mod, shape, target, opts, prec):
    """opts "no_chain" (MAD_OPT_COARSE_NO_CHAIN): the one-plane blocks' chain steps multiply
    by Dinv_i after E_i y instead of by stored KL_i / KU_i (the low-memory form)."""
    import multigridanisotropicdiffusion_amd as M
    P = M.FP64 if prec == "fp64" else M.FP32
    sp = (1.0, 0.8, 1.3)[: len(shape)]
    T = synth.random_spd(shape, seed=31)
    s = M.Solver(shape, sp, time_step=3.0, precision=P, coarse_block_unknowns=target,
                 options=M.capi.OPT_COARSE_NO_CHAIN if opts == "no_chain" else 0)
    s.set_tensor(T)
    s.setup()
    assert s.num_levels == 1  # an axis < 12: the whole grid is the coarsest level
    b = synth.image(shape, seed=7)
    s.upload(0, M.capi.B, b)
    s.coarse_solve()
    got = s.download(0, M.capi.X)
    o = oracle_mod.Oracle(shape, sp, T, 3.0)
    ref = o.direct_solve(b)
    assert relmax(got, ref) < (1e-12 if P == M.FP64 else 2e-6)


def test_block_path_equals_dense_inverse():
    """The same 4800-unknown coarsest level through the dense inverse (default) and forced
    onto the block-plane LU (coarse_dense_max 1): both exact, equal to fp64 rounding."""
    import multigridanisotropicdiffusion_amd as M
    shape = (8, 24, 25)
    T = synth.random_spd(shape, seed=3)
    b = synth.image(shape, seed=4)
    out = []
    for dm in (0, 1):
        s = M.Solver(shape, time_step=2.0, precision=M.FP64, coarse_dense_max=dm)
        s.set_tensor(T)
        s.setup()
        s.upload(0, M.capi.B, b)
        s.coarse_solve()
        out.append(s.download(0, M.capi.X))
        s.close()
    assert relmax(out[1], out[0]) < 1e-12


@pytest.mark.timeout(600)
@pytest.mark.parametrize("shape,coarsest", [
    ((64, 512, 512), (8, 64, 64)),     # 32768 unknowns
    ((40, 256, 256), (10, 64, 64)),    # 40960 unknowns
])
def test_thin_volume_vcycle_matches_oracle(oracle_mod, shape, coarsest):
    """One V-cycle (nu = 2, 4-colour GS) of a thin VED-form volume whose coarsest level is
    beyond the dense inverse, against the oracle's V-cycle in the same colour order:
    fp64 <= 1e-10, fp32 <= 1e-5 (the north-star tolerance)."""
    import multigridanisotropicdiffusion_amd as M
    T = synth.ved_form(shape)
    x = synth.image(shape, seed=5)
    b = synth.image(shape, seed=3)
    got = {}
    for prec in (M.FP64, M.FP32):
        s = M.Solver(shape, time_step=0.5, precision=prec)
        s.set_tensor(T)
        s.setup()
        assert s.shape_at(s.num_levels - 1) == coarsest
        s.upload(0, M.capi.X, x)
        s.upload(0, M.capi.B, b)
        s.vcycle()
        got[prec] = s.download(0, M.capi.X)
        s.close()
    o = oracle_mod.Oracle(shape, (1.0, 1.0, 1.0), T, 0.5)
    del T
    assert o.shape_at(o.num_levels - 1) == coarsest
    ref = o.vcycle(x, b, smoother=oracle_mod.GS_COLOR, ncolors=4, iterations_per_grid=2)
    assert relmax(got[M.FP64], ref) < 1e-10
    assert relmax(got[M.FP32], ref) < 1e-5


@pytest.mark.timeout(900)
def test_depth0_volume_run_matches_oracle(oracle_mod):
    """130x130x10: maxDepth 0, the direct solver covers all 169000 unknowns (planes of 1300,
    one per block).  mad_run to the reference tests' 1e-10 with the default descriptor
    (MAD_PRECISION_AUTO -> FP32_REFINE) and in FP64, against the oracle's GenerateData."""
    import multigridanisotropicdiffusion_amd as M
    shape = (10, 130, 130)
    sp = (0.9, 1.0, 2.5)
    T = synth.random_spd(shape, seed=12)
    img = 100.0 * synth.image(shape, seed=8)
    o = oracle_mod.Oracle(shape, sp, T, 0.8)
    assert o.num_levels == 1
    ref, cyc, rr = o.run(img, tolerance=1e-10, number_of_steps=2)
    assert rr[-1] <= 1e-10
    for prec, tol in ((M.FP64, 1e-11), (M.PRECISION_AUTO, 1e-9)):
        s = M.Solver(shape, sp, time_step=0.8, tolerance=1e-10, number_of_steps=2, precision=prec)
        s.set_tensor(T)
        out, st = s.run(img, out_dtype=np.float64)
        assert st["num_levels"] == 1 and st["last_relres"] <= 1e-10, st
        assert relmax(out, ref) < tol, (prec, relmax(out, ref))
        s.close()


@pytest.mark.parametrize("nranks", [2, 4])
def test_thin_volume_rank_slabs_match_single(nranks):
    """Rank slabs (in-process transport) of a thin volume whose replicated coarsest level takes the
    block-plane LU (32 x 256 x 256 -> 8 x 64 x 64): every rank factors and solves it alike, so two
    V-cycles equal the one-GPU run bit for bit."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (32, 256, 256)
    T = synth.ved_form(shape)
    x = synth.image(shape, seed=1)
    b = synth.image(shape, seed=2)
    s = M.Solver(shape, time_step=0.5, precision=M.FP32)
    s.set_tensor(T)
    s.setup()
    assert s.shape_at(s.num_levels - 1) == (8, 64, 64)
    s.upload(0, M.capi.X, x)
    s.upload(0, M.capi.B, b)
    s.vcycle()
    s.vcycle()
    ref = s.download(0, M.capi.X)
    s.close()
    sl = D.slabs(shape, nranks)

    def body(r, s):
        z0, z1 = sl[r]
        s.set_tensor(T)
        s.setup()
        s.upload(0, M.capi.X, x[z0:z1])
        s.upload(0, M.capi.B, b[z0:z1])
        s.vcycle()
        s.vcycle()
        return s.download(0, M.capi.X)
    outs = D.run_local(nranks, body, shape, time_step=0.5, precision=M.FP32)
    np.testing.assert_array_equal(np.concatenate(outs), ref)


@pytest.mark.timeout(600)
def test_thin_volume_fmg_matches_oracle(oracle_mod):
    """FullMultiGrid (MAD.hxx:300-338) on a volume with a large coarsest level: the coarsest
    'V-cycles' of FMG are repeated direct solves, here the block-plane LU; fp64
    against the oracle's FMG (banded LU) in the same colour order."""
    import multigridanisotropicdiffusion_amd as M
    shape = (40, 256, 256)
    T = synth.ved_form(shape)
    b = synth.image(shape, seed=3)
    s = M.Solver(shape, time_step=0.5, precision=M.FP64)
    s.set_tensor(T)
    s.setup()
    s.upload(0, M.capi.B, b)
    s.fmg()
    got = s.download(0, M.capi.X)
    s.close()
    o = oracle_mod.Oracle(shape, (1.0, 1.0, 1.0), T, 0.5)
    ref = o.fmg(b, smoother=oracle_mod.GS_COLOR, ncolors=4, iterations_per_grid=2)
    assert relmax(got, ref) < 1e-10


@pytest.mark.timeout(300)
def test_ct_slab_whole_grid_direct_solve():
    """A realistic CT slab, 512 x 512 x 8 (an axis < 12: the whole 2.1 M-unknown grid is the
    direct solve, GH.hxx:36-59): planes of q = 4096 unknowns, one per block, whose KL / KU
    would not fit beside the 69 GB of Dinv blocks, so the chain runs through Dinv_i.  The
    oracle's band LU needs ~200 GB of host memory here, so the check is by property: the fp64
    solve's residual ||b - A x|| / ||b|| <= 1e-12 (measured 4e-16)."""
    import multigridanisotropicdiffusion_amd as M
    shape = (8, 512, 512)
    s = M.Solver(shape, time_step=0.1, precision=M.FP64)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    assert s.num_levels == 1
    s.synth_level(0, M.capi.B, 3)
    s.coarse_solve()
    assert s.residual(0) / s.norm(0, M.capi.B) <= 1e-12
    s.close()
