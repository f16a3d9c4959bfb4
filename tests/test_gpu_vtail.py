"""The V-cycle tail (vtail_k): the replicated 3D levels of <= 32768 voxels and everything coarser run
in one workgroup instead of ~19 launches per level (per-colour GS passes, descent, prolongation,
coarsest solve).  It must equal the per-level launches (MAD_OPT_NO_VCYCLE_TAIL) BIT for bit --
same device functions, same order -- on every level, in fp32 and fp64, for every tensor kind and
centring mix, in V-cycles, FMG cycles and a whole mad_run, on one GPU and on rank slabs (where
the tail covers the replicated levels)."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def _cycles(shape, tensor, opts, precision, cycle, seed):
    import multigridanisotropicdiffusion_amd as M
    s = M.Solver(shape, time_step=0.3, precision=precision, options=opts)
    s.set_tensor(tensor)
    s.setup()
    s.upload(0, M.capi.X, synth.image(shape, seed=seed))
    s.upload(0, M.capi.B, synth.image(shape, seed=seed + 1))
    out = []
    for _ in range(2):
        (s.fmg if cycle == "fmg" else s.vcycle)()
        out.append([s.download(l, M.capi.X) for l in range(s.num_levels)])
    names = [s.smooth_kernel_name(l) for l in range(s.num_levels)]
    s.close()
    return out, names


@pytest.mark.parametrize("shape,kind", [((64, 64, 64), "full"), ((40, 52, 36), "full"),
                                        ((33, 47, 29), "diag"), ((48, 40, 44), "iso"),
                                        ((130, 70, 50), "full")])
@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("cycle", ["vcycle", "fmg"])
def test_tail_equals_per_level_launches(shape, kind, prec, cycle):
    import multigridanisotropicdiffusion_amd as M
    if kind == "full":
        T = synth.random_spd(shape, seed=5)
    elif kind == "diag":
        T = synth.random_spd(shape, seed=5, offdiag=False)
    else:
        T = synth.isotropic(shape, seed=5)
    precision = M.FP32 if prec == "fp32" else M.FP64
    a, _ = _cycles(shape, T, 0, precision, cycle, 7)
    b, _ = _cycles(shape, T, M.capi.OPT_NO_VCYCLE_TAIL, precision, cycle, 7)
    for q, (xa, xb) in enumerate(zip(a, b)):
        for l, (u, v) in enumerate(zip(xa, xb)):
            assert np.isfinite(u).all()
            np.testing.assert_array_equal(u, v, err_msg=f"cycle {q + 1}, level {l}")


def test_tail_whole_run_equals_per_level_launches():
    """mad_run (time steps, stopping loop, default precision = FP32_REFINE at 1e-10): same output,
    same cycle counts."""
    import multigridanisotropicdiffusion_amd as M
    shape = (72, 64, 56)
    T = synth.ved_form(shape, seed=3)
    img = synth.image(shape, seed=2).astype(np.float32)
    res = []
    for opts in (0, M.capi.OPT_NO_VCYCLE_TAIL):
        s = M.Solver(shape, time_step=0.5, number_of_steps=2, tolerance=1e-10, options=opts)
        s.set_tensor(T)
        s.setup()
        out, st = s.run(img)
        res.append((out, st["total_cycles"]))
        s.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]


@pytest.mark.parametrize("nranks", [2, 4])
def test_tail_on_rank_slabs(nranks):
    """Rank slabs: the tail covers the replicated levels (every rank the same bits)."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (128, 96, 80)
    outs = {}
    for opts in (0, M.capi.OPT_NO_VCYCLE_TAIL):
        def body(r, s):
            s.synth_tensor(kind=0, seed=4)
            s.setup()
            s.synth_level(0, M.capi.B, 3)
            s.synth_level(0, M.capi.X, 5)
            for _ in range(3):
                s.vcycle()
            return [s.download(l, M.capi.X) for l in range(s.num_levels)]
        outs[opts] = D.run_local(nranks, body, shape, time_step=0.2, precision=M.FP32, options=opts)
    for r in range(nranks):
        for l, (u, v) in enumerate(zip(outs[0][r], outs[M.capi.OPT_NO_VCYCLE_TAIL][r])):
            np.testing.assert_array_equal(u, v, err_msg=f"rank {r}, level {l}")
