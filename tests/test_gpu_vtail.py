"""The V-cycle tail (vtail_k): the replicated 3D levels of <= 32768 voxels and everything coarser in ONE
launch of 16-64 workgroups that keep their planes' records, b and x in LDS, phases separated by
device-wide barriers, instead of ~19 launches per level (per-colour GS passes,
descent, prolongation, coarsest solve).  It must equal the per-level launches (MAD_OPT_NO_VCYCLE_TAIL)
BIT for bit -- same device functions, same order -- on every level, in fp32 and fp64, for every tensor
kind and centring mix, in V-cycles (eager and graph-replayed), FMG cycles and a whole mad_run, on one
GPU and on rank slabs (where the tail covers the replicated levels)."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def _tensor(shape, kind):
    if kind == "full":
        return synth.random_spd(shape, seed=5)
    if kind == "diag":
        return synth.random_spd(shape, seed=5, offdiag=False)
    return synth.isotropic(shape, seed=5)


def _cycles(shape, tensor, opts, precision, cycle, seed, nu=2, ncycles=2):
    import multigridanisotropicdiffusion_amd as M
    s = M.Solver(shape, time_step=0.3, precision=precision, options=opts, iterations_per_grid=nu)
    s.set_tensor(tensor)
    s.setup()
    tail = [s.vcycle_tail(l) for l in range(s.num_levels)]
    s.upload(0, M.capi.X, synth.image(shape, seed=seed))
    s.upload(0, M.capi.B, synth.image(shape, seed=seed + 1))
    out = []
    for _ in range(ncycles):
        (s.fmg if cycle == "fmg" else s.vcycle)()
        out.append([s.download(l, M.capi.X) for l in range(s.num_levels)])
    s.close()
    return out, tail


def _equal(a, b):
    for q, (xa, xb) in enumerate(zip(a, b)):
        for l, (u, v) in enumerate(zip(xa, xb)):
            assert np.isfinite(u).all()
            np.testing.assert_array_equal(u, v, err_msg=f"cycle {q + 1}, level {l}")


@pytest.mark.parametrize("shape,kind", [((64, 64, 64), "full"), ((40, 52, 36), "full"),
                                        ((33, 47, 29), "diag"), ((48, 40, 44), "iso"),
                                        ((130, 70, 50), "full")])
@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("cycle", ["vcycle", "fmg"])
def test_tail_equals_per_level_launches(shape, kind, prec, cycle):
    import multigridanisotropicdiffusion_amd as M
    T = _tensor(shape, kind)
    precision = M.FP32 if prec == "fp32" else M.FP64
    a, ta = _cycles(shape, T, 0, precision, cycle, 7, ncycles=3)
    b, tb = _cycles(shape, T, M.capi.OPT_NO_VCYCLE_TAIL, precision, cycle, 7, ncycles=3)
    print(f"{shape} {kind} {prec} {cycle}: tail per level {ta}")
    assert any(n > 0 for n, _ in ta), "the tail never engages"
    assert all(n == 0 for n, _ in tb)
    assert all(0 < lds <= 160 * 1024 for n, lds in ta if n)
    _equal(a, b)


@pytest.mark.parametrize("nu", [1, 3])
def test_tail_other_sweep_counts(nu):
    import multigridanisotropicdiffusion_amd as M
    shape = (64, 48, 56)
    T = _tensor(shape, "full")
    a, ta = _cycles(shape, T, 0, M.FP32, "vcycle", 11, nu=nu)
    b, _ = _cycles(shape, T, M.capi.OPT_NO_VCYCLE_TAIL, M.FP32, "vcycle", 11, nu=nu)
    assert any(n > 0 for n, _ in ta)
    _equal(a, b)


def test_tail_large_grid_graph_replay():
    """256^3 (7 levels: the tail from 32^3), enough V-cycles that the graph-replayed cycle runs, against
    the per-level launches; the tail's launch uses 16 workgroups there."""
    import multigridanisotropicdiffusion_amd as M
    shape = (256, 256, 256)
    res = []
    for opts in (0, M.capi.OPT_NO_VCYCLE_TAIL):
        s = M.Solver(shape, time_step=0.4, precision=M.FP32, options=opts)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 5)
        tails = [s.vcycle_tail(l) for l in range(s.num_levels)]
        for _ in range(6):
            s.vcycle()
        res.append(([s.download(l, M.capi.X) for l in range(s.num_levels)], tails))
        s.close()
    (xa, ta), (xb, tb) = res
    print("tail per level", ta)
    first = next(l for l, (n, _) in enumerate(ta) if n)
    assert first >= 1 and ta[first][0] == 16 and all(n == 0 for n, _ in tb)
    for l, (u, v) in enumerate(zip(xa, xb)):
        np.testing.assert_array_equal(u, v, err_msg=f"level {l}")


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


def test_tail_not_used_where_it_does_not_apply():
    import multigridanisotropicdiffusion_amd as M
    shape = (64, 64, 64)
    for kw in (dict(verbose=True), dict(smoother=M.WEIGHTED_JACOBI), dict(smoother=M.GAUSS_SEIDEL_LEX),
               dict(options=M.capi.OPT_NO_VCYCLE_TAIL)):
        s = M.Solver(shape, time_step=0.2, precision=M.FP64, **kw)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        assert all(s.vcycle_tail(l) == (0, 0) for l in range(s.num_levels)), kw
        s.close()


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
            tails = [s.vcycle_tail(l) for l in range(s.num_levels)]
            for _ in range(3):
                s.vcycle()
            return [s.download(l, M.capi.X) for l in range(s.num_levels)], tails
        outs[opts] = D.run_local(nranks, body, shape, time_step=0.2, precision=M.FP32, options=opts)
    for r in range(nranks):
        xa, ta = outs[0][r]
        xb, _ = outs[M.capi.OPT_NO_VCYCLE_TAIL][r]
        assert any(n > 0 for n, _ in ta)
        for l, (u, v) in enumerate(zip(xa, xb)):
            np.testing.assert_array_equal(u, v, err_msg=f"rank {r}, level {l}")
