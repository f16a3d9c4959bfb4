"""Oracle known-answer tests (CPU).  The reference has no golden vectors
(test/itk2DDiffusionTest_GS.cxx:151 returns EXIT_SUCCESS without checks), so
the oracle is pinned by analytic properties of the algorithm it restates
 and by regression against the committed fixtures."""
import numpy as np
import pytest

import mf_numpy as mf
import synth
from conftest import load_golden


@pytest.fixture(scope="module")
def O(oracle_mod):
    return oracle_mod


# App. C: depth table computed from include/mad/itkGridsHierarchy.hxx:36-59 (numpy shapes z,y,x)
@pytest.mark.parametrize("shape,depth", [
    ((512, 512), 6), ((256, 256), 5), ((128, 128, 128), 4), ((256, 256, 256), 5),
    ((512, 512, 512), 6), ((512, 1024, 1024), 6), ((69, 77, 69), 3), ((119, 140, 134), 4),
    ((10, 40, 40), 0), ((11, 40, 40), 1), ((12, 12, 12), 1), ((3, 3, 3), 0), ((23, 24, 24), 2),
])
def test_depth_table(O, shape, depth):
    assert O.max_depth(shape) == depth


def test_ved_hierarchy_centering(O):
    o = O.Oracle((69, 77, 69), (0.3125, 0.3125, 0.5), synth.constant((69, 77, 69), [1, 0, 0, 1, 0, 1]), 0.1)
    shapes = [lv["shape"] for lv in o.levels]
    cents = [lv["centering"] for lv in o.levels]
    assert shapes == [(69, 77, 69), (35, 39, 35), (18, 20, 18), (9, 10, 9)]
    assert cents[1] == [0, 0, 0] and cents[2] == [0, 0, 0] and cents[3] == [1, 1, 1]
    assert o.levels[3]["spacing"] == [0.3125 * 8, 0.3125 * 8, 0.5 * 8]


CASES = [
    ((13, 17, 11), (0.7, 1.0, 1.3), 7, True),
    ((24, 26, 28), (1.0, 0.9, 1.2), 15, True),
    ((16, 14, 18), (1.0, 1.0, 1.0), 13, False),
    ((24, 18), (1.0, 0.5), 3, True),
    ((48, 40), (1.0, 1.0), 17, True),
]


@pytest.mark.parametrize("shape,spacing,seed,offdiag", CASES)
def test_row_sums_and_matrix_free(O, shape, spacing, seed, offdiag):
    """A 1 = 1 on every level (App. B.1) and the matrix-free operator the kernels
    evaluate equals the DCA stencil on every level."""
    T = synth.random_spd(shape, seed=seed, offdiag=offdiag)
    dt = 0.4
    o = O.Oracle(shape, spacing, T, dt)
    Tl = T
    rng = np.random.default_rng(seed)
    for l in range(o.num_levels):
        A = o.stencil(l)
        assert np.abs(A.sum(axis=1) - 1.0).max() < 1e-13
        if len(shape) == 3:  # 3D: the 8 corners are identically zero (GH.hxx:632-653)
            for i in (0, 2, 6, 8, 18, 20, 24, 26):
                assert np.all(A[:, i] == 0.0)
        if l > 0:
            Tl = np.stack([o.restrict(l - 1, Tl[c]) for c in range(Tl.shape[0])])
        h = o.levels[l]["spacing"]
        co = mf.coefficients(Tl, h, dt)
        x = rng.random(o.shape_at(l))
        b = rng.random(o.shape_at(l))
        r = o.residual(l, x, b)
        r2 = b - mf.apply(x, co)
        assert np.abs(r - r2).max() <= 1e-13 * max(1.0, np.abs(r).max())


def test_dt_zero_identity(O):
    shape = (12, 14, 13)
    T = synth.random_spd(shape, seed=1)
    o = O.Oracle(shape, (1, 1, 1), T, 0.0)
    A = o.stencil(0)
    e = np.zeros(27)
    e[13] = 1.0
    assert np.all(A == e)
    x = np.random.default_rng(0).random(shape)
    out, cyc, rr = o.run(x, tolerance=1e-12)
    assert np.array_equal(out, x) and cyc == [1]


@pytest.mark.parametrize("shape", [(24, 18), (25, 19), (16, 16, 16), (13, 17, 11), (12, 14, 13)])
def test_transfers_preserve_constants(O, shape):
    """R(1) = 1 and P(1) = 1 for vertex and cell centring (App. B.3)."""
    o = O.Oracle(shape, [1.0] * len(shape), synth.random_spd(shape, seed=2), 0.1)
    ones_f = np.ones(shape)
    ones_c = np.ones(o.shape_at(1))
    assert np.abs(o.restrict(0, ones_f) - 1).max() < 1e-15
    assert np.abs(o.interpolate(0, ones_c) - 1).max() < 1e-15


def _matrix(f, n_in, shape_in):
    cols = []
    for k in range(n_in):
        e = np.zeros(n_in)
        e[k] = 1.0
        cols.append(f(e.reshape(shape_in)).ravel())
    return np.stack(cols, axis=1)


def test_cell_restriction_is_scaled_transpose(O):
    """Cell centring: R = P^T / 2^D, boundaries included."""
    shape = (12, 16)  # even -> cell-centred in both axes
    o = O.Oracle(shape, (1, 1), synth.random_spd(shape, seed=4), 0.1)
    cs = o.shape_at(1)
    R = _matrix(lambda v: o.restrict(0, v), int(np.prod(shape)), shape)
    P = _matrix(lambda v: o.interpolate(0, v), int(np.prod(cs)), cs)
    assert np.abs(R - P.T / 4.0).max() < 1e-15


def test_exact_solution_is_fixed_point(O):
    """If A x = b exactly, one GS or WJ sweep leaves x unchanged (App. B.4)."""
    shape = (10, 11, 9)  # every axis < 12 -> maxDepth 0: the direct solver covers the grid
    o = O.Oracle(shape, (1, 1, 1), synth.random_spd(shape, seed=5), 0.7)
    assert o.num_levels == 1
    b = np.random.default_rng(3).random(shape)
    x = o.direct_solve(b)
    assert np.abs(o.residual(0, x, b)).max() < 1e-13
    assert np.abs(o.gs_lex(0, x, b) - x).max() < 1e-13
    assert np.abs(o.wj(0, x, b) - x).max() < 1e-13
    assert np.abs(o.gs_color(0, x, b) - x).max() < 1e-13


@pytest.mark.parametrize("cycle", [0, 1, 2])
def test_constant_input_stays_constant(O, cycle):
    shape = (16, 18, 20)
    o = O.Oracle(shape, (1, 1, 1), synth.random_spd(shape, seed=6), 0.5)
    x = np.full(shape, 3.25)
    out, cyc, rr = o.run(x, cycle=cycle, tolerance=1e-12, max_cycles=5)
    assert np.abs(out - 3.25).max() < 1e-12


def test_mirror_symmetry(O):
    """Flipping x with an x-mirror-symmetric tensor (M_xy = M_xz = 0) flips the
    converged solution (App. B.6)."""
    shape = (14, 16, 18)
    T = synth.random_spd(shape, seed=8, offdiag=False)
    T = 0.5 * (T + T[..., ::-1])
    o = O.Oracle(shape, (1, 1, 1), T, 0.6)
    x = np.random.default_rng(9).random(shape)
    a, _, _ = o.run(x, tolerance=1e-13)
    b, _, _ = o.run(np.ascontiguousarray(x[..., ::-1]), tolerance=1e-13)
    assert np.abs(a[..., ::-1] - b).max() < 1e-11


def test_lex_gs_is_order_dependent_but_colour_gs_converges_to_same(O):
    """Multicolour GS (GPU smoother) and lexicographic GS (reference) share the fixed
    point: converged solutions agree to solver tolerance."""
    shape = (24, 26, 28)
    o = O.Oracle(shape, (1.0, 0.9, 1.2), synth.random_spd(shape, seed=15), 0.6)
    x = np.random.default_rng(10).random(shape)
    a, _, _ = o.run(x, tolerance=1e-12, smoother=O.GS_LEX)
    b, _, _ = o.run(x, tolerance=1e-12, smoother=O.GS_COLOR)
    c, _, _ = o.run(x, tolerance=1e-12, smoother=O.WJ)
    one_sweep_diff = np.abs(o.gs_lex(0, x, x) - o.gs_color(0, x, x)).max()
    assert one_sweep_diff > 1e-3
    assert np.abs(a - b).max() < 1e-10 * np.abs(a).max()
    assert np.abs(a - c).max() < 1e-10 * np.abs(a).max()


KERNEL_FIXTURES = ["k2d_cell", "k2d_vert", "k3d_vert", "k3d_cell", "k3d_mixed", "k3d_diag",
                   "k3d_iso", "k3d_deep", "k2d_deep"]


@pytest.mark.parametrize("name", KERNEL_FIXTURES)
def test_oracle_matches_golden(O, name):
    """Regression pin of the oracle itself against the committed fixtures."""
    g = load_golden(name)
    shape = tuple(int(s) for s in g["shape"])
    o = O.Oracle(shape, tuple(g["spacing"]), g["tensor"], float(g["dt"]))
    diag = name.endswith("diag") or name.endswith("iso")
    x, b = g["x"], g["b"]
    np.testing.assert_allclose(o.wj(0, x, b), g["wj"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(o.residual(0, x, b), g["residual"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(o.gs_lex(0, x, b), g["gs_lex"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(o.gs_color(0, x, b, ncolors=2 if diag else 4), g["gs_color"],
                               rtol=0, atol=1e-14)
    np.testing.assert_allclose(o.vcycle(x, b, smoother=O.WJ), g["vcycle_wj"], rtol=0, atol=1e-13)


def test_c1_lena_converges(O):
    """itk2DDiffusionTest_{GS,WJ} parameters: both smoothers and both cycles converge to
    the same solution (tolerance 1e-10, test/itk2DDiffusionTest_GS.cxx:88-97)."""
    g = load_golden("lena_c1")
    ref = g["gs_v"].astype(np.float64)
    for k in ("wj_v", "wj_fmg", "gs_fmg"):
        assert np.abs(g[k] - ref).max() < 1e-3  # float32-stored outputs of 0..255 images
    assert int(g["gs_v_cycles"][0]) < int(g["wj_v_cycles"][0])


@pytest.mark.parametrize("nthreads", [1, 3])
def test_openmp_colour_sweep_equals_serial(oracle_mod, nthreads):
    """ora_gs_color_omp (bench.py's parallel CPU baseline) is the serial multicolour sweep."""
    import synth
    for shape, T, nc in [((14, 16, 18), synth.random_spd((14, 16, 18), seed=2), 4),
                         ((14, 16, 18), synth.random_spd((14, 16, 18), seed=2, offdiag=False), 2),
                         ((18, 20), synth.random_spd((18, 20), seed=2), 4)]:
        o = oracle_mod.Oracle(shape, (1.0,) * len(shape), T, 0.3)
        b = synth.image(shape, seed=3)
        np.testing.assert_array_equal(o.gs_color(0, b, b, nc), o.gs_color_omp(0, b, b, nc, nthreads))


def _assembled(o, l):
    """Dense A of level l from the oracle's 27-point stencils (DS.hxx:32-88 assembly)."""
    shape = o.shape_at(l)
    n = list(reversed(shape)) + [1] * (3 - len(shape))
    N = int(np.prod(shape))
    S = o.stencil(l)
    A = np.zeros((N, N))
    for p in range(N):
        i, j, k = p % n[0], (p // n[0]) % n[1], p // (n[0] * n[1])
        for s in range(27):
            if S[p, s] == 0.0:
                continue
            q = (i + s % 3 - 1, j + (s // 3) % 3 - 1, k + s // 9 - 1)
            A[p, q[0] + n[0] * (q[1] + n[1] * q[2])] += S[p, s]
    return A


@pytest.mark.parametrize("shape,spacing", [
    ((10, 22, 24), (1.0, 0.9, 1.2)),   # maxDepth 0, 5280 unknowns: the banded LU
    ((26, 9, 21), (0.8, 1.0, 1.1)),    # short y axis innermost, x / z outer
    ((10, 520), (1.0, 0.7)),           # 2D, 5200 unknowns
])
def test_banded_direct_solve_is_exact(O, shape, spacing):
    """Above 4096 unknowns the oracle's DirectSolver (DS.hxx:32-147) is a banded partial-pivot
    LU of the renumbered operator (shortest axis innermost, LAPACK gbtrf/gbtrs restated); it
    solves A x = b to fp64 rounding like vnl_sparse_lu and numpy's dense LU."""
    o = O.Oracle(shape, spacing, synth.random_spd(shape, seed=21), 2.0)
    assert o.num_levels == 1 and int(np.prod(shape)) > 4096
    b = np.random.default_rng(4).random(shape)
    x = o.direct_solve(b)
    assert np.abs(o.residual(0, x, b)).max() < 1e-12 * np.abs(b).max()
    ref = np.linalg.solve(_assembled(o, 0), b.ravel()).reshape(shape)
    assert np.abs(x - ref).max() < 1e-11 * np.abs(ref).max()
