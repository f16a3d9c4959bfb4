"""The reference's second test volume in full: test/test_data/ved_test_2 (134 x 140 x 119 int16,
spacing .330017; committed unchanged as tests/golden/ved_test_2.mhd / .zraw, input data).

Its hierarchy takes all four mixed centrings, CCV -> VCC -> CVC -> VCV (x, y, z;
include/mad/itkGridsHierarchy.hxx:84-97) -- the committed crop
(test_gpu_ved2.py) stops after CVC, so the VCV level (9 x 9 x 8) and its transfers are only
exercised here.  The whole VED filter with the itkVEDTest_GS parameters (test/itkVEDTest_GS.cxx:
50-99) runs against the oracle (oracle/ved_oracle.py tensor + oracle/mad_oracle.c solve) at test
time; the oracle takes ~80 s of host time for this volume, once per module.  Parity unpinned as
every oracle comparison here."""
import os

import numpy as np
import pytest

import ved_oracle as VO
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

KW = dict(alpha=0.5, beta=0.5, gamma=5.0, epsilon=0.01, sensitivity=10.0, omega=1.5,
          iterations=1, diffusion_iterations=4, diffusion_iterations_per_grid=3,
          time_step=0.1, tolerance=1e-10)
# (z, y, x) shapes and (x, y, z) centring letters of levels 1..4
LEVELS = [((60, 70, 67), "CCV"), ((30, 35, 34), "VCC"), ((15, 18, 17), "CVC"), ((8, 9, 9), "VCV")]


def relmax(a, ref):
    return np.abs(a - ref).max() / np.abs(ref).max()


@pytest.fixture(scope="module")
def M():
    import multigridanisotropicdiffusion_amd as M
    return M


@pytest.fixture(scope="module")
def volume():
    from multigridanisotropicdiffusion_amd import mhd
    arr, info = mhd.read_mhd(os.path.join(GOLDEN, "ved_test_2.mhd"))
    assert arr.shape == (119, 140, 134) and arr.dtype == np.int16
    return arr, tuple(info["spacing"])


@pytest.fixture(scope="module")
def ved_ref(oracle_mod, volume):
    img, sp = volume
    return VO.ved_run(img, sp, oracle_mod, **KW)


@pytest.mark.parametrize("precision,tol", [("FP32", 4 * np.finfo(np.float32).eps), ("FP64", 1e-14)])
def test_full_volume_hierarchy_and_transfers(M, oracle_mod, volume, precision, tol):
    """Level sizes and per-axis centrings (CCV, VCC, CVC, VCV) of the device hierarchy, and
    restriction / interpolation of random arrays on every level against the oracle
    (IGO.hxx:45-304), border rows included -- within the north-star bounds (1e-8 fp64, 1e-5
    fp32) by orders of magnitude: same taps, same order."""
    import synth
    img, sp = volume
    T = synth.ved_form(img.shape)
    s = M.Solver(img.shape, sp, time_step=0.1, precision=getattr(M, precision))
    s.set_tensor(T)
    s.setup()
    assert s.num_levels == 5
    for l, (shape, letters) in enumerate(LEVELS, start=1):
        info = s.level_info(l)
        assert info["shape"] == shape, l
        assert "".join("C" if c else "V" for c in info["centering"]) == letters, l
    o = oracle_mod.Oracle(img.shape, sp, T, 0.1)
    rng = np.random.default_rng(31)
    for l in range(s.num_levels - 1):
        fine = rng.standard_normal(s.shape_at(l))
        s.upload(l, M.capi.R, fine)
        s.restrict(l)
        assert relmax(s.download(l + 1, M.capi.B), o.restrict(l, fine)) < tol, l
        coarse = rng.standard_normal(s.shape_at(l + 1))
        s.upload(l + 1, M.capi.X, coarse)
        s.interpolate(l)
        assert relmax(s.download(l, M.capi.X), o.interpolate(l, coarse)) < tol, l
    s.close()


def _oracle_solve(oracle_mod, x, sp, T):
    """DiffusionStep of the oracle (lexicographic GS, the reference's loop) on a given tensor."""
    o = oracle_mod.Oracle(x.shape, sp, T, KW["time_step"])
    out, cycles, _ = o.run(x, cycle=oracle_mod.VCYCLE, smoother=oracle_mod.GS_LEX,
                           iterations_per_grid=KW["diffusion_iterations_per_grid"], max_cycles=100,
                           number_of_steps=KW["diffusion_iterations"], tolerance=KW["tolerance"])
    return out, cycles


@pytest.mark.timeout(400)
def test_ved_filter_full_volume_fp64(M, oracle_mod, volume, ved_ref):
    """The whole VED filter in fp64 against the oracle.

    - with the reference's smoother order (lexicographic GS, `MAD_GAUSS_SEIDEL_LEX`, hyperplane
      wavefronts; the oracle's GS_LEX): within 1e-8 end to end -- the tensor within 1e-6 of the
      oracle's (the GPU's cyclic Jacobi vs LAPACK's eigh; it moves the output by < 1e-13 here), the
      same cycles per step;
    - with the default multicolour GS (a different sweep order, so parity is at convergence): two
      solutions each converged to relres 1e-10 differ by 2.0e-8 (max-norm, relative) on this volume,
      held to 1e-7; cycle counts within one of the oracle's per step; the short output within one
      grey level of the truncated reference."""
    img, sp = volume
    x = img.astype(np.float64)
    ref, steps = ved_ref
    kw = dict(KW, smoother=M.GAUSS_SEIDEL_LEX)
    v = M.VED(img.shape, sp, precision=M.FP64, **kw)
    out, st = v.run(img, out_dtype=np.float64)
    assert st["last_relres"] <= 1e-10
    assert relmax(out, ref) < 1e-8
    assert st["total_cycles"] == sum(steps[0][0])
    p = dict(VO.DEFAULTS)
    p.update(KW)
    T, _ = v.tensor(img)
    Tr, _ = VO.ved_tensor(x, sp, p["scales"], p["alpha"], p["beta"], p["gamma"], p["epsilon"],
                          p["omega"], p["sensitivity"])
    assert np.abs(T - Tr).max() < 1e-6
    v.close()
    v = M.VED(img.shape, sp, precision=M.FP64, **KW)
    out, st = v.run(img, out_dtype=np.float64)
    assert st["last_relres"] <= 1e-10
    assert relmax(out, ref) < 1e-7
    assert abs(st["total_cycles"] - sum(steps[0][0])) <= len(steps[0][0])
    out16, _ = v.run(img, out_dtype=np.int16)
    assert np.abs(out16.astype(np.float64) - np.trunc(ref)).max() <= 1
    v.close()


@pytest.mark.timeout(400)
def test_ved_filter_full_volume_fp32(M, oracle_mod, volume, ved_ref):
    """fp32 storage: the tensor matches the oracle's within 1e-3 except at scale near-ties (the
    strict argmax over scales, VED.hxx:272, that an fp32 Hessian cannot resolve), and the
    diffusion -- the hot path, solved to the reference's 1e-10 by the default precision
    (MAD_PRECISION_AUTO -> FP32_REFINE) -- matches the oracle's solve of the GPU's own tensor
    within 1e-5."""
    img, sp = volume
    x = img.astype(np.float64)
    v = M.VED(img.shape, sp, **KW)  # precision AUTO: fp32 Hessian, fp32 + fp64 defect correction
    out, st = v.run(img, out_dtype=np.float64)
    assert st["last_relres"] <= 1e-10
    p = dict(VO.DEFAULTS)
    p.update(KW)
    T, _ = v.tensor(img)
    Tr, _ = VO.ved_tensor(x, sp, p["scales"], p["alpha"], p["beta"], p["gamma"], p["epsilon"],
                          p["omega"], p["sensitivity"])
    # every tensor mismatch above 1e-3 must sit on a scale near-tie (both directions valid):
    # the oracle's two best scales within 1e-5 relative, the accuracy of the fp32 vesselness
    # (exp terms of fp32 eigenvalues; measured here: voxel (94, 88, 118), scales 0.775 / 1.245
    # at 0.48292448 / 0.48292526, 1.6e-6 apart, the fp32 mode keeps 0.775, tools/debug_ved2_voxel.py)
    tie = VO.near_ties(x, sp, p["scales"], p["alpha"], p["beta"], p["gamma"], rel=1e-5)
    bad = np.abs(T - Tr).max(axis=0) > 1e-3
    assert not (bad & ~tie).any(), np.argwhere(bad & ~tie)[:5]
    assert tie.mean() < 1e-3
    ref32, _ = _oracle_solve(oracle_mod, x, sp, T)
    assert relmax(out, ref32) < 1e-5
    # and against the oracle's whole pipeline (its own fp64 tensor).  Where the fp32 tensor took the
    # other scale's direction at a near-tie the implicit diffusion spreads that valid difference
    # over its neighbourhood (dt / h^2 ~ 0.9 here), so the bound is on the distribution: 99.9 % of
    # the voxels within 1e-6 of max|ref|, fewer than 0.1 % above the north-star 1e-5, all below
    # 1e-2.  Measured (profiles/r04_ved2_fp32_pipeline.log): median 6.1e-10, 99 % 1.2e-8,
    # 99.9 % 1.8e-7, max 3.8e-3 next to the 1.6e-6 tie at (94, 88, 118).
    ref, _ = ved_ref
    err = np.abs(out - ref) / np.abs(ref).max()
    q = np.quantile(err, [0.5, 0.99, 0.999, 1.0])
    frac = (err > 1e-5).mean()
    print(f"fp32 VED vs the oracle's whole pipeline: median {q[0]:.2e}, 99% {q[1]:.2e}, "
          f"99.9% {q[2]:.2e}, max {q[3]:.2e}, above 1e-5: {frac:.2e} of the voxels "
          f"({int(tie.sum())} near-tie voxels)")
    assert q[2] < 1e-6 and frac < 1e-3 and q[3] < 1e-2
    v.close()
