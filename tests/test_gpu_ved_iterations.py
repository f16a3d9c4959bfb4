"""VED with Iterations >= 2 against the oracle.

With Iterations = n the reference's GenerateData (include/itkVEDMultigridImageFilter.hxx:104-128)
repeats, n times: the multiscale Hessian of the CURRENT (diffused) internal image, the
vesselness maxima over the scales, the tensor, and the diffusion step.  The maxima are reset
after each tensor (:121-123) so the next iteration's first scale starts them afresh
(`firstTime`, :221).  Here, on the reference's own volume (test_data/ved_test.mhd) with the
itkVEDTest_GS parameters (test/itkVEDTest_GS.cxx:61-92) except Iterations = 2:

* fp64, the reference's lexicographic GS (MAD_GAUSS_SEIDEL_LEX): the whole filter against
  oracle/ved_oracle.py:ved_run(iterations=2) -- the oracle's tensor from the oracle's own
  iteration-1 image -- to <= 1e-13 with the same total cycle count (V-cycles).
* fp64, the default multicolour GS: <= 1e-8 (a different, converged, smoother order).
* fp32: the diffusion against the oracle run on the GPU's own per-iteration tensors (the
  fp32 Hessian cannot resolve the argmax near-ties, tests/test_gpu_ved2_full.py), <= 1e-5;
  short output = truncation of the same values, |diff| <= 1.
* Iteration 2 is built from the diffused image with the maxima reset: one filter run with
  Iterations = 2 equals two chained runs with Iterations = 1 (the second fed the first's fp64
  output), bit for bit, and iteration 2's tensor differs from iteration 1's.
"""
import os

import numpy as np
import pytest

import ved_oracle as VO
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

KW = dict(alpha=0.5, beta=0.5, gamma=5.0, epsilon=0.01, sensitivity=10.0, omega=1.5,
          diffusion_iterations=4, diffusion_iterations_per_grid=3, time_step=0.1, tolerance=1e-10,
          scales=(0.300, 0.482, 0.775, 1.245, 2.000))


def relinf(a, ref):
    return np.abs(np.asarray(a, np.float64) - ref).max() / np.abs(ref).max()


@pytest.fixture(scope="module")
def M():
    import multigridanisotropicdiffusion_amd as mod
    return mod


@pytest.fixture(scope="module")
def ved_volume():
    from multigridanisotropicdiffusion_amd import mhd
    arr, info = mhd.read_mhd(os.path.join(GOLDEN, "ved_test.mhd"))
    return arr, tuple(info["spacing"])


@pytest.fixture(scope="module")
def oracle_two(oracle_mod, ved_volume):
    """ved_run with Iterations = 2 and the reference's lexicographic GS, V-cycles"""
    img, sp = ved_volume
    return VO.ved_run(img, sp, oracle_mod, iterations=2, cycle=oracle_mod.VCYCLE,
                      smoother=oracle_mod.GS_LEX, **KW)


def gpu_run(M, img, sp, iterations, precision, smoother, out_dtype=np.float64):
    v = M.VED(img.shape, sp, precision=getattr(M, precision), cycle=M.VCYCLE, smoother=smoother,
              iterations=iterations, **KW)
    try:
        return v.run(img, out_dtype=out_dtype)
    finally:
        v.close()


@pytest.mark.parametrize("smoother,bound,same_order", [("GAUSS_SEIDEL_LEX", 1e-13, True),
                                                        ("GAUSS_SEIDEL", 1e-8, False)])
def test_ved_two_iterations_fp64(M, oracle_two, ved_volume, smoother, bound, same_order):
    img, sp = ved_volume
    ref, steps = oracle_two
    assert len(steps) == 2
    ocycles = [sum(cyc) for cyc, _ in steps]
    out, st = gpu_run(M, img, sp, 2, "FP64", getattr(M, smoother))
    err = relinf(out, ref)
    print(f"VED Iterations=2 fp64 {smoother}: cycles {st['total_cycles']} (oracle {ocycles}), rel err {err:.2e}")
    assert st["iterations"] == 2 and st["converged"]
    if same_order:
        assert st["total_cycles"] == sum(ocycles), (st["total_cycles"], ocycles)
    assert err < bound
    # and iteration 2 did something: the two-iteration image is not the one-iteration image
    one, _ = gpu_run(M, img, sp, 1, "FP64", getattr(M, smoother))
    assert relinf(one, ref) > 100 * bound


def test_ved_two_iterations_fp32_on_gpu_tensors(M, oracle_mod, ved_volume):
    img, sp = ved_volume
    gs = M.GAUSS_SEIDEL
    out2, st2 = gpu_run(M, img, sp, 2, "FP32", gs)
    assert st2["iterations"] == 2
    # iteration by iteration: the GPU's tensor of the image that iteration starts from
    x1, _ = gpu_run(M, img, sp, 1, "FP32", gs)
    v = M.VED(img.shape, sp, precision=M.FP32, cycle=M.VCYCLE, smoother=gs, iterations=1, **KW)
    T1, _ = v.tensor(img)
    T2, _ = v.tensor(x1)
    v.close()
    # iteration 2's tensor is built from the diffused image (not the input's again)
    assert np.abs(T2 - T1).max() > 1e-3

    def diffuse(x, T):
        o = oracle_mod.Oracle(x.shape, sp, T, KW["time_step"])
        y, cyc, _ = o.run(np.asarray(x, np.float64), cycle=oracle_mod.VCYCLE, smoother=oracle_mod.GS_LEX,
                          iterations_per_grid=KW["diffusion_iterations_per_grid"], max_cycles=100,
                          number_of_steps=KW["diffusion_iterations"], tolerance=KW["tolerance"])
        assert all(c <= 100 for c in cyc)
        return y

    ref1 = diffuse(img, T1)
    e1 = relinf(x1, ref1)
    ref2 = diffuse(x1, T2)  # iteration 2 from the GPU's iteration-1 image, on the GPU's tensor
    e2 = relinf(out2, ref2)
    print(f"VED Iterations=2 fp32: iteration 1 rel err {e1:.2e}, iteration 2 rel err {e2:.2e}")
    assert e1 < 1e-5 and e2 < 1e-5
    out16, _ = gpu_run(M, img, sp, 2, "FP32", gs, out_dtype=np.int16)
    assert out16.dtype == np.int16
    assert np.abs(out16.astype(np.float64) - np.trunc(ref2)).max() <= 1


@pytest.mark.parametrize("precision", ["FP64", "FP32"])
def test_ved_iterations_chain_with_maxima_reset(M, ved_volume, precision):
    """Iterations = 2 == two chained Iterations = 1 runs (bitwise): iteration 2 starts from the
    diffused image and its scale maxima start afresh (VED.hxx:121-123, :221)."""
    img, sp = ved_volume
    two, _ = gpu_run(M, img, sp, 2, precision, M.GAUSS_SEIDEL)
    a, _ = gpu_run(M, img, sp, 1, precision, M.GAUSS_SEIDEL)
    b, _ = gpu_run(M, a, sp, 1, precision, M.GAUSS_SEIDEL)
    print(f"VED {precision}: Iterations=2 vs chained max|diff| {np.abs(two - b).max():.2e}")
    assert np.array_equal(two, b)
    assert not np.array_equal(two, a)
