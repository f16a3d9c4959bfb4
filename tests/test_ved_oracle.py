"""VED oracle (oracle/ved_oracle.py) and MetaImage I/O, CPU only.

The Hessian stage is parity-unpinned (ITK's recursive Gaussian is not available);
the restatement is pinned by known answers instead: the recursive filters (ITK's
RecursiveGaussianImageFilter algorithm, the default operator) keep constants, have
slope 1 on ramps and curvature 1 on t^2/2, and their impulse responses are the
Gaussian and its first / second derivatives to the accuracy of Deriche's 4th-order
fit; the FIR kernels are exact on quadratics; the scale-normalised Hessian of a
quadratic image is sigma^2 times its analytic Hessian away from the borders (both
operators; the recursive one's border transient decays as exp(-1.37 t / sigma)),
a bright tube gives a
positive vesselness with its axis as the omega direction, the tensor is
identity where the response vanishes and has eigenvalues {a, a, c} elsewhere
(VED.hxx:327-365).  The MHD reader is checked on the reference's own test volume
(tests/golden/ved_test.mhd, copied data) against the crop fixture."""
import os

import numpy as np
import pytest

import ved_oracle as V
from conftest import GOLDEN
from multigridanisotropicdiffusion_amd import mhd


@pytest.mark.parametrize("sigma,h", [(0.3, 0.3125), (0.482, 1.0), (2.0, 0.5), (1.245, 0.33)])
def test_kernels_are_exact_on_quadratics(sigma, h):
    K0, K1, K2 = V.gauss_kernels(sigma, h)
    R = V.kernel_radius(sigma, h)
    t = np.arange(-R, R + 1, dtype=np.float64)
    assert len(K0) == 2 * R + 1 and R == max(1, int(np.ceil(4 * sigma / h)))
    assert abs(K0.sum() - 1) < 1e-14 and abs((K0 * t).sum()) < 1e-14
    assert abs(K1.sum()) < 1e-14 and abs((K1 * t).sum() - 1) < 1e-14
    assert abs((K1 * t * t).sum()) < 1e-13
    assert abs(K2.sum()) < 1e-13 and abs((K2 * t).sum()) < 1e-13
    assert abs((K2 * t * t).sum() / 2 - 1) < 1e-13
    np.testing.assert_allclose(K0, K0[::-1], rtol=0, atol=1e-17)
    np.testing.assert_allclose(K1, -K1[::-1], rtol=0, atol=1e-17)


@pytest.mark.parametrize("kind,shape,margin,atol", [("fir", (30, 34, 38), 4, 1e-9),
                                                     ("recursive", (64, 66, 72), 12, 1e-5)])
def test_hessian_of_a_quadratic(kind, shape, margin, atol):
    sp = (0.5, 0.75, 1.0)  # hx, hy, hz
    z, y, x = np.meshgrid(*[np.arange(n, dtype=np.float64) for n in shape], indexing="ij")
    X, Y, Z = x * sp[0], y * sp[1], z * sp[2]
    c = dict(xx=0.3, yy=-0.7, zz=1.1, xy=0.4, xz=-0.25, yz=0.6)
    f = (c["xx"] * X * X + c["yy"] * Y * Y + c["zz"] * Z * Z + c["xy"] * X * Y
         + c["xz"] * X * Z + c["yz"] * Y * Z + 2 * X - Y + 5)
    sigma = 1.2
    H = V.hessian(f, sp, sigma, kind)
    R = [max(1, int(np.ceil(margin * sigma / h))) for h in sp]
    inner = (slice(R[2], -R[2]), slice(R[1], -R[1]), slice(R[0], -R[0]))
    want = [2 * c["xx"], c["xy"], c["xz"], 2 * c["yy"], c["yz"], 2 * c["zz"]]
    for q in range(6):
        np.testing.assert_allclose(H[inner + (q,)], sigma * sigma * want[q], rtol=0, atol=atol)


@pytest.mark.parametrize("sd", [0.96, 1.5, 2.49, 4.0, 6.4])
def test_recursive_gaussian_known_answers(sd):
    """ITK RecursiveGaussianImageFilter restated (Deriche 4th order): normalisation and
    impulse responses.  sd is sigma in voxels (the VED scales / spacings give 0.6 .. 6.4)."""
    n = 400
    c0, c1, c2 = (V.recursive_coefficients(sd, o) for o in range(3))
    t = np.arange(n) - n // 2.0
    inner = slice(int(20 * sd), n - int(20 * sd))  # border transients ~exp(-1.37 t / sd)
    # constants kept exactly (initial states assume the end values extend to infinity)
    np.testing.assert_allclose(V.recursive_filter(np.full(n, 3.0), c0, 0), 3.0, rtol=1e-13)
    assert np.abs(V.recursive_filter(np.full(n, 3.0), c1, 0)).max() < 1e-12
    assert np.abs(V.recursive_filter(np.full(n, 3.0), c2, 0)).max() < 1e-12
    # slope 1 on a ramp, curvature 1 on t^2 / 2, zero-order keeps lines (interior)
    np.testing.assert_allclose(V.recursive_filter(t, c1, 0)[inner], 1.0, atol=1e-9)
    np.testing.assert_allclose(V.recursive_filter(0.5 * t * t, c2, 0)[inner], 1.0, atol=1e-7)
    np.testing.assert_allclose(V.recursive_filter(t, c0, 0)[inner], t[inner], atol=1e-8)
    # impulse responses vs the sampled Gaussian and its derivatives, to the accuracy of
    # Deriche's 4th-order fit (measured: 0.3 % of the peak for the Gaussian, 1.1-1.4 % for
    # the derivatives)
    imp = np.zeros(n)
    imp[n // 2] = 1.0
    g = np.exp(-t * t / (2 * sd * sd)) / (np.sqrt(2 * np.pi) * sd)
    for c, ref, tol in ((c0, g, 5e-3), (c1, -t / sd ** 2 * g, 2e-2), (c2, (t * t - sd * sd) / sd ** 4 * g, 2e-2)):
        r = V.recursive_filter(imp, c, 0)
        assert np.abs(r - ref).max() < tol * np.abs(ref).max(), np.abs(r - ref).max() / np.abs(ref).max()
    assert abs(V.recursive_filter(imp, c0, 0).sum() - 1.0) < 1e-12


def tube(shape, r=2.5, axis_yx=(15.0, 17.0)):
    z, y, x = np.meshgrid(*[np.arange(n, dtype=np.float64) for n in shape], indexing="ij")
    d2 = (y - axis_yx[0]) ** 2 + (x - axis_yx[1]) ** 2
    return 200.0 * np.exp(-d2 / (2 * r * r))


def test_bright_tube_is_a_vessel_along_its_axis():
    img = tube((24, 30, 34))
    T, resp = V.ved_tensor(img, (1.0, 1.0, 1.0), scales=(1.0, 2.0, 3.0), omega=1.5)
    c = (12, 15, 17)
    assert resp[c] > 0.3
    # tensor on the axis: eigenvector of the largest eigenvalue (omega branch) is z
    M = np.array([[T[0][c], T[1][c], T[2][c]], [T[1][c], T[3][c], T[4][c]],
                  [T[2][c], T[4][c], T[5][c]]])
    w, v = np.linalg.eigh(M)
    Vv = resp[c] ** 0.1
    np.testing.assert_allclose(w, sorted([1 + (0.01 - 1) * Vv] * 2 + [1 + (1.5 - 1) * Vv]), atol=1e-12)
    assert abs(abs(v[2, 2]) - 1) < 1e-6  # z component (x, y, z order) of the omega direction
    # far from the tube: flat background, no response, identity tensor
    far = (12, 2, 2)
    assert resp[far] == 0.0
    assert [T[q][far] for q in range(6)] == [1, 0, 0, 1, 0, 1]


def test_tensor_is_identity_or_two_level_spd():
    rng = np.random.default_rng(7)
    img = rng.normal(100.0, 30.0, size=(16, 18, 20))
    T, resp = V.ved_tensor(img, (0.5, 0.5, 0.8), scales=(0.5, 1.0), omega=1.5)
    M = np.stack([np.stack([T[0], T[1], T[2]], -1), np.stack([T[1], T[3], T[4]], -1),
                  np.stack([T[2], T[4], T[5]], -1)], -2)
    w = np.linalg.eigvalsh(M)
    Vv = np.power(resp, 0.1)
    a = 1 + (0.01 - 1) * Vv
    cc = 1 + (1.5 - 1) * Vv
    np.testing.assert_allclose(w[..., 0], a, atol=1e-12)
    np.testing.assert_allclose(w[..., 1], a, atol=1e-12)
    np.testing.assert_allclose(w[..., 2], cc, atol=1e-12)
    assert (resp > 0).any() and (resp == 0).any()


def test_vesselness_formula_matches_reference_branches():
    l = np.array([[0.1, -1.0, -2.0], [-0.1, 1.0, -2.0], [0.0, -0.5, 0.3], [-0.01, -3.0, -3.1]])
    v = V.vesselness(l, 0.5, 0.5, 5.0)
    assert v[1] == 0 and v[2] == 0  # lambda1 or lambda2 >= 0 (VED.hxx:183-186)
    a, b, c = l[0]
    ref = (np.exp(-2e-10 / (abs(b) * c * c)) * (1 - np.exp(-(b * b) / (c * c) / 0.5))
           * np.exp(-(a * a) / abs(b * c) / 0.5) * (1 - np.exp(-(a * a + b * b + c * c) / 50.0)))
    assert abs(v[0] - ref) < 1e-15


def test_sort_by_magnitude_three_swaps():
    w = np.array([[-3.0, -1.0, 0.5], [-0.2, 0.1, 4.0], [-5.0, 2.0, 3.0]])
    e = V.sort_by_magnitude(w)
    np.testing.assert_array_equal(e, [[0.5, -1.0, -3.0], [0.1, -0.2, 4.0], [2.0, 3.0, -5.0]])


def test_mhd_reads_reference_test_volume():
    arr, info = mhd.read_mhd(os.path.join(GOLDEN, "ved_test.mhd"))
    assert arr.shape == (69, 77, 69) and arr.dtype == np.int16
    assert info["spacing"] == [0.3125, 0.3125, 0.5]
    assert info["direction"] == [-1, 0, 0, 0, -1, 0, 0, 0, 1]
    crop = np.load(os.path.join(GOLDEN, "ved_crop_i16.npy"))
    np.testing.assert_array_equal(arr[17:52, 19:58, 17:52], crop)


@pytest.mark.parametrize("dtype,compress", [(np.int16, True), (np.float32, False),
                                            (np.uint8, True), (np.float64, True)])
def test_mhd_round_trip(tmp_path, dtype, compress):
    rng = np.random.default_rng(3)
    a = (rng.random((5, 6, 7)) * 100).astype(dtype)
    p = str(tmp_path / "vol.mhd")
    mhd.write_mhd(p, a, spacing=(0.5, 0.25, 2.0), origin=(1, 2, 3), compress=compress)
    b, info = mhd.read_mhd(p)
    assert b.dtype == a.dtype
    np.testing.assert_array_equal(a, b)
    assert info["spacing"] == [0.5, 0.25, 2.0] and info["origin"] == [1, 2, 3]
