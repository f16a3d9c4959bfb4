"""VED tensor generation, fp64 numpy restatement -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this
module, and only as the checker; the product (multigridanisotropicdiffusion_amd/)
never imports it.

Restates itk::VEDMultigridImageFilter (reference include/itkVEDMultigridImageFilter.hxx,
cited below as VED.hxx):
  GenerateData        VED.hxx:63-155   (iterations: multiscale vesselness -> tensor ->
                                         MAD diffusion with NumberOfSteps =
                                         DiffusionIterations, MaxCycles 100)
  ComputeHessian      VED.hxx:158-173  (HessianRecursiveGaussianImageFilter,
                                         NormalizeAcrossScale on)
  VesselnessFunction  VED.hxx:176-212
  UpdateVesselness    VED.hxx:215-299  (vnl_symmetric_eigensystem: ascending
                                         eigenvalues, eigenvector columns; sort by |l|
                                         with three swaps; keep the eigensystem of the
                                         scale with the largest response, first scale
                                         unconditionally, later ones on a strict >)
  GenerateDiffusionTensor VED.hxx:302-378 (V = resp^(1/s); T = Q D Q^T with
                                         D = diag(1+(eps-1)V, 1+(eps-1)V, 1+(omega-1)V)
                                         on vnl's eigenvector order, identity where V = 0)

Hessian (ComputeHessian): the reference runs ITK's HessianRecursiveGaussianImageFilter with
NormalizeAcrossScale on.  Default here (kind="recursive"): ITK's RecursiveGaussianImageFilter
algorithm restated from its published description -- per axis a 4th-order recursive (IIR)
approximation of the Gaussian (order 0) and its first / second derivatives (R. Deriche,
"Recursively implementing the Gaussian and its derivatives", INRIA RR-1893, 1993, with ITK's
coefficient set, see DERICHE), a causal and an anticausal pass per line whose initial states
assume the line's end values extend to infinity, normalised so that order 0 keeps constants,
order 1 returns 1 on a unit ramp and order 2 returns 1 on t^2/2 (voxel units); the Hessian
component H_ij applies order 2 along i (i = j) or order 1 along i and j, order 0 along the
remaining axes, and scales by sigma^2 / (h_i h_j) (scale-normalised physical derivatives,
sigma^order d^order/dx^order, Lindeberg's normalisation that NormalizeAcrossScale names).
PARITY UNPINNED for the Hessian stage: ITK is not available here (its version is not pinned
by the reference either), so nothing ties this restatement to ITK's own numbers; it is
checked against the properties above (tests/test_ved_oracle.py).

kind="fir" keeps the round-1 operator (mad_ved_desc.hessian = MAD_VED_HESSIAN_FIR on the
GPU): separable correlation with moment-normalised sampled Gaussian derivative kernels
(see gauss_kernels), the same continuous operator sigma^2 d2/dxi dxj (G_sigma * I):
  K0 = g / sum g;  K1 = t g / sum t^2 g;  K2 = a (t^2 - m) g,
  g(t) = exp(-t^2 / (2 s^2)), s = sigma / h (voxels), t = -R..R, R = ceil(4 s),
  m = sum t^2 g / sum g,  a = 2 / (sum t^4 g - m sum t^2 g)
(exact on polynomials of degree <= 2: sum K0 = 1, sum t K1 = 1, sum t^2 K2 / 2 = 1),
borders replicated (clamped index), physical derivatives (1/h per order),
multiplied by sigma^2.  The eigen-decomposition uses LAPACK (numpy.linalg.eigh), an
independent method from the GPU's Jacobi rotations; both return vnl's order.

The unqualified abs() on doubles (VED.hxx:197,202,266-268) is read as fabs.
"""
import numpy as np

# VED.hxx:34-58 defaults
DEFAULTS = dict(alpha=0.5, beta=0.5, gamma=5.0, epsilon=0.01, omega=5.0, sensitivity=10.0,
                scales=(0.300, 0.482, 0.775, 1.245, 2.000), iterations=1,
                diffusion_iterations=5, time_step=0.1, tolerance=1e-6,
                diffusion_iterations_per_grid=2)


def kernel_radius(sigma, h):
    return max(1, int(np.ceil(4.0 * sigma / h)))


def gauss_kernels(sigma, h):
    """(K0, K1, K2) for one axis (voxel-unit derivatives), see the module docstring.
    Sums run t = -R..R in order (the GPU path computes its taps with the same code
    in C++ on the host)."""
    R = kernel_radius(sigma, h)
    s = sigma / h
    t = np.arange(-R, R + 1, dtype=np.float64)
    g = np.exp(-(t * t) / (2.0 * s * s))
    S0 = S2 = S4 = 0.0
    for q in range(2 * R + 1):
        S0 += g[q]
        S2 += t[q] * t[q] * g[q]
        S4 += t[q] * t[q] * t[q] * t[q] * g[q]
    m = S2 / S0
    a = 2.0 / (S4 - m * S2)
    return g / S0, t * g / S2, a * (t * t - m) * g


def correlate(f, K, axis):
    """out(i) = sum_t K(t) f(clamp(i + t)) along `axis` (numpy axis)."""
    R = (len(K) - 1) // 2
    n = f.shape[axis]
    out = np.zeros_like(f)
    for q, t in enumerate(range(-R, R + 1)):
        idx = np.clip(np.arange(n) + t, 0, n - 1)
        out += K[q] * np.take(f, idx, axis=axis)
    return out


# ITK RecursiveGaussianImageFilter's coefficient set ("parameters of exponential series"):
# index 0 / 1 / 2 = Gaussian / first / second derivative
DERICHE = dict(A1=(1.3530, -0.6724, -1.3563), B1=(1.8151, -3.4327, 5.2318), W1=0.6681, L1=-1.3932,
               A2=(-0.3531, 0.6724, 0.3446), B2=(0.0902, 0.6100, -2.2355), W2=2.0787, L2=-1.3732)


def _n_coefficients(sd, a1, b1, w1, l1, a2, b2, w2, l2):
    """Causal numerator N0..N3 of one exponential pair, and its moments SN, DN, EN."""
    s1, s2 = np.sin(w1 / sd), np.sin(w2 / sd)
    c1, c2 = np.cos(w1 / sd), np.cos(w2 / sd)
    e1, e2 = np.exp(l1 / sd), np.exp(l2 / sd)
    n0 = a1 + a2
    n1 = e2 * (b2 * s2 - (a2 + 2 * a1) * c2)
    n1 += e1 * (b1 * s1 - (a1 + 2 * a2) * c1)
    n2 = (a1 + a2) * c2 * c1
    n2 -= b1 * c2 * s1 + b2 * c1 * s2
    n2 *= 2 * e1 * e2
    n2 += a2 * e1 * e1 + a1 * e2 * e2
    n3 = e2 * e1 * e1 * (b2 * s2 - a2 * c2)
    n3 += e1 * e2 * e2 * (b1 * s1 - a1 * c1)
    return (n0, n1, n2, n3), n0 + n1 + n2 + n3, n1 + 2 * n2 + 3 * n3, n1 + 4 * n2 + 9 * n3


def _d_coefficients(sd, w1, l1, w2, l2):
    """Denominator D1..D4 (shared by both passes) and its moments SD, DD, ED."""
    c1, c2 = np.cos(w1 / sd), np.cos(w2 / sd)
    e1, e2 = np.exp(l1 / sd), np.exp(l2 / sd)
    d4 = e1 * e1 * e2 * e2
    d3 = -2 * c1 * e1 * e2 * e2
    d3 += -2 * c2 * e2 * e1 * e1
    d2 = 4 * c2 * c1 * e1 * e2
    d2 += e1 * e1 + e2 * e2
    d1 = -2 * (e2 * c2 + e1 * c1)
    D = (d1, d2, d3, d4)
    return D, 1.0 + d1 + d2 + d3 + d4, d1 + 2 * d2 + 3 * d3 + 4 * d4, d1 + 4 * d2 + 9 * d3 + 16 * d4


def recursive_coefficients(sd, order):
    """The 20 coefficients of one axis / order for sigma sd in voxels: N0..N3 (causal),
    M1..M4 (anticausal), D1..D4 and the border terms BN1..BN4, BM1..BM4; voxel-unit
    normalisation (order 0 gain 1, order 1 slope 1, order 2 curvature 1)."""
    P = DERICHE
    pair = lambda o: (P["A1"][o], P["B1"][o], P["W1"], P["L1"], P["A2"][o], P["B2"][o], P["W2"], P["L2"])
    D, SD, DD, ED = _d_coefficients(sd, P["W1"], P["L1"], P["W2"], P["L2"])
    if order == 0:
        N, SN, DN, EN = _n_coefficients(sd, *pair(0))
        alpha = 2 * SN / SD - N[0]
        N = tuple(v / alpha for v in N)
        symmetric = True
    elif order == 1:
        N, SN, DN, EN = _n_coefficients(sd, *pair(1))
        alpha = 2 * (SN * DD - DN * SD) / (SD * SD)
        N = tuple(v / alpha for v in N)
        symmetric = False
    else:
        N0, SN0, DN0, EN0 = _n_coefficients(sd, *pair(0))
        N2, SN2, DN2, EN2 = _n_coefficients(sd, *pair(2))
        beta = -(2 * SN2 - SD * N2[0]) / (2 * SN0 - SD * N0[0])
        a, b, c, d = (N2[q] + beta * N0[q] for q in range(4))
        SN = a + b + c + d
        DN = b + 2 * c + 3 * d
        EN = b + 4 * c + 9 * d
        alpha = EN * SD * SD - ED * SN * SD - 2 * DN * DD * SD + 2 * DD * DD * SN
        alpha /= SD * SD * SD
        N = (a / alpha, b / alpha, c / alpha, d / alpha)
        symmetric = True
    if symmetric:
        M = (N[1] - D[0] * N[0], N[2] - D[1] * N[0], N[3] - D[2] * N[0], -D[3] * N[0])
    else:
        M = (-(N[1] - D[0] * N[0]), -(N[2] - D[1] * N[0]), -(N[3] - D[2] * N[0]), D[3] * N[0])
    SNn = N[0] + N[1] + N[2] + N[3]
    SM = M[0] + M[1] + M[2] + M[3]
    SDn = 1.0 + D[0] + D[1] + D[2] + D[3]
    BN = tuple(D[q] * SNn / SDn for q in range(4))
    BM = tuple(D[q] * SM / SDn for q in range(4))
    return dict(N=N, M=M, D=D, BN=BN, BM=BM)


def recursive_filter(f, c, axis):
    """Causal + anticausal passes along `axis` (numpy axis) with the coefficients c
    (recursive_coefficients); the initial states take the line's first / last value as
    extending to infinity.  Needs >= 4 points along the axis."""
    x = np.moveaxis(np.asarray(f, np.float64), axis, -1)
    n = x.shape[-1]
    if n < 4:
        raise ValueError("recursive Gaussian needs at least 4 points along each axis")
    N0, N1, N2, N3 = c["N"]
    M1, M2, M3, M4 = c["M"]
    D1, D2, D3, D4 = c["D"]
    BN1, BN2, BN3, BN4 = c["BN"]
    BM1, BM2, BM3, BM4 = c["BM"]
    s = np.empty_like(x)
    v = x[..., 0]
    s[..., 0] = v * N0 + v * N1 + v * N2 + v * N3
    s[..., 1] = x[..., 1] * N0 + v * N1 + v * N2 + v * N3
    s[..., 2] = x[..., 2] * N0 + x[..., 1] * N1 + v * N2 + v * N3
    s[..., 3] = x[..., 3] * N0 + x[..., 2] * N1 + x[..., 1] * N2 + v * N3
    s[..., 0] -= v * BN1 + v * BN2 + v * BN3 + v * BN4
    s[..., 1] -= s[..., 0] * D1 + v * BN2 + v * BN3 + v * BN4
    s[..., 2] -= s[..., 1] * D1 + s[..., 0] * D2 + v * BN3 + v * BN4
    s[..., 3] -= s[..., 2] * D1 + s[..., 1] * D2 + s[..., 0] * D3 + v * BN4
    for i in range(4, n):
        s[..., i] = x[..., i] * N0 + x[..., i - 1] * N1 + x[..., i - 2] * N2 + x[..., i - 3] * N3
        s[..., i] -= s[..., i - 1] * D1 + s[..., i - 2] * D2 + s[..., i - 3] * D3 + s[..., i - 4] * D4
    a = np.empty_like(x)
    v = x[..., n - 1]
    a[..., n - 1] = v * M1 + v * M2 + v * M3 + v * M4
    a[..., n - 2] = x[..., n - 1] * M1 + v * M2 + v * M3 + v * M4
    a[..., n - 3] = x[..., n - 2] * M1 + x[..., n - 1] * M2 + v * M3 + v * M4
    a[..., n - 4] = x[..., n - 3] * M1 + x[..., n - 2] * M2 + x[..., n - 1] * M3 + v * M4
    a[..., n - 1] -= v * BM1 + v * BM2 + v * BM3 + v * BM4
    a[..., n - 2] -= a[..., n - 1] * D1 + v * BM2 + v * BM3 + v * BM4
    a[..., n - 3] -= a[..., n - 2] * D1 + a[..., n - 1] * D2 + v * BM3 + v * BM4
    a[..., n - 4] -= a[..., n - 3] * D1 + a[..., n - 2] * D2 + a[..., n - 1] * D3 + v * BM4
    for i in range(n - 4, 0, -1):
        a[..., i - 1] = x[..., i] * M1 + x[..., i + 1] * M2 + x[..., i + 2] * M3 + x[..., i + 3] * M4
        a[..., i - 1] -= a[..., i] * D1 + a[..., i + 1] * D2 + a[..., i + 2] * D3 + a[..., i + 3] * D4
    return np.moveaxis(s + a, -1, axis)


def hessian(img, spacing, sigma, kind="recursive"):
    """Scale-normalised Hessian, components [xx, xy, xz, yy, yz, zz] (ITK
    SymmetricSecondRankTensor order) stacked on the last axis.  img is (z, y, x),
    spacing (hx, hy, hz).  kind: "recursive" (ITK's operator, default) or "fir"."""
    img = np.asarray(img, np.float64)
    hx, hy, hz = spacing
    if kind == "fir":
        Kx, Ky, Kz = (gauss_kernels(sigma, h) for h in (hx, hy, hz))
        fx = lambda f, o: correlate(f, Kx[o], 2)
        fy = lambda f, o: correlate(f, Ky[o], 1)
        fz = lambda f, o: correlate(f, Kz[o], 0)
    else:
        C = {ax: [recursive_coefficients(sigma / h, o) for o in range(3)]
             for ax, h in ((2, hx), (1, hy), (0, hz))}
        fx = lambda f, o: recursive_filter(f, C[2][o], 2)
        fy = lambda f, o: recursive_filter(f, C[1][o], 1)
        fz = lambda f, o: recursive_filter(f, C[0][o], 0)
    Z = [fz(img, o) for o in range(3)]
    A = {(oy, oz): fy(Z[oz], oy) for oy, oz in [(0, 0), (1, 0), (2, 0), (0, 1), (1, 1), (0, 2)]}
    s2 = sigma * sigma
    H = np.empty(img.shape + (6,))
    H[..., 0] = fx(A[(0, 0)], 2) * (s2 / (hx * hx))
    H[..., 1] = fx(A[(1, 0)], 1) * (s2 / (hx * hy))
    H[..., 2] = fx(A[(0, 1)], 1) * (s2 / (hx * hz))
    H[..., 3] = fx(A[(2, 0)], 0) * (s2 / (hy * hy))
    H[..., 4] = fx(A[(1, 1)], 0) * (s2 / (hy * hz))
    H[..., 5] = fx(A[(0, 2)], 0) * (s2 / (hz * hz))
    return H


def vesselness(l, alpha, beta, gamma):
    """VED.hxx:176-212 on eigenvalues sorted by |l| (l[..., 0] smallest)."""
    l0, l1, l2 = l[..., 0], l[..., 1], l[..., 2]
    out = np.zeros(l0.shape)
    ok = ~((l1 >= 0) | (l2 >= 0))
    a, b, c = l0[ok], l1[ok], l2[ok]
    smoothC = 1e-5
    Ra = (b * b) / (c * c)
    Rb = (a * a) / np.abs(b * c)
    S = a * a + b * b + c * c
    sf = np.exp(-(2 * smoothC * smoothC) / (np.abs(b) * c * c))
    out[ok] = (sf * (1.0 - np.exp(-Ra / (2.0 * alpha * alpha)))
               * np.exp(-Rb / (2.0 * beta * beta))
               * (1.0 - np.exp(-S / (2.0 * gamma * gamma))))
    return out


def sort_by_magnitude(w):
    """VED.hxx:266-268: three conditional swaps of the ascending eigenvalues."""
    e = w.copy()
    for i, j in ((0, 1), (1, 2), (0, 1)):
        sw = np.abs(e[..., i]) > np.abs(e[..., j])
        ei, ej = e[..., i].copy(), e[..., j].copy()
        e[..., i] = np.where(sw, ej, ei)
        e[..., j] = np.where(sw, ei, ej)
    return e


def scale_responses(img, spacing, scales, alpha, beta, gamma, kind="recursive"):
    """Vesselness of every scale (UpdateVesselness's candidates, VED.hxx:215-299), stacked:
    (len(scales), *img.shape).  Used to find scale near-ties (the strict argmax, VED.hxx:272)."""
    out = []
    for sigma in scales:
        H = hessian(img, spacing, sigma, kind)
        A = np.empty(img.shape + (3, 3))
        A[..., 0, 0], A[..., 0, 1], A[..., 0, 2] = H[..., 0], H[..., 1], H[..., 2]
        A[..., 1, 0], A[..., 1, 1], A[..., 1, 2] = H[..., 1], H[..., 3], H[..., 4]
        A[..., 2, 0], A[..., 2, 1], A[..., 2, 2] = H[..., 2], H[..., 4], H[..., 5]
        w = np.linalg.eigh(A)[0]
        out.append(vesselness(sort_by_magnitude(w), alpha, beta, gamma))
    return np.stack(out)


def near_ties(img, spacing, scales, alpha, beta, gamma, rel=1e-6):
    """Voxels whose two largest scale responses are within `rel` of each other (positive
    response): where an fp32 Hessian may pick either scale's direction."""
    ves = np.sort(scale_responses(img, spacing, scales, alpha, beta, gamma), axis=0)
    return (ves[-1] > 0) & ((ves[-1] - ves[-2]) <= rel * ves[-1])


def multiscale(img, spacing, scales, alpha, beta, gamma, kind="recursive"):
    """UpdateVesselness over all scales: (response, eigenvector columns Q)."""
    resp = None
    Q = None
    for i, sigma in enumerate(scales):
        H = hessian(img, spacing, sigma, kind)
        M = np.empty(img.shape + (3, 3))
        M[..., 0, 0], M[..., 0, 1], M[..., 0, 2] = H[..., 0], H[..., 1], H[..., 2]
        M[..., 1, 0], M[..., 1, 1], M[..., 1, 2] = H[..., 1], H[..., 3], H[..., 4]
        M[..., 2, 0], M[..., 2, 1], M[..., 2, 2] = H[..., 2], H[..., 4], H[..., 5]
        w, v = np.linalg.eigh(M)  # ascending eigenvalues, eigenvectors as columns
        ves = vesselness(sort_by_magnitude(w), alpha, beta, gamma)
        if i == 0:
            resp, Q = ves, v
        else:
            upd = ves > resp
            resp = np.where(upd, ves, resp)
            Q = np.where(upd[..., None, None], v, Q)
    return resp, Q


def diffusion_tensor(resp, Q, epsilon, omega, sensitivity):
    """GenerateDiffusionTensor (VED.hxx:302-378): SoA (6, *shape), components
    [xx,xy,xz,yy,yz,zz] (the layout oracle.Oracle and Solver.set_tensor take)."""
    V = np.power(resp, 1.0 / sensitivity)
    D = np.stack([1.0 + (epsilon - 1.0) * V, 1.0 + (epsilon - 1.0) * V,
                  1.0 + (omega - 1.0) * V], axis=-1)
    T = np.einsum("...ik,...k,...jk->...ij", Q, D, Q)
    out = np.empty((6,) + resp.shape)
    for c, (d, d2) in enumerate(((0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2))):
        out[c] = np.where(V > 0, T[..., d, d2], 1.0 if d == d2 else 0.0)
    return out


def ved_tensor(img, spacing, scales=DEFAULTS["scales"], alpha=0.5, beta=0.5, gamma=5.0,
               epsilon=0.01, omega=5.0, sensitivity=10.0, kind="recursive"):
    resp, Q = multiscale(img, spacing, scales, alpha, beta, gamma, kind)
    return diffusion_tensor(resp, Q, epsilon, omega, sensitivity), resp


def ved_run(img, spacing, oracle_mod, out_dtype=np.float64, **kw):
    """GenerateData (VED.hxx:63-155) with the C MAD oracle for DiffusionStep."""
    p = dict(DEFAULTS)
    p.update(kw)
    x = np.asarray(img, np.float64).copy()
    steps = []
    for _ in range(p["iterations"]):
        T, _ = ved_tensor(x, spacing, p["scales"], p["alpha"], p["beta"], p["gamma"],
                          p["epsilon"], p["omega"], p["sensitivity"], p.get("hessian", "recursive"))
        o = oracle_mod.Oracle(x.shape, spacing, T, p["time_step"])
        x, cyc, rr = o.run(x, cycle=p.get("cycle", oracle_mod.VCYCLE),
                           smoother=p.get("smoother", oracle_mod.GS_LEX),
                           iterations_per_grid=p["diffusion_iterations_per_grid"],
                           max_cycles=100, number_of_steps=p["diffusion_iterations"],
                           tolerance=p["tolerance"])
        steps.append((cyc, rr))
    if np.issubdtype(np.dtype(out_dtype), np.integer):
        x = np.trunc(x).astype(out_dtype)
    return x, steps
