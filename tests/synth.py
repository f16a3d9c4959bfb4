"""Seeded synthetic inputs shared by tests, fixture scripts and bench (host side).

Tensor fields are returned as (ncomp, *shape) float64 in ITK component order
[xx,xy,xz,yy,yz,zz] (3D) / [xx,xy,yy] (2D).
"""
import numpy as np


def random_spd(shape, seed=0, lo=0.1, hi=2.0, offdiag=True):
    """Smoothly varying SPD field Q diag(l) Q^T (SURVEY §8d C3 form, small sizes)."""
    rng = np.random.default_rng(seed)
    dim = len(shape)
    grids = np.meshgrid(*[np.arange(s, dtype=np.float64) for s in shape], indexing="ij")
    ph = rng.uniform(0, 2 * np.pi, size=8)
    if dim == 3:
        z, y, x = grids
        a1 = 0.9 * np.sin(2 * np.pi * x / 11 + ph[0]) * np.cos(2 * np.pi * z / 13 + ph[1])
        a2 = 0.7 * np.sin(2 * np.pi * y / 9 + ph[2])
        a3 = 0.8 * np.cos(2 * np.pi * (x + z) / 15 + ph[3])
        lam = [lo + (hi - lo) * (0.5 + 0.5 * np.sin(2 * np.pi * g / p + q))
               for g, p, q in ((x, 7, ph[4]), (y, 10, ph[5]), (z, 8, ph[6]))]
        ca, sa = np.cos(a1), np.sin(a1)
        cb, sb = np.cos(a2), np.sin(a2)
        cc, sc = np.cos(a3), np.sin(a3)
        # Q = Rz(a1) Ry(a2) Rx(a3), built elementwise
        Q = np.empty((3, 3) + tuple(shape))
        Q[0, 0] = ca * cb
        Q[0, 1] = ca * sb * sc - sa * cc
        Q[0, 2] = ca * sb * cc + sa * sc
        Q[1, 0] = sa * cb
        Q[1, 1] = sa * sb * sc + ca * cc
        Q[1, 2] = sa * sb * cc - ca * sc
        Q[2, 0] = -sb
        Q[2, 1] = cb * sc
        Q[2, 2] = cb * cc
        if not offdiag:
            Q = np.zeros_like(Q)
            for i in range(3):
                Q[i, i] = 1.0
        T = np.einsum("ik...,k...,jk...->ij...", Q, np.stack(lam), Q)
        return np.stack([T[0, 0], T[0, 1], T[0, 2], T[1, 1], T[1, 2], T[2, 2]])
    y, x = grids
    a = 1.1 * np.sin(2 * np.pi * x / 9 + ph[0]) * np.cos(2 * np.pi * y / 7 + ph[1])
    l1 = lo + (hi - lo) * (0.5 + 0.5 * np.sin(2 * np.pi * x / 6 + ph[2]))
    l2 = lo + (hi - lo) * (0.5 + 0.5 * np.cos(2 * np.pi * y / 5 + ph[3]))
    if not offdiag:
        a = np.zeros_like(a)
    c, s = np.cos(a), np.sin(a)
    txx = c * c * l1 + s * s * l2
    txy = c * s * (l1 - l2)
    tyy = s * s * l1 + c * c * l2
    return np.stack([txx, txy, tyy])


def isotropic(shape, seed=0):
    """c(x) I with c = 1 + 0.5 sin sin sin (SURVEY §8d C2 form)."""
    dim = len(shape)
    grids = np.meshgrid(*[np.arange(s, dtype=np.float64) for s in shape], indexing="ij")
    c = np.ones(shape)
    for g in grids:
        c = c * np.sin(2 * np.pi * g / 32 + 0.3 * seed)
    c = 1.0 + 0.5 * c
    if dim == 3:
        z = np.zeros(shape)
        return np.stack([c, z, z, c, z, c])
    z = np.zeros(shape)
    return np.stack([c, z, c])


def constant(shape, values):
    return np.stack([np.full(shape, float(v)) for v in values])


def ved_form(shape, eps=0.01, omega=1.5, sens=10.0, seed=4):
    """VED-form tensor (include/itkVEDMultigridImageFilter.hxx:327-365) on an analytic
    vesselness / direction field: T = l_perp I + (l_par - l_perp) v v^T with
    l_perp = 1 + (eps-1) V, l_par = 1 + (omega-1) V, V = resp^(1/sens); identity where V = 0."""
    z, y, x = np.meshgrid(*[np.arange(s, dtype=np.float64) for s in shape], indexing="ij")
    resp = vesselness_field(x, y, z, shape, seed)
    V = np.where(resp > 0, np.power(np.maximum(resp, 0), 1.0 / sens), 0.0)
    v = direction_field(x, y, z, shape)
    lp = 1.0 + (eps - 1.0) * V
    la = 1.0 + (omega - 1.0) * V
    d = la - lp
    return np.stack([lp + d * v[0] * v[0], d * v[0] * v[1], d * v[0] * v[2],
                     lp + d * v[1] * v[1], d * v[1] * v[2], lp + d * v[2] * v[2]])


def direction_field(x, y, z, shape):
    nx, ny, nz = shape[2], shape[1], shape[0]
    vx = np.sin(2 * np.pi * y / max(ny, 2) * 1.5) + 0.3
    vy = np.cos(2 * np.pi * z / max(nz, 2) * 1.25)
    vz = 1.0 + 0.5 * np.sin(2 * np.pi * x / max(nx, 2))
    nrm = np.sqrt(vx * vx + vy * vy + vz * vz)
    return np.stack([vx / nrm, vy / nrm, vz / nrm])


def vesselness_field(x, y, z, shape, seed):
    nx, ny, nz = shape[2], shape[1], shape[0]
    s = (np.sin(2 * np.pi * x / max(nx, 2) * 3 + seed) *
         np.sin(2 * np.pi * y / max(ny, 2) * 2 + 0.5 * seed) *
         np.cos(2 * np.pi * z / max(nz, 2) * 2.5))
    return np.maximum(s, 0.0) ** 2  # zero on about half the volume (identity tensor there)


def image(shape, seed=1):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, size=shape)


def tube_phantom(S, seed=4):
    """C4's VED input: bright axis-aligned tubes (radius 2..6 voxels, intensity
    200 on 0) plus N(0, 10^2) noise, fp32 (z, y, x) -- the volume tools/bench_ved.py times.
    S: the cube's edge, or a (z, y, x) shape (C5: (512, 1024, 1024))."""
    shape = (S, S, S) if np.isscalar(S) else tuple(int(n) for n in S)
    cube = len(set(shape)) == 1
    rng = np.random.default_rng(seed)
    img = rng.normal(0.0, 10.0, size=shape).astype(np.float32)
    for axis in range(3):
        n1, n2 = [shape[a] for a in range(3) if a != axis]  # the tube's cross-section axes
        g1 = np.arange(n1, dtype=np.float32)
        g2 = np.arange(n2, dtype=np.float32)
        prof = np.zeros((n1, n2), np.float32)
        for _ in range(64 // 3 + (1 if axis < 64 % 3 else 0)):
            if cube:
                a, b = rng.uniform(8, n1 - 8, size=2)
            else:
                a, b = rng.uniform(8, n1 - 8), rng.uniform(8, n2 - 8)
            r = rng.uniform(2, 6)
            prof += 200.0 * np.exp(-((g1[:, None] - a) ** 2 + (g2[None, :] - b) ** 2) / (2 * r * r))
        if axis == 0:
            img += prof[None, :, :]
        elif axis == 1:
            img += prof[:, None, :]
        else:
            img += prof[:, :, None]
    return img
