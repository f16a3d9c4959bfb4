"""numpy restatement of the matrix-free operator the HIP kernels evaluate.

TEST HELPER.  The GPU never stores the reference's 27-coefficient DCA stencil
(include/mad/itkGridsHierarchy.hxx:298-516); it evaluates the identical
operator from per-level coefficient fields:

  a_d   = dt * M_dd / h_d^2
  e_dd2 = dt * M_dd2 / (2 h_d h_d2)                 (d < d2)
  g_d   = dt / (2 h_d) * sum_d2 delta_d2 M_d,d2 / (2 h_d2)
  delta = central difference inside, one-sided 2nd order on the border
          (GH:447-474)
  (A u)(p) = D u(p) - S(p),  D = 1 + 2 sum_d a_d,
  S(p) = sum_d (a_d + g_d) u~(p+e_d) + (a_d - g_d) u~(p-e_d)
       + sum_{d<d2} e_dd2 [u~(++) - u~(+-) - u~(-+) + u~(--)]
  u~ = mirror ghost about the boundary node: u~(-1)=u(1), u~(n)=u(n-2).

tests/test_oracle.py checks this equals the oracle's DCA stencil to 1e-13.
Arrays are numpy (z, y, x) / (y, x); spacing is given x-first (ITK order).
"""
import numpy as np


def tcomp(dim, d, d2):
    if d > d2:
        d, d2 = d2, d
    return d * dim - d * (d - 1) // 2 + (d2 - d)


def _axis(dim, d):
    """ITK dimension d (x=0) -> numpy axis."""
    return dim - 1 - d


def delta(f, d, dim):
    """2h * derivative of field f along ITK dim d, one-sided at the border (GH:447-474)."""
    ax = _axis(dim, d)
    f = np.moveaxis(f, ax, 0)
    out = np.empty_like(f)
    out[1:-1] = f[2:] - f[:-2]
    out[0] = -3.0 * f[0] + 4.0 * f[1] - 1.0 * f[2]
    out[-1] = 3.0 * f[-1] - 4.0 * f[-2] + 1.0 * f[-3]
    return np.moveaxis(out, 0, ax)


def coefficients(tensor, spacing, dt):
    """Return dict with 'a' (dim fields), 'e' ({(d,d2): field}), 'g' (dim fields)."""
    dim = tensor.ndim - 1
    h = list(spacing)
    a = [dt * tensor[tcomp(dim, d, d)] / (h[d] * h[d]) for d in range(dim)]
    e = {}
    for d in range(dim):
        for d2 in range(d + 1, dim):
            e[(d, d2)] = dt * tensor[tcomp(dim, d, d2)] / (2.0 * h[d] * h[d2])
    g = []
    for d in range(dim):
        s = np.zeros(tensor.shape[1:])
        for d2 in range(dim):
            s = s + delta(tensor[tcomp(dim, d, d2)], d2, dim) / (2.0 * h[d2])
        g.append(dt / (2.0 * h[d]) * s)
    return dict(a=a, e=e, g=g)


def mirror_pad(u):
    p = np.pad(u, 1, mode="reflect")  # reflect: u(-1)=u(1), u(n)=u(n-2)
    return p


def shifted(P, dim, offs):
    """View of padded array P at offset offs (ITK order, each in -1..1)."""
    sl = [slice(None)] * dim
    for d in range(dim):
        ax = _axis(dim, d)
        o = offs[d]
        n = P.shape[ax] - 2
        sl[ax] = slice(1 + o, 1 + o + n)
    return P[tuple(sl)]


def off_sum(u, co):
    dim = u.ndim
    P = mirror_pad(u)
    S = np.zeros_like(u)
    for d in range(dim):
        ep = [0] * dim
        ep[d] = 1
        em = [0] * dim
        em[d] = -1
        S += (co["a"][d] + co["g"][d]) * shifted(P, dim, ep)
        S += (co["a"][d] - co["g"][d]) * shifted(P, dim, em)
    for (d, d2), e in co["e"].items():
        def o(sd, sd2):
            v = [0] * dim
            v[d] = sd
            v[d2] = sd2
            return v
        S += e * (shifted(P, dim, o(1, 1)) - shifted(P, dim, o(1, -1))
                  - shifted(P, dim, o(-1, 1)) + shifted(P, dim, o(-1, -1)))
    return S


def diag(co):
    return 1.0 + 2.0 * sum(co["a"])


def apply(u, co):
    return diag(co) * u - off_sum(u, co)
