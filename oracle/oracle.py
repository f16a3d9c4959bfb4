"""ctypes wrapper for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker.  The product path (the HIP library in
multigridanisotropicdiffusion_amd/) never imports it.

PARITY UNPINNED: the reference (nellogrb/MultigridAnisotropicDiffusion) has
no golden vectors and cannot be built here (ITK/VXL absent); the oracle is
pinned by analytic known-answer tests only (tests/test_oracle.py).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmad_oracle.so")

VCYCLE, FMG, SMOOTHER = 0, 1, 2
GS_LEX, WJ, GS_COLOR = 0, 1, 2
VERTEX, CELL = 0, 1


class OraParams(ctypes.Structure):
    _fields_ = [
        ("cycle", ctypes.c_int),
        ("smoother", ctypes.c_int),
        ("iterations_per_grid", ctypes.c_uint),
        ("max_cycles", ctypes.c_uint),
        ("number_of_steps", ctypes.c_uint),
        ("tolerance", ctypes.c_double),
        ("omega", ctypes.c_double),
        ("verbose", ctypes.c_int),
        ("ncolors", ctypes.c_int),
    ]


def build():
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        lp = ctypes.POINTER(ctypes.c_long)
        ip = ctypes.POINTER(ctypes.c_int)
        L.ora_max_depth.argtypes = [ctypes.c_int, lp]
        L.ora_max_depth.restype = ctypes.c_int
        L.ora_create.argtypes = [ctypes.c_int, lp, dp, dp, ctypes.c_double]
        L.ora_create.restype = ctypes.c_void_p
        L.ora_destroy.argtypes = [ctypes.c_void_p]
        L.ora_num_levels.argtypes = [ctypes.c_void_p]
        L.ora_num_levels.restype = ctypes.c_int
        L.ora_level_info.argtypes = [ctypes.c_void_p, ctypes.c_int, lp, dp, ip]
        L.ora_stencil.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_stencil.restype = dp
        for name in ("ora_gs_lex", "ora_residual"):
            getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_int, dp, dp, dp]
        L.ora_gs_color.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, dp, dp, dp]
        L.ora_gs_color_omp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, dp, dp, dp,
                                       ctypes.c_int]
        L.ora_wj.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, dp, dp, dp]
        L.ora_restrict.argtypes = [ctypes.c_void_p, ctypes.c_int, dp, dp]
        L.ora_interpolate.argtypes = [ctypes.c_void_p, ctypes.c_int, dp, dp]
        L.ora_direct_solve.argtypes = [ctypes.c_void_p, dp, dp]
        L.ora_l2norm.argtypes = [ctypes.c_long, dp]
        L.ora_l2norm.restype = ctypes.c_double
        L.ora_run.argtypes = [ctypes.c_void_p, ctypes.POINTER(OraParams), dp, dp, ip, dp]
        L.ora_run.restype = ctypes.c_int
        L.ora_vcycle.argtypes = [ctypes.c_void_p, ctypes.POINTER(OraParams), dp, dp, dp]
        L.ora_fmg.argtypes = [ctypes.c_void_p, ctypes.POINTER(OraParams), dp, dp]
        L.ora_take_trace.argtypes = [ctypes.c_void_p, ctypes.c_long, ip, ip, dp]
        L.ora_take_trace.restype = ctypes.c_long
        _lib = L
    return _lib


def _dp(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _shape3(shape):
    """numpy shape (z,y,x) or (y,x) -> (dim, n[3] x-fastest)."""
    dim = len(shape)
    n = list(reversed(shape)) + [1] * (3 - dim)
    return dim, n


def max_depth(shape):
    dim, n = _shape3(shape)
    arr = (ctypes.c_long * 3)(*n)
    return lib().ora_max_depth(dim, arr)


def params(cycle=VCYCLE, smoother=GS_LEX, iterations_per_grid=2, max_cycles=100,
           number_of_steps=1, tolerance=1e-6, omega=2.0 / 3.0, verbose=0, ncolors=0):
    return OraParams(cycle, smoother, iterations_per_grid, max_cycles, number_of_steps,
                     tolerance, omega, verbose, ncolors)


class Oracle:
    """Hierarchy + DCA operators + coarsest LU for one (image, tensor, dt)."""

    def __init__(self, shape, spacing, tensor, dt):
        """shape: numpy shape (z,y,x)/(y,x); spacing: per numpy axis order reversed
        (x first, as ITK); tensor: array (ncomp, *shape) in ITK component order."""
        self.shape = tuple(shape)
        self.dim, n = _shape3(shape)
        h = list(spacing) + [1.0] * (3 - self.dim)
        t = np.ascontiguousarray(tensor, dtype=np.float64)
        ncomp = self.dim * (self.dim + 1) // 2
        assert t.shape == (ncomp,) + self.shape
        L = lib()
        self._c = L.ora_create(self.dim, (ctypes.c_long * 3)(*n), (ctypes.c_double * 3)(*h),
                               _dp(t), float(dt))
        if not self._c:
            raise RuntimeError("ora_create failed")
        self.levels = []
        for l in range(L.ora_num_levels(self._c)):
            nn = (ctypes.c_long * 3)()
            hh = (ctypes.c_double * 3)()
            cc = (ctypes.c_int * 3)()
            L.ora_level_info(self._c, l, nn, hh, cc)
            nshape = tuple(reversed(list(nn)[: self.dim]))
            self.levels.append(dict(shape=nshape, spacing=list(hh)[: self.dim],
                                    centering=list(cc)[: self.dim]))

    def __del__(self):
        if getattr(self, "_c", None):
            lib().ora_destroy(self._c)
            self._c = None

    @property
    def num_levels(self):
        return len(self.levels)

    def shape_at(self, l):
        return self.levels[l]["shape"]

    def _out(self, l):
        return np.zeros(self.shape_at(l), dtype=np.float64)

    @staticmethod
    def _in(a):
        return np.ascontiguousarray(a, dtype=np.float64)

    def stencil(self, l):
        """(N, 27) copy of the level-l DCA stencil (Neighborhood index order)."""
        N = int(np.prod(self.shape_at(l)))
        p = lib().ora_stencil(self._c, l)
        return np.ctypeslib.as_array(p, shape=(N * 27,)).reshape(N, 27).copy()

    def gs_lex(self, l, x, b):
        out = self._out(l)
        lib().ora_gs_lex(self._c, l, _dp(self._in(x)), _dp(self._in(b)), _dp(out))
        return out

    def gs_color(self, l, x, b, ncolors=4):
        out = self._out(l)
        lib().ora_gs_color(self._c, l, ncolors, _dp(self._in(x)), _dp(self._in(b)), _dp(out))
        return out

    def gs_color_omp(self, l, x, b, ncolors=4, nthreads=1):
        out = self._out(l)
        lib().ora_gs_color_omp(self._c, l, ncolors, _dp(self._in(x)), _dp(self._in(b)), _dp(out),
                               int(nthreads))
        return out

    def wj(self, l, x, b, omega=2.0 / 3.0):
        out = self._out(l)
        lib().ora_wj(self._c, l, omega, _dp(self._in(x)), _dp(self._in(b)), _dp(out))
        return out

    def residual(self, l, x, b):
        out = self._out(l)
        lib().ora_residual(self._c, l, _dp(self._in(x)), _dp(self._in(b)), _dp(out))
        return out

    def restrict(self, l, fine):
        out = self._out(l + 1)
        lib().ora_restrict(self._c, l, _dp(self._in(fine)), _dp(out))
        return out

    def interpolate(self, l, coarse):
        out = self._out(l)
        lib().ora_interpolate(self._c, l, _dp(self._in(coarse)), _dp(out))
        return out

    def direct_solve(self, b):
        out = self._out(self.num_levels - 1)
        lib().ora_direct_solve(self._c, _dp(self._in(b)), _dp(out))
        return out

    def vcycle(self, x, b, **kw):
        p = params(**kw)
        out = self._out(0)
        lib().ora_vcycle(self._c, ctypes.byref(p), _dp(self._in(x)), _dp(self._in(b)), _dp(out))
        return out

    def vcycle_verbose(self, x, b, **kw):
        """One V-cycle with the verbose trace; returns (output, [(level, it, relres), ...])."""
        L = lib()
        L.ora_take_trace(self._c, 0, None, None, None)
        out = self.vcycle(x, b, verbose=1, **kw)
        cap = 1 << 16
        lv = (ctypes.c_int * cap)()
        it = (ctypes.c_int * cap)()
        rr = (ctypes.c_double * cap)()
        n = L.ora_take_trace(self._c, cap, lv, it, rr)
        return out, [(lv[i], it[i], rr[i]) for i in range(min(n, cap))]

    def fmg(self, b, **kw):
        p = params(**kw)
        out = self._out(0)
        lib().ora_fmg(self._c, ctypes.byref(p), _dp(self._in(b)), _dp(out))
        return out

    def run_benchmark(self, image, **kw):
        """Whole filter with the verbose trace; returns (output, cycles, relres, history) where
        history is the reference's -DBENCHMARK relres sequence of a V-cycle / FMG run: the
        level-0 entries of the trace, i.e. after every level-0 sweep and after the level-0
        coarse-grid correction (MAD.hxx:401-409, 450-458, 477-485)."""
        L = lib()
        L.ora_take_trace(self._c, 0, None, None, None)
        out, cyc, rr = self.run(image, verbose=1, **kw)
        cap = 1 << 20
        lv = (ctypes.c_int * cap)()
        it = (ctypes.c_int * cap)()
        rel = (ctypes.c_double * cap)()
        n = L.ora_take_trace(self._c, cap, lv, it, rel)
        assert n <= cap
        return out, cyc, rr, [rel[i] for i in range(n) if lv[i] == 0 and it[i] >= 0]

    def run(self, image, **kw):
        """Whole filter (GenerateData) in fp64; returns (output, cycles, relres)."""
        p = params(**kw)
        steps = p.number_of_steps
        out = self._out(0)
        cyc = (ctypes.c_int * max(steps, 1))()
        rr = (ctypes.c_double * max(steps, 1))()
        lib().ora_run(self._c, ctypes.byref(p), _dp(self._in(image)), _dp(out), cyc, rr)
        return out, list(cyc)[:steps], list(rr)[:steps]


def l2norm(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().ora_l2norm(x.size, _dp(x))
