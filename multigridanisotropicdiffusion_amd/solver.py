"""Host-side mirror of the reference's operator surface over the C ABI.

``Solver`` exposes the kernel-level entry points of include/mad.h (one
context = hierarchy + operators resident on one GPU); the ITK-shaped filter
classes live in ``filters.py``.  numpy arrays use (z, y, x) / (y, x) order;
the C ABI takes sizes and spacings x first, as ITK does.
"""
import ctypes
import os

import numpy as np

from . import _capi as C

_DT = {np.dtype(np.uint8): C.U8, np.dtype(np.int8): C.I8, np.dtype(np.uint16): C.U16,
       np.dtype(np.int16): C.I16, np.dtype(np.uint32): C.U32, np.dtype(np.int32): C.I32,
       np.dtype(np.float32): C.F32, np.dtype(np.float64): C.F64}


def mad_dtype(dt):
    dt = np.dtype(dt)
    if dt not in _DT:
        raise TypeError(f"unsupported pixel type {dt}")
    return _DT[dt]


def max_depth(shape):
    """GridsHierarchy depth rule (include/mad/itkGridsHierarchy.hxx:36-59)."""
    dim = len(shape)
    n = (ctypes.c_int64 * 3)(*(list(reversed(shape)) + [1] * (3 - dim)))
    return C.load().mad_max_depth(dim, n)


def slab_range(nz, nranks, rank, align=1):
    b, e = ctypes.c_int64(), ctypes.c_int64()
    C.check(C.load().mad_slab_range(nz, nranks, rank, align, ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def tensor_to_aos(tensor, shape):
    """Accept (ncomp, *shape) SoA or (*shape, ncomp) AoS; return contiguous AoS."""
    t = np.asarray(tensor)
    dim = len(shape)
    ncomp = dim * (dim + 1) // 2
    if t.shape == (ncomp,) + tuple(shape):
        t = np.moveaxis(t, 0, -1)
    elif t.shape != tuple(shape) + (ncomp,):
        raise ValueError(f"tensor shape {t.shape} does not match image {shape} "
                         f"(expected {(ncomp,) + tuple(shape)} or {tuple(shape) + (ncomp,)})")
    if t.dtype not in (np.float32, np.float64):
        t = t.astype(np.float64)
    return np.ascontiguousarray(t)


class Solver:
    """One GPU context (mad_ctx).  Parameters mirror the filter setters
    (itkMultigridAnisotropicDiffusionImageFilter.h:133-160) and their defaults."""

    def __init__(self, shape, spacing=None, *, time_step=0.01, cycle=C.VCYCLE,
                 smoother=C.GAUSS_SEIDEL, iterations_per_grid=2, max_cycles=100,
                 number_of_steps=1, tolerance=1e-6, omega=2.0 / 3.0, verbose=False,
                 precision=C.PRECISION_AUTO, stall_guard=None, device=-1, tensor_kind=C.TENSOR_AUTO,
                 nranks=1, rank=0, global_shape=None, gs_kernel=0, options=0, min_slab_planes=0,
                 min_slab_voxels=0, coarse_dense_max=0, coarse_block_unknowns=0):
        L = C.load()
        self.shape = tuple(int(s) for s in shape)  # this rank's slab
        gshape = tuple(global_shape) if global_shape is not None else self.shape
        self.dim = len(gshape)
        if self.dim not in (2, 3):
            raise ValueError("images must be 2D or 3D")
        d = C.default_desc()
        d.dim = self.dim
        size = list(reversed(gshape)) + [1] * (3 - self.dim)
        for q in range(3):
            d.size[q] = size[q]
        sp = list(spacing) if spacing is not None else [1.0] * self.dim
        for q in range(3):
            d.spacing[q] = sp[q] if q < self.dim else 1.0
        d.cycle = int(cycle)
        d.smoother = int(smoother)
        d.iterations_per_grid = int(iterations_per_grid)
        d.max_cycles = int(max_cycles)
        d.number_of_steps = int(number_of_steps)
        d.time_step = float(time_step)
        d.tolerance = float(tolerance)
        d.omega = float(omega)
        d.verbose = int(bool(verbose))
        d.precision = int(precision)
        d.stall_guard = int(precision != C.FP64) if stall_guard is None else int(stall_guard)
        d.device = int(device)
        d.tensor_kind = int(tensor_kind)
        d.nranks = int(nranks)
        d.rank = int(rank)
        d.gs_kernel = int(gs_kernel)
        d.options = int(options)
        d.min_slab_planes = int(min_slab_planes)
        d.min_slab_voxels = int(min_slab_voxels)
        d.coarse_dense_max = int(coarse_dense_max)
        d.coarse_block_unknowns = int(coarse_block_unknowns)
        self._desc = d
        ctx = ctypes.c_void_p()
        C.check(L.mad_create(ctypes.byref(d), ctypes.byref(ctx)))
        self._ctx = ctx
        self._L = L
        self.precision = precision

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.mad_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        return C.check(rc, self._ctx)

    # ------------------------------------------------------------ setup
    def set_tensor(self, tensor):
        """SetDiffusionTensor: (ncomp, *shape) SoA or (*shape, ncomp) AoS, ITK order."""
        gshape = tuple(reversed([self._desc.size[q] for q in range(self.dim)]))
        t = tensor_to_aos(tensor, gshape)
        self._check(self._L.mad_set_tensor(self._ctx, t.ctypes.data_as(ctypes.c_void_p),
                                           C.F64 if t.dtype == np.float64 else C.F32))

    def tensor_planes(self):
        """Global z planes [first, first + n) of the tensor this context stores
        (mad_tensor_planes): the whole grid on one rank, slab + ghost planes on a rank."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._L.mad_tensor_planes(self._ctx, ctypes.byref(a), ctypes.byref(b)))
        return a.value, a.value + b.value

    def set_tensor_planes(self, tensor, first_plane):
        """SetDiffusionTensor from global planes [first_plane, ...) only (AoS (z, y, x, ncomp)
        or SoA (ncomp, z, y, x) of those planes; mad_set_tensor_planes).  The in-plane shape
        must be the grid's; the plane count is the array's."""
        if self.dim != 3:
            raise ValueError("set_tensor_planes takes z planes of a 3D grid; use set_tensor in 2D")
        nc = 6
        plane = tuple(reversed([self._desc.size[q] for q in range(2)]))  # (y, x)
        t = np.asarray(tensor)
        aos_ok = t.ndim == 4 and t.shape[1:3] == plane and t.shape[3] == nc
        soa_ok = t.ndim == 4 and t.shape[0] == nc and t.shape[2:] == plane
        if aos_ok and soa_ok:
            raise ValueError(f"tensor planes of shape {t.shape} are ambiguous (AoS or SoA)")
        if soa_ok:
            t = np.moveaxis(t, 0, -1)
        elif not aos_ok:
            raise ValueError(f"tensor planes of shape {t.shape} do not match the grid: expected "
                             f"AoS (planes, {plane[0]}, {plane[1]}, {nc}) or SoA "
                             f"({nc}, planes, {plane[0]}, {plane[1]})")
        t = np.ascontiguousarray(t, dtype=np.float64 if t.dtype == np.float64 else np.float32)
        self._check(self._L.mad_set_tensor_planes(self._ctx, t.ctypes.data_as(ctypes.c_void_p),
                                                  C.F64 if t.dtype == np.float64 else C.F32,
                                                  int(first_plane), int(t.shape[0])))

    def synth_tensor(self, kind=0, seed=4):
        self._check(self._L.mad_bench_synth_tensor(self._ctx, kind, seed))

    def comm_init(self, uid):
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        self._check(self._L.mad_comm_init(self._ctx, buf))

    def allreduce(self, values, op="sum"):
        """Reduce host floats over the ranks of this solver's communicator (sum / max),
        a barrier as a side effect (mad_comm_allreduce_host)."""
        v = np.ascontiguousarray(np.atleast_1d(np.asarray(values, dtype=np.float64))).copy()
        self._check(self._L.mad_comm_allreduce_host(
            self._ctx, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), v.size,
            {"sum": 0, "max": 1}[op]))
        return v

    def comm_init_local(self, group):
        """In-process transport: contexts sharing `group` exchange slabs directly."""
        self._check(self._L.mad_comm_init_local(self._ctx, int(group)))


    def comm_init_solo(self):
        """Measurement only (mad_comm_init_solo): this rank alone on its device, every
        exchange a device copy of the same bytes; timings, not results."""
        self._check(self._L.mad_comm_init_solo(self._ctx))

    def comm_init_rccl_solo(self):
        """Measurement only (mad_comm_init_rccl_solo): as comm_init_solo, every exchange through a
        single-rank RCCL communicator (ncclSend / ncclRecv to itself, the same bytes): RCCL's
        kernels and launch latency in the per-rank timing."""
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # one node: bootstrap on loopback
        self._check(self._L.mad_comm_init_rccl_solo(self._ctx))

    def setup(self):
        self._check(self._L.mad_setup(self._ctx))

    @property
    def num_levels(self):
        return self._L.mad_num_levels(self._ctx)

    def level_info(self, level):
        n = (ctypes.c_int64 * 3)()
        h = (ctypes.c_double * 3)()
        c = (ctypes.c_int32 * 3)()
        self._check(self._L.mad_level_info(self._ctx, level, n, h, c))
        return dict(shape=tuple(reversed(list(n)[: self.dim])), spacing=list(h)[: self.dim],
                    centering=list(c)[: self.dim])

    def shape_at(self, level):
        return self.level_info(level)["shape"]

    # ------------------------------------------------------------ kernel level
    def upload(self, level, which, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        if a.shape != self.shape_at(level):
            raise ValueError(f"level {level} array must have shape {self.shape_at(level)}")
        self._check(self._L.mad_upload(self._ctx, level, which,
                                       a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))

    def download(self, level, which):
        a = np.empty(self.shape_at(level), dtype=np.float64)
        self._check(self._L.mad_download(self._ctx, level, which,
                                         a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return a

    def fill(self, level, which, value):
        self._check(self._L.mad_fill(self._ctx, level, which, float(value)))

    def smooth(self, level, sweeps=1):
        self._check(self._L.mad_smooth(self._ctx, level, sweeps))

    def residual(self, level):
        v = ctypes.c_double()
        self._check(self._L.mad_residual(self._ctx, level, ctypes.byref(v)))
        return v.value

    def norm(self, level, which):
        v = ctypes.c_double()
        self._check(self._L.mad_norm(self._ctx, level, which, ctypes.byref(v)))
        return v.value

    def restrict(self, level):
        self._check(self._L.mad_restrict(self._ctx, level))

    def residual_restrict(self, level):
        """b[level+1] <- R (b - A x) in one pass where possible; returns True if fused."""
        f = ctypes.c_int32()
        self._check(self._L.mad_residual_restrict(self._ctx, level, ctypes.byref(f)))
        return bool(f.value)

    def interpolate(self, level):
        self._check(self._L.mad_interpolate(self._ctx, level))

    def prolongate_add(self, level):
        self._check(self._L.mad_prolongate_add(self._ctx, level))

    def coarse_solve(self):
        self._check(self._L.mad_coarse_solve(self._ctx))

    def vcycle(self):
        self._check(self._L.mad_vcycle(self._ctx))

    def fmg(self):
        self._check(self._L.mad_fmg(self._ctx))

    def synchronize(self):
        self._check(self._L.mad_synchronize(self._ctx))

    def synth_level(self, level, which, seed):
        self._check(self._L.mad_bench_synth_level(self._ctx, level, which, seed))

    # ------------------------------------------------------------ filter
    def run(self, image, out_dtype=np.float32):
        """GenerateData on a host image (numpy); returns (output, stats dict)."""
        img = np.ascontiguousarray(image)
        if img.shape != self.shape:
            raise ValueError(f"image shape {img.shape} != {self.shape}")
        out = np.empty(self.shape, dtype=out_dtype)
        st = C.MadStats()
        rc = C.check(self._L.mad_run(self._ctx, img.ctypes.data_as(ctypes.c_void_p),
                                     mad_dtype(img.dtype), out.ctypes.data_as(ctypes.c_void_p),
                                     mad_dtype(out_dtype), ctypes.byref(st)),
                     self._ctx, warn_not_converged=True)
        stats = st.as_dict()
        stats["converged"] = rc == C.OK
        stats["step_cycles"], stats["step_relres"] = [], []
        for s in range(st.steps):
            cy, rr = ctypes.c_uint32(), ctypes.c_double()
            self._check(self._L.mad_get_step_stats(self._ctx, s, ctypes.byref(cy),
                                                   ctypes.byref(rr)))
            stats["step_cycles"].append(cy.value)
            stats["step_relres"].append(rr.value)
        return out, stats

    def cycle_trace(self):
        """Convergence history of the last run (mad_get_cycle_trace): list of (time step,
        relres, seconds).  Default: one entry per cycle, seconds since the run started.  With
        options=capi.OPT_BENCHMARK_TRACE: the reference's -DBENCHMARK history -- level 0 after
        every sweep and after the coarse-grid correction of every level-0 V-cycle (2 nu + 1 per
        cycle; SMOOTHER: every sweep), seconds since the time step started
        (itkMultigridAnisotropicDiffusionImageFilter.hxx:147-151, 222-227, 401-409, 450-458,
        477-485)."""
        n = ctypes.c_uint32()
        self._check(self._L.mad_get_cycle_trace(self._ctx, 0, None, None, None, ctypes.byref(n)))
        k = n.value
        st = (ctypes.c_uint32 * max(k, 1))()
        rr = (ctypes.c_double * max(k, 1))()
        sec = (ctypes.c_double * max(k, 1))()
        self._check(self._L.mad_get_cycle_trace(self._ctx, k, st, rr, sec, ctypes.byref(n)))
        return [(st[q], rr[q], sec[q]) for q in range(k)]

    def placement_trials(self):
        """Level-0 sweep ms on each set of level-0 arrays the last setup tried (mad_placement_trials;
        the fastest was kept); [] when nothing was tuned."""
        n = ctypes.c_uint32()
        self._check(self._L.mad_placement_trials(self._ctx, 0, None, ctypes.byref(n)))
        k = n.value
        ms = (ctypes.c_double * max(k, 1))()
        self._check(self._L.mad_placement_trials(self._ctx, k, ms, ctypes.byref(n)))
        return [ms[q] for q in range(k)]

    @property
    def resolved_precision(self):
        """The precision mad_create resolved (PRECISION_AUTO -> FP32 or FP32_REFINE)."""
        d = C.MadDesc()
        self._check(self._L.mad_get_desc(self._ctx, ctypes.byref(d)))
        return d.precision

    def bench_smooth(self, level, sweeps):
        t, k, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint32()
        self._check(self._L.mad_bench_smooth(self._ctx, level, sweeps, ctypes.byref(t),
                                             ctypes.byref(k), ctypes.byref(n)))
        return t.value, k.value, n.value

    def bench_launch_times(self):
        """Per-launch kernel durations (ms) of the last bench_smooth."""
        buf = (ctypes.c_float * 4096)()
        n = ctypes.c_uint32()
        self._check(self._L.mad_bench_launch_times(self._ctx, buf, 4096, ctypes.byref(n)))
        return list(buf[:n.value])

    def smooth_kernel_name(self, level=0):
        buf = ctypes.create_string_buffer(256)
        self._check(self._L.mad_smooth_kernel_name(self._ctx, level, buf, 256))
        return buf.value.decode()

    def bench_vcycle(self, cycles):
        t = ctypes.c_double()
        self._check(self._L.mad_bench_vcycle(self._ctx, cycles, ctypes.byref(t)))
        return t.value


def comm_version():
    """(runtime, compiled) RCCL version codes (major*10000 + minor*100 + patch)."""
    r, c = ctypes.c_int32(), ctypes.c_int32()
    C.check(C.load().mad_comm_version(ctypes.byref(r), ctypes.byref(c)))
    return r.value, c.value


def comm_unique_id():
    buf = ctypes.create_string_buffer(128)
    C.check(C.load().mad_comm_unique_id(buf))
    return buf.raw
