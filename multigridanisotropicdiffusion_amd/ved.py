"""VED (vessel enhancing diffusion) on the GPU: the caller of the multigrid hot path.

Mirrors ``itk::VEDMultigridImageFilter<TIn, TOut, TSmoother>``
(include/itkVEDMultigridImageFilter.h:43-168): the same setters and defaults
(VED.hxx:34-58).  The whole pipeline -- multiscale Hessian, eigen-analysis,
vesselness, tensor and the MAD diffusion steps -- runs in libmad_hip.so through
include/mad_ved.h; there is no CPU fallback.

``VED`` is the low-level context (one image size); ``VEDMultigridImageFilter`` the
ITK-shaped facade.
"""
import ctypes

import numpy as np

from . import _capi as C
from .filters import Image, MultigridGaussSeidelSmoother
from .solver import mad_dtype


class VED:
    """One mad_ved_ctx.  shape: numpy (z, y, x); spacing x first."""

    def __init__(self, shape, spacing=(1.0, 1.0, 1.0), *, alpha=0.5, beta=0.5, gamma=5.0,
                 epsilon=0.01, omega=5.0, sensitivity=10.0,
                 scales=(0.300, 0.482, 0.775, 1.245, 2.000), iterations=1,
                 diffusion_iterations=5, cycle=C.VCYCLE, time_step=0.1, tolerance=1e-6,
                 diffusion_iterations_per_grid=2, verbose=False, smoother=C.GAUSS_SEIDEL,
                 precision=C.PRECISION_AUTO, device=-1, nranks=1, rank=0, hessian="recursive",
                 options=0):
        if len(shape) != 3:
            raise ValueError("VED is 3D (itkVEDMultigridImageFilter.h:46)")
        if len(scales) > C.VED_MAX_SCALES:
            raise ValueError(f"at most {C.VED_MAX_SCALES} scales")
        self._L = C.load()
        self.shape = tuple(int(v) for v in shape)
        d = C.VedDesc()
        C.check(self._L.mad_ved_desc_init(ctypes.byref(d)))
        for q, n in enumerate(reversed(self.shape)):
            d.size[q] = n
        for q in range(3):
            d.spacing[q] = float(spacing[q])
        d.alpha, d.beta, d.gamma = alpha, beta, gamma
        d.epsilon, d.omega, d.sensitivity = epsilon, omega, sensitivity
        d.nscales = len(scales)
        for q, sg in enumerate(scales):
            d.scales[q] = float(sg)
        d.iterations, d.diffusion_iterations = iterations, diffusion_iterations
        d.cycle, d.time_step, d.tolerance = int(cycle), float(time_step), float(tolerance)
        d.diffusion_iterations_per_grid = diffusion_iterations_per_grid
        d.verbose = int(bool(verbose))
        d.smoother, d.precision, d.device = int(smoother), int(precision), int(device)
        d.nranks, d.rank = int(nranks), int(rank)
        # ComputeHessian operator: "recursive" (ITK's HessianRecursiveGaussianImageFilter, the
        # reference's, default) or "fir" (sampled Gaussian derivative taps)
        d.hessian = {"recursive": C.VED_HESSIAN_RECURSIVE, "fir": C.VED_HESSIAN_FIR}[hessian]
        d.options = int(options)  # C.VED_OPT_LINE_WALK: the line-walk parity reference
        self.desc = d
        self.nranks, self.rank = int(nranks), int(rank)
        nz = self.shape[0]
        if nz % self.nranks:
            raise ValueError(f"nz {nz} not divisible by nranks {self.nranks}")
        per = nz // self.nranks
        self.slab = (per * self.rank, per * (self.rank + 1))  # this rank's output planes
        ctx = ctypes.c_void_p()
        rc = self._L.mad_ved_create(ctypes.byref(d), ctypes.byref(ctx))
        if rc != C.OK:
            raise C.MadError(rc, (self._L.mad_ved_last_error(None) or b"").decode())
        self._ctx = ctx

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.mad_ved_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    def comm_init(self, uid):
        """Join the RCCL communicator (uid from solver.comm_unique_id() on rank 0)."""
        self._check(self._L.mad_ved_comm_init(self._ctx, ctypes.c_char_p(bytes(uid))))

    def comm_init_local(self, group):
        """In-process transport: ranks as threads of this process on one device."""
        self._check(self._L.mad_ved_comm_init_local(self._ctx, ctypes.c_uint64(group)))

    def comm_init_solo(self):
        """Measurement only (mad_ved_comm_init_solo): one rank alone on its device."""
        self._check(self._L.mad_ved_comm_init_solo(self._ctx))

    def _check(self, rc):
        if rc != C.OK:
            raise C.MadError(rc, (self._L.mad_ved_last_error(self._ctx) or b"").decode())

    def _img(self, image):
        img = np.ascontiguousarray(image)
        if img.shape != self.shape:
            raise ValueError(f"image shape {img.shape} != {self.shape}")
        return img

    def run(self, image, out_dtype=np.float64):
        """GenerateData on a host image (the whole volume on every rank); returns (this
        rank's z-slab of the output -- the whole volume on one GPU --, stats dict)."""
        img = self._img(image)
        out = np.empty((self.slab[1] - self.slab[0],) + self.shape[1:], dtype=out_dtype)
        st = C.VedStats()
        rc = C.check(self._L.mad_ved_run(self._ctx, img.ctypes.data_as(ctypes.c_void_p),
                                         mad_dtype(img.dtype), out.ctypes.data_as(ctypes.c_void_p),
                                         mad_dtype(out_dtype), ctypes.byref(st)),
                     self._ctx, warn_not_converged=True, last_error=self._L.mad_ved_last_error)
        stats = st.as_dict()
        stats["converged"] = rc == C.OK
        return out, stats

    def tensor(self, image):
        """One tensor generation: (SoA tensor (6, z, y, x), max response (z, y, x))."""
        img = self._img(image)
        T = np.empty((6,) + self.shape)
        resp = np.empty(self.shape)
        dp = ctypes.POINTER(ctypes.c_double)
        self._check(self._L.mad_ved_tensor(self._ctx, img.ctypes.data_as(ctypes.c_void_p),
                                           mad_dtype(img.dtype), T.ctypes.data_as(dp),
                                           resp.ctypes.data_as(dp)))
        return T, resp

    def hessian(self, image, sigma):
        """ComputeHessian at one scale: (6, z, y, x), [xx,xy,xz,yy,yz,zz]."""
        img = self._img(image)
        H = np.empty((6,) + self.shape)
        self._check(self._L.mad_ved_hessian(self._ctx, img.ctypes.data_as(ctypes.c_void_p),
                                            mad_dtype(img.dtype), float(sigma),
                                            H.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return H


class VEDMultigridImageFilter:
    """itk::VEDMultigridImageFilter facade (VED.h:88-106 setters, VED.hxx:34-58 defaults)."""

    VCYCLE, FMG, SMOOTHER = C.VCYCLE, C.FMG, C.SMOOTHER

    def __init__(self, smoother=MultigridGaussSeidelSmoother, output_dtype=None,
                 precision=C.PRECISION_AUTO, device=-1, hessian="recursive"):
        self._smoother = smoother
        self._output_dtype = output_dtype
        self._hessian = hessian
        self._precision = precision
        self._device = device
        self._p = dict(alpha=0.5, beta=0.5, gamma=5.0, epsilon=0.01, omega=5.0, sensitivity=10.0,
                       scales=(0.300, 0.482, 0.775, 1.245, 2.000), iterations=1,
                       diffusion_iterations=5, cycle=C.VCYCLE, time_step=0.1, tolerance=1e-6,
                       diffusion_iterations_per_grid=2, verbose=False)
        self._input = None
        self._output = None
        self.stats = None

    @classmethod
    def New(cls, **kw):
        return cls(**kw)

    def SetAlpha(self, v): self._p["alpha"] = float(v)
    def SetBeta(self, v): self._p["beta"] = float(v)
    def SetGamma(self, v): self._p["gamma"] = float(v)
    def SetEpsilon(self, v): self._p["epsilon"] = float(v)
    def SetOmega(self, v): self._p["omega"] = float(v)
    def SetSensitivity(self, v): self._p["sensitivity"] = float(v)
    def SetScales(self, v): self._p["scales"] = tuple(float(s) for s in v)
    def SetIterations(self, v): self._p["iterations"] = int(v)
    def SetDiffusionIterations(self, v): self._p["diffusion_iterations"] = int(v)
    def SetCycle(self, v): self._p["cycle"] = int(v)
    def SetTimeStep(self, v): self._p["time_step"] = float(v)
    def SetTolerance(self, v): self._p["tolerance"] = float(v)
    def SetDiffusionIterationsPerGrid(self, v): self._p["diffusion_iterations_per_grid"] = int(v)
    def SetVerbose(self, v): self._p["verbose"] = bool(v)

    def SetInput(self, image):
        self._input = image if isinstance(image, Image) else Image(image)

    def GetOutput(self):
        return self._output

    def Update(self):
        """GenerateData (VED.hxx:63-155) on the GPU; output pixel type = input's
        unless output_dtype was given (the reference's TOutputImage)."""
        if self._input is None:
            raise RuntimeError("SetInput must be called before Update")
        img = self._input
        out_dtype = self._output_dtype or img.array.dtype
        v = VED(img.array.shape, img.spacing, smoother=self._smoother.smoother_id,
                precision=self._precision, device=self._device, hessian=self._hessian, **self._p)
        try:
            out, stats = v.run(img.array, out_dtype=out_dtype)
        finally:
            v.close()
        self.stats = stats
        self._output = Image(out, spacing=img.spacing, origin=img.origin)
        return self._output
