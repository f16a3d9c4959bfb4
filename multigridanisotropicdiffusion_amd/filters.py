"""ITK-shaped Python facade of the reference filter surface.

Mirrors ``itk::MultigridAnisotropicDiffusionImageFilter<TIn, TOut, TSmoother>``
(include/itkMultigridAnisotropicDiffusionImageFilter.h:89-160): the same
setter names, CycleType values and defaults, with the smoother chosen by a
class (the reference's template argument).  Images are ``Image`` objects
(numpy buffer + spacing + origin); tensors are ``Image`` objects whose pixel
is the ITK SymmetricSecondRankTensor component vector [xx,xy,xz,yy,yz,zz] /
[xx,xy,yy] (last axis), or plain arrays.  Update() runs on the GPU through the
C ABI (include/mad.h); there is no CPU fallback.
"""
import numpy as np

from . import _capi as C
from .solver import Solver


class Image:
    """Minimal itk::Image stand-in: buffer (numpy, (z,y,x)), spacing and origin x first."""

    def __init__(self, array, spacing=None, origin=None):
        self.array = np.asarray(array)
        nd = self.dim
        self.spacing = tuple(float(s) for s in (spacing if spacing is not None else [1.0] * nd))
        self.origin = tuple(float(o) for o in (origin if origin is not None else [0.0] * nd))

    @property
    def dim(self):
        return self.array.ndim

    def GetSpacing(self):
        return self.spacing

    def GetOrigin(self):
        return self.origin

    def GetBufferAsArray(self):
        return self.array

    def GetLargestPossibleRegion(self):
        return dict(index=(0,) * self.dim, size=tuple(reversed(self.array.shape)))


class TensorImage(Image):
    """Image of SymmetricSecondRankTensor pixels: array shape (*image_shape, ncomp)."""

    @property
    def dim(self):
        return self.array.ndim - 1


# smoother plug-ins (template argument TSmootherType)
class MultigridGaussSeidelSmoother:
    """mad::MultigridGaussSeidelSmoother (include/mad/itkMultigridGaussSeidelSmoother.h).
    GPU form: multicolour GS (red-black for 5/7-point operators, 4 colours for
    9/19-point); same fixed point, parity at convergence."""
    smoother_id = C.GAUSS_SEIDEL
    weight = 2.0 / 3.0


class MultigridGaussSeidelLexSmoother(MultigridGaussSeidelSmoother):
    """Exact lexicographic GS order (hyperplane wavefronts): per-sweep parity mode."""
    smoother_id = C.GAUSS_SEIDEL_LEX


class MultigridWeightedJacobiSmoother:
    """mad::MultigridWeightedJacobiSmoother (weight 2/3 by default,
    include/mad/itkMultigridWeightedJacobiSmoother.hxx:174-191)."""
    smoother_id = C.WEIGHTED_JACOBI
    weight = 2.0 / 3.0

    def __init__(self, weight=2.0 / 3.0):
        self.weight = weight


class MultigridAnisotropicDiffusionImageFilter:
    """Implicit-Euler anisotropic diffusion, (I - dt div(M grad)) u^{n+1} = u^n, by
    multigrid (V-cycle / FMG / smoother only)."""

    # enum CycleType { VCYCLE, FMG, SMOOTHER } (.h:123)
    VCYCLE, FMG, SMOOTHER = C.VCYCLE, C.FMG, C.SMOOTHER

    def __init__(self, smoother=MultigridGaussSeidelSmoother, output_dtype=np.float32,
                 precision=C.PRECISION_AUTO, device=-1, benchmark=False):
        # benchmark: the reference's -DBENCHMARK build (.hxx:145-151): Update() records the
        # relres / seconds history the reference writes to benchmark.txt (GetBenchmarkOutput)
        self._benchmark = bool(benchmark)
        self.benchmark_trace = None
        self._smoother = smoother
        self._output_dtype = np.dtype(output_dtype)
        self._precision = precision
        self._device = device
        # defaults, include/itkMultigridAnisotropicDiffusionImageFilter.hxx:36-52
        self._time_step = 0.01
        self._number_of_steps = 1
        self._cycle = self.VCYCLE
        self._iterations_per_grid = 2
        self._tolerance = 1e-6
        self._max_cycles = 100
        self._verbose = False
        self._input = None
        self._tensor = None
        self._output = None
        self.stats = None

    @classmethod
    def New(cls, **kw):
        return cls(**kw)

    # setters (.h:133-160)
    def SetCycle(self, cycle):
        self._cycle = int(cycle)

    def SetIterationsPerGrid(self, n):
        self._iterations_per_grid = int(n)

    def SetMaxCycles(self, n):
        self._max_cycles = int(n)

    def SetNumberOfSteps(self, n):
        self._number_of_steps = int(n)

    def SetTimeStep(self, dt):
        self._time_step = float(dt)

    def SetTolerance(self, tol):
        self._tolerance = float(tol)

    def SetVerbose(self, v):
        self._verbose = bool(v)

    def SetDiffusionTensor(self, tensor):
        """Copied and cast to fp64 at call time, like .hxx:66-101."""
        arr = tensor.array if isinstance(tensor, Image) else np.asarray(tensor)
        self._tensor = np.array(arr, dtype=np.float64, copy=True)

    def SetInput(self, image):
        self._input = image if isinstance(image, Image) else Image(image)

    def GetOutput(self):
        return self._output

    def GetBenchmarkOutput(self):
        """The lines the reference's -DBENCHMARK build writes to benchmark.txt, "relres_seconds"
        (.hxx:222-227, 401-409, 450-458, 477-485); needs benchmark=True."""
        if self.benchmark_trace is None:
            raise RuntimeError("construct with benchmark=True and call Update first")
        return [f"{rr:g}_{sec:g}" for _, rr, sec in self.benchmark_trace]

    def Update(self):
        """GenerateData (.hxx:104-297) on the GPU."""
        if self._input is None or self._tensor is None:
            raise RuntimeError("SetInput and SetDiffusionTensor must be called before Update")
        img = self._input
        smoother = self._smoother
        weight = getattr(smoother, "weight", 2.0 / 3.0)
        s = Solver(img.array.shape, img.spacing, time_step=self._time_step, cycle=self._cycle,
                   smoother=smoother.smoother_id, iterations_per_grid=self._iterations_per_grid,
                   max_cycles=self._max_cycles, number_of_steps=self._number_of_steps,
                   tolerance=self._tolerance, omega=weight, verbose=self._verbose,
                   precision=self._precision, device=self._device,
                   options=C.OPT_BENCHMARK_TRACE if self._benchmark else 0)
        try:
            s.set_tensor(self._tensor)
            out, stats = s.run(img.array, out_dtype=self._output_dtype)
            if self._benchmark:
                self.benchmark_trace = s.cycle_trace()
        finally:
            s.close()
        self.stats = stats
        self._output = Image(out, spacing=img.spacing, origin=img.origin)  # origin: .hxx:286
        return self._output
