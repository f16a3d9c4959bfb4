"""MI355X-native multigrid anisotropic diffusion (drop-in for the V-cycle hot path of
nellogrb/MultigridAnisotropicDiffusion).

The compute path is libmad_hip.so (hand-written HIP kernels for gfx950 behind the C
ABI in include/mad.h).  This package is the host-side mirror of the reference's
operator surface; it never falls back to a CPU implementation.
"""
from . import _capi as capi
from ._capi import (FMG, FP32, FP32_REFINE, FP64, GAUSS_SEIDEL, GAUSS_SEIDEL_LEX, PRECISION_AUTO,
                    SMOOTHER, VCYCLE, WEIGHTED_JACOBI, MadError, NotConvergedWarning)
from .filters import (Image, MultigridAnisotropicDiffusionImageFilter,
                      MultigridGaussSeidelLexSmoother, MultigridGaussSeidelSmoother,
                      MultigridWeightedJacobiSmoother, TensorImage)
from .solver import Solver, comm_unique_id, max_depth, slab_range
from .ved import VED, VEDMultigridImageFilter
from . import mhd

__all__ = [
    "capi", "Solver", "comm_unique_id", "max_depth", "slab_range", "Image", "TensorImage",
    "MultigridAnisotropicDiffusionImageFilter", "MultigridGaussSeidelSmoother",
    "MultigridGaussSeidelLexSmoother", "MultigridWeightedJacobiSmoother", "MadError",
    "VCYCLE", "FMG", "SMOOTHER", "GAUSS_SEIDEL", "GAUSS_SEIDEL_LEX", "WEIGHTED_JACOBI",
    "FP32", "FP32_REFINE", "FP64", "PRECISION_AUTO", "NotConvergedWarning", "VED", "VEDMultigridImageFilter", "mhd",
]
