"""ctypes binding of include/mad.h (the C ABI of libmad_hip.so).

The shared library is built in-tree (``python -m multigridanisotropicdiffusion_amd.build``
or ``__graft_entry__.build()``).  There is no fallback: if the library is
missing, importing this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmad_hip.so")

ABI_VERSION = 1

# mad_status
OK, ERR_INVALID, ERR_STATE, ERR_DEVICE, ERR_COMM, ERR_SINGULAR, ERR_UNSUPPORTED, ERR_NOMEM, \
    ERR_NUMERIC, ERR_NOT_CONVERGED = range(10)
# mad_cycle (itkMultigridAnisotropicDiffusionImageFilter.h:123)
VCYCLE, FMG, SMOOTHER = 0, 1, 2
# mad_smoother
GAUSS_SEIDEL, GAUSS_SEIDEL_LEX, WEIGHTED_JACOBI = 0, 1, 2
# mad_dtype
U8, I8, U16, I16, U32, I32, F32, F64 = range(8)
# mad_precision (PRECISION_AUTO, the default: FP32_REFINE below tolerance 1e-6, else FP32)
FP32, FP64, FP32_REFINE, PRECISION_AUTO = 0, 1, 2, 3
# mad_ved_hessian_kind
VED_HESSIAN_RECURSIVE, VED_HESSIAN_FIR = 0, 1
# mad_tensor_kind
TENSOR_AUTO, TENSOR_ISOTROPIC, TENSOR_DIAGONAL, TENSOR_FULL = range(4)
# mad_which
X, B, R = 0, 1, 2
# mad_desc.options / mad_ved_desc.options
OPT_EAGER_RANK_VCYCLE = 1
OPT_OVERLAP_RANK_SWEEP = 2
OPT_PEER_HALO = 4
OPT_COARSE_NO_CHAIN = 8
OPT_BENCHMARK_TRACE = 16  # the reference's -DBENCHMARK history in mad_get_cycle_trace (include/mad.h)
OPT_NO_PLACEMENT_TUNE = 32  # keep level 0's first allocation (mad_placement_trials)
OPT_NO_RECORD_B = 64  # SMOOTHER: level-0 records without b (the split-b sweep instead)
VED_OPT_LINE_WALK = 1

EXPORTS = (
    "mad_desc_init", "mad_max_depth", "mad_create", "mad_destroy", "mad_last_error",
    "mad_get_desc", "mad_set_tensor", "mad_set_tensor_device", "mad_tensor_planes",
    "mad_set_tensor_planes", "mad_setup", "mad_run",
    "mad_run_device", "mad_get_step_stats", "mad_get_cycle_trace", "mad_placement_trials", "mad_num_levels", "mad_plan_level",
    "mad_level_info", "mad_upload",
    "mad_download", "mad_fill", "mad_smooth", "mad_residual", "mad_norm", "mad_restrict",
    "mad_residual_restrict",
    "mad_interpolate", "mad_prolongate_add", "mad_coarse_solve", "mad_vcycle", "mad_fmg",
    "mad_synchronize", "mad_bench_smooth", "mad_bench_launch_times", "mad_smooth_kernel_name", "mad_bench_vcycle", "mad_bench_synth_tensor",
    "mad_bench_synth_level", "mad_comm_unique_id", "mad_comm_init", "mad_comm_init_local", "mad_comm_init_solo",
    "mad_comm_init_rccl_solo",
    "mad_comm_selftest", "mad_slab_range", "mad_comm_allreduce_host", "mad_comm_version",
    # include/mad_ved.h
    "mad_ved_desc_init", "mad_ved_create", "mad_ved_destroy", "mad_ved_last_error",
    "mad_ved_run", "mad_ved_run_device", "mad_ved_comm_init", "mad_ved_comm_init_local",
    "mad_ved_comm_init_solo",
    "mad_ved_tensor", "mad_ved_hessian",
)

VED_MAX_SCALES = 16


class MadDesc(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_uint32),
        ("dim", ctypes.c_int32),
        ("size", ctypes.c_int64 * 3),
        ("spacing", ctypes.c_double * 3),
        ("cycle", ctypes.c_int32),
        ("smoother", ctypes.c_int32),
        ("iterations_per_grid", ctypes.c_uint32),
        ("max_cycles", ctypes.c_uint32),
        ("number_of_steps", ctypes.c_uint32),
        ("time_step", ctypes.c_double),
        ("tolerance", ctypes.c_double),
        ("omega", ctypes.c_double),
        ("verbose", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("stall_guard", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("tensor_kind", ctypes.c_int32),
        ("nranks", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("gs_kernel", ctypes.c_int32),
        ("options", ctypes.c_uint32),
        ("min_slab_planes", ctypes.c_int32),
        ("min_slab_voxels", ctypes.c_int32),
        ("coarse_dense_max", ctypes.c_int32),
        ("coarse_block_unknowns", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 3),
    ]


class MadStats(ctypes.Structure):
    _fields_ = [
        ("steps", ctypes.c_uint32),
        ("total_cycles", ctypes.c_uint32),
        ("last_cycles", ctypes.c_uint32),
        ("stalled", ctypes.c_int32),
        ("last_relres", ctypes.c_double),
        ("setup_ms", ctypes.c_double),
        ("solve_ms", ctypes.c_double),
        ("num_levels", ctypes.c_uint32),
        ("tensor_kind", ctypes.c_int32),
        ("colors", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 5),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


class VedDesc(ctypes.Structure):
    """mad_ved_desc (include/mad_ved.h)."""
    _fields_ = [
        ("abi_version", ctypes.c_uint32),
        ("size", ctypes.c_int64 * 3),
        ("spacing", ctypes.c_double * 3),
        ("alpha", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("epsilon", ctypes.c_double),
        ("omega", ctypes.c_double),
        ("sensitivity", ctypes.c_double),
        ("nscales", ctypes.c_int32),
        ("scales", ctypes.c_double * VED_MAX_SCALES),
        ("iterations", ctypes.c_uint32),
        ("diffusion_iterations", ctypes.c_uint32),
        ("cycle", ctypes.c_int32),
        ("time_step", ctypes.c_double),
        ("tolerance", ctypes.c_double),
        ("diffusion_iterations_per_grid", ctypes.c_uint32),
        ("verbose", ctypes.c_int32),
        ("smoother", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("nranks", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("hessian", ctypes.c_int32),
        ("options", ctypes.c_uint32),
        ("reserved", ctypes.c_int32 * 4),
    ]


class VedStats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_uint32),
        ("total_cycles", ctypes.c_uint32),
        ("last_relres", ctypes.c_double),
        ("tensor_ms", ctypes.c_double),
        ("diffusion_ms", ctypes.c_double),
        ("stalled", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 7),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


class MadError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"mad error {code}: {msg}")
        self.code = code


_lib = None


def load():
    """Load libmad_hip.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # MAD_HIP_LIB: an alternative build of the same library (A/B measurements)
    path = os.environ.get("MAD_HIP_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build the HIP library first "
            "(python -m multigridanisotropicdiffusion_amd.build)")
    L = ctypes.CDLL(path)
    vp, i32, u32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64, \
        ctypes.c_double
    dp = ctypes.POINTER(ctypes.c_double)
    i64p = ctypes.POINTER(ctypes.c_int64)
    i32p = ctypes.POINTER(ctypes.c_int32)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    sig = {
        "mad_desc_init": ([ctypes.POINTER(MadDesc)], i32),
        "mad_max_depth": ([i32, i64p], i32),
        "mad_create": ([ctypes.POINTER(MadDesc), ctypes.POINTER(vp)], i32),
        "mad_destroy": ([vp], None),
        "mad_last_error": ([vp], ctypes.c_char_p),
        "mad_get_desc": ([vp, ctypes.POINTER(MadDesc)], i32),
        "mad_set_tensor": ([vp, vp, i32], i32),
        "mad_set_tensor_device": ([vp, vp, i32], i32),
        "mad_tensor_planes": ([vp, i64p, i64p], i32),
        "mad_set_tensor_planes": ([vp, vp, i32, ctypes.c_int64, ctypes.c_int64], i32),
        "mad_setup": ([vp], i32),
        "mad_run": ([vp, vp, i32, vp, i32, ctypes.POINTER(MadStats)], i32),
        "mad_run_device": ([vp, vp, i32, vp, i32, ctypes.POINTER(MadStats)], i32),
        "mad_get_step_stats": ([vp, u32, u32p, dp], i32),
        "mad_get_cycle_trace": ([vp, u32, u32p, dp, dp, u32p], i32),
        "mad_placement_trials": ([vp, u32, dp, u32p], i32),
        "mad_num_levels": ([vp], i32),
        "mad_plan_level": ([ctypes.POINTER(MadDesc), i32, i64p, dp, i32p, i64p, i64p, i32p], i32),
        "mad_level_info": ([vp, i32, i64p, dp, i32p], i32),
        "mad_upload": ([vp, i32, i32, dp], i32),
        "mad_download": ([vp, i32, i32, dp], i32),
        "mad_fill": ([vp, i32, i32, dbl], i32),
        "mad_smooth": ([vp, i32, u32], i32),
        "mad_residual": ([vp, i32, dp], i32),
        "mad_norm": ([vp, i32, i32, dp], i32),
        "mad_restrict": ([vp, i32], i32),
        "mad_residual_restrict": ([vp, i32, ctypes.POINTER(i32)], i32),
        "mad_interpolate": ([vp, i32], i32),
        "mad_prolongate_add": ([vp, i32], i32),
        "mad_coarse_solve": ([vp], i32),
        "mad_vcycle": ([vp], i32),
        "mad_fmg": ([vp], i32),
        "mad_synchronize": ([vp], i32),
        "mad_bench_smooth": ([vp, i32, u32, dp, dp, u32p], i32),
        "mad_bench_launch_times": ([vp, ctypes.POINTER(ctypes.c_float), u32, u32p], i32),
        "mad_smooth_kernel_name": ([vp, i32, ctypes.c_char_p, i32], i32),
        "mad_bench_vcycle": ([vp, u32, dp], i32),
        "mad_bench_synth_tensor": ([vp, i32, ctypes.c_uint64], i32),
        "mad_bench_synth_level": ([vp, i32, i32, ctypes.c_uint64], i32),
        "mad_comm_unique_id": ([vp], i32),
        "mad_comm_init": ([vp, vp], i32),
        "mad_comm_init_local": ([vp, ctypes.c_uint64], i32),
        "mad_comm_init_solo": ([vp], i32),
        "mad_comm_init_rccl_solo": ([vp], i32),
        "mad_comm_selftest": ([i32, dp], i32),
        "mad_slab_range": ([i64, i32, i32, i32, i64p, i64p], i32),
        "mad_comm_allreduce_host": ([vp, dp, u32, i32], i32),
        "mad_comm_version": ([ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)], i32),
        "mad_ved_desc_init": ([ctypes.POINTER(VedDesc)], i32),
        "mad_ved_create": ([ctypes.POINTER(VedDesc), ctypes.POINTER(vp)], i32),
        "mad_ved_destroy": ([vp], None),
        "mad_ved_last_error": ([vp], ctypes.c_char_p),
        "mad_ved_run": ([vp, vp, i32, vp, i32, ctypes.POINTER(VedStats)], i32),
        "mad_ved_run_device": ([vp, vp, i32, vp, i32, ctypes.POINTER(VedStats)], i32),
        "mad_ved_comm_init": ([vp, vp], i32),
        "mad_ved_comm_init_local": ([vp, ctypes.c_uint64], i32),
        "mad_ved_comm_init_solo": ([vp], i32),
        "mad_ved_tensor": ([vp, vp, i32, dp, dp], i32),
        "mad_ved_hessian": ([vp, vp, i32, dbl, dp], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


class NotConvergedWarning(RuntimeWarning):
    """MAD_ERR_NOT_CONVERGED: the stall guard ended a time step above Tolerance (the output
    is still written); the ITK filter would report it as a warning."""


def check(rc, ctx=None, warn_not_converged=False, last_error=None):
    if rc != OK:
        msg = (last_error or load().mad_last_error)(ctx)
        msg = msg.decode() if msg else ""
        if rc == ERR_NOT_CONVERGED and warn_not_converged:
            import warnings
            warnings.warn(msg, NotConvergedWarning, stacklevel=3)
            return rc
        raise MadError(rc, msg)
    return rc


def default_desc():
    d = MadDesc()
    check(load().mad_desc_init(ctypes.byref(d)))
    return d
