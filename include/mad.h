/*
 * mad.h -- C ABI of the MI355X-native multigrid anisotropic-diffusion solver.
 *
 * This is the drop-in boundary for the reference's hot path
 * (nellogrb/MultigridAnisotropicDiffusion, ITK remote module).  Plain C types
 * only: sizes, pointers, enums.  Every entry point names the reference
 * interface it replaces (paths relative to the reference repository root):
 *
 *   MAD = include/itkMultigridAnisotropicDiffusionImageFilter.{h,hxx}
 *   SM  = include/mad/itkMultigridSmoother.h (smoother plug-in interface)
 *   IGO = include/mad/itkInterGridOperators.{h,hxx}
 *   GH  = include/mad/itkGridsHierarchy.{h,hxx}
 *   DS  = include/mad/itkDirectSolver.{h,hxx}
 *
 * Conventions
 *   - status: every call returns MAD_OK (0) or a mad_status error code; the
 *     message is available from mad_last_error(ctx) (or mad_last_error(NULL)
 *     for errors raised before a context exists).  The reference raises no
 *     errors (it has no validation); the checks here are additions.
 *   - images are x-fastest (ITK buffer order), size[] / spacing[] x first.
 *   - a context owns all device memory and one HIP stream; it is not
 *     re-entrant (same as the reference filter, MAD.h:185 m_CurrentLevel).
 */
#ifndef MAD_H
#define MAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAD_ABI_VERSION 1

typedef enum mad_status {
  MAD_OK = 0,
  MAD_ERR_INVALID = 1,     /* bad argument (size, dim, dtype, level, region mismatch) */
  MAD_ERR_STATE = 2,       /* call out of order (e.g. run before set_tensor) */
  MAD_ERR_DEVICE = 3,      /* HIP runtime error */
  MAD_ERR_COMM = 4,        /* RCCL / multi-GPU error */
  MAD_ERR_SINGULAR = 5,    /* coarsest operator singular */
  MAD_ERR_UNSUPPORTED = 6, /* valid request this build does not implement */
  MAD_ERR_NOMEM = 7,
  MAD_ERR_NUMERIC = 8,     /* NaN/Inf residual norm or diffusion tensor */
  MAD_ERR_NOT_CONVERGED = 9 /* warning, not a failure: the stall guard ended a time step above
                               Tolerance (the storage precision's floor, e.g. MAD_FP32 asked for
                               1e-10).  The output image and the stats are written; the reference
                               would have run on to MaxCycles (MAD.hxx:207-246). */
} mad_status;

/* MAD.h:123 enum CycleType { VCYCLE, FMG, SMOOTHER } -- same values */
typedef enum mad_cycle { MAD_VCYCLE = 0, MAD_FMG = 1, MAD_SMOOTHER = 2 } mad_cycle;

/* smoother plug-in (template argument TSmootherType, MAD.h:89-92) */
typedef enum mad_smoother {
  MAD_GAUSS_SEIDEL = 0,      /* multicolour GS: red-black for 5/7-point operators (isotropic or
                                diagonal tensor), 4 colours for 9/19-point (full tensor).
                                Replaces mad::MultigridGaussSeidelSmoother (parity at convergence). */
  MAD_GAUSS_SEIDEL_LEX = 1,  /* exact lexicographic GS order via hyperplane wavefronts
                                (per-sweep parity with the reference; slow, debug/parity mode) */
  MAD_WEIGHTED_JACOBI = 2    /* mad::MultigridWeightedJacobiSmoother (ω = 2/3 default) */
} mad_smoother;

typedef enum mad_dtype {
  MAD_U8 = 0, MAD_I8 = 1, MAD_U16 = 2, MAD_I16 = 3, MAD_U32 = 4, MAD_I32 = 5,
  MAD_F32 = 6, MAD_F64 = 7
} mad_dtype;

/* MAD_FP32_REFINE: fp32 hierarchy (storage + arithmetic) inside a mixed-precision defect
   correction -- level 0's iterate, rhs and residual in fp64 with the fp64 operator, one fp32
   cycle per correction -- so a solve reaches the reference's fp64 tolerances (1e-10).
   MAD_PRECISION_AUTO (the mad_desc_init default) is resolved by mad_create from the tolerance:
   MAD_FP32_REFINE when tolerance < 1e-6 (below what fp32 storage resolves; e.g. the reference
   tests' 1e-10, test/itk2DDiffusionTest_GS.cxx:97, test/itkVEDTest_GS.cxx:85), MAD_FP32
   otherwise; mad_get_desc then reports the resolved value */
typedef enum mad_precision {
  MAD_FP32 = 0, MAD_FP64 = 1, MAD_FP32_REFINE = 2, MAD_PRECISION_AUTO = 3
} mad_precision;
#define MAD_FP32_TOLERANCE_FLOOR 1e-6
/* MAD_FP32_REFINE V-cycle / FMG solves run their first cycles in plain fp32 (fp32 iterate, fp32
   residual norm) until relres drops below this, far above fp32's ~1e-7 floor; the iterate then moves
   to fp64 and the defect correction continues (SMOOTHER runs refine from the first sweep).  The
   fp32 phase also ends when a cycle reduces relres by less than 1 / MAD_REFINE_FP32_MIN_RATE (fp32's
   floor rises with the conditioning: large time steps, strong anisotropy) and one cycle before
   MaxCycles, so the defect correction always gets a turn (MaxCycles 1 refines from the start) */
#define MAD_REFINE_SWITCH_RELRES 1e-5
#define MAD_REFINE_FP32_MIN_RATE 0.5
/* defaults of mad_desc.min_slab_planes / min_slab_voxels (measured: profiles/r03_agglomeration.md,
   profiles/r03_rank_serial_ab.md) */
#define MAD_MIN_SLAB_PLANES 4
#define MAD_MIN_SLAB_VOXELS 131072
/* defaults of mad_desc.coarse_dense_max / coarse_block_unknowns (the DirectSolver, DS.hxx:32-147) */
#define MAD_COARSE_DENSE_MAX 8192
#define MAD_COARSE_BLOCK_UNKNOWNS 2048
/* the largest coarse_dense_max mad_create accepts (a dense inverse of n unknowns: 8 n^2 bytes of
   host memory, 16 n^2 of device memory, checked against hipMemGetInfo at setup) */
#define MAD_COARSE_DENSE_LIMIT 16384

typedef enum mad_tensor_kind {
  MAD_TENSOR_AUTO = 0,       /* detect from the level-0 tensor */
  MAD_TENSOR_ISOTROPIC = 1,  /* M = c(x) I */
  MAD_TENSOR_DIAGONAL = 2,   /* off-diagonals identically 0 */
  MAD_TENSOR_FULL = 3
} mad_tensor_kind;

/* per-level device arrays addressable through the kernel-level entry points */
typedef enum mad_which { MAD_X = 0 /* solution */, MAD_B = 1 /* rhs */, MAD_R = 2 /* residual */ } mad_which;

/* Filter parameters: the MultigridAnisotropicDiffusionImageFilter setters
 * (MAD.h:133-160) plus the image geometry and MI355X execution options.
 * mad_desc_init() fills the reference defaults (MAD.hxx:36-52). */
typedef struct mad_desc {
  uint32_t abi_version;          /* = MAD_ABI_VERSION */
  int32_t dim;                   /* TInputImage::ImageDimension: 2 or 3 */
  int64_t size[3];               /* image size, x first; size[2] = 1 in 2D */
  double spacing[3];             /* image spacing, x first (tensor spacing is ignored, as in GH:131) */
  int32_t cycle;                 /* SetCycle,              default MAD_VCYCLE */
  int32_t smoother;              /* TSmootherType,         default MAD_GAUSS_SEIDEL */
  uint32_t iterations_per_grid;  /* SetIterationsPerGrid,  default 2 */
  uint32_t max_cycles;           /* SetMaxCycles,          default 100 */
  uint32_t number_of_steps;      /* SetNumberOfSteps,      default 1 */
  double time_step;              /* SetTimeStep,           default 0.01 */
  double tolerance;              /* SetTolerance,          default 1e-6 */
  double omega;                  /* WJ weight (MultigridWeightedJacobiSmoother ctor), default 2/3 */
  int32_t verbose;               /* SetVerbose,            default 0 */
  int32_t precision;             /* MAD_PRECISION_AUTO (default), MAD_FP32, MAD_FP64 storage +
                                    arithmetic, or MAD_FP32_REFINE (fp32 cycles, fp64 defect
                                    correction) */
  int32_t stall_guard;           /* 1: end a time step once relres stops improving (a precision
                                    floor) -- mad_run then returns MAD_ERR_NOT_CONVERGED; default 1
                                    (the FP64 path never stalls above 1e-13) */
  int32_t device;                /* HIP device ordinal, -1 = current device */
  int32_t tensor_kind;           /* mad_tensor_kind, default AUTO */
  int32_t nranks;                /* z-slab decomposition: number of ranks (1 = single GPU) */
  int32_t rank;                  /* this rank */
  int32_t gs_kernel;             /* 3D multicolour GS: 0 auto (fused single-launch sweep
                                    gs_fused3_k on large levels, one launch per colour below),
                                    1 one launch per colour, 3 gs_fused3_k, 4 gs_fused3_k with
                                    the last z-chunk marched downward (the rank-slab single-
                                    launch form, selectable on one GPU for parity); all
                                    bit-identical */
  uint32_t options;              /* MAD_OPT_* bits, default 0 */
  int32_t min_slab_planes;       /* z-slab decomposition: a coarse level stays distributed while
                                    every rank keeps >= this many planes of it and >= min_slab_voxels
                                    voxels; the first level below is replicated on every rank
                                    (agglomeration).  0 = default (MAD_MIN_SLAB_PLANES) */
  int32_t min_slab_voxels;       /* 0 = default (MAD_MIN_SLAB_VOXELS): below ~128 K voxels per rank a
                                    level's exchanges (one RCCL round trip per sweep) cost more than
                                    sweeping the whole level on every rank */
  int32_t coarse_dense_max;      /* DirectSolver (DS.hxx:32-147): a coarsest level of up to this many
                                    unknowns is factored densely into an explicit inverse (one GEMV
                                    per solve); a larger one (thin volumes, or any axis < 12: the
                                    whole grid, GH.hxx:36-59) by the block-plane LU.  0 = default
                                    (MAD_COARSE_DENSE_MAX) */
  int32_t coarse_block_unknowns; /* block-plane LU: unknowns per diagonal block (max(1, this / plane
                                    size) planes of the longest axis).  0 = default
                                    (MAD_COARSE_BLOCK_UNKNOWNS) */
  int32_t reserved[3];
} mad_desc;

/* mad_desc.options: MAD_OPT_EAGER_RANK_VCYCLE keeps a multi-rank V-cycle eager instead of
   replaying its captured hipGraph (the reference of the graph-replay parity test) */
#define MAD_OPT_EAGER_RANK_VCYCLE 1u
/* MAD_OPT_OVERLAP_RANK_SWEEP: a rank slab's fused sweep runs split -- its two boundary chunks first,
   then the halo exchange on a communication stream beside the interior launch -- instead of the
   default serial form (one launch, then the exchange on the solver's stream).  Identical results.
   The sweep fills every CU, so an exchange kernel released beside it either waits for the sweep
   or delays the sweep's workgroups on the CUs it takes; the split also costs a short boundary
   launch and, in a captured V-cycle graph, a second stream that slows every node's launch
   (DESIGN.md "Multi-GPU"). */
#define MAD_OPT_OVERLAP_RANK_SWEEP 2u
/* MAD_OPT_PEER_HALO: on rank slabs, a level's fused GS sweep stores its GHOST edge planes straight into
   the neighbours' mailboxes (device memory mapped across processes: hipIpc handles exchanged over the
   communicator) and counts its tiles in their counters while the rest of the sweep runs; the next
   consumer of the ghost planes waits for the neighbours' counters and copies the mailbox in (one small
   launch) -- no exchange after the sweep.  Levels swept colour by colour push their edge planes into the
   mailboxes after the last colour pass instead (one small launch), and every descent into a distributed
   level pushes the new coarse b the same way, so a rank's V-cycle keeps one collective, the all-gather
   at the agglomeration level.  Identical results.  Setup-time option (mad_setup maps the windows,
   collectively). */
#define MAD_OPT_PEER_HALO 4u
/* MAD_OPT_COARSE_NO_CHAIN: the block-plane direct solver (mad_coarse.hpp) without its chain
   matrices KL_i / KU_i even where they fit -- what it does by itself for one-plane blocks whose
   KL / KU would take more than half the free device memory (e.g. a 512 x 512 x 8 whole-grid
   solve: 69 instead of 206 GB); one more launch per chain step, the same result to fp64 rounding.
   Applies to one-plane blocks only: blocks of several planes always keep KL / KU (far smaller than
   their Dinv blocks), and the setup's memory check counts them */
#define MAD_OPT_COARSE_NO_CHAIN 8u
/* MAD_OPT_BENCHMARK_TRACE: mad_get_cycle_trace returns the reference's -DBENCHMARK history instead of
   one entry per cycle -- in VCYCLE / FMG, level 0's relative residual after every pre-smoothing
   sweep, after the coarse-grid correction and after every post-smoothing sweep of every level-0
   V-cycle, FMG's included (MAD.hxx:401-409, 450-458, 477-485: 2 nu + 1 entries per V-cycle), in
   SMOOTHER after every sweep (:222-227); seconds since the time step's start (the reference resets
   m_Time per step, :158-163).  V-cycles then run eagerly with a residual norm read back after every
   level-0 sweep (a measurement mode, as the reference's); off by default.  In MAD_FP32_REFINE the
   correction cycles' entries are the fp32 residual of the correction equation over the step's
   ||b||, i.e. the relres of the updated iterate to fp32 rounding. */
#define MAD_OPT_BENCHMARK_TRACE 16u
/* MAD_OPT_NO_PLACEMENT_TUNE: keep level 0's first ping-pong allocation (mad_placement_trials; the A/B) */
#define MAD_OPT_NO_PLACEMENT_TUNE 32u
/* MAD_OPT_NO_RECORD_B: in CycleType SMOOTHER, level 0's records do not carry b (40-B records); the sweep
   reads b from the split copy the V-cycle layout uses (36-B records + 4 B) -- the A/B of the two forms */
#define MAD_OPT_NO_RECORD_B 64u

typedef struct mad_stats {
  uint32_t steps;                /* time steps run */
  uint32_t total_cycles;         /* V-cycles / FMG cycles / smoother iterations over all steps */
  uint32_t last_cycles;          /* cycles of the last time step */
  int32_t stalled;               /* 1 if the stall guard ended any step before tolerance */
  double last_relres;            /* relative residual ||b - A x|| / ||b|| at the end */
  double setup_ms;               /* hierarchy + operators + coarse LU */
  double solve_ms;               /* time-step loop (device time, host-synchronised) */
  uint32_t num_levels;
  int32_t tensor_kind;           /* resolved mad_tensor_kind */
  int32_t colors;                /* GS colours used (2 or 4) */
  int32_t reserved[5];
} mad_stats;

typedef struct mad_ctx mad_ctx;

/* ---------------------------------------------------------------- setup */
int mad_desc_init(mad_desc *d);                       /* MAD.hxx:36-52 defaults */
int mad_max_depth(int32_t dim, const int64_t size[3]);/* GH.hxx:36-59 depth rule (-1 on error) */
int mad_create(const mad_desc *d, mad_ctx **out);     /* MAD::New() + setters */
void mad_destroy(mad_ctx *ctx);
const char *mad_last_error(const mad_ctx *ctx);
int mad_get_desc(const mad_ctx *ctx, mad_desc *out);

/* SetDiffusionTensor (MAD.hxx:66-101): AoS symmetric tensors, ITK
 * SymmetricSecondRankTensor component order [xx,xy,xz,yy,yz,zz] (3D) /
 * [xx,xy,yy] (2D), dtype MAD_F32 or MAD_F64, of the whole (global) grid.  Copied
 * (cast to fp64) at call time; a rank of a z-slab decomposition copies only the
 * planes it stores (mad_tensor_planes) and keeps them across setups. */
int mad_set_tensor(mad_ctx *ctx, const void *host_aos, int32_t dtype);
int mad_set_tensor_device(mad_ctx *ctx, const void *dev_aos, int32_t dtype);
/* The global z planes [first, first + n) of the tensor this context stores: the whole
 * grid on one rank, the rank's slab plus ghost planes (the operator build's stencil
 * reach) on a z-slab rank.  mad_set_tensor_planes takes just those (or any covering
 * range starting at first_plane), so no process has to hold the global tensor. */
int mad_tensor_planes(const mad_ctx *ctx, int64_t *first_plane, int64_t *nplanes);
int mad_set_tensor_planes(mad_ctx *ctx, const void *host_aos, int32_t dtype,
                          int64_t first_plane, int64_t nplanes);

/* Build the grids hierarchy, per-level operators and the coarsest-grid direct
 * solver (GH.hxx:30-204, DS.hxx:32-88).  Implicit in mad_run; explicit for the
 * kernel-level entry points below. */
int mad_setup(mad_ctx *ctx);

/* ---------------------------------------------------------------- filter */
/* GenerateData (MAD.hxx:104-297): cast input -> internal precision, run
 * NumberOfSteps implicit-Euler steps, each solved by the chosen cycle to
 * Tolerance / MaxCycles, cast to the output type (static_cast semantics:
 * truncation toward zero for integer outputs, saturated to the type's range). */
int mad_run(mad_ctx *ctx, const void *host_in, int32_t in_dtype, void *host_out,
            int32_t out_dtype, mad_stats *stats);
/* same with device-resident input/output buffers (no PCIe in the solve) */
int mad_run_device(mad_ctx *ctx, const void *dev_in, int32_t in_dtype, void *dev_out,
                   int32_t out_dtype, mad_stats *stats);
/* per-time-step history of the last run */
int mad_get_step_stats(const mad_ctx *ctx, uint32_t step, uint32_t *cycles, double *relres);
/* Convergence history of the last run.  Default: one entry per cycle (V-cycle / FMG cycle /
 * smoother sweep): the time step it belongs to, the relative residual ||b - A x|| / ||b|| after it
 * and the seconds since the run started (host wall clock, the norm is read back every cycle).
 * This is the reference's -DBENCHMARK benchmark.txt (MAD.hxx:147-151, 222-227) only in SMOOTHER
 * mode; in VCYCLE / FMG the reference writes 2 nu + 1 entries per level-0 V-cycle (after every
 * sweep and after the correction, :401-409, 450-458, 477-485) and nothing per cycle -- that
 * history, with the reference's per-step clock, is what mad_desc.options MAD_OPT_BENCHMARK_TRACE
 * records.  Copies min(cap, total) entries (any pointer may be NULL); *count = total entries. */
int mad_get_cycle_trace(const mad_ctx *ctx, uint32_t cap, uint32_t *step, double *relres,
                        double *seconds, uint32_t *count);
/* Level-0 placement tuning of the last setup (no reference counterpart).  The level-0 sweep's speed
 * depends on where its ping-pong pair (x, t) landed in HBM: per allocation, each direction of the pair
 * sweeps in ~1.13 or ~1.24 ms at 512^3 (profiles/r06_placement.md).  Setup times both directions and,
 * while one is slower than the fastest direction seen, tries up to 7 fresh allocations of the pair,
 * keeping the fastest.  ms receives (forward, reverse) sweep ms per pair tried, in order; *count =
 * 2 x pairs, 0 when nothing was tuned (levels < 2^24 voxels, rank slabs, MAD_OPT_NO_PLACEMENT_TUNE). */
int mad_placement_trials(const mad_ctx *ctx, uint32_t cap, double *ms, uint32_t *count);

/* ---------------------------------------------------------------- hierarchy */
int mad_num_levels(const mad_ctx *ctx);               /* GH::GetMaxDepth() + 1 */
/* Host-only plan of the hierarchy for a descriptor (no device needed): returns
 * the number of levels (or -status on error) and fills level `level`'s global
 * size, spacing, centring and this rank's z-slab [z_begin, z_end); replicated
 * (agglomerated) levels report the full range with distributed = 0.
 * GH.hxx:36-106 plus the MI355X z-slab rule. */
int mad_plan_level(const mad_desc *d, int32_t level, int64_t size[3], double spacing[3],
                   int32_t centering[3], int64_t *z_begin, int64_t *z_end,
                   int32_t *distributed);
/* GetRegionAtLevel / GetSpacingAtLevel / GetVertexCenteringAtLevel (GH.h:96-106):
 * centering 0 = vertex, 1 = cell (level 0 reports vertex, GH.hxx:207).
 * size is this rank's slab on multi-GPU runs. */
int mad_level_info(const mad_ctx *ctx, int32_t level, int64_t size[3], double spacing[3],
                   int32_t centering[3]);

/* ---------------------------------------------------------------- kernel level */
/* Host <-> device copies of one level array (fp64 on the host, converted). */
int mad_upload(mad_ctx *ctx, int32_t level, int32_t which, const double *host);
int mad_download(mad_ctx *ctx, int32_t level, int32_t which, double *host);
int mad_fill(mad_ctx *ctx, int32_t level, int32_t which, double value);
/* SM.h:60-62 SingleIteration, applied `sweeps` times in place: x <- S(x, b). */
int mad_smooth(mad_ctx *ctx, int32_t level, uint32_t sweeps);
/* SM.h:66-68 ComputeResidual: r <- b - A x; optional ||r||_2 (MAD.hxx:496-515). */
int mad_residual(mad_ctx *ctx, int32_t level, double *norm_out);
/* MAD.hxx:496-515 L2Norm of one level array (fp64 accumulation). */
int mad_norm(mad_ctx *ctx, int32_t level, int32_t which, double *norm_out);
/* IGO.hxx:175-304 Restriction: b[level+1] <- R r[level]. */
int mad_restrict(mad_ctx *ctx, int32_t level);
/* MAD.hxx:389,413 the V-cycle descent b[level+1] <- R (b[level] - A x[level]) in one pass
 * (r[level] is not written) where the level is held whole by this rank (3D, >= 16 x 16);
 * elsewhere residual + restriction.  *fused (optional) = 1 if the one-pass kernel ran.
 * Bit-identical to mad_residual + mad_restrict. */
int mad_residual_restrict(mad_ctx *ctx, int32_t level, int32_t *fused);
/* IGO.hxx:45-172 Interpolation: x[level] <- P x[level+1]. */
int mad_interpolate(mad_ctx *ctx, int32_t level);
/* IGO Interpolation + correction add (MAD.hxx:422-435): x[level] += P x[level+1]. */
int mad_prolongate_add(mad_ctx *ctx, int32_t level);
/* DS.hxx:91-147 DirectSolver::Solve on the coarsest level: x[L] <- A_L^-1 b[L]. */
int mad_coarse_solve(mad_ctx *ctx);
/* MAD.hxx:341-493 VCycle on level 0 (x[0], b[0]) -- one cycle. */
int mad_vcycle(mad_ctx *ctx);
/* MAD.hxx:300-338 FullMultiGrid: x[0] <- FMG(b[0]). */
int mad_fmg(mad_ctx *ctx);
int mad_synchronize(mad_ctx *ctx);

/* ---------------------------------------------------------------- measurement */
/* Time `sweeps` smoother sweeps on `level` with HIP events on the context
 * stream: total wall (device) time, and the mean duration of the dominant
 * (sweep) kernel launches.  Used by bench.py. */
int mad_bench_smooth(mad_ctx *ctx, int32_t level, uint32_t sweeps, double *total_ms,
                     double *kernel_ms_mean, uint32_t *kernel_launches);
/* Per-launch durations (ms, HIP events) of the dominant kernel in the last
 * mad_bench_smooth call: up to `cap` values into `ms`, their count into *n
 * (median / min for the SURVEY 8(d) timing protocol). */
int mad_bench_launch_times(mad_ctx *ctx, float *ms, uint32_t cap, uint32_t *n);
/* Name of the kernel one smoother sweep on `level` launches, as rocprofv3 prints
 * its template arguments (e.g. "gs_fused3_k<float, 3, 64, 32, 1024, 4, 2>"), so a
 * profile summary can be matched to the bench line. */
int mad_smooth_kernel_name(mad_ctx *ctx, int32_t level, char *buf, int32_t len);
/* Time `cycles` V-cycles (device time). */
int mad_bench_vcycle(mad_ctx *ctx, uint32_t cycles, double *total_ms);
/* Deterministic synthetic inputs generated on the device (bench / smoke):
 * kind 0 = VED-form tensor, 1 = isotropic c(x)I, 2 = random-rotation SPD.
 * Counter-based, identical to tests/synth.py's *_dev formulas. */
int mad_bench_synth_tensor(mad_ctx *ctx, int32_t kind, uint64_t seed);
int mad_bench_synth_level(mad_ctx *ctx, int32_t level, int32_t which, uint64_t seed);

/* ---------------------------------------------------------------- multi-GPU */
/* z-slab decomposition over `nranks` processes, one GPU each, RCCL halos.
 * The unique id (128 bytes) is created on rank 0 and broadcast by the host. */
int mad_comm_unique_id(void *uid128);
int mad_comm_init(mad_ctx *ctx, const void *uid128);
/* In-process transport: the contexts of one process that pass the same `group`
 * (each with its own desc.rank, driven from its own host thread) exchange
 * ghost planes by device-to-device copies.  Same bytes as the RCCL path; used to
 * test the z-slab decomposition on a single GPU. */
int mad_comm_init_local(mad_ctx *ctx, uint64_t group);
/* Measurement only: this context runs as rank desc.rank of desc.nranks ALONE on its
 * device.  Every exchange becomes a device copy of the same bytes within its own arrays
 * (and the norm allreduce a no-op), so one rank's device time per sweep / V-cycle --
 * graph replay, boundary + interior launches, communication-stream overlap -- can be
 * timed on a one-GPU machine.  The values it computes are not the solution. */
int mad_comm_init_solo(mad_ctx *ctx);
/* Measurement only, as mad_comm_init_solo, but every exchange goes through RCCL: a single-rank
 * communicator on ctx's device, each grouped exchange a group of ncclSend / ncclRecv pairs to
 * itself moving the same bytes as mad_comm_init_solo's copies, the norm a one-rank
 * ncclAllReduce.  One rank's per-sweep / per-V-cycle time then includes RCCL's kernels, their
 * launch latency and their capture into the V-cycle graph (not the xGMI transfer time).
 * Results equal mad_comm_init_solo's bit for bit. */
int mad_comm_init_rccl_solo(mad_ctx *ctx);
/* Transport self-test on one GPU: a single-rank RCCL communicator runs the halo
 * exchange (grouped ncclSend/ncclRecv, both neighbours = this rank), the fp64
 * allreduce and the slab allgather the solver uses, on `device`, first eagerly and
 * then captured into a hipGraph and replayed twice (the multi-rank V-cycle graph
 * holds these operations); *max_err is the largest deviation from the expected
 * bytes over all runs (0 when the transport works). */
int mad_comm_selftest(int32_t device, double *max_err);
/* Host values reduced over the ranks of ctx's communicator (op 0 = sum, 1 = max),
 * in place; a barrier as a side effect.  Lets a host program (bench.py) synchronise
 * ranks and take its max-over-ranks timing over the solver's own RCCL communicator. */
int mad_comm_allreduce_host(mad_ctx *ctx, double *values, uint32_t n, int32_t op);
/* RCCL version the process bound at run time, and NCCL_VERSION_CODE of the headers
 * the library was compiled with (major*10000 + minor*100 + patch).  mad_comm_init
 * fails with MAD_ERR_COMM when their major.minor differ. */
int mad_comm_version(int32_t *runtime, int32_t *compiled);
/* slab [z_begin, z_end) of this rank for a global nz (even-aligned split) */
int mad_slab_range(int64_t nz, int32_t nranks, int32_t rank, int32_t align, int64_t *z_begin,
                   int64_t *z_end);

#ifdef __cplusplus
}
#endif
#endif /* MAD_H */
