/*
 * mad_ved.h -- C ABI of the VED (vessel enhancing diffusion) pipeline on the GPU:
 * the caller of the multigrid hot path.
 *
 * Replaces itk::VEDMultigridImageFilter (reference include/itkVEDMultigridImageFilter.{h,hxx},
 * cited VED.h / VED.hxx):
 *   multiscale Hessian (ComputeHessian, VED.hxx:158-173), eigen-analysis and Frangi-type
 *   vesselness with the per-voxel maximum over scales (UpdateVesselness / VesselnessFunction,
 *   VED.hxx:176-299), tensor construction (GenerateDiffusionTensor, VED.hxx:302-378) and
 *   the anisotropic-diffusion step through the MAD solver of mad.h (DiffusionStep,
 *   VED.hxx:381-402), iterated m_Iterations times (GenerateData, VED.hxx:63-155).
 *
 * Everything stays on the device between stages: image (fp64, the reference's internal
 * pixel type, VED.h:61), Hessian scratch (storage precision = desc.precision), response
 * and vessel direction (fp64), the fp64 SoA tensor handed to the solver in place.
 *
 * Hessian definition (parity unpinned: ITK's HessianRecursiveGaussianImageFilter is an
 * IIR approximation and ITK is not available to compare with): scale-normalised
 * (sigma^2) Gaussian second derivatives by separable correlation with moment-normalised
 * sampled Gaussian derivative kernels, radius ceil(4 sigma / h) per axis, borders
 * replicated.  See DESIGN.md "VED tensor generation" and oracle/ved_oracle.py.
 */
#ifndef MAD_VED_H
#define MAD_VED_H

#include "mad.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MAD_VED_MAX_SCALES 16

typedef struct mad_ved_desc {
  uint32_t abi_version;            /* MAD_ABI_VERSION */
  int64_t size[3];                 /* x, y, z (the filter is 3D only, VED.h:46) */
  double spacing[3];               /* image spacing (Hessian and solver), x first */
  /* VED parameters, VED.hxx:34-58 defaults */
  double alpha;                    /* 0.5 */
  double beta;                     /* 0.5 */
  double gamma;                    /* 5.0 */
  double epsilon;                  /* 0.01 */
  double omega;                    /* 5.0 */
  double sensitivity;              /* 10.0 */
  int32_t nscales;                 /* 5 */
  double scales[MAD_VED_MAX_SCALES];/* 0.300 0.482 0.775 1.245 2.000 (physical sigma) */
  uint32_t iterations;             /* 1  (outer VED iterations) */
  uint32_t diffusion_iterations;   /* 5  (MAD NumberOfSteps per iteration) */
  /* MAD parameters of DiffusionStep (VED.hxx:386-396; MaxCycles fixed at 100) */
  int32_t cycle;                   /* MAD_VCYCLE */
  double time_step;                /* 0.1 */
  double tolerance;                /* 1e-6 */
  uint32_t diffusion_iterations_per_grid; /* 2 */
  int32_t verbose;                 /* 0 */
  /* additions (no reference counterpart) */
  int32_t smoother;                /* mad_smoother, default MAD_GAUSS_SEIDEL (VED.h:44) */
  int32_t precision;               /* MAD_PRECISION_AUTO (default) / MAD_FP32 / MAD_FP32_REFINE: fp32
                                      Hessian, the diffusion solve as mad_create resolves it (AUTO:
                                      FP32_REFINE below tolerance 1e-6); MAD_FP64: fp64 throughout */
  int32_t device;                  /* HIP device, -1 = current */
  int32_t nranks;                  /* z-slab ranks of the diffusion step (1 = single GPU) */
  int32_t rank;
  int32_t hessian;                 /* mad_ved_hessian_kind: MAD_VED_HESSIAN_RECURSIVE (default, the
                                      reference's HessianRecursiveGaussianImageFilter operator,
                                      VED.hxx:158-173) or MAD_VED_HESSIAN_FIR (sampled Gaussian
                                      derivative taps, round 1) */
  uint32_t options;                /* MAD_VED_OPT_* bits, default 0 */
  int32_t reserved[4];
} mad_ved_desc;

/* mad_ved_desc.options: MAD_VED_OPT_LINE_WALK runs the recursive Hessian as one thread per
   line and output for every axis (ved_iir_k, the slow parity reference of the production passes,
   which equal it bit for bit) */
#define MAD_VED_OPT_LINE_WALK 1u

typedef enum mad_ved_hessian_kind {
  MAD_VED_HESSIAN_RECURSIVE = 0,
  MAD_VED_HESSIAN_FIR = 1
} mad_ved_hessian_kind;

typedef struct mad_ved_stats {
  uint32_t iterations;             /* VED iterations run */
  uint32_t total_cycles;           /* MAD cycles over all iterations and steps */
  double last_relres;              /* relative residual at the end of the last step */
  double tensor_ms;                /* device time: Hessian + vesselness + tensor, all iterations */
  double diffusion_ms;             /* MAD setup + solve, all iterations */
  int32_t stalled;                 /* any step ended by the fp32 stall guard */
  int32_t reserved[7];
} mad_ved_stats;

typedef struct mad_ved_ctx mad_ved_ctx;

int mad_ved_desc_init(mad_ved_desc *d);                    /* VED.hxx:34-58 defaults */
int mad_ved_create(const mad_ved_desc *d, mad_ved_ctx **out); /* VED::New() + setters */
void mad_ved_destroy(mad_ved_ctx *ctx);
const char *mad_ved_last_error(const mad_ved_ctx *ctx);

/* GenerateData (VED.hxx:63-155): host image in (any mad_dtype, x fastest), host image out
 * (static_cast, i.e. truncation for integer types, VED.hxx:145).
 * Multi-GPU (nranks > 1, after mad_ved_comm_init*): every rank passes the WHOLE image and
 * receives ITS z-slab (mad_slab_range planes).  The tensor generation is replicated on
 * every rank (like the solver's operator setup); the diffusion steps run on z-slabs
 * with RCCL halos; between VED iterations the slabs are all-gathered. */
int mad_ved_run(mad_ved_ctx *ctx, const void *in, int32_t in_dtype, void *out,
                int32_t out_dtype, mad_ved_stats *stats);
/* same with device buffers */
int mad_ved_run_device(mad_ved_ctx *ctx, const void *in, int32_t in_dtype, void *out,
                       int32_t out_dtype, mad_ved_stats *stats);

/* Join the ranks of a multi-GPU run (mad_comm_unique_id creates the id on rank 0);
 * the in-process variant runs ranks as threads on one device (tests). */
int mad_ved_comm_init(mad_ved_ctx *ctx, const void *uid128);
int mad_ved_comm_init_local(mad_ved_ctx *ctx, uint64_t group);
/* Measurement only (as mad_comm_init_solo): this rank alone on its device, every exchange a
 * device copy of the same bytes -- one rank's share of a partitioned run, timed on one GPU. */
int mad_ved_comm_init_solo(mad_ved_ctx *ctx);

/* One tensor generation on a host image (parity / inspection): all scales of
 * ComputeHessian + UpdateVesselness, then GenerateDiffusionTensor.  tensor_soa: 6 arrays
 * of N doubles [xx,xy,xz,yy,yz,zz]; response (may be NULL): N doubles, the maximum
 * vesselness over scales. */
int mad_ved_tensor(mad_ved_ctx *ctx, const void *image, int32_t dtype, double *tensor_soa,
                   double *response);
/* ComputeHessian at one scale (VED.hxx:158-173) on a host image: 6 arrays of N doubles. */
int mad_ved_hessian(mad_ved_ctx *ctx, const void *image, int32_t dtype, double sigma,
                    double *hessian_soa);

#ifdef __cplusplus
}
#endif
#endif
