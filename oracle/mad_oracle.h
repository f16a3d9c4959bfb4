/*
 * mad_oracle.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * fp64 CPU restatement of nellogrb/MultigridAnisotropicDiffusion's multigrid
 * anisotropic-diffusion solver (ITK remote module, header-only C++).  It is the
 * checker for the HIP path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * PARITY UNPINNED: the reference ships no golden vectors or assertions
 * (test/itk2DDiffusionTest_GS.cxx:151 just returns EXIT_SUCCESS) and cannot be
 * compiled here (needs ITK + VXL, absent).  This restatement is pinned only by
 * analytic known-answer tests (row sums, dt=0 identity, transfer constants,
 * exact-solve fixed points, depth table) -- see tests/test_oracle.py.
 *
 * Every function cites the reference file:line it follows.
 */
#ifndef MAD_ORACLE_H
#define MAD_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

enum { ORA_VCYCLE = 0, ORA_FMG = 1, ORA_SMOOTHER = 2 };          /* CycleType, .h:123 */
enum { ORA_GS_LEX = 0, ORA_WJ = 1, ORA_GS_COLOR = 2 };            /* smoother plug-ins */
enum { ORA_VERTEX = 0, ORA_CELL = 1 };                             /* CoarseGridCenteringType */

typedef struct ora_ctx ora_ctx;

typedef struct ora_params {
  int cycle;              /* ORA_VCYCLE / ORA_FMG / ORA_SMOOTHER */
  int smoother;           /* ORA_GS_LEX (reference GS) / ORA_WJ / ORA_GS_COLOR (extension) */
  unsigned iterations_per_grid;
  unsigned max_cycles;
  unsigned number_of_steps;
  double tolerance;
  double omega;           /* WJ weight (reference default 2/3) */
  int verbose;
  int ncolors;            /* ORA_GS_COLOR: 2 (5/7-point) or 4 (9/19-point); 0 -> 4 */
} ora_params;

/* depth rule, include/mad/itkGridsHierarchy.hxx:36-59 */
int ora_max_depth(int dim, const long n0[3]);

/* Build hierarchy + DCA operators + coarsest LU (itkGridsHierarchy.hxx:30-204,
 * itkDirectSolver.hxx:32-88).  tensor_soa: ncomp arrays of N doubles, ITK
 * component order [xx,xy,xz,yy,yz,zz] (3D) / [xx,xy,yy] (2D). */
ora_ctx *ora_create(int dim, const long n0[3], const double h0[3],
                    const double *tensor_soa, double dt);
void ora_destroy(ora_ctx *c);
int ora_num_levels(const ora_ctx *c);
void ora_level_info(const ora_ctx *c, int level, long n[3], double h[3], int cent[3]);
/* 27 doubles per voxel, ITK Neighborhood index order (x fastest).  2D uses the oz=0 slice. */
const double *ora_stencil(const ora_ctx *c, int level);

/* smoothers / residual / transfers on one level */
void ora_gs_lex(const ora_ctx *c, int level, const double *x, const double *b, double *out);
void ora_gs_color(const ora_ctx *c, int level, int ncolors, const double *x, const double *b,
                  double *out);
/* ora_gs_color on nthreads host threads (OpenMP; identical result) -- CPU baseline only */
void ora_gs_color_omp(const ora_ctx *c, int level, int ncolors, const double *x, const double *b,
                      double *out, int nthreads);
void ora_wj(const ora_ctx *c, int level, double omega, const double *x, const double *b,
            double *out);
void ora_residual(const ora_ctx *c, int level, const double *x, const double *b, double *r);
/* fine level `level` -> coarse level `level+1` and back (centering of level+1) */
void ora_restrict(const ora_ctx *c, int level, const double *fine, double *coarse);
void ora_interpolate(const ora_ctx *c, int level, const double *coarse, double *fine);
void ora_direct_solve(const ora_ctx *c, const double *b, double *x);
double ora_l2norm(long n, const double *x);

/* whole filter: GenerateData (itkMultigridAnisotropicDiffusionImageFilter.hxx:104-297).
 * cycles_out / relres_out: arrays of number_of_steps entries (may be NULL). */
int ora_run(ora_ctx *c, const ora_params *p, const double *input, double *output,
            int *cycles_out, double *relres_out);

/* single V-cycle / FMG on level 0 (for per-cycle parity checks) */
void ora_vcycle(ora_ctx *c, const ora_params *p, const double *x, const double *b, double *out);
/* Verbose trace of the V-cycles run since the last call (params.verbose != 0): the per-level
 * relative residuals the reference prints (MAD.hxx:356-371, 384-411, 437-487), in print order:
 * level, it (-1 direct solver, 0 "initial" after the correction, n >= 1 after sweep n), relres.
 * Copies min(cap, count) entries, returns count, and clears the trace. */
long ora_take_trace(ora_ctx *c, long cap, int *level, int *it, double *relres);
void ora_fmg(ora_ctx *c, const ora_params *p, const double *b, double *out);

#ifdef __cplusplus
}
#endif
#endif
