/*
 * mad_oracle.c -- TEST INFRASTRUCTURE ONLY.  See mad_oracle.h.
 *
 * Line-faithful fp64 restatement of the reference's algorithm.  Citations are
 * relative to /root/reference (nellogrb/MultigridAnisotropicDiffusion):
 *   GH  = include/mad/itkGridsHierarchy.hxx
 *   GS  = include/mad/itkMultigridGaussSeidelSmoother.hxx
 *   WJ  = include/mad/itkMultigridWeightedJacobiSmoother.hxx
 *   IGO = include/mad/itkInterGridOperators.{h,hxx}
 *   DS  = include/mad/itkDirectSolver.hxx
 *   MAD = include/itkMultigridAnisotropicDiffusionImageFilter.hxx
 *
 * PARITY UNPINNED (no reference golden vectors exist; reference not buildable).
 *
 * Deliberate, documented differences (rounding-level only):
 *  - the direct solver is a partial-pivot LU instead of vnl_sparse_lu
 *    (DS:81-86,129): dense up to ORA_DENSE_MAX unknowns, banded above it (the
 *    unknowns renumbered with the shortest axis innermost, LAPACK gbtrf/gbtrs
 *    restated) -- all are exact solvers, results agree to fp64 rounding;
 *  - Interpolation scatters interior coarse points first and then all border
 *    points in x-fastest order; ITK's ImageBoundaryFacesCalculator visits the
 *    border faces in a different order (IGO.hxx:93-167), which only permutes
 *    fp64 additions into the same fine voxel.
 *  - ORA_GS_COLOR is an extension (multicolour GS, the GPU smoother); the
 *    reference Gauss-Seidel is ORA_GS_LEX.
 */
#include "mad_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MAXLEV 32

typedef struct {
  long n[3];
  double h[3];
  int cent[3]; /* centering of this level w.r.t. the finer one (level 0: vertex, GH:207) */
  long N;
  double *A; /* N*27 stencil (StencilImage, itkStencilImage.h:48-111) */
} ora_level;

struct ora_ctx {
  int dim;
  int nlev; /* maxDepth + 1 */
  ora_level lev[MAXLEV];
  int noff;          /* active offsets: 19 (3D, corners removed GH:632-653) / 9 (2D) */
  int off[27][3];    /* in Neighborhood index order (itkStencilImage.hxx:51-67) */
  /* coarsest-level LU (replaces vnl_sparse_lu, DS:32-88): dense (kl == -1) or banded */
  long nlu;
  double *lu;
  long *piv;
  long kl, ku;  /* banded: sub/super-diagonals of A in the renumbered order */
  long *perm;   /* banded: natural (x-fastest) index -> band index */
  /* verbose trace (ora_take_trace) */
  long ntr, captr;
  int *tr_level, *tr_it;
  double *tr_rel;
};

static void trace_push(ora_ctx *c, int level, int it, double rel) {
  if (c->ntr == c->captr) {
    c->captr = c->captr ? 2 * c->captr : 64;
    c->tr_level = (int *)realloc(c->tr_level, sizeof(int) * c->captr);
    c->tr_it = (int *)realloc(c->tr_it, sizeof(int) * c->captr);
    c->tr_rel = (double *)realloc(c->tr_rel, sizeof(double) * c->captr);
  }
  c->tr_level[c->ntr] = level;
  c->tr_it[c->ntr] = it;
  c->tr_rel[c->ntr] = rel;
  ++c->ntr;
}

/* dense LU up to this many unknowns (the golden fixtures' sizes), banded above */
#define ORA_DENSE_MAX 4096

static inline int nbidx(int ox, int oy, int oz) { return (ox + 1) + 3 * (oy + 1) + 9 * (oz + 1); }

static inline int tcomp(int dim, int d, int d2) {
  if (d > d2) { int t = d; d = d2; d2 = t; }
  return d * dim - d * (d - 1) / 2 + (d2 - d);
}

/* ---------------------------------------------------------------- depth rule */
/* GH:36-59: halve every axis (even -> n/2, odd -> (n-1)/2+1) until one axis < 6 */
int ora_max_depth(int dim, const long n0[3]) {
  unsigned long gs[3] = {(unsigned long)n0[0], (unsigned long)n0[1], (unsigned long)n0[2]};
  int coarsest = 0;
  int numberOfLevels = 1;
  while (!coarsest) {
    for (int d = 0; d < dim; ++d) {
      gs[d] = (gs[d] % 2 == 0) ? gs[d] / 2 : ((gs[d] - 1) / 2) + 1;
      if (gs[d] < 6) coarsest = 1;
    }
    ++numberOfLevels;
  }
  --numberOfLevels;
  return numberOfLevels - 1;
}

/* ---------------------------------------------------------------- transfers */
/* 1-D tables, IGO.h:101-127: [position][offset + radius] */
static const double INT_V[3][3] = {{0., 1., 0.5}, {0.5, 1., 0.5}, {0.5, 1., 0.}};
static const double INT_C[3][5] = {{0., 0., 1., 0.75, 0.25},
                                   {0., 0.25, 0.75, 0.75, 0.25},
                                   {0., 0.25, 0.75, 1., 0.}};
static const double RES_V[3][3] = {{0., 1., 0.}, {0.25, 0.5, 0.25}, {0., 1., 0.}};
static const double RES_C[3][5] = {{0., 0., 0.5, 0.375, 0.125},
                                   {0., 0.125, 0.375, 0.375, 0.125},
                                   {0., 0.125, 0.375, 0.5, 0.}};
enum { P_LEFT = 0, P_INTERIOR = 1, P_RIGHT = 2 };

typedef struct {
  int dim;
  int r[3];          /* stencil radius per dim (vertex 1, cell 2), IGO.hxx:318-319 */
  int size[3];       /* 2r+1 */
  int count;         /* product of sizes */
  int nact;          /* active offsets: nonzero in the interior stencil, IGO.hxx:88-90 */
  int act[125][3];
} xfer_t;

/* GenerateStencil, IGO.hxx:307-353: tensor product of 1-D stencils */
static double gen_weight(const xfer_t *x, const int cent[3], const int pos[3], const int o[3],
                         int interp) {
  double value = 1;
  for (int d = 0; d < x->dim; ++d) {
    int k = o[d] + x->r[d];
    if (cent[d] == ORA_VERTEX)
      value *= interp ? INT_V[pos[d]][k] : RES_V[pos[d]][k];
    else
      value *= interp ? INT_C[pos[d]][k] : RES_C[pos[d]][k];
  }
  return value;
}

static void xfer_init(xfer_t *x, int dim, const int cent[3], int interp) {
  x->dim = dim;
  x->count = 1;
  for (int d = 0; d < 3; ++d) {
    x->r[d] = (d < dim) ? (cent[d] == ORA_VERTEX ? 1 : 2) : 0;
    x->size[d] = 2 * x->r[d] + 1;
    x->count *= x->size[d];
  }
  int pos[3] = {P_INTERIOR, P_INTERIOR, P_INTERIOR};
  x->nact = 0;
  for (int i = 0; i < x->count; ++i) { /* Neighborhood index order, x fastest */
    int o[3];
    int t = i;
    for (int d = 0; d < 3; ++d) {
      o[d] = t % x->size[d] - x->r[d];
      t /= x->size[d];
    }
    if (gen_weight(x, cent, pos, o, interp) != 0.) {
      memcpy(x->act[x->nact], o, sizeof(o));
      x->nact++;
    }
  }
}

static int is_border(int dim, const long I[3], const long n[3]) {
  for (int d = 0; d < dim; ++d)
    if (I[d] < 1 || I[d] > n[d] - 2) return 1;
  return 0;
}

static void positions(int dim, const long I[3], const long n[3], int pos[3]) {
  pos[0] = pos[1] = pos[2] = P_INTERIOR;
  for (int d = 0; d < dim; ++d) {
    if (I[d] == 0) pos[d] = P_LEFT;
    else if (n[d] - I[d] == 1) pos[d] = P_RIGHT;
  }
}

/* Restriction, IGO.hxx:175-304 (gather by coarse index; faces on the coarse image) */
static void restrict_raw(int dim, const int cent[3], const long nf[3], const double *fine,
                         const long nc[3], double *coarse) {
  xfer_t x;
  xfer_init(&x, dim, cent, 0);
  int ipos[3] = {P_INTERIOR, P_INTERIOR, P_INTERIOR};
  double wint[125];
  for (int a = 0; a < x.nact; ++a) wint[a] = gen_weight(&x, cent, ipos, x.act[a], 0);
  long I[3];
  for (I[2] = 0; I[2] < nc[2]; ++I[2])
    for (I[1] = 0; I[1] < nc[1]; ++I[1])
      for (I[0] = 0; I[0] < nc[0]; ++I[0]) {
        long F[3] = {2 * I[0], 2 * I[1], (dim == 3) ? 2 * I[2] : 0};
        double value = 0.;
        if (!is_border(dim, I, nc)) {
          for (int a = 0; a < x.nact; ++a) {
            const int *o = x.act[a];
            long q = (F[0] + o[0]) + nf[0] * ((F[1] + o[1]) + nf[1] * (F[2] + o[2]));
            value += wint[a] * fine[q];
          }
        } else {
          int pos[3];
          positions(dim, I, nc, pos);
          for (int a = 0; a < x.nact; ++a) {
            const int *o = x.act[a];
            long g[3] = {F[0] + o[0], F[1] + o[1], F[2] + o[2]};
            int inside = 1;
            for (int d = 0; d < dim; ++d)
              if (g[d] < 0 || g[d] >= nf[d]) inside = 0;
            if (inside)
              value += gen_weight(&x, cent, pos, o, 0) * fine[g[0] + nf[0] * (g[1] + nf[1] * g[2])];
          }
        }
        coarse[I[0] + nc[0] * (I[1] + nc[1] * I[2])] = value;
      }
}

/* Interpolation, IGO.hxx:45-172 (scatter from coarse points; output zero-filled) */
static void interpolate_raw(int dim, const int cent[3], const long nc[3], const double *coarse,
                            const long nf[3], double *fine) {
  xfer_t x;
  xfer_init(&x, dim, cent, 1);
  int ipos[3] = {P_INTERIOR, P_INTERIOR, P_INTERIOR};
  double wint[125];
  for (int a = 0; a < x.nact; ++a) wint[a] = gen_weight(&x, cent, ipos, x.act[a], 1);
  long Nf = nf[0] * nf[1] * nf[2];
  for (long i = 0; i < Nf; ++i) fine[i] = 0.;
  for (int pass = 0; pass < 2; ++pass) {
    long I[3];
    for (I[2] = 0; I[2] < nc[2]; ++I[2])
      for (I[1] = 0; I[1] < nc[1]; ++I[1])
        for (I[0] = 0; I[0] < nc[0]; ++I[0]) {
          int border = is_border(dim, I, nc);
          if (border != pass) continue;
          long F[3] = {2 * I[0], 2 * I[1], (dim == 3) ? 2 * I[2] : 0};
          double v = coarse[I[0] + nc[0] * (I[1] + nc[1] * I[2])];
          int pos[3];
          positions(dim, I, nc, pos);
          for (int a = 0; a < x.nact; ++a) {
            const int *o = x.act[a];
            long g[3] = {F[0] + o[0], F[1] + o[1], F[2] + o[2]};
            if (border) {
              int inside = 1;
              for (int d = 0; d < dim; ++d)
                if (g[d] < 0 || g[d] >= nf[d]) inside = 0;
              if (!inside) continue;
              fine[g[0] + nf[0] * (g[1] + nf[1] * g[2])] += gen_weight(&x, cent, pos, o, 1) * v;
            } else {
              fine[g[0] + nf[0] * (g[1] + nf[1] * g[2])] += wint[a] * v;
            }
          }
        }
  }
}

/* ---------------------------------------------------------------- DCA */
/* GenerateDCA, GH:298-516.  tensor: SoA (ncomp arrays of N). */
static void generate_dca(int dim, const long n[3], const double h[3], const double *T,
                         double dt, double *A) {
  long N = n[0] * n[1] * n[2];
  long stride[3] = {1, n[0], n[0] * n[1]};
  long idx[3];
  for (idx[2] = 0; idx[2] < n[2]; ++idx[2])
    for (idx[1] = 0; idx[1] < n[1]; ++idx[1])
      for (idx[0] = 0; idx[0] < n[0]; ++idx[0]) {
        long p = idx[0] + n[0] * (idx[1] + n[1] * idx[2]);
        double *S = A + 27 * p;
        for (int i = 0; i < 27; ++i) S[i] = 0; /* GH:344 */
        const int c = nbidx(0, 0, 0);
        S[c] = 1; /* GH:346 */
        for (int d = 0; d < dim; ++d) {
          int offP[3] = {0, 0, 0}, offM[3] = {0, 0, 0};
          offP[d] = 1;
          offM[d] = -1;
          double weight = -dt / (h[d] * h[d]); /* GH:360 */
          if (idx[d] == 0) offM[d] = 1;          /* GH:362 */
          else if (n[d] - idx[d] == 1) offP[d] = -1; /* GH:363 */
          double value = T[tcomp(dim, d, d) * N + p] * weight;
          S[nbidx(offP[0], offP[1], offP[2])] += value;
          S[nbidx(offM[0], offM[1], offM[2])] += value;
          S[c] -= 2 * value;
          for (int d2 = 0; d2 < dim; ++d2) {
            weight = -dt / (4 * h[d] * h[d2]); /* GH:374 */
            int PP[3] = {0, 0, 0}, PM[3] = {0, 0, 0}, MP[3] = {0, 0, 0}, MM[3] = {0, 0, 0};
            PP[d] += 1; PP[d2] += 1;
            PM[d] += 1; PM[d2] -= 1;
            MP[d] -= 1; MP[d2] += 1;
            MM[d] -= 1; MM[d2] -= 1;
            if (idx[d] == 0) { /* GH:388-396 */
              MM[d] += 2; MP[d] += 2;
            } else if (n[d] - idx[d] == 1) {
              PP[d] -= 2; PM[d] -= 2;
            }
            if (idx[d2] == 0) { /* GH:407-418 */
              MM[d2] += 2; PM[d2] += 2;
            } else if (n[d2] - idx[d2] == 1) {
              PP[d2] -= 2; MP[d2] -= 2;
            }
            if (d != d2) { /* mixed derivatives, GH:434-444 */
              value = T[tcomp(dim, d, d2) * N + p] * weight;
              S[nbidx(PP[0], PP[1], PP[2])] += value;
              S[nbidx(PM[0], PM[1], PM[2])] -= value;
              S[nbidx(MP[0], MP[1], MP[2])] -= value;
              S[nbidx(MM[0], MM[1], MM[2])] += value;
            }
            /* first derivatives with one-sided tensor differences at the border, GH:447-474 */
            const double *Tc = T + tcomp(dim, d, d2) * N;
            if (idx[d2] == 0) {
              value = (-3. * Tc[p] + 4. * Tc[p + stride[d2]] - 1. * Tc[p + 2 * stride[d2]]) * weight;
            } else if (n[d2] - idx[d2] == 1) {
              value = (3. * Tc[p] - 4. * Tc[p - stride[d2]] + 1. * Tc[p - 2 * stride[d2]]) * weight;
            } else {
              value = (Tc[p + stride[d2]] - Tc[p - stride[d2]]) * weight;
            }
            S[nbidx(offP[0], offP[1], offP[2])] += value;
            S[nbidx(offM[0], offM[1], offM[2])] -= value;
          }
        }
      }
}

/* ---------------------------------------------------------------- dense LU */
static int lu_factor(long n, double *a, long *piv) {
  for (long k = 0; k < n; ++k) {
    long p = k;
    double best = fabs(a[k * n + k]);
    for (long i = k + 1; i < n; ++i)
      if (fabs(a[i * n + k]) > best) { best = fabs(a[i * n + k]); p = i; }
    piv[k] = p;
    if (best == 0.) return -1;
    if (p != k)
      for (long j = 0; j < n; ++j) { double t = a[k * n + j]; a[k * n + j] = a[p * n + j]; a[p * n + j] = t; }
    double inv = 1. / a[k * n + k];
    for (long i = k + 1; i < n; ++i) {
      double f = a[i * n + k] * inv;
      a[i * n + k] = f;
      if (f != 0.)
        for (long j = k + 1; j < n; ++j) a[i * n + j] -= f * a[k * n + j];
    }
  }
  return 0;
}

static void lu_solve(long n, const double *a, const long *piv, double *x) {
  for (long k = 0; k < n; ++k) { long p = piv[k]; if (p != k) { double t = x[k]; x[k] = x[p]; x[p] = t; } }
  for (long i = 0; i < n; ++i) { double s = x[i]; for (long j = 0; j < i; ++j) s -= a[i * n + j] * x[j]; x[i] = s; }
  for (long i = n - 1; i >= 0; --i) { double s = x[i]; for (long j = i + 1; j < n; ++j) s -= a[i * n + j] * x[j]; x[i] = s / a[i * n + i]; }
}

/* ---------------------------------------------------------------- banded LU */
/* LAPACK dgbtf2 / dgbtrs restated (unblocked, partial pivoting) on column-major band
 * storage: A(i, j) at ab[(kv + i - j) + j * ldab], kv = kl + ku, ldab = 2 kl + ku + 1 (the
 * kl extra super-diagonals hold U's fill from row interchanges). */
static int band_factor(long n, long kl, long ku, double *ab, long *piv) {
  const long kv = kl + ku, ldab = 2 * kl + ku + 1;
  long ju = 0;
  for (long j = 0; j < n; ++j) {
    double *cj = ab + j * ldab;
    long km = kl < n - 1 - j ? kl : n - 1 - j;
    long p = 0;
    double best = fabs(cj[kv]);
    for (long i = 1; i <= km; ++i)
      if (fabs(cj[kv + i]) > best) { best = fabs(cj[kv + i]); p = i; }
    piv[j] = j + p;
    if (best == 0.) return -1;
    long jn = j + ku + p < n - 1 ? j + ku + p : n - 1;
    if (jn > ju) ju = jn;
    if (p != 0)
      for (long c = j; c <= ju; ++c) {
        double *cc = ab + c * ldab + kv - c;
        double t = cc[j]; cc[j] = cc[j + p]; cc[j + p] = t;
      }
    const double inv = 1. / cj[kv];
    for (long i = 1; i <= km; ++i) cj[kv + i] *= inv;
#pragma omp parallel for schedule(static) if ((ju - j) * km > 200000)
    for (long c = j + 1; c <= ju; ++c) {
      double *cc = ab + c * ldab + kv - c;  /* cc[r] = A(r, c) */
      const double f = cc[j];
      if (f != 0.)
        for (long i = 1; i <= km; ++i) cc[j + i] -= cj[kv + i] * f;
    }
  }
  return 0;
}

static void band_solve(long n, long kl, long ku, const double *ab, const long *piv, double *x) {
  const long kv = kl + ku, ldab = 2 * kl + ku + 1;
  for (long j = 0; j < n; ++j) { /* L y = P b */
    long p = piv[j];
    if (p != j) { double t = x[j]; x[j] = x[p]; x[p] = t; }
    long lm = kl < n - 1 - j ? kl : n - 1 - j;
    const double *cj = ab + j * ldab + kv;
    for (long i = 1; i <= lm; ++i) x[j + i] -= cj[i] * x[j];
  }
  for (long j = n - 1; j >= 0; --j) { /* U x = y, U with kl + ku super-diagonals */
    const double *cj = ab + j * ldab + kv - j;  /* cj[r] = U(r, j) */
    x[j] /= cj[j];
    long i0 = j - kv > 0 ? j - kv : 0;
    for (long i = i0; i < j; ++i) x[i] -= cj[i] * x[j];
  }
}

/* band numbering of the coarsest grid: axes ordered by length (shortest innermost, the
 * longest outermost), so the bandwidth is about the product of the two shorter axes */
static void band_order(int dim, const long n[3], long *perm, long *kl_out, long *ku_out,
                       const double *A) {
  int ax[3] = {0, 1, 2};
  for (int a = 0; a < dim; ++a)
    for (int b = a + 1; b < dim; ++b)
      if (n[ax[b]] < n[ax[a]] || (n[ax[b]] == n[ax[a]] && ax[b] < ax[a])) {
        int t = ax[a]; ax[a] = ax[b]; ax[b] = t;
      }
  long st[3] = {0, 0, 0}, s = 1;
  for (int a = 0; a < dim; ++a) { st[ax[a]] = s; s *= n[ax[a]]; }
  long idx[3], kl = 0, ku = 0;
  for (idx[2] = 0; idx[2] < n[2]; ++idx[2])
    for (idx[1] = 0; idx[1] < n[1]; ++idx[1])
      for (idx[0] = 0; idx[0] < n[0]; ++idx[0]) {
        long p = idx[0] + n[0] * (idx[1] + n[1] * idx[2]);
        perm[p] = idx[0] * st[0] + idx[1] * st[1] + idx[2] * st[2];
      }
  for (idx[2] = 0; idx[2] < n[2]; ++idx[2])
    for (idx[1] = 0; idx[1] < n[1]; ++idx[1])
      for (idx[0] = 0; idx[0] < n[0]; ++idx[0]) {
        long p = idx[0] + n[0] * (idx[1] + n[1] * idx[2]);
        for (int i = 0; i < 27; ++i) {
          if (A[27 * p + i] == 0.) continue;
          int o[3] = {i % 3 - 1, (i / 3) % 3 - 1, i / 9 - 1};
          long q[3] = {idx[0] + o[0], idx[1] + o[1], idx[2] + o[2]};
          int inside = 1;
          for (int d = 0; d < 3; ++d)
            if (q[d] < 0 || q[d] >= n[d]) inside = 0;
          if (!inside) continue;
          long d = perm[q[0] + n[0] * (q[1] + n[1] * q[2])] - perm[p];
          if (d > ku) ku = d;
          if (-d > kl) kl = -d;
        }
      }
  *kl_out = kl;
  *ku_out = ku;
}

/* ---------------------------------------------------------------- hierarchy */
ora_ctx *ora_create(int dim, const long n0[3], const double h0[3], const double *tensor,
                    double dt) {
  if (dim != 2 && dim != 3) return NULL;
  ora_ctx *c = (ora_ctx *)calloc(1, sizeof(ora_ctx));
  c->dim = dim;
  int maxDepth = ora_max_depth(dim, n0);
  if (maxDepth + 1 > MAXLEV) { free(c); return NULL; }
  c->nlev = maxDepth + 1;
  /* active offsets: all 27/9 in index order, minus 3D corners (GH:489-513) */
  c->noff = 0;
  for (int i = 0; i < 27; ++i) {
    int o[3] = {i % 3 - 1, (i / 3) % 3 - 1, i / 9 - 1};
    if (dim == 2 && o[2] != 0) continue;
    if (dim == 3 && o[0] != 0 && o[1] != 0 && o[2] != 0) continue;
    memcpy(c->off[c->noff++], o, sizeof(o));
  }
  /* level geometry, GH:61-106 */
  ora_level *L = c->lev;
  for (int d = 0; d < 3; ++d) {
    L[0].n[d] = (d < dim) ? n0[d] : 1;
    L[0].h[d] = (d < dim) ? h0[d] : 1.;
    L[0].cent[d] = ORA_VERTEX;
  }
  for (int l = 1; l < c->nlev; ++l)
    for (int d = 0; d < 3; ++d) {
      L[l].h[d] = L[l - 1].h[d] * 2;
      if (d >= dim) { L[l].n[d] = 1; L[l].cent[d] = ORA_VERTEX; continue; }
      if (L[l - 1].n[d] % 2 == 0) { L[l].n[d] = L[l - 1].n[d] / 2; L[l].cent[d] = ORA_CELL; }
      else { L[l].n[d] = (L[l - 1].n[d] - 1) / 2 + 1; L[l].cent[d] = ORA_VERTEX; }
    }
  for (int l = 0; l < c->nlev; ++l) {
    L[l].N = L[l].n[0] * L[l].n[1] * L[l].n[2];
    L[l].A = (double *)malloc(sizeof(double) * 27 * L[l].N);
  }
  int ncomp = dim * (dim + 1) / 2;
  /* operator on the finest grid (GH:110), then restricted tensors + DCA per level (GH:149-201) */
  generate_dca(dim, L[0].n, L[0].h, tensor, dt, L[0].A);
  double *fine = (double *)malloc(sizeof(double) * ncomp * L[0].N);
  memcpy(fine, tensor, sizeof(double) * ncomp * L[0].N);
  for (int l = 1; l < c->nlev; ++l) {
    double *coarse = (double *)malloc(sizeof(double) * ncomp * L[l].N);
    for (int k = 0; k < ncomp; ++k)
      restrict_raw(dim, L[l].cent, L[l - 1].n, fine + k * L[l - 1].N, L[l].n, coarse + k * L[l].N);
    generate_dca(dim, L[l].n, L[l].h, coarse, dt, L[l].A);
    free(fine);
    fine = coarse;
  }
  free(fine);
  /* DirectSolver on the coarsest operator (DS:32-88): matrix(row, col) from all 27/9 entries */
  ora_level *C = &L[c->nlev - 1];
  long n = C->N;
  c->nlu = n;
  c->kl = -1;
  c->piv = (long *)malloc(sizeof(long) * n);
  long ldab = 0;
  if (n > ORA_DENSE_MAX) {
    c->perm = (long *)malloc(sizeof(long) * n);
    band_order(dim, C->n, c->perm, &c->kl, &c->ku, C->A);
    ldab = 2 * c->kl + c->ku + 1;
    c->lu = (double *)calloc((size_t)n * ldab, sizeof(double));
  } else {
    c->lu = (double *)calloc((size_t)n * n, sizeof(double));
  }
  if (!c->lu) { ora_destroy(c); return NULL; }
  long idx[3];
  for (idx[2] = 0; idx[2] < C->n[2]; ++idx[2])
    for (idx[1] = 0; idx[1] < C->n[1]; ++idx[1])
      for (idx[0] = 0; idx[0] < C->n[0]; ++idx[0]) {
        long row = idx[0] + C->n[0] * (idx[1] + C->n[1] * idx[2]);
        for (int i = 0; i < 27; ++i) {
          int o[3] = {i % 3 - 1, (i / 3) % 3 - 1, i / 9 - 1};
          if (dim == 2 && o[2] != 0) continue;
          long q[3] = {idx[0] + o[0], idx[1] + o[1], idx[2] + o[2]};
          int inside = 1;
          for (int d = 0; d < dim; ++d)
            if (q[d] < 0 || q[d] >= C->n[d]) inside = 0;
          if (!inside) continue;
          long col = q[0] + C->n[0] * (q[1] + C->n[1] * q[2]);
          if (c->kl < 0) {
            c->lu[row * n + col] = C->A[27 * row + i];
          } else if (C->A[27 * row + i] != 0.) {
            long r = c->perm[row], k = c->perm[col];
            c->lu[(c->kl + c->ku + r - k) + k * ldab] = C->A[27 * row + i];
          }
        }
      }
  int fail = (c->kl < 0) ? lu_factor(n, c->lu, c->piv) : band_factor(n, c->kl, c->ku, c->lu, c->piv);
  if (fail != 0) { ora_destroy(c); return NULL; }
  return c;
}

void ora_destroy(ora_ctx *c) {
  if (!c) return;
  for (int l = 0; l < c->nlev; ++l) free(c->lev[l].A);
  free(c->lu);
  free(c->piv);
  free(c->perm);
  free(c->tr_level);
  free(c->tr_it);
  free(c->tr_rel);
  free(c);
}

int ora_num_levels(const ora_ctx *c) { return c->nlev; }

void ora_level_info(const ora_ctx *c, int level, long n[3], double h[3], int cent[3]) {
  for (int d = 0; d < 3; ++d) {
    n[d] = c->lev[level].n[d];
    h[d] = c->lev[level].h[d];
    cent[d] = c->lev[level].cent[d];
  }
}

const double *ora_stencil(const ora_ctx *c, int level) { return c->lev[level].A; }

/* ---------------------------------------------------------------- smoothers */
/* LexOrder, itkMultigridGaussSeidelSmoother.h:87-100 */
static int lex_order(const int *l, const int *r) {
  for (int i = 2; i >= 0; --i) {
    if (l[i] < r[i]) return 1;
    if (l[i] > r[i]) return 0;
  }
  return 0;
}

#define FOR_VOXELS(L)                                      \
  for (long z = 0; z < (L)->n[2]; ++z)                     \
    for (long y = 0; y < (L)->n[1]; ++y)                   \
      for (long x = 0; x < (L)->n[0]; ++x)

static inline int inside3(const ora_level *L, long x, long y, long z) {
  return x >= 0 && x < L->n[0] && y >= 0 && y < L->n[1] && z >= 0 && z < L->n[2];
}

/* GS SingleIteration, GS:33-111: lexicographic, new values for lex-earlier neighbours */
void ora_gs_lex(const ora_ctx *c, int level, const double *in, const double *b, double *out) {
  const ora_level *L = &c->lev[level];
  const int zero[3] = {0, 0, 0};
  const int ic = nbidx(0, 0, 0);
  FOR_VOXELS(L) {
    long p = x + L->n[0] * (y + L->n[1] * z);
    const double *S = L->A + 27 * p;
    double value = b[p];
    for (int k = 0; k < c->noff; ++k) {
      const int *o = c->off[k];
      if (!inside3(L, x + o[0], y + o[1], z + o[2])) continue;
      long q = (x + o[0]) + L->n[0] * ((y + o[1]) + L->n[1] * (z + o[2]));
      if (lex_order(o, zero)) value -= S[nbidx(o[0], o[1], o[2])] * out[q];
      else if (lex_order(zero, o)) value -= S[nbidx(o[0], o[1], o[2])] * in[q];
    }
    out[p] = value / S[ic];
  }
}

static int color_of(int dim, int ncolors, long x, long y, long z) {
  if (ncolors == 2) return (int)((x + y + z) & 1);
  if (dim == 2) return (int)((x & 1) | ((y & 1) << 1));
  return (int)(((x + z) & 1) | (((y + z) & 1) << 1));
}

/* Extension: multicolour GS (2 colours for 5/7-point operators, 4 for 9/19-point).
 * Same per-point update as GS:74-99 with all neighbours taken from the current iterate. */
void ora_gs_color(const ora_ctx *c, int level, int ncolors, const double *in, const double *b,
                  double *out) {
  const ora_level *L = &c->lev[level];
  const int ic = nbidx(0, 0, 0);
  if (out != in) memcpy(out, in, sizeof(double) * L->N);
  for (int col = 0; col < ncolors; ++col) {
    FOR_VOXELS(L) {
      if (color_of(c->dim, ncolors, x, y, z) != col) continue;
      long p = x + L->n[0] * (y + L->n[1] * z);
      const double *S = L->A + 27 * p;
      double value = b[p];
      for (int k = 0; k < c->noff; ++k) {
        const int *o = c->off[k];
        if (o[0] == 0 && o[1] == 0 && o[2] == 0) continue;
        if (!inside3(L, x + o[0], y + o[1], z + o[2])) continue;
        long q = (x + o[0]) + L->n[0] * ((y + o[1]) + L->n[1] * (z + o[2]));
        value -= S[nbidx(o[0], o[1], o[2])] * out[q];
      }
      out[p] = value / S[ic];
    }
  }
}

/* The same multicolour sweep on all host cores (OpenMP over the planes of one colour;
 * the colouring makes the updates of one colour independent, so the result does not
 * depend on the thread count).  CPU baseline only (bench.py cpu_baseline.parallel). */
void ora_gs_color_omp(const ora_ctx *c, int level, int ncolors, const double *in,
                      const double *b, double *out, int nthreads) {
  const ora_level *L = &c->lev[level];
  const int ic = nbidx(0, 0, 0);
  if (out != in) memcpy(out, in, sizeof(double) * L->N);
  for (int col = 0; col < ncolors; ++col) {
#pragma omp parallel for num_threads(nthreads) schedule(static) collapse(2)
    for (long z = 0; z < L->n[2]; ++z)
      for (long y = 0; y < L->n[1]; ++y)
        for (long x = (color_of(c->dim, ncolors, 0, y, z) == col) ? 0 : 1; x < L->n[0]; x += 2) {
          if (color_of(c->dim, ncolors, x, y, z) != col) break;  /* row holds no point of col */
          long p = x + L->n[0] * (y + L->n[1] * z);
          const double *S = L->A + 27 * p;
          double value = b[p];
          for (int k = 0; k < c->noff; ++k) {
            const int *o = c->off[k];
            if (o[0] == 0 && o[1] == 0 && o[2] == 0) continue;
            if (!inside3(L, x + o[0], y + o[1], z + o[2])) continue;
            long q = (x + o[0]) + L->n[0] * ((y + o[1]) + L->n[1] * (z + o[2]));
            value -= S[nbidx(o[0], o[1], o[2])] * out[q];
          }
          out[p] = value / S[ic];
        }
  }
}

/* WJ SingleIteration, WJ:33-102 */
void ora_wj(const ora_ctx *c, int level, double omega, const double *in, const double *b,
            double *out) {
  const ora_level *L = &c->lev[level];
  const int ic = nbidx(0, 0, 0);
  FOR_VOXELS(L) {
    long p = x + L->n[0] * (y + L->n[1] * z);
    const double *S = L->A + 27 * p;
    double value = b[p];
    for (int k = 0; k < c->noff; ++k) {
      const int *o = c->off[k];
      if (o[0] == 0 && o[1] == 0 && o[2] == 0) continue;
      if (!inside3(L, x + o[0], y + o[1], z + o[2])) continue;
      long q = (x + o[0]) + L->n[0] * ((y + o[1]) + L->n[1] * (z + o[2]));
      value -= S[nbidx(o[0], o[1], o[2])] * in[q];
    }
    value *= omega / S[ic];
    value += (1 - omega) * in[p];
    out[p] = value;
  }
}

/* ComputeResidual, GS:114-180 (identical in WJ:105-171): r = b - A x */
void ora_residual(const ora_ctx *c, int level, const double *in, const double *b, double *r) {
  const ora_level *L = &c->lev[level];
  FOR_VOXELS(L) {
    long p = x + L->n[0] * (y + L->n[1] * z);
    const double *S = L->A + 27 * p;
    double value = b[p];
    for (int k = 0; k < c->noff; ++k) {
      const int *o = c->off[k];
      if (!inside3(L, x + o[0], y + o[1], z + o[2])) continue;
      long q = (x + o[0]) + L->n[0] * ((y + o[1]) + L->n[1] * (z + o[2]));
      value -= S[nbidx(o[0], o[1], o[2])] * in[q];
    }
    r[p] = value;
  }
}

void ora_restrict(const ora_ctx *c, int level, const double *fine, double *coarse) {
  restrict_raw(c->dim, c->lev[level + 1].cent, c->lev[level].n, fine, c->lev[level + 1].n, coarse);
}

void ora_interpolate(const ora_ctx *c, int level, const double *coarse, double *fine) {
  interpolate_raw(c->dim, c->lev[level + 1].cent, c->lev[level + 1].n, coarse, c->lev[level].n, fine);
}

/* DirectSolver::Solve, DS:91-147 */
void ora_direct_solve(const ora_ctx *c, const double *b, double *x) {
  if (c->kl < 0) {
    memcpy(x, b, sizeof(double) * c->nlu);
    lu_solve(c->nlu, c->lu, c->piv, x);
    return;
  }
  double *t = (double *)malloc(sizeof(double) * c->nlu);
  for (long p = 0; p < c->nlu; ++p) t[c->perm[p]] = b[p];
  band_solve(c->nlu, c->kl, c->ku, c->lu, c->piv, t);
  for (long p = 0; p < c->nlu; ++p) x[p] = t[c->perm[p]];
  free(t);
}

/* L2Norm, MAD:496-515 */
double ora_l2norm(long n, const double *x) {
  double norm = 0;
  for (long i = 0; i < n; ++i) norm += x[i] * x[i];
  return sqrt(norm);
}

/* ---------------------------------------------------------------- driver */
static void smooth(const ora_ctx *c, const ora_params *p, int level, const double *x,
                   const double *b, double *out) {
  if (p->smoother == ORA_WJ) ora_wj(c, level, p->omega, x, b, out);
  else if (p->smoother == ORA_GS_COLOR) {
    int ncol = p->ncolors ? p->ncolors : 4;
    ora_gs_color(c, level, ncol, x, b, out);
  } else ora_gs_lex(c, level, x, b, out);
}

/* VCycle, MAD:341-493 (the residuals/norms computed there only for verbose
 * output are skipped; the residual after the last pre-smoothing sweep feeds the
 * restriction, MAD:389,413). */
static void vcycle_rec(ora_ctx *c, const ora_params *p, int level, const double *x,
                       const double *b, double *out) {
  ora_level *L = &c->lev[level];
  long N = L->N;
  /* verbose only: rhsNorm (MAD:352) and the relative residual of the current iterate */
  double *vr = p->verbose ? (double *)malloc(sizeof(double) * N) : NULL;
  double rhsNorm = p->verbose ? ora_l2norm(N, b) : 0.;
#define VERBOSE_LINE(it_, sol_)                                   \
  if (p->verbose) {                                               \
    ora_residual(c, level, (sol_), b, vr);                        \
    trace_push(c, level, (it_), ora_l2norm(N, vr) / rhsNorm);     \
  }
  if (level == c->nlev - 1) { /* MAD:356-371 */
    ora_direct_solve(c, b, out);
    VERBOSE_LINE(-1, out);
    free(vr);
    return;
  }
  double *cur = (double *)malloc(sizeof(double) * N);
  double *tmp = (double *)malloc(sizeof(double) * N);
  memcpy(cur, x, sizeof(double) * N); /* ImageDuplicator, MAD:375-379 */
  for (unsigned n = 0; n < p->iterations_per_grid; ++n) { /* MAD:384-411 */
    smooth(c, p, level, cur, b, tmp);
    double *t = cur; cur = tmp; tmp = t;
    VERBOSE_LINE((int)n + 1, cur);
  }
  ora_residual(c, level, cur, b, tmp); /* MAD:389 */
  ora_level *Cl = &c->lev[level + 1];
  double *bc = (double *)malloc(sizeof(double) * Cl->N);
  double *xc = (double *)calloc(Cl->N, sizeof(double)); /* MAD:415-416 */
  double *oc = (double *)malloc(sizeof(double) * Cl->N);
  ora_restrict(c, level, tmp, bc); /* MAD:413 */
  vcycle_rec(c, p, level + 1, xc, bc, oc); /* MAD:418-420 */
  ora_interpolate(c, level, oc, tmp);      /* MAD:422 */
  for (long i = 0; i < N; ++i) cur[i] += tmp[i]; /* MAD:424-435 */
  VERBOSE_LINE(0, cur); /* MAD:437-448 */
  for (unsigned n = 0; n < p->iterations_per_grid; ++n) { /* MAD:460-487 */
    smooth(c, p, level, cur, b, tmp);
    double *t = cur; cur = tmp; tmp = t;
    VERBOSE_LINE((int)n + 1, cur);
  }
#undef VERBOSE_LINE
  memcpy(out, cur, sizeof(double) * N);
  free(cur); free(tmp); free(bc); free(xc); free(oc); free(vr);
}

long ora_take_trace(ora_ctx *c, long cap, int *level, int *it, double *relres) {
  long n = c->ntr;
  for (long i = 0; i < n && i < cap; ++i) {
    if (level) level[i] = c->tr_level[i];
    if (it) it[i] = c->tr_it[i];
    if (relres) relres[i] = c->tr_rel[i];
  }
  c->ntr = 0;
  return n;
}

/* FullMultiGrid, MAD:300-338 */
static void fmg_rec(ora_ctx *c, const ora_params *p, int level, const double *b, double *out) {
  ora_level *L = &c->lev[level];
  long N = L->N;
  double *cur = (double *)malloc(sizeof(double) * N);
  double *tmp = (double *)malloc(sizeof(double) * N);
  if (level == c->nlev - 1) { /* MAD:308-316 */
    memset(cur, 0, sizeof(double) * N);
  } else { /* MAD:317-334 */
    ora_level *Cl = &c->lev[level + 1];
    double *bc = (double *)malloc(sizeof(double) * Cl->N);
    double *xc = (double *)malloc(sizeof(double) * Cl->N);
    ora_restrict(c, level, b, bc);
    fmg_rec(c, p, level + 1, bc, xc);
    ora_interpolate(c, level, xc, cur);
    free(bc); free(xc);
  }
  for (unsigned n = 0; n < p->iterations_per_grid; ++n) {
    vcycle_rec(c, p, level, cur, b, tmp);
    double *t = cur; cur = tmp; tmp = t;
  }
  memcpy(out, cur, sizeof(double) * N);
  free(cur); free(tmp);
}

void ora_vcycle(ora_ctx *c, const ora_params *p, const double *x, const double *b, double *out) {
  vcycle_rec(c, p, 0, x, b, out);
}

void ora_fmg(ora_ctx *c, const ora_params *p, const double *b, double *out) {
  fmg_rec(c, p, 0, b, out);
}

/* GenerateData, MAD:104-297 (casts are the caller's job; input/output are fp64) */
int ora_run(ora_ctx *c, const ora_params *p, const double *input, double *output,
            int *cycles_out, double *relres_out) {
  long N = c->lev[0].N;
  double *rhs = (double *)malloc(sizeof(double) * N);
  double *sol = (double *)malloc(sizeof(double) * N);
  double *tmp = (double *)malloc(sizeof(double) * N);
  memcpy(rhs, input, sizeof(double) * N); /* MAD:110-127 */
  for (unsigned step = 0; step < p->number_of_steps; ++step) { /* MAD:158 */
    if (p->cycle == ORA_FMG) fmg_rec(c, p, 0, rhs, sol); /* MAD:170-176 */
    else memcpy(sol, rhs, sizeof(double) * N);          /* MAD:177-201 */
    double relativeResidual;
    double rhsNorm = ora_l2norm(N, rhs); /* MAD:204 */
    unsigned numberOfIterations = 0;
    do { /* MAD:207-246 */
      if (p->cycle == ORA_SMOOTHER) smooth(c, p, 0, sol, rhs, tmp);
      else vcycle_rec(c, p, 0, sol, rhs, tmp);
      double *t = sol; sol = tmp; tmp = t;
      ora_residual(c, 0, sol, rhs, tmp);
      relativeResidual = ora_l2norm(N, tmp) / rhsNorm;
      ++numberOfIterations;
    } while (relativeResidual > p->tolerance && numberOfIterations < p->max_cycles);
    if (cycles_out) cycles_out[step] = (int)numberOfIterations;
    if (relres_out) relres_out[step] = relativeResidual;
    memcpy(rhs, sol, sizeof(double) * N); /* MAD:248-261 */
  }
  memcpy(output, sol, sizeof(double) * N);
  free(rhs); free(sol); free(tmp);
  return 0;
}
