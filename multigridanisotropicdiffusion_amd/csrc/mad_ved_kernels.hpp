// mad_ved_kernels.hpp -- device kernels of the VED tensor generation (include/mad_ved.h).
//
// Reference: include/itkVEDMultigridImageFilter.hxx (VED.hxx below).
//   ComputeHessian          VED.hxx:158-173  -> ved_iir_k (x3 axes; ITK's recursive operator,
//                                              default) or ved_fir_{z,y}_k + ved_fir_x_k
//   VesselnessFunction      VED.hxx:176-212  -> ved_vesselness
//   UpdateVesselness        VED.hxx:215-299  -> ved_fir_x_k<.., VED_UPDATE> (fused)
//   GenerateDiffusionTensor VED.hxx:302-378  -> ved_tensor_k
//
// The scale-normalised Hessian is three separable correlation passes with sampled,
// moment-normalised Gaussian derivative taps (computed on the host, ved_taps in
// mad_ved.hpp): z (image -> 3 derivative orders), y (-> the 6 (y, z) order pairs the
// Hessian needs), then x, fused with the per-voxel eigen-analysis, vesselness and the
// running maximum over scales, so the 6 Hessian components never reach HBM.
// Storage, FIR and eigen arithmetic in T (fp32 or fp64, explicit fma); response and
// vessel direction are stored in fp64 (the reference's Precision).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mad {

// Hessian scale factors sigma^2 / (h_d h_d2), component order [xx,xy,xz,yy,yz,zz]
struct HessScale {
  double f[6];
};

struct VesselParams {
  double alpha, beta, gamma;
};

// The three passes stage their input lines through LDS once (each input value is read
// from HBM once per pass plus the tile halo) and run the taps out of LDS.  Taps live in
// a small device array read with uniform (scalar) loads: [K0 | K1 | K2], each 2R+1.

// z pass: o_q(i,j,k) = sum_t K_q(t) in(i, j, clamp(k + t)), q = 0, 1, 2 (orders).
// Block = 64 x 4 columns, ZT output planes; LDS holds the ZT + 2R input planes of the
// block's columns (converted from the fp64 image to T on the way in).
template <typename T>
__global__ void __launch_bounds__(256) ved_fir_z_k(const double* __restrict__ in, T* __restrict__ o0,
                                                   T* __restrict__ o1, T* __restrict__ o2,
                                                   const T* __restrict__ taps, int R, int nx, int ny,
                                                   int nz, int ZT) {
#pragma clang fp contract(off)
  extern __shared__ __align__(16) unsigned char ved_smem[];
  T* L = reinterpret_cast<T*>(ved_smem);
  const int tid = threadIdx.x;
  const int i = blockIdx.x * 64 + (tid & 63);
  const int j = blockIdx.y * 4 + (tid >> 6);
  const int z0 = blockIdx.z * ZT;
  const bool ok = i < nx && j < ny;
  const int64_t sz = (int64_t)nx * ny;
  const int64_t col = (int64_t)min(j, ny - 1) * nx + min(i, nx - 1);
  const int np = ZT + 2 * R;
  for (int m = 0; m < np; ++m) {
    const int kk = min(max(z0 - R + m, 0), nz - 1);
    L[m * 256 + tid] = (T)in[kk * sz + col];
  }
  // each thread reads only its own column: no barrier needed
  const int W = 2 * R + 1;
  const int zend = min(ZT, nz - z0);
  for (int o = 0; o < zend; ++o) {
    T a0 = T(0), a1 = T(0), a2 = T(0);
    const T* c = L + o * 256 + tid;
#pragma unroll 4
    for (int q = 0; q < W; ++q) {
      const T v = c[q * 256];
      a0 = fma(taps[q], v, a0);
      a1 = fma(taps[W + q], v, a1);
      a2 = fma(taps[2 * W + q], v, a2);
    }
    if (ok) {
      const int64_t p = (int64_t)(z0 + o) * sz + col;
      o0[p] = a0;
      o1[p] = a1;
      o2[p] = a2;
    }
  }
}

// y pass: the six (y order, z order) pairs of the Hessian:
//   a00 = K0y z0, a10 = K1y z0, a20 = K2y z0, a01 = K0y z1, a11 = K1y z1, a02 = K0y z2
// Block = 64 x-columns of one plane, YT output rows; LDS holds the YT + 2R input rows
// of the three inputs; each thread produces YT / 4 outputs of its column.
template <typename T>
__global__ void __launch_bounds__(256) ved_fir_y_k(const T* __restrict__ z0, const T* __restrict__ z1,
                                                   const T* __restrict__ z2, T* __restrict__ a00,
                                                   T* __restrict__ a10, T* __restrict__ a20,
                                                   T* __restrict__ a01, T* __restrict__ a11,
                                                   T* __restrict__ a02, const T* __restrict__ taps,
                                                   int R, int nx, int ny, int nz, int YT) {
#pragma clang fp contract(off)
  extern __shared__ __align__(16) unsigned char ved_smem[];
  T* L = reinterpret_cast<T*>(ved_smem);
  const int tid = threadIdx.x;
  const int xi = tid & 63;
  const int i = blockIdx.x * 64 + xi;
  const int y0 = blockIdx.y * YT;
  const int k = blockIdx.z;
  const int64_t sz = (int64_t)nx * ny;
  const int64_t pl = (int64_t)k * sz + min(i, nx - 1);
  const int nr = YT + 2 * R;
  const int64_t S3 = (int64_t)nr * 64;  // one input's slab in LDS
  for (int r = tid >> 6; r < nr; r += 4) {
    const int jj = min(max(y0 - R + r, 0), ny - 1);
    const int64_t q = pl + (int64_t)jj * nx;
    L[r * 64 + xi] = z0[q];
    L[S3 + r * 64 + xi] = z1[q];
    L[2 * S3 + r * 64 + xi] = z2[q];
  }
  __syncthreads();
  if (i >= nx) return;
  const int W = 2 * R + 1;
  const int yend = min(YT, ny - y0);
  for (int o = tid >> 6; o < yend; o += 4) {
    T s00 = T(0), s10 = T(0), s20 = T(0), s01 = T(0), s11 = T(0), s02 = T(0);
    const T* c = L + o * 64 + xi;
#pragma unroll 4
    for (int q = 0; q < W; ++q) {
      const T v0 = c[q * 64], v1 = c[S3 + q * 64], v2 = c[2 * S3 + q * 64];
      const T k0 = taps[q], k1 = taps[W + q], k2 = taps[2 * W + q];
      s00 = fma(k0, v0, s00);
      s10 = fma(k1, v0, s10);
      s20 = fma(k2, v0, s20);
      s01 = fma(k0, v1, s01);
      s11 = fma(k1, v1, s11);
      s02 = fma(k0, v2, s02);
    }
    const int64_t p = pl + (int64_t)(y0 + o) * nx;
    a00[p] = s00;
    a10[p] = s10;
    a20[p] = s20;
    a01[p] = s01;
    a11[p] = s11;
    a02[p] = s02;
  }
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi rotations in E (fp64, or fp32
// in the fp32 storage mode): w ascending, V columns the matching unit eigenvectors --
// the order vnl_symmetric_eigensystem returns (VED.hxx:259-264).  Converges
// quadratically; stops when the off-diagonal mass is below ~eps/16 of the diagonal's.
template <typename E>
struct EigLimits;
template <>
struct EigLimits<double> {
  static constexpr double conv = 1e-17, tiny = 1e-300, huge = 1e150;
};
template <>
struct EigLimits<float> {
  static constexpr float conv = 1e-8f, tiny = 1e-30f, huge = 1e18f;
};

// rotation arithmetic: IEEE in fp64; the hardware reciprocal / square-root / reciprocal
// square-root approximations (~1 ulp) in fp32, where the rotation only needs c^2 + s^2 = 1
// to fp32 accuracy
__device__ inline double ei_rcp(double x) { return 1.0 / x; }
__device__ inline double ei_sqrt(double x) { return sqrt(x); }
__device__ inline double ei_rsqrt(double x) { return 1.0 / sqrt(x); }
__device__ inline float ei_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ inline float ei_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ inline float ei_rsqrt(float x) { return __builtin_amdgcn_rsqf(x); }

template <typename E>
__device__ inline void sym3_eigen(E a00, E a01, E a02, E a11, E a12, E a22, E w[3], E V[3][3]) {
#pragma clang fp contract(off)
  using Lim = EigLimits<E>;
  E A[3][3] = {{a00, a01, a02}, {a01, a11, a12}, {a02, a12, a22}};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) V[r][c] = (r == c) ? E(1) : E(0);
  for (int sweep = 0; sweep < 24; ++sweep) {
    const E off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
    const E dia = fabs(A[0][0]) + fabs(A[1][1]) + fabs(A[2][2]);
    if (!(off > Lim::conv * dia) || off < Lim::tiny) break;
#pragma unroll
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0;
      const int q = pq == 0 ? 1 : 2;
      const int r = 3 - p - q;
      const E apq = A[p][q];
      if (fabs(apq) < Lim::tiny) continue;
      const E theta = (A[q][q] - A[p][p]) * ei_rcp(E(2) * apq);
      E t;
      if (fabs(theta) > Lim::huge) {
        t = E(0.5) * ei_rcp(theta);
      } else {
        t = ei_rcp(fabs(theta) + ei_sqrt(theta * theta + E(1)));
        if (theta < E(0)) t = -t;
      }
      const E c = ei_rsqrt(t * t + E(1));
      const E s = t * c;
      A[p][p] -= t * apq;
      A[q][q] += t * apq;
      A[p][q] = A[q][p] = E(0);
      const E arp = A[r][p], arq = A[r][q];
      A[r][p] = A[p][r] = c * arp - s * arq;
      A[r][q] = A[q][r] = s * arp + c * arq;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const E vkp = V[k][p], vkq = V[k][q];
        V[k][p] = c * vkp - s * vkq;
        V[k][q] = s * vkp + c * vkq;
      }
    }
  }
  w[0] = A[0][0];
  w[1] = A[1][1];
  w[2] = A[2][2];
  // ascending, columns with them
  auto sw = [&](int a, int b) {
    if (w[a] > w[b]) {
      const E tw = w[a];
      w[a] = w[b];
      w[b] = tw;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const E tv = V[k][a];
        V[k][a] = V[k][b];
        V[k][b] = tv;
      }
    }
  };
  sw(0, 1);
  sw(1, 2);
  sw(0, 1);
}

// fp32 mode's eigen-analysis: closed-form (trigonometric) eigenvalues of the symmetric 3x3
// matrix, evaluated in fp64 -- the acos of the normalised determinant loses half the digits
// when two eigenvalues cluster (error ~ sqrt(eps) of the spread), which fp32 cannot afford
// (measured: tensor errors 3e-3 against the oracle) and fp64 can (~1e-8).  Ascending in w;
// diagonal input returns the diagonal in the order sym3_eigen's ascending sort produces.
__device__ inline void sym3_eigvals_closed(double a00, double a01, double a02, double a11,
                                           double a12, double a22, double w[3], double& spread) {
#pragma clang fp contract(off)
  const double p1 = a01 * a01 + a02 * a02 + a12 * a12;
  const double q = (a00 + a11 + a22) * (1.0 / 3.0);
  const double b00 = a00 - q, b11 = a11 - q, b22 = a22 - q;
  const double p2 = b00 * b00 + b11 * b11 + b22 * b22 + 2.0 * p1;
  const double p = sqrt(p2 * (1.0 / 6.0));
  spread = p;
  if (!(p > 0.0) || p1 == 0.0) {  // diagonal (or a multiple of I): sort the diagonal
    double d0 = a00, d1 = a11, d2 = a22, t;
    if (d0 > d1) { t = d0; d0 = d1; d1 = t; }
    if (d1 > d2) { t = d1; d1 = d2; d2 = t; }
    if (d0 > d1) { t = d0; d0 = d1; d1 = t; }
    w[0] = d0; w[1] = d1; w[2] = d2;
    return;
  }
  const double ip = 1.0 / p;
  const double c00 = b00 * ip, c11 = b11 * ip, c22 = b22 * ip;
  const double c01 = a01 * ip, c02 = a02 * ip, c12 = a12 * ip;
  const double det = c00 * (c11 * c22 - c12 * c12) - c01 * (c01 * c22 - c12 * c02) +
                     c02 * (c01 * c12 - c11 * c02);
  const double r = fmin(fmax(0.5 * det, -1.0), 1.0);
  const double phi = acos(r) * (1.0 / 3.0);
  const double hi = q + 2.0 * p * cos(phi);
  const double lo = q + 2.0 * p * cos(phi + 2.0943951023931957);  // + 2 pi / 3
  w[2] = hi;
  w[0] = lo;
  w[1] = 3.0 * q - hi - lo;
}

// unit eigenvector of eigenvalue lam (fp64): the largest cross product of two rows of
// A - lam I.  Returns false when lam is within 1e-3 of the spread from another eigenvalue
// (the caller then falls back to the Jacobi iteration for this voxel).
__device__ inline bool sym3_eigvec_closed(double a00, double a01, double a02, double a11,
                                          double a12, double a22, double lam, double gap,
                                          double spread, double v[3]) {
#pragma clang fp contract(off)
  if (!(gap > 1e-3 * spread)) return false;
  const double r0[3] = {a00 - lam, a01, a02};
  const double r1[3] = {a01, a11 - lam, a12};
  const double r2[3] = {a02, a12, a22 - lam};
  auto cross = [](const double* x, const double* y, double* z) {
    z[0] = x[1] * y[2] - x[2] * y[1];
    z[1] = x[2] * y[0] - x[0] * y[2];
    z[2] = x[0] * y[1] - x[1] * y[0];
  };
  double c0[3], c1[3], c2[3];
  cross(r0, r1, c0);
  cross(r0, r2, c1);
  cross(r1, r2, c2);
  const double n0 = c0[0] * c0[0] + c0[1] * c0[1] + c0[2] * c0[2];
  const double n1 = c1[0] * c1[0] + c1[1] * c1[1] + c1[2] * c1[2];
  const double n2 = c2[0] * c2[0] + c2[1] * c2[1] + c2[2] * c2[2];
  const double* c = c0;
  double n = n0;
  if (n1 > n) { c = c1; n = n1; }
  if (n2 > n) { c = c2; n = n2; }
  if (!(n > 0.0)) return false;
  const double in = 1.0 / sqrt(n);
  v[0] = c[0] * in;
  v[1] = c[1] * in;
  v[2] = c[2] * in;
  return true;
}

// VesselnessFunction (VED.hxx:176-212) on eigenvalues sorted by magnitude, in E; the
// reference's unqualified abs() on doubles is fabs.
template <typename E>
__device__ inline E ved_vesselness(E e0, E e1, E e2, const VesselParams& vp) {
  if (e1 >= E(0) || e2 >= E(0)) return E(0);
  const E smoothC = E(1e-5);
  const E aden = E(2.0 * vp.alpha * vp.alpha);
  const E bden = E(2.0 * vp.beta * vp.beta);
  const E gden = E(2.0 * vp.gamma * vp.gamma);
  const E anum = (e1 * e1) / (e2 * e2);
  const E bnum = (e0 * e0) / fabs(e1 * e2);
  const E gnum = (e0 * e0) + (e1 * e1) + (e2 * e2);
  const E sf = exp(-(E(2) * smoothC * smoothC) / (fabs(e1) * e2 * e2));
  return sf * (E(1) - exp(-anum / aden)) * exp(-bnum / bden) * (E(1) - exp(-gnum / gden));
}

enum { VED_HESSIAN = 0, VED_UPDATE = 1 };

template <typename T, int MODE>
__device__ __forceinline__ void ved_point(double H0, double H1, double H2, double H3, double H4,
                                          double H5, int64_t p, int64_t n, double* __restrict__ hess,
                                          double* __restrict__ resp, double* __restrict__ dir,
                                          int first, const VesselParams& vp);

// x pass + (MODE == VED_HESSIAN) write the scale-normalised Hessian, fp64 SoA, or
// (MODE == VED_UPDATE) UpdateVesselness: eigen-analysis, vesselness, keep the response
// and the eigenvector of the largest (algebraic) eigenvalue -- the column
// GenerateDiffusionTensor weights with omega -- of the scale with the largest response
// (first scale unconditionally, later ones on a strict >, VED.hxx:272).
template <typename T, int MODE>
__global__ void __launch_bounds__(256) ved_fir_x_k(const T* __restrict__ a00, const T* __restrict__ a10,
                                                   const T* __restrict__ a20, const T* __restrict__ a01,
                                                   const T* __restrict__ a11, const T* __restrict__ a02,
                                                   const T* __restrict__ taps, int R, int nx, int ny,
                                                   int nz, HessScale hs, double* __restrict__ hess,
                                                   double* __restrict__ resp, double* __restrict__ dir,
                                                   int first, VesselParams vp) {
#pragma clang fp contract(off)
  // block = 256 consecutive x of one row; LDS: the six input rows over [x0-R, x0+256+R)
  extern __shared__ __align__(16) unsigned char ved_smem[];
  T* L = reinterpret_cast<T*>(ved_smem);
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * 256;
  const int i = x0 + tid;
  const int j = blockIdx.y;
  const int k = blockIdx.z;
  const int64_t n = (int64_t)nx * ny * nz;
  const int64_t row = ((int64_t)k * ny + j) * nx;
  const int nw = 256 + 2 * R;
  for (int e = tid; e < nw; e += 256) {
    const int64_t q = row + min(max(x0 - R + e, 0), nx - 1);
    L[e] = a00[q];
    L[nw + e] = a10[q];
    L[2 * nw + e] = a20[q];
    L[3 * nw + e] = a01[q];
    L[4 * nw + e] = a11[q];
    L[5 * nw + e] = a02[q];
  }
  __syncthreads();
  if (i >= nx) return;
  const int W = 2 * R + 1;
  T hxx = T(0), hxy = T(0), hyy = T(0), hxz = T(0), hyz = T(0), hzz = T(0);
  const T* c = L + tid;
#pragma unroll 4
  for (int q = 0; q < W; ++q) {
    const T k0 = taps[q], k1 = taps[W + q], k2 = taps[2 * W + q];
    hxx = fma(k2, c[q], hxx);
    hxy = fma(k1, c[nw + q], hxy);
    hyy = fma(k0, c[2 * nw + q], hyy);
    hxz = fma(k1, c[3 * nw + q], hxz);
    hyz = fma(k0, c[4 * nw + q], hyz);
    hzz = fma(k0, c[5 * nw + q], hzz);
  }
  const double H0 = (double)hxx * hs.f[0], H1 = (double)hxy * hs.f[1], H2 = (double)hxz * hs.f[2];
  const double H3 = (double)hyy * hs.f[3], H4 = (double)hyz * hs.f[4], H5 = (double)hzz * hs.f[5];
  ved_point<T, MODE>(H0, H1, H2, H3, H4, H5, row + i, n, hess, resp, dir, first, vp);
}

// one voxel's scale-normalised Hessian [xx,xy,xz,yy,yz,zz] (fp64): written out (MODE
// VED_HESSIAN) or UpdateVesselness (VED_UPDATE), see ved_fir_x_k
template <typename T, int MODE>
__device__ __forceinline__ void ved_point(double H0, double H1, double H2, double H3, double H4,
                                          double H5, int64_t p, int64_t n, double* __restrict__ hess,
                                          double* __restrict__ resp, double* __restrict__ dir,
                                          int first, const VesselParams& vp) {
#pragma clang fp contract(off)
  if (MODE == VED_HESSIAN) {
    hess[p] = H0;
    hess[n + p] = H1;
    hess[2 * n + p] = H2;
    hess[3 * n + p] = H3;
    hess[4 * n + p] = H4;
    hess[5 * n + p] = H5;
    return;
  }
  // eigen-analysis and vesselness in the storage precision T (fp64 = the reference's
  // Precision, cyclic Jacobi; fp32 in the fp32 mode, like the solver: closed-form
  // eigenvalues, and the eigenvector -- only where this scale's response wins -- from
  // cross products, with the Jacobi iteration as the fallback for near-degenerate cases)
  const T A0 = (T)H0, A1 = (T)H1, A2 = (T)H2, A3 = (T)H3, A4 = (T)H4, A5 = (T)H5;
  T w[3], V[3][3];
  double wd[3], spread = 0.0;
  if constexpr (sizeof(T) == 4) {
    // the fp32 Hessian components, widened: the closed form runs in fp64
    sym3_eigvals_closed(A0, A1, A2, A3, A4, A5, wd, spread);
    w[0] = (T)wd[0]; w[1] = (T)wd[1]; w[2] = (T)wd[2];
  } else {
    sym3_eigen<T>(A0, A1, A2, A3, A4, A5, w, V);
  }
  // sort by magnitude with the reference's three swaps (VED.hxx:266-268)
  T e0 = w[0], e1 = w[1], e2 = w[2], tt;
  if (fabs(e0) > fabs(e1)) { tt = e0; e0 = e1; e1 = tt; }
  if (fabs(e1) > fabs(e2)) { tt = e1; e1 = e2; e2 = tt; }
  if (fabs(e0) > fabs(e1)) { tt = e0; e0 = e1; e1 = tt; }
  const double v = (double)ved_vesselness<T>(e0, e1, e2, vp);
  if (first || v > resp[p]) {
    T d[3];
    if constexpr (sizeof(T) == 4) {
      double dd[3];
      if (sym3_eigvec_closed(A0, A1, A2, A3, A4, A5, wd[2], wd[2] - wd[1], spread, dd)) {
        d[0] = (T)dd[0]; d[1] = (T)dd[1]; d[2] = (T)dd[2];
      } else {
        sym3_eigen<T>(A0, A1, A2, A3, A4, A5, w, V);
        d[0] = V[0][2]; d[1] = V[1][2]; d[2] = V[2][2];
      }
    } else {
      d[0] = V[0][2]; d[1] = V[1][2]; d[2] = V[2][2];
    }
    resp[p] = v;
    dir[p] = (double)d[0];
    dir[n + p] = (double)d[1];
    dir[2 * n + p] = (double)d[2];
  }
}

// ---------------------------------------------------------------------------
// ITK's HessianRecursiveGaussianImageFilter operator (the reference's ComputeHessian,
// VED.hxx:158-173): per axis a recursive (IIR) Gaussian / derivative filter, ITK
// RecursiveGaussianImageFilter's algorithm (Deriche 4th order; coefficients computed on the
// host, ved_iir_coef in mad_ved.hpp, restating oracle/ved_oracle.py recursive_coefficients).
// One thread per line: a causal pass (initial state: the first value extends to -infinity)
// writes the output, an anticausal pass (last value to +infinity) adds its part, then the
// output is scaled (x pass: sigma^2 / (h_i h_j)).  Arithmetic in fp64 (ITK's RealType), in
// the oracle's order with contraction off; the volumes between passes are stored as SI / SO
// (fp64 in the fp64 mode, fp32 in the fp32 mode, where the causal part is rounded once
// before the anticausal part is added).
struct IirCoef {
  double n[4], m[4], d[4], bn[4], bm[4];
};
struct IirPass {
  const void* in[6];  // SI (kernel template argument) volumes
  void* out[6];       // SO volumes
  int src[6];       // input of each output
  IirCoef c[6];     // its filter along this pass's axis
  double scale[6];  // applied to the finished output
  int nout;
};

template <typename SI, typename SO>
__global__ void __launch_bounds__(256) ved_iir_k(IirPass P, int axis, int nx, int ny, int nz) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t base, st;
  int n;
  if (axis == 0) {  // lines along x, one per (y, z)
    if (t >= (int64_t)ny * nz) return;
    base = t * nx;
    st = 1;
    n = nx;
  } else if (axis == 1) {  // along y, one per (x, z): consecutive threads, consecutive x
    if (t >= (int64_t)nx * nz) return;
    const int64_t i = t % nx, k = t / nx;
    base = k * nx * ny + i;
    st = nx;
    n = ny;
  } else {  // along z, one per (x, y)
    if (t >= (int64_t)nx * ny) return;
    base = t;
    st = (int64_t)nx * ny;
    n = nz;
  }
  for (int o = 0; o < P.nout; ++o) {
    const SI* x = static_cast<const SI*>(P.in[P.src[o]]) + base;
    SO* y = static_cast<SO*>(P.out[o]) + base;
    const IirCoef& c = P.c[o];
    const double N0 = c.n[0], N1 = c.n[1], N2 = c.n[2], N3 = c.n[3];
    const double D1 = c.d[0], D2 = c.d[1], D3 = c.d[2], D4 = c.d[3];
    // causal
    {
      const double v = x[0], x1 = x[st], x2 = x[2 * st], x3 = x[3 * st];
      double s0 = v * N0 + v * N1 + v * N2 + v * N3;
      double s1 = x1 * N0 + v * N1 + v * N2 + v * N3;
      double s2 = x2 * N0 + x1 * N1 + v * N2 + v * N3;
      double s3 = x3 * N0 + x2 * N1 + x1 * N2 + v * N3;
      s0 -= v * c.bn[0] + v * c.bn[1] + v * c.bn[2] + v * c.bn[3];
      s1 -= s0 * D1 + v * c.bn[1] + v * c.bn[2] + v * c.bn[3];
      s2 -= s1 * D1 + s0 * D2 + v * c.bn[2] + v * c.bn[3];
      s3 -= s2 * D1 + s1 * D2 + s0 * D3 + v * c.bn[3];
      y[0] = s0;
      y[st] = s1;
      y[2 * st] = s2;
      y[3 * st] = s3;
      double xm1 = x3, xm2 = x2, xm3 = x1, sm1 = s3, sm2 = s2, sm3 = s1, sm4 = s0;
      for (int i = 4; i < n; ++i) {
        const double xi = x[i * st];
        double si = xi * N0 + xm1 * N1 + xm2 * N2 + xm3 * N3;
        si -= sm1 * D1 + sm2 * D2 + sm3 * D3 + sm4 * D4;
        y[i * st] = si;
        xm3 = xm2; xm2 = xm1; xm1 = xi;
        sm4 = sm3; sm3 = sm2; sm2 = sm1; sm1 = si;
      }
    }
    // anticausal, added to the causal part, then scaled
    {
      const double M1 = c.m[0], M2 = c.m[1], M3 = c.m[2], M4 = c.m[3];
      const double sc = P.scale[o];
      const double v = x[(int64_t)(n - 1) * st];
      const double xa = v, xb = x[(int64_t)(n - 2) * st], xc = x[(int64_t)(n - 3) * st];
      double a1 = v * M1 + v * M2 + v * M3 + v * M4;                  // a[n-1]
      double a2 = xa * M1 + v * M2 + v * M3 + v * M4;                 // a[n-2]
      double a3 = xb * M1 + xa * M2 + v * M3 + v * M4;                // a[n-3]
      double a4 = xc * M1 + xb * M2 + xa * M3 + v * M4;               // a[n-4]
      a1 -= v * c.bm[0] + v * c.bm[1] + v * c.bm[2] + v * c.bm[3];
      a2 -= a1 * D1 + v * c.bm[1] + v * c.bm[2] + v * c.bm[3];
      a3 -= a2 * D1 + a1 * D2 + v * c.bm[2] + v * c.bm[3];
      a4 -= a3 * D1 + a2 * D2 + a1 * D3 + v * c.bm[3];
      SO* yp = y + (int64_t)(n - 1) * st;
      yp[0] = (yp[0] + a1) * sc;
      yp[-st] = (yp[-st] + a2) * sc;
      yp[-2 * st] = (yp[-2 * st] + a3) * sc;
      yp[-3 * st] = (yp[-3 * st] + a4) * sc;
      // window: x[i], x[i+1], x[i+2], x[i+3] and a[i], a[i+1], a[i+2], a[i+3], from i = n-4
      double w0 = x[(int64_t)(n - 4) * st], w1 = xc, w2 = xb, w3 = xa;
      double b0 = a4, b1 = a3, b2 = a2, b3 = a1;
      for (int i = n - 4; i > 0; --i) {
        double ai = w0 * M1 + w1 * M2 + w2 * M3 + w3 * M4;  // a[i-1]
        ai -= b0 * D1 + b1 * D2 + b2 * D3 + b3 * D4;
        SO* yi = y + (int64_t)(i - 1) * st;
        yi[0] = (yi[0] + ai) * sc;
        w3 = w2; w2 = w1; w1 = w0; w0 = x[(int64_t)(i - 1) * st];
        b3 = b2; b2 = b1; b1 = b0; b0 = ai;
      }
    }
  }
}

// ved_iir_k for the strided axes (z, y: consecutive threads take consecutive x, so every
// access is a coalesced row) with the K outputs that share an input filtered in one march
// (each input value read twice per group -- causal, anticausal -- instead of twice per
// output), the loads of B points issued together (one memory latency per block, not per
// point).  One launch per group; its filters are kernel arguments indexed at compile time.
// Per output the same expressions in the same order as ved_iir_k (bit-identical).
template <int K>
struct IirGroup {
  const void* in;
  void* out[K];
  IirCoef c[K];
  double scale[K];
};

// Lines of the x columns [xa, xa + nxr) (z lines: all y; y lines: the planes [za, za + nzr))
// only -- the whole grid: xa = 0, nxr = nx, za = 0, nzr = nz: a rank of the partitioned VED
// runs the z pass on its x range and the y pass on its tensor planes (ved_scale_iir).  B:
// points per load block (16 and more put the blocks in scratch memory); PIPE: the next block's
// loads are issued before the current block is filtered (two blocks in flight per line: each
// line's memory round trips are the time, most of all in the partitioned passes' few lines).
template <typename SI, typename SO, int K, int B = 8, bool PIPE = false>
__global__ void __launch_bounds__(256) ved_iir_grp_k(IirGroup<K> G, int axis, int nx, int ny, int nz,
                                                     int xa, int nxr, int za, int nzr) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t base, st;
  int n;
  if (axis == 1) {  // along y, one per (x, z)
    if (t >= (int64_t)nxr * nzr) return;
    const int64_t i = xa + t % nxr, k = za + t / nxr;
    base = k * nx * ny + i;
    st = nx;
    n = ny;
  } else {  // along z, one per (x, y)
    if (t >= (int64_t)nxr * ny) return;
    const int64_t i = xa + t % nxr, j = t / nxr;
    base = j * nx + i;
    st = (int64_t)nx * ny;
    n = nz;
  }
  const SI* __restrict__ x = static_cast<const SI*>(G.in) + base;
  SO* y[K];
#pragma unroll
  for (int q = 0; q < K; ++q) y[q] = static_cast<SO*>(G.out[q]) + base;
  // causal
  {
    const double v = x[0], x1 = x[st], x2 = x[2 * st], x3 = x[3 * st];
    double sm1[K], sm2[K], sm3[K], sm4[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const IirCoef& C = G.c[q];
      const double N0 = C.n[0], N1 = C.n[1], N2 = C.n[2], N3 = C.n[3];
      const double D1 = C.d[0], D2 = C.d[1], D3 = C.d[2];
      double s0 = v * N0 + v * N1 + v * N2 + v * N3;
      double s1 = x1 * N0 + v * N1 + v * N2 + v * N3;
      double s2 = x2 * N0 + x1 * N1 + v * N2 + v * N3;
      double s3 = x3 * N0 + x2 * N1 + x1 * N2 + v * N3;
      s0 -= v * C.bn[0] + v * C.bn[1] + v * C.bn[2] + v * C.bn[3];
      s1 -= s0 * D1 + v * C.bn[1] + v * C.bn[2] + v * C.bn[3];
      s2 -= s1 * D1 + s0 * D2 + v * C.bn[2] + v * C.bn[3];
      s3 -= s2 * D1 + s1 * D2 + s0 * D3 + v * C.bn[3];
      y[q][0] = s0;
      y[q][st] = s1;
      y[q][2 * st] = s2;
      y[q][3 * st] = s3;
      sm1[q] = s3; sm2[q] = s2; sm3[q] = s1; sm4[q] = s0;
    }
    double xm1 = x3, xm2 = x2, xm3 = x1;
    SI xn[B];
    if (PIPE) {
#pragma unroll
      for (int u = 0; u < B; ++u) xn[u] = (4 + u < n) ? x[(int64_t)(4 + u) * st] : SI(0);
    }
    for (int i0 = 4; i0 < n; i0 += B) {
      SI xb[B];
      if (PIPE) {
#pragma unroll
        for (int u = 0; u < B; ++u) {
          xb[u] = xn[u];
          xn[u] = (i0 + B + u < n) ? x[(int64_t)(i0 + B + u) * st] : SI(0);
        }
      } else {
#pragma unroll
        for (int u = 0; u < B; ++u) xb[u] = (i0 + u < n) ? x[(int64_t)(i0 + u) * st] : SI(0);
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int i = i0 + u;
        if (i >= n) break;
        const double xi = xb[u];
#pragma unroll
        for (int q = 0; q < K; ++q) {
          const IirCoef& C = G.c[q];
          double si = xi * C.n[0] + xm1 * C.n[1] + xm2 * C.n[2] + xm3 * C.n[3];
          si -= sm1[q] * C.d[0] + sm2[q] * C.d[1] + sm3[q] * C.d[2] + sm4[q] * C.d[3];
          y[q][(int64_t)i * st] = si;
          sm4[q] = sm3[q]; sm3[q] = sm2[q]; sm2[q] = sm1[q]; sm1[q] = si;
        }
        xm3 = xm2; xm2 = xm1; xm1 = xi;
      }
    }
  }
  // anticausal, added to the causal part, then scaled
  {
    const double v = x[(int64_t)(n - 1) * st];
    const double xa = v, xb = x[(int64_t)(n - 2) * st], xc = x[(int64_t)(n - 3) * st];
    double b0[K], b1[K], b2[K], b3[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const IirCoef& C = G.c[q];
      const double M1 = C.m[0], M2 = C.m[1], M3 = C.m[2], M4 = C.m[3];
      const double D1 = C.d[0], D2 = C.d[1], D3 = C.d[2];
      const double sc = G.scale[q];
      double a1 = v * M1 + v * M2 + v * M3 + v * M4;
      double a2 = xa * M1 + v * M2 + v * M3 + v * M4;
      double a3 = xb * M1 + xa * M2 + v * M3 + v * M4;
      double a4 = xc * M1 + xb * M2 + xa * M3 + v * M4;
      a1 -= v * C.bm[0] + v * C.bm[1] + v * C.bm[2] + v * C.bm[3];
      a2 -= a1 * D1 + v * C.bm[1] + v * C.bm[2] + v * C.bm[3];
      a3 -= a2 * D1 + a1 * D2 + v * C.bm[2] + v * C.bm[3];
      a4 -= a3 * D1 + a2 * D2 + a1 * D3 + v * C.bm[3];
      SO* yp = y[q] + (int64_t)(n - 1) * st;
      yp[0] = (yp[0] + a1) * sc;
      yp[-st] = (yp[-st] + a2) * sc;
      yp[-2 * st] = (yp[-2 * st] + a3) * sc;
      yp[-3 * st] = (yp[-3 * st] + a4) * sc;
      b0[q] = a4; b1[q] = a3; b2[q] = a2; b3[q] = a1;
    }
    double w0 = x[(int64_t)(n - 4) * st], w1 = xc, w2 = xb, w3 = xa;
    // blocks of B points downward from i = n-4 (point i-1 each step), loads first (PIPE: the
    // next block's loads ahead; they read causal outputs below the block being finished)
    SI xpn[B];
    SO ybn[K][B];
    if (PIPE) {
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int i = n - 4 - u;
        xpn[u] = (i > 0) ? x[(int64_t)(i - 1) * st] : SI(0);
#pragma unroll
        for (int q = 0; q < K; ++q) ybn[q][u] = (i > 0) ? y[q][(int64_t)(i - 1) * st] : SO(0);
      }
    }
    for (int i0 = n - 4; i0 > 0; i0 -= B) {
      SI xp[B];
      SO yb[K][B];
      if (PIPE) {
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const int i = i0 - B - u;
          xp[u] = xpn[u];
          xpn[u] = (i > 0) ? x[(int64_t)(i - 1) * st] : SI(0);
#pragma unroll
          for (int q = 0; q < K; ++q) {
            yb[q][u] = ybn[q][u];
            ybn[q][u] = (i > 0) ? y[q][(int64_t)(i - 1) * st] : SO(0);
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const int i = i0 - u;
          xp[u] = (i > 0) ? x[(int64_t)(i - 1) * st] : SI(0);
#pragma unroll
          for (int q = 0; q < K; ++q) yb[q][u] = (i > 0) ? y[q][(int64_t)(i - 1) * st] : SO(0);
        }
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int i = i0 - u;
        if (i <= 0) break;
#pragma unroll
        for (int q = 0; q < K; ++q) {
          const IirCoef& C = G.c[q];
          double ai = w0 * C.m[0] + w1 * C.m[1] + w2 * C.m[2] + w3 * C.m[3];
          ai -= b0[q] * C.d[0] + b1[q] * C.d[1] + b2[q] * C.d[2] + b3[q] * C.d[3];
          y[q][(int64_t)(i - 1) * st] = (yb[q][u] + ai) * G.scale[q];
          b3[q] = b2[q]; b2[q] = b1[q]; b1[q] = b0[q]; b0[q] = ai;
        }
        w3 = w2; w2 = w1; w1 = w0; w0 = xp[u];
      }
    }
  }
}

// The x-axis pass of ved_iir_k with coalesced memory access.  Lines along x are contiguous
// rows, so one thread per line reads 64 different rows per instruction; here one wave
// takes 64 consecutive lines and one output, and every chunk of C points goes through an
// LDS tile [64 lines][C] (+1 pad; one tile, reused for x and y): rows are loaded / stored by the whole wave (C doubles
// per row, contiguous), each lane then runs its line's recursion on the tile.  Same
// recursion, same expressions in the same order as ved_iir_k (bit-identical): the causal
// and anticausal passes are written as per-point state machines over a sliding window,
// with the first four points of each direction taking ved_iir_k's edge formulas.
// lines [lbase, nlines) (x rows, row index j + ny k): all of them on one GPU, a rank's tensor
// planes in the partitioned VED
template <typename SI, typename SO, int C = 128 / (int)sizeof(SO)>
__global__ void __launch_bounds__(64) ved_iir_x_k(IirPass P, int nx, int64_t lbase, int64_t nlines) {
#pragma clang fp contract(off)
  static_assert(sizeof(SI) == sizeof(SO), "the x pass reads and writes the volumes' storage type");
  static_assert(64 % C == 0, "whole rows per wave instruction");
  // tiles of the storage type (x chunk, y chunk), C values per row: LDS per wave bounds the
  // waves per CU; a chunk of half a 128-B line leaves the other half to a later chunk
  __shared__ SO tx[64 * (C + 1)];
  __shared__ SO ty[64 * (C + 1)];
  constexpr int RPI = 64 / C;  // rows per wave instruction
  const int o = blockIdx.y;
  const int lane = threadIdx.x;
  const int64_t line0 = lbase + (int64_t)blockIdx.x * 64;
  const SI* __restrict__ x = static_cast<const SI*>(P.in[P.src[o]]);
  SO* __restrict__ y = static_cast<SO*>(P.out[o]);
  const IirCoef c = P.c[o];
  const double sc = P.scale[o];
  const int n = nx;
  // wave-cooperative row transfers of the chunk [i0, i0 + cnt) of lines line0 .. line0+63:
  // instruction q moves rows RPI q + lrow, column lcol (all loads of a chunk in flight
  // together, then the LDS writes).  Buffer accesses over the block's lines (record range),
  // per-lane byte offsets; rows past the volume are masked (loads give 0, no stores).
  const int lrow = lane / C, lcol = lane % C;
  const int64_t nl = min((int64_t)64, nlines - line0);
  const uint32_t nbytes = (uint32_t)(nl * n * (int64_t)sizeof(SO));
  const uint32_t lofs = (uint32_t)((lrow * n + lcol) * (int)sizeof(SO));
  const uint32_t qstep = (uint32_t)(RPI * n * (int)sizeof(SO));
  auto rsrc = [&](const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
  };
  auto load_tile = [&](const SO* __restrict__ src, SO* t, int i0, int cnt) {
    const auto r = rsrc(src + line0 * n);
    const uint32_t off = lofs + (uint32_t)(i0 * (int)sizeof(SO));
    SO v[C];
#pragma unroll
    for (int q = 0; q < C; ++q) {
      v[q] = SO(0);
      if (RPI * q + lrow < nl) {
        const int vo = (int)(off + (uint32_t)q * qstep);
        if constexpr (sizeof(SO) == 4)
          v[q] = __builtin_bit_cast(SO, __builtin_amdgcn_raw_buffer_load_b32(r, vo, 0, 0));
        else
          v[q] = __builtin_bit_cast(SO, __builtin_amdgcn_raw_buffer_load_b64(r, vo, 0, 0));
      }
    }
#pragma unroll
    for (int q = 0; q < C; ++q) t[(RPI * q + lrow) * (C + 1) + lcol] = v[q];
  };
  auto store_tile = [&](SO* __restrict__ dst, const SO* t, int i0, int cnt) {
    const auto r = rsrc(dst + line0 * n);
    const uint32_t off = lofs + (uint32_t)(i0 * (int)sizeof(SO));
    if (lcol >= cnt) return;
#pragma unroll
    for (int q = 0; q < C; ++q) {
      if (RPI * q + lrow >= nl) continue;
      const SO w = t[(RPI * q + lrow) * (C + 1) + lcol];
      const int vo = (int)(off + (uint32_t)q * qstep);
      if constexpr (sizeof(SO) == 4) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, w), r, vo, 0, 0);
      } else {
        using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, w), r, vo, 0, 0);
      }
    }
  };
  SO* mx = tx + lane * (C + 1);
  SO* my = ty + lane * (C + 1);
  const double N0 = c.n[0], N1 = c.n[1], N2 = c.n[2], N3 = c.n[3];
  const double D1 = c.d[0], D2 = c.d[1], D3 = c.d[2], D4 = c.d[3];
  // ---- causal: s[i] into y
  double v = 0.0, x1 = 0.0, x2 = 0.0;                        // x[0], x[1], x[2] (edge formulas)
  double xm1 = 0.0, xm2 = 0.0, xm3 = 0.0;                    // x[i-1], x[i-2], x[i-3]
  double sm1 = 0.0, sm2 = 0.0, sm3 = 0.0, sm4 = 0.0;         // s[i-1] .. s[i-4]
  for (int i0 = 0; i0 < n; i0 += C) {
    const int cnt = min(C, n - i0);
    load_tile(x, tx, i0, cnt);
    __syncthreads();
    for (int j = 0; j < cnt; ++j) {
      const int i = i0 + j;
      const double xi = mx[j];
      double si;
      if (i == 0) {
        v = xi;
        si = v * N0 + v * N1 + v * N2 + v * N3;
        si -= v * c.bn[0] + v * c.bn[1] + v * c.bn[2] + v * c.bn[3];
      } else if (i == 1) {
        x1 = xi;
        si = x1 * N0 + v * N1 + v * N2 + v * N3;
        si -= sm1 * D1 + v * c.bn[1] + v * c.bn[2] + v * c.bn[3];
      } else if (i == 2) {
        x2 = xi;
        si = x2 * N0 + x1 * N1 + v * N2 + v * N3;
        si -= sm1 * D1 + sm2 * D2 + v * c.bn[2] + v * c.bn[3];
      } else if (i == 3) {
        si = xi * N0 + x2 * N1 + x1 * N2 + v * N3;
        si -= sm1 * D1 + sm2 * D2 + sm3 * D3 + v * c.bn[3];
      } else {
        si = xi * N0 + xm1 * N1 + xm2 * N2 + xm3 * N3;
        si -= sm1 * D1 + sm2 * D2 + sm3 * D3 + sm4 * D4;
      }
      mx[j] = si;  // in place: x[i] is consumed
      xm3 = xm2; xm2 = xm1; xm1 = xi;
      sm4 = sm3; sm3 = sm2; sm2 = sm1; sm1 = si;
    }
    __syncthreads();
    store_tile(y, tx, i0, cnt);
    __syncthreads();
  }
  // ---- anticausal: a[k] from x[k+1 ..] and a[k+1 ..], y[k] = (s[k] + a[k]) * sc
  const double M1 = c.m[0], M2 = c.m[1], M3 = c.m[2], M4 = c.m[3];
  double V = 0.0, xa = 0.0, xb = 0.0;                        // x[n-1], x[n-1], x[n-2] (edge)
  double w0 = 0.0, w1 = 0.0, w2 = 0.0, w3 = 0.0;             // x[k+1] .. x[k+4]
  double b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;             // a[k+1] .. a[k+4]
  const int nch = (n + C - 1) / C;
  for (int ch = nch - 1; ch >= 0; --ch) {
    const int i0 = ch * C, cnt = min(C, n - i0);
    load_tile(x, tx, i0, cnt);
    load_tile(y, ty, i0, cnt);
    __syncthreads();
    for (int j = cnt - 1; j >= 0; --j) {
      const int k = i0 + j, m = n - 1 - k;
      const double xk = mx[j];
      double ak;
      if (m == 0) {
        V = xk;
        xa = xk;
        ak = V * M1 + V * M2 + V * M3 + V * M4;
        ak -= V * c.bm[0] + V * c.bm[1] + V * c.bm[2] + V * c.bm[3];
      } else if (m == 1) {
        ak = xa * M1 + V * M2 + V * M3 + V * M4;
        ak -= b0 * D1 + V * c.bm[1] + V * c.bm[2] + V * c.bm[3];
        xb = xk;
      } else if (m == 2) {
        ak = xb * M1 + xa * M2 + V * M3 + V * M4;
        ak -= b0 * D1 + b1 * D2 + V * c.bm[2] + V * c.bm[3];
      } else if (m == 3) {
        ak = w0 * M1 + xb * M2 + xa * M3 + V * M4;
        ak -= b0 * D1 + b1 * D2 + b2 * D3 + V * c.bm[3];
      } else {
        ak = w0 * M1 + w1 * M2 + w2 * M3 + w3 * M4;
        ak -= b0 * D1 + b1 * D2 + b2 * D3 + b3 * D4;
      }
      my[j] = (my[j] + ak) * sc;
      w3 = w2; w2 = w1; w1 = w0; w0 = xk;
      b3 = b2; b2 = b1; b1 = b0; b0 = ak;
    }
    __syncthreads();
    store_tile(y, ty, i0, cnt);
    __syncthreads();
  }
}

// UpdateVesselness / Hessian output from the six recursive-Hessian volumes
// (points [p0, p1) of the n-point volumes)
template <typename T, int MODE, typename S = double>
__global__ void __launch_bounds__(256) ved_hess_k(const S* __restrict__ H, int64_t n, int64_t p0, int64_t p1,
                                                  double* __restrict__ hess, double* __restrict__ resp,
                                                  double* __restrict__ dir, int first, VesselParams vp) {
  for (int64_t p = p0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < p1;
       p += (int64_t)gridDim.x * blockDim.x)
    ved_point<T, MODE>(H[p], H[n + p], H[2 * n + p], H[3 * n + p], H[4 * n + p], H[5 * n + p], p, n,
                       hess, resp, dir, first, vp);
}

// Partitioned VED transpose: six volumes' block [z0, z0 + nzb) x [0, ny) x [x0, x0 + nxb) to or
// from a contiguous buffer (volume-major, then z, y, x), UNPACK = buffer -> volumes.
template <typename T>
struct Vol6 {
  T* v[6];
};
// nv volumes, one element per thread over the whole block (32-bit indices: a block holds < 2^31
// elements), grid-stride
template <typename T, bool UNPACK>
__global__ void __launch_bounds__(256) ved_block_k(Vol6<T> V, T* __restrict__ buf, int nx, int ny, int x0,
                                                   int nxb, int z0, int nzb, int nv) {
  const uint32_t tot = (uint32_t)nv * nzb * ny * nxb;
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < tot; q += gridDim.x * 256u) {
    const uint32_t row = q / (uint32_t)nxb, i = q - row * (uint32_t)nxb;
    const uint32_t ck = row / (uint32_t)ny, j = row - ck * (uint32_t)ny;
    const uint32_t c = ck / (uint32_t)nzb, kl = ck - c * (uint32_t)nzb;
    T* vp = V.v[c] + ((int64_t)(z0 + (int)kl) * ny + j) * nx + x0 + i;
    if (UNPACK) *vp = buf[q];
    else buf[q] = *vp;
  }
}

// GenerateDiffusionTensor (VED.hxx:302-378) into the solver's fp64 SoA tensor
// [xx,xy,xz,yy,yz,zz]: V = resp^(1/s); where V > 0, T = Q D Q^T with
// D = diag(a, a, c), a = 1 + (eps-1) V, c = 1 + (omega-1) V on vnl's column order,
// i.e. T = a I + (c - a) v v^T with v the third column; identity elsewhere.
__global__ void __launch_bounds__(256) ved_tensor_k(const double* __restrict__ resp,
                                                    const double* __restrict__ dir,
                                                    double* __restrict__ T, int64_t n, int64_t q0,
                                                    int64_t q1, int64_t cs, double eps,
                                                    double omega, double sens) {
  // points [q0, q1) of the n-point grid (a rank slab's tensor planes); T at global point 0 with
  // component stride cs (= n on one GPU)
  for (int64_t q = q0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < q1;
       q += (int64_t)gridDim.x * blockDim.x) {
    const double V = pow(resp[q], 1. / sens);
    if (V > 0) {
      const double a = 1. + (eps - 1.) * V;
      const double c = 1. + (omega - 1.) * V;
      const double d = c - a;
      const double v0 = dir[q], v1 = dir[n + q], v2 = dir[2 * n + q];
      T[q] = a + d * v0 * v0;
      T[cs + q] = d * v0 * v1;
      T[2 * cs + q] = d * v0 * v2;
      T[3 * cs + q] = a + d * v1 * v1;
      T[4 * cs + q] = d * v1 * v2;
      T[5 * cs + q] = a + d * v2 * v2;
    } else {
      T[q] = 1.;
      T[cs + q] = 0.;
      T[2 * cs + q] = 0.;
      T[3 * cs + q] = 1.;
      T[4 * cs + q] = 0.;
      T[5 * cs + q] = 1.;
    }
  }
}

}  // namespace mad
