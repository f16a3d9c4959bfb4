// mad_ved_kernels.hpp -- device kernels of the VED tensor generation (include/mad_ved.h).
//
// Reference: include/itkVEDMultigridImageFilter.hxx (VED.hxx below).
//   ComputeHessian          VED.hxx:158-173  -> ved_fir_{z,y}_k + ved_fir_x_k
//   VesselnessFunction      VED.hxx:176-212  -> ved_vesselness
//   UpdateVesselness        VED.hxx:215-299  -> ved_fir_x_k<.., VED_UPDATE> (fused)
//   GenerateDiffusionTensor VED.hxx:302-378  -> ved_tensor_k
//
// The scale-normalised Hessian is three separable correlation passes with sampled,
// moment-normalised Gaussian derivative taps (computed on the host, ved_taps in
// mad_ved.hpp): z (image -> 3 derivative orders), y (-> the 6 (y, z) order pairs the
// Hessian needs), then x, fused with the per-voxel eigen-analysis, vesselness and the
// running maximum over scales, so the 6 Hessian components never reach HBM.
// Storage / FIR arithmetic in T (fp32 or fp64, explicit fma); the eigen-analysis,
// vesselness, response and vessel direction are fp64 (the reference's Precision).
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

// z pass: o_q(i,j,k) = sum_t K_q(t) in(i, j, clamp(k + t)), q = 0, 1, 2 (orders).
// taps: [K0 | K1 | K2], each 2R+1 long.  Reads of `in` (fp64 image) are coalesced in x.
template <typename T>
__global__ void __launch_bounds__(256) ved_fir_z_k(const double* __restrict__ in, T* __restrict__ o0,
                                                   T* __restrict__ o1, T* __restrict__ o2,
                                                   const T* __restrict__ taps, int R, int nx, int ny,
                                                   int nz) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= nx || j >= ny) return;
  const int64_t sz = (int64_t)nx * ny;
  const int64_t col = (int64_t)j * nx + i;
  const int W = 2 * R + 1;
  T a0 = T(0), a1 = T(0), a2 = T(0);
  for (int t = -R; t <= R; ++t) {
    const int kk = min(max(k + t, 0), nz - 1);
    const T v = (T)in[kk * sz + col];
    a0 = fma(taps[t + R], v, a0);
    a1 = fma(taps[W + t + R], v, a1);
    a2 = fma(taps[2 * W + t + R], v, a2);
  }
  const int64_t p = k * sz + col;
  o0[p] = a0;
  o1[p] = a1;
  o2[p] = a2;
}

// y pass: the six (y order, z order) pairs of the Hessian:
//   a00 = K0y z0, a10 = K1y z0, a20 = K2y z0, a01 = K0y z1, a11 = K1y z1, a02 = K0y z2
template <typename T>
__global__ void __launch_bounds__(256) ved_fir_y_k(const T* __restrict__ z0, const T* __restrict__ z1,
                                                   const T* __restrict__ z2, T* __restrict__ a00,
                                                   T* __restrict__ a10, T* __restrict__ a20,
                                                   T* __restrict__ a01, T* __restrict__ a11,
                                                   T* __restrict__ a02, const T* __restrict__ taps,
                                                   int R, int nx, int ny, int nz) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= nx || j >= ny) return;
  const int64_t sz = (int64_t)nx * ny;
  const int64_t pl = k * sz + i;
  const int W = 2 * R + 1;
  T s00 = T(0), s10 = T(0), s20 = T(0), s01 = T(0), s11 = T(0), s02 = T(0);
  for (int t = -R; t <= R; ++t) {
    const int jj = min(max(j + t, 0), ny - 1);
    const int64_t q = pl + (int64_t)jj * nx;
    const T v0 = z0[q], v1 = z1[q], v2 = z2[q];
    const T k0 = taps[t + R], k1 = taps[W + t + R], k2 = taps[2 * W + t + R];
    s00 = fma(k0, v0, s00);
    s10 = fma(k1, v0, s10);
    s20 = fma(k2, v0, s20);
    s01 = fma(k0, v1, s01);
    s11 = fma(k1, v1, s11);
    s02 = fma(k0, v2, s02);
  }
  const int64_t p = pl + (int64_t)j * nx;
  a00[p] = s00;
  a10[p] = s10;
  a20[p] = s20;
  a01[p] = s01;
  a11[p] = s11;
  a02[p] = s02;
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi rotations (fp64): w ascending,
// V columns the matching unit eigenvectors -- the order vnl_symmetric_eigensystem
// returns (VED.hxx:259-264).  Converges quadratically; stops when the off-diagonal
// mass is below 1e-17 of the diagonal's.
__device__ inline void sym3_eigen(double a00, double a01, double a02, double a11, double a12,
                                  double a22, double w[3], double V[3][3]) {
#pragma clang fp contract(off)
  double A[3][3] = {{a00, a01, a02}, {a01, a11, a12}, {a02, a12, a22}};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) V[r][c] = (r == c) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 24; ++sweep) {
    const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
    const double dia = fabs(A[0][0]) + fabs(A[1][1]) + fabs(A[2][2]);
    if (!(off > 1e-17 * dia) || off < 1e-300) break;
#pragma unroll
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0;
      const int q = pq == 0 ? 1 : 2;
      const int r = 3 - p - q;
      const double apq = A[p][q];
      if (fabs(apq) < 1e-300) continue;
      const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
      double t;
      if (fabs(theta) > 1e150) {
        t = 0.5 / theta;
      } else {
        t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
        if (theta < 0.0) t = -t;
      }
      const double c = 1.0 / sqrt(t * t + 1.0);
      const double s = t * c;
      A[p][p] -= t * apq;
      A[q][q] += t * apq;
      A[p][q] = A[q][p] = 0.0;
      const double arp = A[r][p], arq = A[r][q];
      A[r][p] = A[p][r] = c * arp - s * arq;
      A[r][q] = A[q][r] = s * arp + c * arq;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double vkp = V[k][p], vkq = V[k][q];
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
      const double tw = w[a];
      w[a] = w[b];
      w[b] = tw;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double tv = V[k][a];
        V[k][a] = V[k][b];
        V[k][b] = tv;
      }
    }
  };
  sw(0, 1);
  sw(1, 2);
  sw(0, 1);
}

// VesselnessFunction (VED.hxx:176-212) on eigenvalues sorted by magnitude; the
// reference's unqualified abs() on doubles is fabs.
__device__ inline double ved_vesselness(double e0, double e1, double e2, const VesselParams& vp) {
  if (e1 >= 0.0 || e2 >= 0.0) return 0.0;
  const double smoothC = 1e-5;
  const double aden = 2.0 * vp.alpha * vp.alpha;
  const double bden = 2.0 * vp.beta * vp.beta;
  const double gden = 2.0 * vp.gamma * vp.gamma;
  const double anum = (e1 * e1) / (e2 * e2);
  const double bnum = (e0 * e0) / fabs(e1 * e2);
  const double gnum = (e0 * e0) + (e1 * e1) + (e2 * e2);
  const double sf = exp(-(2 * smoothC * smoothC) / (fabs(e1) * e2 * e2));
  return sf * (1. - exp(-anum / aden)) * exp(-bnum / bden) * (1. - exp(-gnum / gden));
}

enum { VED_HESSIAN = 0, VED_UPDATE = 1 };

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
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= nx || j >= ny) return;
  const int64_t n = (int64_t)nx * ny * nz;
  const int64_t row = ((int64_t)k * ny + j) * nx;
  const int W = 2 * R + 1;
  T hxx = T(0), hxy = T(0), hyy = T(0), hxz = T(0), hyz = T(0), hzz = T(0);
  for (int t = -R; t <= R; ++t) {
    const int64_t q = row + min(max(i + t, 0), nx - 1);
    const T k0 = taps[t + R], k1 = taps[W + t + R], k2 = taps[2 * W + t + R];
    hxx = fma(k2, a00[q], hxx);
    hxy = fma(k1, a10[q], hxy);
    hyy = fma(k0, a20[q], hyy);
    hxz = fma(k1, a01[q], hxz);
    hyz = fma(k0, a11[q], hyz);
    hzz = fma(k0, a02[q], hzz);
  }
  const double H0 = (double)hxx * hs.f[0], H1 = (double)hxy * hs.f[1], H2 = (double)hxz * hs.f[2];
  const double H3 = (double)hyy * hs.f[3], H4 = (double)hyz * hs.f[4], H5 = (double)hzz * hs.f[5];
  const int64_t p = row + i;
  if (MODE == VED_HESSIAN) {
    hess[p] = H0;
    hess[n + p] = H1;
    hess[2 * n + p] = H2;
    hess[3 * n + p] = H3;
    hess[4 * n + p] = H4;
    hess[5 * n + p] = H5;
    return;
  }
  double w[3], V[3][3];
  sym3_eigen(H0, H1, H2, H3, H4, H5, w, V);
  // sort by magnitude with the reference's three swaps (VED.hxx:266-268)
  double e0 = w[0], e1 = w[1], e2 = w[2], tt;
  if (fabs(e0) > fabs(e1)) { tt = e0; e0 = e1; e1 = tt; }
  if (fabs(e1) > fabs(e2)) { tt = e1; e1 = e2; e2 = tt; }
  if (fabs(e0) > fabs(e1)) { tt = e0; e0 = e1; e1 = tt; }
  const double v = ved_vesselness(e0, e1, e2, vp);
  if (first || v > resp[p]) {
    resp[p] = v;
    dir[p] = V[0][2];
    dir[n + p] = V[1][2];
    dir[2 * n + p] = V[2][2];
  }
}

// GenerateDiffusionTensor (VED.hxx:302-378) into the solver's fp64 SoA tensor
// [xx,xy,xz,yy,yz,zz]: V = resp^(1/s); where V > 0, T = Q D Q^T with
// D = diag(a, a, c), a = 1 + (eps-1) V, c = 1 + (omega-1) V on vnl's column order,
// i.e. T = a I + (c - a) v v^T with v the third column; identity elsewhere.
__global__ void __launch_bounds__(256) ved_tensor_k(const double* __restrict__ resp,
                                                    const double* __restrict__ dir,
                                                    double* __restrict__ T, int64_t n, double eps,
                                                    double omega, double sens) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const double V = pow(resp[q], 1. / sens);
    if (V > 0) {
      const double a = 1. + (eps - 1.) * V;
      const double c = 1. + (omega - 1.) * V;
      const double d = c - a;
      const double v0 = dir[q], v1 = dir[n + q], v2 = dir[2 * n + q];
      T[q] = a + d * v0 * v0;
      T[n + q] = d * v0 * v1;
      T[2 * n + q] = d * v0 * v2;
      T[3 * n + q] = a + d * v1 * v1;
      T[4 * n + q] = d * v1 * v2;
      T[5 * n + q] = a + d * v2 * v2;
    } else {
      T[q] = 1.;
      T[n + q] = 0.;
      T[2 * n + q] = 0.;
      T[3 * n + q] = 1.;
      T[4 * n + q] = 0.;
      T[5 * n + q] = 1.;
    }
  }
}

}  // namespace mad
