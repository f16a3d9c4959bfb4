// mad_coarse.hpp -- direct solver of a large coarsest level (DirectSolver,
// include/mad/itkDirectSolver.hxx:32-147).
//
// The reference LU-factors the coarsest operator with vnl_sparse_lu at construction
// (DS.hxx:81-86) and solves with it once per V-cycle (DS.hxx:129).  Small coarsest
// levels (the 512 .. 2048 unknowns of C2-C5) keep the dense explicit inverse in
// mad_solver.hip.  A large one -- the grid stops coarsening when one axis drops below 6,
// so a thin volume (512x512x64 -> 64x64x8, or any axis < 12: the whole grid) leaves
// tens of thousands to millions of unknowns -- is solved here by a block-plane
// factorisation:
//
//   unknowns renumbered with the longest axis outermost ("planes" orthogonal to it,
//   q unknowns each, the two shorter axes inside, shortest fastest); the radius-1
//   stencil couples a plane only to its two neighbours, so with blocks of P planes
//   (mb = P q rows) A is block tridiagonal with couplings between the last plane of
//   block i and the first plane of block i+1 (E_i: block i -> i-1, F_i: i -> i+1,
//   <= 5 entries per row).  Block LU (Schur complements on the first plane only):
//     D_0 = A_00,  D_i = A_ii - E_i D_{i-1}^{-1}[last, last] F_{i-1}   (q x q update)
//   and the explicit inverses Dinv_i = D_i^{-1} (rocSOLVER getrf + getri per block,
//   partial pivoting inside the block) are stored.  Per solve:
//     c_i = Dinv_i b_i                           all blocks at once (one launch)
//     y_i = c_i - Dinv_i[:, first] (E_i y_{i-1}[last])   chain over the last planes,
//                                                then the other rows at once
//     x_i = y_i - Dinv_i[:, last] (F_i x_{i+1}[first])   chain over the first planes,
//                                                then the other rows at once
//   so the sequential part is 2 (nb - 1) q x q products -- with the chain's matrices
//   KL_i = Dinv_i[last, first] E_i and KU_i = Dinv_i[first, last] F_i formed at setup,
//   one GEMV launch per step (blocks of one plane, q >= the block target, whose KL / KU would
//   not fit next to Dinv, multiply by Dinv_i itself after a sparse E_i y: the same q x q read
//   without 2 q^2 of extra memory per block) -- and everything else is bandwidth-parallel.  All arithmetic fp64 (the reference's), deterministic
//   (one wave per row, fixed reduction order): every rank that replicates the
//   coarsest level computes the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include "mad_alloc.hpp"
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

namespace mad {

// bp[r] = b[iperm[r]] (band order, fp64)
template <typename T>
__global__ void __launch_bounds__(256) cs_gather_k(const T* __restrict__ b, const int* __restrict__ iperm,
                                                   double* __restrict__ bp, int n) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < n) bp[r] = (double)b[iperm[r]];
}

// x[p] = cv[perm[p]] (natural order, storage type)
template <typename T>
__global__ void __launch_bounds__(256) cs_scatter_k(const double* __restrict__ cv, const int* __restrict__ perm,
                                                    T* __restrict__ x, int n) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p < n) x[p] = (T)cv[perm[p]];
}

__device__ __forceinline__ double cs_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// c = Dinv_i b_i for every block: one wave per row (row-major blocks, block i at
// i * mb * mb, leading dimension = the block's rows)
__global__ void __launch_bounds__(256) cs_dinv_k(const double* __restrict__ dinv, const double* __restrict__ bp,
                                                 double* __restrict__ cv, int n, int mb) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const int i = r / mb;
  const int r0 = i * mb;
  const int m = min(mb, n - r0);
  const double* a = dinv + (size_t)i * mb * mb + (size_t)(r - r0) * m;
  const double* v = bp + r0;
  double s = 0.0;
  for (int c = lane; c < m; c += 64) s += a[c] * v[c];
  s = cs_wave_sum(s);
  if (lane == 0) cv[r] = s;
}

// One chain step: cv[row0 + r] -= K[r, :] . v[0 .. q), r < q, K q x q row-major with leading
// dimension ld -- KL_i / KU_i (ld q, v the neighbour block's plane of cv), or, in the blocks of
// one plane, Dinv_i itself (ld q, v = E_i y_{i-1} / F_i x_{i+1} from cs_ell_mv_k); one wave per row.
__global__ void __launch_bounds__(256) cs_chain_k(const double* __restrict__ K, int ld, const double* v,
                                                  double* cv, int q, int row0) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= q) return;
  const double* a = K + (size_t)r * ld;
  double s = 0.0;
#pragma unroll 4
  for (int k = lane; k < q; k += 64) s += a[k] * v[k];
  s = cs_wave_sum(s);
  if (lane == 0) cv[row0 + r] -= s;
}

// t = E cv[src .. src + q) for one block's coupling E (ELL, q rows x ew): the vector the
// one-plane blocks' chain step multiplies by Dinv_i (their KL_i = Dinv_i E_i is not stored)
__global__ void __launch_bounds__(256) cs_ell_mv_k(const int* __restrict__ ec, const double* __restrict__ ev,
                                                   int ew, const double* __restrict__ src,
                                                   double* __restrict__ t, int q) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= q) return;
  double s = 0.0;
  for (int e = 0; e < ew; ++e) s += ev[(size_t)k * ew + e] * src[ec[(size_t)k * ew + e]];
  t[k] = s;
}

// The other rows of every coupled block i = iblk0 + blockIdx.y, after its chain:
//   LOWER (UPPER = false): t = E_i cv[last plane of block i-1],  cv[rows] -= Dinv_i[rows, 0:q] t
//   UPPER:                 t = F_i cv[first plane of block i+1], cv[rows] -= Dinv_i[rows, m-q:m] t
// rows: LOWER all but the block's last plane, UPPER all but its first.  t lives in LDS (q
// doubles), formed once per workgroup of 32 rows (8 per wave).
template <bool UPPER>
__global__ void __launch_bounds__(256) cs_couple_k(const double* __restrict__ dinv, const int* __restrict__ ecol,
                                                   const double* __restrict__ eval, int ew,
                                                   double* __restrict__ cv, int n, int mb, int q, int iblk0) {
  extern __shared__ double t[];
  const int i = iblk0 + (int)blockIdx.y;
  const int r0 = i * mb;
  const int m = min(mb, n - r0);
  const int nsel = m - q;
  if ((int)blockIdx.x * 32 >= nsel) return;  // whole workgroup: past the block's rows
  const int src = UPPER ? r0 + m : r0 - q;
  const int* ec = ecol + (size_t)i * q * ew;
  const double* ev = eval + (size_t)i * q * ew;
  for (int k = threadIdx.x; k < q; k += 256) {
    double s = 0.0;
    for (int e = 0; e < ew; ++e) s += ev[k * ew + e] * cv[src + ec[k * ew + e]];
    t[k] = s;
  }
  __syncthreads();
  const int base = UPPER ? q : 0;
  const int col0 = UPPER ? m - q : 0;
  const int lane = threadIdx.x & 63;
  for (int h = 0; h < 8; ++h) {
    const int rr = (int)blockIdx.x * 32 + (threadIdx.x >> 6) * 8 + h;
    if (rr >= nsel) break;
    const int lr = base + rr;
    const double* a = dinv + (size_t)i * mb * mb + (size_t)lr * m + col0;
    double s = 0.0;
#pragma unroll 4
    for (int k = lane; k < q; k += 64) s += a[k] * t[k];
    s = cs_wave_sum(s);
    if (lane == 0) cv[r0 + lr] -= s;
  }
}

// D[row][col] += val from ELL rows (distinct columns per row), D row-major with ld
__global__ void __launch_bounds__(256) cs_ell_add_k(const int* __restrict__ col, const double* __restrict__ val,
                                                    int w, int rows, double* __restrict__ D, int ld) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * w) return;
  const double v = val[t];
  if (v != 0.0) D[(size_t)(t / w) * ld + col[t]] += v;
}

struct CoarseBlocks {
  int n = 0, q = 0, mb = 0, nb = 0, ew = 0;
  double* dinv = nullptr;
  int* perm = nullptr;   // natural -> band index
  int* iperm = nullptr;  // band -> natural index
  int* ecol = nullptr;   // E_i ELL (q rows x ew per block; block 0 unused)
  double* eval = nullptr;
  int* fcol = nullptr;   // F_i ELL (block nb - 1 unused)
  double* fval = nullptr;
  double* kl = nullptr;  // chain matrices KL_i (q x q per block; block 0 unused); only for blocks
  double* ku = nullptr;  // of > 1 plane -- KU_i (block nb - 1 unused)
  double* bp = nullptr;
  double* cv = nullptr;
  double* tv = nullptr;  // one-plane blocks: the chain step's coupled vector (q)
  size_t device_bytes = 0;

  bool active() const { return dinv != nullptr; }

  void release() {
    for (void* p : {(void*)dinv, (void*)perm, (void*)iperm, (void*)ecol, (void*)eval, (void*)fcol,
                    (void*)fval, (void*)kl, (void*)ku, (void*)bp, (void*)cv, (void*)tv})
      if (p) (void)hipFree(p);
    dinv = nullptr;
    perm = iperm = ecol = fcol = nullptr;
    eval = fval = kl = ku = bp = cv = tv = nullptr;
    n = q = mb = nb = ew = 0;
    device_bytes = 0;
  }

  // unknowns per block (rows of a Dinv block): P planes of q, P = max(1, target / q)
  // (default target 2048): the chain has nb - 1 dependent q x q products per direction,
  // the batched product reads P q^2 * 8 B per plane
  static int planes_per_block(int q, int nplanes, int target) {
    return std::max(1, std::min(nplanes, target / q));
  }

  // blocks of > 1 plane keep KL / KU whatever with_chain says: they are much smaller than Dinv_i
  static bool keeps_chain(bool with_chain, int64_t mb, int64_t q) { return with_chain || mb > q; }

  // bytes this solver would hold on the device for a grid (before building it)
  static size_t estimate_bytes(int dim, const int64_t nn[3], int target, bool with_chain) {
    int64_t len[3] = {nn[0], nn[1], dim == 3 ? nn[2] : 1};
    const int64_t N = len[0] * len[1] * len[2];
    const int64_t no = std::max({len[0], len[1], len[2]});
    const int64_t q = N / no;
    const int64_t P = planes_per_block((int)q, (int)no, target);
    const int64_t mb = P * q, nb = (no + P - 1) / P;
    const int64_t last = N - (nb - 1) * mb;
    // Dinv blocks + 3 q^2 of setup workspace (+ 2 nb q^2 of chain matrices: with_chain, or blocks of
    // > 1 plane, which build() always gives them -- the same predicate)
    const int64_t chain = keeps_chain(with_chain, mb, q) ? 2 * nb : 0;
    return (size_t)(((nb - 1) * mb * mb + last * last) * 8 + (chain + 3) * q * q * 8 + N * 160);
  }
  // The chain's KL_i / KU_i (q x q each, formed at setup) make every chain step one GEMV launch.
  // Without them (build's with_chain false) a step is a sparse E_i y launch and a GEMV over
  // Dinv_i's q x q corner -- the same bytes, one more launch per step (130 x 130 x 10: 2.93 vs
  // 2.08 ms per solve), and 2 nb q^2 fewer bytes: blocks of one plane (q >= the block target)
  // need as much for KL / KU as for Dinv (206 instead of 69 GB at 512 x 512 x 8), so the solver
  // drops them when they would not fit (Solver::build_coarse_inverse).
  bool chain_matrices() const { return kl != nullptr; }

  using Emit = std::function<void(int64_t col, double val)>;
  using RowFn = std::function<void(int64_t p, const Emit&)>;

  // row(p, emit): entries A[p][col] += val of natural row p (any order, duplicates add)
  // returns false if a diagonal block is singular
  bool build(int dim, const int64_t nn[3], int target, bool with_chain, const RowFn& row, hipStream_t stream) {
    release();
    int64_t len[3] = {nn[0], nn[1], dim == 3 ? nn[2] : 1};
    const int64_t N = len[0] * len[1] * len[2];
    if (N > INT32_MAX / 2) throw std::runtime_error("coarsest grid too large for the direct solver");
    // axes by length: shortest innermost, longest outermost (ties: lower axis inner)
    int ax[3] = {0, 1, 2};
    std::stable_sort(ax, ax + 3, [&](int a, int b) { return len[a] < len[b]; });
    int64_t st[3];
    int64_t s = 1;
    for (int a = 0; a < 3; ++a) st[ax[a]] = s, s *= len[ax[a]];
    n = (int)N;
    const int64_t no = len[ax[2]];
    q = (int)(N / no);
    // (no bound on q itself: the memory estimate, checked against the device before build, is
    // the wall -- N q 8 B of Dinv blocks)
    const int P = planes_per_block(q, (int)no, target);
    mb = P * q;
    nb = (int)((no + P - 1) / P);
    std::vector<int> hperm(N), hiperm(N);
    for (int64_t k = 0; k < len[2]; ++k)
      for (int64_t j = 0; j < len[1]; ++j)
        for (int64_t i = 0; i < len[0]; ++i) {
          const int64_t p = i + len[0] * (j + len[1] * k);
          const int64_t r = i * st[0] + j * st[1] + k * st[2];
          hperm[p] = (int)r;
          hiperm[r] = (int)p;
        }
    // rows in band order: in-block entries (local column), the coupling toward block i-1
    // (E_i: first plane of i -> last plane of i-1) and toward block i+1 (F_i)
    std::vector<std::vector<std::pair<int, double>>> in(N), lo(N), up(N);
    auto add = [](std::vector<std::pair<int, double>>& v, int c, double x) {
      for (auto& e : v)
        if (e.first == c) { e.second += x; return; }
      v.emplace_back(c, x);
    };
    for (int64_t r = 0; r < N; ++r) {
      const int64_t r0 = (r / mb) * mb;
      const int64_t r1 = std::min<int64_t>(r0 + mb, N);
      row(hiperm[r], [&](int64_t col, double val) {
        const int64_t c = hperm[col];
        if (c >= r0 && c < r1)
          add(in[r], (int)(c - r0), val);
        else if (c < r0 && c >= r0 - q && r < r0 + q)
          add(lo[r], (int)(c - (r0 - q)), val);
        else if (c >= r1 && c < r1 + q && r >= r1 - q)
          add(up[r], (int)(c - r1), val);
        else
          throw std::runtime_error("coarsest operator couples beyond neighbouring planes");
      });
    }
    int wi = 1;
    ew = 1;
    for (int64_t r = 0; r < N; ++r) {
      wi = std::max(wi, (int)in[r].size());
      ew = std::max(ew, (int)std::max(lo[r].size(), up[r].size()));
    }
    std::vector<int> icol((size_t)N * wi, 0);
    std::vector<double> ival((size_t)N * wi, 0.0);
    for (int64_t r = 0; r < N; ++r)
      for (size_t e = 0; e < in[r].size(); ++e) {
        icol[r * wi + e] = in[r][e].first;
        ival[r * wi + e] = in[r][e].second;
      }
    std::vector<int> hec((size_t)nb * q * ew, 0), hfc((size_t)nb * q * ew, 0);
    std::vector<double> hev((size_t)nb * q * ew, 0.0), hfv((size_t)nb * q * ew, 0.0);
    for (int i = 0; i < nb; ++i) {
      const int64_t r0 = (int64_t)i * mb;
      const int64_t r1 = std::min<int64_t>(r0 + mb, N);
      for (int k = 0; k < q; ++k) {
        const size_t o = ((size_t)i * q + k) * ew;
        const auto& l = lo[r0 + k];
        for (size_t e = 0; e < l.size(); ++e) hec[o + e] = l[e].first, hev[o + e] = l[e].second;
        const auto& u = up[r1 - q + k];
        for (size_t e = 0; e < u.size(); ++e) hfc[o + e] = u[e].first, hfv[o + e] = u[e].second;
      }
    }
    in.clear(); lo.clear(); up.clear();

    // device arrays
    const int64_t last = N - (int64_t)(nb - 1) * mb;
    const size_t dinv_elems = (size_t)(nb - 1) * mb * mb + (size_t)last * last;
    auto dmalloc = [&](void** ptr, size_t bytes) {
      if (big_alloc(ptr, bytes) != hipSuccess)
        throw std::runtime_error("direct solver: device allocation of " + std::to_string(bytes) + " B failed");
      device_bytes += bytes;
    };
    dmalloc((void**)&dinv, sizeof(double) * dinv_elems);
    dmalloc((void**)&perm, sizeof(int) * N);
    dmalloc((void**)&iperm, sizeof(int) * N);
    const size_t ne = (size_t)nb * q * ew;
    dmalloc((void**)&ecol, sizeof(int) * ne);
    dmalloc((void**)&eval, sizeof(double) * ne);
    dmalloc((void**)&fcol, sizeof(int) * ne);
    dmalloc((void**)&fval, sizeof(double) * ne);
    if (keeps_chain(with_chain, mb, q)) {  // blocks of > 1 plane: KL / KU are much smaller than Dinv_i
      dmalloc((void**)&kl, sizeof(double) * nb * q * q);
      dmalloc((void**)&ku, sizeof(double) * nb * q * q);
    }
    dmalloc((void**)&bp, sizeof(double) * N);
    dmalloc((void**)&cv, sizeof(double) * N);
    dmalloc((void**)&tv, sizeof(double) * q);
    auto h2d = [&](void* d, const void* h, size_t bytes) {
      if (hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream) != hipSuccess)
        throw std::runtime_error("direct solver: upload failed");
    };
    h2d(perm, hperm.data(), sizeof(int) * N);
    h2d(iperm, hiperm.data(), sizeof(int) * N);
    h2d(ecol, hec.data(), sizeof(int) * ne);
    h2d(eval, hev.data(), sizeof(double) * ne);
    h2d(fcol, hfc.data(), sizeof(int) * ne);
    h2d(fval, hfv.data(), sizeof(double) * ne);
    // setup workspace: in-block ELL, dense E_i / F_{i-1} / E_i W, pivots, info
    int* dicol = nullptr;
    double* dival = nullptr;
    double *dE = nullptr, *dF = nullptr, *dT = nullptr;
    int* ipiv = nullptr;
    int* info = nullptr;
    auto wmalloc = [&](void** ptr, size_t bytes) {
      if (hipMalloc(ptr, bytes) != hipSuccess)
        throw std::runtime_error("direct solver: device allocation of " + std::to_string(bytes) + " B failed");
    };
    rocblas_handle h = nullptr;
    auto cleanup = [&]() {
      for (void* p : {(void*)dicol, (void*)dival, (void*)dE, (void*)dF, (void*)dT, (void*)ipiv, (void*)info})
        if (p) (void)hipFree(p);
      if (h) rocblas_destroy_handle(h);
    };
    try {
      wmalloc((void**)&dicol, sizeof(int) * N * wi);
      wmalloc((void**)&dival, sizeof(double) * N * wi);
      wmalloc((void**)&dE, sizeof(double) * q * q);
      wmalloc((void**)&dF, sizeof(double) * q * q);
      wmalloc((void**)&dT, sizeof(double) * q * q);
      wmalloc((void**)&ipiv, sizeof(int) * mb);
      wmalloc((void**)&info, sizeof(int) * 2 * nb);
      h2d(dicol, icol.data(), sizeof(int) * N * wi);
      h2d(dival, ival.data(), sizeof(double) * N * wi);
      if (hipMemsetAsync(info, 0, sizeof(int) * 2 * nb, stream) != hipSuccess)
        throw std::runtime_error("direct solver: memset failed");
      if (rocblas_create_handle(&h) != rocblas_status_success)
        throw std::runtime_error("rocblas_create_handle failed");
      rocblas_set_stream(h, stream);
      // row-major C(m x n) = alpha A(m x k) B(k x n) + beta C: column-major C^T = B^T A^T
      auto rm_gemm = [&](int m, int nn_, int k, double alpha, const double* A, int lda, const double* B,
                         int ldb, double beta, double* C, int ldc) {
        if (rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, nn_, m, k, &alpha, B, ldb, A, lda,
                          &beta, C, ldc) != rocblas_status_success)
          throw std::runtime_error("rocblas_dgemm failed");
      };
      auto ell_dense = [&](const int* c, const double* v, int w, int rows, double* D, int ld, size_t zero) {
        if (zero && hipMemsetAsync(D, 0, sizeof(double) * zero, stream) != hipSuccess)
          throw std::runtime_error("direct solver: memset failed");
        const int th = rows * w;
        hipLaunchKernelGGL(cs_ell_add_k, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, stream, c, v, w, rows,
                           D, ld);
      };
      for (int i = 0; i < nb; ++i) {
        const int64_t r0 = (int64_t)i * mb;
        const int m = (int)std::min<int64_t>(mb, N - r0);
        double* Di = dinv + (size_t)i * mb * mb;
        ell_dense(dicol + r0 * wi, dival + r0 * wi, wi, m, Di, m, (size_t)m * m);
        if (i > 0) {
          // D_i[first, first] -= E_i Dinv_{i-1}[last, last] F_{i-1}
          const double* Dp = dinv + (size_t)(i - 1) * mb * mb;
          ell_dense(ecol + (size_t)i * q * ew, eval + (size_t)i * q * ew, ew, q, dE, q, (size_t)q * q);
          ell_dense(fcol + (size_t)(i - 1) * q * ew, fval + (size_t)(i - 1) * q * ew, ew, q, dF, q,
                    (size_t)q * q);
          rm_gemm(q, q, q, 1.0, dE, q, Dp + (size_t)(mb - q) * mb + (mb - q), mb, 0.0, dT, q);
          rm_gemm(q, q, q, -1.0, dT, q, dF, q, 1.0, Di, m);
        }
        // rocSOLVER reads the row-major D_i as column-major D_i^T; inv(D_i^T) column-major
        // is inv(D_i) row-major
        if (rocsolver_dgetrf(h, m, m, Di, m, ipiv, info + 2 * i) != rocblas_status_success ||
            rocsolver_dgetri(h, m, Di, m, ipiv, info + 2 * i + 1) != rocblas_status_success)
          throw std::runtime_error("rocsolver getrf/getri failed");
        // chain matrices: KL_i = Dinv_i[last, first] E_i, KU_i = Dinv_i[first, last] F_i
        if (!chain_matrices()) continue;
        if (i > 0)  // dE still holds E_i (the Schur update above)
          rm_gemm(q, q, q, 1.0, Di + (size_t)(m - q) * m, m, dE, q, 0.0, kl + (size_t)i * q * q, q);
        if (i < nb - 1) {
          ell_dense(fcol + (size_t)i * q * ew, fval + (size_t)i * q * ew, ew, q, dF, q, (size_t)q * q);
          rm_gemm(q, q, q, 1.0, Di + (m - q), m, dF, q, 0.0, ku + (size_t)i * q * q, q);
        }
      }
      if (hipGetLastError() != hipSuccess) throw std::runtime_error("direct solver: launch failed");
      std::vector<int> hinfo(2 * nb);
      if (hipMemcpyAsync(hinfo.data(), info, sizeof(int) * 2 * nb, hipMemcpyDeviceToHost, stream) !=
              hipSuccess ||
          hipStreamSynchronize(stream) != hipSuccess)
        throw std::runtime_error("direct solver: setup failed on the device");
      cleanup();
      for (int v : hinfo)
        if (v != 0) return false;
      return true;
    } catch (...) {
      (void)hipStreamSynchronize(stream);
      cleanup();
      release();
      throw;
    }
  }

  // x = A^-1 b on the stream (kernel launches only: graph-capturable)
  template <typename T>
  void solve(const T* b, T* x, hipStream_t stream) const {
    const dim3 b256(256);
    const unsigned g1 = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL((cs_gather_k<T>), dim3(g1), b256, 0, stream, b, iperm, bp, n);
    hipLaunchKernelGGL(cs_dinv_k, dim3((unsigned)((n + 3) / 4)), b256, 0, stream, dinv, bp, cv, n, mb);
    const size_t lds = sizeof(double) * q;
    const unsigned gc = (unsigned)((q + 3) / 4);
    const unsigned gr = (unsigned)((mb - q + 31) / 32);
    const bool km = chain_matrices();  // else one plane per block (mb == q)
    const unsigned ge = (unsigned)((q + 255) / 256);
    for (int i = 1; i < nb; ++i) {  // y_i[last] = c_i[last] - KL_i y_{i-1}[last]
      const int r0 = i * mb, m = std::min(mb, n - r0);
      if (km) {
        hipLaunchKernelGGL(cs_chain_k, dim3(gc), b256, 0, stream, kl + (size_t)i * q * q, q, cv + (r0 - q), cv,
                           q, r0 + m - q);
      } else {  // one plane per block: KL_i y = Dinv_i (E_i y)
        hipLaunchKernelGGL(cs_ell_mv_k, dim3(ge), b256, 0, stream, ecol + (size_t)i * q * ew,
                           eval + (size_t)i * q * ew, ew, cv + (r0 - q), tv, q);
        hipLaunchKernelGGL(cs_chain_k, dim3(gc), b256, 0, stream, dinv + (size_t)i * mb * mb, q, tv, cv, q, r0);
      }
    }
    if (mb > q && nb > 1)
      hipLaunchKernelGGL((cs_couple_k<false>), dim3(gr, (unsigned)(nb - 1)), b256, lds, stream, dinv, ecol, eval,
                         ew, cv, n, mb, q, 1);
    for (int i = nb - 2; i >= 0; --i) {  // x_i[first] = y_i[first] - KU_i x_{i+1}[first]
      if (km) {
        hipLaunchKernelGGL(cs_chain_k, dim3(gc), b256, 0, stream, ku + (size_t)i * q * q, q, cv + (i + 1) * mb,
                           cv, q, i * mb);
      } else {  // KU_i x = Dinv_i (F_i x)
        hipLaunchKernelGGL(cs_ell_mv_k, dim3(ge), b256, 0, stream, fcol + (size_t)i * q * ew,
                           fval + (size_t)i * q * ew, ew, cv + (i + 1) * mb, tv, q);
        hipLaunchKernelGGL(cs_chain_k, dim3(gc), b256, 0, stream, dinv + (size_t)i * mb * mb, q, tv, cv, q, i * mb);
      }
    }
    if (mb > q && nb > 1)
      hipLaunchKernelGGL((cs_couple_k<true>), dim3(gr, (unsigned)(nb - 1)), b256, lds, stream, dinv, fcol, fval,
                         ew, cv, n, mb, q, 0);
    hipLaunchKernelGGL((cs_scatter_k<T>), dim3(g1), b256, 0, stream, cv, perm, x, n);
  }
};

}  // namespace mad
