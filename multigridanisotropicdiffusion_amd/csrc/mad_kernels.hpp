// mad_kernels.hpp -- HIP kernels for the V-cycle hot path (gfx950 / CDNA4).
//
// Operator: the reference assembles a 27-coefficient DCA stencil per voxel
// (include/mad/itkGridsHierarchy.hxx:298-516).  Here it is evaluated
// matrix-free from per-level coefficient fields (SoA, storage type T):
//
//   a_d   = dt M_dd / h_d^2                 (ISO: one field a, a_d = a * rat[d])
//   g_d   = dt/(2h_d) sum_d2 delta_d2 M_d,d2 / (2h_d2)   (one-sided at the border)
//   e_dd2 = dt M_dd2 / (2 h_d h_d2)         (FULL only)
//   (A u)(p) = D u(p) - S(p),   D = 1 + 2 sum a_d
//   S(p) = sum_d (a_d+g_d) u~(p+e_d) + (a_d-g_d) u~(p-e_d)
//        + sum_{d<d2} e_dd2 (u~(++) - u~(+-) - u~(-+) + u~(--))
//   u~ mirrored about the boundary node: u~(-1) = u(1), u~(n) = u(n-2)
//
// which equals the DCA stencil row by row (tests/test_oracle.py checks it to
// 1e-13).  Coefficient field order: [a.. | g.. | e..] (see CoefLayout).
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <type_traits>
#include <cstdint>

namespace mad {

enum { KISO = 1, KDIAG = 2, KFULL = 3 };

template <int DIM, int KIND>
struct CoefLayout {
  static constexpr int NA = (KIND == KISO) ? 1 : DIM;
  static constexpr int NG = DIM;
  static constexpr int NE = (KIND == KFULL) ? DIM * (DIM - 1) / 2 : 0;
  static constexpr int N = NA + NG + NE;
};

inline int coef_count(int dim, int kind) {
  int na = (kind == KISO) ? 1 : dim;
  int ne = (kind == KFULL) ? dim * (dim - 1) / 2 : 0;
  return na + dim + ne;
}

// Geometry of one level slab as seen by a kernel.  Arrays are x-fastest; the
// base pointer addresses local plane 0; in 3D GHOST ghost planes are allocated on
// each side (rank halos; at a global boundary the mirror is used instead).
// Coefficient fields are stored point-interleaved (AoS): the NCF coefficients of a
// point are contiguous, so one point is one 16/24/36-byte record (fp32) read with
// wide loads, and a run of points of one colour is one contiguous byte range
// (a tile halo then costs at most a line at each end of a run, not one per field).
// Points are ordered x-parity split within every row: the even-x points first,
// then the odd-x points (cidx below), so each colour class of a row is one run.
// 3D levels keep GHOST coefficient planes below and above the slab (neighbour data
// on rank slabs, padding for masked border lanes otherwise).
constexpr int GHOST = 4;

struct Geo {
  int nx, ny, nz;       // local sizes
  int zoff;             // global z index of local plane 0 (colour parity)
  int zlo_ghost;        // 1: planes -GHOST..-1 hold the lower neighbour's data
  int zhi_ghost;        // 1: planes nz..nz+GHOST-1 hold the upper neighbour's data
  int hx0;              // (nx + 1) / 2: start of the odd-x half of a coefficient row
  int64_t sy, sz;       // strides
  int64_t N;            // nx*ny*nz (owned points)
  int rs;               // coefficient record stride (ncoef, or ncoef + 1 when the record
                        // also carries the rhs b: level 0, see LevelData::brec)
};

// coefficient record index of point (i, j, k): element cidx * NCF + field
__device__ __forceinline__ int64_t cidx(const Geo& g, int i, int j, int k) {
  return (int64_t)k * g.sz + (int64_t)j * g.sy + ((i & 1) ? g.hx0 + (i >> 1) : (i >> 1));
}

template <typename T>
struct Rat {
  T r[3];  // ISO spacing ratios h_x^2 / h_d^2
};

// ---------------------------------------------------------------------------
// the per-point stencil: D and S of (A u)(p) = D u(p) - S(p)
template <typename T>
struct Coefs {
  T ax, ay, az, gx, gy, gz, exy, exz, eyz;
};

template <typename T, int DIM, int KIND>
__device__ __forceinline__ void coefs_from_raw(const T* raw, const Rat<T>& rat, Coefs<T>& q);

template <typename T, int DIM, int KIND>
__device__ __forceinline__ void load_coefs(const T* __restrict__ cf, int64_t c, int rs,
                                           const Rat<T>& rat, Coefs<T>& q) {
  constexpr int NCF = CoefLayout<DIM, KIND>::N;
  const T* rec = cf + c * rs;
  T raw[NCF];
#pragma unroll
  for (int a = 0; a < NCF; ++a) raw[a] = rec[a];
  coefs_from_raw<T, DIM, KIND>(raw, rat, q);
}

// Neighbour values in a fixed order, mirror-resolved by the caller:
//  0 xp  1 xm  2 yp  3 ym  4 zp  5 zm
//  6 xp,yp  7 xp,ym  8 xm,yp  9 xm,ym   10 xp,zp 11 xp,zm 12 xm,zp 13 xm,zm
// 14 yp,zp 15 yp,zm 16 ym,zp 17 ym,zm
// Every smoother / residual kernel evaluates the operator through this one
// function, so the fused and the per-colour GS kernels are bit-identical.
template <typename T, int DIM, int KIND>
__device__ __forceinline__ void stencil_combine(const Coefs<T>& q, const T* nb, T& D, T& S) {
  // explicit fma chain with contraction off: every kernel (per-colour, fused,
  // Jacobi, residual) rounds this expression identically whatever the context
#pragma clang fp contract(off)
  T s = (q.ax + q.gx) * nb[0];
  s = fma(q.ax - q.gx, nb[1], s);
  s = fma(q.ay + q.gy, nb[2], s);
  s = fma(q.ay - q.gy, nb[3], s);
  T d = T(2) * (q.ax + q.ay);
  if (DIM == 3) {
    s = fma(q.az + q.gz, nb[4], s);
    s = fma(q.az - q.gz, nb[5], s);
    d = fma(T(2), q.az, d);
  }
  if (KIND == KFULL) {
    s = fma(q.exy, (nb[6] - nb[7]) - (nb[8] - nb[9]), s);
    if (DIM == 3) {
      s = fma(q.exz, (nb[10] - nb[11]) - (nb[12] - nb[13]), s);
      s = fma(q.eyz, (nb[14] - nb[15]) - (nb[16] - nb[17]), s);
    }
  }
  D = T(1) + d;
  S = s;
}

// r = b - (D u - S), rounded the same way in every residual kernel
template <typename T>
__device__ __forceinline__ T resid_value(T b, T D, T u, T S) {
#pragma clang fp contract(off)
  const T Du = D * u;
  return b - (Du - S);
}

// n / D for the smoothers: fp32 hardware reciprocal plus one fma correction of the
// quotient (within 1 ulp of the IEEE quotient, 5 VALU instead of ~11); fp64 IEEE
template <typename T>
__device__ __forceinline__ T div_fast(T n, T D) {
#pragma clang fp contract(off)
  if constexpr (sizeof(T) == 4) {
    const float r = __builtin_amdgcn_rcpf(D);
    const float q = n * r;
    const float e = __builtin_fmaf(-q, D, n);
    return __builtin_fmaf(e, r, q);
  } else {
    return n / D;
  }
}

// Gauss-Seidel point update u = (b + S) / D, shared by every GS kernel so they round
// alike.  fp32: hardware reciprocal and one fma correction of the quotient (5 VALU
// instead of the ~11 of the IEEE division sequence; within 1 ulp of the correctly
// rounded quotient for the operator's D >= 1); fp64: IEEE division.
template <typename T>
__device__ __forceinline__ T gs_update(T b, T S, T D) {
#pragma clang fp contract(off)
  const T n = b + S;
  if constexpr (sizeof(T) == 4) {
    const float r = __builtin_amdgcn_rcpf(D);
    const float q = n * r;
    const float e = __builtin_fmaf(-q, D, n);
    return __builtin_fmaf(e, r, q);
  } else {
    return n / D;
  }
}

template <int DIM, int KIND>
struct NbCount {
  static constexpr int N = (KIND == KFULL) ? (DIM == 3 ? 18 : 10) : (DIM == 3 ? 6 : 4);
};

// gather the neighbour values of global-memory point p (i, j, k local)
template <typename T, int DIM, int KIND>
__device__ __forceinline__ void gather_nb(const T* __restrict__ u, const Geo& g, int i, int j,
                                          int k, int64_t p, T* nb) {
  const int64_t dxm = (i == 0) ? 1 : -1;
  const int64_t dxp = (i == g.nx - 1) ? -1 : 1;
  const int64_t dym = (j == 0) ? g.sy : -g.sy;
  const int64_t dyp = (j == g.ny - 1) ? -g.sy : g.sy;
  nb[0] = u[p + dxp];
  nb[1] = u[p + dxm];
  nb[2] = u[p + dyp];
  nb[3] = u[p + dym];
  int64_t dzm = 0, dzp = 0;
  if (DIM == 3) {
    dzm = (k == 0 && !g.zlo_ghost) ? g.sz : -g.sz;
    dzp = (k == g.nz - 1 && !g.zhi_ghost) ? -g.sz : g.sz;
    nb[4] = u[p + dzp];
    nb[5] = u[p + dzm];
  }
  if (KIND == KFULL) {
    nb[6] = u[p + dxp + dyp];
    nb[7] = u[p + dxp + dym];
    nb[8] = u[p + dxm + dyp];
    nb[9] = u[p + dxm + dym];
    if (DIM == 3) {
      nb[10] = u[p + dxp + dzp];
      nb[11] = u[p + dxp + dzm];
      nb[12] = u[p + dxm + dzp];
      nb[13] = u[p + dxm + dzm];
      nb[14] = u[p + dyp + dzp];
      nb[15] = u[p + dyp + dzm];
      nb[16] = u[p + dym + dzp];
      nb[17] = u[p + dym + dzm];
    }
  }
}

template <typename T, int DIM, int KIND>
__device__ __forceinline__ void stencil_terms(const T* __restrict__ u, const T* __restrict__ cf,
                                              const Geo& g, const Rat<T>& rat, int i, int j,
                                              int k, int64_t p, T& D, T& S) {
  Coefs<T> q;
  load_coefs<T, DIM, KIND>(cf, cidx(g, i, j, k), g.rs, rat, q);
  T nb[18];
  gather_nb<T, DIM, KIND>(u, g, i, j, k, p, nb);
  stencil_combine<T, DIM, KIND>(q, nb, D, S);
}

// ---------------------------------------------------------------------------
// multicolour Gauss-Seidel, one colour per launch, in place.
//   ncolors 2: red-black, colour = (i+j+k) & 1        (5/7-point operators)
//   ncolors 4: 3D colour = ((i+k)&1) | ((j+k)&1)<<1   (19-point; corners inactive)
//              2D colour = (i&1) | (j&1)<<1           (9-point)
// Same-colour points are never neighbours, so a colour pass is order-free.
// Thread (x, y, z) -> i' (half row), row index, plane.
// kofs: first local plane of the launch (negative: ghost planes of a rank slab, computed
// redundantly so that one deep halo exchange serves a whole sweep)
template <typename T, int DIM, int KIND>
__global__ void __launch_bounds__(256) gs_color_k(T* __restrict__ u, const T* __restrict__ b,
                                                  const T* __restrict__ cf, Geo g, Rat<T> rat,
                                                  int color, int ncolors, int kofs = 0) {
  const int k = (DIM == 3) ? (int)blockIdx.z + kofs : 0;
  const int kg = k + g.zoff;
  const int jq = blockIdx.y * blockDim.y + threadIdx.y;
  const int iq = blockIdx.x * blockDim.x + threadIdx.x;
  int i, j;
  if (ncolors == 4) {
    if (DIM == 3) {
      j = 2 * jq + (((color >> 1) ^ kg) & 1);
      i = 2 * iq + (((color & 1) ^ kg) & 1);
    } else {
      j = 2 * jq + (color >> 1);
      i = 2 * iq + (color & 1);
    }
  } else {
    j = jq;
    i = 2 * iq + ((color + j + kg) & 1);
  }
  if (i >= g.nx || j >= g.ny) return;
  const int64_t p = i + g.sy * j + g.sz * k;
  T D, S;
  stencil_terms<T, DIM, KIND>(u, cf, g, rat, i, j, k, p, D, S);
  u[p] = gs_update(b[p], S, D);
}

// exact lexicographic GS (reference order, itkMultigridGaussSeidelSmoother.hxx:67-106)
// as hyperplane wavefronts t = i + 2j + 3k (3D) / i + 2j (2D): every lex-earlier
// neighbour lies on an earlier hyperplane, every later one on a later hyperplane.
template <typename T, int DIM, int KIND>
__global__ void __launch_bounds__(256) gs_lex_plane_k(T* __restrict__ u, const T* __restrict__ b,
                                                      const T* __restrict__ cf, Geo g, Rat<T> rat,
                                                      int t) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = (DIM == 3) ? (int)blockIdx.y : 0;
  if (j >= g.ny) return;
  const int i = t - 2 * j - 3 * k;
  if (i < 0 || i >= g.nx) return;
  const int64_t p = i + g.sy * j + g.sz * k;
  T D, S;
  stencil_terms<T, DIM, KIND>(u, cf, g, rat, i, j, k, p, D, S);
  u[p] = gs_update(b[p], S, D);
}

// ---------------------------------------------------------------------------
// Fused multicolour GS sweep (3D): the whole sweep in ONE launch, out of place
// (uin -> uout), bit-identical to NC in-place gs_color_k passes.
//
// Wavefront: at z-step k, stage c updates colour c on plane k-c.  Colour c needs
// colours < c already updated on planes k-c-1..k-c+1 (done in earlier stages of
// this and the previous steps) and colours > c still old (their stages run later),
// so the stage order reproduces the colour-by-colour sweep exactly.
// Tiles: each workgroup owns a TX x TY column of one z-chunk; stage c also
// updates an (NC-1-c)-wide halo redundantly so no workgroup ever needs another
// one's updated values (overlapped tiling); only the tile interior is stored.
// LDS: ring of NC+2 planes of u over the tile + NC halo, rows stored x-parity
// split (even x, then odd x) so every colour stage reads contiguous runs.
// Registers: the next step's u plane and each stage's coefficients / rhs are
// prefetched one step ahead, so HBM latency hides behind the current step.
// z-chunks start NC-1 planes early and run NC-1 planes late (redundant), and read
// up to NC planes beyond the chunk: on a rank slab those are the GHOST planes.
template <typename T, int DIM, int KIND>
__device__ __forceinline__ void coefs_from_raw(const T* raw, const Rat<T>& rat, Coefs<T>& q) {
  using L = CoefLayout<DIM, KIND>;
  if (KIND == KISO) {
    const T a = raw[0];
    q.ax = a;
    q.ay = a * rat.r[1];
    q.az = (DIM == 3) ? a * rat.r[2] : T(0);
  } else {
    q.ax = raw[0];
    q.ay = raw[1];
    q.az = (DIM == 3) ? raw[2] : T(0);
  }
  q.gx = raw[L::NA];
  q.gy = raw[L::NA + 1];
  q.gz = (DIM == 3) ? raw[L::NA + 2] : T(0);
  if (KIND == KFULL) {
    q.exy = raw[L::NA + L::NG];
    q.exz = (DIM == 3) ? raw[L::NA + L::NG + 1] : T(0);
    q.eyz = (DIM == 3) ? raw[L::NA + L::NG + 2] : T(0);
  } else {
    q.exy = q.exz = q.eyz = T(0);
  }
}

// raw buffer access (gfx9 descriptor, no range limit): uniform base in SGPRs,
// 32-bit per-lane byte offset + uniform byte offset -> no VALU address arithmetic
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, -1, 0x00020000);
}
template <typename T, int AUX = 0>
__device__ __forceinline__ T buf_load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, AUX));
  } else {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, AUX);
    return __builtin_bit_cast(T, v);
  }
}
template <typename T, int AUX = 0>
__device__ __forceinline__ void buf_store(T v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  if constexpr (sizeof(T) == 4) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)voff, 0, AUX);
  } else {
    using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, v), r, (int)voff, 0, AUX);
  }
}

// one coefficient record (NCF values of T) at byte offset voff: dword x3 chunks when
// the record is a multiple of 12 bytes, else x4 chunks + remainder (default cache policy:
// the nt policy measured 1.04-1.9x slower on these streams, profiles/r01_policy_ab.log)

template <typename T, int NCF>
__device__ __forceinline__ void buf_load_rec(__amdgpu_buffer_rsrc_t r, uint32_t voff, T* out) {
  constexpr int NB = NCF * (int)sizeof(T);
  constexpr int NW = NB / 4;
  uint32_t w[NW];
  // chunk offsets go in soffset (inline constants), so no VALU add per chunk
  if constexpr (NB % 12 == 0 && NB % 16 != 0) {
#pragma unroll
    for (int q = 0; q < NW / 3; ++q) {
      auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)voff, 12 * q, 0);
      w[3 * q] = v[0]; w[3 * q + 1] = v[1]; w[3 * q + 2] = v[2];
    }
  } else {
    int q = 0;
#pragma unroll
    for (; q + 4 <= NW; q += 4) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 4 * q, 0);
      w[q] = v[0]; w[q + 1] = v[1]; w[q + 2] = v[2]; w[q + 3] = v[3];
    }
    if constexpr (NW % 4 == 3) {
      auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)voff, 4 * (NW - 3), 0);
      w[NW - 3] = v[0]; w[NW - 2] = v[1]; w[NW - 1] = v[2];
    } else if constexpr (NW % 4 == 2) {
      auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, 4 * (NW - 2), 0);
      w[NW - 2] = v[0]; w[NW - 1] = v[1];
    } else if constexpr (NW % 4 == 1) {
      w[NW - 1] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, 4 * (NW - 1), 0);
    }
  }
  __builtin_memcpy(out, w, NB);
}

template <int NC, int TX, int TY>
struct FusedGeom {
  static constexpr int H = NC;
  static constexpr int RX = TX + 2 * H;
  static constexpr int RY = TY + 2 * H;
  // LDS row: even-x half, then odd-x half starting HALF floats later; HALF is
  // padded to 16 (mod 32) so lanes alternating halves hit disjoint banks.
  static constexpr int HALF = ((RX / 2 + 15) / 32) * 32 + 16;
  static constexpr int PITCH = 2 * HALF + 1;
  static constexpr int PLANE = RY * PITCH;
  static constexpr int NP = NC + 2;
  static constexpr int rows(int c) { return (NC == 4) ? (TY + 2 * (NC - 1 - c)) / 2 : TY + 2 * (NC - 1 - c); }
  static constexpr int cols(int c) { return (TX + 2 * (NC - 1 - c)) / 2; }
};

// ---------------------------------------------------------------------------
// Fused multicolour GS sweep, v3: the wavefront / overlapped-tile schedule above and the
// same arithmetic as the per-colour passes (bit-identical results), with a per-step
// instruction stream almost free of address arithmetic:
//  * the x/y mirror boundary lives in the LDS tile: ghost positions at distance 1
//    outside the domain hold mirror copies (loaded mirrored, and rewritten when
//    their source point is updated), so every neighbour read is a ds_read with a
//    compile-time offset;
//  * the z loop is unrolled by two with the plane parity normalised, so every
//    stage point's parity, LDS offset and global offset are compile-time plus one
//    per-thread constant;
//  * global loads use a uniform (SGPR) base + 32-bit per-thread byte offset; points
//    outside the domain load from the padded allocation and are masked at the store.
// Needs: coefficient fields with >= 1 padding plane below and above every field
// (LevelData::cf, GHOST planes) and x/b arrays with their GHOST planes; nx, ny >= 3.
// LDS: dynamic, NP * PLANE * sizeof(T) bytes.
//
// Rank slabs (flip_last, sig): the LAST z-chunk of the launch marches downward -- the
// kernel runs it on a z-reflected view of the slab (negative plane stride, ghost
// sides swapped, +z / -z neighbour planes swapped back at the stencil, colour parity
// from the physical plane), which gives bit-identical results because a multicolour
// sweep does not depend on the order within a colour.  So the slab's first and last
// GHOST planes are both final a few steps into the launch; the workgroups of the two
// edge chunks then count themselves in sig[0] (bottom) / sig[1] (top), and the
// communication stream, waiting on those counters, exchanges the halo while the rest
// of the sweep runs -- one launch per sweep instead of boundary + interior launches.

//
// Peer halo (PEER, MAD_OPT_PEER_HALO): the edge chunks also store their first GHOST output
// planes into the neighbour's mailbox (po.dst[0] bottom edge -> rank - 1, po.dst[1] top edge ->
// rank + 1, addressed with the chunk's own plane stride, so the reflected top chunk fills the
// mailbox downward) and, once a tile's GHOST planes are out, count the tile in the neighbour's
// counter (po.sig[0] / po.sig[1]) with a system-scope release; the neighbour's stream waits on
// that counter and copies the mailbox into its ghost planes (Solver::peer_resolve).

// where a PEER sweep's edge planes go (null: no neighbour on that side)
template <typename T>
struct PeerOut {
  T* dst[2];
  uint32_t* sig[2];
};

//
// BL (dense b, not BREC): b is staged through LDS like u -- one coalesced load of the tile region's
// plane per step into a ring of NC planes (the stages read plane k - c at step k), the stages then
// read their point's b from LDS at the u offset -- instead of one load per stage point of its colour,
// which on the x-parity-interleaved dense b is a stride-2 access (two cache lines per wave load for
// one line's worth of values).  The LDS then holds NP + NC planes (fp32 64 x 32 tiles: 155 KB).
//
// BS (b split, round 6): dense b's values in the records' x-parity-split order (LevelData::bs, cidx), so a
// stage's b values are one contiguous run per row like its records -- one stride-1 load per stage point,
// no LDS ring (BL's 62 KB) and no stride-2 access; the copy is refreshed when b changes (sync_bsplit).
//
// ZU (zero iterate): the sweep's input u is known to be zero (the first sweep of a correction cycle
// whose x was zeroed, or never written, by the step before): its planes enter the LDS ring as
// zeros instead of being loaded -- the same arithmetic on the same values, without the read, and
// without the zero fill the caller would otherwise write first.
template <typename T, int KIND, int TX, int TY, int NT, int MINW, int LEAD = 2, bool BREC = false,
          bool PEER = false, bool BL = false, bool ZU = false, bool BS = false>
__global__ void __launch_bounds__(NT, MINW) gs_fused3_k(const T* __restrict__ uin, T* __restrict__ uout,
                                                        const T* __restrict__ b, const T* __restrict__ cf,
                                                        Geo g, Rat<T> rat, int zc, int ntx, int nty,
                                                        int zbase, int zstride, int flip_last,
                                                        uint32_t* __restrict__ sig, PeerOut<T> po) {
  constexpr int NC = (KIND == KFULL) ? 4 : 2;
  using FG = FusedGeom<NC, TX, TY>;
  constexpr int H = FG::H, RX = FG::RX, RY = FG::RY, HALF = FG::HALF, PITCH = FG::PITCH;
  constexpr int PLANE = FG::PLANE, NP = FG::NP;
  constexpr int UPT = (RX * RY + NT - 1) / NT;
  constexpr int OPT = (TX * TY + NT - 1) / NT;
  constexpr int NCF = CoefLayout<3, KIND>::N;
  constexpr int RS = NCF + (BREC ? 1 : 0);  // record stride; BREC: b is the record's last value
  constexpr uint32_t TS = sizeof(T);
  static_assert(TX % 2 == 0 && TY % 2 == 0 && (H % 2) == 0, "even tile geometry");
  static_assert(FG::rows(0) * FG::cols(0) <= NT, "one stage point per thread");
  static_assert(!(BL && BREC), "b rides in the record");
  static_assert(!(BS && (BL || BREC)), "one form of b");
  constexpr int NB = BL ? NC : 0;  // b ring slots (after the NP u slots)
  extern __shared__ __align__(16) unsigned char fused_smem[];

  int bid = blockIdx.x;
  {
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7, xcd = bid & 7, idx = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int tiles = ntx * nty;
  const int chunk = bid / tiles;
  const int tile = bid - chunk * tiles;
  const int tyi = tile / ntx;
  const int txi = tile - tyi * ntx;
  const int rx0 = txi * TX - H;
  const int ry0 = tyi * TY - H;
  const int tid = threadIdx.x;
  // first thread of this wave (wave-uniform): a stage has fewer points than threads
  // (665..512 of 1024 for the 64x32 tile), so whole waves sit a stage out -- they skip
  // its loads and arithmetic instead of computing masked-off lanes, which leaves the
  // SIMDs' issue slots to the waves that have points
  const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
  auto wave_in = [&](int c) { return wbase < FG::rows(c) * FG::cols(c); };
  const int nx = g.nx, ny = g.ny;
  const int sy = (int)g.sy, hx0 = g.hx0;
  // tile whose region keeps >= 2 points from every x/y face: no masks, no ghost images
  const bool interior = rx0 >= 2 && rx0 + RX <= nx - 2 && ry0 >= 2 && ry0 + RY <= ny - 2;

  // chunk q of this launch covers owned planes [zbase + q*zstride, +zc): one launch
  // may cover a slab's two boundary chunks only, or its interior (rank-slab overlap)
  const int p0 = zbase + chunk * zstride;
  const int p1 = min(p0 + zc, g.nz);
  // z-reflected view for a downward-marching last chunk: logical plane l = physical
  // nz-1-l (all plane addressing below goes through sz, zlo_g / zhi_g, zpar)
  const bool flip = flip_last != 0 && chunk == (int)(gridDim.x / tiles) - 1;
  int64_t sz = g.sz;
  int zlo_g = g.zlo_ghost, zhi_g = g.zhi_ghost, zpar = g.zoff;
  int z0 = p0, z1 = p1;
  if (flip) {
    const int64_t top = (int64_t)(g.nz - 1) * g.sz;
    uin += top;
    uout += top;
    b += top;
    cf += top * RS;
    sz = -g.sz;
    zlo_g = g.zhi_ghost;
    zhi_g = g.zlo_ghost;
    zpar = g.zoff + g.nz - 1;  // global parity of logical l = (l + zpar) & 1
    z0 = g.nz - p1;
    z1 = g.nz - p0;
  }
  const int zlo = zlo_g ? -GHOST : 0;
  const int zhi = zhi_g ? g.nz + GHOST : g.nz;
  const int ulo = zlo_g ? -(GHOST - 1) : 0;
  const int uhi = zhi_g ? g.nz + GHOST - 1 : g.nz;
  // an edge chunk of a rank slab signals once its first GHOST planes are final
  T* const pdst = PEER ? po.dst[flip ? 1 : 0] : nullptr;
  uint32_t* const psig = PEER ? po.sig[flip ? 1 : 0] : (sig ? sig + (flip ? 1 : 0) : nullptr);
  const bool signals = (PEER ? pdst != nullptr : sig != nullptr) && z0 == 0 && zlo_g;
  // first step with its plane parity normalised to even (global z), last step
  const int kbeg = (z0 - (NC - 1)) - ((z0 - (NC - 1) + zpar) & 1);
  const int kend = z1 + NC - 2;

  auto mirror = [](int v, int n) { return v < 0 ? min(-v, n - 1) : (v >= n ? max(2 * (n - 1) - v, 0) : v); };

  // Plane-load (source byte offset in a plane, LDS byte offset in a ring slot) and
  // output (LDS, global) offsets of this thread's elements, computed once: recomputing
  // them every step cost ~60 VALU per wave and step (integer division by RX, mirror),
  // a quarter of the issue-bound sweep's vector instructions.  -1 marks no element.
  uint32_t usrc[UPT];
  int udst[UPT];
#pragma unroll
  for (int e = 0; e < UPT; ++e) {
    const int q = tid + e * NT;
    const int lj = q / RX, li = q - (q / RX) * RX;
    int gi = rx0 + li, gj = ry0 + lj;
    if (!interior) {
      gi = mirror(gi, nx);
      gj = mirror(gj, ny);
    }
    usrc[e] = (uint32_t)(gj * sy + gi) * TS;
    udst[e] = (q < RX * RY) ? (int)((lj * PITCH + (li & 1) * HALF + (li >> 1)) * TS) : -1;
  }
  int olds[OPT], oglb[OPT];
#pragma unroll
  for (int e = 0; e < OPT; ++e) {
    const int q = tid + e * NT;
    const int lj = H + q / TX, li = H + (q - (q / TX) * TX);
    const int gi = rx0 + li, gj = ry0 + lj;
    const bool ok = q < TX * TY && gi < nx && gj < ny;
    olds[e] = (int)((lj * PITCH + (li & 1) * HALF + (li >> 1)) * TS);
    oglb[e] = ok ? (int)((gj * sy + gi) * TS) : -1;
  }

  // ---- stage points.  Stage c covers rows/cols of its colour in the region shrunk
  // by H - (NC-1-c) = c+1 on each side.  For plane parity PM:
  //   NC=4: li = c+1 + (1^PM) + 2t,  lj = c+1 + yb(c,PM) + 2r
  //   NC=2: lj = c+1 + r,            li = c+1 + ((c^PM^r)&1) + 2t
  // Per-thread byte offsets: LDS (within a plane slot), coefficient record (from
  // the tile's record base ry0*sy + rx0/2), rhs (from ry0*sy + rx0).
  // NC=4 keeps only the PM=0 offsets: PM=1 moves every point by a uniform delta
  // (pdelta below), so it is folded into the uniform bases.
  constexpr int NPM = (NC == 4) ? 1 : 2;
  uint32_t pl[NC][NPM], pg[NC][NPM], pb[NC][NPM];
  uint32_t vmask = 0, gmask = 0;  // bit (c*2+PM): valid point; 4 ghost-image bits each
  uint32_t omask = 0;              // bit (c*2+PM): li odd (per thread only for NC=2)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cols = FG::cols(c);
    const bool has = tid < FG::rows(c) * cols;
    const int r = has ? tid / cols : 0;
    const int t = has ? tid - (tid / cols) * cols : 0;
    const int l0 = c + 1;
#pragma unroll
    for (int PM = 0; PM < 2; ++PM) {
      int li, lj;
      if (NC == 4) {
        li = l0 + (1 ^ PM) + 2 * t;
        lj = l0 + (((c >> 1) ^ PM ^ l0) & 1) + 2 * r;
      } else {
        lj = l0 + r;
        li = l0 + ((c ^ PM ^ r) & 1) + 2 * t;
      }
      const int gi = rx0 + li, gj = ry0 + lj;
      const bool ok = has && gi >= 0 && gi < nx && gj >= 0 && gj < ny;
      vmask |= (ok ? 1u : 0u) << (c * 2 + PM);
      const uint32_t gb = (ok && gi == 1 ? 1u : 0u) | (ok && gi == nx - 2 ? 2u : 0u) |
                          (ok && gj == 1 ? 4u : 0u) | (ok && gj == ny - 2 ? 8u : 0u);
      gmask |= gb << (4 * (c * 2 + PM));
      omask |= (uint32_t)(li & 1) << (c * 2 + PM);
      if (PM < NPM) {
        pl[c][PM] = (uint32_t)(lj * PITCH + (li & 1) * HALF + (li >> 1)) * TS;
        pg[c][PM] = (uint32_t)(lj * sy + (li & 1) * hx0 + (li >> 1)) * (TS * RS);
        pb[c][PM] = (uint32_t)(lj * sy + li) * TS;
      }
    }
  }
  // NC=4, PM=1 vs PM=0: li -> li-1, lj -> lj + 1 - 2*yb0 (yb0 = ((c>>1) ^ (c+1)) & 1)
  // deltas: .l LDS elements (compile-time), .g coefficient records, .b rhs elements
  struct PD {
    int l;
    int64_t g, b;
  };
  auto pdelta = [&](int c, int PM) -> PD {
    if (NC != 4 || PM == 0) return PD{0, 0, 0};
    const int dy = 1 - 2 * (((c >> 1) ^ (c + 1)) & 1);
    const bool odd0 = (c & 1) != 0;  // li parity at PM=0: (c+2) & 1
    return PD{dy * PITCH + (odd0 ? -HALF : HALF - 1), (int64_t)dy * sy + (odd0 ? -hx0 : hx0 - 1),
              (int64_t)dy * sy - 1};
  };
  const int64_t cbase = (int64_t)ry0 * sy + (rx0 >> 1);  // rx0 is even
  const int64_t bbase = (int64_t)ry0 * sy + rx0;

  auto slot = [](int m) { return (m + NP * 64) % NP; };
  auto plane_ok = [&](int m) { return m >= zlo && m < zhi; };
  auto stage_on = [&](int c, int m) {
    const int h = NC - 1 - c;
    return m >= z0 - h && m < z1 + h && m >= ulo && m < uhi;
  };
  unsigned char* lbytes = fused_smem;

  T up[UPT];
  T bp[BL ? UPT : 1];
  T raw[NC][RS];
  T bv[NC];
  auto bslot = [](int m) { return NP + (m + NB * 64) % (NB > 0 ? NB : 1); };
  auto load_bplane = [&](int m) {
    if constexpr (BL) {
      m = min(max(m, zlo), zhi - 1);
      const __amdgpu_buffer_rsrc_t rs = buf_rsrc(b + (int64_t)m * sz);
#pragma unroll
      for (int e = 0; e < UPT; ++e) bp[e] = buf_load<T>(rs, usrc[e], 0u);
    }
  };
  auto put_bplane = [&](int m) {
    if constexpr (BL) {
      unsigned char* P = lbytes + bslot(m) * (PLANE * TS);
#pragma unroll
      for (int e = 0; e < UPT; ++e) {
        if (e < UPT - 1 || udst[e] >= 0) *reinterpret_cast<T*>(P + udst[e]) = bp[e];
      }
    }
  };
  auto load_plane = [&](int m) {
    if constexpr (ZU) {
#pragma unroll
      for (int e = 0; e < UPT; ++e) up[e] = T(0);
    } else {
      m = min(max(m, zlo), zhi - 1);
      const __amdgpu_buffer_rsrc_t rs = buf_rsrc(uin + (int64_t)m * sz);
#pragma unroll
      for (int e = 0; e < UPT; ++e) up[e] = buf_load<T>(rs, usrc[e], 0u);
    }
  };
  auto put_plane = [&](int m) {
    unsigned char* P = lbytes + slot(m) * (PLANE * TS);
#pragma unroll
    for (int e = 0; e < UPT; ++e) {
      if (e < UPT - 1 || udst[e] >= 0) *reinterpret_cast<T*>(P + udst[e]) = up[e];
    }
  };
  // stage c data of step k (plane m = k - c, parity PM)
  // unconditional (the plane index clamped into the loadable range): a conditional
  // load makes the compiler copy every prefetch register at the join
  auto load_stage = [&](int c, int k, int PM) {
    const int m = min(max(k - c, zlo), zhi - 1);
    {
      const PD d = pdelta(c, PM);
      buf_load_rec<T, RS>(buf_rsrc(cf + ((int64_t)m * sz + cbase + d.g) * RS), pg[c][PM % NPM],
                          raw[c]);
      if constexpr (BS)  // the split copy: the record's index, stride 1 (pg / RS)
        bv[c] = buf_load<T>(buf_rsrc(b + (int64_t)m * sz + cbase + d.g), pg[c][PM % NPM] / (uint32_t)RS, 0u);
      else if constexpr (!BREC && !BL)
        bv[c] = buf_load<T>(buf_rsrc(b + (int64_t)m * sz + bbase + d.b), pb[c][PM % NPM], 0u);
    }
  };
  auto stage = [&](int c, int k, int PM) {
    const int m = k - c;
    if (!stage_on(c, m) || !wave_in(c)) return;
    const int zm = (m == 0 && !zlo_g) ? 1 : m - 1;
    const int zp = (m == g.nz - 1 && !zhi_g) ? g.nz - 2 : m + 1;
    const uint32_t o = pl[c][PM % NPM] + (uint32_t)(pdelta(c, PM).l * (int)TS);
    unsigned char* A0 = lbytes + slot(m) * (PLANE * TS) + o;
    // physical -z / +z neighbour planes (swapped in the reflected view)
    const unsigned char* Am = lbytes + slot(flip ? zp : zm) * (PLANE * TS) + o;
    const unsigned char* Ap = lbytes + slot(flip ? zm : zp) * (PLANE * TS) + o;
    // li parity: NC=4 compile-time ((c+1+(1^PM)) & 1); NC=2 per thread (row parity)
    bool odd;
    if (NC == 4) {
      odd = ((c + 1 + (1 ^ PM)) & 1) != 0;
    } else {
      odd = ((omask >> (c * 2 + PM)) & 1u) != 0;
    }
    const int ox_p = odd ? 1 - HALF : HALF;
    const int ox_m = odd ? -HALF : HALF - 1;
    auto rd = [](const unsigned char* p, int off) { return *reinterpret_cast<const T*>(p + off * (int)TS); };
    T nb[18];
    nb[0] = rd(A0, ox_p);
    nb[1] = rd(A0, ox_m);
    nb[2] = rd(A0, PITCH);
    nb[3] = rd(A0, -PITCH);
    nb[4] = rd(Ap, 0);
    nb[5] = rd(Am, 0);
    if (KIND == KFULL) {
      nb[6] = rd(A0, ox_p + PITCH);
      nb[7] = rd(A0, ox_p - PITCH);
      nb[8] = rd(A0, ox_m + PITCH);
      nb[9] = rd(A0, ox_m - PITCH);
      nb[10] = rd(Ap, ox_p);
      nb[11] = rd(Am, ox_p);
      nb[12] = rd(Ap, ox_m);
      nb[13] = rd(Am, ox_m);
      nb[14] = rd(Ap, PITCH);
      nb[15] = rd(Am, PITCH);
      nb[16] = rd(Ap, -PITCH);
      nb[17] = rd(Am, -PITCH);
    }
    Coefs<T> q;
    coefs_from_raw<T, 3, KIND>(raw[c], rat, q);
    T D, S;
    stencil_combine<T, 3, KIND>(q, nb, D, S);
    T bval;
    if constexpr (BREC)
      bval = raw[c][NCF];
    else if constexpr (BL)
      bval = *reinterpret_cast<const T*>(lbytes + bslot(m) * (PLANE * TS) + o);
    else
      bval = bv[c];
    const T v = gs_update(bval, S, D);
    const int bit = c * 2 + PM;
    if (interior) {
      if (NC == 2 || FG::rows(c) * FG::cols(c) < NT) {
        if ((vmask >> bit) & 1u) *reinterpret_cast<T*>(A0) = v;
      } else {
        *reinterpret_cast<T*>(A0) = v;
      }
    } else if ((vmask >> bit) & 1u) {
      *reinterpret_cast<T*>(A0) = v;
      const uint32_t gb = (gmask >> (4 * bit)) & 15u;
      if (gb) {
        // mirror images u~(-1) = u(1), u~(n) = u(n-2): same row parity, +-1 in the half
        // row (x) and +-2 rows (y); corners need both
        const int xs[3] = {0, (gb & 1u) ? -1 : 0, (gb & 2u) ? 1 : 0};
        const int ys[3] = {0, (gb & 4u) ? -2 * PITCH : 0, (gb & 8u) ? 2 * PITCH : 0};
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int bq = 0; bq < 3; ++bq) {
            if ((a == 0 && bq == 0) || (a > 0 && xs[a] == 0) || (bq > 0 && ys[bq] == 0)) continue;
            *reinterpret_cast<T*>(A0 + (xs[a] + ys[bq]) * (int)TS) = v;
          }
      }
    }
  };

  // prologue: planes kbeg-1, kbeg into LDS; plane kbeg+1 and step kbeg's stage data
  for (int m = kbeg - 1; m <= kbeg; ++m)
    if (plane_ok(m)) {
      load_plane(m);
      put_plane(m);
    }
  load_plane(kbeg + 1);
  load_bplane(kbeg);
#pragma unroll
  for (int c = 0; c < LEAD; ++c) load_stage(c, kbeg, c & 1);

  for (int k0 = kbeg; k0 <= kend; k0 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = k0 + u;
      if (k <= kend) {
        // keep the per-thread masks in VGPRs: without this the compiler hoists every
        // (stage, parity, flag) test out of the loop as a 64-bit lane mask and spills
        asm volatile("" : "+v"(vmask), "+v"(gmask), "+v"(omask));
        if (plane_ok(k + 1)) put_plane(k + 1);
        load_plane(k + 2);
        put_bplane(k);  // b of plane k: stage c reads plane k - c at step k (ring of NC)
        load_bplane(k + 1);
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          stage(c, k, (u ^ c) & 1);
          // prefetch LEAD stages ahead: (k, c) + LEAD -> (k + dk, c2); raw[c2] was
          // last read at (k + dk - 1, c2), before this point
          {
            constexpr int L = LEAD < NC ? LEAD : NC;
            const int c2 = (c + L) % NC, dk = (c + L) / NC;
            load_stage(c2, k + dk, (u ^ dk ^ c2) & 1);
          }
          __syncthreads();
        }
        const int mo = k - NC + 1;
        if (mo >= z0 && mo < z1) {
          const unsigned char* P = lbytes + slot(mo) * (PLANE * TS);
          const __amdgpu_buffer_rsrc_t ro = buf_rsrc(uout + (int64_t)mo * sz);
#pragma unroll
          for (int e = 0; e < OPT; ++e)
            if (oglb[e] >= 0)
              buf_store<T>(*reinterpret_cast<const T*>(P + olds[e]), ro, (uint32_t)oglb[e]);
          if constexpr (PEER) {
            if (signals && mo < GHOST) {  // an edge plane: also into the neighbour's mailbox
              const __amdgpu_buffer_rsrc_t rp = buf_rsrc(pdst + (int64_t)mo * sz);
#pragma unroll
              for (int e = 0; e < OPT; ++e)
                if (oglb[e] >= 0)
                  buf_store<T>(*reinterpret_cast<const T*>(P + olds[e]), rp, (uint32_t)oglb[e]);
            }
          }
          if (signals && mo == GHOST - 1) {
            // the edge planes 0..GHOST-1 of this tile are stored: release them, count in
            if (PEER) {
              // the mailbox and the counters are uncached memory (no L2 on either GPU holds them):
              // once every thread's mailbox stores have completed (vmcnt 0) the tile is counted
              // in.  A system-scope release fence here would write back the whole L2 (full of
              // this sweep's dirty output) once per tile: 0.30 vs 0.20 ms per 64-plane rank sweep
              __builtin_amdgcn_s_waitcnt(0);
              __syncthreads();
              if (tid == 0) __hip_atomic_fetch_add(psig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
              __threadfence();
              __syncthreads();
              if (tid == 0) __hip_atomic_fetch_add(psig, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
        }
      }
    }
  }
}

// Peer halo self-test at setup (Solver::peer_selftest): every edge fills the WHOLE neighbour
// mailbox it will write (GHOST planes, ghost_n elements) with a pattern of the sending rank,
// through the sweep's own store path -- buffer stores with an SGPR base and per-lane offsets,
// s_waitcnt 0 before a barrier, then one relaxed system-scope counter increment per workgroup
// (peer_ping_k) -- and every receiver waits for all its neighbours' workgroups (bounded) and
// checks every element of both mailboxes (peer_pong_k); a missing count or a single wrong value
// makes every rank fall back to the exchange for that level.  blockIdx.y = side.
__device__ __forceinline__ uint32_t peer_pattern(int rank, int64_t e) {
  return (uint32_t)(rank + 1) * 1021u + (uint32_t)(e % 4093);  // < 2^24: exact in fp32 too
}
template <typename T>
__global__ void __launch_bounds__(256) peer_ping_k(PeerOut<T> po, int64_t ghost_n, int64_t top_off, int rank) {
  const int side = blockIdx.y;
  T* d = po.dst[side];
  if (!d) return;
  T* base = d - (side ? top_off : 0);  // the top edge's pointer is at its mailbox's last plane
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t e0 = (int64_t)blockIdx.x * 256; e0 < ghost_n; e0 += stride) {
    const int64_t e = e0 + threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(base + e0);
    if (e < ghost_n) buf_store<T>((T)peer_pattern(rank, e), r, threadIdx.x * (uint32_t)sizeof(T));
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(po.sig[side], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// okw (plain device memory, 1 before the launch) is cleared on any failure; the counters are
// reset by the host afterwards (nothing writes them again before the collective that follows)
template <typename T>
__global__ void __launch_bounds__(256) peer_pong_k(const T* mlo, const T* mhi, const uint32_t* clo,
                                                   const uint32_t* chi, int rlo, int rhi, int64_t ghost_n,
                                                   uint32_t expect, uint32_t* okw, uint64_t tmo) {
  __shared__ int arrived;
  const int side = blockIdx.y;
  const T* m = side ? mhi : mlo;
  const uint32_t* cnt = side ? chi : clo;
  const int sender = side ? rhi : rlo;
  if (!m) return;
  if (threadIdx.x == 0) {
    int ok = 1;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < expect) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > tmo) {
        ok = 0;
        break;
      }
    }
    arrived = ok;
  }
  __syncthreads();
  bool bad = !arrived;
  if (arrived) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < ghost_n; e += stride)
      bad |= m[e] != (T)peer_pattern(sender, e);
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) atomicAnd(okw, 0u);
}

// Peer halo, consumer side: wait for the neighbours' edge planes, copy the two mailboxes into
// the ghost planes.  blockIdx.y = side (0: from rank - 1 into the lower ghost planes, 1: from
// rank + 1 into the upper ones; a null destination = no neighbour there).  ctl is this rank's
// control block: counters [buffer * 2 + side] the neighbours' sweeps count their tiles into
// (ci = buffer * 2), a ticket, an error word.  Thread 0 of every block polls its side's counter
// until all `tiles` edge tiles are in (system-scope acquire of uncached memory, so the stores of
// the other GPU are visible), giving up after `tmo` wall-clock ticks with the error word set (a
// peer that died must not hang this GPU); the last block to finish resets the counters, which no
// neighbour touches again before this rank's next sweep has signalled it (Solver::peer_resolve).
// The error word is sticky: once a wait has timed out (here or in an earlier launch) the blocks
// neither wait nor copy and the counters are left as they are -- a late tile of the neighbour must
// not release a later batch early -- and the host raises it (Solver::peer_check, called by every
// entry point that returns results: mad_run, the norms, downloads, mad_synchronize).
// The mailboxes are uncached, so the copy reads what the neighbour stored; the ghost planes are
// then ordinary stream-ordered data for the kernels that follow.
#ifndef UNPACK_LOADS
#define UNPACK_LOADS 8
#endif
// grid-strided byte copy with UNPACK_LOADS loads in flight per thread before their stores (16-B
// words where both ends and the length allow, else 4-B): a copy from (or into) the uncached
// mailboxes is latency-bound with one load per iteration -- a 512^2 x 4-plane side per 64 blocks
// took 13.5 us per unpack with one, 8.2-8.7 with eight, 9.3 with sixteen (profiles/r05_unpack_ab.log)
template <typename W>
__device__ __forceinline__ void copy_words(W* __restrict__ d, const W* __restrict__ s, uint64_t n,
                                           uint64_t t0, uint64_t stride) {
  constexpr int NL = UNPACK_LOADS;
  uint64_t i = t0;
  for (; i + (NL - 1) * stride < n; i += NL * stride) {
    W v[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) v[q] = s[i + q * stride];
#pragma unroll
    for (int q = 0; q < NL; ++q) d[i + q * stride] = v[q];
  }
  for (; i < n; i += stride) d[i] = s[i];
}
__device__ __forceinline__ void copy_inflight(char* d, const char* s, uint64_t bytes, uint64_t t0,
                                              uint64_t stride) {
  if ((((uintptr_t)d | (uintptr_t)s | bytes) & 15) == 0)
    copy_words((uint4*)d, (const uint4*)s, bytes / 16, t0, stride);
  else
    copy_words((uint32_t*)d, (const uint32_t*)s, bytes / 4, t0, stride);
}

// Per-colour GS levels (rank slabs, MAD_OPT_PEER_HALO): after a sweep's last colour pass, the
// GHOST edge planes of x into the neighbours' mailboxes of this batch's buffer (blockIdx.y = side:
// 0 the bottom planes for rank - 1, 1 the top planes for rank + 1; po.dst[1] points at its
// mailbox's last plane, where the fused sweep's reflected top chunk starts, so the push steps back
// to the mailbox's first), then -- stores complete (vmcnt 0), barrier -- every workgroup counts
// itself in the neighbour's counter with a relaxed system-scope increment: the fused sweep's and
// peer_ping_k's completion pattern, resolved by the same peer_unpack_k (tiles = push blocks)
template <typename T>
__global__ void __launch_bounds__(256) peer_push_k(const T* __restrict__ x, int64_t top_off, PeerOut<T> po,
                                                   int64_t n, int64_t top_dst_off) {
  const int side = blockIdx.y;
  T* dt = po.dst[side];
  if (!dt) return;
  char* d = (char*)(dt - (side ? top_dst_off : 0));
  const char* s = (const char*)(x + (side ? top_off : 0));
  copy_inflight(d, s, (uint64_t)n * sizeof(T), (uint64_t)blockIdx.x * blockDim.x + threadIdx.x,
                (uint64_t)gridDim.x * blockDim.x);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(po.sig[side], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void __launch_bounds__(256) peer_unpack_k(char* __restrict__ dlo, const char* __restrict__ slo,
                                                     char* __restrict__ dhi, const char* __restrict__ shi,
                                                     uint64_t bytes, uint32_t* __restrict__ ctl, int ci,
                                                     uint32_t tiles, uint64_t tmo) {
  __shared__ int failed;
  const int side = blockIdx.y;
  char* d = side ? dhi : dlo;
  const char* src = side ? shi : slo;
  if (d) {
    if (threadIdx.x == 0) {
      int f = __hip_atomic_load(ctl + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
      uint32_t* cnt = ctl + ci + side;
      const uint64_t t0 = wall_clock64();
      while (!f && __hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < tiles) {
        __builtin_amdgcn_s_sleep(2);
        if (wall_clock64() - t0 > tmo) {
          __hip_atomic_store(ctl + 5, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          f = 1;
        }
      }
      failed = f;
    }
    __syncthreads();
    if (!failed) {
      const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
      const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
      copy_inflight(d, src, bytes, t0, stride);
    }
  }
  if (threadIdx.x == 0) {
    const uint32_t nb = gridDim.x * gridDim.y;
    if (__hip_atomic_fetch_add(ctl + 4, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
      if (__hip_atomic_load(ctl + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        if (dlo) __hip_atomic_store(ctl + ci, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (dhi) __hip_atomic_store(ctl + ci + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __hip_atomic_store(ctl + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// fp64 block reduction helper (wave64 shuffles, then LDS across waves)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

template <int NT>
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double red[NT / 64];
  const int tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
  v = wave_sum(v);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  double s = 0.0;
  if (tid == 0) {
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[w];
  }
  return s;  // valid in thread 0
}

// weighted Jacobi sweep (itkMultigridWeightedJacobiSmoother.hxx:67-98), out of place
template <typename T, int DIM, int KIND>
__global__ void __launch_bounds__(256) wj_k(const T* __restrict__ u, T* __restrict__ uo,
                                            const T* __restrict__ b, const T* __restrict__ cf,
                                            Geo g, Rat<T> rat, T omega) {
  const int k = (DIM == 3) ? (int)blockIdx.z : 0;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.nx || j >= g.ny) return;
  const int64_t p = i + g.sy * j + g.sz * k;
  T D, S;
  stencil_terms<T, DIM, KIND>(u, cf, g, rat, i, j, k, p, D, S);
  T v = (b[p] + S) * div_fast(omega, D);
  v += (T(1) - omega) * u[p];
  uo[p] = v;
}

// residual r = b - A u (itkMultigridGaussSeidelSmoother.hxx:148-176), with optional
// fp64 ||r||^2 block partials (L2Norm, MAD.hxx:496-515)
template <typename T, int DIM, int KIND>
__global__ void __launch_bounds__(256) residual_k(const T* __restrict__ u, const T* __restrict__ b,
                                                  T* __restrict__ r, const T* __restrict__ cf,
                                                  Geo g, Rat<T> rat, double* __restrict__ part) {
  const int k = (DIM == 3) ? (int)blockIdx.z : 0;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double sq = 0.0;
  if (i < g.nx && j < g.ny) {
    const int64_t p = i + g.sy * j + g.sz * k;
    T D, S;
    stencil_terms<T, DIM, KIND>(u, cf, g, rat, i, j, k, p, D, S);
    const T rv = resid_value(b[p], D, u[p], S);
    r[p] = rv;
    sq = (double)rv * (double)rv;
  }
  if (part) {
    const double s = block_sum<256>(sq);
    if (threadIdx.x == 0 && threadIdx.y == 0)
      part[blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)] = s;
  }
}

// residual r = b - A u, 3D, z-marching (the residual_k arithmetic, bit-identical):
// each workgroup owns a TX x TY column of one z-chunk, keeps a 4-slot LDS ring of u
// planes over the tile + 1 (mirror images of the domain faces stored in the ring, as
// in gs_fused3_k), reads each point's coefficient record with wide buffer loads one
// step ahead, and writes r (and optionally fp64 |r|^2 partials per workgroup).
// One barrier per plane.  Needs the GHOST x/b planes and coefficient padding planes
// of LevelData (masked lanes read inside them).  be / xe (MAD_FP32_REFINE's defect
// correction): also be = (TE) r and xe = 0 at every point, the fp32 hierarchy's next rhs and
// zero initial guess (convert_k + fill_k of r folded into this pass).  ue / uo (the defect
// correction's update folded in, one GPU): every loaded u is u + (T) ue -- the fp32 cycle's
// correction -- and the owned points' u + ue go to uo (a second buffer: neighbouring tiles still
// read u); xe is then written by a separate fill, since those tiles also read ue.
// TB: the storage type of b -- float where the refine rhs is an exactly-fp32 image (an 8/16-bit or fp32
// input in its first time step): read as T, the same values in half the bytes.  bse: be's values also in
// the records' x-parity-split order (the fused sweep's split copy of b, gs_fused3_k BS).
template <typename T, int KIND, int TX, int TY, bool BREC = false, typename TE = T, typename TB = T>
__global__ void __launch_bounds__(TX * TY) resid3_k(const T* __restrict__ u, const TB* __restrict__ b,
                                                    T* __restrict__ r, const T* __restrict__ cf,
                                                    Geo g, Rat<T> rat, int zc, int ntx,
                                                    double* __restrict__ part,
                                                    TE* __restrict__ be = nullptr,
                                                    TE* __restrict__ xe = nullptr,
                                                    const TE* __restrict__ ue = nullptr,
                                                    T* __restrict__ uo = nullptr,
                                                    TE* __restrict__ bse = nullptr) {
  constexpr int NT = TX * TY;
  constexpr int RX = TX + 2, RY = TY + 2, PL = RX * RY;
  constexpr int UPT = (PL + NT - 1) / NT;
  constexpr int NCF = CoefLayout<3, KIND>::N;
  constexpr int RS = NCF + (BREC ? 1 : 0);  // record stride; BREC: b is the record's last value
  constexpr uint32_t TS = sizeof(T);
  __shared__ T ring[4 * PL];
  const int tiles_per_plane = ntx * ((g.ny + TY - 1) / TY);
  const int chunk = blockIdx.x / tiles_per_plane;
  const int tile = blockIdx.x - chunk * tiles_per_plane;
  const int tyi = tile / ntx, txi = tile - (tile / ntx) * ntx;
  const int x0 = txi * TX, y0 = tyi * TY;  // x0 even
  const int tid = threadIdx.x;
  const int tx = tid % TX, ty = tid / TX;
  const int nx = g.nx, ny = g.ny, sy = (int)g.sy, hx0 = g.hx0;
  const int64_t sz = g.sz;
  const int z0 = chunk * zc, z1 = min(z0 + zc, g.nz);
  const int zlo = g.zlo_ghost ? -1 : 0, zhi = g.zhi_ghost ? g.nz + 1 : g.nz;
  auto mirror = [](int v, int n) { return v < 0 ? min(-v, n - 1) : (v >= n ? max(2 * (n - 1) - v, 0) : v); };
  // region element e of this thread: LDS index and mirrored in-plane source offset
  int u_dst[UPT];
  uint32_t u_src[UPT];
#pragma unroll
  for (int e = 0; e < UPT; ++e) {
    const int q = tid + e * NT;
    const int lj = q / RX, li = q - (q / RX) * RX;
    u_dst[e] = q < PL ? q : -1;
    u_src[e] = (uint32_t)(mirror(y0 - 1 + lj, ny) * sy + mirror(x0 - 1 + li, nx)) * TS;
  }
  const int i = x0 + tx, j = y0 + ty;
  const bool ok = i < nx && j < ny;
  const uint32_t rec_off = ok ? (uint32_t)(ty * sy + (tx & 1) * hx0 + (tx >> 1)) * (TS * RS) : 0u;
  const uint32_t pt_off = ok ? (uint32_t)(ty * sy + tx) * TS : 0u;
  const uint32_t pt_off_b = ok ? (uint32_t)(ty * sy + tx) * (uint32_t)sizeof(TB) : 0u;
  const int64_t rbase = (int64_t)y0 * sy + (x0 >> 1), pbase = (int64_t)y0 * sy + x0;
  const int il = (ty + 1) * RX + (tx + 1);
  constexpr int oyp = RX, oym = -RX;  // x/y mirror images live in the ring

  T up[UPT];
  T raw[RS];
  T bv = T(0);
  auto load_plane = [&](int m) {
    m = min(max(m, zlo), zhi - 1);
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(u + (int64_t)m * sz);
#pragma unroll
    for (int e = 0; e < UPT; ++e) up[e] = buf_load<T>(rs, u_src[e], 0u);
    if (ue) {  // u + (T) e, as the separate update pass rounds it
      const __amdgpu_buffer_rsrc_t re = buf_rsrc(ue + (int64_t)m * sz);
#pragma unroll
      for (int e = 0; e < UPT; ++e)
        up[e] = up[e] + (T)buf_load<TE>(re, (u_src[e] / TS) * (uint32_t)sizeof(TE), 0u);
    }
  };
  auto put_plane = [&](int m) {
    T* P = ring + (m & 3) * PL;
#pragma unroll
    for (int e = 0; e < UPT; ++e)
      if (e < UPT - 1 || u_dst[e] >= 0) P[u_dst[e]] = up[e];
  };
  auto load_pt = [&](int m) {
    m = min(max(m, 0), g.nz - 1);
    buf_load_rec<T, RS>(buf_rsrc(cf + ((int64_t)m * sz + rbase) * RS), rec_off, raw);
    if constexpr (!BREC) bv = (T)buf_load<TB>(buf_rsrc(b + (int64_t)m * sz + pbase), pt_off_b, 0u);
  };

  // prologue: planes z0-1, z0 in the ring, z0+1 in registers, point data of z0
  if (z0 - 1 >= zlo) {
    load_plane(z0 - 1);
    put_plane(z0 - 1);
  }
  load_plane(z0);
  put_plane(z0);
  load_plane(z0 + 1);
  load_pt(z0);
  double sq = 0.0;
  for (int m = z0; m < z1; ++m) {
    if (m + 1 < zhi) put_plane(m + 1);
    load_plane(m + 2);
    __syncthreads();
    const int zm = (m == 0 && !g.zlo_ghost) ? m + 1 : m - 1;
    const int zp = (m == g.nz - 1 && !g.zhi_ghost) ? m - 1 : m + 1;
    const T* P0 = ring + (m & 3) * PL + il;
    const T* Pm = ring + (zm & 3) * PL + il;
    const T* Pp = ring + (zp & 3) * PL + il;
    T nb[18];
    nb[0] = P0[1];
    nb[1] = P0[-1];
    nb[2] = P0[oyp];
    nb[3] = P0[oym];
    nb[4] = Pp[0];
    nb[5] = Pm[0];
    if (KIND == KFULL) {
      nb[6] = P0[1 + oyp];
      nb[7] = P0[1 + oym];
      nb[8] = P0[-1 + oyp];
      nb[9] = P0[-1 + oym];
      nb[10] = Pp[1];
      nb[11] = Pm[1];
      nb[12] = Pp[-1];
      nb[13] = Pm[-1];
      nb[14] = Pp[oyp];
      nb[15] = Pm[oyp];
      nb[16] = Pp[oym];
      nb[17] = Pm[oym];
    }
    Coefs<T> q;
    coefs_from_raw<T, 3, KIND>(raw, rat, q);
    T D, S;
    stencil_combine<T, 3, KIND>(q, nb, D, S);
    const T rv = resid_value(BREC ? raw[NCF] : bv, D, P0[0], S);
    load_pt(m + 1);
    if (ok) {
      if (r) buf_store<T>(rv, buf_rsrc(r + (int64_t)m * sz + pbase), pt_off);  // null: norm only
      if (be) {
        const int64_t p = (int64_t)m * sz + pbase + ty * sy + tx;
        be[p] = (TE)rv;
        if (bse) bse[(int64_t)m * sz + rbase + rec_off / (TS * RS)] = (TE)rv;
        if (xe) xe[p] = TE(0);
        if (uo) uo[p] = P0[0];
      }
      sq += (double)rv * (double)rv;
    }
  }
  if (part) {
    const double s = block_sum<NT>(sq);
    if (tid == 0) part[blockIdx.x] = s;
  }
}

// wj3_k: one weighted-Jacobi sweep (itkMultigridWeightedJacobiSmoother.hxx:67-98),
// z-marching like resid3_k: u planes staged once in a 4-plane LDS ring with the x/y
// mirror images, the record of the next plane prefetched, uo written out of place.
// Same point update as wj_k: (b + S) * (omega / D) + (1 - omega) u.
template <typename T, int KIND, int TX, int TY, bool BREC = false>
__global__ void __launch_bounds__(TX * TY) wj3_k(const T* __restrict__ u, T* __restrict__ uo,
                                                 const T* __restrict__ b, const T* __restrict__ cf,
                                                 Geo g, Rat<T> rat, T omega, int zc, int ntx) {
  constexpr int NT = TX * TY;
  constexpr int RX = TX + 2, RY = TY + 2, PL = RX * RY;
  constexpr int UPT = (PL + NT - 1) / NT;
  constexpr int NCF = CoefLayout<3, KIND>::N;
  constexpr int RS = NCF + (BREC ? 1 : 0);
  constexpr uint32_t TS = sizeof(T);
  __shared__ T ring[4 * PL];
  const int tiles_per_plane = ntx * ((g.ny + TY - 1) / TY);
  const int chunk = blockIdx.x / tiles_per_plane;
  const int tile = blockIdx.x - chunk * tiles_per_plane;
  const int tyi = tile / ntx, txi = tile - (tile / ntx) * ntx;
  const int x0 = txi * TX, y0 = tyi * TY;
  const int tid = threadIdx.x;
  const int tx = tid % TX, ty = tid / TX;
  const int nx = g.nx, ny = g.ny, sy = (int)g.sy, hx0 = g.hx0;
  const int64_t sz = g.sz;
  const int z0 = chunk * zc, z1 = min(z0 + zc, g.nz);
  const int zlo = g.zlo_ghost ? -1 : 0, zhi = g.zhi_ghost ? g.nz + 1 : g.nz;
  auto mirror = [](int v, int n) { return v < 0 ? min(-v, n - 1) : (v >= n ? max(2 * (n - 1) - v, 0) : v); };
  int u_dst[UPT];
  uint32_t u_src[UPT];
#pragma unroll
  for (int e = 0; e < UPT; ++e) {
    const int q = tid + e * NT;
    const int lj = q / RX, li = q - (q / RX) * RX;
    u_dst[e] = q < PL ? q : -1;
    u_src[e] = (uint32_t)(mirror(y0 - 1 + lj, ny) * sy + mirror(x0 - 1 + li, nx)) * TS;
  }
  const int i = x0 + tx, j = y0 + ty;
  const bool ok = i < nx && j < ny;
  const uint32_t rec_off = ok ? (uint32_t)(ty * sy + (tx & 1) * hx0 + (tx >> 1)) * (TS * RS) : 0u;
  const uint32_t pt_off = ok ? (uint32_t)(ty * sy + tx) * TS : 0u;
  const int64_t rbase = (int64_t)y0 * sy + (x0 >> 1), pbase = (int64_t)y0 * sy + x0;
  const int il = (ty + 1) * RX + (tx + 1);
  constexpr int oyp = RX, oym = -RX;

  T up[UPT];
  T raw[RS];
  T bv = T(0);
  auto load_plane = [&](int m) {
    m = min(max(m, zlo), zhi - 1);
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(u + (int64_t)m * sz);
#pragma unroll
    for (int e = 0; e < UPT; ++e) up[e] = buf_load<T>(rs, u_src[e], 0u);
  };
  auto put_plane = [&](int m) {
    T* P = ring + (m & 3) * PL;
#pragma unroll
    for (int e = 0; e < UPT; ++e)
      if (e < UPT - 1 || u_dst[e] >= 0) P[u_dst[e]] = up[e];
  };
  auto load_pt = [&](int m) {
    m = min(max(m, 0), g.nz - 1);
    buf_load_rec<T, RS>(buf_rsrc(cf + ((int64_t)m * sz + rbase) * RS), rec_off, raw);
    if constexpr (!BREC) bv = buf_load<T>(buf_rsrc(b + (int64_t)m * sz + pbase), pt_off, 0u);
  };

  if (z0 - 1 >= zlo) {
    load_plane(z0 - 1);
    put_plane(z0 - 1);
  }
  load_plane(z0);
  put_plane(z0);
  load_plane(z0 + 1);
  load_pt(z0);
  for (int m = z0; m < z1; ++m) {
    if (m + 1 < zhi) put_plane(m + 1);
    load_plane(m + 2);
    __syncthreads();
    const int zm = (m == 0 && !g.zlo_ghost) ? m + 1 : m - 1;
    const int zp = (m == g.nz - 1 && !g.zhi_ghost) ? m - 1 : m + 1;
    const T* P0 = ring + (m & 3) * PL + il;
    const T* Pm = ring + (zm & 3) * PL + il;
    const T* Pp = ring + (zp & 3) * PL + il;
    T nb[18];
    nb[0] = P0[1];
    nb[1] = P0[-1];
    nb[2] = P0[oyp];
    nb[3] = P0[oym];
    nb[4] = Pp[0];
    nb[5] = Pm[0];
    if (KIND == KFULL) {
      nb[6] = P0[1 + oyp];
      nb[7] = P0[1 + oym];
      nb[8] = P0[-1 + oyp];
      nb[9] = P0[-1 + oym];
      nb[10] = Pp[1];
      nb[11] = Pm[1];
      nb[12] = Pp[-1];
      nb[13] = Pm[-1];
      nb[14] = Pp[oyp];
      nb[15] = Pm[oyp];
      nb[16] = Pp[oym];
      nb[17] = Pm[oym];
    }
    Coefs<T> q;
    coefs_from_raw<T, 3, KIND>(raw, rat, q);
    T D, S;
    stencil_combine<T, 3, KIND>(q, nb, D, S);
    T v = ((BREC ? raw[NCF] : bv) + S) * div_fast(omega, D);
    v += (T(1) - omega) * P0[0];
    load_pt(m + 1);
    if (ok) buf_store<T>(v, buf_rsrc(uo + (int64_t)m * sz + pbase), pt_off);
  }
}

// sum of squares of a contiguous array, grid-stride, fp64 partials per block
template <typename T>
__global__ void __launch_bounds__(256) sumsq_k(const T* __restrict__ x, int64_t n,
                                               double* __restrict__ part) {
  double s = 0.0;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const double v = (double)x[q];
    s += v * v;
  }
  s = block_sum<256>(s);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// deterministic final reduction of partials (one block)
__global__ void __launch_bounds__(256) reduce_final_k(const double* __restrict__ part, int64_t n,
                                                      double* __restrict__ out) {
  double s = 0.0;
  for (int64_t q = threadIdx.x; q < n; q += blockDim.x) s += part[q];
  s = block_sum<256>(s);
  if (threadIdx.x == 0) out[0] = s;
}

// ---------------------------------------------------------------------------
// inter-grid transfers (itkInterGridOperators.{h,hxx}), gather form, separable.
// coarse(I,J,K) = sum w_x w_y w_z fine(...)   (fine: g level geometry, may read ghosts)
// Taps are written tap by tap with selects (no per-branch array stores: with three
// branches each storing all four weights, the compiler merged the tap-3 weight
// wrongly -- observed on gfx950 with ROCm 7.2 -- and the clamped border rows lost
// their folded 1/8).
template <typename W>
__device__ __forceinline__ void rtaps4(int I, int nc, int cell, int* idx, W* w) {
  const bool endv = !cell && (I == 0 || I == nc - 1);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ic = min(max(2 * I - 1 + t, 0), 2 * nc - 1);      // cell: clamped 2I-1+t
    const int iv = endv ? 2 * I : (t == 3 ? 2 * I : 2 * I - 1 + t);  // vertex
    idx[t] = cell ? ic : iv;
    const W wc = (t == 0 || t == 3) ? W(0.125) : W(0.375);
    const W wv = endv ? (t == 0 ? W(1) : W(0)) : (t == 1 ? W(0.5) : (t == 3 ? W(0) : W(0.25)));
    w[t] = cell ? wc : wv;
  }
}

template <typename W>
__device__ __forceinline__ void itaps2(int f, int nc, int cell, int* idx, W* w) {
  const int I = f >> 1;
  const bool odd = (f & 1) != 0;
  idx[0] = I;
  idx[1] = cell ? (odd ? min(I + 1, nc - 1) : max(I - 1, 0)) : (odd ? I + 1 : I);
  w[0] = cell ? W(0.75) : (odd ? W(0.5) : W(1));
  w[1] = cell ? W(0.25) : (odd ? W(0.5) : W(0));
}

template <typename T, typename A, int DIM>
__global__ void __launch_bounds__(256) restrict_k(const T* __restrict__ fine, Geo gf,
                                                  T* __restrict__ coarse, Geo gc, int cx, int cy,
                                                  int cz, int fz_shift) {
#pragma clang fp contract(off)  // explicit fma: every transfer kernel rounds alike
  const int K = (DIM == 3) ? (int)blockIdx.z : 0;
  const int J = blockIdx.y * blockDim.y + threadIdx.y;
  const int I = blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= gc.nx || J >= gc.ny) return;
  int ix[4], iy[4], iz[4] = {0, 0, 0, 0};
  A wx[4], wy[4], wz[4] = {A(1), A(0), A(0), A(0)};
  rtaps4<A>(I, gc.nx, cx, ix, wx);
  rtaps4<A>(J, gc.ny, cy, iy, wy);
  if (DIM == 3) rtaps4<A>(K, gc.nz, cz, iz, wz);
  A v = A(0);
#pragma unroll
  for (int c = 0; c < (DIM == 3 ? 4 : 1); ++c) {
    const T* pl = fine + gf.sz * (int64_t)(iz[c] - fz_shift);
    A vz = A(0);
#pragma unroll
    for (int bq = 0; bq < 4; ++bq) {
      const T* row = pl + gf.sy * iy[bq];
      A vy = A(0);
#pragma unroll
      for (int a = 0; a < 4; ++a) vy = fma(wx[a], (A)row[ix[a]], vy);
      vz = fma(wy[bq], vy, vz);
    }
    v = fma(wz[c], vz, v);
  }
  coarse[I + gc.sy * J + gc.sz * K] = (T)v;
}

// fine(i,j,k) (+)= sum w coarse(...)
template <typename T, int DIM, int ADD>
__global__ void __launch_bounds__(256) interp_k(const T* __restrict__ coarse, Geo gc,
                                                T* __restrict__ fine, Geo gf, int cx, int cy,
                                                int cz) {
#pragma clang fp contract(off)  // explicit fma: every transfer kernel rounds alike
  const int k = (DIM == 3) ? (int)blockIdx.z : 0;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= gf.nx || j >= gf.ny) return;
  int ix[2], iy[2], iz[2] = {0, 0};
  T wx[2], wy[2], wz[2] = {T(1), T(0)};
  itaps2<T>(i, gc.nx, cx, ix, wx);
  itaps2<T>(j, gc.ny, cy, iy, wy);
  if (DIM == 3) itaps2<T>(k, gc.nz, cz, iz, wz);
  T v = T(0);
#pragma unroll
  for (int c = 0; c < (DIM == 3 ? 2 : 1); ++c) {
    const T* pl = coarse + gc.sz * (int64_t)iz[c];
    T vz = T(0);
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const T* row = pl + gc.sy * iy[bq];
      vz = fma(wy[bq], fma(wx[1], row[ix[1]], wx[0] * row[ix[0]]), vz);
    }
    v = fma(wz[c], vz, v);
  }
  const int64_t p = i + gf.sy * j + gf.sz * k;
  if (ADD) fine[p] += v;
  else fine[p] = v;
}

// 3D transfers on a z-slab: z taps are computed from GLOBAL plane indices (zoff) and
// the global coarse depth ncz; local plane -1 / nz are the ghost planes (filled by
// the halo exchange before the launch).  On one GPU zoff = 0 and the slab is the grid.
// Taps are held in registers with a fixed count per axis (4 for restriction, 2 for
// interpolation; unused taps weigh 0) and summed x, then y, then z with explicit fma,
// the same order as the 2D / generic kernels above.  Same inter-grid stencils of the
// reference (itkInterGridOperators.h:101-127; restriction taps IGO.h:115-127,
// interpolation scatter stencils IGO.h:101-113 as gathers):
//   cell-centred restriction = 1/8,3/8,3/8,1/8 on 2I-1..2I+2 with the fine index
//   clamped into the grid (which reproduces the one-sided border rows exactly);
//   vertex-centred = 1/4,1/2,1/4 about 2I, injection at both ends.
//   cell-centred interpolation = 3/4 c(I) + 1/4 c(I -+ 1), coarse index clamped;
//   vertex-centred = c(f/2) for even f, (c(f/2) + c(f/2+1)) / 2 for odd f.
// Both kernels march z: each workgroup owns a tile column, stages one plane at a
// time in LDS (coalesced loads, each fine / coarse value read once from HBM), and
// carries the z dimension in registers.
//
// restrict3_k: coarse tile CX x CY (one thread per coarse point), coarse planes
// [K0, K1).  Marches the fine planes the chunk needs in order: each fine plane is
// staged in LDS once (the next one already in registers), its x-y restricted value
// goes into a 4-entry register window, and a coarse plane is emitted once its last
// fine tap has been seen.
template <typename T, typename A, int CX, int CY>
__global__ void __launch_bounds__(CX * CY) restrict3_k(const T* __restrict__ fine, Geo gf,
                                                       T* __restrict__ coarse, Geo gc, int cx,
                                                       int cy, int cz, int fz_shift, int ncz,
                                                       int kc, int ntx) {
#pragma clang fp contract(off)  // explicit fma: every transfer kernel rounds alike
  constexpr int NT = CX * CY;
  constexpr int FX = 2 * CX + 2, FY = 2 * CY + 2, FP = FX * FY;
  constexpr int EPT = (FP + NT - 1) / NT;
  __shared__ T tile[FP];
  const int tiles = ntx * ((gc.ny + CY - 1) / CY);
  const int chunk = blockIdx.x / tiles;
  const int t = blockIdx.x - chunk * tiles;
  const int tyi = t / ntx, txi = t - (t / ntx) * ntx;
  const int I0 = txi * CX, J0 = tyi * CY;
  const int tid = threadIdx.x;
  const int I = I0 + tid % CX, J = J0 + tid / CX;
  const bool ok = I < gc.nx && J < gc.ny;
  const int fx0 = 2 * I0 - 1, fy0 = 2 * J0 - 1;  // tile origin in fine indices
  int ix[4], iy[4];
  A wx[4], wy[4];
  rtaps4<A>(min(I, gc.nx - 1), gc.nx, cx, ix, wx);
  rtaps4<A>(min(J, gc.ny - 1), gc.ny, cy, iy, wy);
  // this thread's tile elements: clamped in-plane source offsets
  int src_off[EPT];
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = min(tid + q * NT, FP - 1);
    const int ly = e / FX, lx = e - (e / FX) * FX;
    src_off[q] = min(max(fy0 + ly, 0), gf.ny - 1) * (int)gf.sy + min(max(fx0 + lx, 0), gf.nx - 1);
  }
  const int K0 = chunk * kc, K1 = min(K0 + kc, gc.nz);
  int iz[4];
  A wz[4];
  rtaps4<A>(K0 + gc.zoff, ncz, cz, iz, wz);
  const int f_lo = iz[0];
  rtaps4<A>(K1 - 1 + gc.zoff, ncz, cz, iz, wz);
  const int f_hi = max(max(iz[0], iz[1]), max(iz[2], iz[3]));
  T reg[EPT];
  auto fetch = [&](int f) {
    const T* src = fine + gf.sz * (int64_t)(f - fz_shift);
#pragma unroll
    for (int q = 0; q < EPT; ++q) reg[q] = src[src_off[q]];
  };
  A win[4];
  int K = K0;
  rtaps4<A>(K + gc.zoff, ncz, cz, iz, wz);
  fetch(f_lo);
  for (int f = f_lo; f <= f_hi; ++f) {
    __syncthreads();  // the previous plane's reads of `tile` are done
#pragma unroll
    for (int q = 0; q < EPT; ++q)
      if (tid + q * NT < FP) tile[tid + q * NT] = reg[q];
    if (f < f_hi) fetch(f + 1);
    __syncthreads();
    A vz = A(0);
#pragma unroll
    for (int bq = 0; bq < 4; ++bq) {
      const T* row = tile + (iy[bq] - fy0) * FX - fx0;
      A vy = A(0);
#pragma unroll
      for (int a = 0; a < 4; ++a) vy = fma(wx[a], (A)row[ix[a]], vy);
      vz = fma(wy[bq], vy, vz);
    }
    win[f & 3] = vz;
    // emit every coarse plane whose last tap is f (uniform)
    while (K < K1 && max(max(iz[0], iz[1]), max(iz[2], iz[3])) == f) {
      A v = A(0);
#pragma unroll
      for (int c = 0; c < 4; ++c) v = fma(wz[c], win[iz[c] & 3], v);
      if (ok) coarse[I + gc.sy * J + gc.sz * (int64_t)K] = (T)v;
      ++K;
      if (K < K1) rtaps4<A>(K + gc.zoff, ncz, cz, iz, wz);
    }
  }
}

// resid_restrict3_k: the coarse right-hand side b_c = R (b - A u) of one V-cycle descent
// (MAD.hxx:389,413) in one pass, without storing the fine residual.  Coarse tile CX x CY
// and coarse planes [K0, K1) as restrict3_k; each fine plane the chunk's taps need is
// residualised on restrict3_k's fine tile (2CX+2 x 2CY+2, fine indices clamped into
// the grid) from a 4-slot LDS ring of u planes over that tile + 1 (x/y mirror images
// in the ring, as resid3_k), the residuals go to an LDS tile, and restrict3_k's x-y
// taps, z window and emission follow.  Residual arithmetic = resid3_k's, restriction
// arithmetic = restrict3_k's, so b_c is bit-identical to residual + restriction.  With zx
// set, the coarse x is zeroed on the way (the descent's fill, MAD.hxx:415-416), on a rank
// slab with its ghost planes.
// Rank slabs: the coarse planes' taps are taken in global indices (coarse zoff, global coarse
// nz `ncz`) and shifted to local fine planes by fzs (the fine zoff); taps past the slab
// residualise the fine ghost planes (u, b and records current there: >= 2 ghost planes), the
// z mirror only at the global faces.  nx, ny >= 3, nz >= 2.
template <typename T, int KIND, int CX, int CY, int NT, bool BREC = false>
__global__ void __launch_bounds__(NT) resid_restrict3_k(
    const T* __restrict__ u, const T* __restrict__ b, const T* __restrict__ cf, Geo gf, Rat<T> rat,
    T* __restrict__ coarse, T* __restrict__ zx, Geo gc, int cx, int cy, int cz, int kc, int ntx,
    int fzs, int ncz) {
  static_assert(CX * CY <= NT, "one coarse point per thread");
  constexpr int FX = 2 * CX + 2, FY = 2 * CY + 2, FP = FX * FY;  // residual tile
  constexpr int UX = FX + 2, UY = FY + 2, UP = UX * UY;          // u region (tile + 1)
  constexpr int UPT = (UP + NT - 1) / NT;
  constexpr int RPT = (FP + NT - 1) / NT;
  constexpr int NCF = CoefLayout<3, KIND>::N;
  constexpr int RS = NCF + (BREC ? 1 : 0);
  constexpr uint32_t TS = sizeof(T);
  __shared__ T ring[4 * UP];
  __shared__ T rt[FP];
  const int tiles = ntx * ((gc.ny + CY - 1) / CY);
  const int chunk = blockIdx.x / tiles;
  const int t = blockIdx.x - chunk * tiles;
  const int tyi = t / ntx, txi = t - (t / ntx) * ntx;
  const int I0 = txi * CX, J0 = tyi * CY;
  const int tid = threadIdx.x;
  const int nx = gf.nx, ny = gf.ny, nz = gf.nz, sy = (int)gf.sy, hx0 = gf.hx0;
  const int64_t sz = gf.sz;
  const int fx0 = 2 * I0 - 1, fy0 = 2 * J0 - 1;  // residual tile origin (fine indices)
  const int ux0 = fx0 - 1, uy0 = fy0 - 1;        // u region origin
  auto mirror = [](int v, int n) { return v < 0 ? min(-v, n - 1) : (v >= n ? max(2 * (n - 1) - v, 0) : v); };
  // coarse point of this thread (threads < CX * CY)
  const bool cthr = tid < CX * CY;
  const int I = I0 + tid % CX, J = J0 + (tid / CX) % CY;
  const bool ok = cthr && I < gc.nx && J < gc.ny;
  int ix[4], iy[4];
  T wx[4], wy[4];
  rtaps4<T>(min(I, gc.nx - 1), gc.nx, cx, ix, wx);
  rtaps4<T>(min(J, gc.ny - 1), gc.ny, cy, iy, wy);
  // u region elements: LDS index and mirrored in-plane source offset
  int u_dst[UPT];
  uint32_t u_src[UPT];
#pragma unroll
  for (int e = 0; e < UPT; ++e) {
    const int q = tid + e * NT;
    const int lj = min(q, UP - 1) / UX, li = min(q, UP - 1) - (min(q, UP - 1) / UX) * UX;
    u_dst[e] = q < UP ? q : -1;
    u_src[e] = (uint32_t)(mirror(uy0 + lj, ny) * sy + mirror(ux0 + li, nx)) * TS;
  }
  // residual tile elements: the clamped fine point, its ring index, record / b offsets
  int r_il[RPT];
  uint32_t r_rec[RPT], r_pt[RPT];
#pragma unroll
  for (int e = 0; e < RPT; ++e) {
    const int q = min(tid + e * NT, FP - 1);
    const int ry = q / FX, rx = q - (q / FX) * FX;
    const int xf = min(max(fx0 + rx, 0), nx - 1), yf = min(max(fy0 + ry, 0), ny - 1);
    r_il[e] = (yf - uy0) * UX + (xf - ux0);
    r_rec[e] = (uint32_t)(yf * sy + (xf & 1) * hx0 + (xf >> 1)) * (TS * RS);
    r_pt[e] = (uint32_t)(yf * sy + xf) * TS;
  }
  const int K0 = chunk * kc, K1 = min(K0 + kc, gc.nz);
  int iz[4];
  T wz[4];
  // z taps of local coarse plane K as local fine planes
  auto ztaps = [&](int Kl) {
    rtaps4<T>(Kl + gc.zoff, ncz, cz, iz, wz);
#pragma unroll
    for (int c = 0; c < 4; ++c) iz[c] -= fzs;
  };
  ztaps(K0);
  const int f_lo = iz[0];
  ztaps(K1 - 1);
  const int f_hi = max(max(iz[0], iz[1]), max(iz[2], iz[3]));
  // loadable planes: the slab plus 2 ghost planes where a neighbour rank has them
  const int ulo = gf.zlo_ghost ? -2 : 0, uhi = gf.zhi_ghost ? nz + 2 : nz;

  T up[UPT];
  T raw[RPT][RS];
  T bv[RPT];
  auto load_plane = [&](int m) {
    m = min(max(m, ulo), uhi - 1);
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(u + (int64_t)m * sz);
#pragma unroll
    for (int e = 0; e < UPT; ++e) up[e] = buf_load<T>(rs, u_src[e], 0u);
  };
  auto put_plane = [&](int m) {
    T* P = ring + (m & 3) * UP;
#pragma unroll
    for (int e = 0; e < UPT; ++e)
      if (u_dst[e] >= 0) P[u_dst[e]] = up[e];
  };
  // waves whose elements all lie past the tile skip that element's loads and arithmetic
  const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
  auto wave_in = [&](int e) { return wbase + e * NT < FP; };
  auto load_pts = [&](int m) {
    m = min(max(m, ulo), uhi - 1);
    const __amdgpu_buffer_rsrc_t rr = buf_rsrc(cf + (int64_t)m * sz * RS);
    const __amdgpu_buffer_rsrc_t rb = buf_rsrc(b + (int64_t)m * sz);
#pragma unroll
    for (int e = 0; e < RPT; ++e) {
      if (e > 0 && !wave_in(e)) continue;
      buf_load_rec<T, RS>(rr, r_rec[e], raw[e]);
      if constexpr (!BREC) bv[e] = buf_load<T>(rb, r_pt[e], 0u);
    }
  };

  if (f_lo - 1 >= ulo) {
    load_plane(f_lo - 1);
    put_plane(f_lo - 1);
  }
  load_plane(f_lo);
  put_plane(f_lo);
  load_plane(f_lo + 1);
  load_pts(f_lo);
  T win[4];
  int K = K0;
  ztaps(K);
  for (int f = f_lo; f <= f_hi; ++f) {
    if (f + 1 < uhi) put_plane(f + 1);
    load_plane(f + 2);
    __syncthreads();  // ring planes f-1..f+1 staged; last plane's restriction reads of rt done
    const int zm = (f == 0 && !gf.zlo_ghost) ? f + 1 : f - 1;
    const int zp = (f == nz - 1 && !gf.zhi_ghost) ? f - 1 : f + 1;
#pragma unroll
    for (int e = 0; e < RPT; ++e) {
      if (e > 0 && !wave_in(e)) continue;
      const T* P0 = ring + (f & 3) * UP + r_il[e];
      const T* Pm = ring + (zm & 3) * UP + r_il[e];
      const T* Pp = ring + (zp & 3) * UP + r_il[e];
      T nb[18];
      nb[0] = P0[1];
      nb[1] = P0[-1];
      nb[2] = P0[UX];
      nb[3] = P0[-UX];
      nb[4] = Pp[0];
      nb[5] = Pm[0];
      if (KIND == KFULL) {
        nb[6] = P0[1 + UX];
        nb[7] = P0[1 - UX];
        nb[8] = P0[-1 + UX];
        nb[9] = P0[-1 - UX];
        nb[10] = Pp[1];
        nb[11] = Pm[1];
        nb[12] = Pp[-1];
        nb[13] = Pm[-1];
        nb[14] = Pp[UX];
        nb[15] = Pm[UX];
        nb[16] = Pp[-UX];
        nb[17] = Pm[-UX];
      }
      Coefs<T> q;
      coefs_from_raw<T, 3, KIND>(raw[e], rat, q);
      T D, S;
      stencil_combine<T, 3, KIND>(q, nb, D, S);
      const T rv = resid_value(BREC ? raw[e][NCF] : bv[e], D, P0[0], S);
      if (tid + e * NT < FP) rt[tid + e * NT] = rv;
    }
    if (f < f_hi) load_pts(f + 1);
    __syncthreads();  // residual tile of plane f complete
    {
#pragma clang fp contract(off)  // restrict3_k's explicit-fma order
      T vz = T(0);
#pragma unroll
      for (int bq = 0; bq < 4; ++bq) {
        const T* row = rt + (iy[bq] - fy0) * FX - fx0;
        T vy = T(0);
#pragma unroll
        for (int a = 0; a < 4; ++a) vy = fma(wx[a], row[ix[a]], vy);
        vz = fma(wy[bq], vy, vz);
      }
      win[f & 3] = vz;
      while (K < K1 && max(max(iz[0], iz[1]), max(iz[2], iz[3])) == f) {
        T v = T(0);
#pragma unroll
        for (int c = 0; c < 4; ++c) v = fma(wz[c], win[iz[c] & 3], v);
        if (ok) {
          const int64_t o = I + gc.sy * J + gc.sz * (int64_t)K;
          coarse[o] = v;
          if (zx) {
            zx[o] = T(0);
            // a rank slab's edge planes zero the GHOST ghost planes beyond them too: every rank
            // zeroes its own planes, so the neighbours' planes they stand for are zeros (no
            // exchange of the zeroed coarse x)
            if (K == 0 && gc.zlo_ghost) {
#pragma unroll
              for (int g = 1; g <= GHOST; ++g) zx[o - gc.sz * (int64_t)g] = T(0);
            }
            if (K == gc.nz - 1 && gc.zhi_ghost) {
#pragma unroll
              for (int g = 1; g <= GHOST; ++g) zx[o + gc.sz * (int64_t)g] = T(0);
            }
          }
        }
        ++K;
        if (K < K1) ztaps(K);
      }
    }
  }
}

// interp3_k: fine tile TX x TY (one thread per fine point), fine planes [k0, k1),
// marched in groups of G planes: the coarse planes a group's taps span go into an
// 8-slot LDS ring (only the ones not already there), and the fine values of the NEXT
// group are loaded while this group is computed, so each thread keeps G loads in
// flight (one plane at a time left the level-0 launch latency-bound at ~2.5 TB/s).
//
// VX > 1: each thread owns VX consecutive fine points of its row (fine tile TX*VX x TY) and
// moves them with one VX-wide load / store (the caller checks that rows, planes and the base
// are VX-aligned and nx % VX == 0); per point the same taps and the same fma chain as VX = 1.
template <typename T, int V>
struct alignas(sizeof(T) * V) VecT {
  T v[V];
};
template <typename T, int ADD, int TX, int TY, int G = 8, int VX = 1>
__global__ void __launch_bounds__(TX * TY) interp3_k(const T* __restrict__ coarse, Geo gc,
                                                     T* __restrict__ fine, Geo gf, int cx, int cy,
                                                     int cz, int ncz, int kc, int ntx, int kbase,
                                                     int kend) {
#pragma clang fp contract(off)  // explicit fma: every transfer kernel rounds alike
  constexpr int NT = TX * TY;
  constexpr int FX = TX * VX;  // fine points per tile row
  constexpr int CXW = FX / 2 + 2, CYW = TY / 2 + 2, CP = CXW * CYW;
  constexpr int NS = 8;           // ring slots
  constexpr int SPAN = G / 2 + 2;  // most coarse planes one group of G fine planes taps
  static_assert(SPAN <= NS && CP <= NT, "interp3_k ring geometry");
  using V = VecT<T, VX>;
  __shared__ T ring[NS * CP];
  const int tiles = ntx * ((gf.ny + TY - 1) / TY);
  const int chunk = blockIdx.x / tiles;
  const int t = blockIdx.x - chunk * tiles;
  const int tyi = t / ntx, txi = t - (t / ntx) * ntx;
  const int i0 = txi * FX, j0 = tyi * TY;
  const int tid = threadIdx.x;
  const int i = i0 + (tid % TX) * VX, j = j0 + tid / TX;
  const bool ok = i < gf.nx && j < gf.ny;
  const int cx0 = i0 / 2 - 1, cy0 = j0 / 2 - 1;  // coarse tile origin
  int ix[VX][2], iy[2];
  T wx[VX][2], wy[2];
#pragma unroll
  for (int v = 0; v < VX; ++v) itaps2<T>(min(i + v, gf.nx - 1), gc.nx, cx, ix[v], wx[v]);
  itaps2<T>(min(j, gf.ny - 1), gc.ny, cy, iy, wy);
  const int ci = tid < CP ? tid : CP - 1;  // one ring element per thread (CP <= NT)
  const int c_off = min(max(cy0 + ci / CXW, 0), gc.ny - 1) * (int)gc.sy +
                    min(max(cx0 + ci % CXW, 0), gc.nx - 1);
  // fine planes [kbase, kend), local; on a rank slab the range may include the ghost
  // planes (their coarse taps then reach up to 3 coarse ghost planes)
  const int k0 = kbase + chunk * kc, k1 = min(k0 + kc, kend);
  const int64_t pxy = (int64_t)j * gf.sy + i;
  int last = INT_MIN;  // largest coarse plane (global) in the ring
  V xc[G], xn[G];
  auto load_fine = [&](int kk, V* dst) {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (ADD && ok && kk + q < k1) {
        dst[q] = *reinterpret_cast<const V*>(fine + pxy + gf.sz * (int64_t)(kk + q));
      } else {
#pragma unroll
        for (int v = 0; v < VX; ++v) dst[q].v[v] = T(0);
      }
    }
  };
  load_fine(k0, xc);
  for (int k = k0; k < k1; k += G) {
    // coarse taps are monotone in the fine plane: the group spans [min taps(k), max taps(kl)]
    const int kl = min(k + G, k1) - 1;
    int iz[2];
    T wz[2];
    itaps2<T>(k + gf.zoff, ncz, cz, iz, wz);
    const int lo = max(min(iz[0], iz[1]), last + 1);
    itaps2<T>(kl + gf.zoff, ncz, cz, iz, wz);
    const int hi = max(iz[0], iz[1]);
    T cv[SPAN];
#pragma unroll
    for (int q = 0; q < SPAN; ++q)
      cv[q] = (lo + q <= hi) ? coarse[gc.sz * (int64_t)(lo + q - gc.zoff) + c_off] : T(0);
    load_fine(k + G, xn);  // next group, in flight across this one
#pragma unroll
    for (int q = 0; q < SPAN; ++q)
      if (lo + q <= hi && tid < CP) ring[((lo + q) & (NS - 1)) * CP + tid] = cv[q];
    last = max(last, hi);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int kk = k + q;
      if (kk > kl) break;
      itaps2<T>(kk + gf.zoff, ncz, cz, iz, wz);
      V out;
#pragma unroll
      for (int x = 0; x < VX; ++x) {
        T v = T(0);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const T* pl = ring + (iz[c] & (NS - 1)) * CP - cx0;
          T vz = T(0);
#pragma unroll
          for (int bq = 0; bq < 2; ++bq) {
            const T* row = pl + (iy[bq] - cy0) * CXW;
            vz = fma(wy[bq], fma(wx[x][1], row[ix[x][1]], wx[x][0] * row[ix[x][0]]), vz);
          }
          v = fma(wz[c], vz, v);
        }
        out.v[x] = ADD ? xc[q].v[x] + v : v;
      }
      if (ok) *reinterpret_cast<V*>(fine + pxy + gf.sz * (int64_t)kk) = out;
    }
    __syncthreads();  // ring slots are reused by the next group
#pragma unroll
    for (int q = 0; q < G; ++q) xc[q] = xn[q];
  }
}

// copy the dense rhs into the b slot (index ncf) of the coefficient records of local
// planes [p0, p1) (ghost planes included on rank slabs): LevelData::brec levels
// dense b -> its x-parity-split copy (gs_fused3_k BS): the records' point order without the stride
template <typename T>
__global__ void __launch_bounds__(256) bsplit_k(const T* __restrict__ b, T* __restrict__ bs, Geo g, int p0) {
  const int k = p0 + (int)blockIdx.z;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.nx || j >= g.ny) return;
  bs[cidx(g, i, j, k)] = b[i + g.sy * j + g.sz * (int64_t)k];
}

template <typename T>
__global__ void __launch_bounds__(256) brec_scatter_k(const T* __restrict__ b, T* __restrict__ cf,
                                                      Geo g, int ncf, int p0) {
  const int k = p0 + (int)blockIdx.z;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.nx || j >= g.ny) return;
  cf[cidx(g, i, j, k) * g.rs + ncf] = b[i + g.sy * j + g.sz * (int64_t)k];
}

// ---------------------------------------------------------------------------
// coarsest-grid solve x = A^-1 b with the precomputed fp64 inverse: one wave per row.  The row
// dot product: default fp contraction (a kernel that inlines it keeps that, whatever its own pragmas).
template <typename T>
__device__ __forceinline__ double coarse_row_dot(const double* __restrict__ a, const T* __restrict__ b,
                                                 int n, int lane) {
  double s = 0.0;
  for (int c = lane; c < n; c += 64) s += a[c] * (double)b[c];
  return wave_sum(s);
}

template <typename T>
__global__ void __launch_bounds__(256) coarse_solve_k(const double* __restrict__ inv,
                                                      const T* __restrict__ b, T* __restrict__ x,
                                                      int n) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double s = coarse_row_dot(inv + (int64_t)row * n, b, n, lane);
  if (lane == 0) x[row] = (T)s;
}

// ---------------------------------------------------------------------------
// elementwise helpers
template <typename T>
__global__ void __launch_bounds__(256) fill_k(T* __restrict__ x, int64_t n, T v) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x)
    x[q] = v;
}

template <typename S, typename D>
__global__ void __launch_bounds__(256) convert_k(const S* __restrict__ x, D* __restrict__ y,
                                                 int64_t n) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x)
    y[q] = (D)x[q];
}

// defect-correction update u += (double) e (MAD_FP32_REFINE: fp64 iterate, fp32 correction)
template <typename S>
__global__ void __launch_bounds__(256) add_conv_k(double* __restrict__ u, const S* __restrict__ e,
                                                  int64_t n) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x)
    u[q] += (double)e[q];
}

// static_cast<OutputPixelType>(double) for integer outputs: truncation toward zero,
// saturated to the type's range (the reference leaves out-of-range values undefined)
template <typename S, typename D>
__global__ void __launch_bounds__(256) convert_int_k(const S* __restrict__ x, D* __restrict__ y,
                                                     int64_t n, double lo, double hi) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    double v = trunc((double)x[q]);
    v = v < lo ? lo : (v > hi ? hi : v);
    if (v != v) v = 0.0;
    y[q] = (D)v;
  }
}

// ---------------------------------------------------------------------------
// setup (fp64): AoS input tensor -> SoA, kind detection, coefficient fields
// (n points; component c of point q at out[c * cs + q]: cs = n for a whole grid, the slab
// array's component stride on a rank)
template <typename S>
__global__ void __launch_bounds__(256) aos_to_soa_k(const S* __restrict__ in, double* __restrict__ out,
                                                    int64_t n, int ncomp, int64_t cs) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < ncomp; ++c) out[c * cs + q] = (double)in[q * ncomp + c];
}

// flags[0] += any off-diagonal != 0, flags[1] += any diagonal entries differ,
// flags[2] += any entry non-finite (NaN / Inf: MAD_ERR_NUMERIC at setup)
__global__ void __launch_bounds__(256) tensor_kind_k(const double* __restrict__ M, int64_t n, int64_t cs,
                                                     int dim, unsigned int* __restrict__ flags) {
  unsigned int off = 0, aniso = 0, bad = 0;
  const int ncomp = dim * (dim + 1) / 2;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    if (dim == 3) {
      off |= (M[1 * cs + q] != 0.0) | (M[2 * cs + q] != 0.0) | (M[4 * cs + q] != 0.0);
      aniso |= (M[0 * cs + q] != M[3 * cs + q]) | (M[0 * cs + q] != M[5 * cs + q]);
    } else {
      off |= (M[1 * cs + q] != 0.0);
      aniso |= (M[0 * cs + q] != M[2 * cs + q]);
    }
    for (int c = 0; c < ncomp; ++c) bad |= !isfinite(M[c * cs + q]);
  }
  if (__any(off) && (threadIdx.x & 63) == 0) atomicOr(&flags[0], 1u);
  if (__any(aniso) && (threadIdx.x & 63) == 0) atomicOr(&flags[1], 1u);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&flags[2], 1u);
}

__device__ __forceinline__ int tcomp(int dim, int d, int d2) {
  if (d > d2) { const int t = d; d = d2; d2 = t; }
  return d * dim - d * (d - 1) / 2 + (d2 - d);
}

// 2h * d f / dx_d with the reference's border formulas (GH.hxx:447-474)
__device__ __forceinline__ double delta_f(const double* __restrict__ f, int64_t p, int idx, int n,
                                          int64_t st) {
  if (idx == 0) return -3. * f[p] + 4. * f[p + st] - 1. * f[p + 2 * st];
  if (n - idx == 1) return 3. * f[p] - 4. * f[p - st] + 1. * f[p - 2 * st];
  return f[p + st] - f[p - st];
}

// spacing / time-step factors of the coefficient fields, computed once on the host
// (the kernel then multiplies instead of dividing: fp64 division is a long VALU sequence)
struct CoefFactors {
  double fa[3];      // dt / h_d^2                 (a_d = fa[d] M_dd)
  double fg[3];      // 1 / (2 h_d2)               (g_d = fgo[d] sum_d2 delta_d2 M_d,d2 fg[d2])
  double fgo[3];     // dt / (2 h_d)
  double fe[3][3];   // dt / (2 h_d h_d2)          (e_dd2 = fe[d][d2] M_d,d2)
};

inline CoefFactors coef_factors(const double h[3], double dt) {
  CoefFactors f{};
  for (int d = 0; d < 3; ++d) {
    f.fa[d] = dt / (h[d] * h[d]);
    f.fg[d] = 1.0 / (2.0 * h[d]);
    f.fgo[d] = dt / (2.0 * h[d]);
    for (int d2 = 0; d2 < 3; ++d2) f.fe[d][d2] = dt / (2.0 * h[d] * h[d2]);
  }
  return f;
}

// coefficient fields of one (global) level from its fp64 tensor
template <typename T, int DIM, int KIND>
__global__ void __launch_bounds__(256) build_coef_k(const double* __restrict__ M, int nx, int ny,
                                                    int nz, CoefFactors f, T* __restrict__ cf,
                                                    int rs) {
  using L = CoefLayout<DIM, KIND>;
  const int k = (DIM == 3) ? (int)blockIdx.z : 0;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nx || j >= ny) return;
  const int64_t n = (int64_t)nx * ny * nz;
  const int64_t p = i + (int64_t)nx * (j + (int64_t)ny * k);
  // output record in the point-interleaved, x-parity-split coefficient layout (cidx)
  const int64_t o = ((int64_t)nx * (j + (int64_t)ny * k) + ((i & 1) ? (nx + 1) / 2 + (i >> 1) : (i >> 1))) * rs;
  const int nn[3] = {nx, ny, nz};
  const int id[3] = {i, j, k};
  const int64_t st[3] = {1, nx, (int64_t)nx * ny};
  if (KIND == KISO) {
    cf[o] = (T)(f.fa[0] * M[p]);
  } else {
#pragma unroll
    for (int d = 0; d < DIM; ++d) cf[o + d] = (T)(f.fa[d] * M[tcomp(DIM, d, d) * n + p]);
  }
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    double s = 0.0;
#pragma unroll
    for (int d2 = 0; d2 < DIM; ++d2)
      s += delta_f(M + tcomp(DIM, d, d2) * n, p, id[d2], nn[d2], st[d2]) * f.fg[d2];
    cf[o + L::NA + d] = (T)(f.fgo[d] * s);
  }
  if (KIND == KFULL) {
    int e = L::NA + L::NG;
#pragma unroll
    for (int d = 0; d < DIM; ++d)
#pragma unroll
      for (int d2 = d + 1; d2 < DIM; ++d2, ++e)
        cf[o + e] = (T)(f.fe[d][d2] * M[tcomp(DIM, d, d2) * n + p]);
  }
}

// 3D coefficient fields, z-marching: a 64 x 4 block of columns walks its planes and keeps
// the z-derivative components M_xz, M_yz, M_zz of planes k-1, k, k+1 in registers, so the
// z-neighbour reads of g (one plane away, evicted from L2 by the time a per-plane grid
// reaches them) come from the previous iterations; in-plane neighbours and the one-sided
// border formulas read memory as build_coef_k does.  Same arithmetic and order, so the
// coefficients are bit-identical to build_coef_k's.
// Global plane indices throughout: planes [kb, ke) of a level with nz planes are built; M and cf
// point at global plane 0 (on a rank slab: the slab arrays shifted by their first global plane,
// only planes [kb - 2, ke + 2) of M and [kb, ke) of cf are touched); cs is M's component stride.
template <typename T, int KIND>
__global__ void __launch_bounds__(256) build_coef3_k(const double* __restrict__ M, int nx, int ny,
                                                     int nz, CoefFactors f, T* __restrict__ cf,
                                                     int rs, int kc, int kb, int ke, int64_t cs) {
  using L = CoefLayout<3, KIND>;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int k0 = kb + blockIdx.z * kc, k1 = min(k0 + kc, ke);
  if (i >= nx || j >= ny || k0 >= k1) return;
  const int64_t n = cs, sz = (int64_t)nx * ny;
  const int64_t col = i + (int64_t)nx * j;
  const int64_t orow = ((int64_t)nx * j + ((i & 1) ? (nx + 1) / 2 + (i >> 1) : (i >> 1)));
  const int nn[3] = {nx, ny, nz};
  const int64_t st[3] = {1, nx, sz};
  // z-window of M_{d,z}, d = x, y, z (components tcomp(3, d, 2) = 2, 4, 5)
  const double* Mz[3] = {M + 2 * n, M + 4 * n, M + 5 * n};
  double zm[3], z0v[3], zp[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    zm[d] = k0 > 0 ? Mz[d][col + (int64_t)(k0 - 1) * sz] : 0.0;
    z0v[d] = Mz[d][col + (int64_t)k0 * sz];
    zp[d] = k0 + 1 < nz ? Mz[d][col + (int64_t)(k0 + 1) * sz] : 0.0;
  }
  for (int k = k0; k < k1; ++k) {
    const int64_t p = col + (int64_t)k * sz;
    const int64_t o = (orow + (int64_t)k * sz) * rs;
    const int id[3] = {i, j, k};
    if (KIND == KISO) {
      cf[o] = (T)(f.fa[0] * M[p]);
    } else {
#pragma unroll
      for (int d = 0; d < 3; ++d) cf[o + d] = (T)(f.fa[d] * M[tcomp(3, d, d) * n + p]);
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      double s = 0.0;
#pragma unroll
      for (int d2 = 0; d2 < 3; ++d2) {
        double dl;
        if (d2 == 2 && k > 0 && k < nz - 1) {
          dl = zp[d] - zm[d];  // delta_f's interior formula, from the register window
        } else {
          dl = delta_f(M + tcomp(3, d, d2) * n, p, id[d2], nn[d2], st[d2]);
        }
        s += dl * f.fg[d2];
      }
      cf[o + L::NA + d] = (T)(f.fgo[d] * s);
    }
    if (KIND == KFULL) {
      int e = L::NA + L::NG;
#pragma unroll
      for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int d2 = d + 1; d2 < 3; ++d2, ++e)
          cf[o + e] = (T)(f.fe[d][d2] * M[tcomp(3, d, d2) * n + p]);
    }
    // shift the window one plane up
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      zm[d] = z0v[d];
      z0v[d] = zp[d];
      zp[d] = k + 2 < nz ? Mz[d][col + (int64_t)(k + 2) * sz] : 0.0;
    }
  }
}

// ---------------------------------------------------------------------------
// g from the stored (storage-type) a / e coefficients.  With a_d = dt M_dd / h_d^2 and
// e_dd2 = dt M_dd2 / (2 h_d h_d2) the reference's g_d = dt/(2h_d) sum_d2 delta_d2 M_d,d2
// / (2 h_d2) (GH.hxx:447-474) is, exactly,
//   g_x = 1/4 delta_x a_x + 1/2 delta_y e_xy + 1/2 delta_z e_xz   (and cyclically)
// with delta the reference's 2h-scaled differences (central; one-sided second order at
// the border, delta_f).  Every kernel evaluates g through these helpers on the same
// T-typed inputs in the same order.
// At the faces the reference's one-sided second-order differences, in its order
// (GH.hxx:454-462): (-3 f(0) + 4 f(1)) - f(2) at the low face, (3 f(0) - 4 f(-1)) + f(-2)
// at the high face (the fp64 refine build, build_coef*_k, evaluates the same expressions).
template <typename T>
__device__ __forceinline__ T gdelta(T fm2, T fm1, T f0, T fp1, T fp2, bool lo, bool hi) {
#pragma clang fp contract(off)
  if (lo) return (T(-3) * f0 + T(4) * fp1) - fp2;
  if (hi) return (T(3) * f0 - T(4) * fm1) + fm2;
  return fp1 - fm1;
}

// g_d from the differences of the coefficient fields (dA_d2 = delta_d2 of field A)
template <typename T, int DIM, int KIND>
__device__ __forceinline__ void g_combine(T dxax, T dyay, T dzaz, T dxexy, T dyexy, T dxexz,
                                          T dzexz, T dyeyz, T dzeyz, T& gx, T& gy, T& gz) {
#pragma clang fp contract(off)
  if (KIND == KFULL) {
    gx = T(0.25) * dxax + T(0.5) * dyexy;
    gy = T(0.5) * dxexy + T(0.25) * dyay;
    if (DIM == 3) {
      gx = gx + T(0.5) * dzexz;
      gy = gy + T(0.5) * dzeyz;
      gz = (T(0.5) * dxexz + T(0.5) * dyeyz) + T(0.25) * dzaz;
    } else {
      gz = T(0);
    }
  } else {
    gx = T(0.25) * dxax;
    gy = T(0.25) * dyay;
    gz = (DIM == 3) ? T(0.25) * dzaz : T(0);
  }
}

// stored g of one level (records already holding a / e): per point, the neighbours'
// coefficients from memory.  In place: g slots are written, a / e only read.  Planes kb +
// blockIdx.z (global indices, cf at global plane 0; a / e current on planes +-2 around them).
template <typename T, int DIM, int KIND>
__global__ void __launch_bounds__(256) build_g_k(T* __restrict__ cf, int nx, int ny, int nz, int rs,
                                                 Rat<T> rat, int kb) {
  using L = CoefLayout<DIM, KIND>;
  const int k = (DIM == 3) ? kb + (int)blockIdx.z : 0;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nx || j >= ny) return;
  const int hx0 = (nx + 1) / 2;
  auto Q = [&](int ii, int jj, int kk) {
    ii = min(max(ii, 0), nx - 1);
    jj = min(max(jj, 0), ny - 1);
    kk = min(max(kk, 0), nz - 1);
    const int64_t c = ((int64_t)kk * ny + jj) * nx + ((ii & 1) ? hx0 + (ii >> 1) : (ii >> 1));
    Coefs<T> q;
    load_coefs<T, DIM, KIND>(cf, c, rs, rat, q);
    return q;
  };
  const bool xl = i == 0, xh = !xl && i == nx - 1;
  const bool yl = j == 0, yh = !yl && j == ny - 1;
  const bool zl = k == 0, zh = !zl && k == nz - 1;
  const Coefs<T> c0 = Q(i, j, k);
  const Coefs<T> xm1 = Q(i - 1, j, k), xp1 = Q(i + 1, j, k), xm2 = Q(i - 2, j, k), xp2 = Q(i + 2, j, k);
  const Coefs<T> ym1 = Q(i, j - 1, k), yp1 = Q(i, j + 1, k), ym2 = Q(i, j - 2, k), yp2 = Q(i, j + 2, k);
  T dxax = gdelta(xm2.ax, xm1.ax, c0.ax, xp1.ax, xp2.ax, xl, xh);
  T dyay = gdelta(ym2.ay, ym1.ay, c0.ay, yp1.ay, yp2.ay, yl, yh);
  T dxexy = gdelta(xm2.exy, xm1.exy, c0.exy, xp1.exy, xp2.exy, xl, xh);
  T dyexy = gdelta(ym2.exy, ym1.exy, c0.exy, yp1.exy, yp2.exy, yl, yh);
  T dxexz = gdelta(xm2.exz, xm1.exz, c0.exz, xp1.exz, xp2.exz, xl, xh);
  T dyeyz = gdelta(ym2.eyz, ym1.eyz, c0.eyz, yp1.eyz, yp2.eyz, yl, yh);
  T dzaz = T(0), dzexz = T(0), dzeyz = T(0);
  if (DIM == 3) {
    const Coefs<T> zm1 = Q(i, j, k - 1), zp1 = Q(i, j, k + 1), zm2 = Q(i, j, k - 2), zp2 = Q(i, j, k + 2);
    dzaz = gdelta(zm2.az, zm1.az, c0.az, zp1.az, zp2.az, zl, zh);
    dzexz = gdelta(zm2.exz, zm1.exz, c0.exz, zp1.exz, zp2.exz, zl, zh);
    dzeyz = gdelta(zm2.eyz, zm1.eyz, c0.eyz, zp1.eyz, zp2.eyz, zl, zh);
  }
  T gx, gy, gz;
  g_combine<T, DIM, KIND>(dxax, dyay, dzaz, dxexy, dyexy, dxexz, dzexz, dyeyz, dzeyz, gx, gy, gz);
  const int64_t o = (((int64_t)k * ny + j) * nx + ((i & 1) ? hx0 + (i >> 1) : (i >> 1))) * rs;
  cf[o + L::NA] = gx;
  cf[o + L::NA + 1] = gy;
  if (DIM == 3) cf[o + L::NA + 2] = gz;
}

// ---------------------------------------------------------------------------
// deterministic synthetic inputs (bench / smoke), mirrored in tests/synth.py
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ double u01(uint64_t seed, int64_t q) {
  return (double)(splitmix64(seed * 0x100000001B3ull + (uint64_t)q) >> 11) * 0x1.0p-53;
}

// x-fastest global index q over the global grid, written at local plane offset
template <typename T>
__global__ void __launch_bounds__(256) synth_image_k(T* __restrict__ x, Geo g, int64_t nxg,
                                                     int64_t nyg, uint64_t seed) {
  const int k = blockIdx.z;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.nx || j >= g.ny) return;
  const int64_t qg = i + nxg * (j + nyg * (int64_t)(k + g.zoff));
  x[i + g.sy * j + g.sz * k] = (T)u01(seed, qg);
}

// VED-form tensor T = lp I + (la - lp) v v^T (include/itkVEDMultigridImageFilter.hxx:327-365
// with V = resp^(1/s), identity where V == 0) on the analytic fields of tests/synth.py.
// Global planes kb + blockIdx.z of an nz-plane grid; M at global plane 0, component stride cs.
__global__ void __launch_bounds__(256) synth_ved_k(double* __restrict__ M, int nx, int ny, int nz,
                                                   uint64_t seed, double eps, double omega,
                                                   double sens, int kb, int64_t cs) {
  const int k = kb + (int)blockIdx.z;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nx || j >= ny) return;
  const int64_t n = cs;
  const int64_t p = i + (int64_t)nx * (j + (int64_t)ny * k);
  const double PI2 = 6.283185307179586;
  const double x = i, y = j, z = k;
  const double fx = nx > 2 ? nx : 2, fy = ny > 2 ? ny : 2, fz = nz > 2 ? nz : 2;
  const double sd = (double)seed;
  double s = sin(PI2 * x / fx * 3.0 + sd) * sin(PI2 * y / fy * 2.0 + 0.5 * sd) *
             cos(PI2 * z / fz * 2.5);
  s = s > 0.0 ? s : 0.0;
  const double resp = s * s;
  const double V = resp > 0.0 ? pow(resp, 1.0 / sens) : 0.0;
  double vx = sin(PI2 * y / fy * 1.5) + 0.3;
  double vy = cos(PI2 * z / fz * 1.25);
  double vz = 1.0 + 0.5 * sin(PI2 * x / fx);
  const double nrm = sqrt(vx * vx + vy * vy + vz * vz);
  vx /= nrm; vy /= nrm; vz /= nrm;
  const double lp = 1.0 + (eps - 1.0) * V;
  const double la = 1.0 + (omega - 1.0) * V;
  const double d = la - lp;
  M[0 * n + p] = lp + d * vx * vx;
  M[1 * n + p] = d * vx * vy;
  M[2 * n + p] = d * vx * vz;
  M[3 * n + p] = lp + d * vy * vy;
  M[4 * n + p] = d * vy * vz;
  M[5 * n + p] = lp + d * vz * vz;
}

// isotropic c(x) I, c = 1 + 0.5 sin sin sin (period 32)
__global__ void __launch_bounds__(256) synth_iso_k(double* __restrict__ M, int nx, int ny, int nz,
                                                   int dim, uint64_t seed, int kb, int64_t cs) {
  const int k = kb + (int)blockIdx.z;
  const int j = blockIdx.y * blockDim.y + threadIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nx || j >= ny) return;
  const int64_t n = cs;
  (void)nz;
  const int64_t p = i + (int64_t)nx * (j + (int64_t)ny * k);
  const double PI2 = 6.283185307179586;
  const double ph = 0.3 * (double)seed;
  double c = sin(PI2 * i / 32.0 + ph) * sin(PI2 * j / 32.0 + ph);
  if (dim == 3) c *= sin(PI2 * k / 32.0 + ph);
  c = 1.0 + 0.5 * c;
  if (dim == 3) {
    M[0 * n + p] = c; M[1 * n + p] = 0.0; M[2 * n + p] = 0.0;
    M[3 * n + p] = c; M[4 * n + p] = 0.0; M[5 * n + p] = c;
  } else {
    M[0 * n + p] = c; M[1 * n + p] = 0.0; M[2 * n + p] = c;
  }
}

}  // namespace mad
