// mad_tsweep.hpp -- the level-0 4-colour Gauss-Seidel sweep of the full 3D operator that
// reads the 24-B tensor instead of the 36-B coefficient records: g is recomputed in-kernel.
//
// Reference: the sweep is itk::mad::MultigridGaussSeidelSmoother::SingleIteration
// (include/mad/itkMultigridGaussSeidelSmoother.hxx:67-106) on the DCA operator of
// include/mad/itkGridsHierarchy.hxx:298-516, whose first-derivative terms (:447-474) are
//   g_x = 1/4 delta_x a_x + 1/2 delta_y e_xy + 1/2 delta_z e_xz   (and cyclically),
// i.e. central differences of the neighbours' tensors (g_combine / gdelta, mad_kernels.hpp).
//
// Bytes per voxel-sweep: tensor 24 + b 4 + u 4 in + 4 out = 36 (the algorithmic figure),
// against 48 for gs_fused3_k, whose records also carry g.
//
// Schedule.  The z-marching wavefront of gs_fused3_k updates colour c of plane m at step
// m + c; here instance (c, k) (colour c on plane k - c) runs in phase 2k + c, two phases per
// step.  A colour-c point reads colours < c on planes m-1..m+1 NEW and colours > c OLD: colour
// c' of plane m' runs in phase 2m' + 3c', so the worst cases (m' = m+1, c' = c-1 and m' = m-1,
// c' = c+1) are one phase before / after -- a barrier between phases orders everything, and the
// two instances of a phase, (c, k) and (c+2, k-1), touch planes three apart.
// Tiles: 32 x 32 with halo H = 4 (region 40 x 40, overlapped tiling); a 7-plane LDS ring of
// u (x-parity-split rows, domain-face mirror images kept in the ring).
//
// Threads: one per vertical 1 x 2 "domino" (points (i, 2r), (i, 2r+1) of the region).  Class
// 0 threads (waves 0-6) own the even columns, class 1 (waves 7-13) the odd ones.  With the
// colouring ((i+k)&1) | ((j+k)&1)<<1 every instance of step k updates points of class k & 1
// (plane parity), so each phase runs one instance on each class: all 14 waves work in every
// phase.
//
// The tensor: each plane's region (40 rows of the six component segments, x-parity split) is
// copied into one of two LDS buffers by the buffer unit itself (buffer_load ... lds: no VGPRs in
// flight), issued two phases ahead.  In the gap before phase 2k every thread forms the records
// (a, g, e, b) of its two points on plane k: x / y differences from its neighbours in buffer k,
// z differences between buffer k+1 and the previous plane's z components kept in registers.
// A record then waits in registers until its instance, 0..4 steps later (about 5 per thread).
// Domain faces need no code here: the tensor array carries ghost values one point outside every
// face (build_gt_k) whose central difference is the one-sided border difference, rounded as
// build_g_k rounds it (gghost).
//
// Bit-identical to per-colour passes over build_g_k's records (same Coefs, g_combine,
// stencil_combine and gs_update on the same fp32 values).
#pragma once
#include "mad_kernels.hpp"

namespace mad {

struct TSweepGeom {
  static constexpr int TX = 32, TY = 32, H = 4;
  static constexpr int RX = TX + 2 * H, RY = TY + 2 * H;  // 40 x 40 region
  static constexpr int DX = RX / 2;                       // columns per class
  static constexpr int ND = DX * (RY / 2);                // dominoes per class (400)
  static constexpr int CT = ((ND + 63) / 64) * 64;        // threads per class (448)
  static constexpr int NT = 2 * CT;                       // 896 threads, 14 waves
  static constexpr int HALF = DX;                         // u ring row: even-x, then odd-x half
  // 2 * PITCH = 20 (mod 32): the 20 lanes of a domino row pair and the next pair's lanes read
  // disjoint banks with ds_read_b32
  static constexpr int PITCH = 42;
  static constexpr int NP = 7;                            // u ring planes (phase 2k+1 reads k-5..k)
  static constexpr int UPLANE = RY * PITCH;               // floats per ring plane
  static constexpr int NCOMP = 6;                         // a_x a_y a_z e_xy e_xz e_yz
  static constexpr int CSEG = RX * 4;                     // bytes of one component of a region row
  static constexpr int HSEG = CSEG / 2;                   // its even-x / odd-x half
  // LDS row: six component segments of 160 B (even-x half, odd-x half), padded to 250 dwords
  // so that 2 * 250 = 20 (mod 32) as for the ring
  static constexpr int RROW = 1000;
  static constexpr int RBUF = RY * RROW;                  // bytes per tensor buffer
  static constexpr int LDS_BYTES = 2 * RBUF + NP * UPLANE * 4;  // 127,040
  static constexpr int PAD = 4;                           // tensor array padding (points)
};

// Tensor array geometry ("row-SoA", x-parity split): a row of a plane holds the six component
// segments of tpitch floats each, every segment its even-x points then its odd-x points, so one
// region row's half segment is 80 contiguous bytes and a row's twelve half segments reach LDS
// as one 60-lane buffer_load ... lds.  Component c of point (i, j, k) is at
//   k * tplane + (j + PAD) * trow + c * tpitch + ((i + PAD) & 1) * tpitch / 2 + (i + PAD) / 2
// from the plane-0 base; GHOST planes below / above.
struct TGeo {
  int64_t tpitch, trow, tplane;
};

// Tensor array of the g-free sweep from the storage-type coefficient records (their a / e),
// every allocated plane: in-domain points copy [a_x a_y a_z e_xy e_xz e_yz]; the points one
// outside a domain face get, for the components differenced across that face, gghost's value
// (x faces: a_x e_xy e_xz; y: a_y e_xy e_yz; z, global faces only: a_z e_xz e_yz); a rank
// slab's ghost planes hold the neighbour's records.  Everything else is 0.
template <typename T>
__global__ void __launch_bounds__(256) build_gt_k(const T* __restrict__ cf, Geo g, T* __restrict__ gt,
                                                  TGeo tg, int p0) {
  constexpr int NA = 3;
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) - 1;
  const int j = (int)(blockIdx.y * blockDim.y + threadIdx.y) - 1;
  const int k = (int)blockIdx.z + p0;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  if (i > nx || j > ny) return;
  // field of component q: a_x a_y a_z -> 0 1 2, e_xy e_xz e_yz -> 6 7 8
  auto F = [&](int ii, int jj, int q) -> T {
    const int f = q < 3 ? q : NA + 3 + (q - 3);
    return cf[cidx(g, ii, jj, k) * g.rs + f];
  };
  auto FZ = [&](int kk, int q) -> T {
    const int f = q < 3 ? q : NA + 3 + (q - 3);
    return cf[cidx(g, i, j, kk) * g.rs + f];
  };
  const bool inx = i >= 0 && i < nx, iny = j >= 0 && j < ny;
  const bool inz = (k >= 0 && k < nz) || (k < 0 && g.zlo_ghost) || (k >= nz && g.zhi_ghost);
  T out[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};
  if (inx && iny && inz) {
#pragma unroll
    for (int q = 0; q < 6; ++q) out[q] = F(i, j, q);
  } else if (!inx && iny && inz) {  // x ghost column (i = -1 or nx): a_x e_xy e_xz
    const int q3[3] = {0, 3, 4};
#pragma unroll
    for (int t = 0; t < 3; ++t)
      out[q3[t]] = (i < 0) ? gghost(F(0, j, q3[t]), F(1, j, q3[t]), F(2, j, q3[t]))
                           : gghost(F(nx - 1, j, q3[t]), F(nx - 2, j, q3[t]), F(nx - 3, j, q3[t]));
  } else if (inx && !iny && inz) {  // y ghost row: a_y e_xy e_yz
    const int q3[3] = {1, 3, 5};
#pragma unroll
    for (int t = 0; t < 3; ++t)
      out[q3[t]] = (j < 0) ? gghost(F(i, 0, q3[t]), F(i, 1, q3[t]), F(i, 2, q3[t]))
                           : gghost(F(i, ny - 1, q3[t]), F(i, ny - 2, q3[t]), F(i, ny - 3, q3[t]));
  } else if (inx && iny && ((k == -1 && !g.zlo_ghost) || (k == nz && !g.zhi_ghost))) {
    const int q3[3] = {2, 4, 5};  // global z face: a_z e_xz e_yz
#pragma unroll
    for (int t = 0; t < 3; ++t)
      out[q3[t]] = (k < 0) ? gghost(FZ(0, q3[t]), FZ(1, q3[t]), FZ(2, q3[t]))
                           : gghost(FZ(nz - 1, q3[t]), FZ(nz - 2, q3[t]), FZ(nz - 3, q3[t]));
  }
  const int ip = i + TSweepGeom::PAD;
  T* o = gt + (int64_t)k * tg.tplane + (int64_t)(j + TSweepGeom::PAD) * tg.trow + (ip & 1) * (tg.tpitch / 2) +
         (ip >> 1);
#pragma unroll
  for (int q = 0; q < 6; ++q) o[q * tg.tpitch] = out[q];
}

// LDS barrier that leaves buffer loads (the tensor copies into LDS, u / b prefetches) in
// flight: this wave's LDS writes complete, then s_barrier.  __syncthreads() would also wait
// for vmcnt(0), i.e. for the next plane's tensor copy issued this step.
__device__ __forceinline__ void tsweep_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One full 4-colour GS sweep uin -> uout (level-0 layout: dense u / b with GHOST planes,
// tensor array gt0 = plane 0 of build_gt_k's array).  Launch: NT threads, LDS_BYTES dynamic
// LDS, ntx * nty * nchunks workgroups (chunk q covers owned planes [zbase + q*zstride, +zc)).
template <int CLS>
__device__ __forceinline__ void tsweep_body(const float* __restrict__ uin, float* __restrict__ uout,
                                            const float* __restrict__ b, const float* __restrict__ gt0,
                                            const Geo& g, const TGeo& tg, int q, int rx0, int ry0,
                                            int z0, int z1, unsigned char* smem);

__global__ void __launch_bounds__(TSweepGeom::NT, 1)
    gs_tsweep_k(const float* __restrict__ uin, float* __restrict__ uout, const float* __restrict__ b,
                const float* __restrict__ gt0, Geo g, TGeo tg, int zc, int ntx, int nty, int zbase,
                int zstride) {
  using G = TSweepGeom;
  extern __shared__ __align__(16) unsigned char tsweep_smem[];
  int bid = blockIdx.x;
  {  // XCD-aware remap: the tiles of one chunk share an XCD's L2 (as gs_fused3_k)
    const int nb = gridDim.x, qq = nb >> 3, r = nb & 7, xcd = bid & 7, idx = bid >> 3;
    bid = (xcd < r ? xcd * (qq + 1) : r * (qq + 1) + (xcd - r) * qq) + idx;
  }
  const int tiles = ntx * nty;
  const int chunk = bid / tiles;
  const int tile = bid - chunk * tiles;
  const int tyi = tile / ntx;
  const int txi = tile - tyi * ntx;
  const int rx0 = txi * G::TX - G::H;
  const int ry0 = tyi * G::TY - G::H;
  const int p0 = zbase + chunk * zstride;
  const int p1 = min(p0 + zc, g.nz);
  const int tid = threadIdx.x;
  if (tid < G::CT)
    tsweep_body<0>(uin, uout, b, gt0, g, tg, tid, rx0, ry0, p0, p1, tsweep_smem);
  else
    tsweep_body<1>(uin, uout, b, gt0, g, tg, tid - G::CT, rx0, ry0, p0, p1, tsweep_smem);
}

template <int CLS>
__device__ __forceinline__ void tsweep_body(const float* __restrict__ uin, float* __restrict__ uout,
                                            const float* __restrict__ b, const float* __restrict__ gt0,
                                            const Geo& g, const TGeo& tg, int q, int rx0, int ry0,
                                            int z0, int z1, unsigned char* smem) {
  using G = TSweepGeom;
  constexpr int NC = 4;
  constexpr int H = G::H, RX = G::RX, RY = G::RY, HALF = G::HALF, PITCH = G::PITCH;
  constexpr int NP = G::NP, RROW = G::RROW, RBUF = G::RBUF, CSEG = G::CSEG, HSEG = G::HSEG;
  constexpr uint32_t TS = 4;
  constexpr int U = 8;  // steps per unrolled loop body: records of plane m sit in rec[(m - kbeg) % 8]
  // LDS: two tensor buffers, then the u ring (over-reads past a buffer's last row land in the
  // ring, never outside the allocation)
  unsigned char* const tbuf = smem;
  float* const ring = reinterpret_cast<float*>(smem + 2 * RBUF);

  const int nx = g.nx, ny = g.ny, sy = (int)g.sy;
  const bool has = q < G::ND;
  const int dx = has ? q % G::DX : 0;
  const int j0 = 2 * (has ? q / G::DX : 0);  // region rows j0, j0 + 1
  const int li = 2 * dx + CLS;               // region column
  const int gi = rx0 + li;
  // tile region keeps >= 2 points from every x / y face: no mirrored sources, no ghost images
  const bool interior = rx0 >= 2 && rx0 + RX <= nx - 2 && ry0 >= 2 && ry0 + RY <= ny - 2;
  auto mirror = [](int v, int n) { return v < 0 ? min(-v, n - 1) : (v >= n ? max(2 * (n - 1) - v, 0) : v); };

  // u / b source offsets of the two points (mirrored outside the domain: in bounds, the values
  // the reference's mirror images), u ring offset of point 0 (point 1: + PITCH), outputs
  uint32_t usrc[2];
  int oglb[2];
  const int uoff0 = j0 * PITCH + CLS * HALF + dx;
#pragma unroll
  for (int oy = 0; oy < 2; ++oy) {
    const int lj = j0 + oy, gj = ry0 + lj;
    const int gim = interior ? gi : mirror(gi, nx), gjm = interior ? gj : mirror(gj, ny);
    usrc[oy] = (uint32_t)(gjm * sy + gim) * TS;
    const bool out = has && li >= H && li < H + G::TX && lj >= H && lj < H + G::TY && gi < nx && gj < ny;
    oglb[oy] = out ? (int)((gj * sy + gi) * TS) : -1;
  }
  // per (plane parity P, point oy): whether the point is updated by its instance (inside the
  // instance's shrunk region and the domain); face-image bits for the ring
  uint32_t vmask = 0, gmask = 0;
#pragma unroll
  for (int P = 0; P < 2; ++P)
#pragma unroll
    for (int oy = 0; oy < 2; ++oy) {
      const int c = (CLS ^ P) | ((oy ^ P) << 1);
      const int lj = j0 + oy, gj = ry0 + lj;
      const bool ok = has && li >= c + 1 && li < RX - c - 1 && lj >= c + 1 && lj < RY - c - 1 && gi >= 0 &&
                      gi < nx && gj >= 0 && gj < ny;
      const int bit = P * 2 + oy;
      vmask |= (ok ? 1u : 0u) << bit;
      const uint32_t gb = (ok && gi == 1 ? 1u : 0u) | (ok && gi == nx - 2 ? 2u : 0u) |
                          (ok && gj == 1 ? 4u : 0u) | (ok && gj == ny - 2 ? 8u : 0u);
      gmask |= gb << (4 * bit);
    }
  // tensor buffer offset (bytes) of point 0 in component segment 0's own half
  const int boff = j0 * RROW + CLS * HSEG + dx * 4;

  const int zlo = g.zlo_ghost ? -GHOST : 0;
  const int zhi = g.zhi_ghost ? g.nz + GHOST : g.nz;
  const int ulo = g.zlo_ghost ? -(GHOST - 1) : 0;
  const int uhi = g.zhi_ghost ? g.nz + GHOST - 1 : g.nz;
  const int zpar = g.zoff;
  // first step with (k + zpar) even, last step
  const int kbeg = (z0 - (NC - 1)) - ((z0 - (NC - 1) + zpar) & 1);
  const int kend = z1 + NC - 2;
  auto plane_ok = [&](int m) { return m >= zlo && m < zhi; };
  auto clampz = [&](int m) { return min(max(m, zlo), zhi - 1); };
  // the tensor array has all GHOST planes (the z-face ghosts sit in the first of them)
  auto clampt = [&](int m) { return min(max(m, -GHOST), g.nz + GHOST - 1); };
  auto stage_on = [&](int c, int m) {
    const int h = NC - 1 - c;
    return m >= z0 - h && m < z1 + h && m >= ulo && m < uhi;
  };
  auto uslot = [](int m) { return (m + NP * 1024) % NP; };

  // ---- global -> LDS copy of plane m's tensor region into buffer tb: row r by wave (r mod 14);
  // lane l < 60 moves 16 B of component l / 10, half (l % 10) / 5
  const int wave = __builtin_amdgcn_readfirstlane((CLS * G::CT + q) >> 6);
  const int lane = (CLS * G::CT + q) & 63;
  const uint32_t tsrc = (uint32_t)(((int64_t)(ry0 + G::PAD) * tg.trow + (lane / 10) * tg.tpitch +
                                    ((lane % 10) / 5) * (tg.tpitch / 2) + (rx0 + G::PAD) / 2) * 4 +
                                   (lane % 5) * 16);
  auto tload = [&](int m, int tb) {
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(gt0 + (int64_t)clampt(m) * tg.tplane);
    auto* dst = tbuf + tb * RBUF;
    if (lane < 60) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int r = wave + 14 * t;
        if (r < RY)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rs, (__attribute__((address_space(3))) void*)(dst + r * RROW), 16,
              tsrc + (uint32_t)(r * tg.trow * 4), 0, 0, 0);
      }
    }
  };
  float uv[2];
  auto uload = [&](int m) {
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(uin + (int64_t)clampz(m) * g.sz);
#pragma unroll
    for (int oy = 0; oy < 2; ++oy) uv[oy] = buf_load<float>(rs, usrc[oy], 0u);
  };
  auto uput = [&](int m) {
    float* P = ring + uslot(m) * G::UPLANE;
    if (has) {
#pragma unroll
      for (int oy = 0; oy < 2; ++oy) P[uoff0 + oy * PITCH] = uv[oy];
    }
  };
  float bv[2];
  auto bload = [&](int m) {
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(b + (int64_t)clampz(m) * g.sz);
#pragma unroll
    for (int oy = 0; oy < 2; ++oy) bv[oy] = buf_load<float>(rs, usrc[oy], 0u);
  };

  struct Rec {
    Coefs<float> q;
    float b;
  };
  Rec rec[U][2];   // records of plane m in rec[(m - kbeg) % U][oy]
  float zk[2][3];  // a_z e_xz e_yz of the previous plane (own points)
  auto ld = [&](const unsigned char* p, int o) { return *reinterpret_cast<const float*>(p + o); };

  // records of plane m from buffer tb (and tb ^ 1 = plane m+1); z differences against zk, which
  // then takes plane m's z components
  auto form = [&](int tb, Rec (&out)[2]) {
#pragma clang fp contract(off)
    const unsigned char* B0 = tbuf + tb * RBUF + boff;
    const unsigned char* B1 = tbuf + (tb ^ 1) * RBUF + boff;
    // other half: x neighbours at index dx - 1 + CLS (left) and dx + CLS (right)
    const unsigned char* BX = tbuf + tb * RBUF + j0 * RROW + (CLS ^ 1) * HSEG + (dx - 1 + CLS) * 4;
    float own[2][6];
#pragma unroll
    for (int oy = 0; oy < 2; ++oy)
#pragma unroll
      for (int c = 0; c < 6; ++c) own[oy][c] = ld(B0, oy * RROW + c * CSEG);
#pragma unroll
    for (int oy = 0; oy < 2; ++oy) {
      // x: [a_x e_xy e_xz] left / right
      const float xax = ld(BX, oy * RROW + 4) - ld(BX, oy * RROW);
      const float xexy = ld(BX, oy * RROW + 3 * CSEG + 4) - ld(BX, oy * RROW + 3 * CSEG);
      const float xexz = ld(BX, oy * RROW + 4 * CSEG + 4) - ld(BX, oy * RROW + 4 * CSEG);
      // y: [a_y e_xy e_yz] of the rows above / below (the other point of the domino is one)
      const int ro = oy == 0 ? -RROW : 2 * RROW;  // the row outside the domino
      const float yp_a = oy == 0 ? own[1][1] : ld(B0, ro + 1 * CSEG);
      const float ym_a = oy == 0 ? ld(B0, ro + 1 * CSEG) : own[0][1];
      const float yp_xy = oy == 0 ? own[1][3] : ld(B0, ro + 3 * CSEG);
      const float ym_xy = oy == 0 ? ld(B0, ro + 3 * CSEG) : own[0][3];
      const float yp_yz = oy == 0 ? own[1][5] : ld(B0, ro + 5 * CSEG);
      const float ym_yz = oy == 0 ? ld(B0, ro + 5 * CSEG) : own[0][5];
      // z: [a_z e_xz e_yz] of plane m+1 (buffer) and m-1 (zk)
      const float zpa = ld(B1, oy * RROW + 2 * CSEG), zpxz = ld(B1, oy * RROW + 4 * CSEG),
                  zpyz = ld(B1, oy * RROW + 5 * CSEG);
      const float dyay = yp_a - ym_a;
      const float dzaz = zpa - zk[oy][0];
      const float dyexy = yp_xy - ym_xy;
      const float dzexz = zpxz - zk[oy][1];
      const float dyeyz = yp_yz - ym_yz;
      const float dzeyz = zpyz - zk[oy][2];
      Rec& R = out[oy];
      R.q.ax = own[oy][0];
      R.q.ay = own[oy][1];
      R.q.az = own[oy][2];
      R.q.exy = own[oy][3];
      R.q.exz = own[oy][4];
      R.q.eyz = own[oy][5];
      g_combine<float, 3, KFULL>(xax, dyay, dzaz, xexy, dyexy, xexz, dzexz, dyeyz, dzeyz, R.q.gx, R.q.gy,
                                 R.q.gz);
      R.b = bv[oy];
      // materialise g here: left to itself the compiler sinks g_combine into the instances that
      // use it (they are conditional), which keeps the nine differences' operands alive for up
      // to four steps instead of three values
      asm volatile("" : "+v"(R.q.gx), "+v"(R.q.gy), "+v"(R.q.gz));
      zk[oy][0] = own[oy][2];
      zk[oy][1] = own[oy][4];
      zk[oy][2] = own[oy][5];
    }
  };

  // instance (c, k): colour c on plane m = k - c (parity P), the class's point oy
  auto stage = [&](int c, int k, int P, int oy, const Rec& R) {
    const int m = k - c;
    const int bit = P * 2 + oy;
    if (!stage_on(c, m)) return;
    const int zm = (m == 0 && !g.zlo_ghost) ? 1 : m - 1;
    const int zp = (m == g.nz - 1 && !g.zhi_ghost) ? g.nz - 2 : m + 1;
    float* A0 = ring + uslot(m) * G::UPLANE + uoff0 + oy * PITCH;
    const float* Am = ring + uslot(zm) * G::UPLANE + uoff0 + oy * PITCH;
    const float* Ap = ring + uslot(zp) * G::UPLANE + uoff0 + oy * PITCH;
    const int ox_p = CLS ? 1 - HALF : HALF;
    const int ox_m = CLS ? -HALF : HALF - 1;
    float nb[18];
    nb[0] = A0[ox_p];
    nb[1] = A0[ox_m];
    nb[2] = A0[PITCH];
    nb[3] = A0[-PITCH];
    nb[4] = Ap[0];
    nb[5] = Am[0];
    nb[6] = A0[ox_p + PITCH];
    nb[7] = A0[ox_p - PITCH];
    nb[8] = A0[ox_m + PITCH];
    nb[9] = A0[ox_m - PITCH];
    nb[10] = Ap[ox_p];
    nb[11] = Am[ox_p];
    nb[12] = Ap[ox_m];
    nb[13] = Am[ox_m];
    nb[14] = Ap[PITCH];
    nb[15] = Am[PITCH];
    nb[16] = Ap[-PITCH];
    nb[17] = Am[-PITCH];
    float D, S;
    stencil_combine<float, 3, KFULL>(R.q, nb, D, S);
    const float v = gs_update(R.b, S, D);
    if ((vmask >> bit) & 1u) {
      *A0 = v;
      if (!interior) {
        const uint32_t gb = (gmask >> (4 * bit)) & 15u;
        if (gb) {
          // mirror images u~(-1) = u(1), u~(n) = u(n-2): same half row +-1 (x), +-2 rows (y)
          const int xs[3] = {0, (gb & 1u) ? -1 : 0, (gb & 2u) ? 1 : 0};
          const int ys[3] = {0, (gb & 4u) ? -2 * PITCH : 0, (gb & 8u) ? 2 * PITCH : 0};
#pragma unroll
          for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int bq = 0; bq < 3; ++bq) {
              if ((a == 0 && bq == 0) || (a > 0 && xs[a] == 0) || (bq > 0 && ys[bq] == 0)) continue;
              A0[xs[a] + ys[bq]] = v;
            }
        }
      }
    }
  };
  // instance (c, kk) where the unrolled position of step kk is uk (kk - kbeg = uk mod U): the
  // class runs it iff its points carry colour c on that plane (class = plane parity of kk)
  auto instance = [&](int c, int kk, int uk) {
    const int Pk = uk & 1;        // parity of plane kk
    if (Pk != CLS) return;        // compile-time: the other class's step
    const int P = Pk ^ (c & 1);   // parity of plane kk - c
    const int oy = ((c >> 1) ^ P) & 1;
    stage(c, kk, P, oy, rec[(uk - c + 2 * U) % U][oy]);
  };

  // ---- prologue: u planes kbeg-1, kbeg in the ring, kbeg+1 in registers; tensor planes kbeg,
  // kbeg+1 in buffers 0, 1, the z components of plane kbeg-1 in zk; b of plane kbeg
  for (int m = kbeg - 1; m <= kbeg; ++m)
    if (plane_ok(m)) {
      uload(m);
      uput(m);
    }
  uload(kbeg + 1);
  tload(kbeg, 0);
  tload(kbeg + 1, 1);
  {
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(gt0 + (int64_t)clampt(kbeg - 1) * tg.tplane);
#pragma unroll
    for (int oy = 0; oy < 2; ++oy) {
      const uint32_t o = (uint32_t)(((int64_t)(ry0 + j0 + oy + G::PAD) * tg.trow + CLS * (tg.tpitch / 2) +
                                     (rx0 + G::PAD) / 2 + dx) * 4);
      zk[oy][0] = buf_load<float>(rs, o + (uint32_t)(2 * tg.tpitch * 4), 0u);
      zk[oy][1] = buf_load<float>(rs, o + (uint32_t)(4 * tg.tpitch * 4), 0u);
      zk[oy][2] = buf_load<float>(rs, o + (uint32_t)(5 * tg.tpitch * 4), 0u);
    }
  }
  bload(kbeg);
#pragma unroll
  for (int a = 0; a < U; ++a)
#pragma unroll
    for (int oy = 0; oy < 2; ++oy) {
      rec[a][oy].q = Coefs<float>{};
      rec[a][oy].b = 0.f;
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tsweep_barrier();

  // iteration k: gap (the store of plane k-5, u plane k+1 into the ring, records of plane k,
  // next u / b loads), phase 2k: (0, k) and (2, k-1); phase 2k+1: (1, k) and (3, k-1), then the
  // loads land.  Instances of steps past kend or before the chunk are off (stage_on); k runs to
  // kend + 1 for (2, kend) and (3, kend), and to kend + 3 for the store of the last plane.
  for (int k0 = kbeg; k0 <= kend + 3; k0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u;
      asm volatile("" : "+v"(vmask), "+v"(gmask));
      // gap: first the store of the output plane k-5 (final since (3, k-2) in phase 2k-1; its
      // ring slot is rewritten by the next gap's put), so it is done long before the wait at the
      // end of the step
      {
        const int mo = k - 5;
        if (mo >= z0 && mo < z1) {
          const float* Pl = ring + uslot(mo) * G::UPLANE;
          const __amdgpu_buffer_rsrc_t ro = buf_rsrc(uout + (int64_t)mo * g.sz);
#pragma unroll
          for (int oy = 0; oy < 2; ++oy)
            if (oglb[oy] >= 0) buf_store<float>(Pl[uoff0 + oy * PITCH], ro, (uint32_t)oglb[oy]);
        }
      }
      if (plane_ok(k + 1)) uput(k + 1);
#ifndef TSW_PROBE_NO_FORM
      form(u & 1, rec[u]);
#endif
#ifndef TSW_PROBE_NO_ULOAD
      uload(k + 2);
      bload(k + 1);
#endif
      tsweep_barrier();
      // phase 2k; tensor plane k+2 into the buffer plane k leaves (everyone formed plane k)
#ifndef TSW_PROBE_NO_TLOAD  // measurement builds only (tools/probe_tsweep.sh)
      tload(k + 2, u & 1);
#endif
#ifndef TSW_PROBE_NO_STAGE
      instance(0, k, u);
      instance(2, k - 1, (u + U - 1) % U);
#endif
      tsweep_barrier();
      // phase 2k+1
#ifndef TSW_PROBE_NO_STAGE
      instance(1, k, u);
      instance(3, k - 1, (u + U - 1) % U);
#endif
      // this iteration's loads (and the stores, issued three phases ago) have landed
#ifndef TSW_PROBE_NO_WAIT
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      tsweep_barrier();
    }
  }
}

}  // namespace mad
