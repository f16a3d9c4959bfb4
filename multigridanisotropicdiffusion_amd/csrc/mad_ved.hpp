// mad_ved.hpp -- host driver + C ABI of include/mad_ved.h (VED pipeline on the GPU).
// Included at the end of mad_solver.hip: it drives the MAD solver through its
// internal entry points (the same ones mad_run uses), no host round trips between
// the tensor generation and the diffusion step.
//
// Reference: include/itkVEDMultigridImageFilter.{h,hxx} (VED.h / VED.hxx).
#include "../../include/mad_ved.h"
#include "mad_ved_kernels.hpp"
#include <type_traits>

struct mad_ved_ctx {
  mad_ved_desc d{};
  std::string err;
  mad_ctx* mad = nullptr;  // the DiffusionStep filter (VED.hxx:386-398), kept across iterations
  int64_t n[3] = {0, 0, 0};
  int64_t N = 0;
  double* img = nullptr;   // internal image (fp64, VED.h:61)
  double* img2 = nullptr;  // next iterate
  void* fir = nullptr;     // 9 FIR volumes in the storage precision
  double* iir = nullptr;   // 12 volumes (T) of the recursive Hessian passes
  void* taps = nullptr;    // per-axis taps of the current scale (device)
  double* resp = nullptr;  // m_MaxVesselnessResponse
  double* dir = nullptr;   // vessel direction (eigenvector column 2 of the max scale), SoA x3
  void* stage = nullptr;   // host <-> device staging
  size_t stage_bytes = 0;
  void* xbuf = nullptr;    // send + receive blocks of the partitioned Hessian's transpose
  size_t xbuf_bytes = 0;
  ~mad_ved_ctx() {
    if (mad) (void)hipSetDevice(mad->device);
    if (mad && mad->stream) (void)hipStreamSynchronize(mad->stream);
    for (void* p : {(void*)img, (void*)img2, fir, (void*)iir, taps, (void*)resp, (void*)dir, stage, xbuf})
      if (p) (void)hipFree(p);
    if (mad) mad_destroy(mad);
  }
};

namespace {

template <typename F>
int ved_guarded(mad_ved_ctx* v, F&& f) {
  try {
    f();
    return MAD_OK;
  } catch (const MadError& e) {
    g_last_error = e.what();
    if (v) v->err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "out of host memory";
    if (v) v->err = g_last_error;
    return MAD_ERR_NOMEM;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    if (v) v->err = e.what();
    return MAD_ERR_DEVICE;
  }
}

// MAD call inside a VED call: forward its status and message
void mad_call(mad_ctx* c, int rc) {
  if (rc != MAD_OK) throw MadError(rc, "diffusion step: " + c->err);
}

// Gaussian derivative taps for one axis: [K0 | K1 | K2], R = ceil(4 sigma / h)
// (oracle/ved_oracle.py gauss_kernels restates the same definition):
//   K0 = g / S0,  K1 = t g / S2,  K2 = a (t^2 - m) g,  m = S2 / S0,  a = 2 / (S4 - m S2)
int ved_taps(double sigma, double h, std::vector<double>& K) {
  const int R = std::max(1, (int)std::ceil(4.0 * sigma / h));
  const double s = sigma / h;
  const int W = 2 * R + 1;
  std::vector<double> g(W), t(W);
  double S0 = 0.0, S2 = 0.0, S4 = 0.0;
  for (int q = 0; q < W; ++q) {
    t[q] = (double)(q - R);
    g[q] = std::exp(-(t[q] * t[q]) / (2.0 * s * s));
  }
  for (int q = 0; q < W; ++q) {
    S0 += g[q];
    S2 += t[q] * t[q] * g[q];
    S4 += t[q] * t[q] * t[q] * t[q] * g[q];
  }
  const double m = S2 / S0;
  const double a = 2.0 / (S4 - m * S2);
  K.assign(3 * W, 0.0);
  for (int q = 0; q < W; ++q) {
    K[q] = g[q] / S0;
    K[W + q] = t[q] * g[q] / S2;
    K[2 * W + q] = a * (t[q] * t[q] - m) * g[q];
  }
  return R;
}

void* ved_stage(mad_ved_ctx* v, size_t bytes) {
  if (bytes > v->stage_bytes) {
    if (v->stage) HIP_CHECK(hipFree(v->stage));
    v->stage = nullptr;
    HIP_CHECK(hipMalloc(&v->stage, bytes));
    v->stage_bytes = bytes;
  }
  return v->stage;
}

// device image (any dtype) -> v->img (fp64)
void ved_load_image(mad_ved_ctx* v, const void* src, int dt, bool dev) {
  const size_t es = dtype_size(dt);
  REQUIRE(es, MAD_ERR_INVALID, "bad image dtype");
  hipStream_t st = v->mad->stream;
  if (!dev) {
    void* s = ved_stage(v, es * v->N);
    HIP_CHECK(hipMemcpyAsync(s, src, es * v->N, hipMemcpyHostToDevice, st));
    src = s;
  }
  convert_to<double>(src, dt, v->img, v->N, st);
}

constexpr size_t kVedLds = 128 * 1024;  // dynamic LDS cap of the FIR tiles

// allow the FIR kernels more than the default 64 KiB of dynamic LDS (once per type)
template <typename T>
void ved_lds_attr() {
  static bool done = false;
  if (done) return;
  for (const void* k : {(const void*)ved_fir_z_k<T>, (const void*)ved_fir_y_k<T>,
                        (const void*)ved_fir_x_k<T, VED_HESSIAN>, (const void*)ved_fir_x_k<T, VED_UPDATE>})
    HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kVedLds));
  done = true;
}

// ITK RecursiveGaussianImageFilter coefficients of one axis / order, sigma sd in voxels
// (restates oracle/ved_oracle.py recursive_coefficients, same formulas and order)
IirCoef ved_iir_coef(double sd, int order) {
  const double A1[3] = {1.3530, -0.6724, -1.3563}, B1[3] = {1.8151, -3.4327, 5.2318};
  const double W1 = 0.6681, L1 = -1.3932;
  const double A2[3] = {-0.3531, 0.6724, 0.3446}, B2[3] = {0.0902, 0.6100, -2.2355};
  const double W2 = 2.0787, L2 = -1.3732;
  auto ncoef = [&](int o, double N[4], double& SN, double& DN, double& EN) {
    const double a1 = A1[o], b1 = B1[o], a2 = A2[o], b2 = B2[o];
    const double s1 = std::sin(W1 / sd), s2 = std::sin(W2 / sd);
    const double c1 = std::cos(W1 / sd), c2 = std::cos(W2 / sd);
    const double e1 = std::exp(L1 / sd), e2 = std::exp(L2 / sd);
    N[0] = a1 + a2;
    N[1] = e2 * (b2 * s2 - (a2 + 2 * a1) * c2);
    N[1] += e1 * (b1 * s1 - (a1 + 2 * a2) * c1);
    N[2] = (a1 + a2) * c2 * c1;
    N[2] -= b1 * c2 * s1 + b2 * c1 * s2;
    N[2] *= 2 * e1 * e2;
    N[2] += a2 * e1 * e1 + a1 * e2 * e2;
    N[3] = e2 * e1 * e1 * (b2 * s2 - a2 * c2);
    N[3] += e1 * e2 * e2 * (b1 * s1 - a1 * c1);
    SN = N[0] + N[1] + N[2] + N[3];
    DN = N[1] + 2 * N[2] + 3 * N[3];
    EN = N[1] + 4 * N[2] + 9 * N[3];
  };
  IirCoef C{};
  double* D = C.d;
  {
    const double c1 = std::cos(W1 / sd), c2 = std::cos(W2 / sd);
    const double e1 = std::exp(L1 / sd), e2 = std::exp(L2 / sd);
    D[3] = e1 * e1 * e2 * e2;
    D[2] = -2 * c1 * e1 * e2 * e2;
    D[2] += -2 * c2 * e2 * e1 * e1;
    D[1] = 4 * c2 * c1 * e1 * e2;
    D[1] += e1 * e1 + e2 * e2;
    D[0] = -2 * (e2 * c2 + e1 * c1);
  }
  const double SD = 1.0 + D[0] + D[1] + D[2] + D[3];
  const double DD = D[0] + 2 * D[1] + 3 * D[2] + 4 * D[3];
  const double ED = D[0] + 4 * D[1] + 9 * D[2] + 16 * D[3];
  double* N = C.n;
  bool symmetric = true;
  if (order == 0) {
    double SN, DN, EN;
    ncoef(0, N, SN, DN, EN);
    const double alpha = 2 * SN / SD - N[0];
    for (int q = 0; q < 4; ++q) N[q] = N[q] / alpha;
  } else if (order == 1) {
    double SN, DN, EN;
    ncoef(1, N, SN, DN, EN);
    const double alpha = 2 * (SN * DD - DN * SD) / (SD * SD);
    for (int q = 0; q < 4; ++q) N[q] = N[q] / alpha;
    symmetric = false;
  } else {
    double N0[4], N2[4], SN0, DN0, EN0, SN2, DN2, EN2;
    ncoef(0, N0, SN0, DN0, EN0);
    ncoef(2, N2, SN2, DN2, EN2);
    const double beta = -(2 * SN2 - SD * N2[0]) / (2 * SN0 - SD * N0[0]);
    double abcd[4];
    for (int q = 0; q < 4; ++q) abcd[q] = N2[q] + beta * N0[q];
    const double SN = abcd[0] + abcd[1] + abcd[2] + abcd[3];
    const double DN = abcd[1] + 2 * abcd[2] + 3 * abcd[3];
    const double EN = abcd[1] + 4 * abcd[2] + 9 * abcd[3];
    double alpha = EN * SD * SD - ED * SN * SD - 2 * DN * DD * SD + 2 * DD * DD * SN;
    alpha /= SD * SD * SD;
    for (int q = 0; q < 4; ++q) N[q] = abcd[q] / alpha;
  }
  double* M = C.m;
  if (symmetric) {
    M[0] = N[1] - D[0] * N[0];
    M[1] = N[2] - D[1] * N[0];
    M[2] = N[3] - D[2] * N[0];
    M[3] = -D[3] * N[0];
  } else {
    M[0] = -(N[1] - D[0] * N[0]);
    M[1] = -(N[2] - D[1] * N[0]);
    M[2] = -(N[3] - D[2] * N[0]);
    M[3] = D[3] * N[0];
  }
  const double SNn = N[0] + N[1] + N[2] + N[3];
  const double SM = M[0] + M[1] + M[2] + M[3];
  const double SDn = 1.0 + D[0] + D[1] + D[2] + D[3];
  for (int q = 0; q < 4; ++q) {
    C.bn[q] = D[q] * SNn / SDn;
    C.bm[q] = D[q] * SM / SDn;
  }
  return C;
}

// one scale with the recursive (IIR) operator: z pass (image -> orders 0..2), y pass (-> the
// six (y, z) order pairs), x pass (-> the six scaled Hessian components), then the Hessian
// out (VED_HESSIAN) or UpdateVesselness (VED_UPDATE) per voxel.
// Partitioned (dist: a z-slab rank of the VED run): every z line lies in one x column, every
// y and x line in one z plane, so rank r runs the z pass on its x range [xa_r, xb_r) (all
// planes), the three z-pass volumes are transposed -- rank r sends each rank q the block [q's
// tensor planes] x [all y] x [xa_r, xb_r) (Comm::exchange_blocks) -- and the y pass, the x pass
// and the vesselness update run on the rank's tensor planes only (its slab + the TENSOR_GHOST
// planes the solver's tensor slab holds).  Each line sees the same values through the same
// expressions, so the tensor equals the one-GPU tensor bit for bit, at 1 / P of the passes'
// work plus the transpose.
template <typename T>
void ved_scale_iir(mad_ved_ctx* v, double sigma, int mode, bool first, double* hess, bool dist = false) {
  hipStream_t st = v->mad->stream;
  const int nx = (int)v->n[0], ny = (int)v->n[1], nz = (int)v->n[2];
  REQUIRE(nx >= 4 && ny >= 4 && nz >= 4, MAD_ERR_UNSUPPORTED,
          "the recursive Gaussian needs at least 4 points along each axis");
  const int64_t N = v->N;
  if (!v->iir) HIP_CHECK(big_alloc((void**)&v->iir, sizeof(double) * 12 * N));
  // volumes between the passes in T: fp64 in the fp64 mode; fp32 in the fp32 mode (the
  // passes' arithmetic stays fp64; half the bytes of the memory-bound passes)
  T* base = reinterpret_cast<T*>(v->iir);
  // slots: Z 0..2, pairs A 6..11, Hessian 0..5 (over the dead Z: one SoA block)
  T* Z[3] = {base, base + N, base + 2 * N};
  T* A[6];
  T* H[6];
  for (int q = 0; q < 6; ++q) {
    A[q] = base + (6 + q) * N;
    H[q] = base + q * N;
  }
  const double* h = v->d.spacing;
  // MAD_VED_OPT_LINE_WALK (the parity reference): ved_iir_k's one thread per line for every
  // axis, each output marched on its own (whole grid: not partitioned)
  const bool line_walk = (v->d.options & MAD_VED_OPT_LINE_WALK) != 0;
  mad_ctx* c = v->mad;
  dist = dist && !line_walk && c->comm.active() && c->d.nranks > 1;
  const int P_ = dist ? c->d.nranks : 1, me = dist ? c->comm.rank() : 0;
  auto xr = [&](int r) { return std::make_pair((int)((int64_t)nx * r / P_), (int)((int64_t)nx * (r + 1) / P_)); };
  auto tplanes = [&](int r) {  // the tensor planes of rank r (compute_geometry's tensor slab)
    if (!dist) return std::make_pair(0, nz);
    const int per = nz / P_;
    return std::make_pair(std::max(per * r - TENSOR_GHOST, 0), std::min(per * (r + 1) + TENSOR_GHOST, nz));
  };
  const int xa = xr(me).first, nxr = xr(me).second - xr(me).first;
  // SI: the z pass reads the fp64 image, the others the T volumes
  auto launch = [&](const IirPass& P, int axis, auto si) {
    using SI = decltype(si);
    const int64_t lines = axis == 0 ? (int64_t)ny * nz : axis == 1 ? (int64_t)nx * nz : (int64_t)nx * ny;
    if (line_walk) {
      hipLaunchKernelGGL((ved_iir_k<SI, T>), dim3((unsigned)((lines + 255) / 256)), dim3(256), 0, st, P, axis,
                         nx, ny, nz);
    } else if (axis == 0) {
      // contiguous lines: one wave per 64 lines and output, LDS-staged row chunks
      // chunk rows of one 128-B line (3.76 vs 4.15 ms per 512^3 fp32 pass with 64 B)
      if constexpr (std::is_same<SI, T>::value) {
        const dim3 gr((unsigned)((lines + 63) / 64), (unsigned)P.nout);
        const int64_t lb = (int64_t)tplanes(me).first * ny, le = (int64_t)tplanes(me).second * ny;
        const dim3 grl((unsigned)((le - lb + 63) / 64), (unsigned)P.nout);
        (void)gr;
        hipLaunchKernelGGL((ved_iir_x_k<SI, T, 128 / (int)sizeof(T)>), grl, dim3(64), 0, st, P, nx, lb, le);
      }
    } else {
      // strided lines: the outputs sharing an input in one march, one launch per input; when
      // partitioned, the z pass on the rank's x range (all y), the y pass on its tensor planes
      // (all x)
      const int lxa = (axis == 2) ? xa : 0, lnx = (axis == 2) ? nxr : nx;
      const int lza = (axis == 1) ? tplanes(me).first : 0;
      const int lnz = (axis == 1) ? tplanes(me).second - tplanes(me).first : nz;
      const int64_t xl = (int64_t)lnx * (axis == 1 ? lnz : ny);
      const unsigned nb = (unsigned)((xl + 255) / 256);
      bool done[6] = {false, false, false, false, false, false};
      for (int o = 0; o < P.nout; ++o) {
        if (done[o]) continue;
        int outs[3], k = 0;
        for (int o2 = o; o2 < P.nout && k < 3; ++o2)
          if (!done[o2] && P.src[o2] == P.src[o]) {
            outs[k++] = o2;
            done[o2] = true;
          }
        auto go = [&](auto KC) {
          constexpr int K = decltype(KC)::value;
          IirGroup<K> G{};
          G.in = P.in[P.src[o]];
          for (int q = 0; q < K; ++q) {
            G.out[q] = P.out[outs[q]];
            G.c[q] = P.c[outs[q]];
            G.scale[q] = P.scale[outs[q]];
          }
          // two load blocks in flight per line (512^3 tensor generation 65.0 -> 56.3 ms on one GPU,
          // profiles/r03_ved_pipe_ab.log; the partitioned passes' few lines per GPU need it most)
          hipLaunchKernelGGL((ved_iir_grp_k<SI, T, K, 8, true>), dim3(nb), dim3(256), 0, st, G, axis, nx, ny, nz,
                             lxa, lnx, lza, lnz);
        };
        if (k == 3) go(std::integral_constant<int, 3>{});
        else if (k == 2) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 1>{});
      }
    }
    HIP_CHECK(hipGetLastError());
  };
  IirPass P{};
  // z: image -> Z_o, o = 0, 1, 2
  P.in[0] = v->img;
  P.nout = 3;
  for (int o = 0; o < 3; ++o) {
    P.out[o] = Z[o];
    P.src[o] = 0;
    P.c[o] = ved_iir_coef(sigma / h[2], o);
    P.scale[o] = 1.0;
  }
  launch(P, 2, double{});
  if (dist) {
    // transpose the three z-pass volumes: the rank's x range (all planes) -> its tensor planes
    // (all x); every y and x line then lies in the rank's planes
    std::vector<const void*> sp(P_, nullptr);
    std::vector<void*> rp(P_, nullptr);
    std::vector<size_t> sb(P_, 0), rb(P_, 0);
    const auto mp = tplanes(me);
    size_t tot = 0;
    for (int r = 0; r < P_; ++r) {
      if (r == me) continue;
      const auto tp = tplanes(r);
      sb[r] = sizeof(T) * 3 * (size_t)(tp.second - tp.first) * ny * nxr;
      rb[r] = sizeof(T) * 3 * (size_t)(mp.second - mp.first) * ny * (xr(r).second - xr(r).first);
      tot += sb[r] + rb[r];
    }
    if (tot > v->xbuf_bytes) {
      if (v->xbuf) HIP_CHECK(hipFree(v->xbuf));
      v->xbuf = nullptr;
      HIP_CHECK(big_alloc((void**)&v->xbuf, tot));
      v->xbuf_bytes = tot;
    }
    Vol6<T> Z3{};
    for (int q = 0; q < 3; ++q) Z3.v[q] = Z[q];
    char* cur = (char*)v->xbuf;
    for (int r = 0; r < P_; ++r) {
      if (r == me) continue;
      sp[r] = cur;
      cur += sb[r];
      rp[r] = cur;
      cur += rb[r];
      const auto tp = tplanes(r);
      const int nzb = tp.second - tp.first;
      // ved_block_k indexes a block with 32-bit offsets
      REQUIRE(3 * (int64_t)nzb * ny * nxr < ((int64_t)1 << 31), MAD_ERR_UNSUPPORTED,
              "VED transpose block exceeds 2^31 elements (use more ranks)");
      hipLaunchKernelGGL((ved_block_k<T, false>), dim3(flat_blocks(3 * (int64_t)nzb * ny * nxr)), dim3(256), 0, st,
                         Z3, (T*)sp[r], nx, ny, xa, nxr, tp.first, nzb, 3);
    }
    HIP_CHECK(hipGetLastError());
    c->comm.exchange_blocks(sp, sb, rp, rb, st);
    const int nzm = mp.second - mp.first;
    for (int q = 0; q < P_; ++q) {
      if (q == me) continue;
      const int qa = xr(q).first, qn = xr(q).second - xr(q).first;
      REQUIRE(3 * (int64_t)nzm * ny * qn < ((int64_t)1 << 31), MAD_ERR_UNSUPPORTED,
              "VED transpose block exceeds 2^31 elements (use more ranks)");
      hipLaunchKernelGGL((ved_block_k<T, true>), dim3(flat_blocks(3 * (int64_t)nzm * ny * qn)), dim3(256), 0, st, Z3,
                         (T*)rp[q], nx, ny, qa, qn, mp.first, nzm, 3);
    }
    HIP_CHECK(hipGetLastError());
  }
  // y: (oy, oz) = (0,0) (1,0) (2,0) (0,1) (1,1) (0,2)
  const int pairs[6][2] = {{0, 0}, {1, 0}, {2, 0}, {0, 1}, {1, 1}, {0, 2}};
  P = IirPass{};
  for (int q = 0; q < 3; ++q) P.in[q] = Z[q];
  P.nout = 6;
  for (int q = 0; q < 6; ++q) {
    P.out[q] = A[q];
    P.src[q] = pairs[q][1];
    P.c[q] = ved_iir_coef(sigma / h[1], pairs[q][0]);
    P.scale[q] = 1.0;
  }
  launch(P, 1, T{});
  // x: H = [xx, xy, xz, yy, yz, zz] from (ox, pair) and sigma^2 / (h_i h_j)
  const int xsrc[6] = {0, 1, 3, 2, 4, 5};  // pair index feeding each component
  const int xord[6] = {2, 1, 1, 0, 0, 0};
  const int cd[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
  P = IirPass{};
  for (int q = 0; q < 6; ++q) P.in[q] = A[q];
  P.nout = 6;
  const double s2 = sigma * sigma;
  for (int q = 0; q < 6; ++q) {
    P.out[q] = H[q];
    P.src[q] = xsrc[q];
    P.c[q] = ved_iir_coef(sigma / h[0], xord[q]);
    P.scale[q] = s2 / (h[cd[q][0]] * h[cd[q][1]]);
  }
  launch(P, 0, T{});
  const T* Hs = H[0];
  const VesselParams vp{v->d.alpha, v->d.beta, v->d.gamma};
  const int64_t p0 = (int64_t)tplanes(me).first * nx * ny, p1 = (int64_t)tplanes(me).second * nx * ny;
  const unsigned nb = flat_blocks(p1 - p0);
  if (mode == VED_HESSIAN)
    hipLaunchKernelGGL((ved_hess_k<T, VED_HESSIAN, T>), dim3(nb), dim3(256), 0, st, Hs, N, p0, p1, hess, nullptr,
                       nullptr, 0, vp);
  else
    hipLaunchKernelGGL((ved_hess_k<T, VED_UPDATE, T>), dim3(nb), dim3(256), 0, st, Hs, N, p0, p1, nullptr,
                       v->resp, v->dir, first ? 1 : 0, vp);
  HIP_CHECK(hipGetLastError());
}

// one scale: Hessian (MODE VED_HESSIAN, into `hess`) or vesselness update
template <typename T>
void ved_scale(mad_ved_ctx* v, double sigma, int mode, bool first, double* hess, bool dist = false) {
  if (v->d.hessian == MAD_VED_HESSIAN_RECURSIVE) {
    ved_scale_iir<T>(v, sigma, mode, first, hess, dist);
    return;
  }
  hipStream_t st = v->mad->stream;
  const int nx = (int)v->n[0], ny = (int)v->n[1], nz = (int)v->n[2];
  const int64_t N = v->N;
  if (!v->fir) HIP_CHECK(big_alloc((void**)&v->fir, sizeof(T) * 9 * N));
  T* f = (T*)v->fir;
  T *z0 = f, *z1 = f + N, *z2 = f + 2 * N;
  T *a00 = f + 3 * N, *a10 = f + 4 * N, *a20 = f + 5 * N, *a01 = f + 6 * N, *a11 = f + 7 * N,
    *a02 = f + 8 * N;
  std::vector<double> K[3];
  int R[3];
  for (int q = 0; q < 3; ++q) R[q] = ved_taps(sigma, v->d.spacing[q], K[q]);
  const size_t W[3] = {K[0].size(), K[1].size(), K[2].size()};
  std::vector<T> kt;
  for (int q = 0; q < 3; ++q)
    for (double x : K[q]) kt.push_back((T)x);
  if (v->taps) HIP_CHECK(hipFree(v->taps));
  v->taps = nullptr;
  HIP_CHECK(hipMalloc(&v->taps, sizeof(T) * kt.size()));
  HIP_CHECK(hipMemcpyAsync(v->taps, kt.data(), sizeof(T) * kt.size(), hipMemcpyHostToDevice, st));
  const T* tx = (const T*)v->taps;
  const T* ty = tx + W[0];
  const T* tz = ty + W[1];
  // LDS-staged passes: z tiles of ZT planes, y tiles of YT rows (smaller when the taps
  // are long), x rows of 256
  auto lds_for = [](int lines, int width, int copies) { return (size_t)lines * width * copies * sizeof(T); };
  int ZT = 32, YT = 32;
  while (ZT > 4 && lds_for(ZT + 2 * R[2], 256, 1) > kVedLds) ZT /= 2;
  while (YT > 4 && lds_for(YT + 2 * R[1], 64, 3) > kVedLds) YT /= 2;
  const size_t lz = lds_for(ZT + 2 * R[2], 256, 1), ly = lds_for(YT + 2 * R[1], 64, 3);
  const size_t lx = lds_for(256 + 2 * R[0], 1, 6);
  REQUIRE(lz <= kVedLds && ly <= kVedLds && lx <= kVedLds, MAD_ERR_UNSUPPORTED,
          "Gaussian taps too long for the LDS tiles (sigma / spacing > ~18)");
  ved_lds_attr<T>();
  hipLaunchKernelGGL((ved_fir_z_k<T>), dim3((nx + 63) / 64, (ny + 3) / 4, (nz + ZT - 1) / ZT),
                     dim3(256), lz, st, v->img, z0, z1, z2, tz, R[2], nx, ny, nz, ZT);
  hipLaunchKernelGGL((ved_fir_y_k<T>), dim3((nx + 63) / 64, (ny + YT - 1) / YT, nz), dim3(256), ly,
                     st, z0, z1, z2, a00, a10, a20, a01, a11, a02, ty, R[1], nx, ny, nz, YT);
  const dim3 gr((nx + 255) / 256, ny, nz);
  HessScale hs;
  const double s2 = sigma * sigma, *h = v->d.spacing;
  const int cd[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
  for (int c = 0; c < 6; ++c) hs.f[c] = s2 / (h[cd[c][0]] * h[cd[c][1]]);
  const VesselParams vp{v->d.alpha, v->d.beta, v->d.gamma};
  if (mode == VED_HESSIAN)
    hipLaunchKernelGGL((ved_fir_x_k<T, VED_HESSIAN>), gr, dim3(256), lx, st, a00, a10, a20, a01, a11, a02,
                       tx, R[0], nx, ny, nz, hs, hess, nullptr, nullptr, 0, vp);
  else
    hipLaunchKernelGGL((ved_fir_x_k<T, VED_UPDATE>), gr, dim3(256), lx, st, a00, a10, a20, a01, a11, a02,
                       tx, R[0], nx, ny, nz, hs, nullptr, v->resp, v->dir, first ? 1 : 0, vp);
  HIP_CHECK(hipGetLastError());
  // the host tap vector dies here: the copy must have landed
  HIP_CHECK(hipStreamSynchronize(st));
}

// ComputeHessian + UpdateVesselness over all scales, GenerateDiffusionTensor into the
// solver's fp64 tensor (VED.hxx:109-120)
template <typename T>
void ved_tensor_impl(mad_ved_ctx* v) {
  mad_ctx* c = v->mad;
  const int64_t N = v->N;
  if (!v->resp) HIP_CHECK(big_alloc((void**)&v->resp, sizeof(double) * N));
  if (!v->dir) HIP_CHECK(big_alloc((void**)&v->dir, sizeof(double) * 3 * N));
  // the run's tensor: partitioned across the ranks (recursive Hessian; the FIR operator and
  // the line-walk reference stay whole-grid on every rank)
  for (int s = 0; s < v->d.nscales; ++s) ved_scale<T>(v, v->d.scales[s], VED_UPDATE, s == 0, nullptr, true);
  // the tensor planes this rank's solver stores (its slab + ghost planes; all on one GPU)
  tensor_alloc(c);
  const int64_t sz = v->n[0] * v->n[1];
  const int64_t q0 = c->tensor_lo * sz, q1 = c->tensor_hi * sz;
  hipLaunchKernelGGL(ved_tensor_k, dim3(flat_blocks(q1 - q0)), dim3(256), 0, c->stream, v->resp, v->dir,
                     tensor_at0(c), N, q0, q1, c->tensor_cs, v->d.epsilon, v->d.omega, v->d.sensitivity);
  HIP_CHECK(hipGetLastError());
  c->tensor_set = true;
  c->setup_done = false;  // DiffusionStep builds a new filter per iteration (VED.hxx:386)
}

void ved_tensor_any(mad_ved_ctx* v) {
  if (v->d.precision == MAD_FP64) ved_tensor_impl<double>(v);
  else ved_tensor_impl<float>(v);
}

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

// this rank's z-slab of level 0: [z0, z1) planes, element offset and count
struct VedSlab {
  int64_t off, n;
};
VedSlab ved_slab(const mad_ved_ctx* v) {
  const LevelGeom& G = v->mad->geom[0];
  const int64_t plane = v->n[0] * v->n[1];
  return VedSlab{G.z0 * plane, (G.z1 - G.z0) * plane};
}

// GenerateData (VED.hxx:63-155)
void ved_run_impl(mad_ved_ctx* v, const void* in, int in_dt, void* out, int out_dt, bool dev,
                  mad_ved_stats* st) {
  mad_ctx* c = v->mad;
  HIP_CHECK(hipSetDevice(c->device));
  const size_t oes = dtype_size(out_dt);
  REQUIRE(oes, MAD_ERR_INVALID, "bad output dtype");
  const bool dist = c->comm.active();
  REQUIRE(dist || c->d.nranks == 1, MAD_ERR_STATE, "nranks > 1 needs mad_ved_comm_init first");
  const VedSlab sl = ved_slab(v);
  ved_load_image(v, in, in_dt, dev);
  hipEvent_t ev[4];
  for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
  double tensor_ms = 0.0, diff_ms = 0.0, relres = 0.0;
  unsigned cycles = 0;
  int stalled = 0;
  for (uint32_t it = 0; it < v->d.iterations; ++it) {  // VED.hxx:104
    if (v->d.verbose && c->comm.rank() == 0) std::printf("Iteration n.%u...\n", it + 1);
    HIP_CHECK(hipEventRecord(ev[0], c->stream));
    ved_tensor_any(v);  // whole image, every rank
    HIP_CHECK(hipEventRecord(ev[1], c->stream));
    mad_stats ms{};
    mad_call(c, run_impl(c, v->img + sl.off, MAD_F64, v->img2 + sl.off, MAD_F64, &ms, true));
    if (dist) {
      // the next iteration's Hessian (and the caller) see the whole new image
      c->comm.allgather_slabs(v->img2 + sl.off, v->img, v->n[0] * v->n[1], v->n[2], sizeof(double),
                              c->stream);
    } else {
      std::swap(v->img, v->img2);
    }
    HIP_CHECK(hipEventRecord(ev[2], c->stream));
    HIP_CHECK(hipEventSynchronize(ev[2]));
    tensor_ms += elapsed(ev[0], ev[1]);
    diff_ms += elapsed(ev[1], ev[2]);
    cycles += ms.total_cycles;
    relres = ms.last_relres;
    stalled |= ms.stalled;
  }
  for (auto& e : ev) HIP_CHECK(hipEventDestroy(e));
  // static_cast of this rank's slab to the output pixel type (VED.hxx:139-150)
  void* dst = dev ? out : ved_stage(v, oes * sl.n);
  convert_from<double>(v->img + sl.off, dst, out_dt, sl.n, c->stream);
  if (!dev) HIP_CHECK(hipMemcpyAsync(out, dst, oes * sl.n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->iterations = v->d.iterations;
    st->total_cycles = cycles;
    st->last_relres = relres;
    st->tensor_ms = tensor_ms;
    st->diffusion_ms = diff_ms;
    st->stalled = stalled;
  }
}

}  // namespace

extern "C" {

int mad_ved_desc_init(mad_ved_desc* d) {
  if (!d) return MAD_ERR_INVALID;
  std::memset(d, 0, sizeof(*d));
  d->abi_version = MAD_ABI_VERSION;
  d->size[0] = d->size[1] = d->size[2] = 1;
  d->spacing[0] = d->spacing[1] = d->spacing[2] = 1.0;
  d->alpha = 0.5;        // VED.hxx:36
  d->beta = 0.5;         // :37
  d->gamma = 5.0;        // :38
  d->epsilon = 0.01;     // :39
  d->omega = 5.0;        // :40
  d->sensitivity = 10.0; // :41
  d->iterations = 1;     // :42
  d->diffusion_iterations = 5;  // :43
  d->cycle = MAD_VCYCLE; // :44
  d->time_step = 0.1;    // :45
  d->tolerance = 1e-6;   // :46
  d->diffusion_iterations_per_grid = 2;  // :47
  d->nscales = 5;        // :52-58
  const double sc[5] = {0.300, 0.482, 0.775, 1.245, 2.000};
  for (int q = 0; q < 5; ++q) d->scales[q] = sc[q];
  d->smoother = MAD_GAUSS_SEIDEL;
  d->precision = MAD_PRECISION_AUTO;  // Hessian in fp32; the diffusion solve as mad_create resolves it
  d->device = -1;
  d->nranks = 1;
  d->rank = 0;
  return MAD_OK;
}

int mad_ved_create(const mad_ved_desc* d, mad_ved_ctx** out) {
  if (!out) return MAD_ERR_INVALID;
  *out = nullptr;
  std::unique_ptr<mad_ved_ctx> v(new mad_ved_ctx());
  int rc = ved_guarded(nullptr, [&] {
    REQUIRE(d, MAD_ERR_INVALID, "null descriptor");
    REQUIRE(d->abi_version == MAD_ABI_VERSION, MAD_ERR_INVALID, "ABI version mismatch");
    REQUIRE(d->hessian == MAD_VED_HESSIAN_RECURSIVE || d->hessian == MAD_VED_HESSIAN_FIR,
            MAD_ERR_INVALID, "bad Hessian kind");
    REQUIRE(d->nscales >= 1 && d->nscales <= MAD_VED_MAX_SCALES, MAD_ERR_INVALID,
            "nscales must be 1.." + std::to_string(MAD_VED_MAX_SCALES));
    for (int s = 0; s < d->nscales; ++s)
      REQUIRE(d->scales[s] > 0.0, MAD_ERR_INVALID, "scales must be positive");
    REQUIRE(d->sensitivity != 0.0, MAD_ERR_INVALID, "sensitivity must be nonzero");
    v->d = *d;
    mad_desc md;
    mad_desc_init(&md);
    md.dim = 3;
    for (int q = 0; q < 3; ++q) {
      md.size[q] = d->size[q];
      md.spacing[q] = d->spacing[q];
    }
    md.cycle = d->cycle;
    md.smoother = d->smoother;
    md.iterations_per_grid = d->diffusion_iterations_per_grid;
    md.max_cycles = 100;  // VED.hxx:396
    md.number_of_steps = d->diffusion_iterations;
    md.time_step = d->time_step;
    md.tolerance = d->tolerance;
    md.verbose = d->verbose;
    md.precision = d->precision;
    md.device = d->device;
    md.nranks = d->nranks < 1 ? 1 : d->nranks;
    md.rank = d->rank;
    const int mrc = mad_create(&md, &v->mad);
    if (mrc != MAD_OK) throw MadError(mrc, g_last_error);
    for (int q = 0; q < 3; ++q) v->n[q] = d->size[q];
    v->N = v->n[0] * v->n[1] * v->n[2];
    REQUIRE(v->n[0] <= INT32_MAX && v->n[1] <= 65535 && v->n[2] <= 65535, MAD_ERR_INVALID,
            "image too large for the VED grid mapping");
    HIP_CHECK(hipSetDevice(v->mad->device));
    HIP_CHECK(big_alloc((void**)&v->img, sizeof(double) * v->N));
    HIP_CHECK(big_alloc((void**)&v->img2, sizeof(double) * v->N));
  });
  if (rc != MAD_OK) return rc;
  *out = v.release();
  return MAD_OK;
}

void mad_ved_destroy(mad_ved_ctx* v) { delete v; }

const char* mad_ved_last_error(const mad_ved_ctx* v) { return v ? v->err.c_str() : g_last_error.c_str(); }

// as mad_run: MAD_ERR_NOT_CONVERGED (output written) when a diffusion step stalled above Tolerance
static int ved_run_status(mad_ved_ctx* v, int rc, const mad_ved_stats& st) {
  if (rc != MAD_OK || !st.stalled) return rc;
  char buf[200];
  std::snprintf(buf, sizeof buf,
                "tolerance %g not reached: the stall guard ended a diffusion step at relres %g (the "
                "storage precision's floor)", v->d.tolerance, st.last_relres);
  v->err = buf;
  return MAD_ERR_NOT_CONVERGED;
}

int mad_ved_run(mad_ved_ctx* v, const void* in, int32_t in_dtype, void* out, int32_t out_dtype,
                mad_ved_stats* st) {
  if (!v || !in || !out) return MAD_ERR_INVALID;
  mad_ved_stats local{};
  mad_ved_stats* s = st ? st : &local;
  return ved_run_status(v, ved_guarded(v, [&] { ved_run_impl(v, in, in_dtype, out, out_dtype, false, s); }), *s);
}

int mad_ved_run_device(mad_ved_ctx* v, const void* in, int32_t in_dtype, void* out,
                       int32_t out_dtype, mad_ved_stats* st) {
  if (!v || !in || !out) return MAD_ERR_INVALID;
  mad_ved_stats local{};
  mad_ved_stats* s = st ? st : &local;
  return ved_run_status(v, ved_guarded(v, [&] { ved_run_impl(v, in, in_dtype, out, out_dtype, true, s); }), *s);
}

int mad_ved_comm_init(mad_ved_ctx* v, const void* uid128) {
  if (!v || !uid128) return MAD_ERR_INVALID;
  return ved_guarded(v, [&] { mad_call(v->mad, mad_comm_init(v->mad, uid128)); });
}

int mad_ved_comm_init_local(mad_ved_ctx* v, uint64_t group) {
  if (!v) return MAD_ERR_INVALID;
  return ved_guarded(v, [&] { mad_call(v->mad, mad_comm_init_local(v->mad, group)); });
}

int mad_ved_comm_init_solo(mad_ved_ctx* v) {
  if (!v) return MAD_ERR_INVALID;
  return ved_guarded(v, [&] { mad_call(v->mad, mad_comm_init_solo(v->mad)); });
}

int mad_ved_tensor(mad_ved_ctx* v, const void* image, int32_t dtype, double* tensor_soa,
                   double* response) {
  if (!v || !image || !tensor_soa) return MAD_ERR_INVALID;
  return ved_guarded(v, [&] {
    REQUIRE(v->mad->d.nranks == 1, MAD_ERR_UNSUPPORTED, "mad_ved_tensor returns the whole grid: one rank only");
    HIP_CHECK(hipSetDevice(v->mad->device));
    ved_load_image(v, image, dtype, false);
    ved_tensor_any(v);
    hipStream_t st = v->mad->stream;
    HIP_CHECK(hipMemcpyAsync(tensor_soa, v->mad->tensor64, sizeof(double) * 6 * v->N,
                             hipMemcpyDeviceToHost, st));
    if (response)
      HIP_CHECK(hipMemcpyAsync(response, v->resp, sizeof(double) * v->N, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
  });
}

int mad_ved_hessian(mad_ved_ctx* v, const void* image, int32_t dtype, double sigma,
                    double* hessian_soa) {
  if (!v || !image || !hessian_soa) return MAD_ERR_INVALID;
  return ved_guarded(v, [&] {
    REQUIRE(sigma > 0.0, MAD_ERR_INVALID, "sigma must be positive");
    HIP_CHECK(hipSetDevice(v->mad->device));
    ved_load_image(v, image, dtype, false);
    double* H = nullptr;
    HIP_CHECK(big_alloc((void**)&H, sizeof(double) * 6 * v->N));
    if (v->d.precision == MAD_FP64) ved_scale<double>(v, sigma, VED_HESSIAN, true, H);
    else ved_scale<float>(v, sigma, VED_HESSIAN, true, H);
    HIP_CHECK(hipMemcpyAsync(hessian_soa, H, sizeof(double) * 6 * v->N, hipMemcpyDeviceToHost,
                             v->mad->stream));
    HIP_CHECK(hipStreamSynchronize(v->mad->stream));
    HIP_CHECK(hipFree(H));
  });
}

}  // extern "C"
