// mad_solver.hip -- host driver + C ABI (include/mad.h) of the MI355X multigrid
// anisotropic-diffusion solver.
//
// Reference path replaced (nellogrb/MultigridAnisotropicDiffusion):
//   GenerateData / VCycle / FullMultiGrid / L2Norm
//       include/itkMultigridAnisotropicDiffusionImageFilter.hxx:104-515
//   GridsHierarchy (depth rule, centring, tensor coarsening, DCA)
//       include/mad/itkGridsHierarchy.hxx:30-516
//   DirectSolver   include/mad/itkDirectSolver.hxx:32-147
//   smoothers      include/mad/itkMultigrid{GaussSeidel,WeightedJacobi}Smoother.hxx
//   transfers      include/mad/itkInterGridOperators.hxx
// Everything runs on one HIP stream per context; level arrays stay resident in
// HBM across V-cycles and time steps; only norms cross PCIe (8 bytes/cycle).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/mad.h"
#include "mad_alloc.hpp"
#include "mad_coarse.hpp"
#include "mad_comm.hpp"
#include "mad_kernels.hpp"

using namespace mad;

namespace {

struct MadError : std::runtime_error {
  int code;
  MadError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(x)                                                                  \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      throw MadError(MAD_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define REQUIRE(cond, code, msg) \
  do {                           \
    if (!(cond)) throw MadError((code), (msg)); \
  } while (0)

thread_local std::string g_last_error;

size_t dtype_size(int dt) {
  switch (dt) {
    case MAD_U8: case MAD_I8: return 1;
    case MAD_U16: case MAD_I16: return 2;
    case MAD_U32: case MAD_I32: case MAD_F32: return 4;
    case MAD_F64: return 8;
  }
  return 0;
}

inline dim3 grid_for(int nx, int ny, int nz, dim3 blk) {
  return dim3((unsigned)((nx + blk.x - 1) / blk.x), (unsigned)((ny + blk.y - 1) / blk.y),
              (unsigned)std::max(nz, 1));
}

inline unsigned flat_blocks(int64_t n, unsigned cap = 4096) {
  int64_t b = (n + 255) / 256;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

const dim3 BLK(64, 4, 1);

// image casts (MAD.hxx:110-127 in, :270-282 static_cast out) on a stream
template <typename T>
void convert_to(const void* src, int dt, T* dst, int64_t n, hipStream_t stream) {
  const unsigned nb = flat_blocks(n);
  switch (dt) {
    case MAD_U8: hipLaunchKernelGGL((convert_k<uint8_t, T>), dim3(nb), dim3(256), 0, stream, (const uint8_t*)src, dst, n); break;
    case MAD_I8: hipLaunchKernelGGL((convert_k<int8_t, T>), dim3(nb), dim3(256), 0, stream, (const int8_t*)src, dst, n); break;
    case MAD_U16: hipLaunchKernelGGL((convert_k<uint16_t, T>), dim3(nb), dim3(256), 0, stream, (const uint16_t*)src, dst, n); break;
    case MAD_I16: hipLaunchKernelGGL((convert_k<int16_t, T>), dim3(nb), dim3(256), 0, stream, (const int16_t*)src, dst, n); break;
    case MAD_U32: hipLaunchKernelGGL((convert_k<uint32_t, T>), dim3(nb), dim3(256), 0, stream, (const uint32_t*)src, dst, n); break;
    case MAD_I32: hipLaunchKernelGGL((convert_k<int32_t, T>), dim3(nb), dim3(256), 0, stream, (const int32_t*)src, dst, n); break;
    case MAD_F32: hipLaunchKernelGGL((convert_k<float, T>), dim3(nb), dim3(256), 0, stream, (const float*)src, dst, n); break;
    case MAD_F64: hipLaunchKernelGGL((convert_k<double, T>), dim3(nb), dim3(256), 0, stream, (const double*)src, dst, n); break;
    default: throw MadError(MAD_ERR_INVALID, "unknown input dtype");
  }
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void convert_from(const T* src, void* dst, int dt, int64_t n, hipStream_t stream) {
  const unsigned nb = flat_blocks(n);
  switch (dt) {
    case MAD_U8: hipLaunchKernelGGL((convert_int_k<T, uint8_t>), dim3(nb), dim3(256), 0, stream, src, (uint8_t*)dst, n, 0.0, 255.0); break;
    case MAD_I8: hipLaunchKernelGGL((convert_int_k<T, int8_t>), dim3(nb), dim3(256), 0, stream, src, (int8_t*)dst, n, -128.0, 127.0); break;
    case MAD_U16: hipLaunchKernelGGL((convert_int_k<T, uint16_t>), dim3(nb), dim3(256), 0, stream, src, (uint16_t*)dst, n, 0.0, 65535.0); break;
    case MAD_I16: hipLaunchKernelGGL((convert_int_k<T, int16_t>), dim3(nb), dim3(256), 0, stream, src, (int16_t*)dst, n, -32768.0, 32767.0); break;
    case MAD_U32: hipLaunchKernelGGL((convert_int_k<T, uint32_t>), dim3(nb), dim3(256), 0, stream, src, (uint32_t*)dst, n, 0.0, 4294967295.0); break;
    case MAD_I32: hipLaunchKernelGGL((convert_int_k<T, int32_t>), dim3(nb), dim3(256), 0, stream, src, (int32_t*)dst, n, -2147483648.0, 2147483647.0); break;
    case MAD_F32: hipLaunchKernelGGL((convert_k<T, float>), dim3(nb), dim3(256), 0, stream, src, (float*)dst, n); break;
    case MAD_F64: hipLaunchKernelGGL((convert_k<T, double>), dim3(nb), dim3(256), 0, stream, src, (double*)dst, n); break;
    default: throw MadError(MAD_ERR_INVALID, "unknown output dtype");
  }
  HIP_CHECK(hipGetLastError());
}


// dispatch (dim, kind) to compile-time parameters
template <typename F>
void dispatch(int dim, int kind, F&& f) {
  using std::integral_constant;
  if (dim == 3) {
    if (kind == KISO) f(integral_constant<int, 3>(), integral_constant<int, KISO>());
    else if (kind == KDIAG) f(integral_constant<int, 3>(), integral_constant<int, KDIAG>());
    else f(integral_constant<int, 3>(), integral_constant<int, KFULL>());
  } else {
    if (kind == KISO) f(integral_constant<int, 2>(), integral_constant<int, KISO>());
    else if (kind == KDIAG) f(integral_constant<int, 2>(), integral_constant<int, KDIAG>());
    else f(integral_constant<int, 2>(), integral_constant<int, KFULL>());
  }
}

struct LevelGeom {
  int64_t n[3];    // global size
  double h[3];
  int cent[3];     // 0 vertex / 1 cell, w.r.t. the finer level (level 0: vertex)
  int64_t N;       // global voxels
  int64_t z0, z1;  // this rank's slab [z0, z1) at this level
  bool distributed;
};

// GH.hxx:36-59
int max_depth_rule(int dim, const int64_t n0[3]) {
  uint64_t gs[3] = {(uint64_t)n0[0], (uint64_t)n0[1], (uint64_t)n0[2]};
  bool coarsest = false;
  int numberOfLevels = 1;
  while (!coarsest) {
    for (int d = 0; d < dim; ++d) {
      gs[d] = (gs[d] % 2 == 0) ? gs[d] / 2 : ((gs[d] - 1) / 2) + 1;
      if (gs[d] < 6) coarsest = true;
    }
    ++numberOfLevels;
  }
  --numberOfLevels;
  return numberOfLevels - 1;
}

// ---------------------------------------------------------------------------
// dense fp64 LU (partial pivoting) + explicit inverse of the coarsest operator on
// the device (rocSOLVER getrf + getri; replaces vnl_sparse_lu, DS.hxx:81-86; the
// inverse turns each per-cycle solve into one device GEMV).  `a` is row-major A,
// which rocSOLVER reads as column-major A^T: inv(A^T) column-major is inv(A)
// row-major, so the result needs no transpose.  Returns false if A is singular.
bool invert_dense_device(int64_t n, const std::vector<double>& a, double* d_inv,
                         hipStream_t stream) {
  rocblas_handle h = nullptr;
  if (rocblas_create_handle(&h) != rocblas_status_success)
    throw std::runtime_error("rocblas_create_handle failed");
  rocblas_set_stream(h, stream);
  rocblas_int* ipiv = nullptr;
  rocblas_int* info = nullptr;
  HIP_CHECK(hipMalloc(&ipiv, sizeof(rocblas_int) * n));
  HIP_CHECK(hipMalloc(&info, sizeof(rocblas_int) * 2));
  HIP_CHECK(hipMemcpyAsync(d_inv, a.data(), sizeof(double) * n * n, hipMemcpyHostToDevice, stream));
  const rocblas_int N = (rocblas_int)n;
  rocblas_status st = rocsolver_dgetrf(h, N, N, d_inv, N, ipiv, info);
  if (st == rocblas_status_success) st = rocsolver_dgetri(h, N, d_inv, N, ipiv, info + 1);
  rocblas_int hinfo[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(hinfo, info, sizeof hinfo, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  HIP_CHECK(hipFree(ipiv));
  HIP_CHECK(hipFree(info));
  rocblas_destroy_handle(h);
  if (st != rocblas_status_success)
    throw std::runtime_error("rocsolver getrf/getri failed (status " + std::to_string((int)st) + ")");
  return hinfo[0] == 0 && hinfo[1] == 0;
}

}  // namespace

// ---------------------------------------------------------------------------
struct SolverBase;

struct mad_ctx {
  mad_desc d{};
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t comm_stream = nullptr;  // overlapped halo exchanges (rank slabs)
  int dim = 3;
  int nlev = 0;
  std::vector<LevelGeom> geom;
  int kind = KFULL;
  int ncolors = 4;
  // level-0 fp64 tensor (SetDiffusionTensor), SoA on the device.  One rank: the whole grid,
  // component stride N.  Rank slab: per component the slab's planes plus tensor_tg ghost planes
  // per side (tensor_layout), so no rank ever holds the global tensor; the global planes
  // [tensor_lo, tensor_hi) inside the grid are the ones set_tensor / synth fill.
  double* tensor64 = nullptr;
  int64_t tensor_cs = 0;  // component stride (elements)
  int tensor_tg = 0;      // ghost planes per side
  int64_t tensor_lo = 0, tensor_hi = 0;
  bool tensor_set = false;
  bool setup_done = false;
  std::unique_ptr<SolverBase> solver;
  std::vector<uint32_t> step_cycles;
  std::vector<double> step_relres;
  // convergence history of the last run (mad_get_cycle_trace): one entry per cycle, or with
  // MAD_OPT_BENCHMARK_TRACE the reference's -DBENCHMARK entries (MAD.hxx:147-151, 222-227,
  // 401-409, 450-458, 477-485: level 0 after every sweep and after the coarse-grid correction,
  // seconds since the time step's start)
  struct TracePoint {
    uint32_t step;
    double relres, seconds;
  };
  std::vector<TracePoint> trace;
  bool bench_trace() const { return (d.options & MAD_OPT_BENCHMARK_TRACE) != 0; }
  bool trace_active = false;  // inside mad_run (kernel-API V-cycles record nothing)
  uint32_t trace_step = 0;
  double trace_rhs = 1.0;  // ||b|| of the time step (the relres denominator)
  std::chrono::steady_clock::time_point trace_t0{};  // the run's start / the step's (benchmark form)
  void trace_push(double rr) {
    trace.push_back({trace_step, rr, std::chrono::duration<double>(std::chrono::steady_clock::now() - trace_t0).count()});
  }
  double setup_ms = 0.0;
  Comm comm;
  ~mad_ctx();
};

// ghost planes per side of a rank's fp64 tensor slab on every distributed level: GHOST
// coefficient ghost planes, +2 for g's differences of the records (build_g_k), +2 for the
// tensor differences of the records (build_coef3_k)
constexpr int TENSOR_GHOST = GHOST + 4;

struct SolverBase {
  virtual ~SolverBase() {}
  virtual void setup(mad_ctx* c) = 0;
  virtual void upload(int l, int which, const double* h) = 0;
  virtual void download(int l, int which, double* h) = 0;
  virtual void fill(int l, int which, double v) = 0;
  virtual void smooth(int l, unsigned n) = 0;
  virtual double residual(int l, bool want_norm) = 0;
  virtual double norm(int l, int which) = 0;
  virtual void restrict_(int l) = 0;
  virtual bool residual_restrict(int l) = 0;  // fused b[l+1] <- R (b - A x); false: not applicable
  virtual void interpolate(int l, bool add) = 0;
  virtual void coarse_solve() = 0;
  // errors the device reported asynchronously (a peer-halo wait that timed out)
  virtual void check_device_errors() {}
  virtual void vcycle() = 0;
  virtual void fmg() = 0;
  virtual void run(const void* in, int in_dtype, void* out, int out_dtype, bool dev_io,
                   mad_stats* st) = 0;
  virtual void bench_smooth(int l, unsigned n, double* total_ms, double* kern_ms,
                            unsigned* launches) = 0;
  std::vector<float> launch_ms;  // per-launch durations of the last bench_smooth
  virtual void bench_vcycle(unsigned n, double* total_ms) = 0;
  virtual void synth_level(int l, int which, uint64_t seed) = 0;
  virtual std::string smooth_kernel(int l) = 0;
  // level-0 sweep ms of every placement candidate setup timed (Solver::tune_placement)
  virtual std::vector<double> placement_ms() const { return {}; }
};

mad_ctx::~mad_ctx() {
  solver.reset();
  if (tensor64) (void)hipFree(tensor64);
  comm.destroy();
  if (stream) (void)hipStreamDestroy(stream);
  if (comm_stream) (void)hipStreamDestroy(comm_stream);
}

namespace {

template <typename T>
struct LevelData {
  Geo g{};
  int cent[3] = {0, 0, 0};
  T* alloc[4] = {nullptr, nullptr, nullptr, nullptr};
  T* x = nullptr;  // solution
  T* b = nullptr;  // rhs
  T* r = nullptr;  // residual
  T* t = nullptr;  // WJ ping-pong / scratch
  T* cf = nullptr;        // field 0, plane 0 (ghost planes precede it on rank slabs)
  T* cf_alloc = nullptr;
  // level 0 of the V-cycle layout (fp32, fused): b in the records' x-parity-split order for the sweep
  // (gs_fused3_k BS), refreshed from the dense b -- the canonical copy -- by sync_bsplit when b changed
  // (brec_ok doubles as its flag: a level has records carrying b or this copy, never both)
  T* bs = nullptr;
  T* bs_alloc = nullptr;
  Rat<T> rat{};
  int64_t ghost = 0;      // elements of the ghost planes on one side (3D: GHOST * sz)
  bool b_halo_ok = false; // ghost planes of b are current (fused sweep on rank slabs)
  // brec: the coefficient records also carry b (record stride g.rs = ncoef + 1), so the
  // sweep / residual read it with the record instead of as a separate stream.  Used
  // on level 0, whose b changes once per time step; the dense b stays the canonical
  // copy and is scattered into the records on demand (sync_brec).
  bool brec = false;
  bool brec_ok = false;
  // rank slabs: x's GHOST ghost planes hold the neighbours' current x (x_halo_ok),
  // possibly still being written by the overlapped exchange (x_halo_pending, ev_halo)
  bool x_halo_ok = false;
  bool x_halo_pending = false;
  hipEvent_t ev_bnd = nullptr;   // boundary chunks of the fused sweep done
  hipEvent_t ev_halo = nullptr;  // their exchange done (communication stream)
  // single-launch rank-slab sweeps: edge-plane counters the sweep kernel increments
  // (signal memory, [0] bottom / [1] top) and the sweeps issued so far
  uint32_t* sig = nullptr;
  uint32_t sig_epoch = 0;
  // peer halo (MAD_OPT_PEER_HALO, Solver::setup_peer): the fused sweep stores its edge planes
  // straight into the neighbours' mailboxes.  phys: the ping-pong pair's x / t at setup (buffer
  // identity: mailbox and counter index); win: this rank's window (uncached: mailboxes
  // [buffer * 2 + side] of GHOST planes, then the control block: counters [buffer * 2 + side],
  // ticket, error word); win_lo / win_hi: the neighbours' windows mapped here
  T* phys[2] = {nullptr, nullptr};
  char* win = nullptr;
  char* win_lo = nullptr;
  char* win_hi = nullptr;
  bool win_ipc = false;
  bool peer = false;
  bool x_peer_pending = false;  // x's ghost planes arrive by peer stores: resolve before use
  uint32_t peer_tiles = 0;      // counts per side and batch (fused: edge tiles; per-colour: push blocks)
  // per-colour levels (round 5): after a sweep's last colour pass peer_push_k copies the edge planes
  // into the neighbours' mailboxes; the batches alternate between the two buffers by peer_seq
  bool peer_pc = false;
  int peer_seq = 0;
  int peer_buf = 0;  // buffer of the batch in flight (x_peer_pending)
  // b of a distributed coarse level: the descent pushes its edge planes (one buffer, mailboxes
  // [4 + side], counters [8 + side]); the first sweep takes them in
  bool b_peer_pending = false;
  // x is zero but was not written (the V-cycle descent left it to the level's first sweep, which
  // takes its planes as zeros: gs_fused3_k ZU); any other write of x clears it
  bool x_zero_lazy = false;
};
// z-depth of a rank slab's boundary chunks (>= GHOST; 4 measured 0.231 vs 0.228 ms per 8-rank
// sweep, profiles/r02_slab_tiles.log)
constexpr int BOUNDARY_PLANES = 8;
// level 0 of the V-cycle layout reads b from an x-parity-split copy (gs_fused3_k BS) instead of staging
// the dense b through LDS (BL); 0 keeps BL (A/B, profiles/r06_bsplit_ab.log)
#ifndef MAD_FUSED_B_SPLIT
#define MAD_FUSED_B_SPLIT 1
#endif
inline int boundary_planes() { return BOUNDARY_PLANES; }

template <typename T>
class Solver final : public SolverBase {
 public:
  ~Solver() override { release(); }

  void setup(mad_ctx* c) override {
    c_ = c;
    release();
    const int dim = c->dim;
    const int nl = c->nlev;
    lv_.resize(nl);
    ncoef_ = coef_count(dim, c->kind);
    int64_t part_need = 1;
    for (int l = 0; l < nl; ++l) {
      const LevelGeom& G = c->geom[l];
      LevelData<T>& L = lv_[l];
      L.g.nx = (int)G.n[0];
      L.g.ny = (int)G.n[1];
      L.g.nz = (int)(G.z1 - G.z0);
      L.g.zoff = (int)G.z0;
      L.g.zlo_ghost = (G.distributed && G.z0 > 0) ? 1 : 0;
      L.g.zhi_ghost = (G.distributed && G.z1 < G.n[2]) ? 1 : 0;
      L.g.sy = G.n[0];
      L.g.sz = G.n[0] * G.n[1];
      L.g.N = L.g.sz * L.g.nz;
      L.g.hx0 = (L.g.nx + 1) / 2;
      for (int d = 0; d < 3; ++d) L.cent[d] = G.cent[d];
      L.rat.r[0] = T(1);
      L.rat.r[1] = (T)((G.h[0] * G.h[0]) / (G.h[1] * G.h[1]));
      L.rat.r[2] = (T)((G.h[0] * G.h[0]) / (G.h[2] * G.h[2]));
      L.ghost = (dim == 3) ? (int64_t)GHOST * L.g.sz : 0;
      // + a margin of rows at both ends: the fused sweep's masked border lanes read
      // up to a tile halo outside the outermost (ghost) plane
      const int64_t margin = margin_elems(L.g);
      const int64_t tot = L.g.N + 2 * (L.ghost + margin);
      bool brec_on = c->d.cycle == MAD_SMOOTHER && !(c->d.options & MAD_OPT_NO_RECORD_B);
      if (c->d.precision == MAD_FP32_REFINE) brec_on = false;  // b changes every cycle there
      L.brec = (dim == 3 && l == 0 && brec_on);
      L.g.rs = ncoef_ + (L.brec ? 1 : 0);
      const int64_t cplane = L.g.sz * L.g.rs;
      const int64_t cgp = (dim == 3) ? GHOST : 0;
      const int64_t cmargin = margin * L.g.rs;
      const int64_t ctot = (L.g.nz + 2 * cgp) * cplane + 2 * cmargin;
      for (int a = 0; a < 4; ++a) {
        level_alloc((void**)&L.alloc[a], sizeof(T) * tot);
        HIP_CHECK(hipMemsetAsync(L.alloc[a], 0, sizeof(T) * tot, c->stream));
      }
      level_alloc((void**)&L.cf_alloc, sizeof(T) * ctot);
      HIP_CHECK(hipMemsetAsync(L.cf_alloc, 0, sizeof(T) * ctot, c->stream));
      L.x = L.alloc[0] + margin + L.ghost;
      L.b = L.alloc[1] + margin + L.ghost;
      L.r = L.alloc[2] + margin + L.ghost;
      L.t = L.alloc[3] + margin + L.ghost;
      L.phys[0] = L.x;
      L.phys[1] = L.t;
      // coefficient records, point-interleaved (mad_kernels.hpp, cidx); 3D levels keep
      // GHOST coefficient planes per side: neighbour planes on rank slabs (the fused
      // sweep recomputes colours on them), padding for masked border lanes otherwise
      // Level 0's records carry b when b is reused by many sweeps: SMOOTHER mode (up to
      // MaxCycles sweeps of one system per time step; the smoother benchmark) -- the
      // sweeps run 3-6 % faster with one record stream.  V-cycle / FMG solves change b
      // every time step after ~2 cycles (~12 level-0 record passes), where the 2.2 ms
      // scatter of b into the 40-B records (partial-line writes, 512^3) costs more than
      // it saves (VED diffusion 126 -> 116.5 ms without it, profiles/r01_brec_ab.log).
      // (L.brec / L.g.rs are set above, before the allocation)
      L.cf = L.cf_alloc + cmargin + cgp * cplane;
      if (l == 0 && dim == 3 && !L.brec && sizeof(T) == 4 && MAD_FUSED_B_SPLIT) {
        level_alloc((void**)&L.bs_alloc, sizeof(T) * tot);
        HIP_CHECK(hipMemsetAsync(L.bs_alloc, 0, sizeof(T) * tot, c->stream));
        L.bs = L.bs_alloc + margin + L.ghost;
      }
      dim3 gr = grid_for(L.g.nx, L.g.ny, L.g.nz, BLK);
      part_need = std::max<int64_t>(part_need, (int64_t)gr.x * gr.y * gr.z);
    }
    refine_ = sizeof(T) == 4 && c->d.precision == MAD_FP32_REFINE;
    if (refine_) {
      LevelData<T>& L0 = lv_[0];
      const int64_t margin = margin_elems(L0.g);
      const int64_t tot = L0.g.N + 2 * (L0.ghost + margin);
      for (auto& a : r64alloc_) {
        HIP_CHECK(big_alloc((void**)&a, sizeof(double) * tot));
        HIP_CHECK(hipMemsetAsync(a, 0, sizeof(double) * tot, c->stream));
      }
      u64_ = r64alloc_[0] + margin + L0.ghost;
      b64_ = r64alloc_[1] + margin + L0.ghost;
      r64_ = r64alloc_[2] + margin + L0.ghost;
      // b64 as fp32 for the time steps whose rhs is an exactly-fp32 image (residual64)
      HIP_CHECK(big_alloc((void**)&b32alloc_, sizeof(float) * tot));
      HIP_CHECK(hipMemsetAsync(b32alloc_, 0, sizeof(float) * tot, c->stream));
      b32_ = b32alloc_ + margin + L0.ghost;
      const int64_t cgp = (dim == 3) ? GHOST : 0;
      const int64_t cplane = L0.g.sz * ncoef_;
      const int64_t ctot = (L0.g.nz + 2 * cgp) * cplane + 2 * margin * ncoef_;
      HIP_CHECK(big_alloc((void**)&cf64_alloc_, sizeof(double) * ctot));
      HIP_CHECK(hipMemsetAsync(cf64_alloc_, 0, sizeof(double) * ctot, c->stream));
      cf64_ = cf64_alloc_ + margin * ncoef_ + cgp * cplane;
      for (int d = 0; d < 3; ++d) rat64_.r[d] = (c->geom[0].h[0] * c->geom[0].h[0]) / (c->geom[0].h[d] * c->geom[0].h[d]);
    }
    int can_wait = 0;
    if (hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, c->device) !=
        hipSuccess)
      can_wait = 0;
    for (int l = 0; l < nl; ++l)
      if (c->geom[l].distributed) {
        HIP_CHECK(hipEventCreateWithFlags(&lv_[l].ev_bnd, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&lv_[l].ev_halo, hipEventDisableTiming));
        // single-launch rank-slab sweeps (part 3) with gs_kernel 4 only.  Not the
        // default: the communication stream's wait-on-value wakes ~0.25 ms after the
        // signal (tools/overlap_probe.hip, profiles/r01_overlap_probe.log) -- longer
        // than a whole 64-plane rank sweep -- while an event after the short boundary
        // launch releases the exchange within ~0.05 ms, so boundary + interior
        // launches (parts 1, 2) win.
        if (can_wait && c->d.gs_kernel == 4) {
          HIP_CHECK(hipExtMallocWithFlags((void**)&lv_[l].sig, 2 * sizeof(uint32_t),
                                          hipMallocSignalMemory));
          const uint32_t zero[2] = {0u, 0u};
          HIP_CHECK(hipMemcpy(lv_[l].sig, zero, sizeof zero, hipMemcpyHostToDevice));
          lv_[l].sig_epoch = 0;
        }
      }
    part_need = std::max<int64_t>(part_need, 4096);
    HIP_CHECK(hipMalloc(&part_, sizeof(double) * part_need));
    part_cap_ = part_need;
    HIP_CHECK(hipMalloc(&scal_, sizeof(double) * 4));
    HIP_CHECK(hipHostMalloc(&hscal_, sizeof(double) * 4, hipHostMallocDefault));
    build_operators();
    build_coarse_inverse();
    setup_peer();
    tuned_ms_.clear();
    for (int l = 0; l < nl; ++l) tune_placement(l);  // levels of >= 2^24 voxels: 0, and 1 at 512^3
    HIP_CHECK(hipStreamSynchronize(c->stream));
  }

  // ------------------------------------------------------------- level-0 placement
  // The level-0 sweep streams ~7 GB per launch at 512^3, and its speed depends on the arrays it runs on:
  // per allocation, each direction of the ping-pong pair (read x / write t, then read t / write x)
  // settles at ~1.11-1.13 or at ~1.24 ms -- the same kernel, the same HBM bytes, the same L2 hit rate and
  // ~7 K UTCL1 misses per launch in every case, the clocks steady (profiles/r06_placement.md) -- and
  // freshly allocated arrays run slower still for their first ~0.3-1 s of use (profiles/
  // r06_transient_probe.log).  So setup allocates PLACEMENT_TRIES - 1 more sets of the level's arrays (the
  // pair each time, the records -- and the V-cycle layout's split b -- too every second time; contents
  // copied over; 12 sets: 1.10 vs 1.13 ms sweeps, 7.31 vs 7.42 ms V-cycles against 8 on one box,
  // profiles/r06_tries_ab.log), sweeps all of them in turn
  // for MAD_PLACEMENT_AGE_MS of device time, then times both directions of every set and keeps the
  // fastest, the others freed.  3D levels of >= 2^24 voxels (a rank's slab too: 512 x 512 x 64 on 8
  // ranks) whose sweep is the fused GS sweep -- timed as the plain whole-slab launch, no exchange, so
  // every rank decides alone -- or, on one rank, the WJ sweep; as many sets as the free memory allows.
  // Not on the in-process transport (its ranks share one device).  MAD_OPT_NO_PLACEMENT_TUNE keeps the
  // first allocation.  Every level of >= 2^24 voxels is tuned so (level 1 of a 512^3 grid too);
  // mad_placement_trials reports level 0's trials.
#ifndef MAD_PLACEMENT_TRIES
#define MAD_PLACEMENT_TRIES 12
#endif
  static constexpr int PLACEMENT_TRIES = MAD_PLACEMENT_TRIES;
#ifndef MAD_PLACEMENT_AGE_MS
#define MAD_PLACEMENT_AGE_MS 1500.0
#endif
  void tune_placement(int l) {
    if (c_->dim != 3 || (c_->d.options & MAD_OPT_NO_PLACEMENT_TUNE)) return;
    if (c_->comm.active() && c_->comm.mode() == Comm::LOCAL) return;
    LevelData<T>& L = lv_[l];
    const int sm = c_->d.smoother;
    if (L.g.N < ((int64_t)1 << 24) || sm == MAD_GAUSS_SEIDEL_LEX) return;
    const bool fused = sm == MAD_GAUSS_SEIDEL && use_fused(l);
    if (!fused && (sm == MAD_GAUSS_SEIDEL || c_->comm.active())) return;
    const int64_t margin = margin_elems(L.g);
    const size_t pbytes = sizeof(T) * (size_t)(L.g.N + 2 * (L.ghost + margin));
    const int64_t cplane = L.g.sz * L.g.rs;
    const size_t cbytes = sizeof(T) * (size_t)((L.g.nz + 2 * GHOST) * cplane + 2 * margin * L.g.rs);
    struct Set {
      T* x;
      T* t;
      T* cf;
      T* bs;  // the V-cycle layout's split b (nullptr where the level has none): moves with the records
    };
    auto point = [&](const Set& a) {  // after an even number of sweeps alloc[0] is x's, alloc[3] t's
      L.alloc[0] = a.x;
      L.alloc[3] = a.t;
      L.cf_alloc = a.cf;
      L.bs_alloc = a.bs;
      L.bs = a.bs ? a.bs + margin + L.ghost : nullptr;
      L.x = a.x + margin + L.ghost;
      L.t = a.t + margin + L.ghost;
      L.cf = a.cf + margin * L.g.rs + GHOST * cplane;
      L.phys[0] = L.x;
      L.phys[1] = L.t;
    };
    // fused GS: the plain whole-slab launch on the level's arrays (rank slabs: no exchange; the ghost
    // planes hold zeros like everything but the records here), swapping the pair like the sweep
    auto sweeps = [&](unsigned n) {
      if (!fused) {
        double tot_ms = 0.0, kern = 0.0;
        unsigned q = 0;
        bench_smooth(l, n, &tot_ms, &kern, &q);
        return;
      }
      std::vector<hipEvent_t> ev(2 * n);
      for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
      for (unsigned i = 0; i < n; ++i) {
        HIP_CHECK(hipEventRecord(ev[2 * i], c_->stream));
        launch_fused_part(L, 0);
        HIP_CHECK(hipEventRecord(ev[2 * i + 1], c_->stream));
        std::swap(L.x, L.t);
        std::swap(L.alloc[0], L.alloc[3]);
      }
      HIP_CHECK(hipEventSynchronize(ev[2 * n - 1]));
      launch_ms.assign(n, 0.f);
      for (unsigned i = 0; i < n; ++i) HIP_CHECK(hipEventElapsedTime(&launch_ms[i], ev[2 * i], ev[2 * i + 1]));
      for (auto& e : ev) (void)hipEventDestroy(e);
    };
    // mean ms of the two launches in each direction: 0 and 2 read x and write t, 1 and 3 the reverse
    auto time_dirs = [&](double* fwd, double* rev) {
      sweeps(4);
      *fwd = 0.5 * (launch_ms[0] + launch_ms[2]);
      *rev = 0.5 * (launch_ms[1] + launch_ms[3]);
      if (l == 0) {
        tuned_ms_.push_back(*fwd);
        tuned_ms_.push_back(*rev);
      }
    };
    sweeps(16);  // the clocks ramp up over the first ~20 launches after the device idled (r06_clock_summaries)
    // the candidate sets, allocated up front: the pair each time, the records too every second time
    std::vector<Set> sets{Set{L.alloc[0], L.alloc[3], L.cf_alloc, L.bs_alloc}};
    const bool has_bs = L.bs_alloc != nullptr;
    for (int tr = 1; tr < PLACEMENT_TRIES; ++tr) {
      const bool with_cf = (tr % 2) == 0;
      const bool with_bs = with_cf && has_bs;
      size_t free_b = 0, total_b = 0;
      HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
      if (free_b < 2 * (2 * pbytes + (with_cf ? cbytes : 0) + (with_bs ? pbytes : 0)) + ((size_t)1 << 30)) break;
      Set cand{nullptr, nullptr, with_cf ? nullptr : sets[0].cf, with_bs ? nullptr : sets[0].bs};
      bool ok = contiguous_alloc((void**)&cand.x, pbytes) == hipSuccess &&
                contiguous_alloc((void**)&cand.t, pbytes) == hipSuccess &&
                (!with_cf || contiguous_alloc((void**)&cand.cf, cbytes) == hipSuccess) &&
                (!with_bs || contiguous_alloc((void**)&cand.bs, pbytes) == hipSuccess);
      if (!ok) {
        (void)hipGetLastError();
        if (cand.x) (void)hipFree(cand.x);
        if (cand.t) (void)hipFree(cand.t);
        if (with_cf && cand.cf) (void)hipFree(cand.cf);
        if (with_bs && cand.bs) (void)hipFree(cand.bs);
        break;
      }
      HIP_CHECK(hipMemcpyAsync(cand.x, sets[0].x, pbytes, hipMemcpyDeviceToDevice, c_->stream));
      HIP_CHECK(hipMemcpyAsync(cand.t, sets[0].t, pbytes, hipMemcpyDeviceToDevice, c_->stream));
      if (with_cf) HIP_CHECK(hipMemcpyAsync(cand.cf, sets[0].cf, cbytes, hipMemcpyDeviceToDevice, c_->stream));
      if (with_bs) HIP_CHECK(hipMemcpyAsync(cand.bs, sets[0].bs, pbytes, hipMemcpyDeviceToDevice, c_->stream));
      sets.push_back(cand);
    }
    // age them: freshly allocated arrays sweep slower for the first ~0.3-1 s of their use, then settle at
    // their own speed (profiles/r06_transient_probe.log), so the sets are swept in turn for
    // MAD_PLACEMENT_AGE_MS of device time before any is timed
    double aged_ms = 0.0;
    while (sets.size() > 1 && aged_ms < MAD_PLACEMENT_AGE_MS) {
      for (const Set& st : sets) {
        point(st);
        sweeps(4);
        for (float v : launch_ms) aged_ms += v;
      }
    }
    double bf = INFINITY, br = INFINITY;
    size_t kept = 0;
    for (size_t i = 0; i < sets.size(); ++i) {
      point(sets[i]);
      double f = 0.0, r = 0.0;
      time_dirs(&f, &r);
      if (f + r < bf + br) {
        kept = i;
        bf = f;
        br = r;
      }
    }
    const Set best = sets[kept];
    point(best);
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    for (size_t i = 0; i < sets.size(); ++i) {
      if (i == kept) continue;
      HIP_CHECK(hipFree(sets[i].x));
      HIP_CHECK(hipFree(sets[i].t));
      // records (and split b): a set either owns its own or shares the first set's
      const bool owns_cf = i == 0 || sets[i].cf != sets[0].cf;
      if (owns_cf && sets[i].cf != best.cf) HIP_CHECK(hipFree(sets[i].cf));
      const bool owns_bs = sets[i].bs && (i == 0 || sets[i].bs != sets[0].bs);
      if (owns_bs && sets[i].bs != best.bs) HIP_CHECK(hipFree(sets[i].bs));
    }
    x_changed(l);
    L.b_halo_ok = L.brec_ok = false;
  }
  std::vector<double> tuned_ms_;  // per candidate pair: forward, reverse level-0 sweep ms (last setup)
  std::vector<double> placement_ms() const override { return tuned_ms_; }

  // level arrays (x, b, r, t, coefficient records): mad_alloc.hpp
  static void level_alloc(void** p, size_t bytes) { HIP_CHECK(contiguous_alloc(p, bytes)); }

  // ------------------------------------------------------------- peer halo
  // MAD_OPT_PEER_HALO: on every distributed level whose sweeps are fused single launches with
  // both edge chunks reflected outward (>= 2 z-chunks of >= GHOST planes), the sweep itself stores
  // its GHOST edge planes into the neighbours' mailboxes and counts its tiles in their counters;
  // no exchange follows the sweep.  The next consumer of x's ghost planes waits for the
  // neighbours' counters and copies the mailboxes in (peer_resolve, one small launch).  Collective
  // (share_window); every rank takes the same decision (same plane counts on distributed levels).
  static constexpr size_t PEER_CTL = 256;
  // six mailboxes of GHOST planes: x [buffer * 2 + side] (buffers 0, 1), b [4 + side]; then the control block
  size_t window_bytes(const LevelData<T>& L) const { return 6 * (size_t)L.ghost * sizeof(T) + PEER_CTL; }
  T* mailbox(char* w, const LevelData<T>& L, int buf, int side) const {
    return (T*)(w + (size_t)(buf * 2 + side) * (size_t)L.ghost * sizeof(T));
  }
  uint32_t* peer_ctl(char* w, const LevelData<T>& L) const {
    return (uint32_t*)(w + 6 * (size_t)L.ghost * sizeof(T));
  }
  bool peer_eligible(int l) {
    LevelData<T>& L = lv_[l];
    if (!(c_->d.options & MAD_OPT_PEER_HALO) || !c_->comm.active() || !c_->geom[l].distributed) return false;
    if (c_->dim != 3) return false;
    if (!use_fused(l))  // per-colour GS level: pushed after its last colour pass (peer_push)
      return c_->d.smoother == MAD_GAUSS_SEIDEL && colour_ca(l) && L.g.nz >= GHOST;
    int tiles = 0, nchunks = 0;
    fused_shape(L, &tiles, &nchunks);
    const ZRange zr = whole_range(L.g.nz, tiles, fused_cfg());
    return nchunks >= 2 && zr.zc >= GHOST;
  }
  void setup_peer() {
    int wall_khz = 0;
    if (hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, c_->device) != hipSuccess ||
        wall_khz <= 0)
      wall_khz = 100000;
    peer_timeout_ticks_ = (uint64_t)wall_khz * 1000ull * 20ull;  // 20 s
    for (size_t l = 0; l < lv_.size(); ++l) {
      LevelData<T>& L = lv_[l];
      if (!peer_eligible((int)l)) continue;
      const size_t wb = window_bytes(L);
      HIP_CHECK(hipExtMallocWithFlags((void**)&L.win, wb, hipDeviceMallocUncached));
      HIP_CHECK(hipMemsetAsync(L.win, 0, wb, c_->stream));
      void *lo = nullptr, *hi = nullptr;
      c_->comm.share_window(L.win, c_->stream, &lo, &hi, &L.win_ipc);
      L.win_lo = (char*)lo;
      L.win_hi = (char*)hi;
      if ((L.g.zlo_ghost && !lo) || (L.g.zhi_ghost && !hi)) {
        // the windows could not be mapped on every rank (share_window agreed on it): this level
        // exchanges after its sweeps as without the option
        HIP_CHECK(hipFree(L.win));
        L.win = nullptr;
        continue;
      }
      if (!peer_selftest(L)) {
        // a neighbour's token or count did not arrive on some rank: every rank exchanges instead
        Comm::close_window(L.win_lo, L.win_ipc);
        Comm::close_window(L.win_hi, L.win_ipc);
        L.win_lo = L.win_hi = nullptr;
        HIP_CHECK(hipFree(L.win));
        L.win = nullptr;
        peer_fallbacks_ += 1;
        continue;
      }
      if (use_fused((int)l)) {
        int tiles = 0, nchunks = 0;
        fused_shape(L, &tiles, &nchunks);
        L.peer_tiles = (uint32_t)tiles;
      } else {
        L.peer_pc = true;
        L.peer_tiles = push_blocks(L);
      }
      L.peer = true;
    }
  }
  // every mailbox of the window -- x buffers 0 and 1, the b mailboxes (buffer 2) -- filled through
  // the mapped windows by the sweep's store / completion / counter pattern with a pattern of the
  // sending rank and the buffer, every element checked on the receiving rank, every counter pair
  // exercised and reset (collective; peer_ping_k / peer_pong_k)
  bool peer_selftest(LevelData<T>& L) {
    const int r = c_->comm.rank();
    const bool self = c_->comm.stand_in();
    const int64_t n = (int64_t)L.ghost;
    const int64_t top = (int64_t)(GHOST - 1) * L.g.sz;
    const unsigned nblk = (unsigned)std::min<int64_t>(256, std::max<int64_t>(1, (n + 255) / 256));
    uint32_t* ctl = peer_ctl(L.win, L);
    const uint32_t one = 1u;
    HIP_CHECK(hipMemcpyAsync(ctl + 6, &one, sizeof one, hipMemcpyHostToDevice, c_->stream));
    const uint64_t tmo = peer_timeout_ticks_ / 10;  // 2 s
    for (int buf = 0; buf < 3; ++buf) {
      const int salt = 1024 * buf;  // peer_pattern stays < 2^24 (exact in fp32)
      const int cb = buf == 2 ? 8 : 2 * buf;
      // every rank's ok word is set (and the previous buffer's pongs done) before any ping counts in
      c_->comm.local_barrier(c_->stream);
      hipLaunchKernelGGL((peer_ping_k<T>), dim3(nblk, 2), dim3(256), 0, c_->stream, peer_out(L, buf), n, top,
                         r + salt);
      HIP_CHECK(hipGetLastError());
      // the in-process transport's ranks share one device's hardware queues: all pings done first
      c_->comm.local_barrier(c_->stream);
      const T* mlo = L.g.zlo_ghost ? mailbox(L.win, L, buf, 0) : nullptr;
      const T* mhi = L.g.zhi_ghost ? mailbox(L.win, L, buf, 1) : nullptr;
      hipLaunchKernelGGL((peer_pong_k<T>), dim3(nblk, 2), dim3(256), 0, c_->stream, mlo, mhi, ctl + cb,
                         ctl + cb + 1, (self ? r : r - 1) + salt, (self ? r : r + 1) + salt, n, nblk, ctl + 6, tmo);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemsetAsync(ctl + cb, 0, 2 * sizeof(uint32_t), c_->stream));  // this buffer's counters
    }
    uint32_t ok = 0;
    HIP_CHECK(hipMemcpyAsync(&ok, ctl + 6, sizeof ok, hipMemcpyDeviceToHost, c_->stream));
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    return c_->comm.all_true(ok == 1u, c_->stream);
  }
  // where this rank's sweep into buffer `buf` stores its edge planes: the bottom edge chunk into
  // rank - 1's mailbox of planes above it (side 1), the top chunk (reflected: plane stride -sz) into
  // rank + 1's mailbox of planes below it (side 0), filled from its last plane down
  // SOLO / RCCL-SOLO (the own window stands in for both neighbours): each edge chunk fills the
  // own mailbox of its own side, as SOLO's exchange copies the own edge planes into the own ghost
  // planes -- the same bytes, and a rank at either end of the decomposition waits only on the side
  // it has
  // (buf 2: the b mailboxes, counted in counters 8 + side)
  PeerOut<T> peer_out(const LevelData<T>& L, int buf) const {
    PeerOut<T> po{{nullptr, nullptr}, {nullptr, nullptr}};
    const bool self = c_->comm.stand_in();
    const int cbase = buf == 2 ? 8 : buf * 2;
    if (L.g.zlo_ghost && L.win_lo) {
      const int side = self ? 0 : 1;
      po.dst[0] = mailbox(L.win_lo, L, buf, side);
      po.sig[0] = peer_ctl(L.win_lo, L) + cbase + side;
    }
    if (L.g.zhi_ghost && L.win_hi) {
      const int side = self ? 1 : 0;
      po.dst[1] = mailbox(L.win_hi, L, buf, side) + (int64_t)(GHOST - 1) * L.g.sz;
      po.sig[1] = peer_ctl(L.win_hi, L) + cbase + side;
    }
    return po;
  }
  int buffer_index(const LevelData<T>& L, const T* a) const { return a == L.phys[0] ? 0 : 1; }
  // x's ghost planes from the neighbours' last peer sweep: wait for their counters, copy the
  // mailboxes in.  The in-process transport (ranks as threads sharing one device's hardware
  // queues) waits on the host instead: every rank's stream drained, then a barrier.
  void peer_resolve(int l) {
    LevelData<T>& L = lv_[l];
    if (!L.x_peer_pending) return;
    L.x_peer_pending = false;
    const int buf = L.peer_buf;
    if (c_->comm.mode() == Comm::LOCAL) c_->comm.local_barrier(c_->stream);
    const size_t bytes = (size_t)L.ghost * sizeof(T);
    char* dlo = L.g.zlo_ghost ? (char*)(L.x - L.ghost) : nullptr;
    char* dhi = L.g.zhi_ghost ? (char*)(L.x + (int64_t)L.g.nz * L.g.sz) : nullptr;
    // at most 2 x 64 workgroups: while they wait, the other CUs stay free for a neighbour's sweep
    // that shares the device (the one-GPU two-process test; LOCAL ranks wait on the host)
    const unsigned blocks = (unsigned)std::min<size_t>(64, std::max<size_t>(1, (bytes / 16 + 255) / 256));
    hipLaunchKernelGGL(peer_unpack_k, dim3(blocks, 2), dim3(256), 0, c_->stream, dlo,
                       (const char*)mailbox(L.win, L, buf, 0), dhi, (const char*)mailbox(L.win, L, buf, 1),
                       (uint64_t)bytes, peer_ctl(L.win, L), buf * 2, L.peer_tiles, peer_timeout_ticks_);
    HIP_CHECK(hipGetLastError());
  }
  void peer_resolve_all() {
    for (size_t l = 0; l < lv_.size(); ++l) {
      peer_resolve((int)l);
      peer_resolve_b((int)l);
    }
  }
  // b's ghost planes from the neighbours' descents (counters 8 + side, mailboxes [4 + side])
  void peer_resolve_b(int l) {
    LevelData<T>& L = lv_[l];
    if (!L.b_peer_pending) return;
    L.b_peer_pending = false;
    if (c_->comm.mode() == Comm::LOCAL) c_->comm.local_barrier(c_->stream);
    const size_t bytes = (size_t)L.ghost * sizeof(T);
    char* dlo = L.g.zlo_ghost ? (char*)(L.b - L.ghost) : nullptr;
    char* dhi = L.g.zhi_ghost ? (char*)(L.b + (int64_t)L.g.nz * L.g.sz) : nullptr;
    const unsigned blocks = push_blocks(L);
    hipLaunchKernelGGL(peer_unpack_k, dim3(blocks, 2), dim3(256), 0, c_->stream, dlo,
                       (const char*)mailbox(L.win, L, 2, 0), dhi, (const char*)mailbox(L.win, L, 2, 1),
                       (uint64_t)bytes, peer_ctl(L.win, L), 8, blocks, peer_timeout_ticks_);
    HIP_CHECK(hipGetLastError());
  }
  // the descent wrote b of a distributed peer level: its edge planes into the neighbours' b mailboxes
  // (one buffer: the neighbour has taken in the previous cycle's batch before this rank's next
  // descent can run -- this rank's level-l work in between waits for the neighbour's first sweep
  // there, which starts with that unpack)
  void peer_push_b(int l) {
    LevelData<T>& L = lv_[l];
    const int64_t top_off = (int64_t)(L.g.nz - GHOST) * L.g.sz;
    hipLaunchKernelGGL((peer_push_k<T>), dim3(push_blocks(L), 2), dim3(256), 0, c_->stream, L.b, top_off,
                       peer_out(L, 2), (int64_t)L.ghost, (int64_t)(GHOST - 1) * L.g.sz);
    HIP_CHECK(hipGetLastError());
    L.b_halo_ok = true;
    L.b_peer_pending = true;
  }
  // b's ghost planes current for a sweep / descent on a rank slab: the pushed batch, or an exchange
  void b_halo(int l) {
    LevelData<T>& L = lv_[l];
    if (L.b_peer_pending) peer_resolve_b(l);
    if (!L.b_halo_ok) {
      halo(l, L.b, GHOST);
      L.b_halo_ok = true;
    }
  }
  // level l's b is about to change (a batch still in flight for it is taken in first)
  void b_changed(int l) {
    LevelData<T>& L = lv_[l];
    if (L.b_peer_pending) peer_resolve_b(l);
    L.b_halo_ok = L.brec_ok = false;
  }
  // per-colour levels: workgroups per side of peer_push_k (each counts itself in when its stores
  // are complete), as many as the unpack uses
  static uint32_t push_blocks(const LevelData<T>& L) {
    const size_t bytes = (size_t)L.ghost * sizeof(T);
    return (uint32_t)std::min<size_t>(64, std::max<size_t>(1, (bytes / 16 + 255) / 256));
  }
  // after the last colour pass of a per-colour sweep: the GHOST edge planes into the neighbours'
  // mailboxes of the next buffer, no exchange; the next consumer of x's ghost planes resolves it
  void peer_push(int l) {
    LevelData<T>& L = lv_[l];
    const int buf = L.peer_seq & 1;
    ++L.peer_seq;
    const int64_t top_off = (int64_t)(L.g.nz - GHOST) * L.g.sz;
    hipLaunchKernelGGL((peer_push_k<T>), dim3(push_blocks(L), 2), dim3(256), 0, c_->stream, L.x, top_off,
                       peer_out(L, buf), (int64_t)L.ghost, (int64_t)(GHOST - 1) * L.g.sz);
    HIP_CHECK(hipGetLastError());
    L.peer_buf = buf;
    L.x_halo_ok = true;
    L.x_peer_pending = true;
  }
  void check_device_errors() override { peer_check(); }
  // a peer wait that timed out (a neighbour never delivered) is an error, not silent stale halos
  void peer_check() {
    for (auto& L : lv_) {
      if (!L.win) continue;
      uint32_t err = 0;
      HIP_CHECK(hipMemcpyAsync(&err, peer_ctl(L.win, L) + 5, sizeof err, hipMemcpyDeviceToHost, c_->stream));
      HIP_CHECK(hipStreamSynchronize(c_->stream));
      if (err) throw CommError("peer halo: a neighbour's edge planes never arrived (wait timed out)");
    }
  }

  // ------------------------------------------------------------- kernel level
  T* arr(int l, int which) {
    LevelData<T>& L = lv_[l];
    if (which == MAD_X) return L.x;
    if (which == MAD_B) return L.b;
    return L.r;
  }

  void upload(int l, int which, const double* h) override {
    LevelData<T>& L = lv_[l];
    if (which == MAD_B) b_changed(l);
    if (which == MAD_X) x_changed(l);
    double* tmp = scratch64(L.g.N);
    HIP_CHECK(hipMemcpyAsync(tmp, h, sizeof(double) * L.g.N, hipMemcpyHostToDevice, c_->stream));
    hipLaunchKernelGGL((convert_k<double, T>), dim3(flat_blocks(L.g.N)), dim3(256), 0, c_->stream,
                       tmp, arr(l, which), L.g.N);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(c_->stream));
  }

  void download(int l, int which, double* h) override {
    peer_check();
    LevelData<T>& L = lv_[l];
    double* tmp = scratch64(L.g.N);
    hipLaunchKernelGGL((convert_k<T, double>), dim3(flat_blocks(L.g.N)), dim3(256), 0, c_->stream,
                       arr(l, which), tmp, L.g.N);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(h, tmp, sizeof(double) * L.g.N, hipMemcpyDeviceToHost, c_->stream));
    HIP_CHECK(hipStreamSynchronize(c_->stream));
  }

  void fill(int l, int which, double v) override {
    LevelData<T>& L = lv_[l];
    if (which == MAD_B) b_changed(l);
    if (which == MAD_X) x_changed(l);
    hipLaunchKernelGGL((fill_k<T>), dim3(flat_blocks(L.g.N)), dim3(256), 0, c_->stream, arr(l, which),
                       L.g.N, (T)v);
    HIP_CHECK(hipGetLastError());
  }

  void synth_level(int l, int which, uint64_t seed) override {
    LevelData<T>& L = lv_[l];
    if (which == MAD_B) b_changed(l);
    if (which == MAD_X) x_changed(l);
    const LevelGeom& G = c_->geom[l];
    hipLaunchKernelGGL((synth_image_k<T>), grid_for(L.g.nx, L.g.ny, L.g.nz, BLK), BLK, 0, c_->stream,
                       arr(l, which), L.g, G.n[0], G.n[1], seed);
    HIP_CHECK(hipGetLastError());
  }

  // halo exchange of `depth` boundary planes of one array (multi-GPU; no-op on one rank)
  // The main stream waits for every overlapped exchange still in flight.  Called
  // before any communication is issued on the main stream: RCCL operations on one
  // communicator must run in the same order on every rank, so two of them may never
  // be in flight on different streams at once.
  void wait_all_pending() {
    for (auto& L : lv_)
      if (L.x_halo_pending) {
        HIP_CHECK(hipStreamWaitEvent(c_->stream, L.ev_halo, 0));
        L.x_halo_pending = false;
      }
  }

  void halo(int l, T* a, int depth = 1) {
    if (!c_->comm.active() || !c_->geom[l].distributed) return;
    LevelData<T>& L = lv_[l];
    if (a == L.x && L.x_peer_pending) peer_resolve(l);
    wait_all_pending();
    if (a == L.x && L.x_halo_ok && depth <= GHOST) return;  // ghost planes are current
    c_->comm.exchange_planes(a, L.g.sz, L.g.nz, depth, L.g.zlo_ghost, L.g.zhi_ghost, sizeof(T),
                             std::is_same<T, double>::value, c_->stream);
    if (a == L.x && depth == GHOST) L.x_halo_ok = true;
  }

  // level l's x changed without its ghost planes (they must be exchanged again)
  // (a peer batch still in flight for x is taken in first: every batch is consumed exactly once)
  void x_changed(int l) {
    if (lv_[l].x_peer_pending) peer_resolve(l);
    lv_[l].x_halo_ok = false;
    lv_[l].x_zero_lazy = false;
  }

  // target grid size of the z-marching transfer kernels
  static constexpr int XFER_BLOCKS = 1024;
  static int xfer_blocks() { return XFER_BLOCKS; }

  // rows kept beyond the outermost plane of every level array (see setup)
  // (covers a tile region of up to 40 rows x 256 points hanging over the last plane)
  static int64_t margin_elems(const Geo& g) { return 48 * g.sy + 512; }

  bool use_fused(int l) const {
    const int v = c_->d.gs_kernel;  // 0 auto, 1 per-colour passes, 3 / 4 fused
    if (c_->dim != 3 || c_->d.smoother != MAD_GAUSS_SEIDEL) return false;
    if (v == 1) return false;
    if (v >= 2) return true;
    // auto: the fused sweep marches each tile column through z sequentially, so it
    // needs a large slab to fill the chip; below ~4M voxels one launch per colour is
    // faster (measured: 256^3 fused 0.23 ms vs 0.28 ms, 128^3 fused 0.13 vs 0.064 ms)
    const Geo& g = lv_[l].g;
#ifndef MAD_FUSED_RANK_MIN_VOXELS  // rank slabs (A/B knob, tools/rank_fused_ab.sh)
#define MAD_FUSED_RANK_MIN_VOXELS ((int64_t)4 << 20)
#define MAD_FUSED_RANK_MIN_PLANES 64
#endif
    if (c_->geom[l].distributed)
      return (int64_t)g.nx * g.ny * g.nz >= (int64_t)MAD_FUSED_RANK_MIN_VOXELS && g.nz >= MAD_FUSED_RANK_MIN_PLANES;
    return (int64_t)g.nx * g.ny * g.nz >= (int64_t)4 << 20 && g.nz >= 64;
  }

  // fused-sweep launch configuration, the measured best at 512^3 (profiles/r01_*): fp32 full
  // tensor 64x32 tiles of 1024 threads (one block per CU, 93 KB LDS), ~256 blocks (one round,
  // z-chunks of 256 planes: least chunk-overlap re-reads); fp64 full tensor 64x16 / 512 (the
  // 64x32 ring would need 186 KB of LDS); diagonal / isotropic tensors 64x16 / 1024
  struct FusedCfg {
    int blocks = 256;
  };
  // fp64 too (round 4): 256 workgroups -- at 512^3 one z-chunk per 64 x 16 tile column -- against
  // the 2048 of rounds 1-3: level-0 sweep 2.30-2.38 vs 2.77-2.96 ms, V-cycle 15.7-15.9 vs 18.0-18.6 ms
  // (512 / 1024 workgroups in between; profiles/r04_fp64_blocks_ab.log)
#ifndef MAD_FUSED_BLOCKS  // A/B knob
#define MAD_FUSED_BLOCKS 256
#endif
  static FusedCfg fused_cfg() {
    FusedCfg f;
    f.blocks = MAD_FUSED_BLOCKS;
    return f;
  }

  // z-range of one fused launch: chunks q = 0..nchunks-1 cover owned planes
  // [zbase + q*zstride, + zc)
  struct ZRange {
    int zbase, zc, zstride, nchunks;
  };
  // the whole slab in chunks sized for ~fc.blocks workgroups (at least 16 planes: a
  // 128-plane rank slab of a 256^2 level still fills the chip)
  static ZRange whole_range(int nz, int tiles, const FusedCfg& fc) {
    int chunks = (fc.blocks + tiles - 1) / tiles;
    chunks = std::max(1, std::min(chunks, std::max(1, nz / 16)));
    const int zc = (nz + chunks - 1) / chunks;
    return ZRange{0, zc, zc, (nz + zc - 1) / zc};
  }

  // parts: 0 whole slab, 1 the two boundary chunks, 2 the interior between them,
  // 3 whole slab with the last chunk marched downward and the edge-plane signals
  // (single-launch rank-slab sweep); gs_kernel 4 runs part 0 with the downward last
  // chunk (no signals)
  // z-chunks of one launch of `part` over `tiles` tiles per plane: the whole slab, or the
  // two boundary chunks of a rank slab (they produce the halo planes), or the interior
  // between them
  ZRange part_range(LevelData<T>& L, int tiles, const FusedCfg& fc, int part, int* flip,
                    uint32_t** sig) {
    const int nz = L.g.nz;
    ZRange zr = whole_range(nz, tiles, fc);
    *flip = (c_->d.gs_kernel == 4 && part == 0) ? 1 : 0;
    *sig = nullptr;
    if (part == 3 || part == 4) {
      REQUIRE(zr.nchunks >= 2 && zr.zc >= GHOST, MAD_ERR_UNSUPPORTED, "slab too thin for the single-launch sweep");
      *flip = 1;
      *sig = part == 3 ? L.sig : nullptr;
    } else if (part == 1) {
      zr = ZRange{0, boundary_planes(), nz - boundary_planes(), 2};
    } else if (part == 2) {
      const int ni = nz - 2 * boundary_planes();
      int chunks = std::max(1, std::min((fc.blocks + tiles - 1) / tiles, std::max(1, ni / 16)));
      const int zc = (ni + chunks - 1) / chunks;
      zr = ZRange{boundary_planes(), zc, zc, (ni + zc - 1) / zc};
    }
    return zr;
  }

  template <int KD, int TX, int TY, int NT>
  void launch_fused(LevelData<T>& L, const FusedCfg& fc, int part, bool zu = false) {
    const int ntx = (L.g.nx + TX - 1) / TX, nty = (L.g.ny + TY - 1) / TY;
    const int tiles = ntx * nty;
    int flip = 0;
    uint32_t* sig = nullptr;
    const ZRange zr = part_range(L, tiles, fc, part, &flip, &sig);
    const unsigned nb = (unsigned)(tiles * zr.nchunks);
    constexpr int NC = (KD == KFULL) ? 4 : 2;
    using FG = FusedGeom<NC, TX, TY>;
    constexpr size_t lds_u = sizeof(T) * FG::NP * FG::PLANE;
    REQUIRE(lds_u <= 160 * 1024, MAD_ERR_UNSUPPORTED,
            "fused GS tile needs " + std::to_string(lds_u) + " B of LDS (> 160 KiB)");
    // dense b staged through LDS where its ring fits beside the u ring (fp32; fp64 tiles do not)
    constexpr size_t lds_bl = sizeof(T) * (FG::NP + NC) * FG::PLANE;
    constexpr bool bl_fits = lds_bl <= 160 * 1024;
    const bool bl = fused_b_lds(L);
    const size_t lds = bl ? lds_bl : lds_u;
    // fp64 doubles the register footprint: 2 waves per SIMD (one 512-thread block per CU,
    // which is all its LDS allows anyway)
    constexpr int MW = sizeof(T) == 8 ? 2 : 4;
    const PeerOut<T> po = part == 4 ? peer_out(L, buffer_index(L, L.t)) : PeerOut<T>{{nullptr, nullptr}, {nullptr, nullptr}};
    auto run = [&](auto kern) {
      // every instance that can be launched gets its dynamic-LDS opt-in (a kernel pointer
      // set, not one flag per function type: several instances share one signature)
      static std::vector<const void*> attr;
      if (std::find(attr.begin(), attr.end(), (const void*)kern) == attr.end()) {
        HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds));
        attr.push_back((const void*)kern);
      }
      hipLaunchKernelGGL(kern, dim3(nb), dim3(NT), lds, c_->stream, L.x, L.t, L.bs ? L.bs : L.b, L.cf, L.g,
                         L.rat, zr.zc, ntx, nty, zr.zbase, zr.zstride, flip, sig, po);
    };
    if (part == 4) {
      if (L.brec)
        run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, true, true>);
      else if constexpr (bl_fits) {
        if (L.bs)
          run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, true, false, false, true>);
        else
          bl ? run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, true, true>)
             : run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, true>);
      } else
        run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, true>);
    } else if (L.brec) {
      run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, true>);
    } else if constexpr (bl_fits) {
      if (zu) {  // zero iterate (zero_sweep_ok: fp32 whole-slab sweeps only)
        REQUIRE(part == 0, MAD_ERR_STATE, "zero-iterate sweep on a rank slab");
        if (L.bs)
          run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, false, false, true, true>);
        else
          bl ? run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, false, true, true>)
             : run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, false, false, true>);
      } else if (L.bs) {
        run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, false, false, false, true>);
      } else {
        bl ? run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2, false, false, true>)
           : run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2>);
      }
    } else {
      REQUIRE(!zu, MAD_ERR_STATE, "zero-iterate sweep without its instance");
      run(gs_fused3_k<T, KD, TX, TY, NT, MW, 2>);
    }
  }

  // does level L's fused sweep stage its dense b through LDS (gs_fused3_k BL)?  fp32 only: the
  // fp64 tiles' u ring leaves no room for a b ring
#ifndef MAD_FUSED_B_LDS
#define MAD_FUSED_B_LDS 1
#endif
  // (level 0 only: 1249.7 vs 1279.6 us per 512^3 launch, but 195.7 vs 190.8 us at 256^3,
  // profiles/r04_bl_ab.md)
  bool fused_b_lds(const LevelData<T>& L) const {
    return MAD_FUSED_B_LDS && sizeof(T) == 4 && !L.brec && !L.bs && &L == &lv_[0];
  }

  // fp32 full-tensor fused tiles: 64 x 32 in 1024 threads (A/B knob: 16 -> 64 x 16 in 512 threads,
  // the halo-sensitivity probe of profiles/r05_tile_halo_ab.md)
#ifndef MAD_FUSED_F32_TY
#define MAD_FUSED_F32_TY 32
#endif
  // tiles per plane and z-chunks of a whole-slab fused launch at level L
  void fused_shape(const LevelData<T>& L, int* tiles, int* nchunks) const {
    const FusedCfg fc = fused_cfg();
    const int tx = 64, ty = (c_->kind == KFULL && sizeof(T) == 4) ? MAD_FUSED_F32_TY : 16;
    *tiles = ((L.g.nx + tx - 1) / tx) * ((L.g.ny + ty - 1) / ty);
    *nchunks = whole_range(L.g.nz, *tiles, fc).nchunks;
  }

  void launch_fused_part(LevelData<T>& L, int part, bool zu = false) {
    const FusedCfg fc = fused_cfg();
    if (c_->kind == KFULL) {
      if constexpr (sizeof(T) == 4)
        launch_fused<KFULL, 64, MAD_FUSED_F32_TY, MAD_FUSED_F32_TY * 32>(L, fc, part, zu);
      else
        launch_fused<KFULL, 64, 16, 512>(L, fc, part, zu);
    } else if (c_->kind == KDIAG) {
      launch_fused<KDIAG, 64, 16, 1024>(L, fc, part, zu);
    } else {
      launch_fused<KISO, 64, 16, 1024>(L, fc, part, zu);
    }
    HIP_CHECK(hipGetLastError());
  }

  // rocprof-style name of the kernel one level-l sweep launches (bench / profiles)
  std::string smooth_kernel(int l) override {
    (void)l;
    const char* tn = sizeof(T) == 4 ? "float" : "double";
    const int dim = c_->dim, kind = c_->kind;
    char buf[160];
    if (c_->d.smoother == MAD_WEIGHTED_JACOBI) {
      const LevelData<T>& L = lv_[l];
      if (dim == 3 && L.g.nx >= 16 && L.g.ny >= 16)
        std::snprintf(buf, sizeof buf, "wj3_k<%s, %d, 64, 16, %s>", tn, kind, L.brec ? "true" : "false");
      else
        std::snprintf(buf, sizeof buf, "wj_k<%s, %d, %d>", tn, dim, kind);
    } else if (c_->d.smoother == MAD_GAUSS_SEIDEL_LEX) {
      std::snprintf(buf, sizeof buf, "gs_lex_plane_k<%s, %d, %d>", tn, dim, kind);
    } else if (!use_fused(l)) {
      std::snprintf(buf, sizeof buf, "gs_color_k<%s, %d, %d>", tn, dim, kind);
      if (lv_[l].peer) return std::string(buf) + " [rank slab: peer halo, edge planes pushed after the last colour pass]";
    } else {
      const int tx = 64, ty = (kind == KFULL && sizeof(T) == 4) ? MAD_FUSED_F32_TY : 16;
      const int nt = (kind == KFULL && sizeof(T) == 8) ? 512 : (kind == KFULL ? MAD_FUSED_F32_TY * 32 : 1024);
      const bool brec = lv_[l].brec;
      const LevelData<T>& L = lv_[l];
      // every template argument, as rocprofv3 prints the instantiation (BREC, PEER, BL, ZU, BS last; the
      // zero-iterate form is only the first sweep of a refine correction cycle)
      std::snprintf(buf, sizeof buf, "gs_fused3_k<%s, %d, %d, %d, %d, %d, 2, %s, %s, %s, false, %s>", tn, kind, tx,
                    ty, nt, sizeof(T) == 8 ? 2 : 4, brec ? "true" : "false", L.peer ? "true" : "false",
                    fused_b_lds(L) ? "true" : "false", L.bs ? "true" : "false");
      // rank slabs: which sweep form fused_sweep takes
      if (L.peer) return std::string(buf) + " [rank slab: peer halo, edge planes stored by the sweep]";
      if (sweep_overlap(l)) {
        int tiles = 0, nchunks = 0;
        fused_shape(L, &tiles, &nchunks);
        const bool single = L.sig && nchunks >= 2;
        return std::string(buf) + (single ? " [rank slab: single launch, edge signals]"
                                          : " [rank slab: boundary + interior launches]");
      }
    }
    return buf;
  }

  // scatter the dense b into the records' b slot when it changed (brec levels); on a
  // rank slab the ghost planes get the neighbours' b too (exchanged first)
  void sync_brec(int l) {
    LevelData<T>& L = lv_[l];
    if (!L.brec || L.brec_ok) return;
    int p0 = 0, p1 = L.g.nz;
    if (c_->comm.active() && c_->geom[l].distributed) {
      if (!L.b_halo_ok) {
        halo(l, L.b, GHOST);
        L.b_halo_ok = true;
      }
      if (L.g.zlo_ghost) p0 = -GHOST;
      if (L.g.zhi_ghost) p1 = L.g.nz + GHOST;
    }
    dim3 gr = grid_for(L.g.nx, L.g.ny, p1 - p0, BLK);
    hipLaunchKernelGGL((brec_scatter_k<T>), gr, BLK, 0, c_->stream, L.b, L.cf, L.g, ncoef_, p0);
    HIP_CHECK(hipGetLastError());
    L.brec_ok = true;
  }
  // the fused sweep's split copy of b (LevelData::bs), ghost planes included on rank slabs
  void sync_bsplit(int l) {
    LevelData<T>& L = lv_[l];
    if (!L.bs || L.brec_ok) return;
    int p0 = 0, p1 = L.g.nz;
    if (c_->comm.active() && c_->geom[l].distributed) {
      b_halo(l);
      if (L.g.zlo_ghost) p0 = -GHOST;
      if (L.g.zhi_ghost) p1 = L.g.nz + GHOST;
    }
    dim3 gr = grid_for(L.g.nx, L.g.ny, p1 - p0, BLK);
    hipLaunchKernelGGL((bsplit_k<T>), gr, BLK, 0, c_->stream, L.b, L.bs, L.g, p0);
    HIP_CHECK(hipGetLastError());
    L.brec_ok = true;
  }

  // Does the fused sweep of rank-slab level l overlap its halo exchange (boundary chunks
  // first, the exchange beside the interior launch, or gs_kernel 4's single launch)?  Not by
  // default: one launch, then the exchange on the solver's stream.  With
  // MAD_OPT_OVERLAP_RANK_SWEEP, gs_kernel 0 splits only where the boundary launch keeps half
  // the chip busy (2 chunks x tiles per plane >= 128 workgroups): on smaller levels the
  // split's short, under-filled boundary launch costs more than the exchange it hides (a
  // 256^2-plane level at 2 ranks: 56 + 102 us per sweep split, profiles/r02_rank_vcycle.md).
  bool sweep_overlap(int l) const {
    const LevelData<T>& L = lv_[l];
    if (!(c_->comm.active() && c_->geom[l].distributed && L.g.nz >= 3 * boundary_planes()))
      return false;
    if (c_->d.gs_kernel == 4) return true;  // the single-launch form exchanges mid-sweep
    // default serial (profiles/r03_rank_serial_ab.md: per-rank sweep 0.195 vs 0.235 ms and
    // V-cycle 1.52 vs 1.81 ms at 8 ranks; a cycle graph with a communication-stream branch
    // launches every one of its ~130 nodes ~2 us slower)
    if (!(c_->d.options & MAD_OPT_OVERLAP_RANK_SWEEP)) return false;
    if (c_->d.gs_kernel != 0) return true;
    int tiles = 0, nchunks = 0;
    fused_shape(L, &tiles, &nchunks);
    return 2 * tiles >= 128;
  }

  // One fused GS sweep x -> t, then swap.  On a rank slab the next consumer of x's ghost
  // planes exchanges them (halo()), by default right after this one launch.  The overlapped
  // form (sweep_overlap): the two boundary chunks (which produce the planes the neighbours
  // need) run first, the exchange of their output then runs on the communication stream
  // while the interior chunks sweep, and the next consumer waits for it.  gs_kernel 4
  // makes the boundary and interior launches one launch instead (part 3: edge chunks
  // signal their finished edge planes to the communication stream, which waits on the
  // counters).
  float fused_sweep(int l, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
    LevelData<T>& L = lv_[l];
    halo(l, L.x, GHOST);
    if (L.brec) {
      sync_brec(l);
    } else {
      b_halo(l);
      sync_bsplit(l);
    }
    if (e0) HIP_CHECK(hipEventRecord(e0, c_->stream));
    if (L.peer) {
      // the sweep delivers its edge planes to the neighbours itself; no exchange follows
      L.peer_buf = buffer_index(L, L.t);
      launch_fused_part(L, 4);
      if (e1) HIP_CHECK(hipEventRecord(e1, c_->stream));
      std::swap(L.x, L.t);
      std::swap(L.alloc[0], L.alloc[3]);
      L.x_halo_ok = true;
      L.x_peer_pending = true;
      return 0.f;
    }
    const bool overlap = sweep_overlap(l);
    int tiles = 0, nchunks = 0;
    if (overlap) fused_shape(L, &tiles, &nchunks);
    if (overlap && L.sig && nchunks >= 2) {
      // one launch: its two edge chunks march outward-in (the top one downward) and
      // count their finished edge planes; the communication stream waits on those
      // counters and exchanges while the rest of the sweep runs
      launch_fused_part(L, 3);
      wait_all_pending();  // (none expected: halo() above already waited)
      const uint32_t target = ++L.sig_epoch * (uint32_t)tiles;
      if (L.g.zlo_ghost)
        HIP_CHECK(hipStreamWaitValue32(c_->comm_stream, L.sig, target, hipStreamWaitValueGte, 0xFFFFFFFFu));
      if (L.g.zhi_ghost)
        HIP_CHECK(hipStreamWaitValue32(c_->comm_stream, L.sig + 1, target, hipStreamWaitValueGte,
                                       0xFFFFFFFFu));
      c_->comm.exchange_planes(L.t, L.g.sz, L.g.nz, GHOST, L.g.zlo_ghost, L.g.zhi_ghost, sizeof(T),
                               std::is_same<T, double>::value, c_->comm_stream);
      HIP_CHECK(hipEventRecord(L.ev_halo, c_->comm_stream));
    } else if (!overlap) {
      // the first sweep of a refine correction cycle (x zero by construction, run_refine), or of a
      // coarse level whose descent left its zero x unwritten (x_zero_lazy)
      const bool zu = (zero_x0_ && &L == &lv_[0]) || L.x_zero_lazy;
      zero_x0_ = false;
      L.x_zero_lazy = false;
      launch_fused_part(L, 0, zu);
    } else {
      launch_fused_part(L, 1);
      wait_all_pending();  // (none expected: halo() above already waited)
      HIP_CHECK(hipEventRecord(L.ev_bnd, c_->stream));
      HIP_CHECK(hipStreamWaitEvent(c_->comm_stream, L.ev_bnd, 0));
      c_->comm.exchange_planes(L.t, L.g.sz, L.g.nz, GHOST, L.g.zlo_ghost, L.g.zhi_ghost, sizeof(T),
                               std::is_same<T, double>::value, c_->comm_stream);
      HIP_CHECK(hipEventRecord(L.ev_halo, c_->comm_stream));
      launch_fused_part(L, 2);
    }
    if (e1) HIP_CHECK(hipEventRecord(e1, c_->stream));
    std::swap(L.x, L.t);
    std::swap(L.alloc[0], L.alloc[3]);
    if (overlap) {
      L.x_halo_ok = true;
      L.x_halo_pending = true;
    } else {
      L.x_halo_ok = false;
    }
    return 0.f;
  }

  // weighted Jacobi: ghost planes / record b before the sweep, then the sweep kernel --
  // z-marching wj3_k on 3D levels of at least 16 x 16 (LDS-staged u planes), wj_k else
  void prep_wj(int l) {
    LevelData<T>& L = lv_[l];
    halo(l, L.x);
    if (L.brec) sync_brec(l);
  }
  void launch_wj(int l) {
    LevelData<T>& L = lv_[l];
    const T omega = (T)c_->d.omega;
    if (c_->dim == 3 && L.g.nx >= 16 && L.g.ny >= 16) {
      constexpr int TX = 64, TY = 16;
      const int ntx = (L.g.nx + TX - 1) / TX, nty = (L.g.ny + TY - 1) / TY;
      int chunks = std::max(1, std::min((1024 + ntx * nty - 1) / (ntx * nty), L.g.nz / 8));
      const int zc = (L.g.nz + chunks - 1) / chunks;
      chunks = (L.g.nz + zc - 1) / zc;
      const unsigned nb = (unsigned)(ntx * nty * chunks);
      auto go = [&](auto K) {
        constexpr int KD = decltype(K)::value;
        if (L.brec)
          hipLaunchKernelGGL((wj3_k<T, KD, TX, TY, true>), dim3(nb), dim3(TX * TY), 0, c_->stream,
                             L.x, L.t, L.b, L.cf, L.g, L.rat, omega, zc, ntx);
        else
          hipLaunchKernelGGL((wj3_k<T, KD, TX, TY>), dim3(nb), dim3(TX * TY), 0, c_->stream, L.x,
                             L.t, L.b, L.cf, L.g, L.rat, omega, zc, ntx);
      };
      if (c_->kind == KFULL) go(std::integral_constant<int, KFULL>{});
      else if (c_->kind == KDIAG) go(std::integral_constant<int, KDIAG>{});
      else go(std::integral_constant<int, KISO>{});
    } else {
      dispatch(c_->dim, c_->kind, [&](auto D, auto K) {
        hipLaunchKernelGGL((wj_k<T, D.value, K.value>), grid_for(L.g.nx, L.g.ny, L.g.nz, BLK), BLK,
                           0, c_->stream, L.x, L.t, L.b, L.cf, L.g, L.rat, omega);
      });
    }
    HIP_CHECK(hipGetLastError());
  }

  // per-colour GS on a 3D rank slab with one halo exchange per sweep
  bool colour_ca(int l) const {
    return c_->dim == 3 && c_->comm.active() && c_->geom[l].distributed &&
           c_->ncolors <= GHOST;
  }

  void smooth(int l, unsigned n) override {
    LevelData<T>& L = lv_[l];
    const int dim = c_->dim;
    const int sm = c_->d.smoother;
    for (unsigned s = 0; s < n; ++s) {
      if (sm == MAD_WEIGHTED_JACOBI) {
        prep_wj(l);
        launch_wj(l);
        std::swap(L.x, L.t);
        std::swap(L.alloc[0], L.alloc[3]);
        x_changed(l);
      } else if (sm == MAD_GAUSS_SEIDEL_LEX) {
        REQUIRE(!c_->comm.active(), MAD_ERR_UNSUPPORTED,
                "lexicographic GS is a single-GPU parity mode");
        const int tmax = (L.g.nx - 1) + 2 * (L.g.ny - 1) + (dim == 3 ? 3 * (L.g.nz - 1) : 0);
        dim3 gr((unsigned)((L.g.ny + 255) / 256), (unsigned)(dim == 3 ? L.g.nz : 1), 1);
        for (int t = 0; t <= tmax; ++t) {
          dispatch(dim, c_->kind, [&](auto D, auto K) {
            hipLaunchKernelGGL((gs_lex_plane_k<T, D.value, K.value>), gr, dim3(256), 0, c_->stream,
                               L.x, L.b, L.cf, L.g, L.rat, t);
          });
        }
        HIP_CHECK(hipGetLastError());
      } else if (use_fused(l)) {
        fused_sweep(l);
      } else {
        const int nc = c_->ncolors;
        const int rows = (nc == 4) ? (L.g.ny + 1) / 2 : L.g.ny;
        if (colour_ca(l)) {
          // rank slab: one exchange of nc ghost planes per sweep instead of one plane per
          // colour; colour c is computed on the owned planes plus the nc - 1 - c nearest
          // ghost planes (the values the neighbour computes, from the same inputs: the
          // outermost of them reads ghost plane nc), so every later colour finds its ghost
          // neighbours updated -- the fused sweep's scheme
          halo(l, L.x, nc);
          b_halo(l);
          for (int col = 0; col < nc; ++col) {
            const int ext = nc - 1 - col;
            const int k0 = L.g.zlo_ghost ? -ext : 0, k1 = L.g.nz + (L.g.zhi_ghost ? ext : 0);
            dim3 gr = grid_for((L.g.nx + 1) / 2, rows, k1 - k0, BLK);
            dispatch(dim, c_->kind, [&](auto D, auto K) {
              hipLaunchKernelGGL((gs_color_k<T, D.value, K.value>), gr, BLK, 0, c_->stream, L.x, L.b,
                                 L.cf, L.g, L.rat, col, nc, k0);
            });
          }
          if (L.peer)
            peer_push(l);
          else
            x_changed(l);
        } else {
          dim3 gr = grid_for((L.g.nx + 1) / 2, rows, L.g.nz, BLK);
          for (int col = 0; col < nc; ++col) {
            halo(l, L.x);
            dispatch(dim, c_->kind, [&](auto D, auto K) {
              hipLaunchKernelGGL((gs_color_k<T, D.value, K.value>), gr, BLK, 0, c_->stream, L.x,
                                 L.b, L.cf, L.g, L.rat, col, nc, 0);
            });
            x_changed(l);
          }
        }
        HIP_CHECK(hipGetLastError());
      }
    }
  }

  double finish_norm2(int64_t nparts, bool global) {
    hipLaunchKernelGGL(reduce_final_k, dim3(1), dim3(256), 0, c_->stream, part_, nparts, scal_);
    HIP_CHECK(hipGetLastError());
    if (global && c_->comm.active()) {
      wait_all_pending();
      c_->comm.allreduce_sum_f64(scal_, 1, c_->stream);
    }
    HIP_CHECK(hipMemcpyAsync(hscal_, scal_, sizeof(double), hipMemcpyDeviceToHost, c_->stream));
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    return hscal_[0];
  }

  double residual(int l, bool want_norm) override { return residual_impl(l, want_norm, true); }

  // fp64 residual of the refined level-0 system: r64 = b64 - A64 u64 (+ ||r||^2 partials),
  // the reference operator in fp64 (coefficient records cf64_, g from the fp64 tensor).  3D
  // levels of >= 16 x 16 write the fp32 hierarchy's next rhs b = (T) r and x = 0 in the same
  // pass instead of r64 (refine_emitted_; else run_refine converts r64 and fills x)
  bool refine_emitted_ = false;
  bool refine_emitted_bs_ = false;  // ... and the split copy of b (LevelData::bs) with it
  // fold: u += (double) x (the fp32 cycle's correction) in the same pass -- one GPU, resid3_k levels:
  // the updated iterate goes to the second fp64 buffer (r64_, unused by this path) and the pointers
  // swap; x = 0 is then a separate fill (neighbouring tiles read x while the pass runs)
  bool refine_fold_ok() const {
    const LevelData<T>& L = lv_[0];
    return c_->dim == 3 && L.g.nx >= 16 && L.g.ny >= 16 && !c_->geom[0].distributed;
  }
  // zero iterate: the next V-cycle's first level-0 sweep reads x as zero without loading it
  // (gs_fused3_k ZU), so the folded refine pass leaves x as it is instead of filling it --
  // only where that sweep is the first thing of the cycle to touch x: a fused fp32 whole-slab
  // sweep at level 0 of a multi-level V-cycle, with pre-smoothing, on one GPU
  bool zero_x0_ = false;
  // a V-cycle descent into level l (>= 1) may leave x[l] unwritten: its first sweep is a fused fp32
  // whole-slab one-GPU sweep (the ZU instance) and nothing reads x[l] before it (pre-smoothing, not
  // verbose, not the coarsest)
  bool lazy_zero_ok(int l) const {
#ifdef MAD_NO_LAZY_ZERO
    return false;
#else
    const auto& d = c_->d;
    return sizeof(T) == 4 && l >= 1 && l < c_->nlev - 1 && !c_->comm.active() && !d.verbose &&
           d.iterations_per_grid >= 1 && use_fused(l) && d.gs_kernel != 4 && !lv_[l].brec &&
           c_->dim == 3;
#endif
  }
  bool zero_sweep_ok() const {
#ifdef MAD_NO_ZERO_SWEEP
    return false;
#else
    const auto& d = c_->d;
    return sizeof(T) == 4 && refine_fold_ok() && !c_->comm.active() && d.cycle == MAD_VCYCLE &&
           !d.verbose && d.iterations_per_grid >= 1 && c_->nlev > 1 && use_fused(0) && d.gs_kernel != 4 &&
           !lv_[0].brec;
#endif
  }
  double residual64(bool fold = false) {
    LevelData<T>& L = lv_[0];
    if (fold && !refine_fold_ok()) {
      hipLaunchKernelGGL((add_conv_k<T>), dim3(flat_blocks(L.g.N)), dim3(256), 0, c_->stream, u64_, L.x, L.g.N);
      HIP_CHECK(hipGetLastError());
      fold = false;
    }
    if (c_->comm.active() && c_->geom[0].distributed) {
      wait_all_pending();
      c_->comm.exchange_planes(u64_, L.g.sz, L.g.nz, 1, L.g.zlo_ghost, L.g.zhi_ghost, sizeof(double),
                               true, c_->stream);
    }
    Geo g = L.g;
    g.rs = ncoef_;
    int64_t nparts = 0;
    if (c_->dim == 3 && g.nx >= 16 && g.ny >= 16) {
      constexpr int TX = 64, TY = 16;
      const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
      int chunks = std::max(1, std::min((1024 + ntx * nty - 1) / (ntx * nty), g.nz / 8));
      const int zc = (g.nz + chunks - 1) / chunks;
      chunks = (g.nz + zc - 1) / zc;
      nparts = (int64_t)ntx * nty * chunks;
      REQUIRE(nparts <= part_cap_, MAD_ERR_UNSUPPORTED, "residual partials buffer too small");
      // one GPU: the fused sweep's split copy of b written in the same pass (rank slabs refresh it,
      // ghost planes included, from the dense b: sync_bsplit)
      T* const bse = (L.bs && !c_->geom[0].distributed) ? L.bs : nullptr;
      refine_emitted_bs_ = bse != nullptr;
      auto go = [&](auto K) {
        constexpr int KD = decltype(K)::value;
        auto launch = [&](auto bptr) {
          using TB = std::remove_const_t<std::remove_pointer_t<decltype(bptr)>>;
          if (fold)
            hipLaunchKernelGGL((resid3_k<double, KD, TX, TY, false, T, TB>), dim3((unsigned)nparts),
                               dim3(TX * TY), 0, c_->stream, u64_, bptr, (double*)nullptr, cf64_, g, rat64_, zc,
                               ntx, part_, L.b, (T*)nullptr, (const T*)L.x, r64_, bse);
          else
            hipLaunchKernelGGL((resid3_k<double, KD, TX, TY, false, T, TB>), dim3((unsigned)nparts),
                               dim3(TX * TY), 0, c_->stream, u64_, bptr, (double*)nullptr, cf64_, g, rat64_, zc,
                               ntx, part_, L.b, L.x, (const T*)nullptr, (double*)nullptr, bse);
        };
#ifdef MAD_NO_B32_RHS  // A/B: always the fp64 rhs
        launch((const double*)b64_);
#else
        if (b32_exact_)
          launch((const float*)b32_);
        else
          launch((const double*)b64_);
#endif
      };
      refine_emitted_ = true;
      if (c_->kind == KFULL) go(std::integral_constant<int, KFULL>{});
      else if (c_->kind == KDIAG) go(std::integral_constant<int, KDIAG>{});
      else go(std::integral_constant<int, KISO>{});
      if (fold) {
        std::swap(u64_, r64_);
        if (!zero_sweep_ok())
          hipLaunchKernelGGL((fill_k<T>), dim3(flat_blocks(L.g.N)), dim3(256), 0, c_->stream, L.x, L.g.N, T(0));
      }
    } else {
      dim3 gr = grid_for(g.nx, g.ny, g.nz, BLK);
      nparts = (int64_t)gr.x * gr.y * gr.z;
      REQUIRE(nparts <= part_cap_, MAD_ERR_UNSUPPORTED, "residual partials buffer too small");
      dispatch(c_->dim, c_->kind, [&](auto D, auto K) {
        hipLaunchKernelGGL((residual_k<double, D.value, K.value>), gr, BLK, 0, c_->stream, u64_, b64_,
                           r64_, cf64_, g, rat64_, part_);
      });
      refine_emitted_ = refine_emitted_bs_ = false;
    }
    HIP_CHECK(hipGetLastError());
    return std::sqrt(finish_norm2(nparts, c_->geom[0].distributed));
  }

  double norm64(const double* a) {
    const int64_t n = lv_[0].g.N;
    unsigned nb = flat_blocks(n, 2048);
    hipLaunchKernelGGL((sumsq_k<double>), dim3(nb), dim3(256), 0, c_->stream, a, n, part_);
    HIP_CHECK(hipGetLastError());
    return std::sqrt(finish_norm2(nb, c_->geom[0].distributed));
  }

  // write_r false: only ||r|| is wanted (the per-cycle convergence test), r is not
  // stored (z-marching path; the per-point fallback always stores it)
  double residual_impl(int l, bool want_norm, bool write_r) {
    LevelData<T>& L = lv_[l];
    halo(l, L.x);
    int64_t nparts = 0;
    if (c_->dim == 3 && L.g.nx >= 16 && L.g.ny >= 16) {
      // z-marching residual (resid3_k): 64x16 columns, chunks sized for ~1024 blocks
      constexpr int TX = 64, TY = 16;
      const int ntx = (L.g.nx + TX - 1) / TX, nty = (L.g.ny + TY - 1) / TY;
      int chunks = std::max(1, std::min((1024 + ntx * nty - 1) / (ntx * nty), L.g.nz / 8));
      const int zc = (L.g.nz + chunks - 1) / chunks;
      chunks = (L.g.nz + zc - 1) / zc;
      nparts = (int64_t)ntx * nty * chunks;
      REQUIRE(nparts <= part_cap_, MAD_ERR_UNSUPPORTED, "residual partials buffer too small");
      sync_brec(l);
      auto go = [&](auto K) {
        constexpr int KD = decltype(K)::value;
        T* rout = write_r ? L.r : nullptr;
        if (L.brec)
          hipLaunchKernelGGL((resid3_k<T, KD, TX, TY, true>), dim3((unsigned)nparts),
                             dim3(TX * TY), 0, c_->stream, L.x, L.b, rout, L.cf, L.g, L.rat, zc, ntx,
                             want_norm ? part_ : nullptr);
        else
          hipLaunchKernelGGL((resid3_k<T, KD, TX, TY>), dim3((unsigned)nparts), dim3(TX * TY), 0,
                             c_->stream, L.x, L.b, rout, L.cf, L.g, L.rat, zc, ntx,
                             want_norm ? part_ : nullptr);
      };
      if (c_->kind == KFULL) go(std::integral_constant<int, KFULL>{});
      else if (c_->kind == KDIAG) go(std::integral_constant<int, KDIAG>{});
      else go(std::integral_constant<int, KISO>{});
    } else {
      dim3 gr = grid_for(L.g.nx, L.g.ny, L.g.nz, BLK);
      nparts = (int64_t)gr.x * gr.y * gr.z;
      dispatch(c_->dim, c_->kind, [&](auto D, auto K) {
        hipLaunchKernelGGL((residual_k<T, D.value, K.value>), gr, BLK, 0, c_->stream, L.x, L.b,
                           L.r, L.cf, L.g, L.rat, want_norm ? part_ : nullptr);
      });
    }
    HIP_CHECK(hipGetLastError());
    if (!want_norm) return 0.0;
    return std::sqrt(finish_norm2(nparts, c_->geom[l].distributed));
  }

  double norm(int l, int which) override {
    LevelData<T>& L = lv_[l];
    unsigned nb = flat_blocks(L.g.N, 2048);
    hipLaunchKernelGGL((sumsq_k<T>), dim3(nb), dim3(256), 0, c_->stream, arr(l, which), L.g.N, part_);
    HIP_CHECK(hipGetLastError());
    return std::sqrt(finish_norm2(nb, c_->geom[l].distributed));
  }

  // b[l+1] <- R r[l]   (IGO.hxx:175-304)
  void restrict_(int l) override { restrict_arr(l, lv_[l].r, lv_[l + 1].b); }

  // b[l+1] <- R (b[l] - A x[l]) in one pass (resid_restrict3_k, bit-identical to the
  // residual + restriction pair; r[l] is not written).  3D levels held whole by this
  // rank (one GPU, or the replicated coarse levels); false: not applicable, the caller
  // runs residual + restriction.
  bool residual_restrict(int l) override { return resid_restrict(l); }
  // zero_x: also zero x[l+1] (the V-cycle descent's fill, folded into the same pass)
#ifndef MAD_RR_SMALL_VOXELS
#define MAD_RR_SMALL_VOXELS 65536
#endif
  bool resid_restrict(int l, bool zero_x = false) {
    LevelData<T>& F = lv_[l];
    LevelData<T>& C = lv_[l + 1];
    // one GPU (or a replicated level), or a rank slab whose coarse level is a slab too (the
    // taps past the slab residualise the fine ghost planes: x and b ghost planes made current
    // first -- the b exchange stands in for the residual's)
    const bool dist = c_->geom[l].distributed;
    // the agglomeration hand-over (distributed l, replicated l + 1) where the z coarsening is
    // cell-centred and splits evenly: every rank restricts its own slab into its coarse planes
    // (a slab view of the coarse level), then the ranks all-gather those -- 1/8 of the bytes of the
    // fine residual the other path gathers, and one pass instead of residual + restriction
    const LevelGeom& Gc = c_->geom[l + 1];
    const bool handover = dist && !Gc.distributed && C.cent[2] == 1 && F.g.nz % 2 == 0 &&
                          F.g.zoff % 2 == 0 && (int64_t)(F.g.nz / 2) * c_->comm.nranks() == (int64_t)Gc.n[2];
    if (c_->dim != 3 || (dist != Gc.distributed && !handover) || F.g.nx < 16 || F.g.ny < 16 || F.g.nz < 2)
      return false;
    if (dist) {
      halo(l, F.x, GHOST);
      if (!F.brec) b_halo(l);
    }
    sync_brec(l);
    b_changed(l + 1);
    T* zx = (zero_x && !handover) ? C.x : nullptr;
    if (zx && C.x_peer_pending) peer_resolve(l + 1);  // (consumed before the zeros land on its ghost planes)
    if (zx && lazy_zero_ok(l + 1)) {  // the coarse level's first sweep takes x as zero without loading it
      zx = nullptr;
      C.x_zero_lazy = true;
    }
    // the kernel zeroes a rank slab's coarse x ghost planes too (the neighbours' zeros)
    if (zero_x && !handover) C.x_halo_ok = dist;
    // where the coarse planes go: the coarse level, or (hand-over) this rank's planes of it
    T* cb = C.b;
    Geo gcv = C.g;
    if (handover) {
      gcv.nz = F.g.nz / 2;
      gcv.zoff = F.g.zoff / 2;
      gcv.N = gcv.sz * gcv.nz;
      gcv.zlo_ghost = gcv.zhi_ghost = 0;
      cb = coarse_slab((int64_t)gcv.N);
    }
    // 32 x 8 coarse tiles in 512-thread blocks, two per CU (one block's barriers overlap the
    // other's loads), ~1024 blocks: 1.133 vs 1.177 ms per 512^3 launch with 1024-thread blocks
    // (profiles/r01_rr_nt_prof.log, r01_rr_blocks_prof.log)
    constexpr int target = 1024;
    const int ncz = (int)c_->geom[l + 1].n[2];  // global coarse nz (taps in global indices)
    auto run = [&](auto CXc, auto CYc, auto NTc) {
      constexpr int CX = decltype(CXc)::value, CY = decltype(CYc)::value, NT = decltype(NTc)::value;
      const int ntx = (gcv.nx + CX - 1) / CX, nty = (gcv.ny + CY - 1) / CY;
      // small coarse levels (<= 65536 voxels): one coarse plane per workgroup (a few tiles per plane
      // cannot fill the chip, and each z-step of the march is a serial round trip): 8^3..32^3 descents
      // 17.7 / 19.3 / 21.3 -> 9.6 / 9.7 / 10.9 us; at 64^3 it costs (27.2 -> 36.4 us), so 4 planes stay
      // the minimum there (profiles/r04_rr_chunk_ab.md)
      const int zdiv = gcv.N <= MAD_RR_SMALL_VOXELS ? 1 : 4;
      int chunks = std::max(1, std::min((target + ntx * nty - 1) / (ntx * nty), gcv.nz / zdiv));
      const int kc = (gcv.nz + chunks - 1) / chunks;
      chunks = (gcv.nz + kc - 1) / kc;
      const dim3 grid((unsigned)(ntx * nty * chunks)), block(NT);
      auto go = [&](auto K) {
        constexpr int KD = decltype(K)::value;
        if (F.brec)
          hipLaunchKernelGGL((resid_restrict3_k<T, KD, CX, CY, NT, true>), grid, block, 0, c_->stream,
                             F.x, F.b, F.cf, F.g, F.rat, cb, zx, gcv, C.cent[0], C.cent[1], C.cent[2],
                             kc, ntx, F.g.zoff, ncz);
        else
          hipLaunchKernelGGL((resid_restrict3_k<T, KD, CX, CY, NT>), grid, block, 0, c_->stream, F.x,
                             F.b, F.cf, F.g, F.rat, cb, zx, gcv, C.cent[0], C.cent[1], C.cent[2], kc,
                             ntx, F.g.zoff, ncz);
      };
      if (c_->kind == KFULL) go(std::integral_constant<int, KFULL>{});
      else if (c_->kind == KDIAG) go(std::integral_constant<int, KDIAG>{});
      else go(std::integral_constant<int, KISO>{});
    };
    // (32 x 16 and 64 x 8 coarse tiles -- ~6 % fewer halo re-reads -- measured within the noise
    // of 32 x 8 per V-cycle, profiles/r03_rr_tile_ab.log)
    run(std::integral_constant<int, 32>{}, std::integral_constant<int, 8>{},
        std::integral_constant<int, 512>{});
    HIP_CHECK(hipGetLastError());
    if (handover) {
      wait_all_pending();
      c_->comm.allgather_slabs(cb, C.b, (int64_t)gcv.nx * gcv.ny, (int64_t)Gc.n[2], sizeof(T), c_->stream);
      if (zero_x) fill(l + 1, MAD_X, 0.0);
    }
    if (dist && C.peer) peer_push_b(l + 1);  // the neighbours' b ghost planes, no exchange
    return true;
  }

  void restrict_arr(int l, T* fine, T* coarse) {
    LevelData<T>& F = lv_[l];
    LevelData<T>& C = lv_[l + 1];
    b_changed(l + 1);
    REQUIRE(!c_->geom[l].distributed || c_->geom[l + 1].distributed, MAD_ERR_UNSUPPORTED,
            "restriction onto a replicated level");
    halo(l, fine);
    const int fz_shift = (c_->dim == 3) ? F.g.zoff : 0;
    dim3 gr = grid_for(C.g.nx, C.g.ny, C.g.nz, BLK);
    Geo gc = C.g;
    if (c_->dim == 3) gc.zoff = C.g.zoff;
    if (c_->dim == 3) {
      // z-marching (restrict3_k): 32x8 coarse columns, ~1024 blocks
      constexpr int CX = 32, CY = 8;
      const int ntx = (C.g.nx + CX - 1) / CX, nty = (C.g.ny + CY - 1) / CY;
      int chunks = std::max(1, std::min((xfer_blocks() + ntx * nty - 1) / (ntx * nty), C.g.nz / 4));
      const int kc = (C.g.nz + chunks - 1) / chunks;
      chunks = (C.g.nz + kc - 1) / kc;
      hipLaunchKernelGGL((restrict3_k<T, T, CX, CY>), dim3((unsigned)(ntx * nty * chunks)),
                         dim3(CX * CY), 0, c_->stream, fine, F.g, coarse, gc, C.cent[0], C.cent[1],
                         C.cent[2], fz_shift, (int)c_->geom[l + 1].n[2], kc, ntx);
      (void)gr;
    } else {
      hipLaunchKernelGGL((restrict_k<T, T, 2>), gr, BLK, 0, c_->stream, fine, F.g, coarse, C.g,
                         C.cent[0], C.cent[1], C.cent[2], 0);
    }
    HIP_CHECK(hipGetLastError());
  }

  // x[l] (+)= P x[l+1]   (IGO.hxx:45-172, MAD.hxx:422-435)
  void interpolate(int l, bool add) override {
    LevelData<T>& F = lv_[l];
    LevelData<T>& C = lv_[l + 1];
    const bool ghosts = interp_ghosts(l, add);
    halo(l + 1, C.x, ghosts ? 3 : 1);  // fine ghost planes reach 3 coarse planes out
    dim3 gr = grid_for(F.g.nx, F.g.ny, F.g.nz, BLK);
    if (c_->dim == 3) {
      launch_interp3(l, add, ghosts);
      if (ghosts) F.x_halo_ok = true;
      else x_changed(l);
    } else {
      if (add)
        hipLaunchKernelGGL((interp_k<T, 2, 1>), gr, BLK, 0, c_->stream, C.x, C.g, F.x, F.g,
                           C.cent[0], C.cent[1], C.cent[2]);
      else
        hipLaunchKernelGGL((interp_k<T, 2, 0>), gr, BLK, 0, c_->stream, C.x, C.g, F.x, F.g,
                           C.cent[0], C.cent[1], C.cent[2]);
    }
    HIP_CHECK(hipGetLastError());
  }

  // DS.hxx:91-147
  void coarse_solve() override {
    const int l = c_->nlev - 1;
    LevelData<T>& L = lv_[l];
    const int n = (int)L.g.N;
    REQUIRE(!c_->geom[l].distributed, MAD_ERR_UNSUPPORTED, "coarsest level must be replicated");
    if (cblk_.active())
      cblk_.solve<T>(L.b, L.x, c_->stream);  // large coarsest level: block-plane LU (mad_coarse.hpp)
    else
      hipLaunchKernelGGL((coarse_solve_k<T>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0, c_->stream,
                         inv_, L.b, L.x, n);
    HIP_CHECK(hipGetLastError());
  }

  // ------------------------------------------------------------- cycles
  void vcycle_rec(int l) {
    const int nl = c_->nlev;
    if (l == nl - 1) {  // MAD.hxx:356-371
      coarse_solve();
      if (c_->d.verbose) (void)verbose_line(l, -1, "direct solver");
      return;
    }
    const unsigned nu = c_->d.iterations_per_grid;
    const bool bt = l == 0 && c_->bench_trace() && c_->trace_active;  // MAD.hxx:401-409
    if (c_->d.verbose || bt) {
      for (unsigned n = 0; n < nu; ++n) {
        smooth(l, 1);
        per_sweep_line(l, (int)n + 1, nullptr, bt);
      }
    } else {
      smooth(l, nu);  // MAD.hxx:384-411
    }
    if (!resid_restrict(l, true)) {  // x[l+1] zeroed in the same pass
      residual(l, false);  // MAD.hxx:389 (after the last pre-smoothing sweep)
      restrict_down(l);    // MAD.hxx:413
      fill(l + 1, MAD_X, 0.0);  // MAD.hxx:415-416
    }
    vcycle_rec(l + 1);        // MAD.hxx:418-420
    interpolate_up(l, true);  // MAD.hxx:422-435
    if (c_->d.verbose || bt) per_sweep_line(l, 0, "initial", bt);  // MAD.hxx:450-458
    if (c_->d.verbose || bt) {
      for (unsigned n = 0; n < nu; ++n) {
        smooth(l, 1);
        per_sweep_line(l, (int)n + 1, nullptr, bt);  // MAD.hxx:477-485
      }
    } else {
      smooth(l, nu);  // MAD.hxx:460-487
    }
  }

  // restriction / interpolation between a level and the next coarser one,
  // including the hand-over from distributed slabs to a replicated level
  void restrict_down(int l) {
    if (c_->geom[l].distributed && !c_->geom[l + 1].distributed) {
      gather_level(l, lv_[l].r);
      restrict_full(l, gathered_, lv_[l + 1].b);
    } else {
      restrict_arr(l, lv_[l].r, lv_[l + 1].b);
    }
  }

  void restrict_rhs_down(int l) {
    if (c_->geom[l].distributed && !c_->geom[l + 1].distributed) {
      gather_level(l, lv_[l].b);
      restrict_full(l, gathered_, lv_[l + 1].b);
    } else {
      restrict_arr(l, lv_[l].b, lv_[l + 1].b);
    }
  }

  void interpolate_up(int l, bool add) {
    if (c_->geom[l].distributed && !c_->geom[l + 1].distributed) {
      interp_from_replicated(l, add);
    } else {
      interpolate(l, add);
    }
  }

  // MAD.hxx:300-338 (rhs already in b[l])
  void fmg_rec(int l) {
    const int nl = c_->nlev;
    if (l == nl - 1) {
      fill(l, MAD_X, 0.0);
    } else {
      restrict_rhs_down(l);
      fmg_rec(l + 1);
      interpolate_up(l, false);
    }
    for (unsigned n = 0; n < c_->d.iterations_per_grid; ++n) vcycle_rec(l);
  }

  // One V-cycle from level 0, replayed from a captured hipGraph when possible: the
  // cycle is ~40 launches per level and the coarse levels are launch-bound.  The
  // graph bakes in the array pointers, so it is only used when a cycle leaves the
  // ping-pong state (x <-> t swaps of the fused sweep) unchanged, i.e. an even
  // number of fused sweeps per level, and re-captured when a call between cycles
  // swapped a pair.  Verbose runs stay eager (host norms per sweep).
  //
  // Rank slabs over RCCL are captured too: the halo exchanges (grouped
  // ncclSend/ncclRecv), the slab allgather of the agglomeration and the
  // communication-stream overlap of the fused sweep (event fork / join) are all
  // stream-ordered, so one graph per rank holds the whole cycle.  The host's
  // ghost-plane bookkeeping is made canonical around the graph: level 0's x / b ghost
  // planes are made current eagerly before every capture and replay (a no-op when they
  // are), the cycle ends joined (no exchange left in flight), and the bookkeeping the
  // capture left behind is re-applied after every replay.  The first multi-rank cycle
  // runs eagerly (RCCL connects its peers lazily, outside any capture).  The
  // in-process LOCAL transport synchronises on the host and stays eager, as does the
  // wait-on-value single-launch sweep (gs_kernel 4); mad_desc.options MAD_OPT_EAGER_RANK_VCYCLE
  // keeps the multi-rank V-cycle eager (the reference for the graph-replay parity test).
  bool vgraph_ranks_ok() const {
    return !(c_->d.options & MAD_OPT_EAGER_RANK_VCYCLE) &&
           (c_->comm.mode() == Comm::RCCL || c_->comm.mode() == Comm::SOLO) && c_->d.gs_kernel != 4;
  }

  struct HaloFlags {
    bool x_ok, b_ok, brec_ok;
  };
  std::vector<HaloFlags> halo_flags() const {
    std::vector<HaloFlags> v;
    for (auto& L : lv_) v.push_back({L.x_halo_ok, L.b_halo_ok, L.brec_ok});
    return v;
  }
  // canonical entry state of a multi-rank graph cycle (host bookkeeping + level 0's
  // ghost planes made current on the stream)
  void ranks_graph_entry() {
    peer_resolve_all();
    // level 0's x ghost planes: a peer level has them (resolved above); otherwise the graph exchanges
    // them itself (its first sweep), so no eager RCCL call sits between two replays -- such a call
    // must first wait for the previous replay (Comm::settle), which would stall the pipeline
    if (lv_[0].peer)
      halo(0, lv_[0].x, GHOST);
    else
      lv_[0].x_halo_ok = false;
    if (!lv_[0].brec && !lv_[0].b_halo_ok) {
      halo(0, lv_[0].b, GHOST);
      lv_[0].b_halo_ok = true;
    }
    wait_all_pending();
    for (size_t l = 1; l < lv_.size(); ++l) {
      lv_[l].x_halo_ok = false;
      lv_[l].b_halo_ok = lv_[l].brec_ok = false;
    }
  }

  void vcycle_fast() {
    const bool ranks = c_->comm.active();
    if (c_->d.verbose || c_->bench_trace() || vgraph_failed_ || (ranks && !vgraph_ranks_ok()) ||
        (ranks && vcycles_eager_ < 1)) {
      if (ranks) ++vcycles_eager_;
      vcycle_rec(0);
      return;
    }
    sync_brec(0);  // eager: level 0's b changes between cycles (time steps), not inside
    sync_bsplit(0);
    if (ranks) ranks_graph_entry();
    const bool zu = zero_x0_;  // the graph bakes in the first sweep's zero-iterate form too
    if (vgraph_) {
      // the graph baked in every level's x / t buffers: a call between two cycles that
      // swapped a ping-pong pair an odd number of times (mad_smooth with an odd sweep
      // count under WJ, or of the fused GS sweep) leaves it pointing at stale buffers,
      // so it is re-captured for the current pointers
      bool same = vgraph_ptrs_.size() == lv_.size() && vgraph_zu_ == zu;
      for (size_t l = 0; same && l < lv_.size(); ++l)
        same = vgraph_ptrs_[l].first == lv_[l].x && vgraph_ptrs_[l].second == lv_[l].t &&
               vgraph_seq_[l] == (lv_[l].peer_seq & 1);  // per-colour peer levels: mailbox parity
      if (!same) {
        HIP_CHECK(hipStreamSynchronize(c_->stream));
        (void)hipGraphExecDestroy(vgraph_);
        vgraph_ = nullptr;
      }
    }
    if (!vgraph_) {
      struct Snap {
        T* x;
        T* t;
        T* a0;
        T* a3;
        bool bh;
        int seq;
      };
      auto snap = [&] {
        std::vector<Snap> v;
        for (auto& L : lv_) v.push_back({L.x, L.t, L.alloc[0], L.alloc[3], L.b_halo_ok, L.peer_seq});
        return v;
      };
      auto restore = [&](const std::vector<Snap>& v) {
        for (size_t l = 0; l < lv_.size(); ++l) {
          lv_[l].x = v[l].x;
          lv_[l].t = v[l].t;
          lv_[l].alloc[0] = v[l].a0;
          lv_[l].alloc[3] = v[l].a3;
          lv_[l].b_halo_ok = v[l].bh;
          lv_[l].peer_seq = v[l].seq;
        }
      };
      const std::vector<Snap> before = snap();
      const std::vector<HaloFlags> flags_before = halo_flags();
      hipGraph_t gph = nullptr;
      HIP_CHECK(hipStreamBeginCapture(c_->stream, hipStreamCaptureModeThreadLocal));
      bool captured = true;
      try {
        vcycle_rec(0);
        if (ranks) {
          wait_all_pending();  // join the communication stream: no open branch
          peer_resolve_all();  // and no peer batch left to take in
        }
      } catch (...) {
        (void)hipStreamEndCapture(c_->stream, &gph);
        if (gph) (void)hipGraphDestroy(gph);
        gph = nullptr;
        restore(before);
        if (!ranks) throw;
        captured = false;  // a transport that refuses capture: eager from here on
      }
      if (captured && hipStreamEndCapture(c_->stream, &gph) != hipSuccess) {
        gph = nullptr;
        captured = false;
      }
      const std::vector<Snap> after = snap();
      bool same = captured;
      // (a cycle pushes a per-colour peer level's batches an even number of times, 2 nu: a replay
      // leaves the mailbox parity where the capture found it)
      for (size_t l = 0; same && l < before.size(); ++l)
        same = before[l].x == after[l].x && before[l].t == after[l].t &&
               ((before[l].seq ^ after[l].seq) & 1) == 0;
      vgraph_exit_flags_ = halo_flags();  // the bookkeeping one cycle leaves
      restore(before);  // capture issued nothing: the state must not advance
      if (ranks) {
        for (size_t l = 0; l < lv_.size(); ++l) {
          lv_[l].x_halo_ok = flags_before[l].x_ok;
          lv_[l].b_halo_ok = flags_before[l].b_ok;
          lv_[l].brec_ok = flags_before[l].brec_ok;
          lv_[l].x_halo_pending = false;
        }
      }
      if (same && hipGraphInstantiate(&vgraph_, gph, nullptr, nullptr, 0) != hipSuccess) {
        vgraph_ = nullptr;
        same = false;
      }
      if (gph) (void)hipGraphDestroy(gph);
      zero_x0_ = zu;  // (consumed by the capture)
      if (!same) {
        (void)hipGetLastError();
        vgraph_failed_ = true;
        vcycle_rec(0);
        return;
      }
      vgraph_zu_ = zu;
      zero_x0_ = false;
      vgraph_ptrs_.clear();
      vgraph_seq_.clear();
      for (auto& L : lv_) {
        vgraph_ptrs_.emplace_back(L.x, L.t);
        vgraph_seq_.push_back(L.peer_seq & 1);
      }
    }
    HIP_CHECK(hipGraphLaunch(vgraph_, c_->stream));
    zero_x0_ = false;
    if (ranks) c_->comm.graph_launched(c_->stream);
    if (ranks) {
      for (size_t l = 0; l < lv_.size(); ++l) {
        lv_[l].x_halo_ok = vgraph_exit_flags_[l].x_ok;
        lv_[l].b_halo_ok = vgraph_exit_flags_[l].b_ok;
        lv_[l].brec_ok = vgraph_exit_flags_[l].brec_ok;
        lv_[l].x_halo_pending = false;
      }
    } else {
      for (size_t l = 1; l < lv_.size(); ++l) lv_[l].b_halo_ok = lv_[l].brec_ok = false;  // as eager
    }
  }

  void vcycle() override { vcycle_fast(); }

  void fmg() override { fmg_rec(0); }

  // the verbose line and / or the level-0 benchmark-trace entry of one point of a V-cycle
  void per_sweep_line(int l, int it, const char* what, bool bench) {
    if (!c_->d.verbose) {  // benchmark trace only: level 0's relres against the time step's ||b||
      const double rn = residual(l, true);
      c_->trace_push(c_->trace_rhs > 0.0 ? rn / c_->trace_rhs : rn);
      return;
    }
    const double rel = verbose_line(l, it, what);
    if (bench) {
      // the verbose line's ||b|| is level 0's b: the time step's rhs except in the refine mode's
      // correction cycles (b = the fp64 residual), whose relres is taken against the step's rhs
      const double rn = rel * norm(l, MAD_B);
      c_->trace_push(c_->trace_rhs > 0.0 ? rn / c_->trace_rhs : rn);
    }
  }

  double verbose_line(int l, int it, const char* what) {
    // rhsNorm (MAD.hxx:352) and the residual norm of the current iterate
    const double bn = norm(l, MAD_B);
    // keep r intact: the residual kernel writes r, which at this point is scratch
    const double rn = residual(l, true);
    const double rel = rn / bn;
    if (c_->comm.rank() != 0) return rel;
    std::string ind(l + 1, ' ');
    if (what && std::strcmp(what, "direct solver") == 0)
      std::printf("%sLevel %d, direct solver: relative residual = %g\n", ind.c_str(), l, rel);
    else if (what)
      std::printf("%sLevel %d, initial relative residual = %g\n", ind.c_str(), l, rel);
    else
      std::printf("%sLevel %d, iteration %d: relative residual = %g\n", ind.c_str(), l, it, rel);
    std::fflush(stdout);
    return rel;
  }

  // ------------------------------------------------------------- filter
  void run(const void* in, int in_dtype, void* out, int out_dtype, bool dev_io,
           mad_stats* st) override {
    if (refine_) {
      run_refine(in, in_dtype, out, out_dtype, dev_io, st);
      return;
    }
    LevelData<T>& L0 = lv_[0];
    const int64_t N = L0.g.N;
    const mad_desc& d = c_->d;
    // cast input -> internal precision (MAD.hxx:110-127)
    const void* src = in;
    if (!dev_io) {
      void* stage = scratch_bytes(N * dtype_size(in_dtype));
      HIP_CHECK(hipMemcpyAsync(stage, in, N * dtype_size(in_dtype), hipMemcpyHostToDevice,
                               c_->stream));
      src = stage;
    }
    convert_in(src, in_dtype, L0.b, N);
    L0.b_halo_ok = L0.brec_ok = false;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventRecord(e0, c_->stream));
    c_->step_cycles.clear();
    c_->step_relres.clear();
    c_->trace.clear();
    // per-cycle entries (seconds since the run's start); with MAD_OPT_BENCHMARK_TRACE the V-cycle
    // records level 0's entries itself (per_sweep_line) and only SMOOTHER sweeps are recorded here,
    // with seconds since the time step's start (the reference's m_Time, MAD.hxx:158-163)
    const bool bt = c_->bench_trace();
    c_->trace_active = true;
    c_->trace_t0 = std::chrono::steady_clock::now();
    auto trace = [&](unsigned step, double rr) {
      if (bt && d.cycle != MAD_SMOOTHER) return;
      c_->trace_step = step;
      c_->trace_push(rr);
    };
    bool stalled_any = false;
    unsigned total = 0;
    double relres = 0.0;
    for (unsigned step = 0; step < d.number_of_steps; ++step) {  // MAD.hxx:158
      if (d.verbose && d.number_of_steps > 1 && c_->comm.rank() == 0)
        std::printf("\n------------ Time step n. %u / %u------------\n", step + 1, d.number_of_steps);
      if (bt) {
        c_->trace_t0 = std::chrono::steady_clock::now();
        c_->trace_step = step;
        c_->trace_rhs = norm(0, MAD_B);  // the rhsNorm of the step's level-0 V-cycles (MAD.hxx:352)
      }
      if (d.cycle == MAD_FMG) {
        if (d.verbose && c_->comm.rank() == 0) std::printf("|--- Full Multigrid Cycle ---|\n");
        fmg_rec(0);  // MAD.hxx:170-176
      } else {
        HIP_CHECK(hipMemcpyAsync(L0.x, L0.b, sizeof(T) * N, hipMemcpyDeviceToDevice,
                                 c_->stream));  // MAD.hxx:177-201
        x_changed(0);
      }
      const double rhsNorm = norm(0, MAD_B);  // MAD.hxx:204
      REQUIRE(std::isfinite(rhsNorm), MAD_ERR_NUMERIC,
              "non-finite right-hand side norm (NaN/Inf in the input image)");
      unsigned it = 0;
      double best = INFINITY;
      std::vector<double> hist;
      const unsigned window = (d.cycle == MAD_SMOOTHER) ? 50 : 5;
      bool stalled = false;
      do {  // MAD.hxx:207-246
        if (d.cycle == MAD_SMOOTHER) {
          smooth(0, 1);
        } else {
          if (d.verbose && c_->comm.rank() == 0) std::printf("\n|--- VCycle n. %u ---|\n", it + 1);
          vcycle_fast();
        }
        const double resNorm = residual_impl(0, true, false);  // MAD.hxx:221-229 (norm only)
        // NaN > tol is false: without this check a NaN residual ends the do/while as if
        // converged and the call returns MAD_OK with a NaN image
        REQUIRE(std::isfinite(resNorm), MAD_ERR_NUMERIC,
                "non-finite residual norm (NaN/Inf in the tensor or the iterate)");
        // an all-zero image (rhsNorm 0) is its own solution: report relres 0, not 0/0
        relres = (rhsNorm > 0.0) ? resNorm / rhsNorm : resNorm;
        if (d.verbose && d.cycle == MAD_SMOOTHER && c_->comm.rank() == 0)
          std::printf("Smoother iteration n. %u: relative residual = %g\n", it + 1, relres);
        ++it;
        trace(step, relres);
        hist.push_back(relres);
        // fp32 floor guard: best relres not improved by 1% within `window` cycles (only while the
        // tolerance is unmet: a cycle that reaches it ends the step as converged)
        if (d.stall_guard && hist.size() > window && relres < 1e-3 && relres > d.tolerance) {
          double prev_best = INFINITY;
          for (size_t q = 0; q + window < hist.size(); ++q) prev_best = std::min(prev_best, hist[q]);
          double recent = INFINITY;
          for (size_t q = hist.size() - window; q < hist.size(); ++q) recent = std::min(recent, hist[q]);
          if (recent > 0.99 * prev_best) stalled = true;
        }
        best = std::min(best, relres);
      } while (relres > d.tolerance && it < d.max_cycles && !stalled);
      stalled_any |= stalled;
      total += it;
      c_->step_cycles.push_back(it);
      c_->step_relres.push_back(relres);
      HIP_CHECK(hipMemcpyAsync(L0.b, L0.x, sizeof(T) * N, hipMemcpyDeviceToDevice,
                               c_->stream));  // MAD.hxx:248-261
      L0.b_halo_ok = L0.brec_ok = false;
    }
    c_->trace_active = false;
    HIP_CHECK(hipEventRecord(e1, c_->stream));
    // cast solution -> output type (MAD.hxx:266-289)
    void* dst = out;
    if (!dev_io) dst = scratch_bytes(N * dtype_size(out_dtype));
    convert_out(L0.x, dst, out_dtype, N);
    if (!dev_io)
      HIP_CHECK(hipMemcpyAsync(out, dst, N * dtype_size(out_dtype), hipMemcpyDeviceToHost,
                               c_->stream));
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    peer_check();  // a timed-out peer wait fails the run instead of returning stale halos
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    if (st) {
      std::memset(st, 0, sizeof(*st));
      st->steps = d.number_of_steps;
      st->total_cycles = total;
      st->last_cycles = c_->step_cycles.empty() ? 0 : c_->step_cycles.back();
      st->stalled = stalled_any ? 1 : 0;
      st->last_relres = relres;
      st->setup_ms = c_->setup_ms;
      st->solve_ms = ms;
      st->num_levels = (uint32_t)c_->nlev;
      st->tensor_kind = c_->kind;
      st->colors = c_->ncolors;
    }
  }

  // GenerateData (MAD.hxx:104-297) with mixed-precision defect correction (MAD_FP32_REFINE):
  // the iterate u and the rhs b of level 0 stay in fp64; every cycle forms the fp64 residual
  // r = b - A u with the fp64 operator, runs the cycle the CycleType names (one V-cycle, or
  // one smoother sweep) in fp32 on the error equation A e = r from e = 0, and adds u += e in
  // fp64.  The fp32 V-cycle only has to reduce the error by its usual factor each time, so
  // the iteration converges to the fp64 solution (relres to the reference's 1e-10) instead
  // of stalling at the fp32 floor (~1e-7); relres is the fp64 residual's, as in the
  // reference's loop (MAD.hxx:207-246).  FMG: the fp32 FMG cycle gives the first iterate.
  void run_refine(const void* in, int in_dtype, void* out, int out_dtype, bool dev_io,
                  mad_stats* st) {
    LevelData<T>& L0 = lv_[0];
    const int64_t N = L0.g.N;
    const mad_desc& d = c_->d;
    const unsigned nb = flat_blocks(N);
    const void* src = in;
    if (!dev_io) {
      void* stage = scratch_bytes(N * dtype_size(in_dtype));
      HIP_CHECK(hipMemcpyAsync(stage, in, N * dtype_size(in_dtype), hipMemcpyHostToDevice,
                               c_->stream));
      src = stage;
    }
    convert_to(src, in_dtype, b64_, N, c_->stream);
    // an 8/16-bit or fp32 image is exactly an fp32 array: the first time step's fp64 residuals read
    // its fp32 copy (the same values, 4 of the pass's 104 B per voxel saved)
    b32_exact_ = in_dtype == MAD_U8 || in_dtype == MAD_I8 || in_dtype == MAD_U16 || in_dtype == MAD_I16 ||
                 in_dtype == MAD_F32;
    if (b32_exact_) {
      hipLaunchKernelGGL((convert_k<double, float>), dim3(nb), dim3(256), 0, c_->stream, b64_, b32_, N);
      HIP_CHECK(hipGetLastError());
    }
    auto to_fp32_rhs = [&](const double* a) {  // level-0 b (fp32) <- a
      hipLaunchKernelGGL((convert_k<double, T>), dim3(nb), dim3(256), 0, c_->stream, a, L0.b, N);
      HIP_CHECK(hipGetLastError());
      L0.b_halo_ok = L0.brec_ok = false;
    };
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventRecord(e0, c_->stream));
    c_->step_cycles.clear();
    c_->step_relres.clear();
    c_->trace.clear();
    // per-cycle entries (seconds since the run's start); with MAD_OPT_BENCHMARK_TRACE the V-cycle
    // records level 0's entries itself (per_sweep_line) and only SMOOTHER sweeps are recorded here,
    // with seconds since the time step's start (the reference's m_Time, MAD.hxx:158-163)
    const bool bt = c_->bench_trace();
    c_->trace_active = true;
    c_->trace_t0 = std::chrono::steady_clock::now();
    auto trace = [&](unsigned step, double rr) {
      if (bt && d.cycle != MAD_SMOOTHER) return;
      c_->trace_step = step;
      c_->trace_push(rr);
    };
    bool stalled_any = false;
    unsigned total = 0;
    double relres = 0.0;
    for (unsigned step = 0; step < d.number_of_steps; ++step) {  // MAD.hxx:158
      if (d.verbose && d.number_of_steps > 1 && c_->comm.rank() == 0)
        std::printf("\n------------ Time step n. %u / %u------------\n", step + 1, d.number_of_steps);
      // V-cycle / FMG solves start in plain fp32 (the fp32 iterate on the fp32 rhs, fp32 residual
      // norms) while relres is far above fp32's floor: those cycles reduce the error as the refined
      // ones would, at the fp32 cycle's cost; below MAD_REFINE_SWITCH_RELRES the iterate moves to
      // fp64 and the defect correction takes over (SMOOTHER runs refine from the first sweep: their
      // unconverged output depends on every sweep's rounding)
#ifdef MAD_NO_REFINE_FP32_PHASE  // A/B: refine from the first cycle
      const bool fp32_phase = false;
#else
      // (at least two cycles allowed: the fp32 phase always leaves the defect correction a turn)
      const bool fp32_phase = d.cycle != MAD_SMOOTHER && d.max_cycles >= 2;
#endif
      if (bt) {
        c_->trace_t0 = std::chrono::steady_clock::now();
        c_->trace_step = step;
        c_->trace_rhs = norm64(b64_);  // MAD.hxx:204 / 352
      }
      if (d.cycle == MAD_FMG) {
        if (d.verbose && c_->comm.rank() == 0) std::printf("|--- Full Multigrid Cycle ---|\n");
        to_fp32_rhs(b64_);
        fmg_rec(0);  // MAD.hxx:170-176, in fp32
        if (!fp32_phase) {
          hipLaunchKernelGGL((convert_k<T, double>), dim3(nb), dim3(256), 0, c_->stream, L0.x, u64_, N);
          HIP_CHECK(hipGetLastError());
        }
      } else if (fp32_phase) {
        to_fp32_rhs(b64_);
        HIP_CHECK(hipMemcpyAsync(L0.x, L0.b, sizeof(T) * N, hipMemcpyDeviceToDevice,
                                 c_->stream));  // MAD.hxx:177-201
        x_changed(0);
      } else {
        HIP_CHECK(hipMemcpyAsync(u64_, b64_, sizeof(double) * N, hipMemcpyDeviceToDevice,
                                 c_->stream));  // MAD.hxx:177-201
      }
      const double rhsNorm = norm64(b64_);  // MAD.hxx:204
      REQUIRE(std::isfinite(rhsNorm), MAD_ERR_NUMERIC,
              "non-finite right-hand side norm (NaN/Inf in the input image)");
      unsigned it = 0;
      std::vector<double> hist;
      const unsigned window = (d.cycle == MAD_SMOOTHER) ? 50 : 5;
      bool stalled = false;
      if (fp32_phase) {
        do {  // MAD.hxx:207-246 in fp32
          if (d.verbose && c_->comm.rank() == 0) std::printf("\n|--- VCycle n. %u ---|\n", it + 1);
          vcycle_fast();
          const double rn = residual_impl(0, true, false);
          REQUIRE(std::isfinite(rn), MAD_ERR_NUMERIC,
                  "non-finite residual norm (NaN/Inf in the tensor or the iterate)");
          relres = (rhsNorm > 0.0) ? rn / rhsNorm : rn;
          ++it;
          trace(step, relres);
          hist.push_back(relres);
          // plain fp32 levels off at a floor that grows with the conditioning (large time steps,
          // strong anisotropy): once a cycle reduces relres by less than 2x, the fp64 defect
          // correction takes over, and the phase ends one cycle before MaxCycles so it always does
          if (hist.size() >= 2 && relres > MAD_REFINE_FP32_MIN_RATE * hist[hist.size() - 2]) break;
        } while (relres > std::max(d.tolerance, MAD_REFINE_SWITCH_RELRES) && it + 1 < d.max_cycles);
        hipLaunchKernelGGL((convert_k<T, double>), dim3(nb), dim3(256), 0, c_->stream, L0.x, u64_, N);
        HIP_CHECK(hipGetLastError());
      }
      double resNorm = residual64();
      REQUIRE(std::isfinite(resNorm), MAD_ERR_NUMERIC,
              "non-finite residual norm (NaN/Inf in the tensor or the iterate)");
      if (fp32_phase) {  // the switch iterate's relres, now from the fp64 residual
        relres = (rhsNorm > 0.0) ? resNorm / rhsNorm : resNorm;
        if (!hist.empty()) {
          hist.back() = relres;
          // (the per-cycle entry; with the benchmark trace the last post-smoothing sweep's)
          if (!c_->trace.empty()) c_->trace.back().relres = relres;
        }
      }
      if (!fp32_phase || (relres > d.tolerance && it < d.max_cycles)) do {  // MAD.hxx:207-246
        if (refine_emitted_) {  // b = (T) r and x = 0 written by residual64's pass
          L0.b_halo_ok = false;
          L0.brec_ok = refine_emitted_bs_;  // the split copy of b too
          x_changed(0);
        } else {
          to_fp32_rhs(r64_);
          fill(0, MAD_X, 0.0);
        }
        if (d.cycle == MAD_SMOOTHER) {
          smooth(0, 1);
        } else {
          if (d.verbose && c_->comm.rank() == 0) std::printf("\n|--- VCycle n. %u ---|\n", it + 1);
          zero_x0_ = refine_emitted_ && zero_sweep_ok();  // x = 0 (or left stale by the fold)
          vcycle_fast();
          zero_x0_ = false;
        }
        resNorm = residual64(/*fold=*/true);  // u += e, then MAD.hxx:221-229

        REQUIRE(std::isfinite(resNorm), MAD_ERR_NUMERIC,
                "non-finite residual norm (NaN/Inf in the tensor or the iterate)");
        relres = (rhsNorm > 0.0) ? resNorm / rhsNorm : resNorm;
        if (d.verbose && d.cycle == MAD_SMOOTHER && c_->comm.rank() == 0)
          std::printf("Smoother iteration n. %u: relative residual = %g\n", it + 1, relres);
        ++it;
        trace(step, relres);
        // benchmark trace: the last post-smoothing entry is the updated iterate's, now in fp64
        if (bt && d.cycle != MAD_SMOOTHER && !c_->trace.empty()) c_->trace.back().relres = relres;
        hist.push_back(relres);
        // fallback only: the fp64 residual keeps falling where plain fp32 stalls
        if (d.stall_guard && hist.size() > window && relres < 1e-3 && relres > d.tolerance) {
          double prev_best = INFINITY;
          for (size_t q = 0; q + window < hist.size(); ++q) prev_best = std::min(prev_best, hist[q]);
          double recent = INFINITY;
          for (size_t q = hist.size() - window; q < hist.size(); ++q) recent = std::min(recent, hist[q]);
          if (recent > 0.99 * prev_best) stalled = true;
        }
      } while (relres > d.tolerance && it < d.max_cycles && !stalled);
      stalled_any |= stalled;
      total += it;
      c_->step_cycles.push_back(it);
      c_->step_relres.push_back(relres);
      HIP_CHECK(hipMemcpyAsync(b64_, u64_, sizeof(double) * N, hipMemcpyDeviceToDevice,
                               c_->stream));  // MAD.hxx:248-261
      b32_exact_ = false;  // the next step's rhs is the fp64 solution
    }
    c_->trace_active = false;
    HIP_CHECK(hipEventRecord(e1, c_->stream));
    // the last folded residual left x holding the last fp32 correction (the zero-iterate sweep
    // never needed it cleared): leave level-0 x = 0, as the unfolded pass does, for direct
    // kernel-API use after the run (mad_download, mad_smooth, mad_vcycle)
    if (refine_emitted_ && zero_sweep_ok()) fill(0, MAD_X, 0.0);
    void* dst = out;
    if (!dev_io) dst = scratch_bytes(N * dtype_size(out_dtype));
    convert_from(u64_, dst, out_dtype, N, c_->stream);  // MAD.hxx:266-289
    if (!dev_io)
      HIP_CHECK(hipMemcpyAsync(out, dst, N * dtype_size(out_dtype), hipMemcpyDeviceToHost,
                               c_->stream));
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    peer_check();  // a timed-out peer wait fails the run instead of returning stale halos
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    if (st) {
      std::memset(st, 0, sizeof(*st));
      st->steps = d.number_of_steps;
      st->total_cycles = total;
      st->last_cycles = c_->step_cycles.empty() ? 0 : c_->step_cycles.back();
      st->stalled = stalled_any ? 1 : 0;
      st->last_relres = relres;
      st->setup_ms = c_->setup_ms;
      st->solve_ms = ms;
      st->num_levels = (uint32_t)c_->nlev;
      st->tensor_kind = c_->kind;
      st->colors = c_->ncolors;
    }
  }

  // ------------------------------------------------------------- measurement
  void bench_smooth(int l, unsigned n, double* total_ms, double* kern_ms,
                    unsigned* launches) override {
    LevelData<T>& L = lv_[l];
    const int sm = c_->d.smoother;
    const bool fused = use_fused(l);
    const int nc = (sm == MAD_GAUSS_SEIDEL && !fused) ? c_->ncolors : 1;
    REQUIRE(sm != MAD_GAUSS_SEIDEL_LEX, MAD_ERR_UNSUPPORTED, "bench of the lexicographic mode");
    const unsigned nl = n * nc;
    std::vector<hipEvent_t> ev(2 * nl);
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    hipEvent_t a, z;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&z));
    HIP_CHECK(hipEventRecord(a, c_->stream));
    const int rows = (nc == 4) ? (L.g.ny + 1) / 2 : L.g.ny;
    unsigned q = 0;
    for (unsigned s = 0; s < n; ++s) {
      if (sm == MAD_WEIGHTED_JACOBI) {
        prep_wj(l);
        HIP_CHECK(hipEventRecord(ev[2 * q], c_->stream));
        launch_wj(l);
        HIP_CHECK(hipEventRecord(ev[2 * q + 1], c_->stream));
        ++q;
        std::swap(L.x, L.t);
        std::swap(L.alloc[0], L.alloc[3]);
        x_changed(l);
      } else if (fused) {
        fused_sweep(l, ev[2 * q], ev[2 * q + 1]);
        ++q;
      } else {
        dim3 gr = grid_for((L.g.nx + 1) / 2, rows, L.g.nz, BLK);
        for (int col = 0; col < nc; ++col) {
          halo(l, L.x);
          HIP_CHECK(hipEventRecord(ev[2 * q], c_->stream));
          dispatch(c_->dim, c_->kind, [&](auto D, auto K) {
            hipLaunchKernelGGL((gs_color_k<T, D.value, K.value>), gr, BLK, 0, c_->stream, L.x,
                               L.b, L.cf, L.g, L.rat, col, nc);
          });
          HIP_CHECK(hipEventRecord(ev[2 * q + 1], c_->stream));
          ++q;
          x_changed(l);
        }
      }
    }
    HIP_CHECK(hipGetLastError());
    if (L.x_halo_pending) {  // the last overlapped exchange belongs to the timed work
      HIP_CHECK(hipStreamWaitEvent(c_->stream, L.ev_halo, 0));
      L.x_halo_pending = false;
    }
    HIP_CHECK(hipEventRecord(z, c_->stream));
    HIP_CHECK(hipEventSynchronize(z));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, a, z));
    double ksum = 0.0;
    launch_ms.assign(q, 0.f);
    for (unsigned i = 0; i < q; ++i) {
      float km = 0.f;
      HIP_CHECK(hipEventElapsedTime(&km, ev[2 * i], ev[2 * i + 1]));
      ksum += km;
      launch_ms[i] = km;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(z);
    *total_ms = ms;
    *kern_ms = q ? ksum / q : 0.0;
    *launches = q;
  }

  void bench_vcycle(unsigned n, double* total_ms) override {
    hipEvent_t a, z;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&z));
    HIP_CHECK(hipEventRecord(a, c_->stream));
    for (unsigned s = 0; s < n; ++s) vcycle_fast();
    HIP_CHECK(hipEventRecord(z, c_->stream));
    HIP_CHECK(hipEventSynchronize(z));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, a, z));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(z);
    *total_ms = ms;
  }

 private:
  mad_ctx* c_ = nullptr;
  std::vector<LevelData<T>> lv_;
  // MAD_FP32_REFINE (T = float): level 0's iterate, rhs and residual in fp64 (same layout as
  // the level arrays: margin + GHOST planes) and its operator as fp64 coefficient records
  // with the reference's g (from the fp64 tensor); the fp32 hierarchy solves for corrections
  bool refine_ = false;
  double* r64alloc_[3] = {nullptr, nullptr, nullptr};
  double* u64_ = nullptr;
  double* b64_ = nullptr;
  float* b32alloc_ = nullptr;  // b64_ as fp32 where it is exactly that (b32_exact_)
  float* b32_ = nullptr;
  bool b32_exact_ = false;
  double* r64_ = nullptr;
  double* cf64_alloc_ = nullptr;
  double* cf64_ = nullptr;
  Rat<double> rat64_{};
  int64_t part_cap_ = 0;             // entries of part_
  hipGraphExec_t vgraph_ = nullptr;  // captured V-cycle (vcycle_fast)
  bool vgraph_zu_ = false;            // its first level-0 sweep is the zero-iterate form
  std::vector<std::pair<T*, T*>> vgraph_ptrs_;  // per-level (x, t) the graph was captured with
  std::vector<int> vgraph_seq_;                  // per-level peer mailbox parity it was captured with
  bool vgraph_failed_ = false;
  uint64_t peer_timeout_ticks_ = 0;
  int peer_fallbacks_ = 0;  // levels whose peer self-test failed (they exchange instead)
  std::vector<HaloFlags> vgraph_exit_flags_;  // rank slabs: ghost bookkeeping after one cycle
  int vcycles_eager_ = 0;  // rank slabs: cycles run eagerly so far (RCCL peers connected)
  int ncoef_ = 0;
  double* part_ = nullptr;
  double* scal_ = nullptr;
  double* hscal_ = nullptr;
  double* inv_ = nullptr;
  CoarseBlocks cblk_;  // coarsest levels above DENSE_COARSE_MAX unknowns
  void* scratch_ = nullptr;
  size_t scratch_cap_ = 0;
  // replicated-level hand-over (multi-GPU)
  T* gathered_ = nullptr;
  T* full_x_ = nullptr;
  int64_t gathered_cap_ = 0;
  T* cslab_ = nullptr;  // coarse_slab
  int64_t cslab_cap_ = 0;

  void release() {
    if (c_ && c_->comm_stream) (void)hipStreamSynchronize(c_->comm_stream);
    // a neighbour's last peer batch still in flight lands in this rank's window: take it in (the
    // unpack waits until the neighbour's stores are complete) before the window is freed.  The
    // in-process transport's ranks drain their streams at their next barrier instead (no wait here:
    // a barrier in a destructor could hang on a rank that already failed).
    if (c_ && c_->comm.mode() != Comm::LOCAL) {
      try {
        for (size_t l = 0; l < lv_.size(); ++l)
          if (lv_[l].x_peer_pending) peer_resolve((int)l);
      } catch (...) {
      }
    }
    if (c_ && c_->stream) (void)hipStreamSynchronize(c_->stream);
    if (vgraph_) (void)hipGraphExecDestroy(vgraph_);
    vgraph_ = nullptr;
    vgraph_ptrs_.clear();
    vgraph_seq_.clear();
    vgraph_failed_ = false;
    vcycles_eager_ = 0;
    for (auto& L : lv_) {
      if (L.ev_bnd) (void)hipEventDestroy(L.ev_bnd);
      if (L.ev_halo) (void)hipEventDestroy(L.ev_halo);
      if (L.sig) (void)hipFree(L.sig);
      Comm::close_window(L.win_lo, L.win_ipc);
      Comm::close_window(L.win_hi, L.win_ipc);
      if (L.win) (void)hipFree(L.win);
      for (auto& a : L.alloc)
        if (a) (void)hipFree(a);
      if (L.cf_alloc) (void)hipFree(L.cf_alloc);
      if (L.bs_alloc) (void)hipFree(L.bs_alloc);
    }
    lv_.clear();
    for (auto& a : r64alloc_)
      if (a) (void)hipFree(a), a = nullptr;
    if (cf64_alloc_) (void)hipFree(cf64_alloc_);
    cf64_alloc_ = nullptr;
    u64_ = b64_ = r64_ = cf64_ = nullptr;
    if (b32alloc_) (void)hipFree(b32alloc_);
    b32alloc_ = b32_ = nullptr;
    b32_exact_ = false;
    if (part_) (void)hipFree(part_);
    if (scal_) (void)hipFree(scal_);
    if (hscal_) (void)hipHostFree(hscal_);
    if (inv_) (void)hipFree(inv_);
    cblk_.release();
    if (scratch_) (void)hipFree(scratch_);
    if (gathered_) (void)hipFree(gathered_);
    if (cslab_) (void)hipFree(cslab_);
    cslab_ = nullptr;
    cslab_cap_ = 0;
    if (full_x_) (void)hipFree(full_x_);
    part_ = scal_ = hscal_ = inv_ = nullptr;
    scratch_ = nullptr;
    scratch_cap_ = 0;
    gathered_ = full_x_ = nullptr;
    gathered_cap_ = 0;
  }

  void* scratch_bytes(size_t bytes) {
    if (bytes > scratch_cap_) {
      HIP_CHECK(hipStreamSynchronize(c_->stream));
      if (scratch_) HIP_CHECK(hipFree(scratch_));
      scratch_ = nullptr;
      HIP_CHECK(big_alloc((void**)&scratch_, bytes));
      scratch_cap_ = bytes;
    }
    return scratch_;
  }
  double* scratch64(int64_t n) { return (double*)scratch_bytes(sizeof(double) * n); }

  void convert_in(const void* src, int dt, T* dst, int64_t n) { convert_to(src, dt, dst, n, c_->stream); }
  void convert_out(const T* src, void* dst, int dt, int64_t n) { convert_from(src, dst, dt, n, c_->stream); }

  // GH.hxx:110-201: level-0 DCA from the input tensor, then per level: restrict every tensor
  // component (coarse centring) and rediscretise, in fp64.  Rank slabs stay slabs: a
  // distributed level restricts its own planes from the finer slab (taps past the slab read
  // the finer level's ghost planes), fills TENSOR_GHOST ghost planes from the neighbours
  // (Comm::shift_planes, hop by hop where the slab is thinner than that) and builds its
  // records on the owned + GHOST ghost planes; the first replicated level gathers the last
  // distributed one (small by construction, plan_geometry).  Per-rank memory O(slab), and the
  // records are bit-identical to a whole-grid build: global plane indices, the same taps in
  // the same order.
  struct TView {
    double* base;  // component 0, first stored plane
    int64_t cs;    // component stride
    int tg;        // ghost planes per side
    int64_t z0;    // global index of the first owned plane
    int64_t sz;    // plane size
    double* at0() const { return base + (tg - z0) * sz; }    // global-plane-indexed
    double* owned(int k) const { return base + k * cs + tg * sz; }  // component k, plane z0
  };

  void build_operators() {
    const int dim = c_->dim;
    const int ncomp = dim * (dim + 1) / 2;
    const int nl = c_->nlev;
    const LevelGeom& G0 = c_->geom[0];
    TView fine{c_->tensor64, c_->tensor_cs, c_->tensor_tg, G0.z0, G0.n[0] * G0.n[1]};
    double* own = nullptr;  // the level tensor allocated here (freed once superseded)
    for (int l = 0; l < nl; ++l) {
      const LevelGeom& G = c_->geom[l];
      const int64_t sz = G.n[0] * G.n[1];
      if (l > 0) {
        const LevelGeom& Gf = c_->geom[l - 1];
        const int tgc = G.distributed ? TENSOR_GHOST : 0;
        const int64_t nzl = G.z1 - G.z0;
        const int64_t csc = (nzl + 2 * tgc) * sz;
        double* coarse = nullptr;
        HIP_CHECK(hipMalloc(&coarse, sizeof(double) * ncomp * csc));
        if (tgc) HIP_CHECK(hipMemsetAsync(coarse, 0, sizeof(double) * ncomp * csc, c_->stream));
        // a replicated level under a distributed one: gather the finer slabs first
        double* gathered = nullptr;
        TView src = fine;
        if (!G.distributed && Gf.distributed) {
          HIP_CHECK(hipMalloc(&gathered, sizeof(double) * ncomp * Gf.N));
          for (int k = 0; k < ncomp; ++k)
            c_->comm.allgather_slabs(fine.owned(k), gathered + k * Gf.N, fine.sz, Gf.n[2], sizeof(double),
                                     c_->stream);
          src = TView{gathered, Gf.N, 0, 0, fine.sz};
        }
        const bool src_slab = src.tg > 0;
        Geo gf{}, gc{};
        gf.nx = (int)Gf.n[0]; gf.ny = (int)Gf.n[1];
        gf.nz = (int)(src_slab ? Gf.z1 - Gf.z0 : Gf.n[2]);
        gf.sy = Gf.n[0]; gf.sz = fine.sz; gf.N = gf.sz * gf.nz;
        gc.nx = (int)G.n[0]; gc.ny = (int)G.n[1]; gc.nz = (int)nzl;
        gc.zoff = (int)G.z0;
        gc.sy = G.n[0]; gc.sz = sz; gc.N = sz * nzl;
        const int fz_shift = src_slab ? (int)Gf.z0 : 0;
        for (int k = 0; k < ncomp; ++k) {
          const double* fk = src.owned(k);
          double* ck = coarse + k * csc + tgc * sz;
          if (dim == 3) {
            // z-marching restriction (LDS-staged planes; same taps and fma order as
            // restrict_k, bit-identical), ~1024 blocks
            constexpr int CX = 32, CY = 8;
            const int ntx = (gc.nx + CX - 1) / CX, nty = (gc.ny + CY - 1) / CY;
            int chunks = std::max(1, std::min((1024 + ntx * nty - 1) / (ntx * nty), std::max(1, gc.nz / 4)));
            const int kc = (gc.nz + chunks - 1) / chunks;
            chunks = (gc.nz + kc - 1) / kc;
            hipLaunchKernelGGL((restrict3_k<double, double, CX, CY>),
                               dim3((unsigned)(ntx * nty * chunks)), dim3(CX * CY), 0, c_->stream,
                               fk, gf, ck, gc, G.cent[0], G.cent[1], G.cent[2], fz_shift,
                               (int)G.n[2], kc, ntx);
          } else {
            dim3 gr = grid_for(gc.nx, gc.ny, gc.nz, BLK);
            hipLaunchKernelGGL((restrict_k<double, double, 2>), gr, BLK, 0, c_->stream, fk, gf, ck, gc,
                               G.cent[0], G.cent[1], G.cent[2], 0);
          }
          HIP_CHECK(hipGetLastError());
          // the coarse slab's ghost planes, hop by hop (a hop moves at most one slab depth)
          for (int D = 0; D < tgc;) {
            const int d = (int)std::min<int64_t>(nzl, tgc - D);
            c_->comm.shift_planes(ck, sz, (int)nzl, D, d, G.z0 > 0, G.z1 < G.n[2], sizeof(double), true,
                                  c_->stream);
            D += d;
          }
        }
        HIP_CHECK(hipStreamSynchronize(c_->stream));
        if (gathered) HIP_CHECK(hipFree(gathered));
        if (own) HIP_CHECK(hipFree(own));
        own = coarse;
        fine = TView{coarse, csc, tgc, G.z0, sz};
      }
      LevelData<T>& L = lv_[l];
      // records on planes [g0, g1) (owned + GHOST ghost planes on a slab); their a / e on
      // [w0, w1) (g's differences reach two planes further)
      const bool dist = G.distributed;
      const int64_t g0 = dist ? std::max<int64_t>(G.z0 - GHOST, 0) : 0;
      const int64_t g1 = dist ? std::min<int64_t>(G.z1 + GHOST, G.n[2]) : G.n[2];
      const int64_t w0 = dist ? std::max<int64_t>(g0 - 2, 0) : 0;
      const int64_t w1 = dist ? std::min<int64_t>(g1 + 2, G.n[2]) : G.n[2];
      const int64_t cplane = sz * L.g.rs;
      T* win = nullptr;  // slab: the records of [w0, w1); whole grid: L.cf itself
      if (dist) HIP_CHECK(hipMalloc(&win, sizeof(T) * (w1 - w0) * cplane));
      T* rec0 = dist ? win - w0 * cplane : L.cf;  // global-plane-indexed records
      const CoefFactors cfac = coef_factors(G.h, c_->d.time_step);
      // z-marching (build_coef3_k): chunks of planes sized for ~4096 blocks of 64 x 4
      auto coef3 = [&](auto* out, int rs, int64_t kb, int64_t ke) {
        using U = std::remove_pointer_t<decltype(out)>;
        const int bx = ((int)G.n[0] + 63) / 64, by = ((int)G.n[1] + 3) / 4;
        const int nzw = (int)(ke - kb);
        int chunks = std::max(1, std::min(nzw, (4096 + bx * by - 1) / (bx * by)));
        const int kc = (nzw + chunks - 1) / chunks;
        chunks = (nzw + kc - 1) / kc;
        auto go = [&](auto K) {
          hipLaunchKernelGGL((build_coef3_k<U, decltype(K)::value>), dim3(bx, by, chunks), BLK, 0,
                             c_->stream, fine.at0(), (int)G.n[0], (int)G.n[1], (int)G.n[2], cfac, out, rs,
                             kc, (int)kb, (int)ke, fine.cs);
        };
        if (c_->kind == KFULL) go(std::integral_constant<int, KFULL>{});
        else if (c_->kind == KDIAG) go(std::integral_constant<int, KDIAG>{});
        else go(std::integral_constant<int, KISO>{});
      };
      if (dim == 3) {
        coef3(rec0, L.g.rs, w0, w1);
      } else {
        dim3 gr = grid_for((int)G.n[0], (int)G.n[1], (int)G.n[2], BLK);
        dispatch(dim, c_->kind, [&](auto D, auto K) {
          hipLaunchKernelGGL((build_coef_k<T, D.value, K.value>), gr, BLK, 0, c_->stream, fine.base,
                             (int)G.n[0], (int)G.n[1], (int)G.n[2], cfac, rec0, L.g.rs);
        });
      }
      HIP_CHECK(hipGetLastError());
      // g from the stored a / e (build_g_k): the one definition every kernel shares
      {
        dim3 gr = grid_for((int)G.n[0], (int)G.n[1], (int)(g1 - g0), BLK);
        dispatch(dim, c_->kind, [&](auto D, auto K) {
          hipLaunchKernelGGL((build_g_k<T, D.value, K.value>), gr, BLK, 0, c_->stream, rec0,
                             (int)G.n[0], (int)G.n[1], (int)G.n[2], L.g.rs, L.rat, (int)g0);
        });
        HIP_CHECK(hipGetLastError());
      }
      if (dist) {
        HIP_CHECK(hipMemcpyAsync(L.cf + (g0 - G.z0) * cplane, win + (g0 - w0) * cplane,
                                 sizeof(T) * (g1 - g0) * cplane, hipMemcpyDeviceToDevice, c_->stream));
        HIP_CHECK(hipStreamSynchronize(c_->stream));
        HIP_CHECK(hipFree(win));
      }
      if (l == 0 && refine_) {
        // the refined system's operator: fp64 records, g from the fp64 tensor (build_coef*_k
        // restate GH.hxx:298-516 directly; no build_g_k pass), owned + ghost planes
        if (dim == 3) {
          coef3(cf64_ - G.z0 * sz * ncoef_, ncoef_, g0, g1);
        } else {
          dim3 gr = grid_for((int)G.n[0], (int)G.n[1], (int)G.n[2], BLK);
          dispatch(dim, c_->kind, [&](auto D, auto K) {
            hipLaunchKernelGGL((build_coef_k<double, D.value, K.value>), gr, BLK, 0, c_->stream, fine.base,
                               (int)G.n[0], (int)G.n[1], (int)G.n[2], cfac, cf64_, ncoef_);
          });
        }
        HIP_CHECK(hipGetLastError());
      }
      if (l == nl - 1) build_coarsest_matrix(fine.base);  // replicated: the whole grid
    }
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    if (own) HIP_CHECK(hipFree(own));
  }

  std::vector<double> coarse_coef64_;

  void build_coarsest_matrix(const double* tensor_l) {
    const int dim = c_->dim;
    const LevelGeom& G = c_->geom[c_->nlev - 1];
    const int nc = coef_count(dim, c_->kind);
    double* cf64 = nullptr;
    HIP_CHECK(big_alloc((void**)&cf64, sizeof(double) * G.N * nc));
    dim3 gr = grid_for((int)G.n[0], (int)G.n[1], (int)G.n[2], BLK);
    dispatch(dim, c_->kind, [&](auto D, auto K) {
      hipLaunchKernelGGL((build_coef_k<double, D.value, K.value>), gr, BLK, 0, c_->stream,
                         tensor_l, (int)G.n[0], (int)G.n[1], (int)G.n[2],
                         coef_factors(G.h, c_->d.time_step), cf64, nc);
    });
    HIP_CHECK(hipGetLastError());
    coarse_coef64_.resize((size_t)G.N * nc);
    HIP_CHECK(hipMemcpyAsync(coarse_coef64_.data(), cf64, sizeof(double) * G.N * nc,
                             hipMemcpyDeviceToHost, c_->stream));
    HIP_CHECK(hipStreamSynchronize(c_->stream));
    HIP_CHECK(hipFree(cf64));
  }

  // Row p of the coarsest operator from its fp64 coefficient records (mirror ghosts
  // folded): emit(col, v) for A[p][col] += v, in the order the dense matrix was always
  // assembled (DS.hxx:32-88 semantics; GH.hxx:298-516 via the matrix-free coefficients)
  template <typename Emit>
  void coarse_row(int64_t p, Emit&& emit) const {
    const int dim = c_->dim;
    const int kind = c_->kind;
    const LevelGeom& G = c_->geom[c_->nlev - 1];
    const double* cf = coarse_coef64_.data();
    const int na = (kind == KISO) ? 1 : dim;
    const int nc = coef_count(dim, kind);
    const int64_t nx = G.n[0], ny = G.n[1], nz = G.n[2];
    const int64_t i = p % nx, j = (p / nx) % ny, k = p / (nx * ny);
    const double r1 = (G.h[0] * G.h[0]) / (G.h[1] * G.h[1]);
    const double r2 = (G.h[0] * G.h[0]) / (G.h[2] * G.h[2]);
    // point-interleaved, x-parity-split records (mad_kernels.hpp, cidx)
    const double* rec = cf + (nx * (j + ny * k) + ((i & 1) ? (nx + 1) / 2 + (i >> 1) : (i >> 1))) * nc;
    double a[3], g[3], e[3] = {0, 0, 0};
    if (kind == KISO) {
      a[0] = rec[0]; a[1] = rec[0] * r1; a[2] = rec[0] * r2;
    } else {
      for (int d = 0; d < dim; ++d) a[d] = rec[d];
    }
    for (int d = 0; d < dim; ++d) g[d] = rec[na + d];
    if (kind == KFULL)
      for (int qq = 0; qq < dim * (dim - 1) / 2; ++qq) e[qq] = rec[na + dim + qq];
    const int64_t xm = (i == 0) ? 1 : i - 1, xp = (i == nx - 1) ? nx - 2 : i + 1;
    const int64_t ym = (j == 0) ? 1 : j - 1, yp = (j == ny - 1) ? ny - 2 : j + 1;
    const int64_t zm = (k == 0) ? 1 : k - 1, zp = (k == nz - 1) ? nz - 2 : k + 1;
    auto idx = [&](int64_t ii, int64_t jj, int64_t kk) { return ii + nx * (jj + ny * kk); };
    emit(p, 1.0 + 2.0 * (a[0] + a[1] + (dim == 3 ? a[2] : 0.0)));
    // A u = D u - S  =>  A[p][q] -= coefficient of u(q) in S
    emit(idx(xp, j, k), -(a[0] + g[0]));
    emit(idx(xm, j, k), -(a[0] - g[0]));
    emit(idx(i, yp, k), -(a[1] + g[1]));
    emit(idx(i, ym, k), -(a[1] - g[1]));
    if (dim == 3) {
      emit(idx(i, j, zp), -(a[2] + g[2]));
      emit(idx(i, j, zm), -(a[2] - g[2]));
    }
    if (kind == KFULL) {
      emit(idx(xp, yp, k), -e[0]);
      emit(idx(xp, ym, k), e[0]);
      emit(idx(xm, yp, k), e[0]);
      emit(idx(xm, ym, k), -e[0]);
      if (dim == 3) {
        emit(idx(xp, j, zp), -e[1]);
        emit(idx(xp, j, zm), e[1]);
        emit(idx(xm, j, zp), e[1]);
        emit(idx(xm, j, zm), -e[1]);
        emit(idx(i, yp, zp), -e[2]);
        emit(idx(i, yp, zm), e[2]);
        emit(idx(i, ym, zp), e[2]);
        emit(idx(i, ym, zm), -e[2]);
      }
    }
  }

  // DirectSolver setup (DS.hxx:32-88: vnl_sparse_lu of the coarsest operator, any size).
  // Up to mad_desc.coarse_dense_max unknowns: dense LU -> explicit inverse, one GEMV per
  // solve.  Above: the block-plane LU of mad_coarse.hpp (thin volumes: 512x512x64 coarsens
  // to 64x64x8; any axis < 12 leaves the whole grid to the direct solver, GH.hxx:36-59).
  void build_coarse_inverse() {
    const int dim = c_->dim;
    const LevelGeom& G = c_->geom[c_->nlev - 1];
    const int64_t n = G.N;
    const int64_t dense_max = c_->d.coarse_dense_max > 0 ? c_->d.coarse_dense_max : MAD_COARSE_DENSE_MAX;
    const int target = c_->d.coarse_block_unknowns > 0 ? c_->d.coarse_block_unknowns : MAD_COARSE_BLOCK_UNKNOWNS;
    if (n > dense_max) {
      size_t free_b = 0, total_b = 0;
      HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
      // KL / KU chain matrices where they take at most half the free memory (one launch per
      // chain step); without them down to the Dinv blocks alone
      // (every rank that replicates the level takes the same decision: the same bits per solve)
      const bool with_chain = c_->comm.all_true(
          CoarseBlocks::estimate_bytes(dim, G.n, target, true) < free_b / 2 &&
              !(c_->d.options & MAD_OPT_COARSE_NO_CHAIN),
          c_->stream);
      const size_t need = CoarseBlocks::estimate_bytes(dim, G.n, target, with_chain);
      REQUIRE(need < free_b / 10 * 9, MAD_ERR_UNSUPPORTED,
              "coarsest grid has " + std::to_string(n) + " unknowns: its direct solver needs " +
                  std::to_string(need >> 20) + " MiB of device memory, " + std::to_string(free_b >> 20) +
                  " MiB free (an axis shorter than 12 leaves the whole grid to the direct solver, "
                  "GH.hxx:36-59)");
      bool ok = false;
      try {
        ok = cblk_.build(dim, G.n, target, with_chain,
                         [&](int64_t p, const CoarseBlocks::Emit& emit) { coarse_row(p, emit); },
                         c_->stream);
      } catch (const std::runtime_error& e) {
        throw MadError(MAD_ERR_UNSUPPORTED, e.what());
      }
      REQUIRE(ok, MAD_ERR_SINGULAR, "coarsest operator is singular");
      return;
    }
    {  // the dense inverse and getrf / getri's copy of A (2 n^2 fp64) must fit on the device
      const size_t need = 2 * sizeof(double) * (size_t)n * (size_t)n;
      size_t free_b = 0, total_b = 0;
      HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
      REQUIRE(need < free_b / 10 * 9, MAD_ERR_UNSUPPORTED,
              "coarsest grid has " + std::to_string(n) + " unknowns: its dense inverse needs " +
                  std::to_string(need >> 20) + " MiB of device memory, " + std::to_string(free_b >> 20) +
                  " MiB free (lower mad_desc.coarse_dense_max to use the block-plane LU)");
    }
    std::vector<double> A((size_t)n * n, 0.0);
    for (int64_t p = 0; p < n; ++p) {
      double* row = &A[(size_t)p * n];
      coarse_row(p, [&](int64_t col, double v) { row[col] += v; });
    }
    HIP_CHECK(hipMalloc(&inv_, sizeof(double) * n * n));
    REQUIRE(invert_dense_device(n, A, inv_, c_->stream), MAD_ERR_SINGULAR,
            "coarsest operator is singular");
  }

  // ---- distributed -> replicated hand-over (agglomeration of coarse levels)
  void ensure_gather(int64_t n) {
    if (n > gathered_cap_) {
      if (gathered_) HIP_CHECK(hipFree(gathered_));
      if (full_x_) HIP_CHECK(hipFree(full_x_));
      HIP_CHECK(hipMalloc(&gathered_, sizeof(T) * n));
      HIP_CHECK(hipMalloc(&full_x_, sizeof(T) * n));
      gathered_cap_ = n;
    }
  }

  // this rank's planes of the first replicated level (the hand-over descent, resid_restrict)
  T* coarse_slab(int64_t n) {
    if (n > cslab_cap_) {
      if (cslab_) HIP_CHECK(hipFree(cslab_));
      HIP_CHECK(hipMalloc(&cslab_, sizeof(T) * n));
      cslab_cap_ = n;
    }
    return cslab_;
  }

  // all ranks assemble the full level-l array from their slabs
  void gather_level(int l, const T* a) {
    const LevelGeom& G = c_->geom[l];
    ensure_gather(G.N);
    wait_all_pending();
    c_->comm.allgather_slabs(a, gathered_, G.n[0] * G.n[1], G.n[2], sizeof(T), c_->stream);
  }

  void restrict_full(int l, const T* fine_full, T* coarse) {
    const LevelGeom& Gf = c_->geom[l];
    LevelData<T>& C = lv_[l + 1];
    b_changed(l + 1);
    Geo gf{};
    gf.nx = (int)Gf.n[0]; gf.ny = (int)Gf.n[1]; gf.nz = (int)Gf.n[2];
    gf.sy = Gf.n[0]; gf.sz = Gf.n[0] * Gf.n[1]; gf.N = Gf.N;
    if (c_->dim == 3) {
      // z-marching (restrict3_k, the same taps and fma order as restrict_k): 64^3 from the gathered
      // 128^3 of an 8-rank cycle in 8.0 instead of 12-17 us per cycle with one thread per coarse point
      constexpr int CX = 32, CY = 8;
      const int ntx = (C.g.nx + CX - 1) / CX, nty = (C.g.ny + CY - 1) / CY;
      int chunks = std::max(1, std::min((xfer_blocks() + ntx * nty - 1) / (ntx * nty), std::max(1, C.g.nz / 4)));
      const int kc = (C.g.nz + chunks - 1) / chunks;
      chunks = (C.g.nz + kc - 1) / kc;
      hipLaunchKernelGGL((restrict3_k<T, T, CX, CY>), dim3((unsigned)(ntx * nty * chunks)), dim3(CX * CY), 0,
                         c_->stream, fine_full, gf, coarse, C.g, C.cent[0], C.cent[1], C.cent[2], 0,
                         (int)c_->geom[l + 1].n[2], kc, ntx);
    } else {
      dim3 gr = grid_for(C.g.nx, C.g.ny, C.g.nz, BLK);
      hipLaunchKernelGGL((restrict_k<T, T, 3>), gr, BLK, 0, c_->stream, fine_full, gf, coarse, C.g,
                         C.cent[0], C.cent[1], C.cent[2], 0);
    }
    HIP_CHECK(hipGetLastError());
  }

  // fine slab (distributed) from the replicated coarse level
  void interp_from_replicated(int l, bool add) {
    const bool ghosts = interp_ghosts(l, add);
    launch_interp3(l, add, ghosts);
    HIP_CHECK(hipGetLastError());
    if (ghosts) lv_[l].x_halo_ok = true;
    else x_changed(l);
  }

  // x[l] (+)= P x[l+1], 3D, z-marching (interp3_k): 64x16 fine columns, ~1024 blocks.
  // The coarse level may be a slab (ghost planes exchanged) or replicated (zoff 0).
  // fine points per thread in x where rows, planes and the array are aligned to them
#ifndef MAD_INTERP_VX
#define MAD_INTERP_VX 2
#endif
  void launch_interp3(int l, bool add, bool ghosts = false) {
    LevelData<T>& F = lv_[l];
    const int vx = (MAD_INTERP_VX > 1 && F.g.nx % 2 == 0 && F.g.sy % 2 == 0 && F.g.sz % 2 == 0 &&
                    ((uintptr_t)F.x % (2 * sizeof(T))) == 0) ? 2 : 1;
    if (vx == 2)
      launch_interp3_v<2>(l, add, ghosts);
    else
      launch_interp3_v<1>(l, add, ghosts);
  }
  template <int VX>
  void launch_interp3_v(int l, bool add, bool ghosts) {
    LevelData<T>& F = lv_[l];
    LevelData<T>& C = lv_[l + 1];
    constexpr int TX = 64, TY = 16;
    const int kbase = (ghosts && F.g.zlo_ghost) ? -GHOST : 0;
    const int kend = (ghosts && F.g.zhi_ghost) ? F.g.nz + GHOST : F.g.nz;
    const int nk = kend - kbase;
    const int ntx = (F.g.nx + TX * VX - 1) / (TX * VX), nty = (F.g.ny + TY - 1) / TY;
    int chunks = std::max(1, std::min((xfer_blocks() + ntx * nty - 1) / (ntx * nty), nk / 4));
    const int kc = (nk + chunks - 1) / chunks;
    chunks = (nk + kc - 1) / kc;
    const unsigned nb = (unsigned)(ntx * nty * chunks);
    const int ncz = (int)c_->geom[l + 1].n[2];
    if (add)
      hipLaunchKernelGGL((interp3_k<T, 1, TX, TY, 8, VX>), dim3(nb), dim3(TX * TY), 0, c_->stream, C.x,
                         C.g, F.x, F.g, C.cent[0], C.cent[1], C.cent[2], ncz, kc, ntx, kbase, kend);
    else
      hipLaunchKernelGGL((interp3_k<T, 0, TX, TY, 8, VX>), dim3(nb), dim3(TX * TY), 0, c_->stream, C.x,
                         C.g, F.x, F.g, C.cent[0], C.cent[1], C.cent[2], ncz, kc, ntx, kbase, kend);
  }

  // On a rank slab whose ghost planes are current, interpolation updates them too
  // (the neighbours' x + P e, computed from the exchanged x and coarse ghost planes:
  // the same values the neighbours compute), so the post-smoothing sweep needs no
  // exchange first.  Returns whether it does (the caller passes it to launch_interp3).
  bool interp_ghosts(int l, bool add) {
    LevelData<T>& F = lv_[l];
    if (!c_->comm.active() || !c_->geom[l].distributed || c_->dim != 3) return false;
    // a peer batch still in flight for x (the previous time step's last sweep, when FMG's
    // interpolation is the level's first use of x) is taken in first: it must not land on the
    // ghost planes this interpolation writes, and x += P e needs it there
    if (F.x_peer_pending) peer_resolve(l);
    if (add && !F.x_halo_ok) return false;
    wait_all_pending();  // the ghost planes may still be arriving
    return true;
  }
};

// ---------------------------------------------------------------------------
void set_error(mad_ctx* c, const std::string& m) {
  g_last_error = m;
  if (c) c->err = m;
}

template <typename F>
int guarded(mad_ctx* c, F&& f) {
  try {
    f();
    return MAD_OK;
  } catch (const MadError& e) {
    set_error(c, e.what());
    return e.code;
  } catch (const CommError& e) {
    set_error(c, e.what());
    return MAD_ERR_COMM;
  } catch (const std::bad_alloc&) {
    set_error(c, "out of host memory");
    return MAD_ERR_NOMEM;
  } catch (const std::exception& e) {
    set_error(c, e.what());
    return MAD_ERR_DEVICE;
  }
}

void use_device(mad_ctx* c) { HIP_CHECK(hipSetDevice(c->device)); }

// the level-0 tensor indexed by global point: component c of global point p at [c * tensor_cs + p]
// (valid for the planes the slab stores)
double* tensor_at0(const mad_ctx* c) {
  const LevelGeom& G = c->geom[0];
  return c->tensor64 + (c->tensor_tg - G.z0) * G.n[0] * G.n[1];
}

void tensor_alloc(mad_ctx* c) {
  if (c->tensor64) return;
  const int ncomp = c->dim * (c->dim + 1) / 2;
  HIP_CHECK(big_alloc((void**)&c->tensor64, sizeof(double) * ncomp * c->tensor_cs));
  // ghost planes outside the grid stay zero (never read)
  if (c->tensor_tg) HIP_CHECK(hipMemsetAsync(c->tensor64, 0, sizeof(double) * ncomp * c->tensor_cs, c->stream));
}

std::vector<LevelGeom> plan_geometry(const mad_desc& d) {
  const int dim = d.dim;
  int64_t n0[3] = {d.size[0], d.size[1], dim == 3 ? d.size[2] : 1};
  const int nlev = max_depth_rule(dim, n0) + 1;
  std::vector<LevelGeom> geom(nlev, LevelGeom{});
  for (int q = 0; q < 3; ++q) {
    geom[0].n[q] = (q < dim) ? n0[q] : 1;
    geom[0].h[q] = (q < dim) ? d.spacing[q] : 1.0;
    geom[0].cent[q] = 0;
  }
  for (int l = 1; l < nlev; ++l)  // GH.hxx:74-106
    for (int q = 0; q < 3; ++q) {
      const LevelGeom& F = geom[l - 1];
      LevelGeom& G = geom[l];
      G.h[q] = F.h[q] * 2;
      if (q >= dim) { G.n[q] = 1; G.cent[q] = 0; continue; }
      if (F.n[q] % 2 == 0) { G.n[q] = F.n[q] / 2; G.cent[q] = 1; }
      else { G.n[q] = (F.n[q] - 1) / 2 + 1; G.cent[q] = 0; }
    }
  for (auto& G : geom) {
    G.N = G.n[0] * G.n[1] * G.n[2];
    G.z0 = 0;
    G.z1 = G.n[2];
    G.distributed = false;
  }
  // z-slab decomposition: level l is distributed while every rank keeps >= min_slab_planes
  // planes and >= min_slab_voxels voxels (level 0: >= 4 planes), nz divides evenly and every
  // coarsening down to l halves z exactly (cell-centred), so fine planes 2K, 2K+1 and coarse
  // plane K share a rank.  The first level below that and all coarser ones are replicated on
  // every rank (agglomeration).
  if (d.nranks > 1) {
    REQUIRE(dim == 3, MAD_ERR_UNSUPPORTED, "z-slab decomposition needs a 3D image");
    const int P = d.nranks;
    REQUIRE(geom[0].n[2] % P == 0 && geom[0].n[2] / P >= 4, MAD_ERR_INVALID,
            "z size must split into >= 4 planes per rank");
    REQUIRE(nlev >= 2, MAD_ERR_UNSUPPORTED, "multi-GPU needs at least two levels");
    const int64_t minp = std::max(4, d.min_slab_planes > 0 ? d.min_slab_planes : MAD_MIN_SLAB_PLANES);
    const int64_t minv = d.min_slab_voxels > 0 ? d.min_slab_voxels : MAD_MIN_SLAB_VOXELS;
    int ld = 0;
    for (int l = 0; l < nlev - 1; ++l) {
      const LevelGeom& G = geom[l];
      bool ok = (G.n[2] % P == 0) && (G.n[2] / P >= (l == 0 ? 4 : minp));
      if (l > 0) ok = ok && G.n[0] * G.n[1] * (G.n[2] / P) >= minv;
      for (int q = 1; q <= l; ++q) ok = ok && (geom[q].cent[2] == 1);
      if (!ok) break;
      ld = l;
    }
    for (int l = 0; l <= ld; ++l) {
      LevelGeom& G = geom[l];
      const int64_t per = G.n[2] / P;
      G.z0 = per * d.rank;
      G.z1 = G.z0 + per;
      G.distributed = true;
    }
  }
  return geom;
}

void compute_geometry(mad_ctx* c) {
  c->geom = plan_geometry(c->d);
  c->nlev = (int)c->geom.size();
  const LevelGeom& G = c->geom[0];
  c->tensor_tg = G.distributed ? TENSOR_GHOST : 0;
  c->tensor_cs = (G.z1 - G.z0 + 2 * c->tensor_tg) * G.n[0] * G.n[1];
  c->tensor_lo = std::max<int64_t>(G.z0 - c->tensor_tg, 0);
  c->tensor_hi = std::min<int64_t>(G.z1 + c->tensor_tg, G.n[2]);
}

}  // namespace

// ===========================================================================
// C ABI
extern "C" {

int mad_desc_init(mad_desc* d) {
  if (!d) return MAD_ERR_INVALID;
  std::memset(d, 0, sizeof(*d));
  d->abi_version = MAD_ABI_VERSION;
  d->dim = 3;
  d->size[0] = d->size[1] = d->size[2] = 1;
  d->spacing[0] = d->spacing[1] = d->spacing[2] = 1.0;
  d->cycle = MAD_VCYCLE;               // MAD.hxx:41
  d->smoother = MAD_GAUSS_SEIDEL;      // MAD.h:90 default TSmootherType
  d->iterations_per_grid = 2;          // MAD.hxx:42
  d->max_cycles = 100;                 // MAD.hxx:44
  d->number_of_steps = 1;              // MAD.hxx:40
  d->time_step = 0.01;                 // MAD.hxx:39
  d->tolerance = 1e-6;                 // MAD.hxx:43
  d->omega = 2.0 / 3.0;                // itkMultigridWeightedJacobiSmoother.hxx:189
  d->verbose = 0;                      // MAD.hxx:45
  d->precision = MAD_PRECISION_AUTO;  // resolved by mad_create from the tolerance
  d->stall_guard = 1;
  d->device = -1;
  d->tensor_kind = MAD_TENSOR_AUTO;
  d->nranks = 1;
  d->rank = 0;
  return MAD_OK;
}

int mad_max_depth(int32_t dim, const int64_t size[3]) {
  if ((dim != 2 && dim != 3) || !size) return -1;
  for (int q = 0; q < dim; ++q)
    if (size[q] < 1) return -1;
  int64_t n[3] = {size[0], size[1], dim == 3 ? size[2] : 1};
  return max_depth_rule(dim, n);
}

const char* mad_last_error(const mad_ctx* c) { return c ? c->err.c_str() : g_last_error.c_str(); }

int mad_create(const mad_desc* d, mad_ctx** out) {
  if (!out) return MAD_ERR_INVALID;
  *out = nullptr;
  std::unique_ptr<mad_ctx> c(new mad_ctx());
  int rc = guarded(nullptr, [&] {
    REQUIRE(d, MAD_ERR_INVALID, "null descriptor");
    REQUIRE(d->abi_version == MAD_ABI_VERSION, MAD_ERR_INVALID, "ABI version mismatch");
    REQUIRE(d->dim == 2 || d->dim == 3, MAD_ERR_INVALID, "dim must be 2 or 3");
    for (int q = 0; q < d->dim; ++q) {
      REQUIRE(d->size[q] >= 3, MAD_ERR_INVALID,
              "every image axis needs >= 3 voxels (one-sided tensor derivatives, GH.hxx:447-474)");
      REQUIRE(d->spacing[q] > 0.0, MAD_ERR_INVALID, "spacing must be positive");
    }
    REQUIRE(d->size[0] * d->size[1] * (d->dim == 3 ? d->size[2] : 1) < (int64_t)INT32_MAX * 8,
            MAD_ERR_INVALID, "image too large");
    REQUIRE(d->cycle >= MAD_VCYCLE && d->cycle <= MAD_SMOOTHER, MAD_ERR_INVALID, "bad cycle");
    REQUIRE(d->smoother >= MAD_GAUSS_SEIDEL && d->smoother <= MAD_WEIGHTED_JACOBI,
            MAD_ERR_INVALID, "bad smoother");
    REQUIRE(d->precision == MAD_FP32 || d->precision == MAD_FP64 || d->precision == MAD_FP32_REFINE ||
                d->precision == MAD_PRECISION_AUTO,
            MAD_ERR_INVALID, "bad precision");
    REQUIRE(d->nranks >= 1 && d->rank >= 0 && d->rank < d->nranks, MAD_ERR_INVALID,
            "bad rank / nranks");
    REQUIRE(d->gs_kernel == 0 || d->gs_kernel == 1 || d->gs_kernel == 3 || d->gs_kernel == 4,
            MAD_ERR_INVALID, "gs_kernel must be 0, 1, 3 or 4");
    REQUIRE((d->options & ~(MAD_OPT_EAGER_RANK_VCYCLE | MAD_OPT_OVERLAP_RANK_SWEEP | MAD_OPT_PEER_HALO |
                            MAD_OPT_COARSE_NO_CHAIN | MAD_OPT_BENCHMARK_TRACE |
                            MAD_OPT_NO_PLACEMENT_TUNE | MAD_OPT_NO_RECORD_B)) == 0,
            MAD_ERR_INVALID, "unknown option bits");
    REQUIRE(d->min_slab_planes >= 0, MAD_ERR_INVALID, "min_slab_planes must be >= 0");
    REQUIRE(d->min_slab_voxels >= 0, MAD_ERR_INVALID, "min_slab_voxels must be >= 0");
    REQUIRE(d->coarse_dense_max >= 0 && d->coarse_dense_max <= MAD_COARSE_DENSE_LIMIT, MAD_ERR_INVALID,
            "coarse_dense_max must be in [0, " + std::to_string(MAD_COARSE_DENSE_LIMIT) +
                "] (a dense inverse of n unknowns takes 8 n^2 bytes on the host and twice that on the device)");
    REQUIRE(d->coarse_block_unknowns >= 0, MAD_ERR_INVALID, "coarse_block_unknowns must be >= 0");
    REQUIRE(d->tensor_kind >= MAD_TENSOR_AUTO && d->tensor_kind <= MAD_TENSOR_FULL,
            MAD_ERR_INVALID, "bad tensor kind");
    c->d = *d;
    // the default precision: fp32 storage resolves relres down to ~2e-7..8e-7
    // (profiles/r02_refine_cycles.md); a tolerance below MAD_FP32_TOLERANCE_FLOOR (the
    // reference tests ask for 1e-10) needs the fp64 defect correction to be reached
    if (c->d.precision == MAD_PRECISION_AUTO)
      c->d.precision = d->tolerance < MAD_FP32_TOLERANCE_FLOOR ? MAD_FP32_REFINE : MAD_FP32;
    if (c->d.dim == 2) c->d.size[2] = 1;
    c->dim = d->dim;
    int dev = d->device;
    if (dev < 0) HIP_CHECK(hipGetDevice(&dev));
    c->device = dev;
    use_device(c.get());
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    compute_geometry(c.get());
  });
  if (rc != MAD_OK) return rc;
  *out = c.release();
  return MAD_OK;
}

void mad_destroy(mad_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  delete c;
}

int mad_get_desc(const mad_ctx* c, mad_desc* out) {
  if (!c || !out) return MAD_ERR_INVALID;
  *out = c->d;
  return MAD_OK;
}

// p: AoS tensor of global planes [first, ...) covering the planes this context stores
// ([tensor_lo, tensor_hi): the whole grid on one rank, the slab and its ghost planes on a rank)
static int set_tensor_impl(mad_ctx* c, const void* p, int32_t dtype, bool dev, int64_t first,
                           int64_t nplanes) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    REQUIRE(p, MAD_ERR_INVALID, "null tensor");
    REQUIRE(dtype == MAD_F32 || dtype == MAD_F64, MAD_ERR_INVALID, "tensor dtype must be F32/F64");
    REQUIRE(first <= c->tensor_lo && first + nplanes >= c->tensor_hi, MAD_ERR_INVALID,
            "tensor planes [" + std::to_string(first) + ", " + std::to_string(first + nplanes) +
                ") do not cover [" + std::to_string(c->tensor_lo) + ", " + std::to_string(c->tensor_hi) +
                ") (mad_tensor_planes)");
    use_device(c);
    const LevelGeom& G = c->geom[0];
    const int ncomp = c->dim * (c->dim + 1) / 2;
    const int64_t sz = G.n[0] * G.n[1];
    const int64_t n = (c->tensor_hi - c->tensor_lo) * sz;  // points this context stores
    tensor_alloc(c);
    const size_t bytes = dtype_size(dtype) * n * ncomp;
    const void* src = (const char*)p + dtype_size(dtype) * (c->tensor_lo - first) * sz * ncomp;
    void* stage = nullptr;
    if (!dev) {
      HIP_CHECK(hipMalloc(&stage, bytes));
      HIP_CHECK(hipMemcpyAsync(stage, src, bytes, hipMemcpyHostToDevice, c->stream));
      src = stage;
    }
    double* dst = tensor_at0(c) + c->tensor_lo * sz;
    if (dtype == MAD_F64)
      hipLaunchKernelGGL((aos_to_soa_k<double>), dim3(flat_blocks(n)), dim3(256), 0, c->stream,
                         (const double*)src, dst, n, ncomp, c->tensor_cs);
    else
      hipLaunchKernelGGL((aos_to_soa_k<float>), dim3(flat_blocks(n)), dim3(256), 0, c->stream,
                         (const float*)src, dst, n, ncomp, c->tensor_cs);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(c->stream));
    if (stage) HIP_CHECK(hipFree(stage));
    c->tensor_set = true;
    c->setup_done = false;
  });
}

int mad_set_tensor(mad_ctx* c, const void* host_aos, int32_t dtype) {
  return c ? set_tensor_impl(c, host_aos, dtype, false, 0, c->geom[0].n[2]) : MAD_ERR_INVALID;
}

int mad_set_tensor_device(mad_ctx* c, const void* dev_aos, int32_t dtype) {
  return c ? set_tensor_impl(c, dev_aos, dtype, true, 0, c->geom[0].n[2]) : MAD_ERR_INVALID;
}

int mad_set_tensor_planes(mad_ctx* c, const void* host_aos, int32_t dtype, int64_t first_plane,
                          int64_t nplanes) {
  return c ? set_tensor_impl(c, host_aos, dtype, false, first_plane, nplanes) : MAD_ERR_INVALID;
}

int mad_tensor_planes(const mad_ctx* c, int64_t* first_plane, int64_t* nplanes) {
  if (!c || !first_plane || !nplanes) return MAD_ERR_INVALID;
  *first_plane = c->tensor_lo;
  *nplanes = c->tensor_hi - c->tensor_lo;
  return MAD_OK;
}

int mad_bench_synth_tensor(mad_ctx* c, int32_t kind, uint64_t seed) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    use_device(c);
    const LevelGeom& G = c->geom[0];
    tensor_alloc(c);
    const int kb = (int)c->tensor_lo;
    dim3 gr = grid_for((int)G.n[0], (int)G.n[1], (int)(c->tensor_hi - c->tensor_lo), BLK);
    if (kind == 0) {
      REQUIRE(c->dim == 3, MAD_ERR_INVALID, "VED-form synthetic tensor is 3D");
      hipLaunchKernelGGL(synth_ved_k, gr, BLK, 0, c->stream, tensor_at0(c), (int)G.n[0],
                         (int)G.n[1], (int)G.n[2], seed, 0.01, 1.5, 10.0, kb, c->tensor_cs);
    } else if (kind == 1) {
      hipLaunchKernelGGL(synth_iso_k, gr, BLK, 0, c->stream, tensor_at0(c), (int)G.n[0],
                         (int)G.n[1], (int)G.n[2], c->dim, seed, kb, c->tensor_cs);
    } else {
      throw MadError(MAD_ERR_INVALID, "unknown synthetic tensor kind");
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(c->stream));
    c->tensor_set = true;
    c->setup_done = false;
  });
}

static void setup_impl(mad_ctx* c) {
  REQUIRE(c->tensor_set, MAD_ERR_STATE, "SetDiffusionTensor (mad_set_tensor) must come first");
  use_device(c);
  REQUIRE(c->d.nranks == 1 || c->comm.active(), MAD_ERR_STATE,
          "nranks > 1: join the communicator (mad_comm_init*) before mad_setup (the operator "
          "build exchanges tensor ghost planes)");
  auto t0 = std::chrono::steady_clock::now();
  const LevelGeom& G = c->geom[0];
  // resolve the tensor kind (over all ranks: every slab must build the same kind of operator),
  // and reject a non-finite tensor (it would surface later as a singular coarsest operator or
  // a NaN image)
  int kind = KFULL;
  {
    const int64_t sz = G.n[0] * G.n[1];
    const int64_t n = (G.z1 - G.z0) * sz;  // owned points
    unsigned int* flags = nullptr;
    HIP_CHECK(hipMalloc(&flags, sizeof(unsigned int) * 3));
    HIP_CHECK(hipMemsetAsync(flags, 0, sizeof(unsigned int) * 3, c->stream));
    hipLaunchKernelGGL(tensor_kind_k, dim3(flat_blocks(n, 2048)), dim3(256), 0, c->stream,
                       tensor_at0(c) + G.z0 * sz, n, c->tensor_cs, c->dim, flags);
    HIP_CHECK(hipGetLastError());
    unsigned int hf[3];
    HIP_CHECK(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipFree(flags));
    if (c->comm.active()) {
      double v[3] = {(double)hf[0], (double)hf[1], (double)hf[2]};
      c->comm.allreduce_host(v, 3, 1, c->stream);
      for (int q = 0; q < 3; ++q) hf[q] = v[q] != 0.0;
    }
    REQUIRE(hf[2] == 0, MAD_ERR_NUMERIC, "diffusion tensor has non-finite (NaN / Inf) entries");
    if (c->d.tensor_kind == MAD_TENSOR_AUTO) kind = hf[0] ? KFULL : (hf[1] ? KDIAG : KISO);
    else kind = c->d.tensor_kind;  // MAD_TENSOR_* == KISO/KDIAG/KFULL
  }
  c->kind = kind;
  c->ncolors = (kind == KFULL) ? 4 : 2;
  if (!c->solver) {
    if (c->d.precision == MAD_FP64) c->solver.reset(new Solver<double>());
    else c->solver.reset(new Solver<float>());
  }
  c->solver->setup(c);
  c->setup_done = true;
  c->setup_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int mad_setup(mad_ctx* c) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] { setup_impl(c); });
}

static int run_impl(mad_ctx* c, const void* in, int32_t in_dtype, void* out, int32_t out_dtype,
                    mad_stats* st, bool dev) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    REQUIRE(in && out, MAD_ERR_INVALID, "null image buffer");
    REQUIRE(dtype_size(in_dtype) && dtype_size(out_dtype), MAD_ERR_INVALID, "bad dtype");
    if (!c->setup_done) setup_impl(c);
    use_device(c);
    c->solver->run(in, in_dtype, out, out_dtype, dev, st);
  });
}

// MAD_ERR_NOT_CONVERGED when the stall guard ended a step above Tolerance (the output and
// the stats are written): a port that asks fp32 storage for 1e-10 learns it from the status,
// not only from stats.stalled
static int run_status(mad_ctx* c, int rc, const mad_stats& st) {
  if (rc != MAD_OK || !st.stalled) return rc;
  char buf[256];
  std::snprintf(buf, sizeof buf,
                "tolerance %g not reached: the stall guard ended a time step at relres %g (the %s "
                "floor); MAD_FP32_REFINE or MAD_FP64 reach the reference tolerances",
                c->d.tolerance, st.last_relres, c->d.precision == MAD_FP64 ? "fp64" : "fp32");
  c->err = buf;
  return MAD_ERR_NOT_CONVERGED;
}

int mad_run(mad_ctx* c, const void* in, int32_t in_dtype, void* out, int32_t out_dtype,
            mad_stats* st) {
  mad_stats local{};
  mad_stats* s = st ? st : &local;
  return run_status(c, run_impl(c, in, in_dtype, out, out_dtype, s, false), *s);
}

int mad_run_device(mad_ctx* c, const void* in, int32_t in_dtype, void* out, int32_t out_dtype,
                   mad_stats* st) {
  mad_stats local{};
  mad_stats* s = st ? st : &local;
  return run_status(c, run_impl(c, in, in_dtype, out, out_dtype, s, true), *s);
}

int mad_get_step_stats(const mad_ctx* c, uint32_t step, uint32_t* cycles, double* relres) {
  if (!c || step >= c->step_cycles.size()) return MAD_ERR_INVALID;
  if (cycles) *cycles = c->step_cycles[step];
  if (relres) *relres = c->step_relres[step];
  return MAD_OK;
}

int mad_placement_trials(const mad_ctx* c, uint32_t cap, double* ms, uint32_t* count) {
  if (!c || !count) return MAD_ERR_INVALID;
  const std::vector<double> v = c->solver ? c->solver->placement_ms() : std::vector<double>{};
  for (size_t q = 0; q < v.size() && q < cap; ++q)
    if (ms) ms[q] = v[q];
  *count = (uint32_t)v.size();
  return MAD_OK;
}

int mad_get_cycle_trace(const mad_ctx* c, uint32_t cap, uint32_t* step, double* relres,
                        double* seconds, uint32_t* count) {
  if (!c) return MAD_ERR_INVALID;
  const size_t n = c->trace.size();
  for (size_t q = 0; q < n && q < cap; ++q) {
    if (step) step[q] = c->trace[q].step;
    if (relres) relres[q] = c->trace[q].relres;
    if (seconds) seconds[q] = c->trace[q].seconds;
  }
  if (count) *count = (uint32_t)n;
  return MAD_OK;
}

int mad_num_levels(const mad_ctx* c) { return c ? c->nlev : -1; }

int mad_plan_level(const mad_desc* d, int32_t level, int64_t size[3], double spacing[3],
                   int32_t centering[3], int64_t* z_begin, int64_t* z_end,
                   int32_t* distributed) {
  int nl = -1;
  int rc = guarded(nullptr, [&] {
    REQUIRE(d && d->abi_version == MAD_ABI_VERSION, MAD_ERR_INVALID, "bad descriptor");
    REQUIRE(d->dim == 2 || d->dim == 3, MAD_ERR_INVALID, "dim must be 2 or 3");
    REQUIRE(d->nranks >= 1 && d->rank >= 0 && d->rank < d->nranks, MAD_ERR_INVALID,
            "bad rank / nranks");
    for (int q = 0; q < d->dim; ++q) REQUIRE(d->size[q] >= 3, MAD_ERR_INVALID, "axis < 3");
    std::vector<LevelGeom> g = plan_geometry(*d);
    nl = (int)g.size();
    REQUIRE(level >= 0 && level < nl, MAD_ERR_INVALID, "bad level");
    const LevelGeom& G = g[level];
    for (int q = 0; q < 3; ++q) {
      if (size) size[q] = G.n[q];
      if (spacing) spacing[q] = G.h[q];
      if (centering) centering[q] = G.cent[q];
    }
    if (z_begin) *z_begin = G.z0;
    if (z_end) *z_end = G.z1;
    if (distributed) *distributed = G.distributed ? 1 : 0;
  });
  return rc == MAD_OK ? nl : -rc;
}

int mad_level_info(const mad_ctx* c, int32_t level, int64_t size[3], double spacing[3],
                   int32_t centering[3]) {
  if (!c || level < 0 || level >= c->nlev) return MAD_ERR_INVALID;
  const LevelGeom& G = c->geom[level];
  for (int q = 0; q < 3; ++q) {
    if (size) size[q] = (q == 2) ? (G.z1 - G.z0) : G.n[q];
    if (spacing) spacing[q] = G.h[q];
    if (centering) centering[q] = G.cent[q];
  }
  return MAD_OK;
}

#define KERNEL_ENTRY(body)                                                     \
  if (!c) return MAD_ERR_INVALID;                                              \
  return guarded(c, [&] {                                                      \
    REQUIRE(c->setup_done, MAD_ERR_STATE, "mad_setup must be called first");  \
    use_device(c);                                                             \
    body;                                                                      \
  })

#define CHECK_LEVEL(l) REQUIRE((l) >= 0 && (l) < c->nlev, MAD_ERR_INVALID, "bad level")
#define CHECK_WHICH(w) REQUIRE((w) >= MAD_X && (w) <= MAD_R, MAD_ERR_INVALID, "bad array selector")

int mad_upload(mad_ctx* c, int32_t level, int32_t which, const double* host) {
  KERNEL_ENTRY(CHECK_LEVEL(level); CHECK_WHICH(which);
               REQUIRE(host, MAD_ERR_INVALID, "null buffer");
               c->solver->upload(level, which, host));
}

int mad_download(mad_ctx* c, int32_t level, int32_t which, double* host) {
  KERNEL_ENTRY(CHECK_LEVEL(level); CHECK_WHICH(which);
               REQUIRE(host, MAD_ERR_INVALID, "null buffer");
               c->solver->download(level, which, host));
}

int mad_fill(mad_ctx* c, int32_t level, int32_t which, double value) {
  KERNEL_ENTRY(CHECK_LEVEL(level); CHECK_WHICH(which); c->solver->fill(level, which, value));
}

int mad_smooth(mad_ctx* c, int32_t level, uint32_t sweeps) {
  KERNEL_ENTRY(CHECK_LEVEL(level); c->solver->smooth(level, sweeps));
}

int mad_residual(mad_ctx* c, int32_t level, double* norm_out) {
  KERNEL_ENTRY(CHECK_LEVEL(level); double v = c->solver->residual(level, norm_out != nullptr);
               if (norm_out) { c->solver->check_device_errors(); *norm_out = v; });
}

int mad_norm(mad_ctx* c, int32_t level, int32_t which, double* norm_out) {
  KERNEL_ENTRY(CHECK_LEVEL(level); CHECK_WHICH(which);
               REQUIRE(norm_out, MAD_ERR_INVALID, "null output");
               const double v = c->solver->norm(level, which);
               c->solver->check_device_errors(); *norm_out = v);
}

int mad_restrict(mad_ctx* c, int32_t level) {
  KERNEL_ENTRY(REQUIRE(level >= 0 && level < c->nlev - 1, MAD_ERR_INVALID, "bad level");
               c->solver->restrict_(level));
}

int mad_residual_restrict(mad_ctx* c, int32_t level, int32_t* fused) {
  KERNEL_ENTRY(REQUIRE(level >= 0 && level < c->nlev - 1, MAD_ERR_INVALID, "bad level");
               const bool f = c->solver->residual_restrict(level);
               if (!f) {
                 c->solver->residual(level, false);
                 c->solver->restrict_(level);
               }
               if (fused) *fused = f ? 1 : 0);
}

int mad_interpolate(mad_ctx* c, int32_t level) {
  KERNEL_ENTRY(REQUIRE(level >= 0 && level < c->nlev - 1, MAD_ERR_INVALID, "bad level");
               c->solver->interpolate(level, false));
}

int mad_prolongate_add(mad_ctx* c, int32_t level) {
  KERNEL_ENTRY(REQUIRE(level >= 0 && level < c->nlev - 1, MAD_ERR_INVALID, "bad level");
               c->solver->interpolate(level, true));
}

int mad_coarse_solve(mad_ctx* c) { KERNEL_ENTRY(c->solver->coarse_solve()); }

int mad_vcycle(mad_ctx* c) { KERNEL_ENTRY(c->solver->vcycle()); }

int mad_fmg(mad_ctx* c) { KERNEL_ENTRY(c->solver->fmg()); }

int mad_synchronize(mad_ctx* c) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    use_device(c);
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipStreamSynchronize(c->comm_stream));
    if (c->solver) c->solver->check_device_errors();
  });
}

int mad_bench_smooth(mad_ctx* c, int32_t level, uint32_t sweeps, double* total_ms,
                     double* kernel_ms_mean, uint32_t* kernel_launches) {
  KERNEL_ENTRY(CHECK_LEVEL(level);
               REQUIRE(total_ms && kernel_ms_mean && kernel_launches, MAD_ERR_INVALID, "null out");
               unsigned nl = 0; c->solver->bench_smooth(level, sweeps, total_ms, kernel_ms_mean, &nl);
               *kernel_launches = nl);
}

int mad_bench_launch_times(mad_ctx* c, float* ms, uint32_t cap, uint32_t* n) {
  KERNEL_ENTRY(REQUIRE(n && (ms || cap == 0), MAD_ERR_INVALID, "null out");
               const std::vector<float>& v = c->solver->launch_ms;
               const uint32_t k = std::min<uint32_t>(cap, (uint32_t)v.size());
               for (uint32_t i = 0; i < k; ++i) ms[i] = v[i];
               *n = k);
}

int mad_smooth_kernel_name(mad_ctx* c, int32_t level, char* buf, int32_t len) {
  KERNEL_ENTRY(CHECK_LEVEL(level);
               REQUIRE(buf && len > 0, MAD_ERR_INVALID, "null or empty buffer");
               const std::string n = c->solver->smooth_kernel(level);
               std::snprintf(buf, (size_t)len, "%s", n.c_str()));
}

int mad_bench_vcycle(mad_ctx* c, uint32_t cycles, double* total_ms) {
  KERNEL_ENTRY(REQUIRE(total_ms, MAD_ERR_INVALID, "null out");
               c->solver->bench_vcycle(cycles, total_ms));
}

int mad_bench_synth_level(mad_ctx* c, int32_t level, int32_t which, uint64_t seed) {
  KERNEL_ENTRY(CHECK_LEVEL(level); CHECK_WHICH(which); c->solver->synth_level(level, which, seed));
}

int mad_slab_range(int64_t nz, int32_t nranks, int32_t rank, int32_t align, int64_t* z_begin,
                   int64_t* z_end) {
  if (nz < 1 || nranks < 1 || rank < 0 || rank >= nranks || align < 1 || !z_begin || !z_end)
    return MAD_ERR_INVALID;
  if (nz % ((int64_t)nranks * align) != 0) return MAD_ERR_INVALID;
  const int64_t per = nz / nranks;
  *z_begin = per * rank;
  *z_end = per * (rank + 1);
  return MAD_OK;
}

int mad_comm_unique_id(void* uid128) {
  if (!uid128) return MAD_ERR_INVALID;
  return guarded(nullptr, [&] { Comm::unique_id(uid128); });
}

int mad_comm_init(mad_ctx* c, const void* uid128) {
  if (!c || !uid128) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    REQUIRE(!c->setup_done, MAD_ERR_STATE, "mad_comm_init must precede mad_setup");
    use_device(c);
    c->comm.init(uid128, c->d.nranks, c->d.rank, c->device);
  });
}

int mad_comm_selftest(int32_t device, double* max_err) {
  if (!max_err) return MAD_ERR_INVALID;
  return guarded(nullptr, [&] {
    HIP_CHECK(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    char uid[128];
    Comm::unique_id(uid);
    Comm comm;
    comm.init_rccl(uid, 1, 0);
    // a float slab of NZ planes of P elements with GHOST ghost planes per side; plane z
    // (ghosts included) holds z + e / P
    constexpr int NZ = 12, P = 96 * 80;
    const int NT = NZ + 2 * GHOST;
    std::vector<float> h((size_t)NT * P);
    for (int z = 0; z < NT; ++z)
      for (int e = 0; e < P; ++e) h[(size_t)z * P + e] = (float)(z - GHOST) + (float)e / P;
    float* d = nullptr;
    HIP_CHECK(hipMalloc(&d, sizeof(float) * h.size()));
    HIP_CHECK(hipMemcpy(d, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice));
    float* base = d + (size_t)GHOST * P;
    comm.exchange_planes(base, P, NZ, GHOST, 1, 1, sizeof(float), false, s);
    // allreduce of one fp64 value, allgather of the (single) slab
    double* v = nullptr;
    HIP_CHECK(hipMalloc(&v, sizeof(double)));
    const double one = 1.25;
    HIP_CHECK(hipMemcpy(v, &one, sizeof one, hipMemcpyHostToDevice));
    comm.allreduce_sum_f64(v, 1, s);
    float* g = nullptr;
    HIP_CHECK(hipMalloc(&g, sizeof(float) * (size_t)NZ * P));
    comm.allgather_slabs(base, g, P, NZ, sizeof(float), s);
    HIP_CHECK(hipStreamSynchronize(s));
    std::vector<float> o(h.size()), og((size_t)NZ * P);
    double vr = 0.0;
    HIP_CHECK(hipMemcpy(o.data(), d, sizeof(float) * o.size(), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(og.data(), g, sizeof(float) * og.size(), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(&vr, v, sizeof vr, hipMemcpyDeviceToHost));
    // sends and receives between one pair of ranks match in issue order: the lower
    // ghosts receive the slab's first GHOST planes, the upper ghosts its last GHOST
    double err = std::fabs(vr - one);
    for (int z = 0; z < NT; ++z) {
      const int src = z < GHOST ? GHOST + z : (z >= NZ + GHOST ? z - GHOST : z);
      for (int e = 0; e < P; ++e)
        err = std::max(err, (double)std::fabs(o[(size_t)z * P + e] - h[(size_t)src * P + e]));
    }
    for (size_t q = 0; q < og.size(); ++q)
      err = std::max(err, (double)std::fabs(og[q] - h[(size_t)GHOST * P + q]));
    // the same three operations captured into a hipGraph and replayed (the multi-rank
    // V-cycle graph holds them, vcycle_fast): inputs reset, outputs cleared first
    {
      hipGraph_t gph = nullptr;
      hipGraphExec_t gx = nullptr;
      HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      comm.exchange_planes(base, P, NZ, GHOST, 1, 1, sizeof(float), false, s);
      comm.allreduce_sum_f64(v, 1, s);
      comm.allgather_slabs(base, g, P, NZ, sizeof(float), s);
      HIP_CHECK(hipStreamEndCapture(s, &gph));
      HIP_CHECK(hipGraphInstantiate(&gx, gph, nullptr, nullptr, 0));
      for (int rep = 0; rep < 2; ++rep) {
        HIP_CHECK(hipMemcpy(d, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(v, &one, sizeof one, hipMemcpyHostToDevice));
        HIP_CHECK(hipMemset(g, 0, sizeof(float) * (size_t)NZ * P));
        HIP_CHECK(hipGraphLaunch(gx, s));
        HIP_CHECK(hipStreamSynchronize(s));
        HIP_CHECK(hipMemcpy(o.data(), d, sizeof(float) * o.size(), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(og.data(), g, sizeof(float) * og.size(), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(&vr, v, sizeof vr, hipMemcpyDeviceToHost));
        err = std::max(err, std::fabs(vr - one));
        for (int z = 0; z < NT; ++z) {
          const int src = z < GHOST ? GHOST + z : (z >= NZ + GHOST ? z - GHOST : z);
          for (int e = 0; e < P; ++e)
            err = std::max(err, (double)std::fabs(o[(size_t)z * P + e] - h[(size_t)src * P + e]));
        }
        for (size_t q = 0; q < og.size(); ++q)
          err = std::max(err, (double)std::fabs(og[q] - h[(size_t)GHOST * P + q]));
      }
      (void)hipGraphExecDestroy(gx);
      (void)hipGraphDestroy(gph);
    }
    *max_err = err;
    comm.destroy();
    (void)hipFree(d);
    (void)hipFree(v);
    (void)hipFree(g);
    (void)hipStreamDestroy(s);
  });
}

int mad_comm_allreduce_host(mad_ctx* c, double* values, uint32_t n, int32_t op) {
  if (!c || (!values && n) || (op != 0 && op != 1)) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    use_device(c);
    c->comm.allreduce_host(values, n, op, c->stream);
  });
}

int mad_comm_version(int32_t* runtime, int32_t* compiled) {
  if (!runtime || !compiled) return MAD_ERR_INVALID;
  return guarded(nullptr, [&] {
    *runtime = Comm::runtime_version();
    *compiled = NCCL_VERSION_CODE;
  });
}

int mad_comm_init_local(mad_ctx* c, uint64_t group) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    REQUIRE(!c->setup_done, MAD_ERR_STATE, "mad_comm_init_local must precede mad_setup");
    use_device(c);
    c->comm.init_local(group, c->d.nranks, c->d.rank);
  });
}

int mad_comm_init_solo(mad_ctx* c) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    REQUIRE(!c->setup_done, MAD_ERR_STATE, "mad_comm_init_solo must precede mad_setup");
    use_device(c);
    c->comm.init_solo(c->d.nranks, c->d.rank);
  });
}

int mad_comm_init_rccl_solo(mad_ctx* c) {
  if (!c) return MAD_ERR_INVALID;
  return guarded(c, [&] {
    REQUIRE(!c->setup_done, MAD_ERR_STATE, "mad_comm_init_rccl_solo must precede mad_setup");
    use_device(c);
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    c->comm.init_rccl_self(c->d.nranks, c->d.rank, dev);
  });
}

}  // extern "C"

// VED pipeline (include/mad_ved.h): the caller of the hot path, same library
#include "mad_ved.hpp"
