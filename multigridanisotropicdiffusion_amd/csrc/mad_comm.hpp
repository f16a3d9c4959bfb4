// mad_comm.hpp -- transports for the z-slab decomposition.
//
// The reference is single-threaded and has no distributed path; this is the
// MI355X addition.  Two interchangeable backends implement the
// three exchanges the solver uses:
//   exchange_planes   `depth` ghost planes per z face with rank +-1
//   allreduce_sum_f64 ||r||^2 partial sums (8 bytes per V-cycle)
//   allgather_slabs   hand-over from the deepest distributed level to the first
//                     replicated coarse level (a few hundred KiB)
// RCCL   one process per GPU, grouped ncclSend/ncclRecv + collectives over xGMI.
// LOCAL  several ranks as host threads of ONE process (any device, typically the
//        same GPU): device-to-device copies between the ranks' own arrays, host
//        barriers for ordering.  It exists so the decomposition (ghost planes,
//        global colour parity, coarsening alignment, agglomeration) is testable
//        bit-for-bit on a one-GPU machine; RCCL and LOCAL move the same bytes.
// SOLO   measurement only: one rank of an N-rank decomposition alone on its device.
//        Every exchange is one stream-ordered copy launch of the same bytes within the
//        rank's own arrays (its boundary planes into its ghost planes, its slab into every
//        slot of a gather, the allreduce a no-op), so one rank's per-cycle device time --
//        hipGraph replay, boundary / interior launches, comm-stream overlap -- is measurable
//        on a one-GPU box.  The numbers it computes are not the decomposition's results.
//        RCCL-SOLO (init_rccl_self): the same stand-in exchanges through RCCL -- a single-rank
//        communicator, every grouped exchange ncclSend / ncclRecv to itself, the allreduce a
//        one-rank ncclAllReduce -- so the per-rank timing includes RCCL's kernels, their
//        launch latency and their capture into the V-cycle graph (not xGMI bandwidth).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace mad {

struct CommError : std::runtime_error {
  explicit CommError(const std::string& m) : std::runtime_error(m) {}
};

#define NCCL_CHECK(x)                                                                        \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw CommError(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

#define HIPC_CHECK(x)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw CommError(std::string(#x) + ": " + hipGetErrorString(e_));  \
  } while (0)

// process-local rendezvous for the LOCAL backend
struct LocalGroup {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> ptr;   // per-rank published array base (plane 0)
  std::vector<double> val;        // per-rank scalars for allreduce
  explicit LocalGroup(int nranks) : n(nranks), ptr(nranks, nullptr), val(nranks, 0.0) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t gen = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen; })) {
      throw CommError("local group barrier timed out (a rank failed or diverged)");
    }
  }
};

inline std::shared_ptr<LocalGroup> local_group(uint64_t key, int nranks) {
  static std::mutex m;
  static std::map<uint64_t, std::weak_ptr<LocalGroup>> groups;
  std::lock_guard<std::mutex> lk(m);
  auto it = groups.find(key);
  if (it != groups.end()) {
    if (auto g = it->second.lock()) {
      if (g->n != nranks) throw CommError("local group size mismatch");
      return g;
    }
  }
  auto g = std::make_shared<LocalGroup>(nranks);
  groups[key] = g;
  return g;
}

// SOLO's device copies.  One grouped exchange is one kernel launch, as RCCL issues a grouped
// ncclSend/ncclRecv (one kernel per ncclGroupEnd) -- not one copy launch per face or peer.
// Up to 8 segments per launch (blockIdx.y), each a multiple of 4 bytes; a segment whose
// pointers and size are 16-byte aligned moves uint4s.
struct CopyBatch {
  static constexpr int MAX = 8;
  int n = 0;
  char* dst[MAX];
  const char* src[MAX];
  uint64_t bytes[MAX];
};

__global__ void __launch_bounds__(256) copy_batch_k(CopyBatch b) {
  const int q = blockIdx.y;
  char* d = b.dst[q];
  const char* s = b.src[q];
  const uint64_t nb = b.bytes[q];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)d | (uintptr_t)s | nb) & 15) == 0) {
    uint4* d4 = (uint4*)d;
    const uint4* s4 = (const uint4*)s;
    for (uint64_t i = t0; i < nb / 16; i += stride) d4[i] = s4[i];
  } else {
    uint32_t* d1 = (uint32_t*)d;
    const uint32_t* s1 = (const uint32_t*)s;
    for (uint64_t i = t0; i < nb / 4; i += stride) d1[i] = s1[i];
  }
}

inline void copy_batch_flush(CopyBatch& b, hipStream_t st) {
  if (b.n == 0) return;
  uint64_t mx = 0;
  for (int q = 0; q < b.n; ++q) mx = std::max(mx, b.bytes[q]);
  const uint64_t blocks = std::min<uint64_t>(1024, std::max<uint64_t>(1, (mx / 16 + 255) / 256));
  hipLaunchKernelGGL(copy_batch_k, dim3((unsigned)blocks, (unsigned)b.n), dim3(256), 0, st, b);
  HIPC_CHECK(hipGetLastError());
  b.n = 0;
}

inline void copy_batch_add(CopyBatch& b, void* dst, const void* src, uint64_t bytes, hipStream_t st) {
  if (bytes == 0) return;
  if (bytes % 4) throw CommError("device copy of " + std::to_string(bytes) + " bytes (not a multiple of 4)");
  if (b.n == CopyBatch::MAX) copy_batch_flush(b, st);
  b.dst[b.n] = (char*)dst;
  b.src[b.n] = (const char*)src;
  b.bytes[b.n] = bytes;
  ++b.n;
}

class Comm {
 public:
  enum Mode { NONE, RCCL, LOCAL, SOLO };

  static void unique_id(void* out128) {
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
  }

  void init(const void* uid128, int nranks, int rank, int device) {
    destroy();
    if (nranks <= 1) return;
    init_rccl(uid128, nranks, rank, device);
  }

  // RCCL the process bound at run time (major * 10000 + minor * 100 + patch); a
  // process that loaded another librccl.so.1 first (torch bundles its own) binds that one
  static int runtime_version() {
    int v = 0;
    NCCL_CHECK(ncclGetVersion(&v));
    return v;
  }

  // an RCCL communicator of any size, one rank included (the transport self-test,
  // mad_comm_selftest: a single-rank communicator exchanges with itself).  The
  // communicator lives on `device` (>= 0; -1 keeps the current device).
  void init_rccl(const void* uid128, int nranks, int rank, int device = -1) {
    destroy();
    // the library is compiled against the ROCm RCCL headers: refuse a runtime library of
    // another major.minor (argument structs and enum values may differ between them)
    const int v = runtime_version();
    if (v / 100 != NCCL_VERSION_CODE / 100)
      throw CommError("RCCL runtime " + std::to_string(v) + " does not match the headers the "
                      "library was built with (" + std::to_string(NCCL_VERSION_CODE) +
                      "): load libmad_hip.so before anything that brings its own librccl "
                      "(e.g. import torch)");
    if (device >= 0) HIPC_CHECK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, uid128, sizeof(id));
    NCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
    mode_ = RCCL;
    nranks_ = nranks;
    rank_ = rank;
  }

  // RCCL-SOLO: a single-rank communicator standing in for rank `rank` of `nranks`
  void init_rccl_self(int nranks, int rank, int device) {
    destroy();
    if (nranks <= 1) return;
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    init_rccl(&id, 1, 0, device);
    self_ = true;
    nranks_ = nranks;
    rank_ = rank;
  }

  void init_local(uint64_t key, int nranks, int rank) {
    destroy();
    if (nranks <= 1) return;
    group_ = local_group(key, nranks);
    mode_ = LOCAL;
    nranks_ = nranks;
    rank_ = rank;
    group_->barrier();  // everyone joined
  }

  void init_solo(int nranks, int rank) {
    destroy();
    if (nranks <= 1) return;
    mode_ = SOLO;
    nranks_ = nranks;
    rank_ = rank;
  }

  void destroy() {
    if (graph_pending_ && graph_stream_) (void)hipStreamSynchronize(graph_stream_);
    graph_pending_ = false;
    graph_stream_ = nullptr;
    if (comm_) (void)ncclCommDestroy(comm_);
    comm_ = nullptr;
    group_.reset();
    self_ = false;
    mode_ = NONE;
    nranks_ = 1;
    rank_ = 0;
  }

  bool active() const { return mode_ != NONE && nranks_ > 1; }

  // A captured graph holding RCCL operations posts their proxy work when the device reaches
  // them, an eager RCCL call when it is enqueued: an eager call issued while such a graph is still
  // in flight can reach the proxy ahead of the graph's operations on one rank and behind them on
  // another, and the ranks' send / recv pairs no longer match (seen on two rank processes over the
  // socket transport as "message truncated", then a hang).  So the solver marks every launch of
  // such a graph, and the next eager RCCL call first waits for it (settle); calls being captured
  // are only recorded and need no wait.
  void graph_launched(hipStream_t s) {
    if (mode_ == RCCL) {
      graph_stream_ = s;
      graph_pending_ = true;
    }
  }
  void settle(hipStream_t s) {
    if (!graph_pending_) return;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    HIPC_CHECK(hipStreamIsCapturing(s, &st));
    if (st != hipStreamCaptureStatusNone) return;
    HIPC_CHECK(hipStreamSynchronize(graph_stream_));
    graph_pending_ = false;
  }
  // SOLO / RCCL-SOLO: the rank's own arrays stand in for its neighbours'
  bool stand_in() const { return mode_ == SOLO || (mode_ == RCCL && self_); }
  // RCCL peer of neighbour rank q (RCCL-SOLO: every peer is this process's only rank)
  int peer(int q) const { return self_ ? 0 : (q + nranks_) % nranks_; }
  Mode mode() const { return mode_; }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }

  // RCCL-SOLO: the SOLO copies (dst <- src, bytes a multiple of 4) as one group of ncclSend /
  // ncclRecv pairs to this process's only rank (pairs to one peer match in posting order)
  struct SelfPair {
    void* dst;
    const void* src;
    size_t bytes;
  };
  void self_exchange(const std::vector<SelfPair>& pairs, hipStream_t s) {
    NCCL_CHECK(ncclGroupStart());
    for (const SelfPair& q : pairs) {
      if (!q.bytes) continue;
      NCCL_CHECK(ncclSend(q.src, q.bytes / 4, ncclFloat, 0, comm_, s));
      NCCL_CHECK(ncclRecv(q.dst, q.bytes / 4, ncclFloat, 0, comm_, s));
    }
    NCCL_CHECK(ncclGroupEnd());
  }

  // a: base pointer of local plane 0; planes -depth..-1 and nz..nz+depth-1 are ghosts.
  // The first / last `depth` owned planes go to rank -+ 1.
  void exchange_planes(void* a, int64_t plane, int nz, int depth, int has_lo, int has_hi,
                       size_t esz, bool is_double, hipStream_t s) {
    char* base = (char*)a;
    const size_t pb = (size_t)plane * esz;
    settle(s);
    if (mode_ == RCCL && self_) {  // SOLO's bytes: own boundary planes into own ghost planes
      std::vector<SelfPair> q;
      if (has_lo) q.push_back({base - depth * pb, base, depth * pb});
      if (has_hi) q.push_back({base + (size_t)nz * pb, base + (size_t)(nz - depth) * pb, depth * pb});
      self_exchange(q, s);
      return;
    }
    if (mode_ == RCCL) {
      const ncclDataType_t dt = is_double ? ncclDouble : ncclFloat;
      const size_t cnt = (size_t)plane * depth;
      // neighbour ranks (has_lo / has_hi are false at the global ends; the modulo only
      // matters for the single-rank self-test, where both neighbours are this rank)
      const int lo = peer(rank_ - 1), hi = peer(rank_ + 1);
      NCCL_CHECK(ncclGroupStart());
      if (has_lo) {
        NCCL_CHECK(ncclSend(base, cnt, dt, lo, comm_, s));
        NCCL_CHECK(ncclRecv(base - depth * pb, cnt, dt, lo, comm_, s));
      }
      if (has_hi) {
        NCCL_CHECK(ncclSend(base + (size_t)(nz - depth) * pb, cnt, dt, hi, comm_, s));
        NCCL_CHECK(ncclRecv(base + (size_t)nz * pb, cnt, dt, hi, comm_, s));
      }
      NCCL_CHECK(ncclGroupEnd());
      return;
    }
    if (mode_ == SOLO) {  // the same bytes, own boundary planes into own ghost planes
      CopyBatch b;
      if (has_lo) copy_batch_add(b, base - depth * pb, base, depth * pb, s);
      if (has_hi) copy_batch_add(b, base + (size_t)nz * pb, base + (size_t)(nz - depth) * pb, depth * pb, s);
      copy_batch_flush(b, s);
      return;
    }
    // LOCAL: publish, pull the neighbours' boundary planes, wait until all pulled
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->ptr[rank_] = a;
    group_->barrier();
    if (has_lo) {
      const char* nb = (const char*)group_->ptr[rank_ - 1];  // same nz on every rank
      HIPC_CHECK(hipMemcpyAsync(base - depth * pb, nb + (size_t)(nz - depth) * pb, depth * pb,
                                hipMemcpyDeviceToDevice, s));
    }
    if (has_hi) {
      const char* nb = (const char*)group_->ptr[rank_ + 1];
      HIPC_CHECK(hipMemcpyAsync(base + (size_t)nz * pb, nb, depth * pb, hipMemcpyDeviceToDevice, s));
    }
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->barrier();
  }

  // One hop of a deep ghost exchange (ghost regions deeper than a slab, filled hop by hop): every
  // rank sends its planes [D, D + d) down (received at [nz + D, nz + D + d) by rank - 1) and
  // [nz - D - d, nz - D) up (received at [-D - d, -D) by rank + 1).  D = 0 is exchange_planes;
  // hop h (D = (h - 1) nz, d <= nz) forwards the ghosts hop h - 1 brought in.  Read and written
  // planes are disjoint, so the in-process transport pulls straight from the neighbours.
  void shift_planes(void* a, int64_t plane, int nz, int D, int d, int has_lo, int has_hi, size_t esz,
                    bool is_double, hipStream_t s) {
    if (D == 0) {
      exchange_planes(a, plane, nz, d, has_lo, has_hi, esz, is_double, s);
      return;
    }
    char* base = (char*)a;
    const size_t pb = (size_t)plane * esz;
    char* send_dn = base + (size_t)D * pb;
    char* recv_hi = base + (size_t)(nz + D) * pb;
    char* send_up = base + (ptrdiff_t)(nz - D - d) * (ptrdiff_t)pb;
    char* recv_lo = base - (ptrdiff_t)(D + d) * (ptrdiff_t)pb;
    settle(s);
    if (mode_ == RCCL && self_) {  // SOLO's bytes
      std::vector<SelfPair> q;
      if (has_lo) q.push_back({recv_lo, send_up, d * pb});
      if (has_hi) q.push_back({recv_hi, send_dn, d * pb});
      self_exchange(q, s);
      return;
    }
    if (mode_ == RCCL) {
      const ncclDataType_t dt = is_double ? ncclDouble : ncclFloat;
      const size_t cnt = (size_t)plane * d;
      const int lo = peer(rank_ - 1), hi = peer(rank_ + 1);
      NCCL_CHECK(ncclGroupStart());
      if (has_lo) {
        NCCL_CHECK(ncclSend(send_dn, cnt, dt, lo, comm_, s));
        NCCL_CHECK(ncclRecv(recv_lo, cnt, dt, lo, comm_, s));
      }
      if (has_hi) {
        NCCL_CHECK(ncclSend(send_up, cnt, dt, hi, comm_, s));
        NCCL_CHECK(ncclRecv(recv_hi, cnt, dt, hi, comm_, s));
      }
      NCCL_CHECK(ncclGroupEnd());
      return;
    }
    if (mode_ == SOLO) {  // the same bytes from this rank's own planes
      CopyBatch b;
      if (has_lo) copy_batch_add(b, recv_lo, send_up, d * pb, s);
      if (has_hi) copy_batch_add(b, recv_hi, send_dn, d * pb, s);
      copy_batch_flush(b, s);
      return;
    }
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->ptr[rank_] = a;
    group_->barrier();
    if (has_lo) {
      const char* nb = (const char*)group_->ptr[rank_ - 1];
      HIPC_CHECK(hipMemcpyAsync(recv_lo, nb + (ptrdiff_t)(nz - D - d) * (ptrdiff_t)pb, d * pb,
                                hipMemcpyDeviceToDevice, s));
    }
    if (has_hi) {
      const char* nb = (const char*)group_->ptr[rank_ + 1];
      HIPC_CHECK(hipMemcpyAsync(recv_hi, nb + (size_t)D * pb, d * pb, hipMemcpyDeviceToDevice, s));
    }
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->barrier();
  }

  // All-to-all of device buffers (the partitioned VED's transpose): send[r] (sbytes[r]) goes to
  // rank r, recv[q] (rbytes[q]) comes from rank q; entries of this rank are not moved.  Byte
  // counts are multiples of 4 (fp32 / fp64 volumes).
  void exchange_blocks(const std::vector<const void*>& send, const std::vector<size_t>& sbytes,
                       const std::vector<void*>& recv, const std::vector<size_t>& rbytes, hipStream_t s) {
    settle(s);
    if (mode_ == RCCL && self_) {  // the own blocks stand in for the peers' (as SOLO)
      std::vector<SelfPair> q;
      for (int r = 0; r < nranks_; ++r)
        if (r != rank_ && rbytes[r]) q.push_back({recv[r], send[r], std::min(sbytes[r], rbytes[r])});
      self_exchange(q, s);
      return;
    }
    if (mode_ == RCCL) {
      NCCL_CHECK(ncclGroupStart());
      for (int r = 0; r < nranks_; ++r) {
        if (r == rank_) continue;
        if (sbytes[r]) NCCL_CHECK(ncclSend(send[r], sbytes[r] / 4, ncclFloat, r, comm_, s));
        if (rbytes[r]) NCCL_CHECK(ncclRecv(recv[r], rbytes[r] / 4, ncclFloat, r, comm_, s));
      }
      NCCL_CHECK(ncclGroupEnd());
      return;
    }
    if (mode_ == SOLO) {  // the same bytes: this rank's own blocks stand in for the peers'
      CopyBatch b;
      for (int r = 0; r < nranks_; ++r)
        if (r != rank_ && rbytes[r]) copy_batch_add(b, recv[r], send[r], std::min(sbytes[r], rbytes[r]), s);
      copy_batch_flush(b, s);
      return;
    }
    // LOCAL: publish the send table, pull every peer's block addressed to this rank
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->ptr[rank_] = (void*)send.data();
    group_->barrier();
    for (int q = 0; q < nranks_; ++q) {
      if (q == rank_ || !rbytes[q]) continue;
      const void* const* peer = (const void* const*)group_->ptr[q];
      HIPC_CHECK(hipMemcpyAsync(recv[q], peer[rank_], rbytes[q], hipMemcpyDeviceToDevice, s));
    }
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->barrier();
  }

  void allreduce_sum_f64(double* p, size_t n, hipStream_t s) {
    settle(s);
    if (mode_ == RCCL) {
      NCCL_CHECK(ncclAllReduce(p, p, n, ncclDouble, ncclSum, comm_, s));
      return;
    }
    if (mode_ == SOLO) return;  // the rank's own partial stands for the sum
    if (n != 1) throw CommError("local allreduce supports one value");
    double v = 0.0;
    HIPC_CHECK(hipMemcpyAsync(&v, p, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->val[rank_] = v;
    group_->barrier();
    double sum = 0.0;
    for (int r = 0; r < nranks_; ++r) sum += group_->val[r];  // rank order: deterministic
    group_->barrier();
    HIPC_CHECK(hipMemcpyAsync(p, &sum, sizeof(double), hipMemcpyHostToDevice, s));
    HIPC_CHECK(hipStreamSynchronize(s));
  }

  // host-side reduction of n doubles over the ranks (op 0 sum, 1 max), through a device
  // buffer on stream s: the bench's barrier and max-over-ranks timing without torch
  void allreduce_host(double* v, size_t n, int op, hipStream_t s) {
    settle(s);
    if (mode_ == RCCL) {
      double* d = nullptr;
      HIPC_CHECK(hipMalloc(&d, sizeof(double) * n));
      HIPC_CHECK(hipMemcpyAsync(d, v, sizeof(double) * n, hipMemcpyHostToDevice, s));
      NCCL_CHECK(ncclAllReduce(d, d, n, ncclDouble, op ? ncclMax : ncclSum, comm_, s));
      HIPC_CHECK(hipMemcpyAsync(v, d, sizeof(double) * n, hipMemcpyDeviceToHost, s));
      HIPC_CHECK(hipStreamSynchronize(s));
      HIPC_CHECK(hipFree(d));
      return;
    }
    if (mode_ != LOCAL) return;  // one rank (or SOLO): nothing to reduce
    for (size_t q = 0; q < n; ++q) {
      group_->val[rank_] = v[q];
      group_->barrier();
      double r = group_->val[0];
      for (int k = 1; k < nranks_; ++k) r = op ? std::max(r, group_->val[k]) : r + group_->val[k];
      group_->barrier();
      v[q] = r;
    }
  }

  // Peer windows (MAD_OPT_PEER_HALO).  Every rank exposes one device allocation `base`; the
  // neighbours' windows mapped into this process come back as lo (rank - 1) / hi (rank + 1), null
  // where there is no neighbour.  RCCL: IPC handles all-gathered over the communicator and opened
  // here (*ipc = true: close them with close_window); LOCAL: the pointers themselves; SOLO and
  // RCCL-SOLO: the rank's own window stands in for both neighbours.  Collective.
  void share_window(void* base, hipStream_t s, void** lo, void** hi, bool* ipc) {
    *lo = *hi = nullptr;
    *ipc = false;
    if (mode_ == SOLO || (mode_ == RCCL && self_)) {
      *lo = *hi = base;
      return;
    }
    if (mode_ == LOCAL) {
      HIPC_CHECK(hipStreamSynchronize(s));
      group_->ptr[rank_] = base;
      group_->barrier();
      if (rank_ > 0) *lo = const_cast<void*>(group_->ptr[rank_ - 1]);
      if (rank_ < nranks_ - 1) *hi = const_cast<void*>(group_->ptr[rank_ + 1]);
      group_->barrier();
      return;
    }
    if (mode_ != RCCL) return;
    settle(s);
    // a handle this rank cannot export still takes part in the gather (zeros) and votes no below,
    // so no rank is left waiting in a collective the others skipped
    hipIpcMemHandle_t mine;
    std::memset(&mine, 0, sizeof mine);
    bool ok = hipIpcGetMemHandle(&mine, base) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    const size_t hb = sizeof(hipIpcMemHandle_t);
    std::vector<char> all(hb * nranks_);
    char* d = nullptr;
    HIPC_CHECK(hipMalloc(&d, hb * (nranks_ + 1)));
    HIPC_CHECK(hipMemcpyAsync(d + hb * nranks_, &mine, hb, hipMemcpyHostToDevice, s));
    NCCL_CHECK(ncclAllGather(d + hb * nranks_, d, hb, ncclChar, comm_, s));
    HIPC_CHECK(hipMemcpyAsync(all.data(), d, hb * nranks_, hipMemcpyDeviceToHost, s));
    HIPC_CHECK(hipStreamSynchronize(s));
    HIPC_CHECK(hipFree(d));
    // a neighbour's window this process cannot map (no peer access between the two GPUs) makes
    // every rank give the windows up together -- the caller falls back to the exchange -- instead
    // of one rank throwing while the others wait in their next collective
    auto open = [&](int r, void** p) {
      hipIpcMemHandle_t h;
      std::memcpy(&h, all.data() + hb * r, hb);
      if (hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        ok = false;
      }
    };
    if (ok && rank_ > 0) open(rank_ - 1, lo);
    if (ok && rank_ < nranks_ - 1) open(rank_ + 1, hi);
    *ipc = true;
    if (!all_true(ok, s)) {
      close_window(*lo, true);
      close_window(*hi, true);
      *lo = *hi = nullptr;
      *ipc = false;
    }
  }

  // logical AND of one flag over the ranks (collective)
  bool all_true(bool v, hipStream_t s) {
    settle(s);
    if (mode_ == RCCL && !self_) {
      int32_t* d = nullptr;
      int32_t h = v ? 1 : 0;
      HIPC_CHECK(hipMalloc(&d, sizeof(int32_t)));
      HIPC_CHECK(hipMemcpyAsync(d, &h, sizeof h, hipMemcpyHostToDevice, s));
      NCCL_CHECK(ncclAllReduce(d, d, 1, ncclInt32, ncclMin, comm_, s));
      HIPC_CHECK(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, s));
      HIPC_CHECK(hipStreamSynchronize(s));
      HIPC_CHECK(hipFree(d));
      return h != 0;
    }
    if (mode_ == LOCAL) {
      group_->val[rank_] = v ? 1.0 : 0.0;
      group_->barrier();
      bool all = true;
      for (int r = 0; r < nranks_; ++r) all = all && group_->val[r] != 0.0;
      group_->barrier();
      return all;
    }
    return v;
  }
  static void close_window(void* p, bool ipc) {
    if (p && ipc) (void)hipIpcCloseMemHandle(p);
  }

  // host barrier of the in-process transport (no-op for the others)
  void local_barrier(hipStream_t s) {
    if (mode_ != LOCAL) return;
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->barrier();
  }

  // every rank holds nz_global / nranks planes; gather all slabs in rank order
  void allgather_slabs(const void* slab, void* full, int64_t plane, int64_t nz_global, size_t esz,
                       hipStream_t s) {
    const size_t bytes = (size_t)plane * (size_t)(nz_global / nranks_) * esz;
    settle(s);
    if (mode_ == RCCL && self_) {  // the own slab into every rank's slot (as SOLO)
      std::vector<SelfPair> q;
      for (int r = 0; r < nranks_; ++r) q.push_back({(char*)full + r * bytes, slab, bytes});
      self_exchange(q, s);
      return;
    }
    if (mode_ == RCCL) {
      NCCL_CHECK(ncclAllGather(slab, full, bytes / 4, ncclFloat, comm_, s));
      return;
    }
    if (mode_ == SOLO) {  // the same bytes: the own slab into every rank's slot
      CopyBatch b;
      for (int r = 0; r < nranks_; ++r) copy_batch_add(b, (char*)full + r * bytes, slab, bytes, s);
      copy_batch_flush(b, s);
      return;
    }
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->ptr[rank_] = slab;
    group_->barrier();
    for (int r = 0; r < nranks_; ++r)
      HIPC_CHECK(hipMemcpyAsync((char*)full + r * bytes, group_->ptr[r], bytes,
                                hipMemcpyDeviceToDevice, s));
    HIPC_CHECK(hipStreamSynchronize(s));
    group_->barrier();
  }

 private:
  Mode mode_ = NONE;
  ncclComm_t comm_ = nullptr;
  std::shared_ptr<LocalGroup> group_;
  int nranks_ = 1;
  int rank_ = 0;
  bool self_ = false;
  bool graph_pending_ = false;        // a graph with RCCL operations may still be running
  hipStream_t graph_stream_ = nullptr;
};

}  // namespace mad
