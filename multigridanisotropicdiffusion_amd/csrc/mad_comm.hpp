// mad_comm.hpp -- RCCL transport for the z-slab decomposition (one process per
// GPU, collectives over xGMI).  The reference is single-threaded and has no
// distributed path; this is the MI355X addition.
//
// Exchanges used by the solver:
//   exchange_planes   one ghost plane per z face with rank +-1 (grouped send/recv)
//   allreduce_sum_f64 ||r||^2 partial sums (8 bytes per V-cycle)
//   allgather_slabs   hand-over from the deepest distributed level to the first
//                     replicated coarse level (<= a few hundred KiB)
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace mad {

struct CommError : std::runtime_error {
  explicit CommError(const std::string& m) : std::runtime_error(m) {}
};

#define NCCL_CHECK(x)                                                                        \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw CommError(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

class Comm {
 public:
  static void unique_id(void* out128) {
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
  }

  void init(const void* uid128, int nranks, int rank, int device) {
    destroy();
    if (nranks <= 1) return;
    ncclUniqueId id;
    std::memcpy(&id, uid128, sizeof(id));
    (void)device;
    NCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
    nranks_ = nranks;
    rank_ = rank;
  }

  void destroy() {
    if (comm_) (void)ncclCommDestroy(comm_);
    comm_ = nullptr;
    nranks_ = 1;
    rank_ = 0;
  }

  bool active() const { return comm_ != nullptr && nranks_ > 1; }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }

  // a: base pointer of local plane 0; planes -depth..-1 and nz..nz+depth-1 are ghosts.
  // Sends the first / last `depth` owned planes to rank -+ 1 (one grouped call).
  void exchange_planes(void* a, int64_t plane, int nz, int depth, int has_lo, int has_hi,
                       size_t esz, bool is_double, hipStream_t s) {
    char* base = (char*)a;
    const ncclDataType_t dt = is_double ? ncclDouble : ncclFloat;
    const size_t pb = (size_t)plane * esz;
    const size_t cnt = (size_t)plane * depth;
    NCCL_CHECK(ncclGroupStart());
    if (has_lo) {
      NCCL_CHECK(ncclSend(base, cnt, dt, rank_ - 1, comm_, s));
      NCCL_CHECK(ncclRecv(base - depth * pb, cnt, dt, rank_ - 1, comm_, s));
    }
    if (has_hi) {
      NCCL_CHECK(ncclSend(base + (size_t)(nz - depth) * pb, cnt, dt, rank_ + 1, comm_, s));
      NCCL_CHECK(ncclRecv(base + (size_t)nz * pb, cnt, dt, rank_ + 1, comm_, s));
    }
    NCCL_CHECK(ncclGroupEnd());
  }

  void allreduce_sum_f64(double* p, size_t n, hipStream_t s) {
    NCCL_CHECK(ncclAllReduce(p, p, n, ncclDouble, ncclSum, comm_, s));
  }

  // every rank holds nz_global / nranks planes; gather all slabs in rank order
  void allgather_slabs(const void* slab, void* full, int64_t plane, int64_t nz_global, size_t esz,
                       hipStream_t s) {
    const size_t count = (size_t)plane * (size_t)(nz_global / nranks_) * (esz / 4);
    NCCL_CHECK(ncclAllGather(slab, full, count, ncclFloat, comm_, s));
  }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_ = 1;
  int rank_ = 0;
};

}  // namespace mad
