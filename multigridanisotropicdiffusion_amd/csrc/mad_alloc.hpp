// mad_alloc.hpp -- device allocation of the large streamed arrays.
//
// The level-0 sweep streams ~6.9 GB per launch at 512^3; how those arrays are mapped decides a
// measurable part of its speed.  Allocated with hipDeviceMallocContiguous (physically contiguous,
// so the GPU page tables can map them with the largest fragments and the UTCL2 misses far less
// often on a kernel that touches every page of its arrays each sweep) the SMOOTHER-layout 512^3
// sweep took 1.12-1.18 ms against 1.18-1.26 ms with the default allocation, the V-cycle 7.63-7.84
// against 7.93-8.04 ms and the FP32_REFINE cycle 10.26 against 10.49-10.83 ms, alternated on one
// box (profiles/r05_contiguous_ab.md).  Buffers below 64 MiB, and any request the driver cannot
// satisfy contiguously (fragmented device memory), take the default allocation.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstdlib>

namespace mad {

constexpr size_t BIG_ALLOC_MIN = (size_t)64 << 20;

// 0 on success (hipMalloc's error code otherwise); never leaves a sticky HIP error behind
inline hipError_t contiguous_alloc(void** p, size_t bytes) {
#ifndef MAD_NO_CONTIGUOUS
  if (bytes >= BIG_ALLOC_MIN) {
    if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    std::fprintf(stderr, "[mad] no physically contiguous block of %zu MiB: default allocation\n", bytes >> 20);
  }
#endif
  return hipMalloc(p, bytes);
}

// the other large buffers (tensor, fp64 refine arrays, VED volumes, direct-solver blocks); making
// only the level arrays contiguous measured the same (profiles/r05_contiguous_ab.md)
inline hipError_t big_alloc(void** p, size_t bytes) { return contiguous_alloc(p, bytes); }

// Placement of level 0's five arrays (x, b, r, t, records) relative to each other: carved from
// ONE contiguous allocation, each starting `align` after the previous array's end rounded up to
// `align`, plus its own offset `off[i]` (bytes).  Physical offsets inside a contiguous block equal
// the virtual ones, so the arrays' relative placement over the HBM channels is fixed instead of
// being whatever the driver's separate allocations happen to give.  Probe form: the environment
// variable MAD_LEVEL0_PLACE="align_kib:x,b,r,t,cf" (offsets in KiB; -1: that array is a separate
// allocation, not in the block) overrides the default.
struct Placement {
  bool on = false;
  size_t align = 0;
  size_t off[5] = {0, 0, 0, 0, 0};
  bool own[5] = {false, false, false, false, false};  // separate allocation
};

inline Placement level0_placement() {
  Placement p;
  const char* e = std::getenv("MAD_LEVEL0_PLACE");
  if (!e || !*e) return p;
  long a = 0, o[5] = {0, 0, 0, 0, 0};
  if (std::sscanf(e, "%ld:%ld,%ld,%ld,%ld,%ld", &a, &o[0], &o[1], &o[2], &o[3], &o[4]) != 6 || a <= 0) {
    std::fprintf(stderr, "[mad] MAD_LEVEL0_PLACE=\"%s\" is not align_kib:x,b,r,t,cf (KiB): ignored\n", e);
    return p;
  }
  p.on = true;
  p.align = (size_t)a << 10;
  for (int i = 0; i < 5; ++i) {
    p.own[i] = o[i] < 0;
    p.off[i] = o[i] < 0 ? 0 : (size_t)o[i] << 10;
  }
  return p;
}

// byte offsets of the arrays of sizes bytes[i] in the pool, and the pool's size
inline size_t place_offsets(const Placement& p, const size_t bytes[5], size_t at[5]) {
  size_t cur = 0;
  for (int i = 0; i < 5; ++i) {
    if (p.own[i]) continue;
    cur = (cur + p.align - 1) / p.align * p.align;
    at[i] = cur + p.off[i];
    cur = at[i] + bytes[i];
  }
  return cur;
}

}  // namespace mad
