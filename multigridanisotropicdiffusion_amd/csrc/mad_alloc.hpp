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

}  // namespace mad
