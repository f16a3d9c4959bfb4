// Overlap probe (tools only): while a sweep-shaped kernel holds every CU (one 1024-thread
// workgroup per CU, ~93 KB LDS, ~100 VGPRs, ~1 ms), can a small kernel on another stream
// run next to it?  The big kernel signals a counter early (like the rank-slab sweep's
// edge chunks); stream B waits on the counter (hipStreamWaitValue32) or on an event of a
// preceding short launch, then runs a halo-sized copy kernel (8 MB).  Prints when the
// copy finishes relative to the big kernel's start and end.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/overlap_probe tools/overlap_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

// device timestamps (constant wall clock) independent of event packets: ts[0] busy start
// (block 0), ts[1] max copy end
__device__ unsigned long long g_ts[2];

// busy kernel: each workgroup streams its own slice `iters` times; signals after iter 1
__global__ void __launch_bounds__(1024) busy(const float4* __restrict__ a, float* __restrict__ out,
                                             long per_wg4, int iters, unsigned* sig, int early) {
  extern __shared__ float4 lds[];
  if (blockIdx.x == 0 && threadIdx.x == 0) g_ts[0] = wall_clock64();
  if (early && sig && threadIdx.x == 0)
    __hip_atomic_fetch_add(sig, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  float acc = 0.f;
  float r[88];  // keep ~100 VGPRs live, like the sweep kernel
#pragma unroll
  for (int q = 0; q < 88; ++q) r[q] = (float)(threadIdx.x + q);
  const float4* base = a + (long)blockIdx.x * per_wg4;
  for (int it = 0; it < iters; ++it) {
    for (long i = threadIdx.x; i < per_wg4; i += 1024) {
      float4 v = base[i];
      lds[threadIdx.x] = v;
      acc += v.x + lds[(threadIdx.x + 1) & 1023].y;
#pragma unroll
      for (int q = 0; q < 88; ++q) r[q] = fmaf(r[q], v.y, v.z);
    }
    __syncthreads();
    if (it == 0 && sig && !early) {
      __threadfence();
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(sig, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#pragma unroll
  for (int q = 0; q < 88; ++q) acc += r[q];
  if (acc == 1234.5f) out[blockIdx.x] = acc;
}

__global__ void tiny(float* o) {
  if (threadIdx.x == 1000) o[0] = 1.f;
}

__global__ void __launch_bounds__(256) copyk(const float4* __restrict__ s, float4* __restrict__ d, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) d[i] = s[i];
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&g_ts[1], (unsigned long long)wall_clock64());
}

int main() {
  const long per_wg = 16L << 20;  // 16 MB per workgroup per iteration
  const int iters = 1;
  float4 *a, *s, *d;
  float* o;
  unsigned* sig;
  CK(hipMalloc(&a, per_wg * 256));
  CK(hipMalloc(&s, 8 << 20));
  CK(hipMalloc(&d, 8 << 20));
  CK(hipMalloc(&o, 4096));
  CK(hipMemset(a, 0, per_wg * 256));
  CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
  // mode 3: the counter in coherent host memory, polled by the host thread
  unsigned* hsig = nullptr;
  unsigned* hsig_d = nullptr;
  CK(hipHostMalloc((void**)&hsig, 8, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&hsig_d, hsig, 0));
  hsig[0] = 0;
  unsigned htarget = 0;
  unsigned zero = 0;
  CK(hipMemcpy(sig, &zero, 4, hipMemcpyHostToDevice));
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  std::printf("{\"can_use_stream_wait_value\": %d}\n", can);
  CK(hipFuncSetAttribute((const void*)busy, hipFuncAttributeMaxDynamicSharedMemorySize, 93 * 1024));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  unsigned target = 0;
  for (int mode = 0; mode < 7; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
      // mode 0: signal after the first quarter; 1: signal at kernel start; 2: event after a tiny
      // kernel that precedes the big one on stream A (the boundary-launch pattern); 3: signal
      // at kernel start into host memory, the host thread polls it and then launches the copy
      CK(hipEventRecord(e0, A));
      // 4: as 3 with 248 workgroups (one CU per XCD left free); 5: as 1 with 248 workgroups
      // 6: as 1 with a 1024-workgroup copy (is the delay the copy's own run under the big
      // kernel's HBM load rather than the wake-up?)
      if (mode == 5) {
        hipLaunchKernelGGL(busy, dim3(248), dim3(1024), 93 * 1024, A, a, o, per_wg / 16, iters + 3, sig, 1);
        target += 248u;
        CK(hipStreamWaitEvent(B, e0, 0));
        CK(hipStreamWaitValue32(B, sig, target, hipStreamWaitValueGte, 0xFFFFFFFFu));
      } else if (mode == 3 || mode == 4) {
        const unsigned nb = mode == 3 ? 256u : 248u;
        hipLaunchKernelGGL(busy, dim3(nb), dim3(1024), 93 * 1024, A, a, o, per_wg / 16, iters + 3, hsig_d,
                           1);
        htarget += nb;
        while (__atomic_load_n(hsig, __ATOMIC_ACQUIRE) < htarget) {
        }
      } else if (mode == 2) {
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, A, o);
        CK(hipEventRecord(e1, A));
        CK(hipStreamWaitEvent(B, e1, 0));
        hipLaunchKernelGGL(busy, dim3(256), dim3(1024), 93 * 1024, A, a, o, per_wg / 16, iters + 3,
                           (unsigned*)nullptr, 0);
      } else {
        hipLaunchKernelGGL(busy, dim3(256), dim3(1024), 93 * 1024, A, a, o, per_wg / 16, iters + 3, sig,
                           mode == 6 ? 1 : mode);
        target += 256u;
        CK(hipStreamWaitEvent(B, e0, 0));
        CK(hipStreamWaitValue32(B, sig, target, hipStreamWaitValueGte, 0xFFFFFFFFu));
      }
      hipLaunchKernelGGL(copyk, dim3(mode == 6 ? 1024 : 64), dim3(256), 0, B, s, d, (8 << 20) / 16);
      CK(hipEventRecord(e2, B));
      hipEvent_t e3;
      CK(hipEventCreate(&e3));
      CK(hipEventRecord(e3, A));
      CK(hipDeviceSynchronize());
      float big = 0, cp = 0;
      CK(hipEventElapsedTime(&big, e0, e3));
      CK(hipEventElapsedTime(&cp, e0, e2));
      CK(hipEventDestroy(e3));
      unsigned long long ts[2];
      CK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_ts), sizeof(ts)));
      int khz = 0;
      CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
      const double dev_ms = (double)((long long)(ts[1] - ts[0])) / (double)khz;
      std::printf("{\"mode\": %d, \"rep\": %d, \"big_kernel_ms\": %.3f, \"copy_done_ms_after_start\": %.3f, "
                  "\"copy_end_after_busy_start_ms_device_clock\": %.3f}\n",
                  mode, rep, big, cp, dev_ms);
    }
  // copy kernel alone
  CK(hipEventRecord(e0, B));
  hipLaunchKernelGGL(copyk, dim3(64), dim3(256), 0, B, s, d, (8 << 20) / 16);
  CK(hipEventRecord(e2, B));
  CK(hipDeviceSynchronize());
  float cp = 0;
  CK(hipEventElapsedTime(&cp, e0, e2));
  std::printf("{\"copy_alone_ms\": %.3f}\n", cp);
  return 0;
}
