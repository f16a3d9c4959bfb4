// Does freeing (or allocating) device memory slow the kernels that run right after it?  A streaming copy
// (1 GiB read + 1 GiB written per launch, ~0.35 ms) is timed launch by launch in windows of 100 ms:
// first undisturbed, then after hipMalloc + hipMemset + hipFree of B bytes, then after hipMalloc +
// hipMemset of B bytes kept.  A slowdown that follows the free / the allocation for a while is device
// work the runtime / driver does on those pages (clearing), not the kernel's own placement.
//    hipcc --offload-arch=gfx950 -O3 -o tools/pbin/free_probe tools/free_probe.hip
//    tools/pbin/free_probe [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void __launch_bounds__(256) copy_k(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

int main(int argc, char** argv) {
  const size_t gib = argc > 1 ? (size_t)std::atoi(argv[1]) : 4;
  const size_t n = ((size_t)1 << 30) / sizeof(float4);
  float4 *a, *b;
  CK(hipMalloc(&a, n * sizeof(float4)));
  CK(hipMalloc(&b, n * sizeof(float4)));
  CK(hipMemset(a, 0, n * sizeof(float4)));
  CK(hipMemset(b, 0, n * sizeof(float4)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<hipEvent_t> ev(2 * 400);
  for (auto& e : ev) CK(hipEventCreate(&e));
  auto windows = [&](const char* tag, int nwin) {
    for (int w = 0; w < nwin; ++w) {
      const int L = 280;  // ~100 ms of copies
      for (int i = 0; i < L; ++i) {
        CK(hipEventRecord(ev[2 * i], s));
        hipLaunchKernelGGL(copy_k, dim3(4096), dim3(256), 0, s, a, b, n);
        CK(hipEventRecord(ev[2 * i + 1], s));
      }
      CK(hipStreamSynchronize(s));
      double sum = 0.0, mx = 0.0, mn = 1e9;
      for (int i = 0; i < L; ++i) {
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
        sum += ms;
        mx = ms > mx ? ms : mx;
        mn = ms < mn ? ms : mn;
      }
      std::printf("{\"phase\": \"%s\", \"window\": %d, \"mean_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, "
                  "\"GBs\": %.0f}\n", tag, w, sum / L, mn, mx, 2.0 * n * sizeof(float4) / (sum / L * 1e-3) / 1e9);
      std::fflush(stdout);
    }
  };
  windows("baseline", 10);
  {
    void* p;
    CK(hipMalloc(&p, gib << 30));
    CK(hipMemset(p, 1, gib << 30));
    CK(hipDeviceSynchronize());
    windows("after_memset", 3);
    CK(hipFree(p));
  }
  windows("after_free", 20);
  {
    void* p;
    CK(hipMalloc(&p, gib << 30));
    windows("after_malloc", 10);
    CK(hipMemset(p, 1, gib << 30));
    CK(hipDeviceSynchronize());
    windows("after_malloc_memset", 10);
    CK(hipFree(p));
  }
  windows("after_free2", 20);
  return 0;
}
