// Read-modify-write streaming probe (tools only): what the prolongation's byte mix -- fine x
// read and written in place, plus a small coarse read -- reaches with one float per lane (as
// interp3_k does) against two / four consecutive floats per lane and a float4 copy.
//    hipcc --offload-arch=gfx950 -O3 -o tools/rmw_probe tools/rmw_probe.hip && ./tools/rmw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

template <int V>
struct Vec;
template <>
struct Vec<1> { using t = float; };
template <>
struct Vec<2> { using t = float2; };
template <>
struct Vec<4> { using t = float4; };

// x[i] += 0.25 * c[i / 8] (coarse read: 1/8 of the fine elements, as the 3D prolongation's)
template <int V>
__global__ void __launch_bounds__(256) rmw_k(float* __restrict__ x, const float* __restrict__ c, long n) {
  using VT = typename Vec<V>::t;
  const long nv = n / V;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    VT v = reinterpret_cast<VT*>(x)[i];
    float* f = reinterpret_cast<float*>(&v);
#pragma unroll
    for (int q = 0; q < V; ++q) f[q] += 0.25f * c[(i * V + q) >> 3];
    reinterpret_cast<VT*>(x)[i] = v;
  }
}

__global__ void __launch_bounds__(256) copy4_k(const float4* __restrict__ a, float4* __restrict__ o, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) o[i] = a[i];
}

int main() {
  const long n = 512L * 512 * 512;
  float *x, *y, *c;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&c, n / 2));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(y, 0, n * 4));
  CK(hipMemset(c, 0, n / 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int grid : {1024, 2048, 4096, 8192}) {
    auto time = [&](auto launch, double bytes, const char* name) {
      for (int w = 0; w < 3; ++w) launch();
      CK(hipEventRecord(e0));
      const int reps = 20;
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      std::printf("{\"probe\": \"%s\", \"grid\": %d, \"us\": %.1f, \"TBs\": %.3f}\n", name, grid, ms * 1e3,
                  bytes / (ms * 1e-3) / 1e12);
    };
    const double rmw_bytes = n * 8.0 + n / 2.0;
    time([&] { hipLaunchKernelGGL(rmw_k<1>, dim3(grid), dim3(256), 0, 0, x, c, n); }, rmw_bytes, "rmw_f1");
    time([&] { hipLaunchKernelGGL(rmw_k<2>, dim3(grid), dim3(256), 0, 0, x, c, n); }, rmw_bytes, "rmw_f2");
    time([&] { hipLaunchKernelGGL(rmw_k<4>, dim3(grid), dim3(256), 0, 0, x, c, n); }, rmw_bytes, "rmw_f4");
    time([&] { hipLaunchKernelGGL(copy4_k, dim3(grid), dim3(256), 0, 0, (const float4*)y, (float4*)x, n / 4); },
         n * 8.0, "copy4");
  }
  CK(hipGetLastError());
  return 0;
}
