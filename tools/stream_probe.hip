// Streaming-bandwidth probe for the smoother's byte mix (tools only, not the library).
// Measures what a plain coalesced kernel achieves when it moves the same bytes per
// voxel as one GS / Jacobi sweep at 512^3 fp32:
//   copy4   : float4 copy (read 4 + write 4 B/voxel)           -> HBM reference point
//   soa12   : 9 coefficient fields + b + u read, u' written (SoA, float4 per lane)
//   aos     : 36-byte coefficient record (3 x dwordx3) + b + u read, u' written
//   aos_rd  : the same reads, write skipped (read-only mix)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

__global__ void __launch_bounds__(256) copy4(const float4* __restrict__ a, float4* __restrict__ o,
                                             long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    o[i] = a[i];
}

__global__ void __launch_bounds__(256) soa12(const float4* __restrict__ cf, const float4* __restrict__ b,
                                             const float4* __restrict__ u, float4* __restrict__ o,
                                             long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 s = b[i];
    const float4 x = u[i];
#pragma unroll
    for (int f = 0; f < 9; ++f) {
      const float4 c = cf[f * n4 + i];
      s.x += c.x * x.x; s.y += c.y * x.y; s.z += c.z * x.z; s.w += c.w * x.w;
    }
    o[i] = s;
  }
}

template <bool WRITE>
__global__ void __launch_bounds__(256) aos(const float* __restrict__ rec, const float* __restrict__ b,
                                           const float* __restrict__ u, float* __restrict__ o,
                                           long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float3* r = reinterpret_cast<const float3*>(rec + 9 * i);
    const float3 c0 = r[0], c1 = r[1], c2 = r[2];
    const float x = u[i];
    float s = b[i] + x * (c0.x + c0.y + c0.z + c1.x + c1.y + c1.z + c2.x + c2.y + c2.z);
    if (WRITE) {
      o[i] = s;
    } else if (s == 12345.678f) {
      o[i] = s;
    }
  }
}

int main(int argc, char** argv) {
  const long N = 512L * 512 * 512;
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  float *cf, *b, *u, *o;
  CK(hipMalloc(&cf, sizeof(float) * 9 * N));
  CK(hipMalloc(&b, sizeof(float) * N));
  CK(hipMalloc(&u, sizeof(float) * N));
  CK(hipMalloc(&o, sizeof(float) * N));
  CK(hipMemset(cf, 0, sizeof(float) * 9 * N));
  CK(hipMemset(b, 0, sizeof(float) * N));
  CK(hipMemset(u, 0, sizeof(float) * N));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 16;
  auto time = [&](const char* name, double bytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f, \"bytes_per_voxel\": %.1f}\n", name, ms,
                bytes / (ms * 1e-3) / 1e9, bytes / N);
  };
  time("copy4", 8.0 * N, [&] {
    hipLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, 0, (const float4*)u, (float4*)o, N / 4);
  });
  time("soa12", 48.0 * N, [&] {
    hipLaunchKernelGGL(soa12, dim3(grid), dim3(256), 0, 0, (const float4*)cf, (const float4*)b,
                       (const float4*)u, (float4*)o, N / 4);
  });
  time("aos", 48.0 * N, [&] {
    hipLaunchKernelGGL(aos<true>, dim3(grid), dim3(256), 0, 0, cf, b, u, o, N);
  });
  time("aos_rd", 44.0 * N, [&] {
    hipLaunchKernelGGL(aos<false>, dim3(grid), dim3(256), 0, 0, cf, b, u, o, N);
  });
  return 0;
}
