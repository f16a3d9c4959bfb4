// Re-read probe (tools only): can the MI355X last-level cache (MALL) serve the record
// re-reads a two-sweep temporal-blocked GS kernel would make?  Each of 256 workgroups
// (one per CU) marches its own contiguous region in steps of STEP bytes; variants:
//   fresh  : read step k only                          (the one-sweep kernel's stream)
//   reread : read step k and step k - LAG again         (two sweeps, second LAG steps behind)
//   twice  : read step k and a DIFFERENT fresh step     (same bytes, no reuse: the control)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/reread_probe tools/reread_probe.hip
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

template <int MODE>
__global__ void __launch_bounds__(1024) march(const float4* __restrict__ a, const float4* __restrict__ b,
                                              float* __restrict__ out, long steps, long step4, int lag) {
  const float4* base = a + (long)blockIdx.x * steps * step4;
  const float4* base2 = b + (long)blockIdx.x * steps * step4;
  float acc = 0.f;
  for (long k = 0; k < steps; ++k) {
    for (long i = threadIdx.x; i < step4; i += 1024) {
      float4 v = base[k * step4 + i];
      acc += v.x + v.y + v.z + v.w;
      if (MODE == 1 && k >= lag) {
        float4 w = base[(k - lag) * step4 + i];
        acc += w.x + w.y + w.z + w.w;
      }
      if (MODE == 2) {
        float4 w = base2[k * step4 + i];
        acc += w.x + w.y + w.z + w.w;
      }
    }
    __syncthreads();
  }
  if (acc == 1234.5f) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
  const long step_bytes = argc > 1 ? std::atol(argv[1]) : 80 * 1024;  // per-WG bytes per step
  const int lag = argc > 2 ? std::atoi(argv[2]) : 4;
  const long total = 5L << 30;  // 5 GB region (the sweep's record array size at 512^3)
  const long steps = total / (256 * step_bytes);
  const long step4 = step_bytes / 16;
  float4 *a, *b;
  float* o;
  CK(hipMalloc(&a, total));
  CK(hipMalloc(&b, total));
  CK(hipMalloc(&o, 4096));
  CK(hipMemset(a, 0, total));
  CK(hipMemset(b, 0, total));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern, double bytes) {
    hipLaunchKernelGGL(kern, dim3(256), dim3(1024), 0, 0, a, b, o, steps, step4, lag);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r)
      hipLaunchKernelGGL(kern, dim3(256), dim3(1024), 0, 0, a, b, o, steps, step4, lag);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    std::printf("{\"probe\": \"%s\", \"step_KB\": %ld, \"lag\": %d, \"ms\": %.3f, \"GBs_loaded\": %.0f}\n",
                name, step_bytes / 1024, lag, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const double T = (double)steps * 256 * step_bytes;
  run("fresh", march<0>, T);
  run("reread", march<1>, 2 * T);
  run("twice", march<2>, 2 * T);
  return 0;
}
