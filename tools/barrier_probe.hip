// Cost of a device-wide workgroup barrier on MI355X (gfx950) against a kernel launch: what a
// multi-workgroup persistent V-cycle tail would pay per phase.
//
// barrier_k: NWG workgroups of 256 threads (only those with blockIdx.x % 8 == 0 take part when
// one_xcd is set: the dispatcher deals workgroups to the 8 XCDs round robin), K phases; each phase
// every participating workgroup reads and writes `words` floats of a shared array (the small-level
// data a tail phase touches), then meets the others at an agent-scope barrier (release increment,
// acquire spin: the compiler's buffer_wbl2 sc1 / buffer_inv sc1), with a wall-clock bound so a
// workgroup that never arrives cannot hang the GPU.  empty_k: K launches of a one-workgroup kernel
// doing the same per-phase work, back to back in a captured graph.
//    hipcc --offload-arch=gfx950 -O3 -o tools/barrier_probe tools/barrier_probe.hip && ./tools/barrier_probe
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


__global__ void __launch_bounds__(256) barrier_k(unsigned* bar, unsigned* err, float* data, int words, int K,
                                                  int one_xcd, unsigned npart) {
  __shared__ int dead;
  if (one_xcd && (blockIdx.x & 7)) return;
  const unsigned me = one_xcd ? blockIdx.x >> 3 : blockIdx.x;
  if (threadIdx.x == 0) dead = 0;
  for (int k = 0; k < K; ++k) {
    for (int i = threadIdx.x; i < words; i += 256) {
      float* p = data + (size_t)me * words + i;
      *p = *p * 0.5f + (float)k;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned target = (unsigned)(k + 1) * npart;
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = wall_clock64();  // 100 MHz
      while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > 200000000ull) {  // 2 s: a missing workgroup is an error, not a hang
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = 1;
          break;
        }
      }
    }
    __syncthreads();
    if (dead) return;
  }
}

__global__ void __launch_bounds__(256) phase_k(float* data, int words, int k) {
  for (int i = threadIdx.x; i < words; i += 256) data[i] = data[i] * 0.5f + (float)k;
}

int main() {
  const int K = 200;
  unsigned *bar, *err;
  float* data;
  CK(hipMalloc(&bar, sizeof(unsigned)));
  CK(hipMalloc(&err, sizeof(unsigned)));
  CK(hipMalloc(&data, sizeof(float) * 4096 * 256));
  CK(hipMemset(data, 0, sizeof(float) * 4096 * 256));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int words : {0, 1024}) {
    for (int one_xcd : {1, 0}) {
      for (int nwg : {8, 32, 128, 256}) {
        const int launch = one_xcd ? nwg * 8 : nwg;
        if (launch > 2048) continue;
        const unsigned nparts = (unsigned)nwg;
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CK(hipMemsetAsync(bar, 0, sizeof(unsigned), s));
          CK(hipMemsetAsync(err, 0, sizeof(unsigned), s));
          CK(hipEventRecord(e0, s));
          hipLaunchKernelGGL(barrier_k, dim3(launch), dim3(256), 0, s, bar, err, data, words, K, one_xcd, nparts);
          CK(hipEventRecord(e1, s));
          CK(hipStreamSynchronize(s));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, e0, e1));
          unsigned herr = 0;
          CK(hipMemcpy(&herr, err, sizeof herr, hipMemcpyDeviceToHost));
          if (herr) std::printf("barrier timed out (nwg %d one_xcd %d)\n", nwg, one_xcd);
          if (ms < best) best = ms;
        }
        std::printf("{\"probe\": \"grid barrier\", \"workgroups\": %d, \"one_xcd\": %d, \"words_per_wg\": %d, "
                    "\"us_per_phase\": %.3f}\n", nwg, one_xcd, words, best * 1e3f / K);
      }
    }
    // K dependent one-workgroup launches, graph-captured
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(phase_k, dim3(1), dim3(256), 0, s, data, words, k);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    std::printf("{\"probe\": \"graph launches\", \"words\": %d, \"us_per_launch\": %.3f}\n", words, best * 1e3f / K);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
