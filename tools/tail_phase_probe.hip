// What one phase of an LDS-resident multi-workgroup V-cycle tail would cost: NWG
// workgroups of 1024 threads, each holding one 32 x 32 plane of a 32^3-class level (x, b and a stand-in
// for the 9-coefficient record) in LDS for the whole launch, plus the neighbours' planes as ghosts.
// Per phase: (c) a colour update of the plane from LDS (half the points, 7-point weights), (x) the
// plane published to global memory and the two neighbour planes read back after (b) a device-wide
// barrier -- agent-scope release increment / acquire spin, which on gfx950 writes back and invalidates
// the XCD's L2 so the neighbours' stores are seen across XCDs.  Variants drop (c) or (x) to split the
// cost.  Compared with the per-colour launch it would replace (gs_color_k on levels <= 32^3: 4.7-5.9 us
// per launch in the V-cycle traces, profiles/r06b_vcycle_breakdown.md).
//    hipcc --offload-arch=gfx950 -O3 -o tools/pbin/tail_phase_probe tools/tail_phase_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int P = 32 * 32;  // one plane

__global__ void __launch_bounds__(1024) tail_k(unsigned* bar, unsigned* err, float* pub, const float* init,
                                                int K, int nwg, int do_compute, int do_exchange) {
  __shared__ float x[3 * P];  // ghost below, own plane, ghost above
  __shared__ float bc[10 * P];  // b + 9 coefficients
  __shared__ int dead;
  const int me = blockIdx.x, t = threadIdx.x;
  if (t == 0) dead = 0;
  x[P + t] = init[me * P + t];
  x[t] = 0.f;
  x[2 * P + t] = 0.f;
  for (int f = 0; f < 10; ++f) bc[f * P + t] = 0.1f + 0.01f * (float)f + 1e-6f * (float)(t & 31);
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    if (do_compute) {  // one colour of the plane (checkerboard, phase parity)
      const int i = t & 31, j = t >> 5;
      if (((i + j + k) & 1) == 0) {
        const float* c = bc;
        const float xm = i > 0 ? x[P + t - 1] : x[P + t + 1];
        const float xp = i < 31 ? x[P + t + 1] : x[P + t - 1];
        const float ym = j > 0 ? x[P + t - 32] : x[P + t + 32];
        const float yp = j < 31 ? x[P + t + 32] : x[P + t - 32];
        const float s = c[1 * P + t] * xm + c[2 * P + t] * xp + c[3 * P + t] * ym + c[4 * P + t] * yp +
                        c[5 * P + t] * x[t] + c[6 * P + t] * x[2 * P + t];
        x[P + t] = (c[t] + s) * (1.0f / (1.0f + c[7 * P + t] + c[8 * P + t] + c[9 * P + t]));
      }
      __syncthreads();
    }
    if (do_exchange) pub[((size_t)(k & 1) * nwg + me) * P + t] = x[P + t];
    __syncthreads();
    if (t == 0) {
      const unsigned target = (unsigned)(k + 1) * (unsigned)nwg;
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = wall_clock64();
      while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > 200000000ull) {  // 2 s bound: a missing workgroup is an error
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = 1;
          break;
        }
      }
    }
    __syncthreads();
    if (dead) return;
    if (do_exchange) {
      const float* src = pub + (size_t)(k & 1) * nwg * P;
      x[t] = me > 0 ? src[(me - 1) * P + t] : 0.f;
      x[2 * P + t] = me < nwg - 1 ? src[(me + 1) * P + t] : 0.f;
      __syncthreads();
    }
  }
  pub[(size_t)2 * nwg * P + me * P + t] = x[P + t];
}

int main() {
  const int K = 400;
  unsigned *bar, *err;
  float *pub, *init;
  CK(hipMalloc(&bar, sizeof(unsigned)));
  CK(hipMalloc(&err, sizeof(unsigned)));
  CK(hipMalloc(&pub, sizeof(float) * 3 * 64 * P));
  CK(hipMalloc(&init, sizeof(float) * 64 * P));
  CK(hipMemset(init, 0, sizeof(float) * 64 * P));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int nwg : {8, 16, 32}) {
    for (int v = 0; v < 4; ++v) {
      const int comp = v & 1, exch = (v >> 1) & 1;
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemsetAsync(bar, 0, sizeof(unsigned), s));
        CK(hipMemsetAsync(err, 0, sizeof(unsigned), s));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(tail_k, dim3(nwg), dim3(1024), 0, s, bar, err, pub, init, K, nwg, comp, exch);
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned herr = 0;
        CK(hipMemcpy(&herr, err, sizeof herr, hipMemcpyDeviceToHost));
        if (herr) std::printf("barrier timed out (nwg %d)\n", nwg);
        if (ms < best) best = ms;
      }
      std::printf("{\"probe\": \"tail phase\", \"workgroups\": %d, \"compute\": %d, \"exchange\": %d, "
                  "\"us_per_phase\": %.3f}\n", nwg, comp, exch, best * 1e3f / K);
    }
  }
  return 0;
}
