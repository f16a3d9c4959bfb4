// Per-phase cost of the solver's V-cycle tail kernel (mad::vtail_k, included from the solver's own header):
// the 512^3 bench hierarchy's tail -- 32^3 and 16^3 cell-centred levels, 8^3 coarsest (dense inverse),
// full tensor, fp32, nu = 2 -- on synthetic records, launched back to back, optionally after a kernel that
// dirties the L2s (as the V-cycle's big launches leave them).  Workgroup 0's wall-clock stamps give the
// time of the loads, of every phase and of the whole launch; events give the launch-to-launch time.
//    hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pbin/tail_probe tools/tail_probe.hip
//    tools/pbin/tail_probe [nwg ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../multigridanisotropicdiffusion_amd/csrc/mad_kernels.hpp"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

using namespace mad;

__global__ void dirty_k(float4* p, size_t n, float v) {  // writes n float4 (a big kernel's dirty L2 lines)
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(v, v, v, v);
}

int main(int argc, char** argv) {
  using T = float;
  constexpr int NCF = CoefLayout<3, KFULL>::N;
  std::vector<int> nwgs;
  bool ucx = false;  // "ucx": uncached hand-over buffers (with the relaxed-barrier kernel variant of the r06 log)
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "ucx") ucx = true;
    else nwgs.push_back(std::atoi(argv[i]));
  }
  if (nwgs.empty()) nwgs = {8, 16, 32};
  const int sizes[3] = {32, 16, 8};
  TailArgs<T> a{};
  a.nlev = 3;
  a.nu = 2;
  a.ncolors = 4;
  int wall_khz = 100000;
  (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  a.tmo = (uint64_t)wall_khz * 2000ull;
  for (int q = 0; q < 3; ++q) {
    const int n = sizes[q];
    TailLevel<T>& L = a.lv[q];
    L.g.nx = L.g.ny = L.g.nz = n;
    L.g.sy = n;
    L.g.sz = (int64_t)n * n;
    L.g.N = L.g.sz * n;
    L.g.hx0 = (n + 1) / 2;
    L.g.rs = NCF;
    L.rat.r[0] = L.rat.r[1] = L.rat.r[2] = 1.f;
    L.cent[0] = L.cent[1] = L.cent[2] = 1;
    std::vector<T> h((size_t)L.g.N * NCF);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01f + 0.05f * (float)((i * 2654435761u) % 1000) / 1000.f;
    T* cf;
    CK(hipMalloc(&cf, h.size() * sizeof(T)));
    CK(hipMemcpy(cf, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    L.cf = cf;
    CK(hipMalloc(&L.x, L.g.N * sizeof(T)));
    CK(hipMalloc(&L.b, L.g.N * sizeof(T)));
    CK(ucx ? hipExtMallocWithFlags((void**)&L.xch, 2 * L.g.N * sizeof(T), hipDeviceMallocUncached)
           : hipMalloc(&L.xch, 2 * L.g.N * sizeof(T)));
    CK(hipMemset(L.x, 0, L.g.N * sizeof(T)));
    std::vector<T> hb(L.g.N, 1.f);
    CK(hipMemcpy(L.b, hb.data(), hb.size() * sizeof(T), hipMemcpyHostToDevice));
  }
  const int nc = 512;
  std::vector<double> hinv((size_t)nc * nc, 1e-4);
  double* inv;
  CK(hipMalloc(&inv, hinv.size() * sizeof(double)));
  CK(hipMemcpy(inv, hinv.data(), hinv.size() * sizeof(double), hipMemcpyHostToDevice));
  a.inv = inv;
  CK(ucx ? hipExtMallocWithFlags((void**)&a.xy, 32 * 256 * sizeof(T), hipDeviceMallocUncached)
         : hipMalloc(&a.xy, 32 * 256 * sizeof(T)));
  CK(ucx ? hipExtMallocWithFlags((void**)&a.sync, 4 * sizeof(unsigned), hipDeviceMallocUncached)
         : hipMalloc(&a.sync, 4 * sizeof(unsigned)));
  CK(hipMemset(a.sync, 0, 4 * sizeof(unsigned)));
  uint64_t* stamps;
  CK(hipMalloc(&stamps, 256 * sizeof(uint64_t)));
  const size_t ndirty = (size_t)64 << 20;  // 1 GiB of float4
  float4* dirty;
  CK(hipMalloc(&dirty, ndirty * sizeof(float4) / 16));
  auto kern = vtail_k<T, KFULL>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int nwg : nwgs) {
    size_t off = 0;
    for (int q = 0; q < 2; ++q) {
      TailLevel<T>& L = a.lv[q];
      L.ppw = (L.g.nz + nwg - 1) / nwg;
      L.lds = (uint32_t)off;
      off += ((size_t)(L.ppw + 2) + 2 * L.ppw + NCF * L.ppw) * L.g.sz * sizeof(T);
      off = (off + 15) & ~(size_t)15;
    }
    if (off > 160 * 1024 - 256) {
      std::printf("{\"ucx\": %d, \"workgroups\": %d, \"skipped\": \"LDS %zu B\"}\n", nwg, off);
      continue;
    }
    for (int dirt = 0; dirt < 2; ++dirt) {
      const int reps = 40;
      for (int q = 0; q < 3; ++q) CK(hipMemset(a.lv[q].x, 0, a.lv[q].g.N * sizeof(T)));
      float tot = 0.f;
      std::vector<double> phase_us;
      double load_us = 0.0, launch_us = 0.0;
      for (int r = 0; r < reps; ++r) {
        if (dirt) hipLaunchKernelGGL(dirty_k, dim3(1024), dim3(256), 0, s, dirty, ndirty / 16, (float)r);
        a.stamps = (r == reps - 1) ? stamps : nullptr;
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), off, s, a);
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 5) tot += ms;
      }
      unsigned err[3];
      CK(hipMemcpy(err, a.sync, sizeof err, hipMemcpyDeviceToHost));
      uint64_t h[256];
      CK(hipMemcpy(h, stamps, sizeof h, hipMemcpyDeviceToHost));
      // stamps: start, loads done, every barrier (36), end: 39 entries
      const double tick_us = 1000.0 / wall_khz;
      int ns = 0;
      while (ns + 1 < 256 && h[ns + 1] > h[ns] && h[ns + 1] - h[ns] < 100000000ull) ++ns;
      load_us = (h[1] - h[0]) * tick_us;
      launch_us = (h[ns] - h[0]) * tick_us;
      std::printf("{\"ucx\": %d, \"workgroups\": %d, \"ppw32\": %d, \"lds\": %zu, \"dirty_l2_before\": %d, \"event_us\": %.2f, "
                  "\"stamped_us\": %.2f, \"load_us\": %.2f, \"phases\": %d, \"phase_us\": [",
                  (int)ucx, nwg, a.lv[0].ppw, off, dirt, tot * 1e3f / (reps - 5), launch_us, load_us, ns - 1);
      for (int i = 1; i < ns; ++i) std::printf("%s%.2f", i > 1 ? ", " : "", (h[i + 1] - h[i]) * tick_us);
      std::vector<T> hx(a.lv[0].g.N);  // the top level's x after the launches: equal across variants
      CK(hipMemcpy(hx.data(), a.lv[0].x, hx.size() * sizeof(T), hipMemcpyDeviceToHost));
      uint64_t hsum = 1469598103934665603ull;
      for (T v : hx) hsum = (hsum ^ __builtin_bit_cast(uint32_t, v)) * 1099511628211ull;
      std::printf("], \"err\": %u, \"x_hash\": \"%016llx\"}\n", err[2], (unsigned long long)hsum);
      std::fflush(stdout);
    }
  }
  return 0;
}
