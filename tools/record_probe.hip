// Record-load probe (tools only, not the library): does the sweep's per-lane 40-byte record
// load (b128 + b128 + b64 at a 40-B lane stride, gs_fused3_k's buf_load_rec) stream HBM as
// fast as the same bytes read coalesced?  Each variant moves 48 B per point (40 B record +
// 4 B u read, 4 B written) over N points, several points in flight per lane:
//   copy4     float4 copy, 8 B per point (the HBM reference)
//   strided   per-lane record loads at a 40-B stride (the sweep's pattern)
//   coal      the same record bytes read as consecutive float4 per lane (coalesced)
//   lds       coalesced float4 loads into LDS, then per-lane 40-B records read from LDS
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/record_probe tools/record_probe.hip
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

constexpr int BLK = 256;
constexpr int PPT = 4;  // points in flight per lane

__global__ void __launch_bounds__(BLK) copy4(const float4* __restrict__ a, float4* __restrict__ o, long n4) {
  for (long i = blockIdx.x * (long)BLK + threadIdx.x; i < n4; i += (long)gridDim.x * BLK) o[i] = a[i];
}

// one chunk = BLK * PPT points; lane t handles points t, t + BLK, ... of its chunk.  Record loads
// as gs_fused3_k's buf_load_rec<float, 10>: raw buffer b128 + b128 + b64, SGPR base, lane offset
__global__ void __launch_bounds__(BLK) strided(const float* __restrict__ rec, const float* __restrict__ u,
                                               float* __restrict__ o, long n) {
  const long nch = n / (BLK * PPT);
  for (long ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rec + ch * BLK * PPT * 10), (short)0, -1, 0x00020000);
    float s[PPT];
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int voff = (q * BLK + threadIdx.x) * 40;
      auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
      auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 16, 0);
      auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 32, 0);
      const float* f0 = reinterpret_cast<const float*>(&v0);
      const float* f1 = reinterpret_cast<const float*>(&v1);
      const float* f2 = reinterpret_cast<const float*>(&v2);
      s[q] = u[ch * BLK * PPT + q * BLK + threadIdx.x] *
             (f0[0] + f0[1] + f0[2] + f0[3] + f1[0] + f1[1] + f1[2] + f1[3] + f2[0] + f2[1]);
    }
#pragma unroll
    for (int q = 0; q < PPT; ++q) o[ch * BLK * PPT + q * BLK + threadIdx.x] = s[q];
  }
}

// the same record bytes as consecutive float4 per lane: a chunk's BLK*PPT records are
// 10*BLK*PPT floats = 2.5*BLK*PPT float4
__global__ void __launch_bounds__(BLK) coal(const float4* __restrict__ rec4, const float* __restrict__ u,
                                            float* __restrict__ o, long n) {
  const long nch = n / (BLK * PPT);
  constexpr int F4 = 10 * BLK * PPT / 4;  // float4 per chunk
  constexpr int PER = F4 / BLK;           // 10 per lane
  for (long ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const float4 v = rec4[ch * F4 + q * BLK + threadIdx.x];
      acc += v.x + v.y + v.z + v.w;
    }
    float s[PPT];
#pragma unroll
    for (int q = 0; q < PPT; ++q) s[q] = u[ch * BLK * PPT + q * BLK + threadIdx.x] * acc;
#pragma unroll
    for (int q = 0; q < PPT; ++q) o[ch * BLK * PPT + q * BLK + threadIdx.x] = s[q];
  }
}

// coalesced float4 loads into LDS, per-point records read back from LDS
__global__ void __launch_bounds__(BLK) lds(const float4* __restrict__ rec4, const float* __restrict__ u,
                                           float* __restrict__ o, long n) {
  const long nch = n / (BLK * PPT);
  constexpr int F4 = 10 * BLK * PPT / 4;
  constexpr int PER = F4 / BLK;
  __shared__ float4 sm[F4];
  for (long ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    float4 v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) v[q] = rec4[ch * F4 + q * BLK + threadIdx.x];
    float uu[PPT];
#pragma unroll
    for (int q = 0; q < PPT; ++q) uu[q] = u[ch * BLK * PPT + q * BLK + threadIdx.x];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) sm[q * BLK + threadIdx.x] = v[q];
    __syncthreads();
    const float* f = reinterpret_cast<const float*>(sm);
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const float2* r2 = reinterpret_cast<const float2*>(f + 10 * (q * BLK + threadIdx.x));
      const float2 a0 = r2[0], a1 = r2[1], a2 = r2[2], a3 = r2[3], a4 = r2[4];
      o[ch * BLK * PPT + q * BLK + threadIdx.x] =
          uu[q] * (a0.x + a0.y + a1.x + a1.y + a2.x + a2.y + a3.x + a3.y + a4.x + a4.y);
    }
  }
}

int main() {
  const long n = 512L * 512 * 512;
  float *rec, *u, *o;
  CK(hipMalloc(&rec, sizeof(float) * 10 * n));
  CK(hipMalloc(&u, sizeof(float) * n));
  CK(hipMalloc(&o, sizeof(float) * n));
  CK(hipMemset(rec, 0, sizeof(float) * 10 * n));
  CK(hipMemset(u, 0, sizeof(float) * n));
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  auto run = [&](const char* name, double bytes, auto&& launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(a));
    const int R = 20;
    for (int r = 0; r < R; ++r) launch();
    CK(hipEventRecord(z));
    CK(hipEventSynchronize(z));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, z));
    ms /= R;
    std::printf("%-8s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  for (int grid : {1024, 2048, 4096, 8192}) {
    std::printf("grid %d\n", grid);
    run("copy4", 8.0 * n, [&] { hipLaunchKernelGGL(copy4, dim3(grid), dim3(BLK), 0, 0, (const float4*)u, (float4*)o, n / 4); });
    run("strided", 48.0 * n, [&] { hipLaunchKernelGGL(strided, dim3(grid), dim3(BLK), 0, 0, rec, u, o, n); });
    run("coal", 48.0 * n, [&] { hipLaunchKernelGGL(coal, dim3(grid), dim3(BLK), 0, 0, (const float4*)rec, u, o, n); });
    run("lds", 48.0 * n, [&] { hipLaunchKernelGGL(lds, dim3(grid), dim3(BLK), 0, 0, (const float4*)rec, u, o, n); });
  }
  CK(hipGetLastError());
  return 0;
}
