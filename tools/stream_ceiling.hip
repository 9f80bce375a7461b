// stream_ceiling.hip — HBM read-stream ceilings on MI355X for the chain kernels'
// access pattern: persistent waves, each owning 8 KiB tiles (64 rows x 128 B) of
// one large buffer, the next tile prefetched while the current one is "used".
//   mode 0: global_load_dwordx4 into registers, default cache policy
//   mode 1: the same, non-temporal
//   mode 2: global_load_lds_dwordx4 (LDS-DMA) into a per-wave LDS slot, nt
//   mode 3: LDS-DMA, default policy
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_ceiling.hip -o tools/stream_ceiling
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <vector>
#include <algorithm>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int NV>
__global__ void __launch_bounds__(256) stream_kernel(const float* __restrict__ src, int64_t ntiles,
                                                     float* __restrict__ sink) {
  __shared__ f32x4 slot[4][2][512];  // per wave: two 8 KiB slots
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 acc = {0, 0, 0, 0};
  if constexpr (MODE <= 1) {
    f32x4 buf[NV];
    int64_t t = w0;
    auto issue = [&](int64_t tile) {
      const f32x4* p = reinterpret_cast<const f32x4*>(src + tile * 2048) + lane;
#pragma unroll
      for (int k = 0; k < NV; ++k) buf[k] = MODE == 1 ? __builtin_nontemporal_load(p + k * 64) : p[k * 64];
    };
    if (t < ntiles) issue(t);
    for (; t < ntiles; t += ws) {
      f32x4 cur[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) cur[k] = buf[k];
      if (t + ws < ntiles) issue(t + ws);
#pragma unroll
      for (int k = 0; k < NV; ++k) acc += cur[k];
    }
  } else {
    int64_t t = w0;
    int sl = 0;
    auto issue = [&](int64_t tile, int s) {
      const float* p = src + tile * 2048 + lane * 4;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        __builtin_amdgcn_global_load_lds(p + k * 256, (__attribute__((address_space(3))) void*)&slot[wid][s][k * 64],
                                         16, 0, MODE == 2 ? 2 : 0);
    };
    if (t < ntiles) issue(t, 0);
    for (; t < ntiles; t += ws) {
      if (t + ws < ntiles) {
        issue(t + ws, sl ^ 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_wave_barrier();
      acc += slot[wid][sl][lane * 8];
      sl ^= 1;
    }
  }
  if (acc.x == 123.456f) sink[threadIdx.x] = acc.y + acc.z + acc.w;
}

template <int MODE>
float run(const float* d, int64_t ntiles, float* sink, int grid, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((stream_kernel<MODE, 8>), dim3(grid), dim3(256), 0, 0, d, ntiles, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const int64_t B = 1 << 24, P = 32;
  const int64_t bytes = B * P * 4;
  const int64_t ntiles = B / 64;
  float *d, *sink;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(d, 0, bytes));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // warm the clocks: ~400 ms of streaming
  for (int i = 0; i < 1000; ++i)
    hipLaunchKernelGGL((stream_kernel<1, 8>), dim3(cus * 4), dim3(256), 0, 0, d, ntiles, sink);
  CHECK(hipDeviceSynchronize());
  for (int wpc : {1, 2, 3, 4}) {
    const int grid = cus * wpc;
    float m0 = run<0>(d, ntiles, sink, grid, 30);
    float m1 = run<1>(d, ntiles, sink, grid, 30);
    float m2 = run<2>(d, ntiles, sink, grid, 30);
    float m3 = run<3>(d, ntiles, sink, grid, 30);
    printf("wg/CU=%d  regs-default %.4f ms %.0f GB/s | regs-nt %.4f ms %.0f GB/s | lds-dma-nt %.4f ms %.0f GB/s | "
           "lds-dma-default %.4f ms %.0f GB/s\n",
           wpc, m0, bytes / m0 / 1e6, m1, bytes / m1 / 1e6, m2, bytes / m2 / 1e6, m3, bytes / m3 / 1e6);
  }
  return 0;
}
