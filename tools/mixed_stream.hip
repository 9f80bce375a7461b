// mixed_stream.hip — the C2 backward's mixed read / write stream as a stream (verdict r04,
// item 6): per 64-sample tile the backward reads y (256 B) + t (8 KiB) + the upstream
// gradient (256 B) and writes d/dt (8 KiB) + d/dy (256 B): 268 B per sample, 4.50 GB per
// 2^24-sample launch, as much written as read.  Persistent 4-wave workgroups; every wave
// walks units of K consecutive tiles and
//   PF = 0 : reads the unit's K tiles, then writes its K tiles (phase-grouped, no prefetch:
//            a wave alternates a K-tile read burst and a K-tile write burst);
//   PF = 1 : reads the NEXT unit's K tiles before writing the current unit's (the shipped
//            kernel's structure at K = 1: chain_grad_wave_kernel prefetches one tile ahead).
// The question: does grouping reads and writes into K-tile phases recover, at the 8-16
// resident waves per CU the chain needs, the rate a copy reaches at 4?  Tiles live in
// registers (32 VGPRs per tile and buffer), so K and PF bound the occupancy; the line
// prints the occupancy the runtime reports for each variant.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mixed_stream.hip -o tools/mixed_stream
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

template <int K, int PF, int SPOL = 2>
__global__ void __launch_bounds__(256) mixed_kernel(const float* __restrict__ t, const float* __restrict__ y,
                                                    const float* __restrict__ g, float* __restrict__ gt,
                                                    float* __restrict__ gy, int64_t nunits) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 buf[K][8];
  float yb[K], gb[K];
  auto issue = [&](int64_t u) {
    const bool ok = u < nunits;
    const int64_t tile0 = ok ? u * K : 0;
    const auto rt = rsrc(t + tile0 * 2048, ok ? 8192 * K : 0);
    const auto ry = rsrc(y + tile0 * 64, ok ? 256 * K : 0);
    const auto rg = rsrc(g + tile0 * 64, ok ? 256 * K : 0);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      yb[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, lane * 4, j * 256, 2));
      gb[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, lane * 4, j * 256, 2));
#pragma unroll
      for (int k = 0; k < 8; ++k)
        buf[j][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rt, lane * 16, j * 8192 + k * 1024, 2));
    }
  };
  auto store = [&](int64_t u, const f32x4 (&cur)[K][8], const float (&dy)[K]) {
    const int64_t tile0 = u * K;
    const auto rt = rsrc(gt + tile0 * 2048, 8192 * K);
    const auto ry = rsrc(gy + tile0 * 64, 256 * K);
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        __builtin_amdgcn_raw_buffer_store_b128(cur[j][k], rt, lane * 16, j * 8192 + k * 1024, SPOL);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, dy[j]), ry, lane * 4, j * 256, SPOL);
    }
  };
  if (PF) issue(w0);
  for (int64_t u = w0; u < nunits; u += ws) {
    if (!PF) issue(u);
    f32x4 cur[K][8];
    float dy[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      dy[j] = yb[j] * gb[j];
#pragma unroll
      for (int k = 0; k < 8; ++k) cur[j][k] = buf[j][k] * gb[j];
    }
    if (PF) issue(u + ws);
    store(u, cur, dy);
  }
}

template <int K, int PF, int SPOL = 2>
void measure(const float* t, const float* y, const float* g, float* gt, float* gy, int64_t ntiles, int cus,
             double bytes) {
  const int64_t nunits = ntiles / K;
  int occ = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(mixed_kernel<K, PF, SPOL>), 256, 0));
  printf("K=%d PF=%d stores aux %2d (max %d wg/CU = %2d waves/CU) |", K, PF, SPOL, occ, 4 * occ);
  for (int wpc = 1; wpc <= 4; ++wpc) {
    if (wpc > occ) {
      printf(" wg/CU=%d       -            |", wpc);
      continue;
    }
    const int grid = cus * wpc;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < 15; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((mixed_kernel<K, PF, SPOL>), dim3(grid), dim3(256), 0, 0, t, y, g, gt, gy, nunits);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float m = ts[ts.size() / 2];
    printf(" wg/CU=%d %.4f ms %4.0f GB/s |", wpc, m, bytes / m / 1e6);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
  }
  printf("\n");
  fflush(stdout);
}

int main() {
  const int64_t B = 1 << 24, P = 32;
  const int64_t ntiles = B / 64;
  const int64_t tb = B * P * 4;
  float *t, *y, *g, *gt, *gy;
  CHECK(hipMalloc(&t, tb));
  CHECK(hipMalloc(&gt, tb));
  CHECK(hipMalloc(&y, B * 4));
  CHECK(hipMalloc(&g, B * 4));
  CHECK(hipMalloc(&gy, B * 4));
  CHECK(hipMemset(t, 0, tb));
  CHECK(hipMemset(y, 0, B * 4));
  CHECK(hipMemset(g, 0, B * 4));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double bytes = 268.0 * B;  // the backward's algorithmic bytes at C2
  for (int i = 0; i < 300; ++i)     // let the clocks ramp
    hipLaunchKernelGGL((mixed_kernel<1, 1>), dim3(cus * 2), dim3(256), 0, 0, t, y, g, gt, gy, ntiles);
  CHECK(hipDeviceSynchronize());
  printf("C2 backward-shaped stream: %.3f GB per launch (268 B x 2^24), median of 15 launches\n", bytes / 1e9);
  measure<1, 1>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<1, 0>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<2, 0>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<2, 1>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<4, 0>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<4, 1>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<8, 0>(t, y, g, gt, gy, ntiles, cus, bytes);
  // the gradient stores write-through (sc1: the line leaves L2) instead of non-temporal
  measure<1, 1, 16>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<4, 0, 16>(t, y, g, gt, gy, ntiles, cus, bytes);
  measure<1, 1, 0>(t, y, g, gt, gy, ntiles, cus, bytes);
  CHECK(hipFree(t));
  CHECK(hipFree(gt));
  CHECK(hipFree(y));
  CHECK(hipFree(g));
  CHECK(hipFree(gy));
  return 0;
}
