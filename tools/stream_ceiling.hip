// stream_ceiling.hip — HBM stream ceilings on MI355X for the chain kernels' access
// pattern: persistent waves, each owning 8 KiB tiles (64 rows x 128 B) of one large
// buffer, the next tile prefetched into registers while the current one is "used".
// Axes (one line per combination):
//   extra : 0 = t rows only, 1 = + a 256 B y load per tile, 2 = + y + a 256 B log_prob
//           store per tile (nt), 3 = as 2 with a default-policy store
//   work  : a dependent chain of `work` v_fma per tile after the hand-off (emulates
//           the flow math; ~300 VALU per sample is the C2 chain)
//   wg/CU : resident 4-wave workgroups per CU
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_ceiling.hip -o tools/stream_ceiling
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

template <int EXTRA, int POL = 2>
__global__ void __launch_bounds__(256) stream_kernel(const float* __restrict__ t, const float* __restrict__ y,
                                                     float* __restrict__ out, int64_t ntiles, int work,
                                                     float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 buf[8];
  float yb = 0.f, acc = 0.f;
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const int nb = tile < ntiles ? 8192 : 0;
    if (EXTRA >= 1)
      yb = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(y + tc * 64, nb ? 256 : 0), lane * 4, 0, 0));
    const auto r = rsrc(t + tc * 2048, nb);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(w0);
  float pv = 0.f;
  auto pr = rsrc(out, 0);
  for (int64_t tile = w0; tile < ntiles; tile += ws) {
    f32x4 s = buf[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += buf[k];
    float v = s.x + s.y + s.z + s.w + yb;
    if (EXTRA >= 2) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pv), pr, lane * 4, 0, EXTRA == 2 ? POL : 0);
    issue(tile + ws);
    for (int i = 0; i < work; ++i) v = fmaf(v, 0.999f, 0.5f);
    acc += v;
    pv = v;
    pr = rsrc(out + tile * 64, 256);
  }
  if (EXTRA >= 2) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pv), pr, lane * 4, 0, 2);
  if (acc == 123.456f) sink[threadIdx.x] = acc;
}

// G consecutive tiles per wave step; the step's G x 256 B of log_prob leave as
// G/4 contiguous 1 KiB stores (float4 per lane) after the step's last tile.
template <int G>
__global__ void __launch_bounds__(256) stream_group_kernel(const float* __restrict__ t, const float* __restrict__ y,
                                                           float* __restrict__ out, int64_t ntiles,
                                                           float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  const int64_t nunits = ntiles / G;
  f32x4 buf[8];
  float yb = 0.f, acc = 0.f;
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const int nb = tile < ntiles ? 8192 : 0;
    yb = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(y + tc * 64, nb ? 256 : 0), lane * 4, 0, 0));
    const auto r = rsrc(t + tc * 2048, nb);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(w0 * G);
  f32x4 pv[G / 4];
  auto pr = rsrc(out, 0);
  for (int64_t u = w0; u < nunits; u += ws) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      f32x4 s = buf[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) s += buf[k];
      const float v = s.x + s.y + s.z + s.w + yb;
      issue(g + 1 < G ? u * G + g + 1 : (u + ws) * G);
      if (g == 0) {
#pragma unroll
        for (int i = 0; i < G / 4; ++i)
          __builtin_amdgcn_raw_buffer_store_b128(pv[i], pr, lane * 16, i * 1024, 2);
      }
      acc += v;
      pv[g / 4][g % 4] = v;
    }
    pr = rsrc(out + u * G * 64, G * 256);
  }
#pragma unroll
  for (int i = 0; i < G / 4; ++i) __builtin_amdgcn_raw_buffer_store_b128(pv[i], pr, lane * 16, i * 1024, 2);
  if (acc == 123.456f) sink[threadIdx.x] = acc;
}

// Backward-shaped stream: read a tile (8 KiB), write a tile (8 KiB) to a second
// buffer.  ORDER 0: the tile's stores right after its hand-off, BEFORE the next
// prefetch (the next hand-off waits for them); 1: after the next prefetch (never
// waited on).  AUX: store cache policy (2 = nt, 0 = default).
template <int ORDER, int AUX>
__global__ void __launch_bounds__(256) copy_kernel(const float* __restrict__ t, float* __restrict__ g, int64_t ntiles,
                                                   float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 buf[8], cur[8];
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const auto r = rsrc(t + tc * 2048, tile < ntiles ? 8192 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(w0);
  for (int64_t tile = w0; tile < ntiles; tile += ws) {
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = buf[k] * 1.5f;
    const auto rg = rsrc(g + tile * 2048, 8192);
    if (ORDER == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(cur[k], rg, lane * 16, k * 1024, AUX);
    }
    issue(tile + ws);
    if (ORDER == 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(cur[k], rg, lane * 16, k * 1024, AUX);
    }
    if (ORDER == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // generic kernel: stores drained per tile
  }
  if (cur[0].x == 123.456f) sink[threadIdx.x] = cur[0].y;
}

template <int ORDER, int AUX>
float run_copy(const float* t, float* g, int64_t ntiles, float* sink, int grid, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((copy_kernel<ORDER, AUX>), dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ts[ts.size() / 2];
}

template <int G>
float run_group(const float* t, const float* y, float* out, int64_t ntiles, float* sink, int grid, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(stream_group_kernel<G>, dim3(grid), dim3(256), 0, 0, t, y, out, ntiles, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ts[ts.size() / 2];
}

template <int POL>
float run_pol(const float* t, const float* y, float* out, int64_t ntiles, float* sink, int grid, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((stream_kernel<2, POL>), dim3(grid), dim3(256), 0, 0, t, y, out, ntiles, 0, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ts[ts.size() / 2];
}

template <int EXTRA>
float run(const float* t, const float* y, float* out, int64_t ntiles, int work, float* sink, int grid, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(stream_kernel<EXTRA>, dim3(grid), dim3(256), 0, 0, t, y, out, ntiles, work, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ts[ts.size() / 2];
}

int main() {
  const int64_t B = 1 << 24, P = 32;
  const int64_t tbytes = B * P * 4;
  const int64_t ntiles = B / 64;
  float *t, *y, *out, *sink;
  CHECK(hipMalloc(&t, tbytes));
  CHECK(hipMalloc(&y, B * 4));
  CHECK(hipMalloc(&out, B * 4));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(t, 0, tbytes));
  CHECK(hipMemset(y, 0, B * 4));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int i = 0; i < 1000; ++i)  // ~0.4 s: let the clocks ramp
    hipLaunchKernelGGL(stream_kernel<0>, dim3(cus * 2), dim3(256), 0, 0, t, y, out, ntiles, 0, sink);
  CHECK(hipDeviceSynchronize());
  const double bytes[4] = {(double)tbytes, (double)tbytes + 4.0 * B, (double)tbytes + 8.0 * B, (double)tbytes + 8.0 * B};
  for (int wpc : {1, 2}) {  // log_prob store cache policy (aux bits: 1 sc0, 2 nt, 16 sc1)
    const int grid = cus * wpc;
    const double b = (double)tbytes + 8.0 * B;
    const int pols[8] = {0, 1, 2, 3, 16, 17, 18, 19};
    float m[8];
    m[0] = run_pol<0>(t, y, out, ntiles, sink, grid, 20);
    m[1] = run_pol<1>(t, y, out, ntiles, sink, grid, 20);
    m[2] = run_pol<2>(t, y, out, ntiles, sink, grid, 20);
    m[3] = run_pol<3>(t, y, out, ntiles, sink, grid, 20);
    m[4] = run_pol<16>(t, y, out, ntiles, sink, grid, 20);
    m[5] = run_pol<17>(t, y, out, ntiles, sink, grid, 20);
    m[6] = run_pol<18>(t, y, out, ntiles, sink, grid, 20);
    m[7] = run_pol<19>(t, y, out, ntiles, sink, grid, 20);
    printf("t+y+out store policy wg/CU=%d |", wpc);
    for (int i = 0; i < 8; ++i) printf(" aux%d %.4f ms %.0f GB/s |", pols[i], m[i], b / m[i] / 1e6);
    printf("\n");
    fflush(stdout);
  }
  {
    float* g2;
    CHECK(hipMalloc(&g2, tbytes));
    for (int wpc : {1, 2, 3, 4, 6, 7}) {
      const int grid = cus * wpc;
      const double b = 2.0 * (double)tbytes;
      const float a0 = run_copy<0, 2>(t, g2, ntiles, sink, grid, 10);
      const float a1 = run_copy<1, 2>(t, g2, ntiles, sink, grid, 10);
      const float a2 = run_copy<0, 0>(t, g2, ntiles, sink, grid, 10);
      const float a3 = run_copy<1, 0>(t, g2, ntiles, sink, grid, 10);
      const float a4 = run_copy<0, 16>(t, g2, ntiles, sink, grid, 10);
      const float a5 = run_copy<0, 18>(t, g2, ntiles, sink, grid, 10);
      printf("copy (read 8 KiB + write 8 KiB per tile) wg/CU=%d | drained nt %.4f ms %.0f GB/s | pipelined nt %.4f ms "
             "%.0f GB/s | drained def %.4f ms %.0f GB/s | pipelined def %.4f ms %.0f GB/s | drained sc1 %.4f ms %.0f GB/s"
             " | drained sc1+nt %.4f ms %.0f GB/s\n",
             wpc, a0, b / a0 / 1e6, a1, b / a1 / 1e6, a2, b / a2 / 1e6, a3, b / a3 / 1e6, a4, b / a4 / 1e6, a5,
             b / a5 / 1e6);
      fflush(stdout);
    }
    CHECK(hipFree(g2));
  }
  for (int wpc : {1, 2, 4}) {
    const int grid = cus * wpc;
    const double b = (double)tbytes + 8.0 * B;
    const float g4 = run_group<4>(t, y, out, ntiles, sink, grid, 20);
    const float g16 = run_group<16>(t, y, out, ntiles, sink, grid, 20);
    const float g32 = run_group<32>(t, y, out, ntiles, sink, grid, 20);
    printf("grouped stores wg/CU=%d | 1KiB/4 tiles %.4f ms %.0f GB/s | 4KiB/16 tiles %.4f ms %.0f GB/s | "
           "8KiB/32 tiles %.4f ms %.0f GB/s\n", wpc, g4, b / g4 / 1e6, g16, b / g16 / 1e6, g32, b / g32 / 1e6);
    fflush(stdout);
  }
  for (int work : {0, 40}) {
    for (int wpc : {1, 2, 3, 4}) {
      const int grid = cus * wpc;
      float m[4];
      m[0] = run<0>(t, y, out, ntiles, work, sink, grid, 20);
      m[1] = run<1>(t, y, out, ntiles, work, sink, grid, 20);
      m[2] = run<2>(t, y, out, ntiles, work, sink, grid, 20);
      m[3] = run<3>(t, y, out, ntiles, work, sink, grid, 20);
      printf("work=%4d wg/CU=%d |", work, wpc);
      const char* nm[4] = {"t", "t+y", "t+y+out(nt)", "t+y+out(def)"};
      for (int e = 0; e < 4; ++e) printf(" %s %.4f ms %.0f GB/s |", nm[e], m[e], bytes[e] / m[e] / 1e6);
      printf("\n");
      fflush(stdout);
    }
  }
  return 0;
}
