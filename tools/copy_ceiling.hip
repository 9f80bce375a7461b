// copy_ceiling.hip — the backward's copy-shaped HBM ceiling under other launch
// structures than stream_ceiling.hip's persistent waves: read an 8 KiB tile
// (64 rows x 128 B) and write 8 KiB to a second buffer, 2^24 rows of 32 floats
// (the C2 backward's t -> grad_t stream, 4.29 GB moved).
//   oneshot<W> : one tile per wave, no prefetch, W waves per workgroup, grid =
//                ntiles / W (the hardware dispatcher refills CUs as waves retire)
//   multi<T>   : one workgroup of 4 waves walks T consecutive tiles per wave with
//                every load of the T tiles issued before the first store
//   flat       : one float4 per lane, grid over the whole buffer (the guide's
//                float4 copy)
//   persist<D> : stream_ceiling's persistent copy with prefetch depth D (1 or 2)
// Build: hipcc --offload-arch=gfx950 -O3 tools/copy_ceiling.hip -o tools/copy_ceiling
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

template <int W, int LP, int SP>
__global__ void __launch_bounds__(64 * W) oneshot_kernel(const float* __restrict__ t, float* __restrict__ g) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tile = (int64_t)blockIdx.x * W + wid;
  const auto r = rsrc(t + tile * 2048, 8192);
  f32x4 buf[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, LP));
  const auto rg = rsrc(g + tile * 2048, 8192);
#pragma unroll
  for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(buf[k] * 1.5f, rg, lane * 16, k * 1024, SP);
}

template <int T>
__global__ void __launch_bounds__(256) multi_kernel(const float* __restrict__ t, float* __restrict__ g) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tile0 = ((int64_t)blockIdx.x * 4 + wid) * T;
  const auto r = rsrc(t + tile0 * 2048, 8192 * T);
  f32x4 buf[8 * T];
#pragma unroll
  for (int k = 0; k < 8 * T; ++k)
    buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  const auto rg = rsrc(g + tile0 * 2048, 8192 * T);
#pragma unroll
  for (int k = 0; k < 8 * T; ++k) __builtin_amdgcn_raw_buffer_store_b128(buf[k] * 1.5f, rg, lane * 16, k * 1024, 2);
}

__global__ void __launch_bounds__(256) flat_kernel(const f32x4* __restrict__ t, f32x4* __restrict__ g) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  g[i] = t[i] * 1.5f;
}

template <int D>
__global__ void __launch_bounds__(256) persist_kernel(const float* __restrict__ t, float* __restrict__ g,
                                                      int64_t ntiles, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 buf[D][8], cur[8];
  auto issue = [&](int64_t tile, f32x4 (&b)[8]) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const auto r = rsrc(t + tc * 2048, tile < ntiles ? 8192 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      b[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
#pragma unroll
  for (int i = 0; i < D; ++i) issue(w0 + i * ws, buf[i]);
  for (int64_t tile = w0; tile < ntiles; tile += ws) {
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = buf[0][k] * 1.5f;
#pragma unroll
    for (int i = 0; i + 1 < D; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) buf[i][k] = buf[i + 1][k];
    issue(tile + D * ws, buf[D - 1]);
    const auto rg = rsrc(g + tile * 2048, 8192);
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b128(cur[k], rg, lane * 16, k * 1024, 2);
  }
  if (cur[0].x == 123.456f) sink[threadIdx.x] = cur[0].y;
}

template <typename F>
float timeit(F launch, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    launch();
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
  float *t, *g, *sink;
  CHECK(hipMalloc(&t, tbytes));
  CHECK(hipMalloc(&g, tbytes));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(t, 0, tbytes));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double b = 2.0 * (double)tbytes;
  for (int i = 0; i < 300; ++i)  // let the clocks ramp
    hipLaunchKernelGGL((oneshot_kernel<4, 2, 2>), dim3(ntiles / 4), dim3(256), 0, 0, t, g);
  CHECK(hipDeviceSynchronize());
  auto rep = [&](const char* name, float ms) {
    printf("%-32s %.4f ms %.0f GB/s\n", name, ms, b / ms / 1e6);
    fflush(stdout);
  };
  for (int pass = 0; pass < 2; ++pass) {
    rep("oneshot W=1 nt/nt", timeit([&] { hipLaunchKernelGGL((oneshot_kernel<1, 2, 2>), dim3(ntiles), dim3(64), 0, 0, t, g); }, 20));
    rep("oneshot W=4 nt/nt", timeit([&] { hipLaunchKernelGGL((oneshot_kernel<4, 2, 2>), dim3(ntiles / 4), dim3(256), 0, 0, t, g); }, 20));
    rep("oneshot W=4 def/def", timeit([&] { hipLaunchKernelGGL((oneshot_kernel<4, 0, 0>), dim3(ntiles / 4), dim3(256), 0, 0, t, g); }, 20));
    rep("oneshot W=4 nt/def", timeit([&] { hipLaunchKernelGGL((oneshot_kernel<4, 2, 0>), dim3(ntiles / 4), dim3(256), 0, 0, t, g); }, 20));
    rep("oneshot W=8 nt/nt", timeit([&] { hipLaunchKernelGGL((oneshot_kernel<8, 2, 2>), dim3(ntiles / 8), dim3(512), 0, 0, t, g); }, 20));
    rep("oneshot W=16 nt/nt", timeit([&] { hipLaunchKernelGGL((oneshot_kernel<16, 2, 2>), dim3(ntiles / 16), dim3(1024), 0, 0, t, g); }, 20));
    rep("multi T=2", timeit([&] { hipLaunchKernelGGL((multi_kernel<2>), dim3(ntiles / 8), dim3(256), 0, 0, t, g); }, 20));
    rep("multi T=4", timeit([&] { hipLaunchKernelGGL((multi_kernel<4>), dim3(ntiles / 16), dim3(256), 0, 0, t, g); }, 20));
    rep("flat float4", timeit([&] { hipLaunchKernelGGL(flat_kernel, dim3(tbytes / 16 / 256), dim3(256), 0, 0, (const f32x4*)t, (f32x4*)g); }, 20));
    for (int wpc : {2, 3, 4}) {
      char nm[64];
      snprintf(nm, sizeof nm, "persist D=1 wg/CU=%d", wpc);
      rep(nm, timeit([&] { hipLaunchKernelGGL((persist_kernel<1>), dim3(cus * wpc), dim3(256), 0, 0, t, g, ntiles, sink); }, 20));
      snprintf(nm, sizeof nm, "persist D=2 wg/CU=%d", wpc);
      rep(nm, timeit([&] { hipLaunchKernelGGL((persist_kernel<2>), dim3(cus * wpc), dim3(256), 0, 0, t, g, ntiles, sink); }, 20));
    }
  }
  return 0;
}
