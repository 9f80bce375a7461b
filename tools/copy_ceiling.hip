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

// Forward-shaped persistent stream (read an 8 KiB tile, write 256 B per tile) with
// the tile walk as a parameter: WALK 0 = grid stride (the kernels' walk), 1 = each
// wave owns one contiguous range of tiles.  OUT 0: no output stores.
template <int WALK, int OUT>
__global__ void __launch_bounds__(256) fwd_kernel(const float* __restrict__ t, float* __restrict__ out,
                                                  int64_t ntiles, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * 4 + wid, nw = (int64_t)gridDim.x * 4;
  const int64_t per = (ntiles + nw - 1) / nw;
  const int64_t first = WALK ? wv * per : wv;
  const int64_t last = WALK ? (wv + 1) * per < ntiles ? (wv + 1) * per : ntiles : ntiles;
  const int64_t step = WALK ? 1 : nw;
  f32x4 buf[8];
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < last ? tile : 0;
    const auto r = rsrc(t + tc * 2048, tile < last ? 8192 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(first);
  float acc = 0.f;
  for (int64_t tile = first; tile < last; tile += step) {
    f32x4 s = buf[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += buf[k];
    const float v = s.x + s.y + s.z + s.w;
    issue(tile + step);
    if (OUT) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rsrc(out + tile * 64, 256), lane * 4, 0, 2);
    acc += v;
  }
  if (acc == 123.456f) sink[threadIdx.x] = acc;
}

// Forward-shaped stream whose 256 B-per-tile output is written in one phase at the
// END of the kernel (the bound on separating the output stores from the read stream:
// the values are the last tile's, the bytes and addresses are every tile's).
__global__ void __launch_bounds__(256) fwd_endwrite_kernel(const float* __restrict__ t, float* __restrict__ out,
                                                           int64_t ntiles, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 buf[8];
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const auto r = rsrc(t + tc * 2048, tile < ntiles ? 8192 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(w0);
  float v = 0.f;
  for (int64_t tile = w0; tile < ntiles; tile += ws) {
    f32x4 s = buf[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += buf[k];
    v = s.x + s.y + s.z + s.w;
    issue(tile + ws);
  }
  for (int64_t tile = w0; tile < ntiles; tile += ws)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rsrc(out + tile * 64, 256), lane * 4, 0, 2);
  if (v == 123.456f) sink[threadIdx.x] = v;
}

// Forward-shaped stream in PHASES of T tiles per wave: the phase's outputs are held
// in the wave's LDS (T x 256 B), then every wave arrives at a grid-wide counter and
// waits (bounded: at most `spin` polls, so the barrier is only a hint and can never
// deadlock) before writing its phase's outputs in one burst.  BAR 0: no barrier
// (per-wave bursts only).
template <int T, int BAR>
__global__ void __launch_bounds__(256) fwd_phase_kernel(const float* __restrict__ t, float* __restrict__ out,
                                                        int64_t ntiles, unsigned* __restrict__ counter, int spin,
                                                        float* __restrict__ sink) {
  __shared__ float lo[4][T * 64];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  const unsigned nwaves = gridDim.x * 4;
  f32x4 buf[8];
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const auto r = rsrc(t + tc * 2048, tile < ntiles ? 8192 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(w0);
  float acc = 0.f;
  unsigned phase = 0;
  for (int64_t tb = w0; tb < ntiles; tb += (int64_t)T * ws) {
    int n = 0;
    for (int64_t tile = tb; n < T && tile < ntiles; tile += ws, ++n) {
      f32x4 s = buf[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) s += buf[k];
      const float v = s.x + s.y + s.z + s.w;
      issue(tile + ws);
      lo[wid][n * 64 + lane] = v;
      acc += v;
    }
    ++phase;
    if (BAR) {
      if (lane == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int i = 0; i < spin; ++i) {
        const unsigned c = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c >= phase * nwaves) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    for (int i = 0; i < n; ++i)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, lo[wid][i * 64 + lane]),
                                            rsrc(out + (tb + (int64_t)i * ws) * 64, 256), lane * 4, 0, 2);
  }
  if (acc == 123.456f) sink[threadIdx.x] = acc;
}

// persist_kernel with the contiguous-range walk (D = 1)
__global__ void __launch_bounds__(256) persist_range_kernel(const float* __restrict__ t, float* __restrict__ g,
                                                            int64_t ntiles, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * 4 + wid, nw = (int64_t)gridDim.x * 4;
  const int64_t per = (ntiles + nw - 1) / nw;
  const int64_t first = wv * per, last = (wv + 1) * per < ntiles ? (wv + 1) * per : ntiles;
  f32x4 buf[8], cur[8];
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < last ? tile : 0;
    const auto r = rsrc(t + tc * 2048, tile < last ? 8192 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(first);
  for (int64_t tile = first; tile < last; ++tile) {
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = buf[k] * 1.5f;
    issue(tile + 1);
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
  const double bf = (double)tbytes + 4.0 * B;
  for (int pass = 0; pass < 2; ++pass) {
    for (int wpc : {1, 2, 4}) {
      const int grid = cus * wpc;
      float m[4];
      m[0] = timeit([&] { hipLaunchKernelGGL((fwd_kernel<0, 1>), dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink); }, 20);
      m[1] = timeit([&] { hipLaunchKernelGGL((fwd_kernel<1, 1>), dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink); }, 20);
      m[2] = timeit([&] { hipLaunchKernelGGL((fwd_kernel<0, 0>), dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink); }, 20);
      m[3] = timeit([&] { hipLaunchKernelGGL((fwd_kernel<1, 0>), dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink); }, 20);
      printf("fwd-shape wg/CU=%d | stride+out %.4f ms %.0f GB/s | range+out %.4f ms %.0f GB/s | stride %.4f ms %.0f GB/s"
             " | range %.4f ms %.0f GB/s\n", wpc, m[0], bf / m[0] / 1e6, m[1], bf / m[1] / 1e6, m[2],
             (double)tbytes / m[2] / 1e6, m[3], (double)tbytes / m[3] / 1e6);
      fflush(stdout);
      char nm[64];
      snprintf(nm, sizeof nm, "fwd-shape end-write wg/CU=%d", wpc);
      {
        const float me = timeit([&] { hipLaunchKernelGGL(fwd_endwrite_kernel, dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink); }, 20);
        printf("%-32s %.4f ms %.0f GB/s\n", nm, me, bf / me / 1e6);
      }
      if (wpc == 2) {
        unsigned* ctr;
        CHECK(hipMalloc(&ctr, 4));
        auto ph = [&](auto kern, const char* label) {
          const float mp = timeit([&] {
            CHECK(hipMemsetAsync(ctr, 0, 4));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, t, g, ntiles, ctr, 4000, sink);
          }, 20);
          printf("%-32s %.4f ms %.0f GB/s\n", label, mp, bf / mp / 1e6);
          fflush(stdout);
        };
        ph(fwd_phase_kernel<32, 1>, "fwd phase T=32 barrier");
        ph(fwd_phase_kernel<32, 0>, "fwd phase T=32 no barrier");
        ph(fwd_phase_kernel<16, 1>, "fwd phase T=16 barrier");
        ph(fwd_phase_kernel<64, 1>, "fwd phase T=64 barrier");
        CHECK(hipFree(ctr));
      }
      snprintf(nm, sizeof nm, "persist range wg/CU=%d", wpc);
      rep(nm, timeit([&] { hipLaunchKernelGGL(persist_range_kernel, dim3(grid), dim3(256), 0, 0, t, g, ntiles, sink); }, 20));
    }
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
