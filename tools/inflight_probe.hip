// inflight_probe.hip — does the C2 stream want fewer bytes in flight than 8 waves per CU hold?
// The pure stream of the C2 tiles (8 KiB rows + 256 B y in, 256 B log_prob out per 64-sample
// tile, sc1 stores) runs faster at 4 waves per CU than at 8 (tools/stream_ceiling.hip), but the
// chain needs 8 to hide its latency.  Here every wave does `work` x 8 independent v_fma per tile
// (the chain's VALU time, no memory) between the hand-off and the next hand-off, and issues the
// next tile's rows either at once after the hand-off (SPLIT = 0, the shipped pipeline) or in two
// halves, the second after half of the work (SPLIT = 1: at most ~4 KiB in flight per wave once
// the first half has landed).  A compute-only line (every tile re-reads the wave's first tile)
// calibrates the work.  Median of 15 launches over 2^24 samples.
// Build: hipcc --offload-arch=gfx950 -O3 tools/inflight_probe.hip -o tools/inflight_probe
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

__device__ __forceinline__ void busy(float (&x)[8], int n) {
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = fmaf(x[j], 0.999f, 0.5f);
  }
}

// HO: the chain kernels' LDS hand-off instead of an in-register reduction: the tile's row pieces
// go to the wave's LDS slot (odd row stride 33), each lane then reads its own row's 30 floats.
template <int SPLIT, bool CONLY, bool HO = false>
__global__ void __launch_bounds__(256) probe_kernel(const float* __restrict__ t, const float* __restrict__ y,
                                                    float* __restrict__ out, int64_t ntiles, int work,
                                                    float* __restrict__ sink) {
  constexpr int S = 33;
  __shared__ float lds[4 * 64 * S];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* tl = lds + wid * 64 * S;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  f32x4 buf[8];
  float yb = 0.f;
  auto issue = [&](int64_t tile, int k0, int k1) {
    if (CONLY) tile = w0;
    const int64_t tc = tile < ntiles ? tile : 0;
    const int nb = tile < ntiles ? 8192 : 0;
    if (k0 == 0)
      yb = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(y + tc * 64, nb ? 256 : 0), lane * 4, 0, 0));
    const auto r = rsrc(t + tc * 2048, nb);
#pragma unroll
    for (int k = k0; k < k1; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  issue(w0, 0, 8);
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)(lane + j);
  for (int64_t tile = w0; tile < ntiles; tile += ws) {
    float v;
    if (HO) {
      const int r0 = lane / 8, c4 = lane % 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float* dst = tl + r0 * S + 4 * c4 + k * 8 * S;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      v = yb;
#pragma unroll
      for (int j = 0; j < 30; ++j) v += tl[lane * S + j];
    } else {
      f32x4 s = buf[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) s += buf[k];
      v = s.x + s.y + s.z + s.w + yb;
    }
    if (SPLIT) {
      issue(tile + ws, 0, 4);
      busy(x, work / 2);
      issue(tile + ws, 4, 8);
      busy(x, work - work / 2);
    } else {
      issue(tile + ws, 0, 8);
      busy(x, work);
    }
    float o = v;
#pragma unroll
    for (int j = 0; j < 8; ++j) o += x[j];
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, o), rsrc(out + tile * 64, 256), lane * 4, 0, 16);
    if (HO) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (x[0] == 123.456f) sink[threadIdx.x] = x[1];
}

// G consecutive tiles per wave unit (the unit's G x 256 B of log_prob contiguous): the values
// leave as one float4 store per lane per 4 tiles after the unit's last tile (lane l writes
// samples 4l..4l+3 of a 4-tile group, transposed through LDS), policy POL.
template <int G, int POL>
__global__ void __launch_bounds__(256) group_kernel(const float* __restrict__ t, const float* __restrict__ y,
                                                    float* __restrict__ out, int64_t ntiles, int work,
                                                    float* __restrict__ sink) {
  __shared__ float xl[4][G * 64];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  const int64_t nunits = ntiles / G;
  f32x4 buf[8];
  float yb = 0.f;
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const int nb = tile < ntiles ? 8192 : 0;
    yb = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(y + tc * 64, nb ? 256 : 0), lane * 4, 0, 0));
    const auto r = rsrc(t + tc * 2048, nb);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)(lane + j);
  issue(w0 * G);
  for (int64_t u = w0; u < nunits; u += ws) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      f32x4 s = buf[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) s += buf[k];
      const float v = s.x + s.y + s.z + s.w + yb;
      issue(g + 1 < G ? u * G + g + 1 : (u + ws) * G);
      busy(x, work);
      xl[wid][g * 64 + lane] = v + x[g & 7];
    }
    __builtin_amdgcn_wave_barrier();
    const auto pr = rsrc(out + u * G * 64, G * 256);
#pragma unroll
    for (int i = 0; i < G / 4; ++i) {
      const f32x4 o = *reinterpret_cast<const f32x4*>(&xl[wid][i * 256 + 4 * lane]);
      __builtin_amdgcn_raw_buffer_store_b128(o, pr, lane * 16, i * 1024, POL);
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (x[0] == 123.456f) sink[threadIdx.x] = x[1];
}

template <int G, int POL>
float run_group(const float* t, const float* y, float* out, int64_t ntiles, int work, float* sink, int grid) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 15; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((group_kernel<G, POL>), dim3(grid), dim3(256), 0, 0, t, y, out, ntiles, work, sink);
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

// Dynamic tail: steps k < Ks as the static walk, then the last D steps' tiles handed out C at a
// time by one agent-scope fetch-add on a counter (zeroed before the launch), each grab issued
// one chunk ahead of its use.
template <int C, int NCTR = 1>
__global__ void __launch_bounds__(256) dyn_kernel(const float* __restrict__ t, const float* __restrict__ y,
                                                  float* __restrict__ out, int64_t ntiles, int work, int dsteps,
                                                  unsigned long long* __restrict__ ctr, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wid, ws = (int64_t)gridDim.x * 4;
  const int64_t ks = max((int64_t)1, ntiles / ws - dsteps), pool0 = ks * ws;
  const int64_t nchunks = (ntiles - pool0 + C - 1) / C;
  const int q = (int)(w0 % NCTR);
  ctr += 16 * q;  // 128 B apart
  f32x4 buf[8];
  float yb = 0.f;
  auto issue = [&](int64_t tile) {
    const int64_t tc = tile < ntiles ? tile : 0;
    const int nb = tile < ntiles ? 8192 : 0;
    yb = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(y + tc * 64, nb ? 256 : 0), lane * 4, 0, 0));
    const auto r = rsrc(t + tc * 2048, nb);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, k * 1024, 2));
  };
  unsigned long long fut = 0;
  auto grab = [&]() {
    if (lane == 0) fut = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)(lane + j);
  int64_t knext = 1, cpos = 0, cleft = 0;
  bool more = true;
  if (ks == 1) grab();
  issue(w0);
  for (int64_t tile = w0, tnext; tile < ntiles; tile = tnext) {
    f32x4 s = buf[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += buf[k];
    const float v = s.x + s.y + s.z + s.w + yb;
    if (knext < ks) {
      tnext = knext * ws + w0;
      if (++knext == ks) grab();
    } else if (cleft > 0) {
      tnext = cpos++;
      --cleft;
    } else if (more) {
      const int64_t c = (int64_t)__builtin_amdgcn_readfirstlane((unsigned)fut) * NCTR + q;
      if (c < nchunks) {
        cpos = pool0 + c * C;
        cleft = min((int64_t)C, ntiles - cpos);
        tnext = cpos++;
        --cleft;
        grab();
      } else {
        more = false;
        tnext = ntiles;
      }
    } else {
      tnext = ntiles;
    }
    issue(tnext);
    busy(x, work);
    float o = v;
#pragma unroll
    for (int j = 0; j < 8; ++j) o += x[j];
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, o), rsrc(out + tile * 64, 256), lane * 4, 0, 16);
  }
  if (x[0] == 123.456f) sink[threadIdx.x] = x[1];
}

template <int C, int NCTR = 1>
float run_dyn(const float* t, const float* y, float* out, int64_t ntiles, int work, int dsteps,
              unsigned long long* ctr, float* sink, int grid) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 15; ++r) {
    CHECK(hipMemsetAsync(ctr, 0, 16 * 8 * NCTR, 0));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((dyn_kernel<C, NCTR>), dim3(grid), dim3(256), 0, 0, t, y, out, ntiles, work, dsteps, ctr, sink);
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

template <int SPLIT, bool CONLY, bool HO = false>
float run(const float* t, const float* y, float* out, int64_t ntiles, int work, float* sink, int grid) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 15; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((probe_kernel<SPLIT, CONLY, HO>), dim3(grid), dim3(256), 0, 0, t, y, out, ntiles, work, sink);
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
  const int64_t tbytes = B * P * 4, ntiles = B / 64;
  float *t, *y, *out, *sink;
  CHECK(hipMalloc(&t, tbytes));
  CHECK(hipMalloc(&y, B * 4));
  CHECK(hipMalloc(&out, B * 4));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(t, 0, tbytes));
  CHECK(hipMemset(y, 0, B * 4));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int i = 0; i < 1000; ++i)  // let the clocks ramp
    hipLaunchKernelGGL((probe_kernel<0, false>), dim3(cus * 2), dim3(256), 0, 0, t, y, out, ntiles, 0, sink);
  CHECK(hipDeviceSynchronize());
  const double bytes = (double)tbytes + 8.0 * B;
  printf("C2-shaped stream (%.3f GB per launch) with `work` x 8 independent fma per tile\n", bytes / 1e9);
  if (getenv("PROBE_DYN")) {  // dynamic tail, 8 waves per CU, at the C2 chain's VALU time
    const int grid = cus * 2;
    unsigned long long* ctr;
    CHECK(hipMalloc(&ctr, 16 * 8 * 8));
    const int work = 80;
    for (int rep = 0; rep < 2; ++rep) {
      printf("work=%d static %.4f | D=4: C=4 %.4f C=8 %.4f C=16 %.4f, C=4 x8 ctr %.4f, C=8 x8 ctr %.4f |", work,
             run_dyn<4>(t, y, out, ntiles, work, 0, ctr, sink, grid),
             run_dyn<4>(t, y, out, ntiles, work, 4, ctr, sink, grid), run_dyn<8>(t, y, out, ntiles, work, 4, ctr, sink, grid),
             run_dyn<16>(t, y, out, ntiles, work, 4, ctr, sink, grid),
             run_dyn<4, 8>(t, y, out, ntiles, work, 4, ctr, sink, grid), run_dyn<8, 8>(t, y, out, ntiles, work, 4, ctr, sink, grid));
      printf(" D=8: C=8 %.4f C=16 %.4f, C=4 x8 ctr %.4f, C=8 x8 ctr %.4f | D=16: C=8 x8 ctr %.4f C=16 x8 %.4f | D=2 C=4 %.4f ms\n",
             run_dyn<8>(t, y, out, ntiles, work, 8, ctr, sink, grid), run_dyn<16>(t, y, out, ntiles, work, 8, ctr, sink, grid),
             run_dyn<4, 8>(t, y, out, ntiles, work, 8, ctr, sink, grid), run_dyn<8, 8>(t, y, out, ntiles, work, 8, ctr, sink, grid),
             run_dyn<8, 8>(t, y, out, ntiles, work, 16, ctr, sink, grid), run_dyn<16, 8>(t, y, out, ntiles, work, 16, ctr, sink, grid),
             run_dyn<4>(t, y, out, ntiles, work, 2, ctr, sink, grid));
      fflush(stdout);
    }
    return 0;
  }
  if (getenv("PROBE_GROUP")) {  // grouped log_prob stores, 8 waves per CU
    const int grid = cus * 2;
    for (int work : {0, 80}) {
      const float a1 = run<0, false>(t, y, out, ntiles, work, sink, grid);
      printf("wg/CU=2 work=%3d | per tile (b32 sc1) %.4f |", work, a1);
      printf(" G=4 sc1 %.4f nt %.4f |", run_group<4, 16>(t, y, out, ntiles, work, sink, grid),
             run_group<4, 2>(t, y, out, ntiles, work, sink, grid));
      printf(" G=8 sc1 %.4f nt %.4f |", run_group<8, 16>(t, y, out, ntiles, work, sink, grid),
             run_group<8, 2>(t, y, out, ntiles, work, sink, grid));
      printf(" G=16 sc1 %.4f nt %.4f |", run_group<16, 16>(t, y, out, ntiles, work, sink, grid),
             run_group<16, 2>(t, y, out, ntiles, work, sink, grid));
      printf(" G=32 sc1 %.4f nt %.4f ms\n", run_group<32, 16>(t, y, out, ntiles, work, sink, grid),
             run_group<32, 2>(t, y, out, ntiles, work, sink, grid));
      fflush(stdout);
    }
    return 0;
  }
  if (getenv("PROBE_HO")) {  // the hand-off form beside the register form, 8 waves per CU
    const int grid = cus * 2;
    for (int work : {0, 48, 64, 80, 96, 128}) {
      const float c = run<0, true, true>(t, y, out, ntiles, work, sink, grid);
      const float a = run<0, false, false>(t, y, out, ntiles, work, sink, grid);
      const float b = run<1, false, false>(t, y, out, ntiles, work, sink, grid);
      const float ah = run<0, false, true>(t, y, out, ntiles, work, sink, grid);
      const float bh = run<1, false, true>(t, y, out, ntiles, work, sink, grid);
      printf("wg/CU=2 work=%3d | hand-off compute-only %.4f | registers: whole %.4f halves %.4f | LDS hand-off: whole %.4f halves %.4f ms\n",
             work, c, a, b, ah, bh);
      fflush(stdout);
    }
    return 0;
  }
  for (int wpc : {1, 2}) {
    const int grid = cus * wpc;
    for (int work : {0, 32, 64, 96, 128, 160, 192, 256, 320}) {
      const float c = run<0, true>(t, y, out, ntiles, work, sink, grid);
      const float a = run<0, false>(t, y, out, ntiles, work, sink, grid);
      const float b = run<1, false>(t, y, out, ntiles, work, sink, grid);
      printf("wg/CU=%d work=%3d | compute-only %.4f ms | issue whole %.4f ms %4.0f GB/s | issue in halves %.4f ms %4.0f GB/s\n",
             wpc, work, c, a, bytes / a / 1e6, b, bytes / b / 1e6);
      fflush(stdout);
    }
  }
  CHECK(hipFree(t));
  CHECK(hipFree(y));
  CHECK(hipFree(out));
  CHECK(hipFree(sink));
  return 0;
}
