// sector_probe.hip — what a sparse read of every 128-B row costs on MI355X (the per-flow
// Bijector API reads one flow's 8-12 B block of every parameter row: PlanarFlow.py:68-80,
// RadialFlow.py:50-70 called one flow at a time).  2^24 rows of 128 B (2 GiB, far beyond
// the caches); each lane owns one row and reads W bytes of it at a byte offset, then
// writes 4 B per row.  If HBM fills arrive in 64-B pieces, reading bytes [64, 76) costs
// about half of reading the whole row.
//   hipcc --offload-arch=gfx950 -O3 -o tools/sector_probe tools/sector_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kRowFloats = 32;

// NDW dwords starting at float OFF of the lane's row; NT: non-temporal loads.
template <int OFF, int NDW, bool NT>
__global__ void __launch_bounds__(256) probe(const float* __restrict__ t, float* __restrict__ out, int64_t rows) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* p = t + r * kRowFloats + OFF;
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NDW; ++i) s += NT ? __builtin_nontemporal_load(p + i) : p[i];
  out[r] = s;
}

// the whole row as 8 float4 per lane (the fused chain's bytes, no LDS)
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) probe_full(const f32x4* __restrict__ t, float* __restrict__ out, int64_t rows) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f32x4 v = __builtin_nontemporal_load(t + r * 8 + i);
    s += v.x + v.y + v.z + v.w;
  }
  out[r] = s;
}

template <typename F>
float time_it(F launch, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) launch();
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms / reps;
}

int main() {
  const int64_t rows = int64_t(1) << 24;
  float *t = nullptr, *out = nullptr;
  CHECK(hipMalloc(&t, rows * kRowFloats * sizeof(float)));
  CHECK(hipMalloc(&out, rows * sizeof(float)));
  CHECK(hipMemset(t, 0, rows * kRowFloats * sizeof(float)));
  const dim3 grid((unsigned)((rows + 255) / 256)), block(256);
  const int reps = 20;
  struct Case {
    const char* name;
    float ms;
  };
  std::vector<Case> cs;
#define RUN(NAME, KERNEL)                                                                  \
  cs.push_back({NAME, time_it([&] { hipLaunchKernelGGL(KERNEL, grid, block, 0, 0, t, out, rows); }, reps)}); \
  CHECK(hipGetLastError());
  for (int pass = 0; pass < 2; ++pass) {
    cs.clear();
    RUN("1 dword @ float 29 (bytes 116-119)", (probe<29, 1, true>));
    RUN("3 dwords @ float 29 (bytes 116-127: one 64-B half)", (probe<29, 3, true>));
    RUN("3 dwords @ float 14 (bytes 56-67: both halves)", (probe<14, 3, true>));
    RUN("3 dwords @ float 2 (bytes 8-19: first half)", (probe<2, 3, true>));
    RUN("3 dwords @ float 29, default policy", (probe<29, 3, false>));
    RUN("16 dwords @ float 16 (the second 64-B half)", (probe<16, 16, true>));
    cs.push_back({"whole 128-B row (8 x float4)",
                  time_it([&] { hipLaunchKernelGGL(probe_full, grid, block, 0, 0, (const f32x4*)t, out, rows); }, reps)});
    CHECK(hipGetLastError());
  }
  for (const Case& c : cs) {
    const double row_gb = rows * 128.0 / 1e9;
    printf("%-55s %8.4f ms   whole-row-equivalent %7.1f GB/s\n", c.name, c.ms, row_gb / (c.ms * 1e-3));
  }
  hipFree(t);
  hipFree(out);
  return 0;
}
