// Does v_mfma_f32_16x16x4_f32 issued by one wave overlap plain fp32 VALU work of another
// wave on the same SIMD?  (The fused Dense backward's SQ counters showed
// SQ_VALU_MFMA_COEXEC_CYCLES = 0.)  8 waves per workgroup, waves w and w + 4 share a SIMD
// (cyclic wave placement); mode 0: every wave MFMA only, 1: every wave VALU only,
// 2: waves 0-3 MFMA and 4-7 VALU, 3: as 2 with the bf16 MFMA (16x16x32) instead,
// 4: waves 0-3 MFMA and 4-7 idle, 5: waves 0-3 idle and 4-7 VALU (the one-wave baselines),
// 6: as 5 with the VALU work as packed fp32 (v_pk_fma_f32 on float2: the same FMAs in half
// the instructions) — does packed math raise the fp32 VALU rate?
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_valu_coexec tools/mfma_valu_coexec.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ void __launch_bounds__(512) coexec(float* out, int n_mfma, int n_valu) {
  const int w = threadIdx.x >> 6;
  const bool mfma_wave = MODE == 0 ? true : (MODE == 1 ? false : w < 4);
  float r = 0.0f;
  if ((MODE == 4 && w >= 4) || ((MODE == 5 || MODE == 6) && w < 4)) {
    out[blockIdx.x * blockDim.x + threadIdx.x] = 0.0f;
    return;
  }
  if (mfma_wave) {
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const float a = threadIdx.x * 1e-3f, b = 1.0f - a;
    if constexpr (MODE == 3) {
      bf16x8 av, bv;
      for (int i = 0; i < 8; ++i) { av[i] = (__bf16)(a + i); bv[i] = (__bf16)(b - i); }
      for (int i = 0; i < n_mfma / 4; ++i) {  // 16x16x32 bf16 = 16 x the FLOP of 16x16x4 f32
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c3, 0, 0, 0);
      }
    } else {
      for (int i = 0; i < n_mfma / 4; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
      }
    }
    r = c0[0] + c1[1] + c2[2] + c3[3];
  } else if constexpr (MODE == 6) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 x0 = {(float)threadIdx.x, 1.0f}, x1 = x0 + 2.0f, x2 = x0 + 4.0f, x3 = x0 + 6.0f;
    const f2 m = {0.999f, 0.999f}, k = {1e-3f, 1e-3f};
    for (int i = 0; i < n_valu / 8; ++i) {
      x0 = __builtin_elementwise_fma(x0, m, k); x1 = __builtin_elementwise_fma(x1, m, k);
      x2 = __builtin_elementwise_fma(x2, m, k); x3 = __builtin_elementwise_fma(x3, m, k);
    }
    r = x0[0] + x0[1] + x1[0] + x1[1] + x2[0] + x2[1] + x3[0] + x3[1];
  } else {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const float m = 0.999f, k = 1e-3f;
    for (int i = 0; i < n_valu / 8; ++i) {
      x0 = fmaf(x0, m, k); x1 = fmaf(x1, m, k); x2 = fmaf(x2, m, k); x3 = fmaf(x3, m, k);
      x4 = fmaf(x4, m, k); x5 = fmaf(x5, m, k); x6 = fmaf(x6, m, k); x7 = fmaf(x7, m, k);
    }
    r = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
float run(float* out, int blocks, int n_mfma, int n_valu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(coexec<MODE>, dim3(blocks), dim3(512), 0, 0, out, n_mfma, n_valu);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(coexec<MODE>, dim3(blocks), dim3(512), 0, 0, out, n_mfma, n_valu);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus;  // one 8-wave workgroup per CU: 2 waves per SIMD
  float* out;
  hipMalloc(&out, (size_t)blocks * 512 * sizeof(float));
  const int nm = 8192, nv = 65536;
  // warm the clocks
  for (int i = 0; i < 20; ++i) run<2>(out, blocks, nm, nv);
  for (int rep = 0; rep < 2; ++rep) {
    const float t0 = run<0>(out, blocks, nm, nv), t1 = run<1>(out, blocks, nm, nv), t2 = run<2>(out, blocks, nm, nv),
                t3 = run<3>(out, blocks, nm, nv), t4 = run<4>(out, blocks, nm, nv), t5 = run<5>(out, blocks, nm, nv), t6 = run<6>(out, blocks, nm, nv);
    printf("{\"mfma_2w_ms\": %.4f, \"valu_2w_ms\": %.4f, \"mfma_1w_ms\": %.4f, \"valu_1w_ms\": %.4f, "
           "\"mixed_f32_mfma_ms\": %.4f, \"mixed_bf16_mfma_ms\": %.4f, \"mixed_over_sum_1w\": %.3f, "
           "\"mixed_over_max_1w\": %.3f, \"valu_packed_1w_ms\": %.4f}\n",
           t0, t1, t4, t5, t2, t3, t2 / (t4 + t5), t2 / fmaxf(t4, t5), t6);
  }
  hipFree(out);
  return 0;
}
