// nfn_bf16.h — exact 3-way bf16 splits of fp32 operands for v_mfma_f32_16x16x32_bf16
// (the fused Dense kernels' GEMMs, nfn_dense.hip / nfn_dense_grad.hip).
// Every operand x is split EXACTLY into three bf16 parts, x = x1 + x2 + x3
// (v_cvt_pk_bf16_f32 round-to-nearest-even, residuals exact in fp32: x1 holds 8 significant
// bits, x2 the next 8, x3 the rest); a product keeps the six terms x_i y_j with i + j <= 4,
// the dropped ones (x2 y3, x3 y2, x3 y3) below 2^-23 |x y|: fp32-level products, accumulated
// in fp32 by the matrix cores.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nfn {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4v;

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const bf16x2v v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32: round to nearest even
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// (a, b) = (hi + mi + lo) exactly, each a packed bf16 pair (element 0 = a in the low half)
__device__ __forceinline__ void split3_pk(float a, float b, uint32_t& hi, uint32_t& mi, uint32_t& lo) {
  hi = pk_bf16(a, b);
  const float ra = a - bf16_lo(hi), rb = b - bf16_hi(hi);
  mi = pk_bf16(ra, rb);
  lo = pk_bf16(ra - bf16_lo(mi), rb - bf16_hi(mi));
}
__device__ __forceinline__ bf16x8v frag8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const u32x4v v = {a, b, c, d};
  return __builtin_bit_cast(bf16x8v, v);
}
__device__ __forceinline__ bf16x8v frag8(u32x4v v) { return __builtin_bit_cast(bf16x8v, v); }
__device__ __forceinline__ f32x4v mfma_bf16(bf16x8v a, bf16x8v b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace nfn
