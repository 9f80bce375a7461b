// nfn_misc.hip — reductions (fp64 partial sums -> score) and the draw-split
// posterior merge.
#include "nfn_launch.h"

namespace nfn {
namespace {

// Finishes a partials-only launch: ws[0] = number n of (sum, non-finite count) pairs
// at ws[2 .. 2n+1]; out = {sum, count}, in the fixed order of sum_pairs (the same bits
// as the in-kernel finish).
__global__ void __launch_bounds__(256) reduce_partials_kernel(const double* __restrict__ ws, double* __restrict__ out) {
  __shared__ double red[2 * kSumWaves];
  sum_pairs(ws + 2, (int64_t)ws[0], red, out);
}

__global__ void __launch_bounds__(1024) reduce_f64_kernel(const double* __restrict__ in, int64_t n,
                                                          double* __restrict__ out) {
  __shared__ double red[1024 / 64];
  constexpr int U = 8;  // independent loads in flight per thread
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.0;
  const int64_t step = (int64_t)blockDim.x * U;
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * (int64_t)blockDim.x < n; i += step) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += in[i + u * (int64_t)blockDim.x];
  }
  for (; i < n; i += blockDim.x) acc[0] += in[i];
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) s += acc[u];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

}  // namespace

void launch_reduce_partials(const double* ws, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(256), 0, s, ws, out);
}

void launch_reduce_f64(const double* in, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_f64_kernel, dim3(1), dim3(1024), 0, s, in, n, out);
}

void launch_posterior_merge(bool fast, const float2* parts, int nsplit, int S, int64_t B, float* out, double* partials,
                            double* out_sum, uint32_t epoch, hipStream_t s) {
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  if (fast)
    hipLaunchKernelGGL(posterior_merge_kernel<true>, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, parts, nsplit, S, B,
                       out, partials, out_sum, epoch);
  else
    hipLaunchKernelGGL(posterior_merge_kernel<false>, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, parts, nsplit, S,
                       B, out, partials, out_sum, epoch);
}

}  // namespace nfn
