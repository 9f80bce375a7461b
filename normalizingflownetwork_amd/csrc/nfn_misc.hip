// nfn_misc.hip — reductions (fp64 partial sums -> score) and the draw-split
// posterior merge.
#include "nfn_launch.h"

namespace nfn {
namespace {

// Sums the partials of a self-describing workspace: ws[0] = number n of
// (sum, non-finite count) pairs at ws[2 .. 2n+1].  out[0] = total sum; the total
// non-finite count goes to ws[1] (the workspace header) and, if given, out_nf[0].
// Fixed order: bitwise deterministic for a given n.
__global__ void __launch_bounds__(1024) reduce_partials_kernel(double* __restrict__ ws, double* __restrict__ out,
                                                              double* __restrict__ out_nf) {
  __shared__ double red[2 * 1024 / 64];
  const int64_t n = (int64_t)ws[0];
  const double* in = ws + 2;  // 8-byte alignment only is guaranteed
  constexpr int U = 4;
  double acc[U], cnt[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = cnt[u] = 0.0;
  const int64_t step = (int64_t)blockDim.x * U;
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * (int64_t)blockDim.x < n; i += step) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = 2 * (i + u * (int64_t)blockDim.x);
      acc[u] += in[k];
      cnt[u] += in[k + 1];
    }
  }
  for (; i < n; i += blockDim.x) {
    acc[0] += in[2 * i];
    cnt[0] += in[2 * i + 1];
  }
  double s = 0.0, c = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    s += acc[u];
    c += cnt[u];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    c += __shfl_xor(c, off);
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * wid] = s;
    red[2 * wid + 1] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tc = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      ts += red[2 * w];
      tc += red[2 * w + 1];
    }
    out[0] = ts;
    ws[1] = tc;
    if (out_nf) out_nf[0] = tc;
  }
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

void launch_reduce_partials(double* ws, double* out, double* out_nf, hipStream_t s) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(1024), 0, s, ws, out, out_nf);
}

void launch_reduce_f64(const double* in, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_f64_kernel, dim3(1), dim3(1024), 0, s, in, n, out);
}

void launch_posterior_merge(bool fast, const float2* parts, int nsplit, int S, int64_t B, float* out, double* partials,
                            hipStream_t s) {
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  if (fast)
    hipLaunchKernelGGL(posterior_merge_kernel<true>, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, parts, nsplit, S, B,
                       out, partials);
  else
    hipLaunchKernelGGL(posterior_merge_kernel<false>, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, parts, nsplit, S,
                       B, out, partials);
}

}  // namespace nfn
