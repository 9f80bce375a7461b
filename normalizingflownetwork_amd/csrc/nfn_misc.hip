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

// nfn_split_blocks_f32: one workgroup per R-row tile.  When the rows are dense (row stride
// rs at most W + 32 floats: the gap columns share the blocks' cache lines, so reading them
// costs no HBM bytes) the tile's whole span [row0 * rs, (row0 + R - 1) * rs + W) is read as
// 16-byte buffer loads, every lane active, from the 16-byte-aligned address at or below its
// first float (`mis` floats lower; the descriptor is bounded at the last valid float, so
// nothing past the tile is read; below it, the first tile reads the 0-3 floats between that
// aligned address and t — inside t's 16-byte granule, so inside any allocation whose base is
// 16-byte aligned, as every HIP and torch allocation is, but outside t itself: a host-side
// checker that tracks t's exact span would flag them); otherwise row by row (one row's W dwords per wave
// instruction).  The tile goes to LDS, then each block is written as its own contiguous
// (rows x w) run, lanes over consecutive floats (row = e / w by a float reciprocal: e <
// 2^18, so the quotient never rounds across an integer).  R * (span of a row) <= 16384
// floats: 64 KiB of LDS.
constexpr int kSplitTileFloats = 16384;

__host__ __device__ inline bool split_dense(int64_t rs, int W) { return rs <= (int64_t)W + 32; }

__host__ __device__ inline int split_rows(int64_t rs, int W) {
  const int64_t span = split_dense(rs, W) ? max(rs, (int64_t)W) : (int64_t)W;
  return (int)max((int64_t)4, min((int64_t)256, ((kSplitTileFloats - 8) / span) & ~(int64_t)3));
}

__global__ void __launch_bounds__(256) split_blocks_kernel(SplitArgs sa) {
  extern __shared__ float tile[];
  const int W = sa.W;
  const int64_t rs = sa.rs;
  const bool dense = split_dense(rs, W);
  const int R = split_rows(rs, W);
  const int64_t b0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, sa.B - b0);
  int mis = 0;       // floats between the aligned load base and the tile's first float
  int64_t lrs = W;   // row stride of the LDS tile
  if (dense) {
    mis = (int)((reinterpret_cast<uintptr_t>(sa.t) & 15) >> 2);
    lrs = max(rs, (int64_t)W);
    const float* base = sa.t + b0 * rs - mis;  // 16-byte aligned: R * rs * 4 is a multiple of 16
    const int n = mis + (int)((nr - 1) * lrs) + W;  // floats of the tile's span from base
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, n * 4, 0x00020000);
    float4* t4 = reinterpret_cast<float4*>(tile);
    for (int v = threadIdx.x; v < (n + 3) / 4; v += blockDim.x)
      t4[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, v * 16, 0, 2));
  } else {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int r = wid; r < nr; r += nw) {
      const float* row = sa.t + (b0 + r) * rs;
      for (int c = lane; c < W; c += 64) tile[r * W + c] = __builtin_nontemporal_load(row + c);
    }
  }
  __syncthreads();
  int off = mis;
  int64_t dofs = 0;
  for (int k = 0; k < sa.nblocks; ++k) {
    const int w = sa.widths[k];
    const float rw = 1.0f / (float)w;
    float* dst = sa.dst + dofs + b0 * w;
    const int n = nr * w;
    auto at = [&](int e) {
      const int r = (int)(((float)e + 0.5f) * rw);
      return tile[r * lrs + off + (e - r * w)];
    };
    int e0 = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {  // 16-byte stores for the run's whole float4s
      const int n4 = n >> 2;
      for (int q = threadIdx.x; q < n4; q += blockDim.x) {
        const int e = 4 * q;
        const f32x4 v = {at(e), at(e + 1), at(e + 2), at(e + 3)};
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst + e));
      }
      e0 = 4 * n4;
    }
    for (int e = e0 + threadIdx.x; e < n; e += blockDim.x) __builtin_nontemporal_store(at(e), dst + e);
    off += w;
    dofs += sa.B * w;
  }
}

}  // namespace

void launch_split_blocks(const SplitArgs& sa, hipStream_t s) {
  const int R = split_rows(sa.rs, sa.W);
  const int64_t span = split_dense(sa.rs, sa.W) ? std::max<int64_t>(sa.rs, sa.W) : sa.W;
  const size_t lds = (size_t)(R * span + 8) * sizeof(float);  // + the aligned span's up to 5 extra floats
  const int64_t nblk = (sa.B + R - 1) / R;
  nfn_launch(split_blocks_kernel, dim3((unsigned)nblk), dim3(256), lds, s, sa);
}

void launch_reduce_partials(const double* ws, double* out, hipStream_t s) {
  nfn_launch(reduce_partials_kernel, dim3(1), dim3(256), 0, s, ws, out);
}

void launch_reduce_f64(const double* in, int64_t n, double* out, hipStream_t s) {
  nfn_launch(reduce_f64_kernel, dim3(1), dim3(1024), 0, s, in, n, out);
}

void launch_posterior_merge(bool fast, const float2* parts, int nsplit, int S, int64_t B, float* out, double* partials,
                            double* out_sum, uint32_t epoch, hipStream_t s) {
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  if (fast)
    nfn_launch(posterior_merge_kernel<true>, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, parts, nsplit, S, B,
                       out, partials, out_sum, epoch);
  else
    nfn_launch(posterior_merge_kernel<false>, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, parts, nsplit, S,
                       B, out, partials, out_sum, epoch);
}

}  // namespace nfn

#ifdef NFN_DIAG
// Diagnostic build only (not in include/nfn.h): tanh_fast — the planar flows' tanh in every
// fast-math kernel — over n points, so tests/diag_modes.py can pin its ulp bound on the
// device against fp64.
namespace nfn {
namespace {
__global__ void __launch_bounds__(256) tanh_fast_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = tanh_fast(x[i]);
}
}  // namespace
}  // namespace nfn

extern "C" int32_t nfn_diag_tanh_fast(const float* x, float* y, int64_t n, void* stream) {
  const nfn::HookScope hook_scope;
  if (n <= 0) return NFN_OK;
  nfn::nfn_launch(nfn::tanh_fast_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                  reinterpret_cast<hipStream_t>(stream), x, y, n);
  return hipGetLastError() == hipSuccess ? NFN_OK : NFN_E_HIP;
}
#endif
