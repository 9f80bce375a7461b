// nfn_tile.hip — one-tile-per-workgroup fallback kernels (unaligned / strided /
// broadcast parameter rows) and the single-bijector kernel of the Bijector API.
#include "nfn_launch.h"

namespace nfn {

// Single bijector over a batch (the per-flow Bijector API).  Parameters are read
// straight from global memory: this path serves the Python Bijector objects,
// not the fused chain.
template <int DM, bool FAST, int V = 1>
__global__ void __launch_bounds__(kMaxBlock)
    flow_fwd_ldj_kernel(int32_t flow_id, const float* __restrict__ z_in, int64_t z_bstride,
                        const float* __restrict__ tk, int64_t t_rowstride, int64_t B, int32_t d,
                        float* __restrict__ z_out, float* __restrict__ ldj_out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if constexpr (DM == 1 && FAST && V != 0) {
    // d = 1: the chain kernels' d = 1 bijectors on the block's 2-3 floats.  Each launch
    // reads every row's 128-B line of t once — a 12-B span costs a whole-line fetch
    // (tools/sector_probe.hip: 1-3 dwords of every row of 2^24 take as long as streaming
    // all 2.15 GB), so ten single-flow launches at C2 are bounded by ~3.6 ms of line fetches.
    // Default-policy loads: the block arrives as two requests (x2 + x1) to the same line,
    // and non-temporal ones let the second refetch it (5.9 vs 4.3 ms for the ten flows,
    // tools/microbench.py flows, profiles/r03/); z and the log-det are stored with the
    // default policy too: the next flow's launch reads this z back.
    const float* p = tk + b * t_rowstride;
    float pv[3];
    pv[0] = p[0];
    pv[1] = p[1];
    pv[2] = flow_id == NFN_FLOW_AFFINE ? 0.0f : p[2];
    float z1 = z_in[b * z_bstride];
    const float det = flow1_fast(flow_id, z1, pv);
    if (z_out) z_out[b] = z1;
    if (ldj_out) ldj_out[b] = __builtin_amdgcn_logf(fabsf(det)) * kLn2;
    return;
  }
  float z[DM];
  const float* zr = z_in + b * z_bstride;
#pragma unroll
  for (int j = 0; j < DM; ++j) z[j] = (j < d) ? zr[j] : 0.0f;
  const float ldj = flow_step<DM, FAST>(flow_id, z, tk + b * t_rowstride, d);
  if (z_out) {
#pragma unroll
    for (int j = 0; j < DM; ++j)
      if (j < d) z_out[b * d + j] = z[j];
  }
  if (ldj_out) ldj_out[b] = ldj;
}

namespace {

// Row staging for the per-flow tile kernel with eight loads in flight per lane before
// their LDS writes (stage_rows' loop waits for each load in turn: at ps = 17 and d = 8
// that is 25 dependent round trips per workgroup, and the kernel is latency-bound).
__device__ __forceinline__ void stage_rows_x8(float* lds, const float* __restrict__ src, int64_t rs, int nr,
                                              int P, int S) {
  const int nth = blockDim.x, tid = threadIdx.x;
  const int n = nr * P;
  const int step_r = nth / P, step_c = nth - (nth / P) * P;
  int r = tid / P, c = tid - (tid / P) * P;
  for (int i0 = tid; i0 < n; i0 += 8 * nth) {
    float v[8];
    int o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      o[u] = r * S + c;
      v[u] = (i0 + u * nth < n) ? src[(int64_t)r * rs + c] : 0.0f;
      r += step_r;
      c += step_c;
      if (c >= P) {
        c -= P;
        r += 1;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u * nth < n) lds[o[u]] = v[u];
  }
}

// The same single bijector for d > 1 with coalesced row traffic: a workgroup's 256 samples
// stage their parameter rows (ps floats at t_rowstride) and their z rows (d floats at
// z_bstride) into LDS at odd strides — whole-tile spans, coalesced — each lane evaluates
// its sample from LDS, and z_out leaves through the same LDS region as one contiguous
// (rows x d) run.  (One lane per row straight from global memory, the generic kernel
// above, makes every wave instruction touch 64 rows' lines.)
template <int DM, bool FAST, bool X8>
__global__ void __launch_bounds__(kMaxBlock)
    flow_fwd_ldj_tile_kernel(int32_t flow_id, const float* __restrict__ z_in, int64_t z_bstride,
                             const float* __restrict__ tk, int64_t t_rowstride, int64_t B, int32_t d, int32_t ps,
                             float* __restrict__ z_out, float* __restrict__ ldj_out) {
  extern __shared__ float lds[];
  const int rows = blockDim.x;
  const int tid = threadIdx.x;
  const int SP = ps | 1, SZ = d | 1;
  float* tp = lds;               // rows x SP parameters
  float* tz = lds + rows * SP;   // rows x SZ inputs, then outputs
  const int64_t b0 = (int64_t)blockIdx.x * rows;
  const int nr = (int)min((int64_t)rows, B - b0);
  const bool tb = t_rowstride == 0, zb = z_bstride == 0;
  if constexpr (X8) {
    stage_rows_x8(tp, tk + (tb ? 0 : b0 * t_rowstride), t_rowstride, tb ? 1 : nr, ps, SP);
    stage_rows_x8(tz, z_in + (zb ? 0 : b0 * z_bstride), z_bstride, zb ? 1 : nr, d, SZ);
  } else {
    stage_rows(tp, tk + (tb ? 0 : b0 * t_rowstride), t_rowstride, tb ? 1 : nr, ps, SP, false);
    stage_rows(tz, z_in + (zb ? 0 : b0 * z_bstride), z_bstride, zb ? 1 : nr, d, SZ, false);
  }
  __syncthreads();
  const bool act = tid < nr;
  float z[DM];
  float ldj = 0.0f;
  if (act) {
    const float* zr = tz + (zb ? 0 : tid * SZ);
#pragma unroll
    for (int j = 0; j < DM; ++j) z[j] = (j < d) ? zr[j] : 0.0f;
    ldj = flow_step<DM, FAST>(flow_id, z, tp + (tb ? 0 : tid * SP), d);
  }
  __syncthreads();  // every lane has read its z row (a broadcast row is shared) before any write
  if (act) {
    if (ldj_out) ldj_out[b0 + tid] = ldj;
#pragma unroll
    for (int j = 0; j < DM; ++j)
      if (j < d) tz[tid * SZ + j] = z[j];
  }
  __syncthreads();
  if (z_out) {
    for (int i = tid; i < nr * d; i += rows) {
      const int r = i / d, c = i - (i / d) * d;
      z_out[b0 * d + i] = tz[r * SZ + c];
    }
  }
}

// The Bijector API's Chain (tfp Chain of the flows that InverseNormalizingFlowLayer.
// _get_bijector builds, DistributionLayers.py:267-278): forward and
// forward_log_det_jacobian in ONE launch instead of one or two per flow.  A tile of
// parameter-row spans is staged in LDS (coalesced, odd stride), then every lane applies
// the flows in application order (the program's block offsets are relative to the
// span) and writes z_K and sum_k log|det J_k| (summed in application order, as TFP's
// Chain does).  `a.y` / `a.y_bstride` carry the input z.
template <int DM, bool FAST>
__global__ void __launch_bounds__(kMaxBlock) chain_fwd_ldj_kernel(ChainArgs a, float* __restrict__ z_out,
                                                                  float* __restrict__ ldj_out) {
  extern __shared__ float lds[];
  const int rows = a.tile_rows > 0 ? a.tile_rows : blockDim.x;
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * rows;
  const int nr = (int)min((int64_t)rows, a.B - b0);
  const bool tb = a.t_rowstride == 0;
  if (a.P > 0) {
    stage_rows(lds, a.t + (tb ? 0 : b0 * a.t_rowstride), a.t_rowstride, tb ? 1 : nr, a.P, a.lds_stride,
               a.vec4 != 0);
  }
  __syncthreads();
  if (tid >= nr) return;
  const int64_t b = b0 + tid;
  const int d = a.d;
  float z[DM];
  const float* zr = a.y + b * a.y_bstride;
#pragma unroll
  for (int j = 0; j < DM; ++j) z[j] = j < d ? zr[j] : 0.0f;
  const float* row = lds + (tb ? 0 : tid * a.lds_stride);
  float ldj = 0.0f;
  for (int k = 0; k < a.prog.K; ++k) {
    const int st = a.prog.step[k];  // wave-uniform (kernel argument)
    ldj = ldj + flow_step<DM, FAST>(st & 3, z, row + (st >> 2), d);
  }
  if (z_out) {
#pragma unroll
    for (int j = 0; j < DM; ++j)
      if (j < d) z_out[b * d + j] = z[j];
  }
  if (ldj_out) ldj_out[b] = ldj;
}

template <bool FAST>
void launch_c_dm(int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, float* z_out, float* ldj_out,
                 hipStream_t s) {
  switch (dm) {
    case 1: nfn_launch((chain_fwd_ldj_kernel<1, FAST>), grid, block, lds, s, a, z_out, ldj_out); break;
    case 2: nfn_launch((chain_fwd_ldj_kernel<2, FAST>), grid, block, lds, s, a, z_out, ldj_out); break;
    case 4: nfn_launch((chain_fwd_ldj_kernel<4, FAST>), grid, block, lds, s, a, z_out, ldj_out); break;
    case 8: nfn_launch((chain_fwd_ldj_kernel<8, FAST>), grid, block, lds, s, a, z_out, ldj_out); break;
    case 16: nfn_launch((chain_fwd_ldj_kernel<16, FAST>), grid, block, lds, s, a, z_out, ldj_out); break;
    default: nfn_launch((chain_fwd_ldj_kernel<32, FAST>), grid, block, lds, s, a, z_out, ldj_out); break;
  }
}

template <int DM, bool FAST>
void launch_t(const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s, bool posterior) {
  if (posterior)
    nfn_launch((posterior_lse_kernel<DM, FAST>), grid, block, lds, s, a);
  else
    nfn_launch((chain_logprob_kernel<DM, FAST>), grid, block, lds, s, a);
}

template <bool FAST>
void launch_t_dm(int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s, bool post) {
  switch (dm) {
    case 1: launch_t<1, FAST>(a, grid, block, lds, s, post); break;
    case 2: launch_t<2, FAST>(a, grid, block, lds, s, post); break;
    case 4: launch_t<4, FAST>(a, grid, block, lds, s, post); break;
    case 8: launch_t<8, FAST>(a, grid, block, lds, s, post); break;
    case 16: launch_t<16, FAST>(a, grid, block, lds, s, post); break;
    default: launch_t<32, FAST>(a, grid, block, lds, s, post); break;
  }
}

template <int DM, bool FAST>
void launch_f(int32_t flow_id, const float* z, int64_t zs, const float* tk, int64_t ts, int64_t B, int32_t d,
              float* z_out, float* ldj_out, hipStream_t s) {
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  if constexpr (DM > 1) {
    // d > 1: LDS-staged rows (NFN_FLOW_VARIANT=0, diag A/B: the per-lane global reads;
    // NFN_FLOW_STAGE=0: one load in flight per lane while staging)
    if (env_int("NFN_FLOW_VARIANT", 1) != 0) {
      const int ps = flow_id == NFN_FLOW_PLANAR ? 2 * d + 1 : (flow_id == NFN_FLOW_RADIAL ? d + 2 : 2 * d);
      const size_t lds = (size_t)kMaxBlock * ((ps | 1) + (d | 1)) * sizeof(float);
      auto kt = env_int("NFN_FLOW_STAGE", 1) != 0 ? flow_fwd_ldj_tile_kernel<DM, FAST, true>
                                                  : flow_fwd_ldj_tile_kernel<DM, FAST, false>;
      nfn_launch((kt), dim3((unsigned)nblk), dim3(kMaxBlock), lds, s, flow_id, z, zs, tk, ts, B, d, ps, z_out, ldj_out);
      return;
    }
  }
  // NFN_FLOW_VARIANT=0 (diag A/B): the generic bijector code for d = 1 too
  auto k = env_int("NFN_FLOW_VARIANT", 1) == 0 ? flow_fwd_ldj_kernel<DM, FAST, 0> : flow_fwd_ldj_kernel<DM, FAST, 1>;
  nfn_launch(k, dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, flow_id, z, zs, tk, ts, B, d, z_out, ldj_out);
}

template <bool FAST>
void launch_f_dm(int dm, int32_t flow_id, const float* z, int64_t zs, const float* tk, int64_t ts, int64_t B,
                 int32_t d, float* z_out, float* ldj_out, hipStream_t s) {
  switch (dm) {
    case 1: launch_f<1, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 2: launch_f<2, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 4: launch_f<4, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 8: launch_f<8, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 16: launch_f<16, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    default: launch_f<32, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
  }
}

}  // namespace

void launch_tile(bool fast, bool post, int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  if (fast)
    launch_t_dm<true>(dm, a, grid, block, lds, s, post);
  else
    launch_t_dm<false>(dm, a, grid, block, lds, s, post);
}

void launch_chain_fwd_ldj(bool fast, int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, float* z_out,
                          float* ldj_out, hipStream_t s) {
  if (fast)
    launch_c_dm<true>(dm, a, grid, block, lds, z_out, ldj_out, s);
  else
    launch_c_dm<false>(dm, a, grid, block, lds, z_out, ldj_out, s);
}

void launch_flow(bool fast, int dm, int32_t flow_id, const float* z, int64_t z_bstride, const float* tk,
                 int64_t t_rowstride, int64_t B, int32_t d, float* z_out, float* ldj_out, hipStream_t s) {
  if (fast)
    launch_f_dm<true>(dm, flow_id, z, z_bstride, tk, t_rowstride, B, d, z_out, ldj_out, s);
  else
    launch_f_dm<false>(dm, flow_id, z, z_bstride, tk, t_rowstride, B, d, z_out, ldj_out, s);
}

}  // namespace nfn
