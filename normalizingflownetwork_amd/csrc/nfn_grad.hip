// nfn_grad.hip — fused BACKWARD of the chain log-density:
// per sample, d log_prob / d t (the whole parameter row) and d log_prob / d y,
// scaled by an upstream gradient g_b.  This is what Keras autodiff computes when
// the reference trains (estimators/BaseEstimator.py:19-31, NLL loss :55-59;
// MaximumLikelihoodNNEstimator.py:33-35) through PlanarFlow.py:43-80,
// RadialFlow.py:44-84, AffineFlow.py:4-9 and DistributionLayers.py:245-294.
//
// One wave per workgroup owns R (<= 64) samples: the parameter rows are staged
// in LDS (odd row stride, coalesced), the chain runs forward once keeping every
// flow's input z_k in LDS, then runs in reverse with closed-form adjoints; each
// flow overwrites its own parameter block in LDS with its gradient (its
// parameters are dead afterwards), so the tile becomes the d/dt tile and is
// written back coalesced.  HBM traffic per sample: y + t in, t-gradient +
// y-gradient + log_prob out.
#include "nfn_grad_device.h"
#include "nfn_launch.h"

namespace nfn {
namespace {

// LDS tile rows -> global rows (the mirror of stage_rows).
__device__ __forceinline__ void store_rows(const float* lds, float* __restrict__ dst, int64_t rs, int nr, int P,
                                           int S, bool vec4) {
  const int nth = blockDim.x;
  const int tid = threadIdx.x;
  if (vec4) {
    const int q = P >> 2;
    const int n = nr * q;
    for (int i = tid; i < n; i += nth) {
      const int r = i / q, c = i - (i / q) * q;
      const float* src = lds + r * S + 4 * c;
      const f32x4 v = {src[0], src[1], src[2], src[3]};
      __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst + (int64_t)r * rs + 4 * c));
    }
  } else {
    const int n = nr * P;
    for (int i = tid; i < n; i += nth) {
      const int r = i / P, c = i - (i / P) * P;
      dst[(int64_t)r * rs + c] = lds[r * S + c];
    }
  }
}

template <int DM, bool FAST>
__device__ __forceinline__ void store_grad_y(const GradArgs& ga, int64_t b, const float (&adj)[DM]) {
  const ChainArgs& a = ga.c;
#pragma unroll
  for (int j = 0; j < DM; ++j)
    if (j < a.d) ga.grad_y[b * a.d + j] = a.y_std ? f_div<FAST>(adj[j], a.y_std[j]) : adj[j];
}

// General form: one wave-sized workgroup per tile of R <= 64 samples, any d, any
// row stride (incl. broadcast t).
template <int DM, bool FAST>
__global__ void __launch_bounds__(64) chain_grad_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  const int R = ga.rows;
  const int S = a.lds_stride;
  float* tile = lds;          // R rows x S
  float* zh = lds + R * S;    // flow inputs: zh[(k * d + j) * R + lane]
  const int lane = threadIdx.x;
  const int64_t b0 = diag_ablate_loads(a) ? 0 : (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, a.B - b0);
  const bool tb = a.t_rowstride == 0;
  if (a.P > 0) stage_rows(tile, a.t + (tb ? 0 : b0 * a.t_rowstride), a.t_rowstride, nr, a.P, S, a.vec4 != 0);
  __syncthreads();
  if (lane < nr) {
    const int64_t b = b0 + lane;
    float z[DM];
    const float corr = load_y<DM, FAST>(z, a, b);
    const float gl = ga.g_out ? ga.g_out[b] : 1.0f;
    float adj[DM];
    const float lp = grad_sample<DM, FAST>(z, tile + lane * S, zh + lane, R, a, gl, adj) - corr;
    if (a.out) a.out[b] = lp;
    if (ga.grad_y) store_grad_y<DM, FAST>(ga, b, adj);
  }
  __syncthreads();
  if (ga.grad_t && a.P > 0) store_rows(tile, ga.grad_t + b0 * ga.gt_rowstride, ga.gt_rowstride, nr, a.P, S,
                                       ga.gt_vec4 != 0);
}

// Streaming form for 16-byte-aligned rows with P/4 a power of two <= 16 (C1, C2):
// a persistent grid whose every WAVE owns a stream of 64-sample tiles with its own
// LDS slot (rows at an odd stride, then the K*d flow inputs) — no workgroup
// barriers.  The next tile's rows, y and upstream gradient are prefetched into
// registers (non-temporal) while the current tile runs forward + reverse; the
// gradient tile is then written back from LDS with coalesced non-temporal
// float4 stores (lane -> (row, 16-byte column) as for the loads).
// NTL / NTS (diag A/B only): non-temporal row loads / gradient stores (the release default).
template <int DM, bool FAST, int NV, int MINW, int CM = kChainLoop, bool NTL = true, bool NTS = true>
__global__ void __launch_bounds__(kMaxBlock, MINW) chain_grad_wave_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  const int S = a.lds_stride;
  const int Q = a.P >> 2;
  const int d = a.d;
  const int slot = 64 * S + a.prog.K * d * 64;
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float* tl = lds + wid * slot;
  float* zh = tl + 64 * S + lane;
  const int r0 = lane / Q;
  const int c4 = lane - r0 * Q;
  const int rstep = 64 / Q;
  const int64_t rs = a.t_rowstride;
  const int64_t gts = ga.gt_rowstride;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);

  float4 buf[NV];
  float ybuf[DM];
  float gbuf = 1.0f;
  bool issued_once = false;
  auto issue = [&](int64_t tile) {
    if (diag_ablate_loads(a) && issued_once) return;  // diagnostic: compute-only timing
    issued_once = true;
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
    const float* base = a.t + b0 * rs + 4 * c4;
#pragma unroll
    for (int k = 0; k < NV; ++k)
      if (r0 + k * rstep < nr) buf[k] = load_row4<NTL>(base + (int64_t)(r0 + k * rstep) * rs);
    if (lane < nr) {
      const float* yr = a.y + (b0 + lane) * a.y_bstride;
#pragma unroll
      for (int j = 0; j < DM; ++j) ybuf[j] = j < d ? yr[j] : 0.0f;
      if (ga.g_out) gbuf = __builtin_nontemporal_load(ga.g_out + b0 + lane);
    }
  };

  const int64_t ntiles = a.ntiles;
  // rotated tile slots as in chain_wave1_kernel: the plain grid stride (rot = 0) in the release
  // library (the rotation loses 0.8 % here, profiles/r05/r05zx_grad_bench_diag.txt); diag NFN_TILE_ROT_B
  const int64_t rot = diag_tile_rot_b(a) % ustep;
  if (u0 < ntiles) issue(u0);
  for (int64_t tile = u0, base = 0, slot = u0, tnext; tile < ntiles; tile = tnext) {
    slot += rot;
    if (slot >= ustep) slot -= ustep;
    base += ustep;
    tnext = base + slot;
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
    if (a.prio) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (r0 + k * rstep < nr) {
        float* dst = tl + (r0 + k * rstep) * S + 4 * c4;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
    }
    float z[DM];
    float corr = 0.0f;
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z[j] = ybuf[j];
      if (a.y_mean && j < d) {
        z[j] = f_div<FAST>(z[j] - a.y_mean[j], a.y_std[j]);
        corr += f_log<FAST>(a.y_std[j]);
      }
    }
    const float gl = gbuf;
    wave_lds_sync();
    if (tnext < ntiles) issue(tnext);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    if (lane < nr) {
      const int64_t b = b0 + lane;
      float adj[DM];
      const float lp = grad_sample<DM, FAST, CM>(z, tl + lane * S, zh, 64, a, gl, adj) - corr;
      if (a.out) __builtin_nontemporal_store(lp, a.out + b);
      if (ga.grad_y) store_grad_y<DM, FAST>(ga, b, adj);
    }
    wave_lds_sync();
    if (ga.grad_t) {
      float* gbase = ga.grad_t + b0 * gts + 4 * c4;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int r = r0 + k * rstep;
        if (r < nr) {
          const float* src = tl + r * S + 4 * c4;
          const f32x4 v = {src[0], src[1], src[2], src[3]};
          if constexpr (NTS)
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(gbase + (int64_t)r * gts));
          else
            *reinterpret_cast<f32x4*>(gbase + (int64_t)r * gts) = v;
        }
      }
    }
  }
}

#ifdef NFN_DIAG
// DIAGNOSTIC A/B (NFN_DIAG build, NFN_GRAD_WAVE1=1; measured and not adopted, DESIGN.md
// "C2 backward: the straight-line pipeline"): bitwise the release kernel's results.
// d = 1, fast math, P = 4Q (Q in {2, 4, 8, 16}): chain_grad_wave_kernel's walk with
// chain_wave1_kernel's memory pipeline (C1, C2 backward).  Every tile access is a
// buffer instruction through a wave-uniform descriptor bounded at B, so the loop body
// is straight-line code: each iteration issues the same loads (y, g, Q row pieces) and
// the same stores (log_prob, d/dy, Q gradient pieces; absent outputs go through empty
// descriptors), the next hand-off waits with vmcnt(#stores) for its prefetched rows and
// never for the previous tile's gradient stores.  (The generic wave kernel's per-slot
// branches made the waitcnt pass drain every store before the hand-off.)
// SPLIT = 2: the next tile's rows are issued in two halves, the second between the
// chain's forward and reverse passes (half the bytes in flight per wave).
template <int Q, int CM, int SPLIT = 1>
__global__ void __launch_bounds__(kMaxBlock) chain_grad_wave1_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  constexpr int RSTEP = 64 / Q;  // rows per wave instruction
  constexpr int kNT = 2;         // non-temporal: streamed once
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = a.lds_stride;
  const int K = a.prog.K;
  const int P = a.P;
  const int64_t rs = a.t_rowstride;
  const int64_t gts = ga.gt_rowstride;
  const int r0 = lane / Q, c4 = lane % Q;
  float* tl = lds + wid * (64 * S + K * 64);
  float* zh = tl + 64 * S + lane;
  const int l0 = r0 * S + 4 * c4;
  const int64_t ntiles = a.ntiles;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const bool has_g = ga.g_out != nullptr;
  const bool want_lp = a.out != nullptr;
  const uint32_t types = a.prog.types[0];
  const int64_t abl_tile = diag_ablate_loads(a) ? u0 : -1;  // diagnostic: compute-only timing
  // loop-invariant byte offsets (the host guarantees 64 rows of a tile span < 2 GiB)
  const int yoff = lane * (int)a.y_bstride * 4;
  const int toff = (r0 * (int)rs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)rs * 4;
  const int goff = (r0 * (int)gts + 4 * c4) * 4;
  const int gkstep = RSTEP * (int)gts * 4;

  constexpr int QA = SPLIT == 2 && Q >= 2 ? Q / 2 : Q;  // row pieces issued with y and g
  float4 buf[Q];
  float ybuf, gbuf;
  auto rows_rsrc = [&](int64_t tile) {
    if (abl_tile >= 0) tile = abl_tile;
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    return tile_rsrc(a.t + (nr > 0 ? b0 : 0) * rs, nr > 0 ? ((nr - 1) * rs + P) * 4 : 0);
  };
  auto issue = [&](int64_t tile) {
    if (abl_tile >= 0) tile = abl_tile;
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    const auto rg = tile_rsrc(has_g ? ga.g_out + b0c : ga.g_out, has_g ? nr * 4 : 0);
    const auto rt = rows_rsrc(tile);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    gbuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, lane * 4, 0, 0));
#pragma unroll
    for (int k = 0; k < QA; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, toff, k * kstep, kNT));
  };
  auto issue_rest = [&](int64_t tile) {
    const auto rt = rows_rsrc(tile);
#pragma unroll
    for (int k = QA; k < Q; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, toff, k * kstep, kNT));
  };

  // A tile's stores: log_prob, d/dy and the gradient rows (read back from the LDS
  // tile), through descriptors bounded at B — empty ones for absent outputs and for
  // nr = 0, so every path issues the same stores.
  auto flush = [&](int64_t b0, int64_t nr, float lp, float gy) {
    const int64_t no = want_lp ? nr : 0, ny = ga.grad_y ? nr : 0, nt = ga.grad_t ? nr : 0;
    const auto ro = tile_rsrc(no > 0 ? a.out + b0 : a.out, no * 4);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, lp), ro, lane * 4, 0, kNT);
    const auto rgy = tile_rsrc(ny > 0 ? ga.grad_y + b0 : ga.grad_y, ny * 4);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, gy), rgy, lane * 4, 0, kNT);
    const auto rgt = tile_rsrc(nt > 0 ? ga.grad_t + b0 * gts : ga.grad_t, nt > 0 ? ((nt - 1) * gts + P) * 4 : 0);
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      const float* src = tl + l0 + k * RSTEP * S;
      __builtin_amdgcn_raw_buffer_store_b128(f32x4{src[0], src[1], src[2], src[3]}, rgt, goff, k * gkstep, kNT);
    }
  };

  issue(u0);
  issue_rest(u0);
  flush(0, 0, 0.0f, 0.0f);  // empty: every path into the loop ends [loads][stores] (counted waits)
  for (int64_t tile = u0; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int64_t nr = min((int64_t)64, a.B - b0);
    if (a.prio) __builtin_amdgcn_s_setprio(3);  // hand-off + next prefetch at high priority
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      float* dst = tl + l0 + k * RSTEP * S;
      dst[0] = buf[k].x;
      dst[1] = buf[k].y;
      dst[2] = buf[k].z;
      dst[3] = buf[k].w;
    }
    float z = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
    const float gl = has_g ? gbuf : 1.0f;
    wave_lds_sync();
    issue(tile + ustep);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    const int64_t next = tile + ustep;
    auto mid = [&]() {
      if constexpr (QA < Q) issue_rest(next);
    };
    float adj;
    // rows past B (the last tile) run on zeros; their stores fall outside the descriptors
    float lp;
    if constexpr (CM == kStaticProg) {
      mid();
      lp = grad1_static<kStaticTypes[0], kStaticK[0]>(z, tl + lane * S, zh, 64, P, a.trainable != 0, gl, want_lp, adj);
    } else if constexpr (CM == kChainPairs) {
      lp = grad1_pairs(z, tl + lane * S, zh, 64, types, K, P, a.trainable != 0, gl, want_lp, adj, mid);
    } else {
      lp = grad1_packed(z, tl + lane * S, zh, 64, types, K, P, a.trainable != 0, gl, want_lp, adj, mid);
    }
    lp -= corr;
    wave_lds_sync();
    flush(b0, nr, lp, norm ? f_div<true>(adj, ystd) : adj);
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
}

// d = 1 backward with a producer / consumer workgroup (diag A/B, NFN_GRAD_PC=1): wave 0
// STREAMS — it holds the next unit's C tiles (y, g, rows) in registers while the others
// compute and writes them into the C LDS slots between two workgroup barriers — and waves
// 1..C each COMPUTE one tile per unit from their slot (forward, then the reverse pass in
// place) and store their own gradient tile, log_prob and d/dy (each prefetches its next
// tile's y and upstream gradient itself: 2 registers).  The memory stream is then
// issued by one wave per workgroup (the backward's loads stream fastest from few waves:
// DESIGN "C2 backward"), the chain by C.  Every wave of a workgroup walks the same units
// (u = blockIdx.x, + gridDim.x, ...), so both barriers are reached by all of them.
// LDS slot j: 64 rows at the odd stride S, then the K x 64 flow inputs.
__device__ __forceinline__ void wg_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int Q, int C, int CM>
__global__ void __launch_bounds__(kMaxBlock, 4) chain_grad_pc_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  constexpr int RSTEP = 64 / Q;
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = a.lds_stride;
  const int K = a.prog.K;
  const int P = a.P;
  const int64_t rs = a.t_rowstride;
  const int64_t gts = ga.gt_rowstride;
  const int r0 = lane / Q, c4 = lane % Q;
  const int l0 = r0 * S + 4 * c4;
  const int slot = 64 * S + K * 64;
  const int64_t ntiles = a.ntiles;
  const int64_t nunits = (ntiles + C - 1) / C;
  const int64_t ustep = gridDim.x;
  const bool norm = a.y_mean != nullptr;
  const bool has_g = ga.g_out != nullptr;
  const int yoff = lane * (int)a.y_bstride * 4;
  const int toff = (r0 * (int)rs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)rs * 4;
  const int64_t abl_unit = diag_ablate_loads(a) ? (int64_t)blockIdx.x : -1;  // diagnostic: compute-only timing
  if (wid == 0) {
    // ---- streamer ----
    float4 buf[C][Q];
    auto issue = [&](int64_t unit) {
      if (abl_unit >= 0) unit = abl_unit;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int64_t b0 = (unit * C + j) * 64;
        const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
        const auto rt = tile_rsrc(a.t + (nr > 0 ? b0 : 0) * rs, nr > 0 ? ((nr - 1) * rs + P) * 4 : 0);
#pragma unroll
        for (int k = 0; k < Q; ++k)
          buf[j][k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, toff, k * kstep, kNT));
      }
    };
    int64_t unit = blockIdx.x;
    issue(unit);
    for (; unit < nunits; unit += ustep) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        float* tl = lds + j * slot;
#pragma unroll
        for (int k = 0; k < Q; ++k) {
          float* dst = tl + l0 + k * RSTEP * S;
          dst[0] = buf[j][k].x;
          dst[1] = buf[j][k].y;
          dst[2] = buf[j][k].z;
          dst[3] = buf[j][k].w;
        }
      }
      wg_lds_barrier();  // A: the unit's inputs are in the slots
      issue(unit + ustep);  // past the end: empty descriptors
      wg_lds_barrier();  // B: the computing waves are done with their slots
    }
  } else if (wid <= C) {
    // ---- computing wave: tile (unit * C + wid - 1) from slot wid - 1 ----
    float* tl = lds + (wid - 1) * slot;
    float* zh = tl + 64 * S + lane;
    float ybuf, gbuf;
    auto issue_yg = [&](int64_t unit) {
      if (abl_unit >= 0) unit = abl_unit;
      const int64_t b0 = (unit * C + wid - 1) * 64;
      const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
      const int64_t b0c = nr > 0 ? b0 : 0;
      const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
      const auto rg = tile_rsrc(has_g ? ga.g_out + b0c : ga.g_out, has_g ? nr * 4 : 0);
      ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
      gbuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, lane * 4, 0, 0));
    };
    const float ymean = norm ? a.y_mean[0] : 0.0f, ystd = norm ? a.y_std[0] : 1.0f;
    const float corr = norm ? f_log<true>(ystd) : 0.0f;
    const bool want_lp = a.out != nullptr;
    const uint32_t types = a.prog.types[0];
    const int goff = (r0 * (int)gts + 4 * c4) * 4;
    const int gkstep = RSTEP * (int)gts * 4;
    auto flush = [&](int64_t b0, int64_t nr, float lp, float gy) {
      const int64_t no = want_lp ? nr : 0, ny = ga.grad_y ? nr : 0, nt = ga.grad_t ? nr : 0;
      const auto ro = tile_rsrc(no > 0 ? a.out + b0 : a.out, no * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, lp), ro, lane * 4, 0, kNT);
      const auto rgy = tile_rsrc(ny > 0 ? ga.grad_y + b0 : ga.grad_y, ny * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, gy), rgy, lane * 4, 0, kNT);
      const auto rgt =
          tile_rsrc(nt > 0 ? ga.grad_t + b0 * gts : ga.grad_t, nt > 0 ? ((nt - 1) * gts + P) * 4 : 0);
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        const float* src = tl + l0 + k * RSTEP * S;
        __builtin_amdgcn_raw_buffer_store_b128(f32x4{src[0], src[1], src[2], src[3]}, rgt, goff, k * gkstep, kNT);
      }
    };
    issue_yg(blockIdx.x);
    flush(0, 0, 0.0f, 0.0f);  // empty: every path into the loop ends [y, g][stores] (counted waits)
    for (int64_t unit = blockIdx.x; unit < nunits; unit += ustep) {
      wg_lds_barrier();  // A
      const int64_t b0 = (unit * C + wid - 1) * 64;
      const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
      float z = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
      const float gl = has_g ? gbuf : 1.0f;
      issue_yg(unit + ustep);
      float adj;
      float lp = CM == kChainPairs
                     ? grad1_pairs(z, tl + lane * S, zh, 64, types, K, P, a.trainable != 0, gl, want_lp, adj)
                     : grad1_packed(z, tl + lane * S, zh, 64, types, K, P, a.trainable != 0, gl, want_lp, adj);
      lp -= corr;
      wave_lds_sync();
      flush(b0, nr, lp, norm ? f_div<true>(adj, ystd) : adj);
      wg_lds_barrier();  // B
    }
  }
}

template <int Q>
bool launch_pc_q(const GradArgs& ga, hipStream_t s, int64_t* grid) {
  constexpr int C = 3;
  const int cm = env_int("NFN_CHAIN_FORM", ga.c.prog.K <= kPairsMaxKStream ? kChainPairs : kChainLoop);
  auto k = cm == kChainPairs ? chain_grad_pc_kernel<Q, C, kChainPairs> : chain_grad_pc_kernel<Q, C, kChainLoop>;
  const size_t lds = (size_t)C * (64 * ga.c.lds_stride + ga.c.prog.K * 64) * sizeof(float);
  const int64_t nunits = (ga.c.ntiles + C - 1) / C;
  *grid = std::max<int64_t>(1, persistent_grid(k, 64 * (C + 1), lds, nunits));
  nfn_launch((k), dim3((unsigned)*grid), dim3(64 * (C + 1)), lds, s, ga);
  return true;
}

template <int Q>
bool launch_wave1_q(const GradArgs& ga, size_t lds_block, int wpb, hipStream_t s, int64_t* grid) {
  const int cm = env_int("NFN_CHAIN_FORM", ga.c.prog.K <= kPairsMaxKStream ? kChainPairs : kChainLoop);
  auto k = cm == kChainPairs ? chain_grad_wave1_kernel<Q, kChainPairs> : chain_grad_wave1_kernel<Q, kChainLoop>;
  if (env_int("NFN_GRAD_SPLIT", 1) == 2)
    k = cm == kChainPairs ? chain_grad_wave1_kernel<Q, kChainPairs, 2> : chain_grad_wave1_kernel<Q, kChainLoop, 2>;
  if (cm == kStaticProg && ga.c.prog.K == kStaticK[0] && ga.c.prog.types[0] == kStaticTypes[0])
    k = chain_grad_wave1_kernel<Q, kStaticProg>;
  const int T = 64 * wpb;
  *grid = std::max<int64_t>(1, persistent_grid(k, T, lds_block, (ga.c.ntiles + wpb - 1) / wpb));
  nfn_launch((k), dim3((unsigned)*grid), dim3(T), lds_block, s, ga);
  return true;
}
#endif  // NFN_DIAG

template <bool FAST>
void launch_grad_t(int dm, const GradArgs& ga, dim3 grid, size_t lds, hipStream_t s) {
  switch (dm) {
    case 1: nfn_launch((chain_grad_kernel<1, FAST>), grid, 64, lds, s, ga); break;
    case 2: nfn_launch((chain_grad_kernel<2, FAST>), grid, 64, lds, s, ga); break;
    case 4: nfn_launch((chain_grad_kernel<4, FAST>), grid, 64, lds, s, ga); break;
    case 8: nfn_launch((chain_grad_kernel<8, FAST>), grid, 64, lds, s, ga); break;
    case 16: nfn_launch((chain_grad_kernel<16, FAST>), grid, 64, lds, s, ga); break;
    default: nfn_launch((chain_grad_kernel<32, FAST>), grid, 64, lds, s, ga); break;
  }
}

template <int DM, bool FAST, int NV>
bool launch_wave_nv(const GradArgs& ga, size_t lds_block, int waves_per_block, hipStream_t s, int64_t* grid) {
  // tuning knob: NFN_GRAD_CAP=1 caps registers at 4 waves per SIMD (d = 1, 8 float4 / lane)
  auto k = chain_grad_wave_kernel<DM, FAST, NV, 1>;
  if constexpr (DM == 1 && NV == 8) {
    if (env_int("NFN_GRAD_CAP", 0) == 1) k = chain_grad_wave_kernel<DM, FAST, NV, 4>;
  }
  if constexpr (DM == 1 && FAST) {
    const int cm = env_int("NFN_CHAIN_FORM", ga.c.prog.K <= kPairsMaxKStream ? kChainPairs : kChainLoop);
    if (cm == kChainPairs && env_int("NFN_GRAD_CAP", 0) != 1) k = chain_grad_wave_kernel<DM, FAST, NV, 1, kChainPairs>;
#ifdef NFN_DIAG
    // the compile-time pair bodies of an alternating program (hpair_types; at P = 4 NV only
    // K = 2 and 10 are), NFN_CHAIN_FORM=8: C2 0.846-0.851 vs 0.861-0.870 ms in one process
    // (r04m_hpair_pf.log), but as a library build 0.847-0.873 vs 0.847-0.863, and C1 0.214-0.235
    // vs 0.219-0.227 (r04o_library_ab.txt): not adopted
    const int hp = (NV == 2 || NV == 8) && env_int("NFN_GRAD_CAP", 0) != 1 ? hpair_types(ga.c) : -1;
    if constexpr (NV == 2 || NV == 8) {
      if (cm == kChainHPair && hp >= 0) {
        switch (hp) {
          case 0: k = chain_grad_wave_kernel<DM, FAST, NV, 1, hpair_form(0, 0, 1)>; break;
          case 1: k = chain_grad_wave_kernel<DM, FAST, NV, 1, hpair_form(0, 1, 1)>; break;
          case 3: k = chain_grad_wave_kernel<DM, FAST, NV, 1, hpair_form(1, 0, 1)>; break;
          default: k = chain_grad_wave_kernel<DM, FAST, NV, 1, hpair_form(1, 1, 1)>; break;
        }
      }
    }
    if (cm == kStaticProg && ga.c.prog.K == kStaticK[0] && ga.c.prog.types[0] == kStaticTypes[0])
      k = chain_grad_wave_kernel<DM, FAST, NV, 1, kStaticProg>;
    // cache-policy A/B for the row loads and gradient stores (loop form, C2's)
    const int ntl = env_int("NFN_GRAD_NTL", 1), nts = env_int("NFN_GRAD_NTS", 1);
    if (cm == kChainLoop && (ntl == 0 || nts == 0)) {
      if (ntl == 0 && nts == 0) k = chain_grad_wave_kernel<DM, FAST, NV, 1, kChainLoop, false, false>;
      else if (ntl == 0) k = chain_grad_wave_kernel<DM, FAST, NV, 1, kChainLoop, false, true>;
      else k = chain_grad_wave_kernel<DM, FAST, NV, 1, kChainLoop, true, false>;
    }
#endif
  }
  const int T = 64 * waves_per_block;
  const int64_t teams = persistent_grid(k, T, lds_block, (ga.c.ntiles + waves_per_block - 1) / waves_per_block);
  *grid = std::max<int64_t>(1, teams);
  nfn_launch((k), dim3((unsigned)*grid), dim3(T), lds_block, s, ga);
  return true;
}

template <bool FAST>
bool launch_wave_t(int dm, int nv, const GradArgs& ga, size_t lds_block, int wpb, hipStream_t s, int64_t* grid) {
  if (dm == 1) {
    switch (nv) {
      case 1: return launch_wave_nv<1, FAST, 1>(ga, lds_block, wpb, s, grid);
      case 2: return launch_wave_nv<1, FAST, 2>(ga, lds_block, wpb, s, grid);
      case 4: return launch_wave_nv<1, FAST, 4>(ga, lds_block, wpb, s, grid);
      case 8: return launch_wave_nv<1, FAST, 8>(ga, lds_block, wpb, s, grid);
      case 16: return launch_wave_nv<1, FAST, 16>(ga, lds_block, wpb, s, grid);
    }
  } else if (dm == 2) {
    switch (nv) {
      case 4: return launch_wave_nv<2, FAST, 4>(ga, lds_block, wpb, s, grid);
      case 8: return launch_wave_nv<2, FAST, 8>(ga, lds_block, wpb, s, grid);
      case 16: return launch_wave_nv<2, FAST, 16>(ga, lds_block, wpb, s, grid);
    }
  }
  return false;
}

// The per-flow Bijector API's backward (nfn_flow_vjp_f32): one bijector's vector-Jacobian
// product, what TF's tape takes through PlanarFlow._forward / _forward_log_det_jacobian
// (PlanarFlow.py:68-80), RadialFlow's (RadialFlow.py:50-70) and tfp Affine's when a loss
// reads a flow's output.  A workgroup's rows of t_k are staged in LDS (coalesced, odd
// stride; a broadcast row is copied to every lane's row), each lane runs the flow's adjoint
// with a = dL/dz_out and gl = dL/dldj — the adjoint overwrites its row with dL/dt_k and
// leaves dL/dz in `a` — and the gradient rows leave through LDS as one contiguous run.
template <int DM, bool FAST>
__global__ void __launch_bounds__(kMaxBlock) flow_vjp_kernel(FlowVjpArgs v) {
  extern __shared__ float lds[];
  const int rows = blockDim.x;
  const int tid = threadIdx.x;
  const int SP = v.ps | 1;
  const int d = v.d;
  const int64_t b0 = (int64_t)blockIdx.x * rows;
  const int nr = (int)min((int64_t)rows, v.B - b0);
  stage_rows(lds, v.t + (v.t_rowstride == 0 ? 0 : b0 * v.t_rowstride), v.t_rowstride, nr, v.ps, SP, false);
  __syncthreads();
  if (tid < nr) {
    const int64_t b = b0 + tid;
    float z[DM], a[DM];
    const float* zr = v.z + b * v.z_bstride;
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z[j] = j < d ? zr[j] : 0.0f;
      a[j] = (j < d && v.g_z) ? v.g_z[b * d + j] : 0.0f;
    }
    const float gl = v.g_ldj ? v.g_ldj[b] : 0.0f;
    float* p = lds + tid * SP;
    if (v.flow_id == NFN_FLOW_PLANAR)
      planar_bwd<DM, FAST>(z, a, p, d, gl);
    else if (v.flow_id == NFN_FLOW_RADIAL)
      radial_bwd<DM, FAST>(z, a, p, d, gl);
    else
      affine_bwd<DM, FAST>(z, a, p, d, gl);
    if (v.dz) {
#pragma unroll
      for (int j = 0; j < DM; ++j)
        if (j < d) v.dz[b * d + j] = a[j];
    }
  }
  __syncthreads();
  if (v.dt) store_rows(lds, v.dt + b0 * v.ps, v.ps, nr, v.ps, SP, false);
}

template <bool FAST>
void launch_vjp_t(int dm, const FlowVjpArgs& v, dim3 grid, size_t lds, hipStream_t s) {
  const dim3 block(kMaxBlock);
  switch (dm) {
    case 1: nfn_launch((flow_vjp_kernel<1, FAST>), grid, block, lds, s, v); break;
    case 2: nfn_launch((flow_vjp_kernel<2, FAST>), grid, block, lds, s, v); break;
    case 4: nfn_launch((flow_vjp_kernel<4, FAST>), grid, block, lds, s, v); break;
    case 8: nfn_launch((flow_vjp_kernel<8, FAST>), grid, block, lds, s, v); break;
    case 16: nfn_launch((flow_vjp_kernel<16, FAST>), grid, block, lds, s, v); break;
    default: nfn_launch((flow_vjp_kernel<32, FAST>), grid, block, lds, s, v); break;
  }
}

}  // namespace

void launch_flow_vjp(bool fast, int dm, const FlowVjpArgs& v, hipStream_t s) {
  const int64_t nblk = (v.B + kMaxBlock - 1) / kMaxBlock;
  const size_t lds = (size_t)kMaxBlock * (v.ps | 1) * sizeof(float);
  if (fast)
    launch_vjp_t<true>(dm, v, dim3((unsigned)nblk), lds, s);
  else
    launch_vjp_t<false>(dm, v, dim3((unsigned)nblk), lds, s);
}

void launch_grad(bool fast, int dm, const GradArgs& ga, dim3 grid, size_t lds, hipStream_t s) {
  if (fast)
    launch_grad_t<true>(dm, ga, grid, lds, s);
  else
    launch_grad_t<false>(dm, ga, grid, lds, s);
}

bool launch_grad_wave(bool fast, int dm, int nv, const GradArgs& ga, size_t lds_block, int waves_per_block,
                      hipStream_t s, int64_t* grid) {
#ifdef NFN_DIAG
  // diagnostic A/B: d = 1 fast math with 64-row tiles spanning < 2 GiB on the straight-line
  // buffer pipeline (NFN_GRAD_WAVE1=1)
  const ChainArgs& a = ga.c;
  if (fast && dm == 1 && a.d == 1 && a.prog.K <= 16 && a.t_rowstride * 64 * 4 < ((int64_t)1 << 31) &&
      ga.gt_rowstride * 64 * 4 < ((int64_t)1 << 31) && a.y_bstride * 64 * 4 < ((int64_t)1 << 31) &&
      env_int("NFN_GRAD_PC", 0) == 1) {
    switch (nv) {
      case 2: return launch_pc_q<2>(ga, s, grid);
      case 4: return launch_pc_q<4>(ga, s, grid);
      case 8: return launch_pc_q<8>(ga, s, grid);
    }
  }
  if (fast && dm == 1 && a.d == 1 && a.prog.K <= 16 && a.t_rowstride * 64 * 4 < ((int64_t)1 << 31) &&
      ga.gt_rowstride * 64 * 4 < ((int64_t)1 << 31) && a.y_bstride * 64 * 4 < ((int64_t)1 << 31) &&
      env_int("NFN_GRAD_WAVE1", 0) == 1) {
    switch (nv) {
      case 2: return launch_wave1_q<2>(ga, lds_block, waves_per_block, s, grid);
      case 4: return launch_wave1_q<4>(ga, lds_block, waves_per_block, s, grid);
      case 8: return launch_wave1_q<8>(ga, lds_block, waves_per_block, s, grid);
      case 16: return launch_wave1_q<16>(ga, lds_block, waves_per_block, s, grid);
    }
  }
#endif
  return fast ? launch_wave_t<true>(dm, nv, ga, lds_block, waves_per_block, s, grid)
              : launch_wave_t<false>(dm, nv, ga, lds_block, waves_per_block, s, grid);
}


}  // namespace nfn
