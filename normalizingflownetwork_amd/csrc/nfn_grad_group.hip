// nfn_grad_group.hip — the fused backward for wide events (d >= 4; config C3),
// structured like chain_group_kernel: a persistent grid whose every wave owns a
// stream of R = 64/G-sample tiles, one G-lane group per sample (lane j holds the
// DPL dimensions j, j + G, ...), inner products as DPP group sums.
// Per wave LDS slot: the tile's parameter rows (stride S from group_lds_stride)
// followed by the lanes' flow inputs zh[(k * DPL + i) * 64 + lane].  The next
// tile's rows (NV float4 per lane), y and upstream gradients are prefetched into
// registers (non-temporal) while the current tile runs forward + reverse; the
// reverse pass overwrites each flow's block with its gradient in LDS and the tile
// goes back to HBM with the load's (row, 16-byte column) slot map.
// Compiled twice: -DNFN_FAST=1 and -DNFN_FAST=0.
#include "nfn_grad_device.h"
#include "nfn_launch.h"

#ifndef NFN_FAST
#error "compile with -DNFN_FAST=0 or -DNFN_FAST=1"
#endif

namespace nfn {
namespace {

constexpr bool kFast = NFN_FAST != 0;

__device__ __forceinline__ int flow_width(int id, int d) {
  return id == NFN_FLOW_PLANAR ? 2 * d + 1 : (id == NFN_FLOW_RADIAL ? d + 2 : 2 * d);
}

template <int G, int DPL, bool FAST, int NV, bool FULL>
__global__ void __launch_bounds__(kMaxBlock) chain_grad_group_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int R = 64 / G;
  const int sl = lane / G;
  const int j = lane - sl * G;
  const int d = FULL ? G * DPL : a.d;  // FULL: d == G * DPL (no per-dimension activity tests)
  const int K = a.prog.K;
  const int Q = a.P >> 2;
  const int S = a.lds_stride;
  const bool lds4 = (S & 3) == 0;
  // float4 view for the 16-byte-aligned slots (lds4): b128 LDS accesses, not ds_*2_b32 pairs
  float4* const l4v = reinterpret_cast<float4*>(__builtin_assume_aligned(lds, 16));
  const int64_t rs = a.t_rowstride;
  const int64_t gts = ga.gt_rowstride;
  const int slot = R * S + K * DPL * 64;
  float* tl = lds + wid * slot;
  float* zh = tl + R * S + lane;
  const int r00 = lane / Q, c00 = lane - (lane / Q) * Q;
  const int sq = 64 / Q, sc = 64 - (64 / Q) * Q;
  const int nslots = R * Q;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  uint32_t tw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) tw[q] = a.prog.types[q];
  float corr = 0.0f;
  if (a.y_mean) {
    for (int i = 0; i < d; ++i) corr += f_log<FAST>(a.y_std[i]);
  }

  float4 buf[NV];
  float ybuf[DPL];
  float gbuf = 1.0f;
  bool issued_once = false;
  auto issue = [&](int64_t tile) {
    if (diag_ablate_loads(a) && issued_once) return;  // diagnostic: compute-only timing
    issued_once = true;
    const int64_t b0 = tile * R;
    const int nr = (int)min((int64_t)R, a.B - b0);
    const float* base = a.t + b0 * rs;
    int r = r00, c = c00;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (lane + k * 64 < nslots && r < nr) buf[k] = load_row4<true>(base + (int64_t)r * rs + 4 * c);
      r += sq;
      c += sc;
      if (c >= Q) {
        c -= Q;
        r += 1;
      }
    }
    if (sl < nr) {
#pragma unroll
      for (int i = 0; i < DPL; ++i)
        ybuf[i] = (j + G * i < d) ? a.y[(b0 + sl) * a.y_bstride + j + G * i] : 0.0f;
      if (ga.g_out) gbuf = ga.g_out[b0 + sl];
    }
  };

  int64_t tile = u0;
  if (tile < a.ntiles) issue(tile);
  for (; tile < a.ntiles; tile += ustep) {
    const int64_t b0 = tile * R;
    const int nr = (int)min((int64_t)R, a.B - b0);
    if (a.prio) __builtin_amdgcn_s_setprio(2);
    {
      int r = r00, c = c00;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (lane + k * 64 < nslots && r < nr) {
          float* dst = tl + r * S + 4 * c;
          if (lds4) {
            l4v[(int)(dst - lds) >> 2] = buf[k];
          } else {
            dst[0] = buf[k].x;
            dst[1] = buf[k].y;
            dst[2] = buf[k].z;
            dst[3] = buf[k].w;
          }
        }
        r += sq;
        c += sc;
        if (c >= Q) {
          c -= Q;
          r += 1;
        }
      }
    }
    float z[DPL];
#pragma unroll
    for (int i = 0; i < DPL; ++i) {
      const int jj = j + G * i;
      z[i] = ybuf[i];
      if (a.y_mean && jj < d) z[i] = f_div<FAST>(z[i] - a.y_mean[jj], a.y_std[jj]);
    }
    const float gl = gbuf;
    wave_lds_sync();
    if (tile + ustep < a.ntiles) issue(tile + ustep);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    if (sl < nr) {
      float* row = tl + sl * S;
      // forward, keeping each flow's input
      float ildj = 0.0f, dimterm = 0.0f;
      int off = a.P;
      for (int k = 0; k < K; ++k) {
        const int id = flow_type_at(tw, k);
        off -= flow_width(id, d);
        const float* p = row + off;
#pragma unroll
        for (int i = 0; i < DPL; ++i) zh[(k * DPL + i) * 64] = z[i];
        if (id == NFN_FLOW_PLANAR) {
          ildj = ildj + planar_gd<G, DPL, FAST, FULL>(z, p, d, j);
        } else if (id == NFN_FLOW_RADIAL) {
          ildj = ildj + radial_gd<G, DPL, FAST, FULL>(z, p, d, j);
        } else {
#pragma unroll
          for (int i = 0; i < DPL; ++i) {
            if (FULL || j + G * i < d) {
              const float s1 = 1.0f + p[d + j + G * i];
              z[i] = z[i] * s1 + p[j + G * i];
              dimterm += f_log<FAST>(fabsf(s1));
            }
          }
        }
      }
      if (a.out) {
        float bt = 0.0f;
#pragma unroll
        for (int i = 0; i < DPL; ++i) {
          const int jj = j + G * i;
          if (FULL || jj < d) {
            if (a.trainable) {
              const float s1 = 1e-3f + softplus_tf<FAST>(kLogExpm1One + 0.1f * row[d + jj]);
              const float zz = f_div<FAST>(z[i] - row[jj], s1);
              bt += -0.5f * (zz * zz) - f_log<FAST>(s1);
            } else {
              bt += -0.5f * (z[i] * z[i]);
            }
          }
        }
        const float lp = ((gsum<G>(dimterm + bt) - kHalfLog2Pi * (float)d) + ildj) - corr;
        if (j == 0) __builtin_nontemporal_store(lp, a.out + b0 + sl);
      }
      // reverse pass: flow K-1's block follows the base, flow k-1's follows flow k's
      float adj[DPL];
      base_gd_bwd<G, DPL, FAST, FULL>(z, adj, row, d, j, a.trainable != 0, gl);
      off = a.trainable ? 2 * d : 0;
      for (int k = K - 1; k >= 0; --k) {
        const int id = flow_type_at(tw, k);
        float zk[DPL];
#pragma unroll
        for (int i = 0; i < DPL; ++i) zk[i] = zh[(k * DPL + i) * 64];
        float* p = row + off;
        if (id == NFN_FLOW_PLANAR)
          planar_gd_bwd<G, DPL, FAST, FULL>(zk, adj, p, d, j, gl);
        else if (id == NFN_FLOW_RADIAL)
          radial_gd_bwd<G, DPL, FAST, FULL>(zk, adj, p, d, j, gl);
        else
          affine_gd_bwd<G, DPL, FAST, FULL>(zk, adj, p, d, j, gl);
        off += flow_width(id, d);
      }
      if (ga.grad_y) {
#pragma unroll
        for (int i = 0; i < DPL; ++i) {
          const int jj = j + G * i;
          if (FULL || jj < d) ga.grad_y[(b0 + sl) * d + jj] = a.y_std ? f_div<FAST>(adj[i], a.y_std[jj]) : adj[i];
        }
      }
    }
    wave_lds_sync();
    if (ga.grad_t) {
      float* gbase = ga.grad_t + b0 * gts;
      int r = r00, c = c00;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (lane + k * 64 < nslots && r < nr) {
          const float* src = tl + r * S + 4 * c;
          f32x4 v;
          if (lds4) {
            const float4 t4 = l4v[(int)(src - lds) >> 2];
            v = f32x4{t4.x, t4.y, t4.z, t4.w};
          } else {
            v = f32x4{src[0], src[1], src[2], src[3]};
          }
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(gbase + (int64_t)r * gts + 4 * c));
        }
        r += sq;
        c += sc;
        if (c >= Q) {
          c -= Q;
          r += 1;
        }
      }
    }
  }
}

// chain_grad_group_kernel for contiguous rows (t and grad_t at row stride P): the
// memory pipeline of chain_group1_kernel.  A wave tile of R rows is one contiguous
// block, read and written back at lane-linear offsets (lane * 16 + k * 1 KiB)
// through descriptors bounded at B, so no per-slot address or predicate lives in
// registers across the tile (the generic kernel's row/column walk costs ~11 VGPRs
// per float4 slot); lanes whose slot lies past the tile park it in a per-lane pad.
// y, g_out, log_prob and grad_y go through buffer instructions too, and nothing
// branches between a load and its use (rows past B compute on zeros; their
// stores fall outside the descriptors).
// SPLIT (diagnostic build only): the tile's LDS accesses through float pointers at runtime
// offsets, as before the float4 view (ds_*2_b32 pairs) — the A/B reference.
template <int G, int DPL, bool FAST, int NV, bool FULL, bool SPLIT = false>
__global__ void __launch_bounds__(kMaxBlock) chain_grad_group1_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  constexpr int R = 64 / G;
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwave = blockDim.x >> 6;
  const int sl = lane / G;
  const int j = lane - sl * G;
  const int d = FULL ? G * DPL : a.d;
  const int K = a.prog.K;
  const int P = a.P;
  const int Q = P >> 2;
  const int S = a.lds_stride;
  const int slot = R * S + K * DPL * 64;
  float* tl = lds + wid * slot;
  float* zh = tl + R * S + lane;
  float* pad = lds + nwave * slot + 4 * lane;
  const int nslots = R * Q;
  // the tile's float4 slots: S, the slot size and the pad are multiples of 4 floats and
  // the dynamic LDS starts at 0 (no static LDS), so every slot is 16-byte aligned.
  // Indexing a float4 view (not a float pointer at a runtime offset) lets the compiler
  // emit ds_write_b128 / ds_read_b128; the split ds_*2_b32 pairs it emits otherwise put
  // lanes 16 B apart on the same banks (4-way conflicts: SQ_LDS_BANK_CONFLICT 1.1e8).
  float4* lds4 = reinterpret_cast<float4*>(__builtin_assume_aligned(lds, 16));
  int loff[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = lane + 64 * k;
    loff[k] = q < nslots ? (int)(tl - lds) + (q / Q) * S + 4 * (q % Q) : (int)(pad - lds);
  }
  const int64_t u0 = (int64_t)blockIdx.x * nwave + wid;
  const int64_t ustep = (int64_t)gridDim.x * nwave;
  const int64_t ybs = a.y_bstride;
  uint32_t tw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) tw[q] = a.prog.types[q];
  float corr = 0.0f;
  if (a.y_mean) {
    for (int i = 0; i < d; ++i) corr += f_log<FAST>(a.y_std[i]);
  }
  const bool norm = a.y_mean != nullptr;
  float ymean[DPL], ystd[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    ymean[i] = (norm && jj < d) ? a.y_mean[jj] : 0.0f;
    ystd[i] = (norm && jj < d) ? a.y_std[jj] : 1.0f;
  }
  const bool abl = diag_ablate_loads(a);
  float4 buf[NV];
  float ybuf[DPL];
  float gbuf;
  auto issue = [&](int64_t tile) {
    if (abl) tile = u0;  // diagnostic: compute-only timing (the same tile over and over)
    const int64_t b0 = tile * R;
    const int64_t nr = max((int64_t)0, min((int64_t)R, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * ybs, nr > 0 ? ((nr - 1) * ybs + a.d) * 4 : 0);
#pragma unroll
    for (int i = 0; i < DPL; ++i)
      ybuf[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             ry, (int)((sl * ybs + j + G * i) * 4), 0, 0));
    if (ga.g_out) {
      const auto rg = tile_rsrc(ga.g_out + b0c, nr * 4);
      gbuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, sl * 4, 0, 0));
    } else {
      gbuf = 1.0f;
    }
    const auto rt = tile_rsrc(a.t + b0c * P, nr * P * 4);
#pragma unroll
    for (int k = 0; k < NV; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, lane * 16, k * 1024, kNT));
  };

  issue(u0);
  for (int64_t tile = u0; tile < a.ntiles; tile += ustep) {
    const int64_t b0 = tile * R;
    const int64_t nr = max((int64_t)0, min((int64_t)R, a.B - b0));
    if (a.prio) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if constexpr (SPLIT)
        *reinterpret_cast<float4*>(lds + loff[k]) = buf[k];
      else
        lds4[loff[k] >> 2] = buf[k];
    }
    float z[DPL];
#pragma unroll
    for (int i = 0; i < DPL; ++i) z[i] = norm ? f_div<FAST>(ybuf[i] - ymean[i], ystd[i]) : ybuf[i];
    const float gl = gbuf;
    wave_lds_sync();
    issue(tile + ustep);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    float* row = tl + sl * S;
    // forward, keeping each flow's input
    float ildj = 0.0f, dimterm = 0.0f;
    int off = P;
    // without a log_prob output the forward recompute only needs each flow's input
    // (z-only steps: no log-determinants)
    const bool want_lp = a.out != nullptr || !a.zonly;
    for (int k = 0; k < K; ++k) {
      const int id = flow_type_at(tw, k);
      off -= flow_width(id, d);
      const float* p = row + off;
#pragma unroll
      for (int i = 0; i < DPL; ++i) zh[(k * DPL + i) * 64] = z[i];
      if (id == NFN_FLOW_PLANAR) {
        if (want_lp)
          ildj = ildj + planar_gd<G, DPL, FAST, FULL>(z, p, d, j);
        else
          planar_gd<G, DPL, FAST, FULL, false>(z, p, d, j);
      } else if (id == NFN_FLOW_RADIAL) {
        if (want_lp)
          ildj = ildj + radial_gd<G, DPL, FAST, FULL>(z, p, d, j);
        else
          radial_gd<G, DPL, FAST, FULL, false>(z, p, d, j);
      } else {
#pragma unroll
        for (int i = 0; i < DPL; ++i) {
          if (FULL || j + G * i < d) {
            const float s1 = 1.0f + p[d + j + G * i];
            z[i] = z[i] * s1 + p[j + G * i];
            if (want_lp) dimterm += f_log<FAST>(fabsf(s1));
          }
        }
      }
    }
    float lp = 0.0f;
    if (a.out) {
      float bt = 0.0f;
#pragma unroll
      for (int i = 0; i < DPL; ++i) {
        const int jj = j + G * i;
        if (FULL || jj < d) {
          if (a.trainable) {
            const float s1 = 1e-3f + softplus_tf<FAST>(kLogExpm1One + 0.1f * row[d + jj]);
            const float zz = f_div<FAST>(z[i] - row[jj], s1);
            bt += -0.5f * (zz * zz) - f_log<FAST>(s1);
          } else {
            bt += -0.5f * (z[i] * z[i]);
          }
        }
      }
      lp = ((gsum<G>(dimterm + bt) - kHalfLog2Pi * (float)d) + ildj) - corr;
    }
    // reverse pass: flow K-1's block follows the base, flow k-1's follows flow k's
    float adj[DPL];
    base_gd_bwd<G, DPL, FAST, FULL>(z, adj, row, d, j, a.trainable != 0, gl);
    off = a.trainable ? 2 * d : 0;
    for (int k = K - 1; k >= 0; --k) {
      const int id = flow_type_at(tw, k);
      float zk[DPL];
#pragma unroll
      for (int i = 0; i < DPL; ++i) zk[i] = zh[(k * DPL + i) * 64];
      float* p = row + off;
      if (id == NFN_FLOW_PLANAR)
        planar_gd_bwd<G, DPL, FAST, FULL>(zk, adj, p, d, j, gl);
      else if (id == NFN_FLOW_RADIAL)
        radial_gd_bwd<G, DPL, FAST, FULL>(zk, adj, p, d, j, gl);
      else
        affine_gd_bwd<G, DPL, FAST, FULL>(zk, adj, p, d, j, gl);
      off += flow_width(id, d);
    }
    wave_lds_sync();
    // lane i < R takes sample i's log_prob (one store per sample); rows past B are dropped
    const float lpv = __shfl(lp, (lane * G) & 63);
    if (a.out) {
      const auto ro = tile_rsrc(nr > 0 ? a.out + b0 : a.out, nr * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, lpv), ro, lane * 4, 0, kNT);
    }
    if (ga.grad_y) {
      const auto rgy = tile_rsrc(nr > 0 ? ga.grad_y + b0 * d : ga.grad_y, nr * d * 4);
#pragma unroll
      for (int i = 0; i < DPL; ++i) {
        const int jj = j + G * i;
        const float v = norm ? f_div<FAST>(adj[i], ystd[i]) : adj[i];
        // dimensions past d (FULL == false) point past the row: out of range only on the last row
        if (FULL || jj < d)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rgy, (sl * d + jj) * 4, 0, 0);
      }
    }
    if (ga.grad_t) {
      const auto rgt = tile_rsrc(nr > 0 ? ga.grad_t + b0 * P : ga.grad_t, nr * P * 4);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const float4 t4 = SPLIT ? *reinterpret_cast<const float4*>(lds + loff[k]) : lds4[loff[k] >> 2];
        __builtin_amdgcn_raw_buffer_store_b128(f32x4{t4.x, t4.y, t4.z, t4.w}, rgt, lane * 16, k * 1024, kNT);
      }
    }
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
}

template <int G, int DPL, int NV>
void launch_gg1(const GradArgs& ga, hipStream_t s, int64_t* grid_out) {
  auto kfn = ga.c.d == G * DPL ? chain_grad_group1_kernel<G, DPL, kFast, NV, true>
                                : chain_grad_group1_kernel<G, DPL, kFast, NV, false>;
#ifdef NFN_DIAG
  if (env_int("NFN_LDS_SPLIT", 0) == 1)
    kfn = ga.c.d == G * DPL ? chain_grad_group1_kernel<G, DPL, kFast, NV, true, true>
                            : chain_grad_group1_kernel<G, DPL, kFast, NV, false, true>;
#endif
  const int wpb = env_int("NFN_GRAD_GROUP_WPB", 4) == 2 ? 2 : 4;
  const int R = 64 / G;
  const size_t lds_b = ((size_t)wpb * (R * ga.c.lds_stride + ga.c.prog.K * DPL * 64) + 64 * 4) * sizeof(float);
  const int T = 64 * wpb;
  const int64_t grid = persistent_grid(kfn, T, lds_b, (ga.c.ntiles + wpb - 1) / wpb);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(T), lds_b, s, ga);
}

template <int G, int DPL, int NV>
void launch_gg(const GradArgs& ga, size_t lds, hipStream_t s, int64_t* grid_out) {
  // contiguous rows: the lane-linear buffer pipeline (NFN_GRAD_GROUP1=0: the generic walk)
  const ChainArgs& a = ga.c;
  if (a.t_rowstride == a.P && (!ga.grad_t || ga.gt_rowstride == a.P) && !a.partials &&
      (int64_t)(64 / G) * a.P * 4 < (int64_t)1 << 31 && a.y_bstride * (64 / G) * 4 < (int64_t)1 << 31 &&
      env_int("NFN_GRAD_GROUP1", 1) != 0) {
    launch_gg1<G, DPL, NV>(ga, s, grid_out);
    return;
  }
  // Four-wave workgroups (C3 with the FULL specialisation: 1.004-1.018 ms vs
  // 1.007-1.068 with two; two-wave groups had won by 2.5 % before it); a register
  // cap at 3 waves per SIMD spills (2.07 ms).  NFN_GRAD_GROUP_WPB=2 for two.
  auto kfn = ga.c.d == G * DPL ? chain_grad_group_kernel<G, DPL, kFast, NV, true>
                                : chain_grad_group_kernel<G, DPL, kFast, NV, false>;
  const int wpb = env_int("NFN_GRAD_GROUP_WPB", 4) == 2 ? 2 : 4;
  const size_t lds_b = lds / 4 * wpb;  // `lds` holds four wave slots
  const int T = 64 * wpb;
  const int64_t grid = persistent_grid(kfn, T, lds_b, (ga.c.ntiles + wpb - 1) / wpb);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(T), lds_b, s, ga);
}

template <int G, int DPL>
bool launch_gg_nv(int nv, const GradArgs& ga, size_t lds, hipStream_t s, int64_t* g) {
  if (nv <= 4)
    launch_gg<G, DPL, 4>(ga, lds, s, g);
  else if (nv <= 6)
    launch_gg<G, DPL, 6>(ga, lds, s, g);
  else if (nv <= 9)
    launch_gg<G, DPL, 9>(ga, lds, s, g);
  else if (nv <= 12)
    launch_gg<G, DPL, 12>(ga, lds, s, g);
  else if (nv <= 16)
    launch_gg<G, DPL, 16>(ga, lds, s, g);
  else
    return false;
  return true;
}

}  // namespace

#if NFN_FAST
bool launch_grad_group_fast(int G, int DPL, int nv, const GradArgs& ga, size_t lds, hipStream_t s, int64_t* grid) {
#else
bool launch_grad_group_precise(int G, int DPL, int nv, const GradArgs& ga, size_t lds, hipStream_t s,
                               int64_t* grid) {
#endif
  if (G == 4 && DPL == 1) return launch_gg_nv<4, 1>(nv, ga, lds, s, grid);
  if (G == 4 && DPL == 2) return launch_gg_nv<4, 2>(nv, ga, lds, s, grid);
  if (G == 4 && DPL == 4) return launch_gg_nv<4, 4>(nv, ga, lds, s, grid);
  if (G == 8 && DPL == 4) return launch_gg_nv<8, 4>(nv, ga, lds, s, grid);
  if constexpr (kFast) {  // alternates for tuning runs (NFN_GROUP_LANES=8)
    if (G == 8 && DPL == 1) return launch_gg_nv<8, 1>(nv, ga, lds, s, grid);
    if (G == 8 && DPL == 2) return launch_gg_nv<8, 2>(nv, ga, lds, s, grid);
  }
  return false;
}

}  // namespace nfn
