// nfn_dense.hip — the reference's output Dense layer fused into the chain
// (SURVEY.md §8(f) row 2): t = h W + b (MaximumLikelihoodNNEstimator.py:43, linear
// activation) is formed on chip from the last hidden activations h (B, H), so the
// kernel streams 4H bytes of h per sample instead of the 4P bytes of t
// (C2 with H = 16: 64 B instead of 128 B).
//
// Persistent grid, every wave owns a stream of 64-sample tiles.  Per tile:
//   1. the tile's h rows (prefetched into registers one tile ahead, non-temporal,
//      coalesced 16-byte pieces) go to the wave's LDS slot at an odd row stride;
//   2. the 64 x P tile of t is computed with v_mfma_f32_16x16x4_f32 (exact fp32,
//      = an fmaf chain): A = h from LDS (lane l: row 16 mt + l % 16, k = 4 ks + l / 16),
//      B = W from the workgroup's LDS copy, four 16-row M tiles per 16-column N tile;
//      accumulators + bias are written into the wave's t tile (odd stride);
//   3. the chain runs per lane exactly as in chain_persistent_kernel.
#include "nfn_bf16.h"
#include "nfn_launch.h"

namespace nfn {
namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int DM, bool FAST, int NVH>
__global__ void __launch_bounds__(kMaxBlock) chain_dense_kernel(DenseArgs da) {
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int H = da.H;
  const int QH = H >> 2;             // float4 pieces per h row (power of two, <= 16)
  const int SH = da.h_lds_stride;    // odd
  const int S = a.lds_stride;        // odd, >= P
  const int P = a.P;
  const int NN = (P + 15) >> 4;      // 16-column N tiles
  const int NK = QH;                 // k-steps of 4
  const int NP = NN * 16;
  // LDS: [W: H x NP, zero-padded] [per wave: h tile 64 x SH | t tile 64 x S]
  float* wl = lds;
  float* hl = lds + H * NP + wid * (64 * SH + 64 * S);
  float* tl = hl + 64 * SH;
  for (int i = tid; i < H * NP; i += blockDim.x) {
    const int k = i / NP, n = i - (i / NP) * NP;
    wl[i] = n < P ? da.W[(int64_t)k * P + n] : 0.0f;
  }
  __syncthreads();
  const int r0 = lane / QH;
  const int c4 = lane - r0 * QH;
  const int rstep = 64 / QH;
  const int64_t hs = da.h_rowstride;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  float corr = 0.0f;
  if (a.y_mean) {
    for (int j = 0; j < a.d; ++j) corr += f_log<FAST>(a.y_std[j]);
  }

  float4 buf[NVH];
  float ybuf[DM];
  auto issue = [&](int64_t tile) {
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
    const float* base = da.h + b0 * hs + 4 * c4;
#pragma unroll
    for (int k = 0; k < NVH; ++k)
      if (r0 + k * rstep < nr) buf[k] = load_row4<true>(base + (int64_t)(r0 + k * rstep) * hs);
    if (lane < nr) {
      const float* yr = a.y + (b0 + lane) * a.y_bstride;
#pragma unroll
      for (int j = 0; j < DM; ++j) ybuf[j] = j < a.d ? yr[j] : 0.0f;
    }
  };

  double acc_sum = 0.0;
  int nfc = 0;  // non-finite log_prob values
  int64_t tile = u0;
  if (tile < a.ntiles) issue(tile);
  for (; tile < a.ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
#pragma unroll
    for (int k = 0; k < NVH; ++k) {
      const int r = r0 + k * rstep;
      float* dst = hl + r * SH + 4 * c4;
      const float4 v = r < nr ? buf[k] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      dst[0] = v.x;
      dst[1] = v.y;
      dst[2] = v.z;
      dst[3] = v.w;
    }
    float z[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z[j] = ybuf[j];
      if (a.y_mean && j < a.d) z[j] = f_div<FAST>(z[j] - a.y_mean[j], a.y_std[j]);
    }
    wave_lds_sync();
    if (tile + ustep < a.ntiles) issue(tile + ustep);
    // t = h W + b on the matrix cores, 16 columns at a time
    const int am = lane & 15;      // A row within an M tile / B and C column
    const int ak = lane >> 4;      // A column (k) within a k-step / B row / C row quad
    for (int nt = 0; nt < NN; ++nt) {
      f32x4v acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      for (int ks = 0; ks < NK; ++ks) {
        const float bv = wl[(4 * ks + ak) * NP + 16 * nt + am];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const float av = hl[(16 * mt + am) * SH + 4 * ks + ak];
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[mt], 0, 0, 0);
        }
      }
      const int n = 16 * nt + am;
      if (n < P) {
        const float bn = da.bias ? da.bias[n] : 0.0f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) tl[(16 * mt + 4 * ak + i) * S + n] = acc[mt][i] + bn;
        }
      }
    }
    wave_lds_sync();
    if (lane < nr) {
      const float* row = tl + lane * S;
      float lp;
      if constexpr (DM == 1 && FAST)
        lp = (a.prog.K <= 16 ? eval_chain1_fast<true, 1, kChainLoop, false>(z[0], row, a)
                             : eval_chain1_fast<false, 1, kChainLoop, false>(z[0], row, a)) - corr;
      else
        lp = eval_chain<DM, FAST>(z, row, a) - corr;
      if (a.out) __builtin_nontemporal_store(lp, a.out + b0 + lane);
      acc_sum += (double)lp;
      nfc += nonfinite1(lp);
    }
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
  if (a.partials) {
    write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// d = 1, fast math: chain_dense_kernel with chain_wave1_kernel's memory pipeline —
// the tile's h rows and y through buffer descriptors bounded at B (tiles past the
// end empty), one counted wait per hand-off, the previous tile's log_prob stored
// after the next prefetch, no branch between a load and its use.  QH = H / 4.
// NN = 16-column N tiles of t (P <= 16 NN), a compile-time count so the GEMM unrolls
// and the tile's A fragments are read from LDS once for all N tiles.
// SB (H = 16, P <= 32): t = h W on v_mfma_f32_16x16x32_bf16 with exact 3-way splits
// (nfn_bf16.h) instead of v_mfma_f32_16x16x4_f32.  K = 32 holds two parts of the 16 hidden
// units, so the six products take three MFMAs per 16 x 16 block of t:
//   [h3 | h2] x [W1 ; W2],  [h1 | h1] x [W3 ; W2],  [h2 | h1] x [W1 ; W1]  (smallest first),
// lane group g = lane >> 4 holding K slots 8 g .. 8 g + 7 = hidden 8 (g & 1) + j of part
// (g < 2 ? first : second).  W is split once per launch into registers; h is split once per
// tile at the hand-off, each loading lane writing its float4's three parts (ds_write_b64)
// into three bf16 planes [row][16] of the wave's slot, read back as one ds_read_b128 per
// fragment (rows 16 mt + lane % 16, chunk g & 1: conflict-free in the guide's b128 lane
// groups).
constexpr int kSbPlane = 64 * 8;  // dwords per bf16 plane of the h tile (64 rows x 16 bf16)
__host__ __device__ inline int dense1_sb_wave_floats(int P, int SH) {
  return std::max(dense1_wave_floats(P, SH), 3 * kSbPlane);
}
template <int QH, int NN, int CM = kChainLoop, bool SB = false>
__global__ void __launch_bounds__(kMaxBlock) chain_dense1_kernel(DenseArgs da) {
  static_assert(!SB || (QH == 4 && NN <= 2), "split-bf16 t: H = 16, P <= 32");
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int H = 4 * QH;
  constexpr int RSTEP = 64 / QH;  // h rows per wave-instruction
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int SH = da.h_lds_stride;  // odd
  const int P = a.P;
  constexpr int NP = NN * 16;
  // t tile column-major at the padded column stride kCS (== 4 mod 32 dwords: the
  // MFMA results leave as conflict-free ds_write_b128 of 4 rows, and the chain's
  // per-lane reads of one column are consecutive), one spare column for the packed
  // chain's read-ahead, overlaying the h tile: a wave's t writes follow its own A
  // fragment reads of h in LDS program order
  float* wl = lds;
  float* hl = lds + H * NP + wid * (SB ? dense1_sb_wave_floats(P, SH) : dense1_wave_floats(P, SH));
  float* tl = hl;
  for (int i = tid; i < H * NP; i += blockDim.x) {
    const int k = i / NP, n = i - (i / NP) * NP;
    wl[i] = n < P ? da.W[(int64_t)k * P + n] : 0.0f;
  }
  __syncthreads();
  const int r0 = lane / QH, c4 = lane % QH;
  const int l0 = r0 * SH + 4 * c4;
  const int am = lane & 15;  // A row within an M tile / B and C column
  const int ak = lane >> 4;  // A column (k) within a k-step / B row / C row quad
  // B fragments (W) stay in registers for the whole launch when they are few
  constexpr bool kBReg = QH * NN <= 16;
  float bvr[kBReg ? QH : 1][kBReg ? NN : 1];
  if constexpr (kBReg && !SB) {
#pragma unroll
    for (int ks = 0; ks < QH; ++ks)
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) bvr[ks][nt] = wl[(4 * ks + ak) * NP + 16 * nt + am];
  }
  // SB: the B fragments of the three MFMAs per N tile, [W1 ; W2], [W3 ; W2], [W1 ; W1]
  // (lane: column 16 nt + am, hidden 8 (ak & 1) + j, part by ak < 2)
  bf16x8v wsb[SB ? NN : 1][3];
  if constexpr (SB) {
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      uint32_t w1[4], w2[4], w3[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k0 = 8 * (ak & 1) + 2 * q;
        split3_pk(wl[k0 * NP + 16 * nt + am], wl[(k0 + 1) * NP + 16 * nt + am], w1[q], w2[q], w3[q]);
      }
      const bool lo = ak < 2;
      wsb[nt][0] = lo ? frag8(w1[0], w1[1], w1[2], w1[3]) : frag8(w2[0], w2[1], w2[2], w2[3]);
      wsb[nt][1] = lo ? frag8(w3[0], w3[1], w3[2], w3[3]) : frag8(w2[0], w2[1], w2[2], w2[3]);
      wsb[nt][2] = frag8(w1[0], w1[1], w1[2], w1[3]);
    }
  }
  const int64_t hs = da.h_rowstride;
  const int64_t ntiles = a.ntiles;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const int yoff = lane * (int)a.y_bstride * 4;
  const int hoff = (r0 * (int)hs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)hs * 4;
  float4 buf[QH];
  float ybuf;
  auto issue = [&](int64_t tile) {
    if (diag_ablate_loads(a)) tile = u0;  // diagnostic: compute-only timing (the first tile re-read)
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    const auto rh = tile_rsrc(da.h + b0c * hs, nr > 0 ? ((nr - 1) * hs + H) * 4 : 0);
#pragma unroll
    for (int k = 0; k < QH; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, hoff, k * kstep, kNT));
  };
  double acc_sum = 0.0;
  int nfc = 0;  // non-finite log_prob values
  __amdgpu_buffer_rsrc_t pend_r = tile_rsrc(a.out, 0);
  float pend_v = 0.0f;
  auto flush = [&]() {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pend_v), pend_r, lane * 4, 0, kNT);
  };
  issue(u0);
  flush();  // empty: every path into the loop ends [loads][store] (counted waits)
  for (int64_t tile = u0; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    if constexpr (SB) {  // the three bf16 planes of the h tile: row r0 + 16 k, hidden 4 c4 .. 4 c4 + 3
#pragma unroll
      for (int k = 0; k < QH; ++k) {
        uint32_t p1[2], p2[2], p3[2];
        split3_pk(buf[k].x, buf[k].y, p1[0], p2[0], p3[0]);
        split3_pk(buf[k].z, buf[k].w, p1[1], p2[1], p3[1]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(hl) + (r0 + k * RSTEP) * 8 + 2 * c4;
        *reinterpret_cast<uint2*>(dst) = make_uint2(p1[0], p1[1]);
        *reinterpret_cast<uint2*>(dst + kSbPlane) = make_uint2(p2[0], p2[1]);
        *reinterpret_cast<uint2*>(dst + 2 * kSbPlane) = make_uint2(p3[0], p3[1]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < QH; ++k) {
        float* dst = hl + l0 + k * RSTEP * SH;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
    }
    const float z0 = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
    wave_lds_sync();
    issue(tile + ustep);
    flush();
    if constexpr (SB) {
      // A fragments [h3 | h2], [h1 | h1], [h2 | h1]: plane (ak < 2 ? 2 : 1), 0, (ak < 2 ? 1 : 0)
      const uint32_t* pl = reinterpret_cast<const uint32_t*>(hl) + 4 * (ak & 1);
      const int pa = ak < 2 ? 2 * kSbPlane : kSbPlane, pc = ak < 2 ? kSbPlane : 0;
      f32x4v acc[NN][4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {  // one M tile's fragments live at a time
        const uint32_t* row = pl + (16 * mt + am) * 8;
        const bf16x8v h0 = frag8(*reinterpret_cast<const u32x4v*>(row + pa));
        const bf16x8v h1 = frag8(*reinterpret_cast<const u32x4v*>(row));
        const bf16x8v h2 = frag8(*reinterpret_cast<const u32x4v*>(row + pc));
#pragma unroll
        for (int nt = 0; nt < NN; ++nt) {
          acc[nt][mt] = mfma_bf16(h0, wsb[nt][0], f32x4v{0.0f, 0.0f, 0.0f, 0.0f});
          acc[nt][mt] = mfma_bf16(h1, wsb[nt][1], acc[nt][mt]);
          acc[nt][mt] = mfma_bf16(h2, wsb[nt][2], acc[nt][mt]);
        }
      }
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) {  // every plane read is done: t overlays the planes
        const int n = 16 * nt + am;
        if (n < P) {
          const float bn = da.bias ? da.bias[n] : 0.0f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            *reinterpret_cast<f32x4v*>(tl + n * kCS + 16 * mt + 4 * ak) = acc[nt][mt] + bn;
        }
      }
    } else {
    // t = h W + b on the matrix cores, 16 columns at a time (exact fp32); the A
    // fragments (4 M tiles x QH k-steps) are shared by every N tile
    float av[4][QH];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int ks = 0; ks < QH; ++ks) av[mt][ks] = hl[(16 * mt + am) * SH + 4 * ks + ak];
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      f32x4v acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < QH; ++ks) {
        const float bv = kBReg ? bvr[kBReg ? ks : 0][kBReg ? nt : 0] : wl[(4 * ks + ak) * NP + 16 * nt + am];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][ks], bv, acc[mt], 0, 0, 0);
      }
      const int n = 16 * nt + am;
      if (n < P) {
        const float bn = da.bias ? da.bias[n] : 0.0f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          *reinterpret_cast<f32x4v*>(tl + n * kCS + 16 * mt + 4 * ak) = acc[mt] + bn;
      }
    }
    }
    wave_lds_sync();
    const float lp = (a.prog.K <= 16 ? eval_chain1_fast<true, kCS, CM, false>(z0, tl + lane, a)
                                     : eval_chain1_fast<false, kCS, kChainLoop, false>(z0, tl + lane, a)) - corr;
    if (lane < nr) {
      acc_sum += (double)lp;
      nfc += nonfinite1(lp);
    }
    pend_v = lp;
    pend_r = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
  flush();
  if (a.partials) {
    write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// (Measured and removed: the split-bf16 t_s of chain_dense1_kernel<SB> here, W_s split per unit
// in registers and h_s into LDS planes, ran C5 at 0.2285 vs 0.2186 ms — W_s changes every
// unit, so the splits cost more than the MFMAs save; commit 5510a5c, profiles/r06/r06u/.)
// Bayesian posterior with the output DenseVariational layer fused
// (BayesianNNEstimator.py:65-76 score over draws, :136-145 the variational output
// layer): per sample, logsumexp over S draws of log_prob(y | t_s = h_s W_s + b_s) - log S.
// d = 1, fast math.  A wave walks (tile, draw) units — its 64-sample tile through all
// S draws — with chain_dense1_kernel's memory pipeline: the NEXT unit's h tile, y and
// W / bias fragments are prefetched (buffer loads, counted waits) while the current
// unit runs the MFMA GEMM and the chain; the tile's result leaves once, after its
// last draw (the per-unit store of the other draws goes through an empty descriptor).
template <int QH, int NN, int CM = kChainLoop>
__global__ void __launch_bounds__(kMaxBlock) posterior_dense1_kernel(DenseArgs da) {
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int RSTEP = 64 / QH;
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int SH = da.h_lds_stride;
  const int P = a.P;
  const int S = a.S;
  float* hl = lds + wid * dense1_wave_floats(P, SH);
  float* tl = hl;
  const int r0 = lane / QH, c4 = lane % QH;
  const int l0 = r0 * SH + 4 * c4;
  const int am = lane & 15, ak = lane >> 4;
  const int64_t hs = da.h_rowstride;
  const int64_t ntiles = a.ntiles;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const int yoff = lane * (int)a.y_bstride * 4;
  const int hoff = (r0 * (int)hs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)hs * 4;
  int woff[QH][NN];  // this lane's B-fragment offsets in W_s (bytes); columns >= P read row 0 and are zeroed
  bool wcol[NN];
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    wcol[nt] = 16 * nt + am < P;
#pragma unroll
    for (int ks = 0; ks < QH; ++ks) woff[ks][nt] = wcol[nt] ? ((4 * ks + ak) * P + 16 * nt + am) * 4 : 0;
  }
  float4 buf[QH];
  float ybuf;
  float wbuf[QH][NN], bbuf[NN];
  auto issue = [&](int64_t tile, int sd) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    const auto rh = tile_rsrc(da.h + sd * da.h_drawstride + b0c * hs, nr > 0 ? ((nr - 1) * hs + 4 * QH) * 4 : 0);
#pragma unroll
    for (int k = 0; k < QH; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, hoff, k * kstep, kNT));
    const auto rw = tile_rsrc(da.W + sd * da.w_drawstride, nr > 0 ? (int64_t)4 * QH * P * 4 : 0);
#pragma unroll
    for (int ks = 0; ks < QH; ++ks)
#pragma unroll
      for (int nt = 0; nt < NN; ++nt)
        wbuf[ks][nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, woff[ks][nt], 0, 0));
    const auto rb = tile_rsrc(da.bias ? da.bias + sd * da.b_drawstride : da.W, (da.bias && nr > 0) ? P * 4 : 0);
#pragma unroll
    for (int nt = 0; nt < NN; ++nt)
      bbuf[nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, (16 * nt + am) * 4, 0, 0));
  };
  double acc_sum = 0.0;
  int nfc = 0;  // non-finite log_prob values
  __amdgpu_buffer_rsrc_t pend_r = tile_rsrc(a.out, 0);
  float pend_v = 0.0f;
  auto flush = [&]() {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pend_v), pend_r, lane * 4, 0, kNT);
  };
  issue(u0, 0);
  flush();  // empty: every path into the loop ends [loads][store]
  for (int64_t tile = u0; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    float m = -INFINITY, lacc = 0.0f;
    for (int sd = 0; sd < S; ++sd) {
#pragma unroll
      for (int k = 0; k < QH; ++k) {
        float* dst = hl + l0 + k * RSTEP * SH;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
      float wv[QH][NN], bv[NN];
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) {
        bv[nt] = bbuf[nt];
#pragma unroll
        for (int ks = 0; ks < QH; ++ks) wv[ks][nt] = wcol[nt] ? wbuf[ks][nt] : 0.0f;
      }
      const float z0 = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
      wave_lds_sync();
      const bool last = sd + 1 == S;
      issue(last ? tile + ustep : tile, last ? 0 : sd + 1);
      flush();
      pend_r = tile_rsrc(a.out, 0);  // later draws of this tile store nothing
      float av[4][QH];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int ks = 0; ks < QH; ++ks) av[mt][ks] = hl[(16 * mt + am) * SH + 4 * ks + ak];
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) {
        f32x4v acc[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < QH; ++ks)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][ks], wv[ks][nt], acc[mt], 0, 0, 0);
        const int n = 16 * nt + am;
        if (n < P) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            *reinterpret_cast<f32x4v*>(tl + n * kCS + 16 * mt + 4 * ak) = acc[mt] + bv[nt];
        }
      }
      wave_lds_sync();
      const float lp = (a.prog.K <= 16 ? eval_chain1_fast<true, kCS, CM, false>(z0, tl + lane, a)
                                       : eval_chain1_fast<false, kCS, kChainLoop, false>(z0, tl + lane, a)) - corr;
      lse_push<true>(m, lacc, lp);
      wave_lds_sync();  // this unit's LDS reads done before the next unit's writes
    }
    const float res = lse_finish<true>(m, lacc, S);
    if (lane < nr) {
      acc_sum += (double)res;
      nfc += nonfinite1(res);
    }
    pend_v = res;
    pend_r = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
  }
  flush();
  if (a.partials) {
    write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// The posterior for any d <= 8 and either math mode: one tile of 64 samples per
// wave, the S draws in turn (h_s rows staged to LDS, W_s fragments read from
// global memory / L2, t_s = h_s W_s + b_s on the matrix cores, the chain, the
// online logsumexp).  Plain synchronous loads: the generality path.
template <int DM, bool FAST>
__global__ void __launch_bounds__(kMaxBlock) posterior_dense_kernel(DenseArgs da) {
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int H = da.H;
  const int QH = H >> 2;
  const int SH = da.h_lds_stride;
  const int S = a.lds_stride;
  const int P = a.P;
  const int NN = (P + 15) >> 4;
  float* hl = lds + wid * (64 * SH + 64 * S);
  float* tl = hl + 64 * SH;
  const int am = lane & 15, ak = lane >> 4;
  const int64_t hs = da.h_rowstride;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  float corr = 0.0f;
  if (a.y_mean) {
    for (int j = 0; j < a.d; ++j) corr += f_log<FAST>(a.y_std[j]);
  }
  double acc_sum = 0.0;
  int nfc = 0;  // non-finite log_prob values
  for (int64_t tile = u0; tile < a.ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
    float z0[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z0[j] = (lane < nr && j < a.d) ? a.y[(b0 + lane) * a.y_bstride + j] : 0.0f;
      if (a.y_mean && j < a.d) z0[j] = f_div<FAST>(z0[j] - a.y_mean[j], a.y_std[j]);
    }
    float m = -INFINITY, lacc = 0.0f;
    for (int sd = 0; sd < a.S; ++sd) {
      const float* hsrc = da.h + sd * da.h_drawstride + b0 * hs;
      for (int i = lane; i < 64 * QH; i += 64) {
        const int r = i / QH, c = i - (i / QH) * QH;
        const float4 v = r < nr ? load_row4<true>(hsrc + (int64_t)r * hs + 4 * c) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float* dst = hl + r * SH + 4 * c;
        dst[0] = v.x;
        dst[1] = v.y;
        dst[2] = v.z;
        dst[3] = v.w;
      }
      wave_lds_sync();
      const float* Ws = da.W + sd * da.w_drawstride;
      for (int nt = 0; nt < NN; ++nt) {
        const int n = 16 * nt + am;
        f32x4v acc[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
        for (int ks = 0; ks < QH; ++ks) {
          const float bv = n < P ? Ws[(4 * ks + ak) * P + n] : 0.0f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const float av = hl[(16 * mt + am) * SH + 4 * ks + ak];
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[mt], 0, 0, 0);
          }
        }
        if (n < P) {
          const float bn = da.bias ? da.bias[sd * da.b_drawstride + n] : 0.0f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
            for (int i = 0; i < 4; ++i) tl[(16 * mt + 4 * ak + i) * S + n] = acc[mt][i] + bn;
          }
        }
      }
      wave_lds_sync();
      float z[DM];
#pragma unroll
      for (int j = 0; j < DM; ++j) z[j] = z0[j];
      const float lp = eval_chain<DM, FAST>(z, tl + lane * S, a) - corr;
      lse_push<FAST>(m, lacc, lp);
      wave_lds_sync();
    }
    if (lane < nr) {
      const float res = lse_finish<FAST>(m, lacc, a.S);
      if (a.out) __builtin_nontemporal_store(res, a.out + b0 + lane);
      acc_sum += (double)res;
      nfc += nonfinite1(res);
    }
  }
  if (a.partials) {
    write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// The posterior with the output DenseVariational layer fused for d >= 2 (fast math, H in
// {4, 8, 16}, P <= 64): posterior_dense1_kernel's memory pipeline around the generic chain.
// A wave walks (tile, draw) units — its 64-sample tile through all S draws; the NEXT
// unit's h tile (QH float4 per lane), W_s B-fragments (QH x NN per lane) and bias are
// buffer-prefetched through descriptors bounded at B (counted waits, no per-lane
// branches) while the current unit runs t_s = h_s W_s + b_s on the matrix cores
// (v_mfma_f32_16x16x4_f32, exact fp32) into the wave's row-major t tile, the chain
// (eval_chain, one sample per lane) and the online logsumexp; the tile's y rows are
// prefetched with its first draw and its score leaves once, after its last draw.
// posterior_dense_kernel (synchronous loads, W_s fragments from L2) stays the precise-math
// and wide-H form.
template <int DM, int QH>
__global__ void __launch_bounds__(kMaxBlock) posterior_densep_kernel(DenseArgs da) {
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int RSTEP = 64 / QH;
  constexpr int kNT = 2;
  constexpr int NNMAX = 4;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int SH = da.h_lds_stride;
  const int S = a.lds_stride;
  const int P = a.P;
  const int d = a.d;
  const int NN = (P + 15) >> 4;
  const int ND = a.S;  // draws
  float* hl = lds + wid * (64 * SH + 64 * S);
  float* tl = hl + 64 * SH;
  const int r0 = lane / QH, c4 = lane % QH;
  const int l0 = r0 * SH + 4 * c4;
  const int am = lane & 15, ak = lane >> 4;
  const int64_t hs = da.h_rowstride;
  const int64_t ntiles = a.ntiles;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool norm = a.y_mean != nullptr;
  float corr = 0.0f;
  if (norm) {
    for (int j = 0; j < d; ++j) corr += f_log<true>(a.y_std[j]);
  }
  const int yoff = lane * (int)a.y_bstride * 4;
  const int hoff = (r0 * (int)hs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)hs * 4;
  int woff[QH][NNMAX];  // this lane's B-fragment offsets in W_s (bytes); columns >= P read row 0 and are zeroed
  bool wcol[NNMAX];
#pragma unroll
  for (int nt = 0; nt < NNMAX; ++nt) {
    wcol[nt] = 16 * nt + am < P;
#pragma unroll
    for (int ks = 0; ks < QH; ++ks) woff[ks][nt] = wcol[nt] ? ((4 * ks + ak) * P + 16 * nt + am) * 4 : 0;
  }
  float4 buf[QH];
  float ybuf[DM];
  float wbuf[QH][NNMAX], bbuf[NNMAX];
  auto issue = [&](int64_t tile, int sd) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    if (sd == 0) {  // the tile's y rows, with its first draw
      const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + d) * 4 : 0);
#pragma unroll
      for (int j = 0; j < DM; ++j)
        ybuf[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff + 4 * min(j, d - 1), 0, 0));
    }
    const auto rh = tile_rsrc(da.h + sd * da.h_drawstride + b0c * hs, nr > 0 ? ((nr - 1) * hs + 4 * QH) * 4 : 0);
#pragma unroll
    for (int k = 0; k < QH; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, hoff, k * kstep, kNT));
    const auto rw = tile_rsrc(da.W + sd * da.w_drawstride, nr > 0 ? (int64_t)4 * QH * P * 4 : 0);
#pragma unroll
    for (int ks = 0; ks < QH; ++ks)
#pragma unroll
      for (int nt = 0; nt < NNMAX; ++nt)
        wbuf[ks][nt] = nt < NN ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, woff[ks][nt], 0, 0))
                               : 0.0f;
    const auto rb = tile_rsrc(da.bias ? da.bias + sd * da.b_drawstride : da.W, (da.bias && nr > 0) ? P * 4 : 0);
#pragma unroll
    for (int nt = 0; nt < NNMAX; ++nt)
      bbuf[nt] = nt < NN ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, (16 * nt + am) * 4, 0, 0))
                         : 0.0f;
  };
  double acc_sum = 0.0;
  int nfc = 0;  // non-finite log_prob values
  __amdgpu_buffer_rsrc_t pend_r = tile_rsrc(a.out, 0);
  float pend_v = 0.0f;
  auto flush = [&]() {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pend_v), pend_r, lane * 4, 0, kNT);
  };
  issue(u0, 0);
  flush();  // empty: every path into the loop ends [loads][store]
  for (int64_t tile = u0; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    float z0[DM];
    float m = -INFINITY, lacc = 0.0f;
    for (int sd = 0; sd < ND; ++sd) {
#pragma unroll
      for (int k = 0; k < QH; ++k) {
        float* dst = hl + l0 + k * RSTEP * SH;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
      float wv[QH][NNMAX], bv[NNMAX];
#pragma unroll
      for (int nt = 0; nt < NNMAX; ++nt) {
        bv[nt] = bbuf[nt];
#pragma unroll
        for (int ks = 0; ks < QH; ++ks) wv[ks][nt] = wcol[nt] ? wbuf[ks][nt] : 0.0f;
      }
      if (sd == 0) {
#pragma unroll
        for (int j = 0; j < DM; ++j) {
          z0[j] = j < d ? ybuf[j] : 0.0f;
          if (norm && j < d) z0[j] = f_div<true>(z0[j] - a.y_mean[j], a.y_std[j]);
        }
      }
      wave_lds_sync();
      const bool last = sd + 1 == ND;
      issue(last ? tile + ustep : tile, last ? 0 : sd + 1);
      flush();
      pend_r = tile_rsrc(a.out, 0);  // later draws of this tile store nothing
      float av[4][QH];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int ks = 0; ks < QH; ++ks) av[mt][ks] = hl[(16 * mt + am) * SH + 4 * ks + ak];
#pragma unroll
      for (int nt = 0; nt < NNMAX; ++nt) {
        if (nt < NN) {
          f32x4v acc[4];
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int ks = 0; ks < QH; ++ks)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
              acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][ks], wv[ks][nt], acc[mt], 0, 0, 0);
          const int n = 16 * nt + am;
          if (n < P) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
              for (int i = 0; i < 4; ++i) tl[(16 * mt + 4 * ak + i) * S + n] = acc[mt][i] + bv[nt];
            }
          }
        }
      }
      wave_lds_sync();
      float z[DM];
#pragma unroll
      for (int j = 0; j < DM; ++j) z[j] = z0[j];
      const float lp = eval_chain<DM, true>(z, tl + lane * S, a) - corr;
      lse_push<true>(m, lacc, lp);
      wave_lds_sync();  // this unit's LDS reads done before the next unit's writes
    }
    const float res = lse_finish<true>(m, lacc, ND);
    if (lane < nr) {
      acc_sum += (double)res;
      nfc += nonfinite1(res);
    }
    pend_v = res;
    pend_r = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
  }
  flush();
  if (a.partials) {
    write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

template <int DM, int QH>
void launch_pdp(const DenseArgs& da, hipStream_t s, int64_t* grid_out) {
  auto kfn = posterior_densep_kernel<DM, QH>;
  const size_t lds = (size_t)(4 * (64 * da.h_lds_stride + 64 * da.c.lds_stride) + 16) * sizeof(float);
  const int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (da.c.ntiles + 3) / 4);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, da);
}

template <int DM>
bool launch_pdp_h(const DenseArgs& da, hipStream_t s, int64_t* g) {
  switch (da.H >> 2) {
    case 1: launch_pdp<DM, 1>(da, s, g); return true;
    case 2: launch_pdp<DM, 2>(da, s, g); return true;
    case 4: launch_pdp<DM, 4>(da, s, g); return true;
  }
  return false;
}

template <int QH, int CM>
void launch_pd1_form(const DenseArgs& da, hipStream_t s, int64_t* grid_out) {
  const int nn = (da.c.P + 15) >> 4;
  const size_t lds = (size_t)(4 * dense1_wave_floats(da.c.P, da.h_lds_stride) + 16) * sizeof(float);
  auto kfn = nn <= 1 ? posterior_dense1_kernel<QH, 1, CM>
                     : (nn == 2 ? posterior_dense1_kernel<QH, 2, CM> : (nn == 3 ? posterior_dense1_kernel<QH, 3, CM>
                                                                                : posterior_dense1_kernel<QH, 4, CM>));
  int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (da.c.ntiles + 3) / 4);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, da);
}

#ifndef NFN_DENSE_HP
template <int QH>
void launch_pd1(const DenseArgs& da, hipStream_t s, int64_t* grid_out) {
  // an alternating program (hpair_types): the compile-time pair bodies, built in their own
  // units (nfn_dense.hip -DNFN_DENSE_HP=sel); C5 with its DenseVariational layer 0.238 ->
  // 0.224 ms (profiles/r04/r04l_hpair_all.log)
  int cm = env_int("NFN_CHAIN_FORM", -1);
  if (cm < 0 && hpair_types(da.c) >= 0) cm = kChainHPair;
  if (cm == kChainHPair && launch_dense1_hpair(hpair_types(da.c), true, da, s, grid_out)) return;
  if (cm == kChainLoop)
    launch_pd1_form<QH, kChainLoop>(da, s, grid_out);  // diag A/B
  else
    launch_pd1_form<QH, kChainPairs>(da, s, grid_out);
}

template <int DM, bool FAST>
void launch_pd(const DenseArgs& da, hipStream_t s, int64_t* grid_out) {
  auto kfn = posterior_dense_kernel<DM, FAST>;
  const size_t lds = (size_t)(4 * (64 * da.h_lds_stride + 64 * da.c.lds_stride) + 16) * sizeof(float);
  const int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (da.c.ntiles + 3) / 4);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, da);
}

template <bool FAST>
bool launch_pd_dm(int dm, const DenseArgs& da, hipStream_t s, int64_t* g) {
  const ChainArgs& a = da.c;
  if constexpr (FAST) {
    if (dm == 1 && a.d == 1 && env_int("NFN_DENSE1", 1) != 0 && da.h_rowstride * 256 < ((int64_t)1 << 31) &&
        a.y_bstride * 256 < ((int64_t)1 << 31)) {
      switch (da.H >> 2) {
        case 1: launch_pd1<1>(da, s, g); return true;
        case 2: launch_pd1<2>(da, s, g); return true;
        case 4: launch_pd1<4>(da, s, g); return true;
        case 8: launch_pd1<8>(da, s, g); return true;
      }
    }
  }
  if constexpr (FAST) {
    // d >= 2, H <= 16: the prefetching pipeline (NFN_DENSEP=0, diag: the synchronous kernel)
    if (dm >= 2 && a.d >= 2 && da.H <= 16 && env_int("NFN_DENSEP", 1) != 0 && da.h_rowstride * 256 < ((int64_t)1 << 31) &&
        a.y_bstride * 256 < ((int64_t)1 << 31)) {
      bool ok = false;
      switch (dm) {
        case 2: ok = launch_pdp_h<2>(da, s, g); break;
        case 4: ok = launch_pdp_h<4>(da, s, g); break;
        case 8: ok = launch_pdp_h<8>(da, s, g); break;
      }
      if (ok) return true;
    }
  }
  switch (dm) {
    case 1: launch_pd<1, FAST>(da, s, g); return true;
    case 2: launch_pd<2, FAST>(da, s, g); return true;
    case 4: launch_pd<4, FAST>(da, s, g); return true;
    case 8: launch_pd<8, FAST>(da, s, g); return true;
  }
  return false;
}

#endif  // NFN_DENSE_HP

// the split-bf16 t GEMM for H = 16, P <= 32 (release default; diag NFN_DENSE_SB=0: fp32 MFMA)
constexpr int kDenseSplitBf16 = 1;
template <int QH, int CM>
void launch_d1_form(const DenseArgs& da, hipStream_t s, int64_t* grid_out) {
  const int nn = (da.c.P + 15) >> 4;
  bool sb = false;
  if constexpr (QH == 4) sb = nn <= 2 && env_int("NFN_DENSE_SB", kDenseSplitBf16) != 0;
  const int wf = sb ? dense1_sb_wave_floats(da.c.P, da.h_lds_stride) : dense1_wave_floats(da.c.P, da.h_lds_stride);
  const size_t lds = (size_t)(4 * QH * nn * 16 + 4 * wf + 16) * sizeof(float);
  auto kfn = nn <= 1 ? chain_dense1_kernel<QH, 1, CM>
                     : (nn == 2 ? chain_dense1_kernel<QH, 2, CM> : (nn == 3 ? chain_dense1_kernel<QH, 3, CM>
                                                                           : chain_dense1_kernel<QH, 4, CM>));
  if constexpr (QH == 4) {
    if (sb) kfn = nn <= 1 ? chain_dense1_kernel<QH, 1, CM, true> : chain_dense1_kernel<QH, 2, CM, true>;
  }
  int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (da.c.ntiles + 3) / 4);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, da);
}

#ifndef NFN_DENSE_HP
template <int QH>
void launch_d1(const DenseArgs& da, size_t /*generic kernel's LDS*/, hipStream_t s, int64_t* grid_out) {
  // an alternating program (hpair_types): the compile-time pair bodies (own units), C2's
  // Dense(H = 16) -> chain 0.445 -> 0.427 ms (profiles/r04/r04l_hpair_all.log)
  int cm = env_int("NFN_CHAIN_FORM", -1);
  if (cm < 0 && hpair_types(da.c) >= 0) cm = kChainHPair;
  if (cm == kChainHPair && launch_dense1_hpair(hpair_types(da.c), false, da, s, grid_out)) return;
#ifdef NFN_DIAG
  if (cm == kStaticProg && (da.c.P + 15) >> 4 == 2 && da.c.prog.K == kStaticK[0] &&
      da.c.prog.types[0] == kStaticTypes[0]) {
    launch_d1_form<QH, kStaticProg>(da, s, grid_out);
    return;
  }
  if (cm == kChainLoop) {
    launch_d1_form<QH, kChainLoop>(da, s, grid_out);
    return;
  }
#endif
  launch_d1_form<QH, kChainPairs>(da, s, grid_out);
}
#endif

#ifndef NFN_DENSE_HP
template <int DM, bool FAST, int NVH>
void launch_d(const DenseArgs& da, size_t lds, hipStream_t s, int64_t* grid_out) {
  auto kfn = chain_dense_kernel<DM, FAST, NVH>;
  const int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (da.c.ntiles + 3) / 4);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, da);
}

template <int DM, bool FAST>
bool launch_d_h(int nvh, const DenseArgs& da, size_t lds, hipStream_t s, int64_t* g) {
  switch (nvh) {
    case 1: launch_d<DM, FAST, 1>(da, lds, s, g); return true;
    case 2: launch_d<DM, FAST, 2>(da, lds, s, g); return true;
    case 4: launch_d<DM, FAST, 4>(da, lds, s, g); return true;
    case 8: launch_d<DM, FAST, 8>(da, lds, s, g); return true;
    case 16: launch_d<DM, FAST, 16>(da, lds, s, g); return true;
  }
  return false;
}

template <bool FAST>
bool launch_d_dm(int dm, int nvh, const DenseArgs& da, size_t lds, hipStream_t s, int64_t* g) {
  const ChainArgs& a = da.c;
  if constexpr (FAST) {
    if (dm == 1 && a.d == 1 && env_int("NFN_DENSE1", 1) != 0 && da.h_rowstride * 256 < ((int64_t)1 << 31) &&
        a.y_bstride * 256 < ((int64_t)1 << 31)) {
      switch (nvh) {
        case 1: launch_d1<1>(da, lds, s, g); return true;
        case 2: launch_d1<2>(da, lds, s, g); return true;
        case 4: launch_d1<4>(da, lds, s, g); return true;
        case 8: launch_d1<8>(da, lds, s, g); return true;
      }
    }
  }
  switch (dm) {
    case 1: return launch_d_h<1, FAST>(nvh, da, lds, s, g);
    case 2: return launch_d_h<2, FAST>(nvh, da, lds, s, g);
    case 4: return launch_d_h<4, FAST>(nvh, da, lds, s, g);
    case 8: return launch_d_h<8, FAST>(nvh, da, lds, s, g);
  }
  return false;
}

#endif  // NFN_DENSE_HP

}  // namespace

#ifdef NFN_DENSE_HP
#define NFN_CAT2(a, b) a##b
#define NFN_CAT(a, b) NFN_CAT2(a, b)
#define NFN_DENSE_HP_FN NFN_CAT(launch_dense1_hpair_, NFN_DENSE_HP)
// This unit: the d = 1 fused Dense kernels (forward and posterior) with the compile-time pair
// bodies of ONE alternating program, sel = NFN_DENSE_HP = 3 * IA + IB (hpair_types).
bool NFN_DENSE_HP_FN(bool post, const DenseArgs& da, hipStream_t s, int64_t* g) {
  constexpr int CM = hpair_form(NFN_DENSE_HP / 3, NFN_DENSE_HP % 3, 1);
  switch (da.H >> 2) {
    case 1: post ? launch_pd1_form<1, CM>(da, s, g) : launch_d1_form<1, CM>(da, s, g); return true;
    case 2: post ? launch_pd1_form<2, CM>(da, s, g) : launch_d1_form<2, CM>(da, s, g); return true;
    case 4: post ? launch_pd1_form<4, CM>(da, s, g) : launch_d1_form<4, CM>(da, s, g); return true;
    case 8: post ? launch_pd1_form<8, CM>(da, s, g) : launch_d1_form<8, CM>(da, s, g); return true;
  }
  return false;
}
#else
bool launch_dense1_hpair(int sel, bool post, const DenseArgs& da, hipStream_t s, int64_t* grid) {
  switch (sel) {
    case 0: return launch_dense1_hpair_0(post, da, s, grid);
    case 1: return launch_dense1_hpair_1(post, da, s, grid);
    case 3: return launch_dense1_hpair_3(post, da, s, grid);
    case 4: return launch_dense1_hpair_4(post, da, s, grid);
  }
  return false;
}

bool launch_dense(bool fast, int dm, int nvh, const DenseArgs& da, size_t lds, hipStream_t s, int64_t* grid) {
  return fast ? launch_d_dm<true>(dm, nvh, da, lds, s, grid) : launch_d_dm<false>(dm, nvh, da, lds, s, grid);
}

bool launch_posterior_dense(bool fast, int dm, const DenseArgs& da, hipStream_t s, int64_t* grid) {
  return fast ? launch_pd_dm<true>(dm, da, s, grid) : launch_pd_dm<false>(dm, da, s, grid);
}
#endif

}  // namespace nfn
