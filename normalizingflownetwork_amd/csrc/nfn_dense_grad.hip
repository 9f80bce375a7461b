// nfn_dense_grad.hip — backward of the fused output Dense layer + flow chain
// (SURVEY.md §8(f) rows 1 + 2 together): what Keras autodiff computes through
// Dense(P) (MaximumLikelihoodNNEstimator.py:37-44) and the layer's log_prob when the
// reference trains (BaseEstimator.py:19-31), without t ever being written:
//   t = h W + b                          (v_mfma_f32_16x16x4_f32, exact fp32)
//   dt = g * d logp / d t                (the closed-form chain backward, grad_sample)
//   dh = dt W^T                          (MFMA, per tile, streamed out)
//   dW = sum_b h_b^T dt_b, db = sum_b dt_b   (MFMA accumulated in registers across the
//                                        wave's tiles; fixed-order workgroup and grid
//                                        reductions: bitwise deterministic)
// Persistent grid, every wave owns a stream of 64-sample tiles; per wave LDS: the h
// tile (odd stride SH), the t / dt tile (odd stride S) and the flow inputs z_k.
#include "nfn_grad_device.h"
#include "nfn_bf16.h"
#include "nfn_launch.h"

namespace nfn {
namespace {

template <int DM, bool FAST, int MH, int NN>
__global__ void __launch_bounds__(kMaxBlock) chain_dense_grad_kernel(DenseGradArgs g) {
  const DenseArgs& da = g.da;
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int nwave = blockDim.x >> 6;
  const int H = da.H;
  const int QH = H >> 2;
  const int SH = da.h_lds_stride;  // odd
  const int S = a.lds_stride;      // odd, >= P
  const int P = a.P;
  const int d = a.d;
  const int K = a.prog.K;
  constexpr int NP = NN * 16;
  constexpr int HP = MH * 16;  // H padded to the 16-row M tiles of dW
  // LDS: [W: H x NP, zero-padded] [per wave: h 64 x SH | t 64 x S | z_k K*d*64] [reduction H*P+P]
  float* wl = lds;
  const int wslot = 64 * SH + 64 * S + K * d * 64;
  float* hl = lds + H * NP + wid * wslot;
  float* tl = hl + 64 * SH;
  float* zh = tl + 64 * S + lane;
  float* rl = lds + H * NP + nwave * wslot;
  for (int i = tid; i < H * NP; i += blockDim.x) {
    const int k = i / NP, n = i - (i / NP) * NP;
    wl[i] = n < P ? da.W[(int64_t)k * P + n] : 0.0f;
  }
  for (int i = tid; i < H * P + P; i += blockDim.x) rl[i] = 0.0f;
  __syncthreads();
  const int am = lane & 15, ak = lane >> 4;
  const int64_t hs = da.h_rowstride;
  const int64_t u0 = (int64_t)blockIdx.x * nwave + wid;
  const int64_t ustep = (int64_t)gridDim.x * nwave;
  float corr = 0.0f;
  if (a.y_mean) {
    for (int j = 0; j < d; ++j) corr += f_log<FAST>(a.y_std[j]);
  }
  f32x4v dw[MH][NN];
#pragma unroll
  for (int mh = 0; mh < MH; ++mh)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) dw[mh][nt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  float db = 0.0f;  // lane p < P: column p of sum_b dt_b

  // the next tile's h rows, y and upstream gradient are prefetched into registers
  // (non-temporal) while the current tile runs; QH = H / 4 <= 4 * MH float4 per lane
  const int r0 = lane / QH, c4 = lane - (lane / QH) * QH, rstep = 64 / QH;
  float4 hbuf[4 * MH];
  float ybuf[DM];
  float gbuf = 1.0f;
  auto issue = [&](int64_t tile) {
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
#pragma unroll
    for (int k = 0; k < 4 * MH; ++k) {
      const int r = r0 + k * rstep;
      hbuf[k] = (k < QH && r < nr) ? load_row4<true>(da.h + (b0 + r) * hs + 4 * c4) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < DM; ++j) ybuf[j] = (lane < nr && j < d) ? a.y[(b0 + lane) * a.y_bstride + j] : 0.0f;
    gbuf = (lane < nr && g.g_out) ? g.g_out[b0 + lane] : 1.0f;
  };
  if (u0 < a.ntiles) issue(u0);
  for (int64_t tile = u0; tile < a.ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int nr = (int)min((int64_t)64, a.B - b0);
    // 1. h tile -> LDS (rows past B are zero: they add nothing to dW)
#pragma unroll
    for (int k = 0; k < 4 * MH; ++k) {
      if (k < QH) {
        float* dst = hl + (r0 + k * rstep) * SH + 4 * c4;
        dst[0] = hbuf[k].x;
        dst[1] = hbuf[k].y;
        dst[2] = hbuf[k].z;
        dst[3] = hbuf[k].w;
      }
    }
    float z[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z[j] = ybuf[j];
      if (a.y_mean && j < d) z[j] = f_div<FAST>(z[j] - a.y_mean[j], a.y_std[j]);
    }
    const float gl = gbuf;
    wave_lds_sync();
    if (tile + ustep < a.ntiles) issue(tile + ustep);
    // 2. t = h W + b
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      f32x4v acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      for (int ks = 0; ks < QH; ++ks) {
        const float bv = wl[(4 * ks + ak) * NP + 16 * nt + am];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(hl[(16 * mt + am) * SH + 4 * ks + ak], bv, acc[mt], 0, 0, 0);
      }
      const int n = 16 * nt + am;
      if (n < P) {
        const float bn = da.bias ? da.bias[n] : 0.0f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) tl[(16 * mt + 4 * ak + i) * S + n] = acc[mt][i] + bn;
      }
    }
    wave_lds_sync();
    // 3. the chain forward + reverse per lane: the t row becomes g * d logp / d t
    {
      float* row = tl + lane * S;
      if (lane < nr) {
        float adj[DM];
        const float lp = grad_sample<DM, FAST>(z, row, zh, 64, a, gl, adj) - corr;
        if (a.out) __builtin_nontemporal_store(lp, a.out + b0 + lane);
        if (g.grad_y) {
#pragma unroll
          for (int j = 0; j < DM; ++j)
            if (j < d) g.grad_y[(b0 + lane) * d + j] = a.y_std ? f_div<FAST>(adj[j], a.y_std[j]) : adj[j];
        }
      } else {
        for (int p = 0; p < S; ++p) row[p] = 0.0f;  // rows past B: no gradient
      }
    }
    wave_lds_sync();
    // 4. dh = dt W^T (k = p over NP, B[p][h] = W[h][p] from the zero-padded LDS copy)
    if (g.grad_h) {
      for (int nh = 0; nh < MH; ++nh) {
        f32x4v acc[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
        const int hc = 16 * nh + am;
#pragma unroll
        for (int ks = 0; ks < 4 * NN; ++ks) {
          const int p = 4 * ks + ak;
          const float bv = hc < H ? wl[hc * NP + p] : 0.0f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const float av = p < P ? tl[(16 * mt + am) * S + p] : 0.0f;
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[mt], 0, 0, 0);
          }
        }
        if (hc < H) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 16 * mt + 4 * ak + i;
              if (r < nr) __builtin_nontemporal_store(acc[mt][i], g.grad_h + (b0 + r) * g.gh_rowstride + hc);
            }
        }
      }
    }
    // 5. dW += h^T dt (k = the tile's 64 samples), db += column sums of dt
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int r = 4 * ks + ak;
#pragma unroll
      for (int mh = 0; mh < MH; ++mh) {
        const int hr = 16 * mh + am;
        const float av = hr < H ? hl[r * SH + hr] : 0.0f;
#pragma unroll
        for (int nt = 0; nt < NN; ++nt) {
          const int p = 16 * nt + am;
          const float bv = p < P ? tl[r * S + p] : 0.0f;
          dw[mh][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, dw[mh][nt], 0, 0, 0);
        }
      }
    }
    if (NN <= 2) {  // P <= 32: two lanes per column, 32 rows each, combined across the halves
      const int p = lane & 31, r0h = (lane >> 5) * 32;
      float cs = 0.0f;
      if (p < P) {
#pragma unroll 8
        for (int r = 0; r < 32; ++r) cs += tl[(r0h + r) * S + p];
      }
      cs += __shfl_xor(cs, 32);
      if (lane < P) db += cs;
    } else if (lane < P) {
      float cs = 0.0f;
      for (int r = 0; r < 64; ++r) cs += tl[r * S + lane];
      db += cs;
    }
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
  if (g.part == nullptr) return;  // no grad_W / grad_b requested (uniform: every thread returns)
  // workgroup reduction in wave order (deterministic), then one partial per workgroup
  for (int w = 0; w < nwave; ++w) {
    if (wid == w) {
#pragma unroll
      for (int mh = 0; mh < MH; ++mh)
#pragma unroll
        for (int nt = 0; nt < NN; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int hr = 16 * mh + 4 * ak + i, p = 16 * nt + am;  // C layout: row 4 ak + i, column am
            if (hr < H && p < P) rl[hr * P + p] += dw[mh][nt][i];
          }
      if (lane < P) rl[H * P + lane] += db;
    }
    __syncthreads();
  }
  float* out = g.part + (int64_t)blockIdx.x * (H * P + P);
  for (int i = tid; i < H * P + P; i += blockDim.x) out[i] = rl[i];
  (void)HP;
}

// d = 1, fast math, H = 16 MH (MH in {1, 2}), P <= 16 NN: the same backward with
// every operand placed for the matrix cores and chain_dense1_kernel's memory pipeline.
// Per 64-sample wave tile (all MFMAs v_mfma_f32_16x16x4_f32, exact fp32):
//   * h arrives by b128 buffer loads (lane (am, ak): h[16 mt + am][16 j + 4 ak .. + 3])
//     and goes to LDS (row stride SH = H + 4: conflict-free b128 writes), to be read
//     back as the A fragments of t = h W (in chain_dense1_kernel's hidden-unit order:
//     t is bitwise the forward kernel's) and, transposed, as those of dW = h^T dt
//     (contraction over samples in the order s = 16 kq + 4 ak + i, so that dt is read
//     as b128), kept in registers across the chain; the W fragments of both GEMMs
//     that read W (t = h W, dh^T = W dt^T) stay in registers for the whole launch;
//   * t = h W + b leaves the matrix cores as b128 writes into a column-major t tile
//     (stride kCS, overlaying the dead h rows); the chain backward runs per lane
//     (grad1_packed on the column stride), turning t into dt in place;
//   * dh^T = W dt^T (contraction over p in the order 16 (ks/4) + 4 ak + ks % 4: the
//     two 16-lane halves of each ds_read_b32 group land on disjoint banks) — each lane
//     then holds 4 consecutive hidden units of one sample: dh leaves as b128 stores;
//   * dW += h^T dt, with db's column sums taken from the same b128 dt reads (VALU
//     adds, lanes of one column combined once at the end).
// Per wave LDS: the t tile ((P + 2) columns, the packed reverse pass reads up to two
// past the last block) and the flow inputs z_k.  Every workgroup writes one partial
// [dW | db], summed across waves in wave order: bitwise deterministic.
// AB (diagnostic builds only): bit 0 replaces the dh^T MFMAs, bit 1 the dW MFMAs, by a VALU
// touch of the same operands — the ceiling any faster form of those two GEMMs could reach.
template <int MH, int NN, int CM = kChainLoop, int AB = 0>
__global__ void __launch_bounds__(kMaxBlock) chain_dense1_grad_kernel(DenseGradArgs g) {
  const DenseArgs& da = g.da;
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  constexpr int H = 16 * MH;
  constexpr int QH = 4 * MH;
  constexpr int SH = H + 4;  // h rows in LDS: 16-byte aligned, == 4 mod 8 (see above)
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwave = blockDim.x >> 6;
  const int P = a.P;
  const int K = a.prog.K;
  const int wfl = dense1_grad_wave_floats(P, SH, K);
  float* tl = lds + wid * wfl;  // t / dt tile, column-major; the h rows overlay it
  float* hl = tl;
  float* zh = tl + (P + 2) * kCS + lane;
  const int am = lane & 15, ak = lane >> 4;

  // W fragments: t GEMM B[k = hidden(ks)][n = p] and dh GEMM A[m = hidden][k = p(ks)]
  float wB[QH][NN], wA[MH][4 * NN], bn[NN];
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    const int p = 16 * nt + am;
    bn[nt] = (p < P && da.bias) ? da.bias[p] : 0.0f;
#pragma unroll
    for (int ks = 0; ks < QH; ++ks) wB[ks][nt] = p < P ? da.W[(4 * ks + ak) * P + p] : 0.0f;
  }
#pragma unroll
  for (int mh = 0; mh < MH; ++mh)
#pragma unroll
    for (int ks = 0; ks < 4 * NN; ++ks) {
      const int p = 16 * (ks >> 2) + 4 * ak + (ks & 3);
      wA[mh][ks] = p < P ? da.W[(16 * mh + am) * P + p] : 0.0f;
    }

  const int64_t hs = da.h_rowstride;
  const int64_t ghs = g.gh_rowstride;
  const int64_t ntiles = a.ntiles;
  const int64_t u0 = (int64_t)blockIdx.x * nwave + wid;
  const int64_t ustep = (int64_t)gridDim.x * nwave;
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const bool trainable = a.trainable != 0;
  const uint32_t types = a.prog.types[0];
  // loop-invariant byte offsets (the host guarantees 64 rows span < 2 GiB)
  const int yoff = lane * (int)a.y_bstride * 4;
  const int hoff = (am * (int)hs + 4 * ak) * 4;      // + mt * 16 rows + j * 16 floats
  const int hmt = 16 * (int)hs * 4;
  const int ghoff = (am * (int)ghs + 4 * ak) * 4;    // dh: row 16 mt + am, hidden 16 mh + 4 ak
  const int ghmt = 16 * (int)ghs * 4;

  float4 hb[4][MH];
  float ybuf, gbuf;
  auto issue = [&](int64_t tile) {
    if (diag_ablate_loads(a)) tile = u0;  // diagnostic: compute-only timing (the first tile re-read)
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    const auto rg = tile_rsrc(g.g_out ? g.g_out + b0c : a.y, g.g_out ? nr * 4 : 0);
    gbuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, lane * 4, 0, 0));
    const auto rh = tile_rsrc(da.h + b0c * hs, nr > 0 ? ((nr - 1) * hs + H) * 4 : 0);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < MH; ++j)
        hb[mt][j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, hoff, mt * hmt + 64 * j, kNT));
  };

  f32x4v dw[MH][NN];
  float db[NN];
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    db[nt] = 0.0f;
#pragma unroll
    for (int mh = 0; mh < MH; ++mh) dw[mh][nt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  }

  issue(u0);
  for (int64_t tile = u0; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    // 1. h rows -> LDS (row-major); read back: the A fragments of t = h W (hidden units
    // in chain_dense1_kernel's order, so t is bitwise the forward kernel's) and, transposed,
    // those of dW (kept in registers across the chain)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < MH; ++j)
        *reinterpret_cast<float4*>(hl + (16 * mt + am) * SH + 16 * j + 4 * ak) = hb[mt][j];
    const float z0 = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
    const float gl = g.g_out ? gbuf : 1.0f;
    wave_lds_sync();
    issue(tile + ustep);  // the next tile's loads (hb is free once in LDS)
    float av[4][QH], hA[MH][16];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int ks = 0; ks < QH; ++ks) av[mt][ks] = hl[(16 * mt + am) * SH + 4 * ks + ak];
#pragma unroll
    for (int mh = 0; mh < MH; ++mh)
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) hA[mh][ks] = hl[(16 * (ks >> 2) + 4 * ak + (ks & 3)) * SH + 16 * mh + am];
    wave_lds_sync();  // every h read done before the t tile overwrites the rows
    // 2. t = h W + b
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      f32x4v acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < QH; ++ks)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][ks], wB[ks][nt], acc[mt], 0, 0, 0);
      if (16 * nt + am < P) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          *reinterpret_cast<f32x4v*>(tl + (16 * nt + am) * kCS + 16 * mt + 4 * ak) = acc[mt] + bn[nt];
      }
    }
    wave_lds_sync();
    // 3. the chain forward + reverse per lane: the t column entries become g * d logp / d t
    float adj, z = z0;
    float lp;
    if constexpr (CM == kStaticProg)
      lp = grad1_static<kStaticTypes[0], kStaticK[0], kCS>(z, tl + lane, zh, 64, P, trainable, gl, a.out != nullptr,
                                                           adj) - corr;
    else if constexpr (CM >= kChainHPair && (CM - kChainHPair) / 9 == 2)  // flow inputs in registers
      lp = grad1_hpairs_regs<((CM - kChainHPair) % 9) / 3, (CM - kChainHPair) % 3, kCS>(
               z, tl + lane, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    else if constexpr (CM >= kChainHPair)
      lp = grad1_hpairs<((CM - kChainHPair) % 9) / 3, (CM - kChainHPair) % 3, kCS>(
               z, tl + lane, zh, 64, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    else if constexpr (CM == kChainPairs)
      lp = grad1_pairs<kCS>(z, tl + lane, zh, 64, types, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    else
      lp = grad1_packed<kCS>(z, tl + lane, zh, 64, types, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    if (nr < 64 && lane >= nr) {  // rows past B carry no gradient
      for (int p = 0; p < P; ++p) tl[p * kCS + lane] = 0.0f;
    }
    {
      const auto ro = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, lp), ro, lane * 4, 0, kNT);
      const auto rdy = tile_rsrc(g.grad_y && nr > 0 ? g.grad_y + b0 : g.grad_y, g.grad_y ? nr * 4 : 0);
      const float gy = norm ? f_div<true>(adj, ystd) : adj;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, gy), rdy, lane * 4, 0, kNT);
    }
    wave_lds_sync();
    // 4. dh^T = W dt^T: lane (am, ak) ends with dh[16 mt + am][16 mh + 4 ak .. + 3]
    {
      const auto rdh = tile_rsrc(g.grad_h && nr > 0 ? g.grad_h + b0 * ghs : g.grad_h,
                                 g.grad_h && nr > 0 ? ((nr - 1) * ghs + H) * 4 : 0);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        float bv[4 * NN];
#pragma unroll
        for (int ks = 0; ks < 4 * NN; ++ks) {
          const int p = 16 * (ks >> 2) + 4 * ak + (ks & 3);
          bv[ks] = p < P ? tl[p * kCS + 16 * mt + am] : 0.0f;
        }
#pragma unroll
        for (int mh = 0; mh < MH; ++mh) {
          f32x4v acc = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int ks = 0; ks < 4 * NN; ++ks) {
            if constexpr (AB & 1)
              acc[ks & 3] = fmaf(wA[mh][ks], bv[ks], acc[ks & 3]);
            else
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[mh][ks], bv[ks], acc, 0, 0, 0);
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc), rdh, ghoff, mt * ghmt + 64 * mh, kNT);
        }
      }
    }
    // 5. dW += h^T dt (contraction over the tile's samples), db += the same dt values
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      const bool col = 16 * nt + am < P;
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        f32x4v q = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
        if (col) q = *reinterpret_cast<const f32x4v*>(tl + (16 * nt + am) * kCS + 16 * kq + 4 * ak);
        db[nt] += (q[0] + q[1]) + (q[2] + q[3]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int mh = 0; mh < MH; ++mh)
            if constexpr ((AB & 2) != 0)
              dw[mh][nt][i] = fmaf(hA[mh][4 * kq + i], q[i], dw[mh][nt][i]);
            else
              dw[mh][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(hA[mh][4 * kq + i], q[i], dw[mh][nt], 0, 0, 0);
      }
    }
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
  if (g.part == nullptr) return;  // no grad_W / grad_b requested (uniform: every thread returns)
  // db: the four lanes of a column (ak = 0..3) combined in a fixed order
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    db[nt] += __shfl_xor(db[nt], 16);
    db[nt] += __shfl_xor(db[nt], 32);
  }
  // each wave's [dW | db] into its own LDS region, then summed in wave order
  const int nWb = H * P + P;
  __syncthreads();
  float* mine = lds + wid * wfl;
#pragma unroll
  for (int mh = 0; mh < MH; ++mh)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hr = 16 * mh + 4 * ak + i, p = 16 * nt + am;  // C layout: row 4 ak + i, column am
        if (p < P) mine[hr * P + p] = dw[mh][nt][i];
      }
#pragma unroll
  for (int nt = 0; nt < NN; ++nt)
    if (ak == 0 && 16 * nt + am < P) mine[H * P + 16 * nt + am] = db[nt];
  __syncthreads();
  float* out = g.part + (int64_t)blockIdx.x * nWb;
  for (int i = tid; i < nWb; i += blockDim.x) {
    float s = lds[i];
    for (int w = 1; w < nwave; ++w) s += lds[w * wfl + i];
    out[i] = s;
  }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 weight-gradient GEMMs (the release form; diag NFN_DGRAD_SB=0 runs the f32
// kernel): chain_dense1_grad_kernel (H = 16,
// P <= 32) with dh^T = W dt^T and dW += h^T dt on v_mfma_f32_16x16x32_bf16 instead of
// v_mfma_f32_16x16x4_f32 (t = h W stays f32: the chain amplifies t's rounding, and a
// split-bf16 t — a few ulp, not bitwise numpy's / the forward kernel's — put one
// ill-conditioned sample of test_dense_grad_matches_oracle 5.4x over its dh bound,
// profiles/r06/r06b_densetests.log).
// Why: the f32 MFMA runs at the f32 vector rate and holds the SIMD's vector issue for all of
// its 32 cycles, so the GEMMs serialise with the chain's VALU work
// (profiles/r02/r02j_mfma_valu_coexec.log: 0.989 of the sum); a 16x16x32 bf16 MFMA takes 16
// cycles and holds vector issue for 8 of them.
// Numerics: every operand x is split EXACTLY into three bf16 parts, x = x1 + x2 + x3
// (v_cvt_pk_bf16_f32 round-to-nearest-even, residuals exact in fp32: x1 holds 8 significant
// bits, x2 the next 8, x3 the rest), and each product keeps the six terms x_i y_j with
// i + j <= 4; the dropped ones (x2 y3, x3 y2, x3 y3) are below 2^-23 |x y|: fp32-level
// products, accumulated in fp32 by the matrix cores.
// Per 64-sample wave tile, after the chain (which is the f32 kernel's, on the f32 t tile):
//   * each lane re-reads ITS sample's dt row; db's column sums come from the f32 tile;
//   * h's transposed A fragments (read from the LDS h rows before the chain, as the f32
//     kernel keeps them) are split; dW's K-slot j of lane group ak is sample
//     32 kc + 16 (j >> 2) + 4 ak + (j & 3) (conflict-free transposed reads below);
//   * one dt part at a time (x1, x2, x3, each split off the running residual), the part goes
//     to a bf16 plane [sample][32] over the dead f32 tile (16-byte chunk c of row s at chunk
//     c ^ swz(s), swz = a bit swap of (s >> 2) & 3: conflict-free row reads and transposed
//     reads), and every product with it runs: dh^T += W_i dt_j (B = plane rows,
//     ds_read_b128; A = W's parts, registers) and dW += h_i^T dt_j (B = the plane read
//     transposed, ds_read_b64_tr_b16).
// LDS per wave: the f32 kernel's (the plane needs 64 x 16 dwords).
// two transposed 4 x 16 reads (ds_read_b64_tr_b16 at two LDS addresses) as one fragment
__device__ __forceinline__ bf16x8v tr_frag(const float* base0, const float* base1) {
  const s16x4v x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4v*)((__attribute__((address_space(3))) float*)base0));
  const s16x4v y = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4v*)((__attribute__((address_space(3))) float*)base1));
  const s16x4v v[2] = {x, y};
  return __builtin_bit_cast(bf16x8v, v);
}
// The bf16 planes' 16-byte chunk swizzle (chunk c of row r sits at chunk c ^ swz(r)): bit 0 =
// bit 1 of the row, bit 1 = bit 2 of the row.  Checked exhaustively against the gfx950 LDS
// lane groups (MI355X_MICROARCH.md, LDS table): conflict-free ds_read_b128 row reads (rows
// 16 mt + am, chunk ak; the W parts' rows am), ds_read_b64_tr_b16 transposed reads (rows
// 4 g + q of a half-wave: the two groups in different chunk pairs) and ds_write_b128 row
// writes (one row per lane); rows r and r + 16 share the swizzle.
__device__ __forceinline__ int dt_swz(int row) { return ((row >> 1) & 1) | ((row >> 1) & 2); }

constexpr int kSbDRow = 16;   // dwords per dt-plane row (32 bf16)
// a wave's LDS: chain_dense1_grad_kernel's (h rows / t tile + flow inputs) or the three dt planes
__host__ __device__ inline int dense1_grad_sb_wave_floats(int P, int K) {
  return std::max(dense1_grad_wave_floats(P, 20, K), 3 * 64 * kSbDRow);
}
constexpr int kSbWRow = 16;  // dwords per hidden unit of the W parts (16 pairs of p, chunks swizzled as the planes)
constexpr int kSbWFloats = 3 * 16 * kSbWRow + 32;  // the workgroup's W bf16 parts [part][hidden][pairs of p] and bias
// The programs the fused Dense backward runs as compile-time blocks with the parameter-scalar
// cache (SP indexes them): C2's (planar, radial) x 5, and the estimator's default
// NormalizingFlowNetwork(n_dims, n_flows=10), radial x 10 (NormalizingFlowNetwork.py:10-17).
constexpr uint32_t kCacheTypes[] = {0x44444u, 0x55555u};
constexpr int kCacheK[] = {10, 10};
constexpr int kNumCached = 2;

// CM: the chain form.  The compile-time C2 program (diag kStaticProg, grad1_static) and its
// parameter-scalar cache (kStaticCache, grad1_static_cache: the release form for C2's program;
// diag kStaticCacheX, the cache bitwise grad1_static's) run at 2 waves per SIMD (the static
// form spills at 3), every other form at 3.
template <int NN, int CM = kChainPairs, int SP = 0>
__global__ void __launch_bounds__(kMaxBlock, (CM == kStaticCache || CM == kStaticCacheX || CM == kStaticProg) ? 2 : 3)
    chain_dense1_grad_sb_kernel(DenseGradArgs g) {
  static_assert(NN == 1 || NN == 2, "P <= 32");
  const DenseArgs& da = g.da;
  const ChainArgs& a = da.c;
  extern __shared__ float lds[];
  constexpr int H = 16;
  constexpr int QH = 4;
  constexpr int SH = H + 4;  // h rows in LDS (as chain_dense1_grad_kernel)
  constexpr int NP = 16 * NN;
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwave = blockDim.x >> 6;
  const int P = a.P;
  const int K = a.prog.K;
  const int wfl = dense1_grad_sb_wave_floats(P, K);  // the f32 kernel's region, or the three dt planes
  float* const wb = lds + wid * wfl;
  float* const tl = wb;  // t / dt tile, column-major; the h rows overlay it, then the dt plane
  float* const hl = wb;
  float* const zh = tl + (P + 2) * kCS + lane;
  const int am = lane & 15, ak = lane >> 4;

  // t = h W (f32 MFMA, bitwise chain_dense1_kernel's t): B fragments W[hidden 4 ks + ak][p]
  // (registers); the bias from the workgroup's LDS copy (after the W parts), read per tile
  float wB[QH][NN];
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    const int p = 16 * nt + am;
#pragma unroll
    for (int ks = 0; ks < QH; ++ks) wB[ks][nt] = p < P ? da.W[(4 * ks + ak) * P + p] : 0.0f;
  }
  float* const bl = lds + nwave * wfl + 3 * 16 * kSbWRow;
  for (int i = tid; i < NP; i += blockDim.x) bl[i] = (i < P && da.bias) ? da.bias[i] : 0.0f;
  // dh^T = W dt^T (bf16 parts): A fragments W_i[hidden am][p = 8 ak + j], i = 1, 2, 3, in the
  // workgroup's LDS after the waves' regions ([part][hidden][kSbWRow]), read per use
  uint32_t* const wpl = reinterpret_cast<uint32_t*>(lds + nwave * wfl);
  for (int i = tid; i < 16 * 16; i += blockDim.x) {
    const int hh = i >> 4, q = i & 15, p = 2 * q;
    const float x0 = p < P ? da.W[hh * P + p] : 0.0f, x1 = p + 1 < P ? da.W[hh * P + p + 1] : 0.0f;
    uint32_t w1, w2, w3;
    split3_pk(x0, x1, w1, w2, w3);
    const int at = hh * kSbWRow + 4 * ((q >> 2) ^ dt_swz(hh)) + (q & 3);
    wpl[at] = w1;
    wpl[16 * kSbWRow + at] = w2;
    wpl[32 * kSbWRow + at] = w3;
  }
  __syncthreads();
  const int64_t hs = da.h_rowstride;
  const int64_t ghs = g.gh_rowstride;
  const int64_t ntiles = a.ntiles;
  const int64_t u0 = (int64_t)blockIdx.x * nwave + wid;
  const int64_t ustep = (int64_t)gridDim.x * nwave;
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const bool trainable = a.trainable != 0;
  const uint32_t types = a.prog.types[0];
  const int yoff = lane * (int)a.y_bstride * 4;
  const int hoff = (am * (int)hs + 4 * ak) * 4;
  const int hmt = 16 * (int)hs * 4;
  const int ghoff = (am * (int)ghs + 4 * ak) * 4;
  const int ghmt = 16 * (int)ghs * 4;
  // transposed reads: lane 4 q + p' of group ak supplies row q, columns 4 p' .. 4 p' + 3
  const int trq = (lane & 15) >> 2, trp = lane & 3;
  const int swz_w = dt_swz(am);  // plane-row reads: rows 16 mt + am share their low 4 bits with am
  const int swz_l = dt_swz(lane);

  float4 hb[4];
  float ybuf, gbuf;
  auto issue = [&](int64_t tile) {
    if (diag_ablate_loads(a)) tile = u0;  // diagnostic: compute-only timing (the first tile re-read)
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    const auto rg = tile_rsrc(g.g_out ? g.g_out + b0c : a.y, g.g_out ? nr * 4 : 0);
    gbuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, lane * 4, 0, 0));
    const auto rh = tile_rsrc(da.h + b0c * hs, nr > 0 ? ((nr - 1) * hs + H) * 4 : 0);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      hb[mt] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, hoff, mt * hmt, kNT));
  };

  f32x4v dw[NN];
  float db[NN];
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    db[nt] = 0.0f;
    dw[nt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  }

  issue(u0);
  for (int64_t tile = u0; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    // 1. h rows -> LDS (row-major); read back: t = h W's A fragments and, transposed, dW's
    //    h[sample 32 kc + 16 (j >> 2) + 4 ak + (j & 3)][hidden am] (kept in registers)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) *reinterpret_cast<float4*>(hl + (16 * mt + am) * SH + 4 * ak) = hb[mt];
    const float z0 = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
    const float gl = g.g_out ? gbuf : 1.0f;
    wave_lds_sync();
    issue(tile + ustep);  // the next tile's loads (hb is free once in LDS)
    float av[4][QH], hA[16];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int ks = 0; ks < QH; ++ks) av[mt][ks] = hl[(16 * mt + am) * SH + 4 * ks + ak];
#pragma unroll
    for (int j = 0; j < 16; ++j) hA[j] = hl[(32 * (j >> 3) + 16 * ((j >> 2) & 1) + 4 * ak + (j & 3)) * SH + am];
    wave_lds_sync();  // every h read done before the t tile overwrites the rows
    // 2. t = h W + b (f32 MFMA)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      f32x4v acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < QH; ++ks)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][ks], wB[ks][nt], acc[mt], 0, 0, 0);
      if (16 * nt + am < P) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          *reinterpret_cast<f32x4v*>(tl + (16 * nt + am) * kCS + 16 * mt + 4 * ak) = acc[mt] + bl[16 * nt + am];
      }
    }
    wave_lds_sync();
    // 3. the chain forward + reverse per lane: the t column entries become g * d logp / d t
    float adj, z = z0;
    float lp;
    if constexpr (CM == kStaticCache || CM == kStaticCacheX)
      lp = grad1_static_cache<kCacheTypes[SP], kCacheK[SP], kCS, CM == kStaticCache>(z, tl + lane, P, trainable, gl,
                                                                                      a.out != nullptr, adj) - corr;
    else if constexpr (CM == kStaticProg)
      lp = grad1_static<kStaticTypes[0], kStaticK[0], kCS>(z, tl + lane, zh, 64, P, trainable, gl, a.out != nullptr,
                                                            adj) - corr;
    else if constexpr (CM >= kChainHPair)
      lp = grad1_hpairs<((CM - kChainHPair) % 9) / 3, (CM - kChainHPair) % 3, kCS>(
               z, tl + lane, zh, 64, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    else if constexpr (CM == kChainPairs)
      lp = grad1_pairs<kCS>(z, tl + lane, zh, 64, types, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    else
      lp = grad1_packed<kCS>(z, tl + lane, zh, 64, types, K, P, trainable, gl, a.out != nullptr, adj) - corr;
    {
      const auto ro = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, lp), ro, lane * 4, 0, kNT);
      const auto rdy = tile_rsrc(g.grad_y && nr > 0 ? g.grad_y + b0 : g.grad_y, g.grad_y ? nr * 4 : 0);
      const float gy = norm ? f_div<true>(adj, ystd) : adj;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, gy), rdy, lane * 4, 0, kNT);
    }
    // 4. this lane's dt row and db's column sums, from the f32 tile (rows past B carry no
    //    gradient: zeroed first, as in chain_dense1_grad_kernel)
    if (nr < 64 && lane >= nr) {
      for (int p = 0; p < P; ++p) tl[p * kCS + lane] = 0.0f;
    }
    float v[32];  // the dt row
#pragma unroll
    for (int p = 0; p < 32; ++p) v[p] = (p < NP && p < P) ? tl[p * kCS + lane] : 0.0f;
    wave_lds_sync();  // the chain's dt writes (other lanes' columns) are visible to the column reads
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      const bool col = 16 * nt + am < P;
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        f32x4v q = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
        if (col) q = *reinterpret_cast<const f32x4v*>(tl + (16 * nt + am) * kCS + 16 * kq + 4 * ak);
        db[nt] += (q[0] + q[1]) + (q[2] + q[3]);
      }
    }
    // 5. dt's three bf16 parts -> three planes [sample][32] over the dead f32 tile (16-byte
    //    chunk c of row s at chunk c ^ swz(s))
    wave_lds_sync();  // every f32 read done before the planes overwrite the tile
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t d1[4], d2[4], d3[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split3_pk(v[8 * c + 2 * q], v[8 * c + 2 * q + 1], d1[q], d2[q], d3[q]);
      float* row = wb + lane * kSbDRow + 4 * (c ^ swz_l);
      *reinterpret_cast<u32x4v*>(row) = u32x4v{d1[0], d1[1], d1[2], d1[3]};
      *reinterpret_cast<u32x4v*>(row + 64 * kSbDRow) = u32x4v{d2[0], d2[1], d2[2], d2[3]};
      *reinterpret_cast<u32x4v*>(row + 128 * kSbDRow) = u32x4v{d3[0], d3[1], d3[2], d3[3]};
    }
    wave_lds_sync();
    // 6. dh^T = W dt^T (B = plane rows): lane (am, ak) ends with dh[16 mt + am][4 ak .. 4 ak + 3];
    //    the six terms small first: (3,1) (2,2) (1,3) (2,1) (1,2) (1,1)
    {
      const auto rdh = tile_rsrc(g.grad_h && nr > 0 ? g.grad_h + b0 * ghs : g.grad_h,
                                 g.grad_h && nr > 0 ? ((nr - 1) * ghs + H) * 4 : 0);
      const uint32_t* wr = wpl + am * kSbWRow + 4 * (ak ^ swz_w);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const float* row = wb + (16 * mt + am) * kSbDRow + 4 * (ak ^ swz_w);
        const bf16x8v d1 = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(row));
        const bf16x8v d2 = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(row + 64 * kSbDRow));
        const bf16x8v d3 = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(row + 128 * kSbDRow));
        const bf16x8v w1 = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(wr));
        const bf16x8v w2 = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(wr + 16 * kSbWRow));
        const bf16x8v w3 = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4v*>(wr + 32 * kSbWRow));
        f32x4v acc = mfma_bf16(w3, d1, f32x4v{0.0f, 0.0f, 0.0f, 0.0f});
        acc = mfma_bf16(w2, d2, acc);
        acc = mfma_bf16(w1, d3, acc);
        acc = mfma_bf16(w2, d1, acc);
        acc = mfma_bf16(w1, d2, acc);
        acc = mfma_bf16(w1, d1, acc);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc), rdh, ghoff, mt * ghmt, kNT);
      }
    }
    // 7. dW += h^T dt: A = h's parts (split from the transposed reads kept since step 1),
    //    B = the planes read transposed [8 samples][16 columns]
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      uint32_t x1[4], x2[4], x3[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split3_pk(hA[8 * kc + 2 * q], hA[8 * kc + 2 * q + 1], x1[q], x2[q], x3[q]);
      const bf16x8v h1 = frag8(x1[0], x1[1], x1[2], x1[3]);
      const bf16x8v h2 = frag8(x2[0], x2[1], x2[2], x2[3]);
      const bf16x8v h3 = frag8(x3[0], x3[1], x3[2], x3[3]);
      const int r = 32 * kc + 4 * ak + trq;  // r and r + 16 share the swizzle
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) {
        const float* bp = wb + r * kSbDRow + 4 * ((2 * nt + (trp >> 1)) ^ dt_swz(r)) + 2 * (trp & 1);
        const bf16x8v e1 = tr_frag(bp, bp + 16 * kSbDRow);
        const bf16x8v e2 = tr_frag(bp + 64 * kSbDRow, bp + 80 * kSbDRow);
        const bf16x8v e3 = tr_frag(bp + 128 * kSbDRow, bp + 144 * kSbDRow);
        f32x4v acc = dw[nt];
        acc = mfma_bf16(h3, e1, acc);
        acc = mfma_bf16(h2, e2, acc);
        acc = mfma_bf16(h1, e3, acc);
        acc = mfma_bf16(h2, e1, acc);
        acc = mfma_bf16(h1, e2, acc);
        dw[nt] = mfma_bf16(h1, e1, acc);
      }
    }
    wave_lds_sync();  // this tile's LDS reads done before the next tile's writes
  }
  if (g.part == nullptr) return;  // no grad_W / grad_b requested (uniform: every thread returns)
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    db[nt] += __shfl_xor(db[nt], 16);
    db[nt] += __shfl_xor(db[nt], 32);
  }
  const int nWb = H * P + P;
  __syncthreads();
  float* mine = lds + wid * wfl;
#pragma unroll
  for (int nt = 0; nt < NN; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hr = 4 * ak + i, p = 16 * nt + am;  // C layout: row 4 ak + i, column am
      if (p < P) mine[hr * P + p] = dw[nt][i];
    }
#pragma unroll
  for (int nt = 0; nt < NN; ++nt)
    if (ak == 0 && 16 * nt + am < P) mine[H * P + 16 * nt + am] = db[nt];
  __syncthreads();
  float* out = g.part + (int64_t)blockIdx.x * nWb;
  for (int i = tid; i < nWb; i += blockDim.x) {
    float s = lds[i];
    for (int w = 1; w < nwave; ++w) s += lds[w * wfl + i];
    out[i] = s;
  }
}

// grad_W | grad_b = the sum of the per-workgroup partials (fp64, deterministic): a
// workgroup owns 64 consecutive elements (lane = element, coalesced rows of the
// partials); its 16 waves take the partials w, w + 16, ... and are combined in wave order
__global__ void __launch_bounds__(1024) sum_partials_kernel(const float* __restrict__ part, int nparts, int n,
                                                            float* __restrict__ gW, float* __restrict__ gb, int nW) {
  __shared__ double red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  double s = 0.0;
  if (i < n) {
#pragma unroll 4
    for (int k = w; k < nparts; k += 16) s += (double)part[(int64_t)k * n + i];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w != 0 || i >= n) return;
  double t = red[0][lane];
  for (int v = 1; v < 16; ++v) t += red[v][lane];
  if (i < nW) {
    if (gW) gW[i] = (float)t;
  } else if (gb) {
    gb[i - nW] = (float)t;
  }
}

template <int MH, int NN>
int64_t launch_dg1(const DenseGradArgs& g, int64_t max_parts, hipStream_t s) {
  auto kfn = chain_dense1_grad_kernel<MH, NN, kChainPairs>;
#ifdef NFN_DIAG
  if (env_int("NFN_CHAIN_FORM", kChainPairs) == kChainLoop) kfn = chain_dense1_grad_kernel<MH, NN>;
  if (env_int("NFN_CHAIN_FORM", kChainPairs) == kChainHPair && hpair_types(g.da.c) == 1)  // (planar, radial)
    kfn = env_int("NFN_HPAIR_U", 1) == 2 ? chain_dense1_grad_kernel<MH, NN, hpair_form(0, 1, 2)>
                                         : chain_dense1_grad_kernel<MH, NN, hpair_form(0, 1, 1)>;
  if constexpr (NN == 2) {
    if (env_int("NFN_CHAIN_FORM", kChainPairs) == kStaticProg && g.da.c.prog.K == kStaticK[0] &&
        g.da.c.prog.types[0] == kStaticTypes[0])
      kfn = chain_dense1_grad_kernel<MH, NN, kStaticProg>;
    if constexpr (MH == 1) {
      const int ab = env_int("NFN_DGRAD_ABLATE", 0);
      if (ab == 1) kfn = chain_dense1_grad_kernel<MH, NN, kChainPairs, 1>;
      if (ab == 2) kfn = chain_dense1_grad_kernel<MH, NN, kChainPairs, 2>;
      if (ab == 3) kfn = chain_dense1_grad_kernel<MH, NN, kChainPairs, 3>;
    }
  }
#endif
  const size_t lds = (size_t)4 * dense1_grad_wave_floats(g.da.c.P, 16 * MH + 4, g.da.c.prog.K) * sizeof(float);
  int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (g.da.c.ntiles + 3) / 4);
  grid = std::max<int64_t>(1, std::min<int64_t>(grid, max_parts));
  nfn_launch(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, g);
  return grid;
}

// the split-bf16 form (H = 16, P <= 32); kDgradSplitBf16 = its release default, diag NFN_DGRAD_SB
constexpr int kDgradSplitBf16 = 1;
template <int NN>
int64_t launch_dg1_sb(const DenseGradArgs& g, int64_t max_parts, hipStream_t s) {
  auto kfn = chain_dense1_grad_sb_kernel<NN, kChainPairs>;
  // a cached program (kCacheTypes) at compile time with the parameter-scalar cache: C2's 0.950 vs
  // 1.066 ms without the cache and 1.158 for the runtime program's pair form in one bench-harness
  // A/B (profiles/r06/r06k/); the diag build's NFN_CHAIN_FORM picks the others
  int sp = -1;
  for (int i = 0; i < kNumCached; ++i)
    if (g.da.c.prog.K == kCacheK[i] && g.da.c.prog.types[0] == kCacheTypes[i]) sp = i;
  if constexpr (NN == 2) {
    if (sp == 0) kfn = chain_dense1_grad_sb_kernel<NN, kStaticCache, 0>;
    if (sp == 1) kfn = chain_dense1_grad_sb_kernel<NN, kStaticCache, 1>;
  }
#ifdef NFN_DIAG
  const int cf = env_int("NFN_CHAIN_FORM", -1);
  if (cf == kChainLoop) kfn = chain_dense1_grad_sb_kernel<NN, kChainLoop>;
  if (cf == kChainPairs) kfn = chain_dense1_grad_sb_kernel<NN, kChainPairs>;
  if constexpr (NN == 2) {
    if (sp == 0 && cf == kStaticProg) kfn = chain_dense1_grad_sb_kernel<NN, kStaticProg>;
    if (sp == 0 && cf == kStaticCacheX) kfn = chain_dense1_grad_sb_kernel<NN, kStaticCacheX, 0>;
    if (sp == 1 && cf == kStaticCacheX) kfn = chain_dense1_grad_sb_kernel<NN, kStaticCacheX, 1>;
  }
#endif
  const size_t lds = ((size_t)4 * dense1_grad_sb_wave_floats(g.da.c.P, g.da.c.prog.K) + kSbWFloats) * sizeof(float);
  int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (g.da.c.ntiles + 3) / 4);
  grid = std::max<int64_t>(1, std::min<int64_t>(grid, max_parts));
  nfn_launch(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, g);
  return grid;
}

template <int MH>
int64_t launch_dg1_n(const DenseGradArgs& g, int64_t max_parts, hipStream_t s) {
  if (MH == 1 && g.da.c.P <= 32 && env_int("NFN_DGRAD_SB", kDgradSplitBf16) != 0 &&
      ((size_t)4 * dense1_grad_sb_wave_floats(g.da.c.P, g.da.c.prog.K) + kSbWFloats) * sizeof(float) <= (size_t)64 * 1024)
    return g.da.c.P <= 16 ? launch_dg1_sb<1>(g, max_parts, s) : launch_dg1_sb<2>(g, max_parts, s);
  switch ((g.da.c.P + 15) / 16) {
    case 1: return launch_dg1<MH, 1>(g, max_parts, s);
    case 2: return launch_dg1<MH, 2>(g, max_parts, s);
    case 3: return launch_dg1<MH, 3>(g, max_parts, s);
    case 4: return launch_dg1<MH, 4>(g, max_parts, s);
  }
  return 0;
}

template <int DM, bool FAST, int MH, int NN>
int64_t launch_dg(const DenseGradArgs& g, size_t lds, int64_t max_parts, hipStream_t s) {
  auto kfn = chain_dense_grad_kernel<DM, FAST, MH, NN>;
  int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (g.da.c.ntiles + 3) / 4);
  grid = std::max<int64_t>(1, std::min<int64_t>(grid, max_parts));
  nfn_launch(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, g);
  return grid;
}

template <int DM, bool FAST>
int64_t launch_dg_shape(const DenseGradArgs& g, size_t lds, int64_t max_parts, hipStream_t s) {
  const int mh = (g.da.H + 15) / 16, nn = (g.da.c.P + 15) / 16;
#define NFN_DG(MHv, NNv) \
  if (mh == MHv && nn == NNv) return launch_dg<DM, FAST, MHv, NNv>(g, lds, max_parts, s);
  NFN_DG(1, 1) NFN_DG(1, 2) NFN_DG(1, 3) NFN_DG(1, 4)
  NFN_DG(2, 1) NFN_DG(2, 2) NFN_DG(2, 3) NFN_DG(2, 4)
  NFN_DG(4, 1) NFN_DG(4, 2) NFN_DG(4, 3) NFN_DG(4, 4)
#undef NFN_DG
  return 0;
}

template <bool FAST>
int64_t launch_dg_dm(int dm, const DenseGradArgs& g, size_t lds, int64_t max_parts, hipStream_t s) {
  switch (dm) {
    case 1: return launch_dg_shape<1, FAST>(g, lds, max_parts, s);
    case 2: return launch_dg_shape<2, FAST>(g, lds, max_parts, s);
    case 4: return launch_dg_shape<4, FAST>(g, lds, max_parts, s);
    case 8: return launch_dg_shape<8, FAST>(g, lds, max_parts, s);
  }
  return 0;
}

}  // namespace

int64_t launch_dense_grad(bool fast, int dm, const DenseGradArgs& g, size_t lds, int64_t max_parts, hipStream_t s) {
  const ChainArgs& a = g.da.c;
  const int H = g.da.H;
  if (fast && a.d == 1 && a.prog.K <= 16 && (H == 16 || H == 32) && a.P <= 64 &&
      g.da.h_rowstride * 256 < ((int64_t)1 << 31) && g.gh_rowstride * 256 < ((int64_t)1 << 31) &&
      a.y_bstride * 256 < ((int64_t)1 << 31) && (reinterpret_cast<uintptr_t>(g.grad_h) & 15) == 0 &&
      (g.gh_rowstride & 3) == 0 && env_int("NFN_DENSE1_GRAD", 1) != 0 &&
      (size_t)4 * dense1_grad_wave_floats(a.P, H + 4, a.prog.K) * sizeof(float) <= (size_t)160 * 1024)
    return H == 16 ? launch_dg1_n<1>(g, max_parts, s) : launch_dg1_n<2>(g, max_parts, s);
  return fast ? launch_dg_dm<true>(dm, g, lds, max_parts, s) : launch_dg_dm<false>(dm, g, lds, max_parts, s);
}

void launch_sum_partials(const float* part, int64_t nparts, int n, float* gW, float* gb, int nW, hipStream_t s) {
  nfn_launch(sum_partials_kernel, dim3((unsigned)((n + 63) / 64)), dim3(1024), 0, s, part, (int)nparts, n,
                     gW, gb, nW);
}

}  // namespace nfn
