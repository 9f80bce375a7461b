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
#include "nfn_launch.h"

namespace nfn {
namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

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

// grad_W | grad_b = the sum of the per-workgroup partials, one thread per element,
// workgroups in order (fp64 accumulation, deterministic)
__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ part, int nparts, int n,
                                                           float* __restrict__ gW, float* __restrict__ gb, int nW) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int k = 0; k < nparts; ++k) s += (double)part[(int64_t)k * n + i];
  if (i < nW) {
    if (gW) gW[i] = (float)s;
  } else if (gb) {
    gb[i - nW] = (float)s;
  }
}

template <int DM, bool FAST, int MH, int NN>
int64_t launch_dg(const DenseGradArgs& g, size_t lds, int64_t max_parts, hipStream_t s) {
  auto kfn = chain_dense_grad_kernel<DM, FAST, MH, NN>;
  int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (g.da.c.ntiles + 3) / 4);
  grid = std::max<int64_t>(1, std::min<int64_t>(grid, max_parts));
  hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, g);
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
  return fast ? launch_dg_dm<true>(dm, g, lds, max_parts, s) : launch_dg_dm<false>(dm, g, lds, max_parts, s);
}

void launch_sum_partials(const float* part, int64_t nparts, int n, float* gW, float* gb, int nW, hipStream_t s) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, (int)nparts, n,
                     gW, gb, nW);
}

}  // namespace nfn
