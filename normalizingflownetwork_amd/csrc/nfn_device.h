// nfn_device.h — device code of the gfx950 (MI355X) conditional normalizing-flow
// log_prob kernels: math, bijectors, chain evaluators and kernel templates.
//
// Reference semantics (paths in the reference checkout):
//   PlanarFlow  estimators/normalizing_flows/PlanarFlow.py:20-80
//   RadialFlow  estimators/normalizing_flows/RadialFlow.py:20-84
//   AffineFlow  estimators/normalizing_flows/AffineFlow.py:4-17  (tfp Affine, diag scale)
//   layer       estimators/DistributionLayers.py:245-294  (reversed param layout,
//               Invert(Chain(...)), MultivariateNormalDiag base)
//   estimator   estimators/BaseEstimator.py:77-86  (y normalisation, -sum(log y_std))
//   posterior   estimators/BayesianNNEstimator.py:65-76, evaluation/scorers.py:13-27
//
// Design (DESIGN.md has the full story):
//   * Persistent kernels walk tiles of consecutive samples.  A tile's parameter
//     rows are one contiguous HBM region, streamed with coalesced non-temporal
//     16-byte loads into registers one tile AHEAD of use, then written to LDS with
//     a bank-conflict-free row stride; each lane then reads its own sample's
//     parameters from LDS.
//   * d = 1 (configs C1/C2/C5): one sample per lane, 64-row tiles owned by single
//     waves (no workgroup barriers), flow types packed 2 bits per flow so block
//     offsets are scalar arithmetic, next-flow parameter reads overlapped with
//     the current flow's math.
//   * d >= 4 (config C3): G-lane groups per sample with DPP butterfly reductions.
//   * z and the running log|det J| stay in VGPRs for the whole chain; only
//     log_prob and one fp64 partial sum per workgroup are written back.
// Kernel templates are instantiated by the launch translation units
// (nfn_persistent.hip, nfn_group.hip, nfn_tile.hip, nfn_misc.hip); the C ABI and
// the dispatch live in nfn_api.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "nfn.h"

// Contraction of a * b + c into an fma only within one source expression, as written —
// never by the backend across statements, whose choices follow the surrounding code (the
// build default, fast-honor-pragmas).  Every kernel that inlines these evaluators — one
// flow per loop trip, pairs, compile-time pair bodies, the grid's split form — then rounds
// the same way, so their results agree bit for bit.  Restored at the end of this header.
#pragma clang fp contract(on)

// The memory-pipeline details (buffer descriptors, counted vmcnt waits, the agent-scope
// partial sums across the XCDs' L2s) are validated on gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "the nfn kernels are written for gfx950 (MI355X) only"
#endif

namespace nfn {

constexpr int kMaxBlock = 256;
constexpr int kLdsTileBudget = 48 * 1024;  // bytes of LDS per workgroup for the tile
constexpr int kLdsMaxBytes = 156 * 1024;   // dynamic LDS a tile workgroup may take (160 KiB - static)
constexpr float kSoftplusThr = 13.942384719848633f;  // -(log(FLT_EPSILON) + 2), TF SoftplusOp
constexpr float kLogExpm1One = 0.54132485461291810f; // log(expm1(1))
constexpr float kHalfLog2Pi = 0.91893853320467274f;   // 0.5*log(2*pi)
constexpr float kLn2 = 0.69314718055994531f;
constexpr float kLog2e = 1.44269504088896341f;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// 16-byte load of a parameter-row piece; NT = non-temporal (streamed once).
template <bool NT>
__device__ __forceinline__ float4 load_row4(const float* p) {
  if constexpr (NT) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}

struct FlowProgram {
  int32_t K;
  uint32_t types[4];            // flow ids, 2 bits each, application order (64 flows)
  int32_t step[NFN_MAX_FLOWS];  // (param offset << 2) | flow id, application order
};

struct ChainArgs {
  const float* y;
  const float* t;
  const float* y_mean;
  const float* y_std;
  float* out;
  double* partials;
  double* out_sum;     // {sum, non-finite count} finished in-kernel by the last workgroup, or NULL
  int64_t y_bstride;
  int64_t t_rowstride;
  int64_t t_drawstride;
  int64_t B;
  int32_t d;
  int32_t P;
  int32_t lds_stride;  // odd, >= P
  int32_t trainable;
  int32_t S;           // posterior draws (1 for the plain chain)
  int32_t vec4;        // tile rows can be streamed as float4
  int32_t ownrow;      // persistent kernel: each lane streams its own row (else cooperative)
  int64_t ntiles;      // persistent kernel: number of `blockDim.x`-row tiles
  int32_t nt;          // non-temporal parameter-row loads
  int32_t nt_store;    // non-temporal log_prob stores
  int32_t nsplit;      // posterior: draw ranges per tile (1 = no split)
  int32_t dps;         // posterior: draws per range
  float2* split_out;   // posterior split: (max, scaled sum) per (range, sample)
  int32_t tile_rows;   // tile kernels: samples per tile when < blockDim.x (very wide rows)
  int32_t prio;        // raise wave priority around the tile hand-off (1 in the release library)
  int32_t tile_rot;    // chain_wave1_kernel: step k's tile slot for wave w is (w + k tile_rot) mod waves (>= 0)
#ifdef NFN_DIAG
  // diagnostic build only (libnfn_hip_diag.so; the release kernels compile these paths out)
  int32_t ablate_loads;  // NFN_ABLATE_LOADS: stream only the first tile (compute-only timing)
  int32_t tile_rot_g;    // NFN_TILE_ROT_G: chain_group1_kernel's rotated slots (release: the plain walk)
  int32_t tile_rot_b;    // NFN_TILE_ROT_B: chain_grad_wave_kernel's rotated slots (release: the plain walk)
#endif
  int64_t grid_cap;    // > 0: persistent grids are capped here (the workspace's partial slots)
  float* z_out;        // Chain bijector form (chain_wave1_kernel<..., FWD>): z_K per sample
  int32_t zonly;       // backward: z-only forward recompute when no log_prob is wanted (tuning knob)
  int64_t pair_base;   // chunked batch: this launch's first partial slot (earlier chunks' pairs precede it)
  uint32_t epoch;      // summed launch: this call's ticket epoch (non-zero, see write_partial)
  FlowProgram prog;
};

// The diagnostic build's knobs (ChainArgs' NFN_DIAG block); the release library sees the
// constants, so every such path folds away at compile time.
#ifdef NFN_DIAG
__host__ __device__ inline bool diag_ablate_loads(const ChainArgs& a) { return a.ablate_loads != 0; }
__host__ __device__ inline int diag_tile_rot_g(const ChainArgs& a) { return a.tile_rot_g; }
__host__ __device__ inline int diag_tile_rot_b(const ChainArgs& a) { return a.tile_rot_b; }
#else
__host__ __device__ inline bool diag_ablate_loads(const ChainArgs&) { return false; }
__host__ __device__ inline int diag_tile_rot_g(const ChainArgs&) { return 0; }
__host__ __device__ inline int diag_tile_rot_b(const ChainArgs&) { return 0; }
#endif

// Output Dense layer fused into the chain (nfn_dense.hip): t = h W + b on chip.
struct DenseArgs {
  ChainArgs c;           // t / t_rowstride unused
  const float* h;        // (B, H) rows at h_rowstride floats
  int64_t h_rowstride;
  const float* W;        // (H, P) row-major
  const float* bias;     // (P,) or NULL
  int32_t H;
  int32_t h_lds_stride;  // odd, > H
  // posterior (c.S draws): draw s uses h + s*h_drawstride (0 = shared h),
  // W + s*w_drawstride and bias + s*b_drawstride
  int64_t h_drawstride;
  int64_t w_drawstride;
  int64_t b_drawstride;
};

// Fused output Dense layer, backward (nfn_dense_grad.hip).
struct DenseGradArgs {
  DenseArgs da;
  const float* g_out;    // upstream gradient (B,) or NULL = ones
  float* grad_h;         // (B, H) at gh_rowstride, or NULL
  int64_t gh_rowstride;
  float* grad_y;         // (B, d) contiguous, or NULL
  float* part;           // per-workgroup partial [grad_W (H x P) | grad_b (P)]
};

// Sampling through the inverted flows (nfn_sample.hip).
struct SampleArgs {
  ChainArgs c;
  const float* eps;      // (B, d) standard-normal draws at eps_bstride floats
  int64_t eps_bstride;
  float* y_out;          // (B, d) contiguous
  float* logp;           // (B,) log-density of each sample, or NULL
};

// Density grid (nfn_grid.hip): y values shared by all parameter rows.
struct GridArgs {
  ChainArgs c;
  const float* y_grid;   // (G, d) rows at y_gstride floats
  int64_t y_gstride;
  float* out;            // (G, B): out[g * out_gstride + b]
  int64_t out_gstride;
  int32_t G;
  int32_t gchunk;        // grid points per workgroup (blockIdx.y walks the chunks)
};

// Backward (nfn_grad.hip): the forward's arguments plus the gradient outputs.
struct GradArgs {
  ChainArgs c;
  const float* g_out;    // upstream gradient (B,) or NULL = ones
  float* grad_t;         // (B, P) at gt_rowstride, or NULL
  float* grad_y;         // (B, d) contiguous, or NULL
  int64_t gt_rowstride;
  int32_t gt_vec4;       // grad_t rows can be written as float4
  int32_t rows;          // samples per workgroup (<= 64, one wave)
};

// ---------------------------------------------------------------------------
// Math.  FAST uses the gfx950 transcendental unit directly (v_exp_f32, v_log_f32,
// v_rcp_f32) with algebraic rewrites chosen to keep ABSOLUTE error ~1e-7 on every
// quantity that is later added into log_prob; the precise path uses OCML.
// ---------------------------------------------------------------------------

template <bool FAST>
__device__ __forceinline__ float f_exp(float x) {
  if constexpr (FAST) {
    return __builtin_amdgcn_exp2f(x * kLog2e);
  } else {
    return expf(x);
  }
}

template <bool FAST>
__device__ __forceinline__ float f_log(float x) {
  if constexpr (FAST) {
    return __builtin_amdgcn_logf(x) * kLn2;
  } else {
    return logf(x);
  }
}

template <bool FAST>
__device__ __forceinline__ float f_div(float a, float b) {
  if constexpr (FAST) {
    return a * __builtin_amdgcn_rcpf(b);
  } else {
    return a / b;
  }
}

// a / b correctly rounded in practice (rcp + one Newton step): used where the
// reference's own arithmetic cancels afterwards (planar u_hat), so the 1-ulp
// v_rcp_f32 error would be amplified.
template <bool FAST>
__device__ __forceinline__ float f_div_acc(float a, float b) {
  if constexpr (FAST) {
    const float r = __builtin_amdgcn_rcpf(b);
    const float q = a * r;
    return fmaf(fmaf(-b, q, a), r, q);
  } else {
    return a / b;
  }
}

// tf.nn.softplus (TF SoftplusOp): x if x > 13.94, exp(x) if x < -13.94, else log1p(exp(x)).
template <bool FAST>
__device__ __forceinline__ float softplus_tf(float x) {
  if constexpr (FAST) {
    // max(x,0) + ln(1 + e^{-|x|}): same function, exp argument <= 0; absolute
    // error ~1 ulp of 1, which is what every consumer (-1 + sp + 1e-5, alpha, beta,
    // 1e-3 + sp) is sensitive to.  Above TF's 13.94 threshold this equals x to
    // within 1 ulp, so no select is needed.
    const float e = __builtin_amdgcn_exp2f(-fabsf(x) * kLog2e);
    return fmaf(__builtin_amdgcn_logf(1.0f + e), kLn2, fmaxf(x, 0.0f));
  } else {
    if (x > kSoftplusThr) return x;
    const float e = expf(x);
    if (x < -kSoftplusThr) return e;
    return log1pf(e);
  }
}

// Radial alpha = softplus(0.3 a - 2) (RadialFlow.py:24-27) feeds h = 1 / (alpha + r),
// so it needs RELATIVE accuracy as alpha -> 0: in the plain fast form ln(1 + e) rounds
// to 0 once e < 2^-24 (alpha = 0, h = inf at z == gamma, where TF stays finite).  The
// rounding error of u = 1 + e is recovered exactly (c = e - (u - 1)) and added back:
// ln(1 + e) = ln(u) + c / u ~ ln(u) + c.  Three VALU ops, no select, no transcendental.
__device__ __forceinline__ float softplus_acc_fast(float x, float e) {
  const float u = 1.0f + e;
  const float c = e - (u - 1.0f);
  return fmaf(__builtin_amdgcn_logf(u), kLn2, fmaxf(x, 0.0f) + c);
}

template <bool FAST>
__device__ __forceinline__ float softplus_alpha(float x) {
  if constexpr (FAST) {
    return softplus_acc_fast(x, __builtin_amdgcn_exp2f(-fabsf(x) * kLog2e));
  } else {
    return softplus_tf<false>(x);
  }
}

// tanh with RELATIVE accuracy everywhere.  An absolute error of ~1e-7 is a large relative one
// as a -> 0; a planar step multiplies tanh by u_hat, which reaches ~1 / |w| when w -> 0
// (u_hat ~ m / w), so the absolute error became a z error of ~1e-7 / |w| (C2 full batch:
// log_prob off by up to 2e-4 on 2e-5 of the samples, tests/test_gpu_fullbatch.py).
// Below |a| = 0.3 an odd polynomial (tanh(a) / a - 1 as three terms in a^2, fitted for relative
// error on [0, 0.3]: <= 0.69 ulp, 0.26 on average); above it 1 - 2 / (1 + e^{2|a|}) with the
// sign copied back (<= 2.9 ulp on [0.3, 1), <= 1.2 past 1; e^{2|a|} -> inf saturates to 1; ulp
// figures with correctly rounded v_exp / v_rcp, both signs alike; with the hardware's, measured
// on MI355X: 3.19 ulp at most on [-1, 1], pinned at 3.25 by tests/test_gpu_diag.py).  Evaluating the exp form
// at |a| is what round 4's accuracy gain came from: round 3 evaluated it at signed a, where
// 2 / (1 + e^{2a}) > 1 has twice the ulp (5.2 ulp).  Round 4's five-term polynomial on [0, 0.55]
// bought nothing over this one in the fp32 emulation of the C2 chain (tools/kernel_emu.py: 200
// vs 206 of 2^21 samples beyond 3e-6 relative, 5 vs 5 beyond 1e-5) and cost two VALU per planar
// flow, which the C2 stream pays for (profiles/r05/).
__device__ __forceinline__ float tanh_poly03(float a) {  // |a| < 0.3
  const float a2 = a * a;
  float p = fmaf(a2, -0.050372913f, 0.13314915f);
  p = fmaf(a2, p, -0.33333063f);
  return fmaf(a * a2, p, a);
}
__device__ __forceinline__ float tanh_fast(float a) {
  const float x = fabsf(a);
  const float E = __builtin_amdgcn_exp2f(x * (2.0f * kLog2e));
  const float te = copysignf(1.0f - __builtin_amdgcn_rcpf(fmaf(E, 0.5f, 0.5f)), a);
  const float tp = tanh_poly03(a);
  return x < 0.3f ? tp : te;
}

template <bool FAST>
__device__ __forceinline__ float f_tanh(float a) {
  if constexpr (FAST) {
    return tanh_fast(a);
  } else {
    return tanhf(a);
  }
}

// Online logsumexp over draws, branch-free: one exp per draw
// (scorers.py:25 / BayesianNNEstimator.py:75 take scipy / tf logsumexp over axis 0).
template <bool FAST>
__device__ __forceinline__ void lse_push(float& m, float& acc, float lp) {
  const float dlt = lp - m;
  const float e = f_exp<FAST>(-fabsf(dlt));
  const bool up = dlt > 0.0f;  // false for NaN
  const float acc_new = up ? fmaf(acc, e, 1.0f) : acc + e;
  acc = (lp == -INFINITY) ? acc : acc_new;
  m = (lp != lp) ? lp : (up ? lp : m);
}

template <bool FAST>
__device__ __forceinline__ float lse_finish(float m, float acc, int S) {
  const float r = (m == -INFINITY || m != m) ? m : m + f_log<FAST>(acc);
  return r - f_log<FAST>((float)S);
}

// ---------------------------------------------------------------------------
// Bijectors.  `p` points at the flow's parameter block (LDS in the chain kernels,
// global memory in the single-flow kernel).  Each updates z in place (forward)
// and returns forward_log_det_jacobian evaluated at the input z.
// ---------------------------------------------------------------------------

// PlanarFlow.py:23-33 (u, w = t+1, b), _u_circ :49-53, _wzb :59, _forward :72,
// _forward_log_det_jacobian :78-80.
template <int DM, bool FAST, typename PTR>
__device__ __forceinline__ float planar_step(float (&z)[DM], PTR p, int d) {
  float u[DM], w[DM];
  float wtu = 0.0f, nw2 = 0.0f, wz = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      u[j] = p[j];
      w[j] = p[d + j] + 1.0f;
      wtu += w[j] * u[j];
      nw2 += w[j] * w[j];
      wz += w[j] * z[j];
    }
  }
  const float b = p[2 * d];
  // softplus with RELATIVE accuracy as w.u -> -inf: it is the leading term of
  // w.u_hat + 1 below once the constraint is active
  const float sp = softplus_alpha<FAST>(wtu);
  const float m_wtu = (-1.0f + sp) + 1e-5f;
  const float norm_w2 = nw2 + 1e-9f;
  const float coef = m_wtu - wtu;
  const float th = f_tanh<FAST>(wz + b);
  const float dth = 1.0f - th * th;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      // d = 1: u + (m - wu) w / (w^2 + 1e-9) = (1e-9 u + m w) / (w^2 + 1e-9) exactly, with
      // no cancellation between u and the correction as the constraint binds (w u -> -inf)
      const float uh = d == 1 ? f_div_acc<FAST>(fmaf(u[j], 1e-9f, m_wtu * w[j]), norm_w2)
                              : u[j] + coef * f_div_acc<FAST>(w[j], norm_w2);
      z[j] = z[j] + uh * th;
    }
  }
  // 1 + (1 - th^2) w.u_hat with w.u_hat = m - coef 1e-9 / |w|^2 (PlanarFlow.py:49-53):
  // th^2 + (1 - th^2)(softplus(w.u) + 1e-5 - coef 1e-9 / |w|^2), a sum of non-negative
  // terms, where the reference's 1 + sum(u_hat psi) cancels as w.u_hat -> -1
  const float qd = fmaf(-coef * 1e-9f, f_div<FAST>(1.0f, norm_w2), sp + 1e-5f);
  return f_log<FAST>(fabsf(fmaf(th, th, dth * qd)));
}

// RadialFlow.py:24-33 (alpha, beta constraints), _r :45 (L1 norm), _h :48,
// _forward :54-56, _forward_log_det_jacobian :62-70 (der_h = RealDiv grad ((-1/y)/y)).
template <int DM, bool FAST, typename PTR>
__device__ __forceinline__ float radial_step(float (&z)[DM], PTR p, int d) {
  const float alpha = softplus_alpha<FAST>(0.3f * p[0] - 2.0f);
  const float beta = softplus_tf<FAST>(0.1f * p[1] + kLogExpm1One) - 1.0f;
  float r = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) r += fabsf(z[j] - p[2 + j]);
  }
  const float yv = alpha + r;
  float h, der_h;
  if constexpr (FAST) {
    h = __builtin_amdgcn_rcpf(yv);
    der_h = -h * h;
  } else {
    h = 1.0f / yv;
    der_h = (-1.0f / yv) / yv;
  }
  const float ab = alpha * beta;
  const float abh = ab * h;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) z[j] = z[j] + abh * (z[j] - p[2 + j]);
  }
  const float A = 1.0f + abh;
  const float Bv = A + (ab * der_h) * r;
  float Ap = 1.0f;  // (1 + ab*h) ** (d - 1)
  for (int j = 1; j < d; ++j) Ap *= A;
  return f_log<FAST>(Ap * Bv);
}

// tfp.bijectors.Affine(shift=t[:d], scale_diag=1+t[d:2d]) — AffineFlow.py:5-9.
template <int DM, bool FAST, typename PTR>
__device__ __forceinline__ float affine_step(float (&z)[DM], PTR p, int d) {
  float ldj = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      const float sc = 1.0f + p[d + j];
      z[j] = z[j] * sc + p[j];
      ldj += f_log<FAST>(fabsf(sc));
    }
  }
  return ldj;
}

template <int DM, bool FAST, typename PTR>
__device__ __forceinline__ float flow_step(int id, float (&z)[DM], PTR p, int d) {
  if (id == NFN_FLOW_PLANAR) return planar_step<DM, FAST>(z, p, d);
  if (id == NFN_FLOW_RADIAL) return radial_step<DM, FAST>(z, p, d);
  return affine_step<DM, FAST>(z, p, d);
}

// MultivariateNormalDiag(loc=t[:d], scale=1e-3+softplus(log(expm1(1))+0.1 t[d:2d]))
// .log_prob(x) — DistributionLayers.py:281-294; N(0, I) when not trainable.
template <int DM, bool FAST, typename PTR>
__device__ __forceinline__ float base_log_prob(const float (&x)[DM], PTR p, int d, bool trainable) {
  float sq = 0.0f, logdet = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      if (trainable) {
        const float s = 1e-3f + softplus_tf<FAST>(kLogExpm1One + 0.1f * p[d + j]);
        const float zz = f_div<FAST>(x[j] - p[j], s);
        sq += zz * zz;
        logdet += f_log<FAST>(s);
      } else {
        sq += x[j] * x[j];
      }
    }
  }
  return -0.5f * sq - (kHalfLog2Pi * (float)d + logdet);
}

// z_0 = y (or (y - mean)/std, BaseEstimator.py:85); returns -sum(log std) or 0.
template <int DM, bool FAST>
__device__ __forceinline__ float load_y(float (&z)[DM], const ChainArgs& a, int64_t b) {
  const float* yr = a.y + b * a.y_bstride;
  float corr = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < a.d) {
      z[j] = yr[j];
      if (a.y_mean) {
        z[j] = f_div<FAST>(z[j] - a.y_mean[j], a.y_std[j]);
        corr += f_log<FAST>(a.y_std[j]);
      }
    } else {
      z[j] = 0.0f;
    }
  }
  return corr;
}

// log_prob of one sample whose parameter row sits at `row` (LDS).
template <int DM, bool FAST>
__device__ __forceinline__ float eval_chain(float (&z)[DM], const float* row, const ChainArgs& a) {
  float ildj = 0.0f;
  const int d = a.d;
  for (int k = 0; k < a.prog.K; ++k) {
    const int st = a.prog.step[k];  // wave-uniform (kernel argument)
    ildj = ildj + flow_step<DM, FAST>(st & 3, z, row + (st >> 2), d);
  }
  return base_log_prob<DM, FAST>(z, row, d, a.trainable != 0) + ildj;
}

// ---------------------------------------------------------------------------
// d = 1 fast path (configs C1, C2, C5).  Every flow has <= 3 parameters at d = 1,
// so the chain is software-pipelined: while flow k is evaluated, flow k+1's
// step word (scalar load) and its three parameters (LDS reads) are already in
// flight.  Log-determinants are accumulated in log2 and scaled by ln 2 once, and
// softplus uses log2(1 + e) directly (absolute error ~1 ulp of 1, which is what
// every softplus consumer here — -1 + softplus + 1e-5, alpha, beta, the base
// scale — is sensitive to).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sp_fast1(float x) { return softplus_tf<true>(x); }

// The d = 1 bijectors return their Jacobian determinant (the caller accumulates
// log2|det|); algebra is rearranged for fewer VALU issues, never for less accuracy.
// Planar (PlanarFlow.py:23-33, :49-53, :72, :78-80), in forms that stay well
// conditioned where the reference's own fp32 order cancels (w u_hat -> -1):
//   m = -1 + softplus(wu) + 1e-5 (softplus relative-accurate as wu -> -inf),
//   u_hat = u + (m - wu) w / (w^2 + 1e-9) = (1e-9 u + m w) / (w^2 + 1e-9),
//   det = 1 + (1 - th^2) w u_hat = th^2 + (1 - th^2)(softplus(wu) + 1e-5 - (m - wu) 1e-9 / (w^2 + 1e-9)),
//   th = tanh_fast(w z + b) (relative accuracy: u_hat th with u_hat ~ m / w)
// (no cancellation follows the quotient, so v_rcp_f32's 1-ulp error is not amplified:
// no Newton step)
__device__ __forceinline__ float planar1_uh(float u, float w, float rn, float m) {
  return fmaf(u, 1e-9f, m * w) * rn;
}

// m = -1 + softplus(w u) + 1e-5 without the cancellation of softplus - 1 near
// w u = log(e - 1) (where m -> 1e-5 and u_hat ~ m / w carries m's relative error into z):
// with d = w u - log(e - 1), one fma against the two-float constant (the product w u is exact
// inside it, so no rounding of w u enters d), m = log1p((1 - 1/e) expm1(d)) + 1e-5
// = d P(d) + 1e-5, P a degree-7 polynomial fitted for relative error on |d| <= 0.75 (<= 2.1
// ulp in fp32 Horner); outside that range softplus - (1 - 1e-5) is not cancellation-limited.
// fp32 emulation of the C2 chain (tools/kernel_emu.py "r6" vs "r5", 2^20 random samples,
// correctly rounded transcendentals): beyond 3e-6 relative 110 -> 31, beyond 1e-5 4 -> 1
// (profiles/r06/r06_kernel_emu_m_forms.txt); on the GPU, every sample of C2 / C4 against the
// fp64 oracle: beyond 1e-5 relative 36 / 317 -> 19 / 138 (profiles/r06/r06h/r06h_parity.json).
// The d = 1 fast-math forwards of log_prob, the posterior, the grid and the Bijector API form
// m here (planar1_fast<true>, grid1_prepare), so their per-sample values stay bitwise one
// another's.
constexpr float kX0H = 0.54132485f, kX0L = 7.158233e-10f;  // log(e - 1) = kX0H + kX0L
__device__ __forceinline__ float planar1_m(float w, float u, float sp) {
  const float d = fmaf(w, u, -kX0H) - kX0L;
  float p = fmaf(d, -5.34155e-06f, -7.2508854e-05f);
  p = fmaf(d, p, 0.00016604575f);
  p = fmaf(d, p, 0.00091448176f);
  p = fmaf(d, p, -0.0038299547f);
  p = fmaf(d, p, -0.010241022f);
  p = fmaf(d, p, 0.116272084f);
  p = fmaf(d, p, 0.63212055f);
  return fabsf(d) <= 0.75f ? fmaf(d, p, 1e-5f) : sp - (1.0f - 1e-5f);
}

// ACCM: the cancellation-aware m (planar1_m) — every d = 1 fast-math forward except the
// compute-bound fused Dense kernels and the backward (ACCM = false: m = softplus - (1 - 1e-5),
// round 5's form; measured costs of the accurate m, profiles/r06/r06g/ and r06h/: fused Dense
// forward +6 %, backward +1 %; C2 +0.3 %, C5 +1.7 %).  Not adopted on top (r06o): a Newton step
// on 1 / |w|^2 (C2 / C4 beyond 1e-5 19 / 138 -> 20 / 126 for C2 +1 %, C5 +5.6 %).
template <bool ACCM = true>
__device__ __forceinline__ float planar1_fast(float& z, float u, float wraw, float b) {
  const float w = wraw + 1.0f;
  const float wtu = w * u;
  const float nw2 = fmaf(w, w, 1e-9f);
  const float rn = __builtin_amdgcn_rcpf(nw2);
  const float sp = softplus_alpha<true>(wtu);
  const float m = ACCM ? planar1_m(w, u, sp) : sp - (1.0f - 1e-5f);
  const float uh = planar1_uh(u, w, rn, m);
  const float qd = fmaf((wtu - m) * 1e-9f, rn, sp + 1e-5f);
  const float th = tanh_fast(fmaf(w, z, b));
  z = fmaf(uh, th, z);
  return fmaf(th, th, fmaf(-th, th, 1.0f) * qd);
}

// Radial (RadialFlow.py:24-33, :45-70) at d = 1: beta = softplus(.) - 1, so
// alpha * beta = alpha * sp - alpha, and 1 + abh + ab * (-h^2) * r = 1 + abh * (alpha h)
// because 1 - h r = alpha h.
__device__ __forceinline__ float radial1_fast(float& z, float a0, float b0, float g) {
  const float alpha = softplus_alpha<true>(fmaf(0.3f, a0, -2.0f));
  const float ab = fmaf(alpha, sp_fast1(fmaf(0.1f, b0, kLogExpm1One)), -alpha);
  const float dz = z - g;
  const float h = __builtin_amdgcn_rcpf(alpha + fabsf(dz));
  const float abh = ab * h;
  z = fmaf(abh, dz, z);
  return fmaf(abh, alpha * h, 1.0f);
}

__device__ __forceinline__ float affine1_fast(float& z, float sh, float scraw) {
  const float sc = 1.0f + scraw;
  z = fmaf(z, sc, sh);
  return sc;
}

// ST: floats between consecutive parameters of one sample (1 = row-major tile; the
// fused Dense kernel's column-major t tile uses its padded column stride).
template <int ST = 1>
__device__ __forceinline__ void read3(float (&v)[3], const float* row, int st) {
  const float* p = row + (st >> 2) * ST;
  v[0] = p[0];
  v[1] = p[ST];
  v[2] = (st & 3) == NFN_FLOW_AFFINE ? 0.0f : p[2 * ST];
}

// Chains of up to 16 flows: the flow types are packed 2 bits per flow in one
// 32-bit kernel argument and every block offset is derived with scalar
// arithmetic (blocks are stored in reverse application order, so
// off_0 = P - size(f_0) and off_{k+1} = off_k - size(f_{k+1})).  The unrolled
// chain body then holds no memory access for the program at all — only in-order
// LDS parameter reads, which for flow k+1 are issued before flow k's math.
__device__ __forceinline__ int size1(int id) { return id == NFN_FLOW_AFFINE ? 2 : 3; }

template <bool ACCM = true>
__device__ __forceinline__ float flow1_fast(int id, float& z, const float (&p)[3]) {
  if (id == NFN_FLOW_PLANAR) return planar1_fast<ACCM>(z, p[0], p[1], p[2]);
  if (id == NFN_FLOW_RADIAL) return radial1_fast(z, p[0], p[1], p[2]);
  return affine1_fast(z, p[0], p[1]);
}

template <int ST = 1>
__device__ __forceinline__ void read3c(float (&v)[3], const float* row, int off) {
  v[0] = row[off * ST];
  v[1] = row[(off + 1) * ST];
  v[2] = row[(off + 2) * ST];
}

template <int ST = 1, bool ACCM = true>
__device__ __forceinline__ float chain1_fast_packed(float& z, const float* row, uint32_t types, int K, int P) {
  float l2 = 0.0f;
  int id = (int)(types & 3u);
  int off = P - size1(id);
  // Parameter reads are unconditional (3 floats, offset clamped at 0; the LDS
  // tile is padded) so that no control flow separates a read from its use and
  // the waitcnt pass can count the in-order LDS returns instead of draining.
  float pc[3];
  read3c<ST>(pc, row, off);
#pragma unroll 1
  for (int k = 0; k < 16; ++k) {
    if (k < K) {
      const int idn = (int)((types >> (2 * (k + 1) & 31)) & 3u);
      const int offn = max(off - size1(idn), 0);
      float pn[3];
      read3c<ST>(pn, row, offn);
      l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<ACCM>(id, z, pc)));
      id = idn;
      off = offn;
      pc[0] = pn[0];
      pc[1] = pn[1];
      pc[2] = pn[2];
    }
  }
  return l2;
}

// A program fixed at compile time (TYPES, K): straight-line code, no dispatch.
template <uint32_t TYPES, int K, int ST = 1, bool ACCM = true>
__device__ __forceinline__ float chain1_fast_static(float& z, const float* row, int P) {
  float l2 = 0.0f;
  int off = P;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int id = (int)((TYPES >> (2 * k)) & 3u);
    off -= size1(id);
    float pc[3];
    read3c<ST>(pc, row, off);
    l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<ACCM>(id, z, pc)));
  }
  return l2;
}

// Two flows per dispatch: each of the nine (type, type) pairs is straight-line code,
// so the second flow's parameter-only work (softplus, u_hat, alpha, beta) can issue
// under the first flow's z chain, and the type dispatch runs once per pair.  The
// next pair's parameters are read (LDS) before the current pair is evaluated.
template <int IA, int IB, bool ACCM = true>
__device__ __forceinline__ void flow_pair1(float& z, float& l2, const float (&pa)[3], const float (&pb)[3]) {
  const float da = flow1_fast<ACCM>(IA, z, pa);
  l2 += __builtin_amdgcn_logf(fabsf(da));
  const float db = flow1_fast<ACCM>(IB, z, pb);
  l2 += __builtin_amdgcn_logf(fabsf(db));
}

#define NFN_PAIR_SWITCH(sel, CALL) \
  switch (sel) {                   \
    case 0: CALL(0, 0); break;     \
    case 1: CALL(0, 1); break;     \
    case 2: CALL(0, 2); break;     \
    case 3: CALL(1, 0); break;     \
    case 4: CALL(1, 1); break;     \
    case 5: CALL(1, 2); break;     \
    case 6: CALL(2, 0); break;     \
    case 7: CALL(2, 1); break;     \
    default: CALL(2, 2); break;    \
  }

// Flow k's type; flows past the program read as planar (offsets then clamp at 0:
// harmless in-row reads of the padded tile).
__device__ __forceinline__ int type1(uint32_t types, int k) { return (int)((types >> ((2 * k) & 31)) & 3u); }

template <int ST = 1, bool ACCM = true>
__device__ __forceinline__ float chain1_fast_pairs(float& z, const float* row, uint32_t types, int K, int P) {
  float l2 = 0.0f;
  int ia = type1(types, 0), ib = type1(types, 1);
  int offa = max(P - size1(ia), 0), offb = max(offa - size1(ib), 0);
  float pa[3], pb[3];
  read3c<ST>(pa, row, offa);
  read3c<ST>(pb, row, offb);
#pragma unroll 1
  for (int k = 0; k + 1 < K; k += 2) {
    const int ian = type1(types, k + 2), ibn = type1(types, k + 3);
    const int offan = max(offb - size1(ian), 0), offbn = max(offan - size1(ibn), 0);
    float pna[3], pnb[3];
    read3c<ST>(pna, row, offan);
    read3c<ST>(pnb, row, offbn);
#define NFN_FWD(A, B) flow_pair1<A, B, ACCM>(z, l2, pa, pb)
    NFN_PAIR_SWITCH(ia * 3 + ib, NFN_FWD)
#undef NFN_FWD
    ia = ian;
    ib = ibn;
    offb = offbn;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pa[i] = pna[i];
      pb[i] = pnb[i];
    }
  }
  if (K & 1) l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<ACCM>(ia, z, pa)));  // the last flow: already read
  return l2;
}

// chain1_fast_pairs for a program that alternates two types (IA, IB, IA, IB, ...; IA == IB
// covers a homogeneous chain): the pair's types and offsets are compile-time, the loop body
// one basic block (no dispatch); U pairs per trip, the remainder pair by pair.  The same
// flow_pair1 calls on the same values as chain1_fast_pairs.
template <int IA, int IB, int U, int ST = 1, bool ACCM = true>
__device__ __forceinline__ float chain1_fast_hpairs(float& z, const float* row, int K, int P) {
  constexpr int SA = IA == NFN_FLOW_AFFINE ? 2 : 3, SB = IB == NFN_FLOW_AFFINE ? 2 : 3, SP = SA + SB;
  float l2 = 0.0f;
  int off = P;  // the current pair's block ends here
  const int np = K >> 1;
  int p = 0;
  if constexpr (U == 0) {  // one pair per trip, the next pair's parameters read first
    float pa[3], pb[3];
    read3c<ST>(pa, row, max(off - SA, 0));
    read3c<ST>(pb, row, max(off - SP, 0));
#pragma unroll 1
    for (; p < np; ++p) {
      off -= SP;
      float pna[3], pnb[3];
      read3c<ST>(pna, row, max(off - SA, 0));  // past flow 0: harmless in-row reads
      read3c<ST>(pnb, row, max(off - SP, 0));
      flow_pair1<IA, IB, ACCM>(z, l2, pa, pb);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pa[i] = pna[i];
        pb[i] = pnb[i];
      }
    }
    if (K & 1) l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<ACCM>(IA, z, pa)));  // already read
    return l2;
  }
#pragma unroll 1
  for (; p + U <= np; p += U) {
    float pa[U > 0 ? U : 1][3], pb[U > 0 ? U : 1][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      read3c<ST>(pa[u], row, off - u * SP - SA);
      read3c<ST>(pb[u], row, off - u * SP - SP);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) flow_pair1<IA, IB, ACCM>(z, l2, pa[u], pb[u]);
    off -= U * SP;
  }
#pragma unroll 1
  for (; p < np; ++p) {
    float pa[3], pb[3];
    read3c<ST>(pa, row, off - SA);
    read3c<ST>(pb, row, off - SP);
    flow_pair1<IA, IB, ACCM>(z, l2, pa, pb);
    off -= SP;
  }
  if (K & 1) {
    float pa[3];
    read3c<ST>(pa, row, off - SA);
    l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<ACCM>(IA, z, pa)));
  }
  return l2;
}

// chain1_fast_pairs over TWO rows that share the program (two draws of one sample in the
// posterior): one dispatch per pair of flows for both, two independent dependency chains
// for the scheduler to interleave.  Per row the same arithmetic as chain1_fast_pairs.
template <int ST = 1>
__device__ __forceinline__ void chain1_fast_pairs2(float& za, float& zb, const float* rowa, const float* rowb,
                                                   uint32_t types, int K, int P, float& l2a, float& l2b) {
  l2a = 0.0f;
  l2b = 0.0f;
  int ia = type1(types, 0), ib = type1(types, 1);
  int offa = max(P - size1(ia), 0), offb = max(offa - size1(ib), 0);
  float pa[3], pb[3], qa[3], qb[3];
  read3c<ST>(pa, rowa, offa);
  read3c<ST>(pb, rowa, offb);
  read3c<ST>(qa, rowb, offa);
  read3c<ST>(qb, rowb, offb);
#pragma unroll 1
  for (int k = 0; k + 1 < K; k += 2) {
    const int ian = type1(types, k + 2), ibn = type1(types, k + 3);
    const int offan = max(offb - size1(ian), 0), offbn = max(offan - size1(ibn), 0);
    float pna[3], pnb[3], qna[3], qnb[3];
    read3c<ST>(pna, rowa, offan);
    read3c<ST>(pnb, rowa, offbn);
    read3c<ST>(qna, rowb, offan);
    read3c<ST>(qnb, rowb, offbn);
#define NFN_FWD2(A, B)                   \
  flow_pair1<A, B>(za, l2a, pa, pb);     \
  flow_pair1<A, B>(zb, l2b, qa, qb)
    NFN_PAIR_SWITCH(ia * 3 + ib, NFN_FWD2)
#undef NFN_FWD2
    ia = ian;
    ib = ibn;
    offb = offbn;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pa[i] = pna[i];
      pb[i] = pnb[i];
      qa[i] = qna[i];
      qb[i] = qnb[i];
    }
  }
  if (K & 1) {
    l2a += __builtin_amdgcn_logf(fabsf(flow1_fast(ia, za, pa)));
    l2b += __builtin_amdgcn_logf(fabsf(flow1_fast(ia, zb, qa)));
  }
}

// Chain-evaluation form of the d = 1 kernels: the packed loop, two flows per dispatch,
// or one compile-time program, C2's: without (diagnostic) / with the backward's
// parameter-scalar cache (grad1_static_cache: kStaticCache shares planar tanh between
// the passes, kStaticCacheX is bitwise grad1_static).
constexpr int kChainLoop = 0, kStaticProg = 2, kChainPairs = 3, kStaticCache = 4, kStaticCacheX = 5;
// Alternating-type programs (chain1_fast_hpairs): CM = hpair_form(IA, IB, U), U pairs per
// loop trip.
constexpr int kChainHPair = 8;
constexpr int hpair_form(int ia, int ib, int u) { return kChainHPair + 9 * u + 3 * ia + ib; }
// The pair form is bitwise the loop's.  It runs in the compute-bound d = 1 kernels
// (posterior, fused Dense forward / backward: -5 to -11 %) and, in the streaming
// kernels, for chains of at most this many flows (C1, K = 2: forward -18 %, backward
// -11 %); at K = 10 (C2) the streaming kernels stream 3-7 % slower with it.
constexpr int kPairsMaxKStream = 4;
constexpr uint32_t kStaticTypes[] = {0x44444u};  // (planar, radial) x 5
constexpr int kStaticK[] = {10};

// Base log-density at d = 1 (fast math), shared by every d = 1 evaluator.
template <int ST = 1>
__device__ __forceinline__ float base1_fast(float z, const float* row, bool trainable) {
  if (trainable) {
    const float sc = 1e-3f + sp_fast1(kLogExpm1One + 0.1f * row[ST]);
    const float zz = f_div<true>(z - row[0], sc);
    return -0.5f * (zz * zz) - (kHalfLog2Pi + __builtin_amdgcn_logf(sc) * kLn2);
  }
  return -0.5f * (z * z) - kHalfLog2Pi;
}

template <bool PACKED, int ST = 1, int CM = kChainLoop, bool ACCM = true>
__device__ __forceinline__ float eval_chain1_fast(float z, const float* row, const ChainArgs& a) {
  const int K = a.prog.K;
  float l2 = 0.0f;  // sum of log2|det J_k|
  if constexpr (CM >= kChainHPair) {
    constexpr int c = CM - kChainHPair;
    l2 = chain1_fast_hpairs<(c % 9) / 3, c % 3, c / 9, ST, ACCM>(z, row, K, a.P);
  } else if constexpr (CM == kChainPairs) {
    if (K > 0) l2 = chain1_fast_pairs<ST, ACCM>(z, row, a.prog.types[0], K, a.P);
  } else if constexpr (CM == kStaticProg) {
    l2 = chain1_fast_static<kStaticTypes[0], kStaticK[0], ST, ACCM>(z, row, a.P);
  } else if constexpr (PACKED) {
    if (K > 0) l2 = chain1_fast_packed<ST, ACCM>(z, row, a.prog.types[0], K, a.P);
  } else if (K > 0) {
    int st = a.prog.step[0];
    float pc[3];
    read3<ST>(pc, row, st);
    for (int k = 0; k < K; ++k) {
      const int stn = (k + 1 < K) ? a.prog.step[k + 1] : 0;
      float pn[3];
      if (k + 1 < K) read3<ST>(pn, row, stn);
      const int id = st & 3;
      float l;
      if (id == NFN_FLOW_PLANAR)
        l = planar1_fast<ACCM>(z, pc[0], pc[1], pc[2]);
      else if (id == NFN_FLOW_RADIAL)
        l = radial1_fast(z, pc[0], pc[1], pc[2]);
      else
        l = affine1_fast(z, pc[0], pc[1]);
      l2 += __builtin_amdgcn_logf(fabsf(l));
      st = stn;
      pc[0] = pn[0];
      pc[1] = pn[1];
      pc[2] = pn[2];
    }
  }
  return base1_fast<ST>(z, row, a.trainable != 0) + l2 * kLn2;
}

// One evaluator per (DM, FAST) for every kernel, so all tile-streaming strategies
// produce bitwise-identical per-sample results.
template <int DM, bool FAST>
__device__ __forceinline__ float eval_sample(float (&z)[DM], const float* row, const ChainArgs& a) {
  if constexpr (DM == 1 && FAST)
    return eval_chain1_fast<false>(z[0], row, a);
  else
    return eval_chain<DM, FAST>(z, row, a);
}

// Stream `nr` parameter rows of width P (global row stride rs) into LDS rows of
// stride S.  Coalesced: consecutive lanes take consecutive 16-byte (or 4-byte)
// pieces of the contiguous row block.
__device__ __forceinline__ void stage_rows(float* lds, const float* __restrict__ src, int64_t rs, int nr,
                                           int P, int S, bool vec4) {
  const int nth = blockDim.x;
  const int tid = threadIdx.x;
  if (vec4) {
    const int q = P >> 2;
    const int n = nr * q;
    const int step_r = nth / q, step_c = nth - (nth / q) * q;
    int r = tid / q, c = tid - (tid / q) * q;
    for (int i = tid; i < n; i += nth) {
      const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)r * rs + 4 * c);
      float* dst = lds + r * S + 4 * c;
      dst[0] = v.x;
      dst[1] = v.y;
      dst[2] = v.z;
      dst[3] = v.w;
      r += step_r;
      c += step_c;
      if (c >= q) {
        c -= q;
        r += 1;
      }
    }
  } else {
    const int n = nr * P;
    const int step_r = nth / P, step_c = nth - (nth / P) * P;
    int r = tid / P, c = tid - (tid / P) * P;
    for (int i = tid; i < n; i += nth) {
      lds[r * S + c] = src[(int64_t)r * rs + c];
      r += step_r;
      c += step_c;
      if (c >= P) {
        c -= P;
        r += 1;
      }
    }
  }
}

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) s += red[w];
  }
  return s;
}

// 1 for a non-finite log_prob (inf / NaN), else 0: every kernel that writes partial
// sums also counts these (SURVEY.md §5 — the reference only notices them in training,
// TerminateOnNaN, BaseEstimator.py:29; score's .mean() silently returns -inf / NaN).
__device__ __forceinline__ int nonfinite1(float v) { return __builtin_isfinite(v) ? 0 : 1; }

// Fixed-order sum of n (sum, non-finite count) pairs by ONE workgroup of any size
// (64..256 threads): virtual wave k in [0, kSumWaves) sums pairs 64 k + lane, + 256, ...
// and is combined by a butterfly, the waves in order by thread 0 — so the in-kernel
// finish and nfn_reduce_partials_f64 give bitwise-identical results.  `red` holds
// 2 * kSumWaves doubles; contains a __syncthreads.  out[0] = sum, out[1] = count.
constexpr int kSumWaves = 4;
template <bool ATOMIC = false>
__device__ __forceinline__ void sum_pairs(const double* __restrict__ pairs, int64_t n, double* red, double* out) {
  const int lane = threadIdx.x & 63, nw = (int)(blockDim.x >> 6), wid = (int)(threadIdx.x >> 6);
  for (int k = wid; k < kSumWaves; k += nw) {
    double s = 0.0, c = 0.0;
    for (int64_t i = 64 * k + lane; i < n; i += 64 * kSumWaves) {
      if constexpr (ATOMIC) {  // agent-coherent loads: pairs written by workgroups on other XCDs
        s += __hip_atomic_load(pairs + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c += __hip_atomic_load(pairs + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        s += pairs[2 * i];
        c += pairs[2 * i + 1];
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      s += __shfl_xor(s, off);
      c += __shfl_xor(c, off);
    }
    if (lane == 0) {
      red[2 * k] = s;
      red[2 * k + 1] = c;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tc = 0.0;
    for (int k = 0; k < kSumWaves; ++k) {
      ts += red[2 * k];
      tc += red[2 * k + 1];
    }
    out[0] = ts;
    out[1] = tc;
  }
}

// Workspace partials: pairs (sum, non-finite count) per workgroup at partials[2 blk],
// partials[2 blk + 1]; the header partials[-2] (= workspace[0]) is the number of
// pairs.  With out_sum, the LAST workgroup to finish sums every pair in fixed order into
// out_sum = {sum, non-finite count}: no reduction launch.  The last workgroup is found
// on a 64-bit ticket at partials[-1] = workspace[1], (epoch << 32 | count): the host
// gives every summed call a non-zero epoch, a workgroup that finds another epoch there
// (a finished call leaves 0; a fresh workspace holds anything) starts this call's count
// at 1 (compare-and-swap from what it saw), the others add 1; the workgroup that brings
// the count to gridDim.x is the last and clears the ticket.  So the workspace needs no
// initialisation and the call no memset launch (a replayed graph repeats its epoch,
// which the clear makes safe).
// Only the pairs cross workgroups, so they are written and read as agent-scope
// atomics (coherent across the XCDs' separate L2s) and ordered before the ticket by a
// vmcnt(0) wait: no release / acquire fence, which would write back / invalidate the
// whole L2 in every workgroup.  The ticket is a vector atomic.  `red` holds
// 2 * kMaxBlock / 64 doubles.  Contains __syncthreads: call from every thread.
__device__ __forceinline__ void write_partial(double* partials, double acc, int nf, double* red,
                                              double* out_sum, uint32_t epoch, int64_t base = 0) {
  double c = (double)nf;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc += __shfl_xor(acc, off);
    c += __shfl_xor(c, off);
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * wid] = acc;
    red[2 * wid + 1] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0, n = 0.0;
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) {
      s += red[2 * w];
      n += red[2 * w + 1];
    }
    const int64_t slot = base + blockIdx.x;
    __hip_atomic_store(partials + 2 * slot, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(partials + 2 * slot + 1, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) partials[-2] = (double)(base + gridDim.x);  // workspace header: number of pairs
  }
  if (out_sum == nullptr) return;  // partials-only launch (nfn_reduce_partials_f64 finishes it)
  unsigned long long* ticket = reinterpret_cast<unsigned long long*>(partials - 1);
  int* flag = reinterpret_cast<int*>(red);
  __syncthreads();  // red is free again
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pair has reached the coherence point
    // Only a workgroup that still sees another epoch tries to install this one (a CAS from
    // the value it saw, so it cannot undo another's install); every other workgroup adds 1.
    // A CAS per workgroup would serialise the whole grid's finish (+0.7 ms at C2, measured).
    unsigned long long cur = __hip_atomic_load(ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned count = 0u;
    if ((unsigned)(cur >> 32) != epoch &&
        __hip_atomic_compare_exchange_strong(ticket, &cur, ((unsigned long long)epoch << 32) | 1ull,
                                             __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      count = 1u;
    else
      count = (unsigned)__hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    flag[0] = count == gridDim.x;
  }
  __syncthreads();
  const bool last = flag[0] != 0;
  __syncthreads();
  if (!last) return;
  // Only the winning workgroup acquires (agent scope): the other workgroups' pairs,
  // stored before their ticket increments, are visible to its loads below.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  sum_pairs<true>(partials, base + gridDim.x, red, out_sum);
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

template <int DM, bool FAST>
__global__ void __launch_bounds__(kMaxBlock) chain_logprob_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
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
  float lp = 0.0f;
  if (tid < nr) {
    float z[DM];
    const int64_t b = b0 + tid;
    const float corr = load_y<DM, FAST>(z, a, b);
    lp = eval_sample<DM, FAST>(z, lds + (tb ? 0 : tid * a.lds_stride), a) - corr;
    if (a.out) a.out[b] = lp;
  }
  if (a.partials) write_partial(a.partials, tid < nr ? (double)lp : 0.0, tid < nr ? nonfinite1(lp) : 0, red, a.out_sum, a.epoch, a.pair_base);
}

// Posterior: the same tile walk once per draw, with an online logsumexp over draws.
template <int DM, bool FAST>
__global__ void __launch_bounds__(kMaxBlock) posterior_lse_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  const int rows = a.tile_rows > 0 ? a.tile_rows : blockDim.x;
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * rows;
  const int nr = (int)min((int64_t)rows, a.B - b0);
  const bool tb = a.t_rowstride == 0;
  float y0[DM];
  float corr = 0.0f;
  if (tid < nr) corr = load_y<DM, FAST>(y0, a, b0 + tid);
  float m = -INFINITY, acc = 0.0f;
  for (int s = 0; s < a.S; ++s) {
    if (s > 0) __syncthreads();  // previous draw's tile fully consumed
    if (a.P > 0) {
      stage_rows(lds, a.t + (int64_t)s * a.t_drawstride + (tb ? 0 : b0 * a.t_rowstride), a.t_rowstride,
                 tb ? 1 : nr, a.P, a.lds_stride, a.vec4 != 0);
    }
    __syncthreads();
    if (tid < nr) {
      float z[DM];
#pragma unroll
      for (int j = 0; j < DM; ++j) z[j] = y0[j];
      const float lp = eval_sample<DM, FAST>(z, lds + (tb ? 0 : tid * a.lds_stride), a) - corr;
      lse_push<FAST>(m, acc, lp);
    }
  }
  float res = 0.0f;
  if (tid < nr) {
    res = lse_finish<FAST>(m, acc, a.S);
    if (a.out) a.out[b0 + tid] = res;
  }
  if (a.partials) write_partial(a.partials, tid < nr ? (double)res : 0.0, tid < nr ? nonfinite1(res) : 0, red, a.out_sum, a.epoch, a.pair_base);
}

// Persistent, software-pipelined version of the two kernels above (the hot path).
// Each workgroup walks tiles blockIdx.x, blockIdx.x + gridDim.x, ...; for every
// (tile, draw) unit the NEXT unit's parameter rows are already in flight in
// registers (`buf`) while the current unit is evaluated from LDS, so HBM loads
// never wait on the flow math.  Rows are moved as float4 (Q = P/4 per row); a
// thread owns Q float4 slots whose addresses are affine in the slot index:
//   cooperative (ownrow = 0, needs Q | T): slot k = float4 (tid % Q) of row
//     tid / Q + k * T / Q — each wave instruction reads 1 KiB contiguous;
//   own-row (ownrow = 1): slot k = float4 k of row tid — each lane streams its
//     own row, no workgroup barrier is needed at all.
// Orders this wave's earlier LDS writes before its later LDS reads (and reads
// before later writes): the wave-tile mode needs no workgroup barrier because a
// wave only ever reads LDS rows that it wrote itself.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <int DM, bool FAST, int NV, bool POST, bool PACKED>
__global__ void __launch_bounds__(kMaxBlock, 4) chain_persistent_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  const int Q = a.P >> 2;
  const int S = a.lds_stride;
  const int64_t rs = a.t_rowstride;
  // Tile teams: the workgroup (cooperative / own-row modes) or each wave on its
  // own 64-row tile stream (wave mode: no workgroup barriers at all).
  const int mode = a.ownrow;  // 0 coop, 1 own-row, 2 wave
  const bool own = mode == 1;
  const bool wave = mode == 2;
  const bool wg_sync = mode == 0;
  const int wid = tid >> 6;
  const int TR = wave ? 64 : T;          // rows per tile
  const int lt = wave ? (tid & 63) : tid;  // thread index inside its team
  float* tl = wave ? lds + wid * 64 * S : lds;
  const int r0 = own ? lt : lt / Q;
  const int c4 = own ? 0 : lt - (lt / Q) * Q;
  const int rstep = own ? 0 : TR / Q;
  const int64_t g0 = (int64_t)r0 * rs + 4 * c4;
  const int64_t gstep = own ? 4 : (int64_t)rstep * rs;
  const int l0 = r0 * S + 4 * c4;
  const int lstep = own ? 4 : rstep * S;
  // Work units: (tile, draw range).  The plain chain has one draw and one range;
  // the posterior may split its S draws into `nsplit` ranges of `dps` draws
  // (merged by posterior_merge_kernel) to expose more parallelism than B allows.
  const int nsp = POST ? a.nsplit : 1;
  const int dps = POST ? a.dps : 1;
  const int64_t nunits = a.ntiles * nsp;
  const int64_t u0 = wave ? (int64_t)blockIdx.x * (T >> 6) + wid : blockIdx.x;
  const int64_t ustep = wave ? (int64_t)gridDim.x * (T >> 6) : gridDim.x;

  // y normalisation constants and -sum(log y_std), per launch
  float ymean[DM], yrstd[DM];
  float corr = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    ymean[j] = 0.0f;
    yrstd[j] = 1.0f;
    if (a.y_mean && j < a.d) {
      ymean[j] = a.y_mean[j];
      yrstd[j] = a.y_std[j];
      corr += f_log<FAST>(yrstd[j]);
    }
  }

  float4 buf[NV];
  float ybuf[DM];
  bool issued_once = false;
  auto issue = [&](int64_t unit, int s, bool first) {
    const int64_t tile = POST ? unit / nsp : unit;
    const int64_t b0 = tile * TR;
    const int nr = (int)min((int64_t)TR, a.B - b0);
    const float* base = a.t + (int64_t)s * a.t_drawstride + b0 * rs;
    if (diag_ablate_loads(a) && issued_once) return;  // diagnostic: compute-only timing
    issued_once = true;
    if (a.nt) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (k < Q && r0 + k * rstep < nr) buf[k] = load_row4<true>(base + g0 + k * gstep);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (k < Q && r0 + k * rstep < nr) buf[k] = load_row4<false>(base + g0 + k * gstep);
      }
    }
    if (first && lt < nr) {
      const float* yr = a.y + (b0 + lt) * a.y_bstride;
#pragma unroll
      for (int j = 0; j < DM; ++j) ybuf[j] = (j < a.d) ? yr[j] : 0.0f;
    }
  };
  auto range_of = [&](int64_t unit, int& sb, int& se) {
    const int rg = POST ? (int)(unit % nsp) : 0;
    sb = rg * dps;
    se = POST ? min(a.S, sb + dps) : 1;
  };
  auto store_out = [&](int64_t b, float v) {
    if (a.out) {
      if (a.nt_store)
        __builtin_nontemporal_store(v, a.out + b);
      else
        a.out[b] = v;
    }
  };

  double acc = 0.0;
  int nfc = 0;  // non-finite log_prob values
  // The store of a unit's results is deferred to the next unit and issued BEFORE
  // that unit's prefetch: vmcnt counts stores and loads in issue order, so a
  // store issued after the prefetch would make the next wait for the prefetched
  // rows also wait for the store's full latency.
  int64_t pend_b = -1;
  float pend_v = 0.0f, pend_m = 0.0f;
  int64_t unit = u0;
  if (unit < nunits) {
    int sb, se;
    range_of(unit, sb, se);
    issue(unit, sb, true);
  }
  for (; unit < nunits; unit += ustep) {
    const int64_t tile = POST ? unit / nsp : unit;
    const int64_t b0 = tile * TR;
    const int nr = (int)min((int64_t)TR, a.B - b0);
    int sb, se;
    range_of(unit, sb, se);
    float z0[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z0[j] = ybuf[j];
      if (a.y_mean && j < a.d) z0[j] = f_div<FAST>(z0[j] - ymean[j], yrstd[j]);
    }
    float m = -INFINITY, accl = 0.0f, lp = 0.0f;
    for (int s = sb; s < se; ++s) {
      if (wg_sync) __syncthreads();  // previous unit's LDS rows fully consumed
      if (a.prio) __builtin_amdgcn_s_setprio(3);  // tuning: hand-off + next prefetch at high priority
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (k < Q && r0 + k * rstep < nr) {
          float* dst = tl + l0 + k * lstep;
          dst[0] = buf[k].x;
          dst[1] = buf[k].y;
          dst[2] = buf[k].z;
          dst[3] = buf[k].w;
        }
      }
      if (wg_sync)
        __syncthreads();
      else if (wave)
        wave_lds_sync();
      if (pend_b >= 0) {
        if (!POST || nsp == 1) {
          store_out(pend_b, pend_v);
        } else {
          a.split_out[pend_b] = make_float2(pend_m, pend_v);
        }
        pend_b = -1;
      }
      // prefetch the next unit's rows while this one is evaluated
      if (s + 1 < se) {
        issue(unit, s + 1, false);
      } else if (unit + ustep < nunits) {
        int nb, ne;
        range_of(unit + ustep, nb, ne);
        issue(unit + ustep, nb, true);
      }
      if (a.prio == 2 && (wid & 1)) __builtin_amdgcn_s_setprio(1);  // static: odd waves compute first
      else if (a.prio) __builtin_amdgcn_s_setprio(0);
      if (lt < nr) {
        float z[DM];
#pragma unroll
        for (int j = 0; j < DM; ++j) z[j] = z0[j];
        if constexpr (DM == 1 && FAST)
          lp = eval_chain1_fast<PACKED>(z[0], tl + lt * S, a) - corr;
        else
          lp = eval_chain<DM, FAST>(z, tl + lt * S, a) - corr;
        if constexpr (POST) lse_push<FAST>(m, accl, lp);
      }
      if (wave) wave_lds_sync();  // this tile's LDS reads done before the next writes
    }
    if (lt < nr) {
      if (POST && nsp > 1) {
        const int rg = (int)(unit % nsp);
        pend_b = (int64_t)rg * a.B + b0 + lt;
        pend_m = m;
        pend_v = accl;
      } else {
        float res = lp;
        if constexpr (POST) res = lse_finish<FAST>(m, accl, a.S);
        pend_b = b0 + lt;
        pend_v = res;
        acc += (double)res;
        nfc += nonfinite1(res);
      }
    }
  }
  if (pend_b >= 0) {
    if (!POST || nsp == 1) {
      store_out(pend_b, pend_v);
    } else {
      a.split_out[pend_b] = make_float2(pend_m, pend_v);
    }
  }
  if (a.partials && (!POST || nsp == 1)) {
    write_partial(a.partials, acc, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// d = 1, wave-owned tiles, P = 4Q floats per row (Q = 2, 4, 8, 16): the hot path of
// configs C1 and C2 (forward; the posterior stays on chain_persistent_kernel).  Same walk as chain_persistent_kernel's wave mode, written
// so that the memory pipeline is straight-line code the waitcnt pass can count:
//   * every tile access is a BUFFER instruction whose descriptor (wave-uniform SGPRs)
//     spans exactly the tile's valid bytes: loads past B return 0 and stores past B
//     are dropped by the range check, so the last partial tile needs no branch and
//     no clamping, and addresses are loop-invariant 32-bit lane offsets (+ an SGPR
//     offset per row piece) — no VALU address arithmetic per load;
//   * y is issued FIRST with a tile's rows, one tile ahead; the rows are written to
//     LDS at the hand-off behind one counted wait;
//   * log_prob leaves in batches (see `flush`), never waited on by the next hand-off
//     (in the generic kernel a y use after the store, behind a branchy hand-off, made
//     the compiler wait for the store's full round trip on every tile).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// The per-tile log_prob (and, for the Chain bijector, z_K) stores of the streaming forward
// kernels (wave1, posterior_wave1, group1).  Cache policy kOutAux = sc1 (aux bits 16: write-through, the line is dropped from
// the XCD's L2) instead of non-temporal (2): in the bench harness the C2 stream with the
// compile-time pair bodies runs 0.378-0.380 ms with sc1 stores against 0.389-0.391 with nt
// (three boxes, profiles/r05/r05u / r05v / r05w_*), C3 -0.5 %, C5 unchanged; the memory-only
// form gains the same 2.5 %.  (The backward's gradient stores stay nt: a backward-shaped stream
// gains nothing from sc1, r05w_mixed_stream.log.)
constexpr int kOutAux = 16;
__device__ __forceinline__ void store_out32(float v, __amdgpu_buffer_rsrc_t r, int off, const ChainArgs&) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, kOutAux);
}

// FWD: the Bijector API's Chain forward + forward_log_det_jacobian instead of log_prob
// (nfn_chain_fwd_ldj_f32 over the layer's flow blocks; needs FAST and PACKED): z_K goes to
// a.z_out and sum_k log|det J_k| to a.out; no base density, no partial sums.
// (Round 5's rejected studies of this loop — LDS-DMA row fill, split / early issue, load and
// store cache policies, pacing, XCD skew, per-wave timestamps — are documented in DESIGN.md
// with their logs under profiles/r05/; they are no longer compiled.)
template <bool FAST, int Q, bool PACKED, bool FWD = false, int CM = kChainLoop>
__global__ void __launch_bounds__(kMaxBlock, 4) chain_wave1_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int RSTEP = 64 / Q;  // rows per wave-instruction
  constexpr int kNT = 2;         // buffer cache policy: non-temporal (streamed once)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: SGPR descriptors
  const int S = a.lds_stride;
  const int64_t rs = a.t_rowstride;
  const int r0 = lane / Q, c4 = lane % Q;
  float* tl = lds + wid * 64 * S;
  const int l0 = r0 * S + 4 * c4;
  const int64_t ntiles = a.ntiles;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<FAST>(ystd);
  }
  // diagnostic build (NFN_ABLATE_LOADS): every tile re-reads the wave's first tile
  const int64_t abl_tile = diag_ablate_loads(a) ? u0 : -1;
  // loop-invariant byte offsets (the host guarantees 64 rows of a tile span < 2 GiB)
  const int yoff = lane * (int)a.y_bstride * 4;
  const int toff = (r0 * (int)rs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)rs * 4;

  // Tiles past the end are issued too, through empty descriptors (no memory traffic,
  // zeros returned): every path then holds the same loads in the same order and the
  // waitcnt pass counts each hand-off's wait exactly.
  float4 buf[Q];
  float ybuf;
  auto issue = [&](int64_t tile) {
    if (abl_tile >= 0) tile = abl_tile;
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    const auto rt = tile_rsrc(a.t + b0c * rs, nr > 0 ? ((nr - 1) * rs + a.P) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
#pragma unroll
    for (int k = 0; k < Q; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, toff, k * kstep, kNT));
  };

  double acc = 0.0;
  int nfc = 0;  // non-finite log_prob values
  // The previous tile's log_prob, stored through a descriptor bounded at B (empty
  // before the first tile: the store is always issued).  It is issued right AFTER
  // the next prefetch, so the next hand-off's wait (vmcnt(1)) does not cover it.
  __amdgpu_buffer_rsrc_t pend_r = tile_rsrc(a.out, 0), pend_rz = tile_rsrc(a.z_out, 0);
  float pend_v = 0.0f, pend_z = 0.0f;
  auto flush = [&]() {
    store_out32(pend_v, pend_r, lane * 4, a);
    if constexpr (FWD)
      store_out32(pend_z, pend_rz, lane * 4, a);
  };
  // Step k covers tiles [k W, (k + 1) W) (W = ustep, the grid's waves); the wave takes slot
  // (u0 + k rot) mod W of it, so with rot > 0 a workgroup's waves visit every part of each
  // step's address range in turn instead of always the same one.
  // (The slot advances incrementally: 0 <= rot < W, no division.)
  const int64_t rot = a.tile_rot % ustep;
  issue(u0);
  flush();  // empty: every path into the loop ends [loads][store] (counted waits)
  for (int64_t tile = u0, base = 0, slot = u0, tnext; tile < ntiles; tile = tnext) {
    slot += rot;
    if (slot >= ustep) slot -= ustep;
    base += ustep;
    tnext = base + slot;  // the next step's tile
    const int64_t b0 = tile * 64;
    const int64_t nr = max((int64_t)0, min((int64_t)64, a.B - b0));
    if (a.prio) __builtin_amdgcn_s_setprio(3);  // hand-off + next prefetch at high priority
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      float* dst = tl + l0 + k * RSTEP * S;
      dst[0] = buf[k].x;
      dst[1] = buf[k].y;
      dst[2] = buf[k].z;
      dst[3] = buf[k].w;
    }
    const float z0 = norm ? f_div<FAST>(ybuf - ymean, ystd) : ybuf;
    wave_lds_sync();
    issue(tnext);
    flush();
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    float lp;
    if constexpr (FWD) {
      static_assert(FAST && PACKED, "the Chain bijector form uses the packed fast-math chain");
      float z = z0;
      lp = (a.prog.K > 0 ? chain1_fast_packed(z, tl + lane * S, a.prog.types[0], a.prog.K, a.P) : 0.0f) * kLn2;
      pend_z = z;
      pend_rz = tile_rsrc(a.z_out && nr > 0 ? a.z_out + b0 : a.z_out, a.z_out ? nr * 4 : 0);
    } else if constexpr (FAST) {
      lp = eval_chain1_fast<PACKED, 1, CM>(z0, tl + lane * S, a) - corr;
    } else {
      float z[1] = {z0};
      lp = eval_chain<1, false>(z, tl + lane * S, a) - corr;
    }
    if (!FWD && lane < nr) {
      acc += (double)lp;
      nfc += nonfinite1(lp);
    }
    pend_v = lp;
    pend_r = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
    wave_lds_sync();  // this tile's LDS reads done before the next writes
  }
  flush();
  if (a.partials) {
    write_partial(a.partials, acc, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// d = 1 Bayesian posterior (config C5) with chain_wave1_kernel's memory pipeline.  A
// wave owns (tile, draw range) units — the 64 samples of a tile through draws
// [sb, se) — and walks them DRAW-INNER: every (unit, draw) step hands its prefetched
// rows (draw s of the tile: one contiguous 64 x P block of t (S, B, P)) to LDS behind
// one counted wait, issues the NEXT step's rows (draw s + 1, or the next unit's first
// draw) and y through buffer descriptors bounded at B, and stores the previous unit's
// result, before the chain and the online logsumexp run on the current draw.  Every
// step issues the same loads and one store (an empty descriptor except right after a
// unit ends), so the pipeline is straight-line code with exact counted waits.  With
// nsplit == 1 (enough tiles for every resident wave: C5 at 2^17 samples) a unit is a
// whole tile, its score leaves once and there is no merge pass; otherwise units write
// (max, scaled sum) pairs for posterior_merge_kernel.
template <int Q, bool PACKED, int CM = kChainLoop>
__global__ void __launch_bounds__(kMaxBlock, 4) posterior_wave1_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int RSTEP = 64 / Q;
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int LS = a.lds_stride;
  const int64_t rs = a.t_rowstride, ds = a.t_drawstride;
  const int r0 = lane / Q, c4 = lane % Q;
  float* tl = lds + wid * 64 * LS;
  const int l0 = r0 * LS + 4 * c4;
  const int S = a.S, nsp = a.nsplit, dps = a.dps;
  const int64_t ntiles = a.ntiles;
  // units (tile, range) are visited as tile-major (tile, rg) pairs advanced by the
  // grid stride without 64-bit divisions: stride = (ut tiles, ur ranges)
  const int wstride = (int)(gridDim.x * (blockDim.x >> 6));
  const int ut = wstride / nsp, ur = wstride - ut * nsp;
  const int w0 = (int)(blockIdx.x * (blockDim.x >> 6)) + wid;
  int64_t tile = w0 / nsp;
  int rg = w0 - (int)tile * nsp;
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const int yoff = lane * (int)a.y_bstride * 4;
  const int toff = (r0 * (int)rs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)rs * 4;
  const float logS = f_log<true>((float)S);

  float4 buf[Q];
  float ybuf;
  // rows of draw s of tile `tl_`, and its y; tiles past the end issue empty descriptors
  auto issue = [&](int64_t tl_, int s) {
    const int64_t b0 = tl_ * 64;
    const int64_t nr = tl_ < ntiles ? min((int64_t)64, a.B - b0) : 0;
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    const auto rt = tile_rsrc(a.t + (nr > 0 ? s * ds + b0c * rs : 0), nr > 0 ? ((nr - 1) * rs + a.P) * 4 : 0);
#pragma unroll
    for (int k = 0; k < Q; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, toff, k * kstep, kNT));
  };

  double acc_sum = 0.0;
  int nfc = 0;
  // the previous unit's result: log_prob (nsplit == 1) or its (max, scaled sum) pair
  const __amdgpu_buffer_rsrc_t empty_r = tile_rsrc(a.out, 0);
  __amdgpu_buffer_rsrc_t pend_r = empty_r;
  float pend_v = 0.0f, pend_m = 0.0f;
  auto flush = [&]() {
    if (nsp == 1)
      store_out32(pend_v, pend_r, lane * 4, a);
    else
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_float2(pend_m, pend_v)), pend_r,
                                            lane * 8, 0, kNT);
  };
  issue(tile, rg * dps);
  flush();
  while (tile < ntiles) {
    const int64_t b0 = tile * 64;
    const int64_t nr = min((int64_t)64, a.B - b0);
    const int sb = rg * dps, se = min(S, sb + dps);
    // the next unit
    int rgn = rg + ur;
    int64_t tilen = tile + ut;
    if (rgn >= nsp) {
      rgn -= nsp;
      tilen += 1;
    }
    float m = -INFINITY, lacc = 0.0f, z0 = 0.0f;
    for (int s = sb; s < se; ++s) {
      if (a.prio) __builtin_amdgcn_s_setprio(3);
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        float* dst = tl + l0 + k * RSTEP * LS;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
      if (s == sb) z0 = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
      wave_lds_sync();
      if (s + 1 < se)
        issue(tile, s + 1);
      else
        issue(tilen, rgn * dps);
      flush();
      pend_r = empty_r;
      if (a.prio) __builtin_amdgcn_s_setprio(0);
      const float lp = eval_chain1_fast<PACKED, 1, CM>(z0, tl + lane * LS, a) - corr;
      lse_push<true>(m, lacc, lp);
      wave_lds_sync();  // this draw's LDS reads done before the next draw's writes
    }
    if (nsp == 1) {
      const float res = ((m == -INFINITY || m != m) ? m : m + f_log<true>(lacc)) - logS;
      if (lane < nr) {
        acc_sum += (double)res;
        nfc += nonfinite1(res);
      }
      pend_v = res;
      pend_r = tile_rsrc(a.out ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
    } else {
      pend_m = m;
      pend_v = lacc;
      pend_r = tile_rsrc(a.split_out + (int64_t)rg * a.B + b0, nr * 8);
    }
    tile = tilen;
    rg = rgn;
  }
  flush();
  if (a.partials && nsp == 1) write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
}

// posterior_wave1_kernel with TWO draws per step (diagnostic experiment, nsplit == 1):
// each lane evaluates its sample under draws s and s + 1 (chain1_fast_pairs2), the rows
// of both draws go to two LDS slots behind one counted wait, and the next step's two
// draws are in flight meanwhile (16 KiB per wave).  The logsumexp takes the draws in the
// same order, so the score is bitwise posterior_wave1_kernel<Q, true, kChainPairs>'s.
template <int Q>
__global__ void __launch_bounds__(kMaxBlock, 2) posterior_wave1x2_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int RSTEP = 64 / Q;
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int LS = a.lds_stride;
  const int64_t rs = a.t_rowstride, ds = a.t_drawstride;
  const int r0 = lane / Q, c4 = lane % Q;
  float* tl0 = lds + wid * 2 * 64 * LS;
  float* tl1 = tl0 + 64 * LS;
  const int l0 = r0 * LS + 4 * c4;
  const int S = a.S;
  const int64_t ntiles = a.ntiles;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const bool norm = a.y_mean != nullptr;
  float ymean = 0.0f, ystd = 1.0f, corr = 0.0f;
  if (norm) {
    ymean = a.y_mean[0];
    ystd = a.y_std[0];
    corr = f_log<true>(ystd);
  }
  const int yoff = lane * (int)a.y_bstride * 4;
  const int toff = (r0 * (int)rs + 4 * c4) * 4;
  const int kstep = RSTEP * (int)rs * 4;
  const float logS = f_log<true>((float)S);
  const bool trainable = a.trainable != 0;
  const uint32_t types = a.prog.types[0];
  const int K = a.prog.K;

  float4 buf0[Q], buf1[Q];
  float ybuf;
  // rows of draws s and s + 1 of tile `tl_` (an empty descriptor past S or past the end)
  auto issue = [&](int64_t tl_, int s) {
    const int64_t b0 = tl_ * 64;
    const int64_t nr = tl_ < ntiles ? min((int64_t)64, a.B - b0) : 0;
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * a.y_bstride, nr > 0 ? ((nr - 1) * a.y_bstride + 1) * 4 : 0);
    ybuf = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff, 0, 0));
    const int64_t span = nr > 0 ? ((nr - 1) * rs + a.P) * 4 : 0;
    const auto rt0 = tile_rsrc(a.t + (nr > 0 ? s * ds + b0c * rs : 0), span);
    const bool has1 = s + 1 < S;
    const auto rt1 = tile_rsrc(a.t + (nr > 0 && has1 ? (s + 1) * ds + b0c * rs : 0), has1 ? span : 0);
#pragma unroll
    for (int k = 0; k < Q; ++k)
      buf0[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt0, toff, k * kstep, kNT));
#pragma unroll
    for (int k = 0; k < Q; ++k)
      buf1[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt1, toff, k * kstep, kNT));
  };

  double acc_sum = 0.0;
  int nfc = 0;
  const __amdgpu_buffer_rsrc_t empty_r = tile_rsrc(a.out, 0);
  __amdgpu_buffer_rsrc_t pend_r = empty_r;
  float pend_v = 0.0f;
  auto flush = [&]() {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pend_v), pend_r, lane * 4, 0, kNT);
  };
  issue(tile, 0);
  flush();
  while (tile < ntiles) {
    const int64_t b0 = tile * 64;
    const int64_t nr = min((int64_t)64, a.B - b0);
    const int64_t tilen = tile + ustep;
    float m = -INFINITY, lacc = 0.0f, z0 = 0.0f;
    for (int s = 0; s < S; s += 2) {
      if (a.prio) __builtin_amdgcn_s_setprio(3);
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        float* d0 = tl0 + l0 + k * RSTEP * LS;
        d0[0] = buf0[k].x;
        d0[1] = buf0[k].y;
        d0[2] = buf0[k].z;
        d0[3] = buf0[k].w;
        float* d1 = tl1 + l0 + k * RSTEP * LS;
        d1[0] = buf1[k].x;
        d1[1] = buf1[k].y;
        d1[2] = buf1[k].z;
        d1[3] = buf1[k].w;
      }
      if (s == 0) z0 = norm ? f_div<true>(ybuf - ymean, ystd) : ybuf;
      wave_lds_sync();
      if (s + 2 < S)
        issue(tile, s + 2);
      else
        issue(tilen, 0);
      flush();
      pend_r = empty_r;
      if (a.prio) __builtin_amdgcn_s_setprio(0);
      float za = z0, zb = z0, l2a = 0.0f, l2b = 0.0f;
      if (K > 0) chain1_fast_pairs2<1>(za, zb, tl0 + lane * LS, tl1 + lane * LS, types, K, a.P, l2a, l2b);
      const float lpa = (base1_fast<1>(za, tl0 + lane * LS, trainable) + l2a * kLn2) - corr;
      lse_push<true>(m, lacc, lpa);
      if (s + 1 < S) {
        const float lpb = (base1_fast<1>(zb, tl1 + lane * LS, trainable) + l2b * kLn2) - corr;
        lse_push<true>(m, lacc, lpb);
      }
      wave_lds_sync();
    }
    const float res = ((m == -INFINITY || m != m) ? m : m + f_log<true>(lacc)) - logS;
    if (lane < nr) {
      acc_sum += (double)res;
      nfc += nonfinite1(res);
    }
    pend_v = res;
    pend_r = tile_rsrc(a.out ? a.out + b0 : a.out, a.out ? nr * 4 : 0);
    tile = tilen;
  }
  flush();
  if (a.partials) write_partial(a.partials, acc_sum, nfc, red, a.out_sum, a.epoch, a.pair_base);
}

// Combines the per-range (max, scaled sum) pairs of a draw-split posterior:
// out[b] = M + log(sum_r acc_r * exp(m_r - M)) - log S, M = max_r m_r.
template <bool FAST>
__global__ void __launch_bounds__(kMaxBlock) posterior_merge_kernel(const float2* __restrict__ parts, int nsplit,
                                                                     int S, int64_t B, float* __restrict__ out,
                                                                     double* __restrict__ partials,
                                                                     double* __restrict__ out_sum, uint32_t epoch) {
  __shared__ double red[2 * kMaxBlock / 64];
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float res = 0.0f;
  if (b < B) {
    float M = -INFINITY;
    bool nan = false;
    for (int r = 0; r < nsplit; ++r) {
      const float mr = parts[(int64_t)r * B + b].x;
      nan |= (mr != mr);
      M = fmaxf(M, mr);
    }
    if (nan) {
      res = NAN;
    } else if (M == -INFINITY) {
      res = -INFINITY;
    } else {
      float A = 0.0f;
      for (int r = 0; r < nsplit; ++r) {
        const float2 pr = parts[(int64_t)r * B + b];
        if (pr.x > -INFINITY) A += pr.y * f_exp<FAST>(pr.x - M);
      }
      res = (M + f_log<FAST>(A)) - f_log<FAST>((float)S);
    }
    if (out) out[b] = res;
  }
  if (partials) write_partial(partials, b < B ? (double)res : 0.0, b < B ? nonfinite1(res) : 0, red, out_sum, epoch);
}

// ---------------------------------------------------------------------------
// Lane-group kernel for wide events (d >= 4; config C3 is d = 8, P = 140).
// G = DM lanes cooperate on one sample and lane j owns z_j, so a 560-byte
// parameter row is spread over 8 lanes instead of one: per-thread prefetch stays
// at ceil(P / 4G) float4 and the LDS tile at (256 / G) rows, which keeps ~32
// waves per CU resident.  The inner products of the flows (w.u, |w|^2, w.z,
// u_hat.psi, |z - gamma|_1) are xor-shuffle reductions inside the G-lane group;
// per-sample scalars (softplus, tanh, log det) are evaluated redundantly by the
// group's lanes.  Per-dimension log terms (affine log|s_j|, the base density)
// are accumulated per lane and reduced once at the end.
// ---------------------------------------------------------------------------

// Butterfly sum inside G-lane groups with DPP (one VALU op per step, no LDS):
// quad_perm [1,0,3,2] (xor 1), quad_perm [2,3,0,1] (xor 2), row_half_mirror
// (8-lane combine), row_mirror (16-lane combine); xor 16 via a lane shuffle.
// Every lane of a group ends with the bitwise-identical sum (fp add commutes).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

template <int G>
__device__ __forceinline__ float gsum(float v) {
  if constexpr (G >= 2) v += dpp_mov<0xB1>(v);
  if constexpr (G >= 4) v += dpp_mov<0x4E>(v);
  if constexpr (G >= 8) v += dpp_mov<0x141>(v);
  if constexpr (G >= 16) v += dpp_mov<0x140>(v);
  if constexpr (G >= 32) v += __shfl_xor(v, 16, 32);
  return v;
}

// A G-lane group owns one sample; lane j owns the DPL dimensions
// j, j + G, ..., j + (DPL-1) G (interleaved, so each per-dimension LDS read by a
// group touches G consecutive floats).  G trades redundant per-sample scalar
// work (softplus / tanh / logs are evaluated by every lane of the group) against
// per-lane vector work (DPL dims each) and tile size.
// FULL: d == G * DPL (every lane's dimensions exist; config C3), so the per-dimension
// activity tests and their divergent branches compile away.
// LDJ = false: the z step only (the backward's forward recompute when log_prob is not
// wanted); returns 0.
template <int G, int DPL, bool FAST, bool FULL = false, bool LDJ = true>
__device__ __forceinline__ float planar_gd(float (&z)[DPL], const float* p, int d_, int j) {
  const int d = FULL ? G * DPL : d_;
  float u[DPL], w[DPL];
  float swu = 0.0f, sww = 0.0f, swz = 0.0f;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const bool act = FULL || j + G * i < d;
    u[i] = act ? p[j + G * i] : 0.0f;
    w[i] = act ? p[d + j + G * i] + 1.0f : 0.0f;
    swu += w[i] * u[i];
    sww += w[i] * w[i];
    swz += w[i] * z[i];
  }
  const float b = p[2 * d];
  const float wtu = gsum<G>(swu);
  const float nw2 = gsum<G>(sww);
  const float wz = gsum<G>(swz);
  // The det is th^2 + (1 - th^2)(softplus(w.u) + 1e-5 - coef 1e-9 / |w|^2) (planar_step):
  // no group sum of u_hat . w, and no cancellation as w.u_hat -> -1.
  if constexpr (FAST) {
    // u_hat_i = u_i + (coef / |w|^2) w_i
    const float sp = softplus_alpha<true>(wtu);
    const float c2 = f_div_acc<true>(sp - (wtu + (1.0f - 1e-5f)), nw2 + 1e-9f);
    const float th = f_tanh<true>(wz + b);
#pragma unroll
    for (int i = 0; i < DPL; ++i) {
      const float uh = fmaf(c2, w[i], u[i]);  // 0 on inactive dims
      z[i] = fmaf(uh, th, z[i]);
    }
    if constexpr (!LDJ) return 0.0f;
    const float qd = fmaf(-c2, 1e-9f, sp + 1e-5f);
    return f_log<true>(fabsf(fmaf(th, th, fmaf(-th, th, 1.0f) * qd)));
  }
  const float sp = softplus_alpha<FAST>(wtu);
  const float m_wtu = (-1.0f + sp) + 1e-5f;
  const float norm_w2 = nw2 + 1e-9f;
  const float coef = m_wtu - wtu;
  const float th = f_tanh<FAST>(wz + b);
  const float dth = 1.0f - th * th;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const float uh = u[i] + coef * f_div_acc<FAST>(w[i], norm_w2);  // 0 on inactive dims
    z[i] = z[i] + uh * th;
  }
  const float qd = fmaf(-coef * 1e-9f, f_div<FAST>(1.0f, norm_w2), sp + 1e-5f);
  return f_log<FAST>(fabsf(fmaf(th, th, dth * qd)));
}

template <int G, int DPL, bool FAST, bool FULL = false, bool LDJ = true>
__device__ __forceinline__ float radial_gd(float (&z)[DPL], const float* p, int d_, int j) {
  const int d = FULL ? G * DPL : d_;
  const float alpha = softplus_alpha<FAST>(0.3f * p[0] - 2.0f);
  const float beta = softplus_tf<FAST>(0.1f * p[1] + kLogExpm1One) - 1.0f;
  float g[DPL];
  float sr = 0.0f;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const bool act = FULL || j + G * i < d;
    g[i] = act ? p[2 + j + G * i] : 0.0f;
    sr += act ? fabsf(z[i] - g[i]) : 0.0f;
  }
  const float r = gsum<G>(sr);
  if constexpr (FAST) {
    // 1 + abh + ab (-h^2) r = 1 + abh (alpha h) since 1 - h r = alpha h;
    // (1 + abh)^(d-1) through one extra log instead of a runtime product loop.
    const float h = __builtin_amdgcn_rcpf(alpha + r);
    const float abh = (alpha * beta) * h;
#pragma unroll
    for (int i = 0; i < DPL; ++i) {
      if (FULL || j + G * i < d) z[i] = fmaf(abh, z[i] - g[i], z[i]);
    }
    if constexpr (!LDJ) return 0.0f;
    const float l2 = fmaf((float)(d - 1), __builtin_amdgcn_logf(1.0f + abh),
                          __builtin_amdgcn_logf(fmaf(abh, alpha * h, 1.0f)));
    return l2 * kLn2;
  }
  const float yv = alpha + r;
  float h, der_h;
  if constexpr (FAST) {
    h = __builtin_amdgcn_rcpf(yv);
    der_h = -h * h;
  } else {
    h = 1.0f / yv;
    der_h = (-1.0f / yv) / yv;
  }
  const float ab = alpha * beta;
  const float abh = ab * h;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    if (FULL || j + G * i < d) z[i] = z[i] + abh * (z[i] - g[i]);
  }
  const float A = 1.0f + abh;
  const float Bv = A + (ab * der_h) * r;
  float Ap = 1.0f;
  for (int i = 1; i < d; ++i) Ap *= A;
  return f_log<FAST>(Ap * Bv);
}

// Flow types of the (up to 64-flow) program, 2 bits each, from the 4 packed words.
__device__ __forceinline__ int flow_type_at(const uint32_t (&tw)[4], int k) {
  const uint32_t w = k < 16 ? tw[0] : (k < 32 ? tw[1] : (k < 48 ? tw[2] : tw[3]));
  return (int)((w >> (2 * (k & 15))) & 3u);
}

// FLOWS_ONLY: the Chain bijector's forward + fldj (no base density): z leaves as z_K and
// the return value is sum_k log|det J_k| (group-summed, every lane of the group).
template <int G, int DPL, bool FAST, bool FULL = false, bool FLOWS_ONLY = false>
__device__ __forceinline__ float eval_chain_gd(float (&z)[DPL], const float* row, const ChainArgs& a, int j) {
  const int d = FULL ? G * DPL : a.d;
  const int K = a.prog.K;
  uint32_t tw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) tw[q] = a.prog.types[q];
  float ildj = 0.0f, dimterm = 0.0f;
  // blocks are stored in reverse application order: off_0 = P - size(f_0), ...
  int off = a.P;
  for (int k = 0; k < K; ++k) {
    const int id = flow_type_at(tw, k);
    off -= id == NFN_FLOW_PLANAR ? 2 * d + 1 : (id == NFN_FLOW_RADIAL ? d + 2 : 2 * d);
    const float* p = row + off;
    if (id == NFN_FLOW_PLANAR) {
      ildj = ildj + planar_gd<G, DPL, FAST, FULL>(z, p, d, j);
    } else if (id == NFN_FLOW_RADIAL) {
      ildj = ildj + radial_gd<G, DPL, FAST, FULL>(z, p, d, j);
    } else {
#pragma unroll
      for (int i = 0; i < DPL; ++i) {
        if (FULL || j + G * i < d) {
          const float sc = 1.0f + p[d + j + G * i];
          z[i] = z[i] * sc + p[j + G * i];
          dimterm += f_log<FAST>(fabsf(sc));
        }
      }
    }
  }
  if constexpr (FLOWS_ONLY) return gsum<G>(dimterm) + ildj;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    if (FULL || jj < d) {
      if (a.trainable) {
        const float sc = 1e-3f + softplus_tf<FAST>(kLogExpm1One + 0.1f * row[d + jj]);
        const float zz = f_div<FAST>(z[i] - row[jj], sc);
        dimterm += -0.5f * (zz * zz) - f_log<FAST>(sc);
      } else {
        dimterm += -0.5f * (z[i] * z[i]);
      }
    }
  }
  return (gsum<G>(dimterm) - kHalfLog2Pi * (float)d) + ildj;
}

// Each WAVE owns its own tile stream of R = 64 / G samples (no workgroup
// barriers, as in the d = 1 wave mode): the next tile's rows are prefetched into
// registers while the current one is evaluated from the wave's LDS slot.
template <int G, int DPL, bool FAST, int NV, bool POST>
__global__ void __launch_bounds__(kMaxBlock) chain_group_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int R = 64 / G;  // samples per wave tile
  const int sl = lane / G;
  const int j = lane - sl * G;
  const int Q = a.P >> 2;
  const int S = a.lds_stride;
  const bool lds4 = (S & 3) == 0;
  const int64_t rs = a.t_rowstride;
  const int ndraw = POST ? a.S : 1;
  float* tl = lds + wid * R * S;
  // tile-invariant slot map: slot k = float4 q = lane + 64k of the wave tile, i.e.
  // row q / Q, piece q % Q, stepped incrementally (64 = sq*Q + sc)
  const int r00 = lane / Q, c00 = lane - (lane / Q) * Q;
  const int sq = 64 / Q, sc = 64 - (64 / Q) * Q;
  const int nslots = R * Q;
  const int64_t u0 = (int64_t)blockIdx.x * (T >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (T >> 6);
  float4 buf[NV];
  float ybuf[DPL];
  bool issued_once = false;
  auto issue = [&](int64_t tile, int s) {
    const int64_t b0 = tile * R;
    const int nr = (int)min((int64_t)R, a.B - b0);
    const float* base = a.t + (int64_t)s * a.t_drawstride + b0 * rs;
    if (diag_ablate_loads(a) && issued_once) return;  // diagnostic: compute-only timing
    issued_once = true;
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
    if (s == 0 && sl < nr) {
#pragma unroll
      for (int i = 0; i < DPL; ++i)
        ybuf[i] = (j + G * i < a.d) ? a.y[(b0 + sl) * a.y_bstride + j + G * i] : 0.0f;
    }
  };
  float corr = 0.0f;
  if (a.y_mean) {
    for (int i = 0; i < a.d; ++i) corr += f_log<FAST>(a.y_std[i]);
  }
  double acc = 0.0;
  int nfc = 0;  // non-finite log_prob values
  int64_t pend_b = -1;  // deferred store, see chain_persistent_kernel
  float pend_v = 0.0f;
  int64_t tile = u0;
  if (tile < a.ntiles) issue(tile, 0);
  for (; tile < a.ntiles; tile += ustep) {
    const int64_t b0 = tile * R;
    const int nr = (int)min((int64_t)R, a.B - b0);
    float z0[DPL];
#pragma unroll
    for (int i = 0; i < DPL; ++i) {
      const int jj = j + G * i;
      z0[i] = ybuf[i];
      if (a.y_mean && jj < a.d) z0[i] = f_div<FAST>(z0[i] - a.y_mean[jj], a.y_std[jj]);
    }
    float m = -INFINITY, accl = 0.0f, lp = 0.0f;
    for (int s = 0; s < ndraw; ++s) {
      if (a.prio) __builtin_amdgcn_s_setprio(2);
      {
        int r = r00, c = c00;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          if (lane + k * 64 < nslots && r < nr) {
            float* dst = tl + r * S + 4 * c;
            if (lds4) {
              *reinterpret_cast<float4*>(dst) = buf[k];
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
      wave_lds_sync();
      if (pend_b >= 0) {
        if (a.out) {
          if (a.nt_store)
            __builtin_nontemporal_store(pend_v, a.out + pend_b);
          else
            a.out[pend_b] = pend_v;
        }
        pend_b = -1;
      }
      if (s + 1 < ndraw)
        issue(tile, s + 1);
      else if (tile + ustep < a.ntiles)
        issue(tile + ustep, 0);
      if (a.prio) __builtin_amdgcn_s_setprio(0);
      if (sl < nr) {
        float z[DPL];
#pragma unroll
        for (int i = 0; i < DPL; ++i) z[i] = z0[i];
        lp = eval_chain_gd<G, DPL, FAST>(z, tl + sl * S, a, j) - corr;
        if constexpr (POST) lse_push<FAST>(m, accl, lp);
      }
      wave_lds_sync();  // this tile's LDS reads done before the next writes
    }
    if (sl < nr && j == 0) {
      float res = lp;
      if constexpr (POST) res = lse_finish<FAST>(m, accl, ndraw);
      pend_b = b0 + sl;
      pend_v = res;
      acc += (double)res;
      nfc += nonfinite1(res);
    }
  }
  if (pend_b >= 0 && a.out) a.out[pend_b] = pend_v;
  if (a.partials) {
    write_partial(a.partials, acc, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

// chain_group_kernel's walk for contiguous parameter rows (row stride == P), with the
// memory pipeline of chain_wave1_kernel: a wave tile of R = 64 / G rows is one
// contiguous block streamed by buffer loads at lane-linear offsets through a
// descriptor bounded at B (zeros past the end, empty descriptors past the last
// tile), y and log_prob by buffer instructions too, and no branch between a load
// and its use: lanes whose slot lies past the tile write their float4 to a per-lane
// pad after the last wave slot (distinct addresses: no same-address write conflicts).  Plain chain only (the posterior keeps chain_group_kernel).
// FWD: the Bijector API's Chain forward + fldj over the layer's rows (nfn_chain_fwd_ldj_f32):
// z_K leaves to a.z_out (each lane its DPL dims), sum_k log|det J_k| to a.out; no base density.
template <int G, int DPL, bool FAST, int NV, bool FULL, bool FWD = false>
__global__ void __launch_bounds__(kMaxBlock) chain_group1_kernel(ChainArgs a) {
  extern __shared__ float lds[];
  __shared__ double red[2 * kMaxBlock / 64];
  constexpr int R = 64 / G;  // samples per wave tile
  constexpr int kNT = 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sl = lane / G;
  const int j = lane - sl * G;
  const int Q = a.P >> 2;
  const int S = a.lds_stride;
  const int nslots = R * Q;  // float4 pieces per tile
  float* tl = lds + wid * R * S;
  float* pad = lds + (kMaxBlock / 64) * R * S + 4 * lane;  // per-lane scratch for out-of-tile slots
  int loff[NV];  // LDS float offset of this lane's slot k (tile-invariant)
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = lane + 64 * k;
    loff[k] = q < nslots ? (int)(tl - lds) + (q / Q) * S + 4 * (q % Q) : (int)(pad - lds);
  }
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int tbytes = R * a.P * 4;  // one full tile (< 2 GiB: P <= 2^24 / R)
  const int64_t ybs = a.y_bstride;
  const bool abl = diag_ablate_loads(a);
  float4 buf[NV];
  float ybuf[DPL];
  auto issue = [&](int64_t tile) {
    if (abl) tile = u0;
    const int64_t b0 = tile * R;
    const int64_t nr = max((int64_t)0, min((int64_t)R, a.B - b0));
    const int64_t b0c = nr > 0 ? b0 : 0;
    const auto ry = tile_rsrc(a.y + b0c * ybs, nr > 0 ? ((nr - 1) * ybs + a.d) * 4 : 0);
#pragma unroll
    for (int i = 0; i < DPL; ++i)
      ybuf[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             ry, (int)((sl * ybs + j + G * i) * 4), 0, 0));
    const auto rt = tile_rsrc(a.t + b0c * a.P, (int)(nr * a.P * 4));
#pragma unroll
    for (int k = 0; k < NV; ++k)
      buf[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, lane * 16, k * 1024, kNT));
    (void)tbytes;
  };
  float corr = 0.0f;
  if (a.y_mean) {
    for (int i = 0; i < a.d; ++i) corr += f_log<FAST>(a.y_std[i]);
  }
  float ymean[DPL], yrstd[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    ymean[i] = (a.y_mean && jj < a.d) ? a.y_mean[jj] : 0.0f;
    yrstd[i] = (a.y_mean && jj < a.d) ? a.y_std[jj] : 1.0f;
  }
  const bool norm = a.y_mean != nullptr;
  double acc = 0.0;
  int nfc = 0;  // non-finite log_prob values
  __amdgpu_buffer_rsrc_t pend_r = tile_rsrc(a.out, 0);
  float pend_v = 0.0f;
  // rotated tile slots as in chain_wave1_kernel: the plain walk (rot = 0) in the release library
  // (no gain for this kernel, profiles/r05/r05zr_c3_bench_diag.txt); diag NFN_TILE_ROT_G
  const int64_t rot = diag_tile_rot_g(a) % ustep;
  issue(u0);
  // an (empty) store behind the first prefetch too: every path into the loop then
  // ends [loads][store] and the hand-off waits with vmcnt(1), not vmcnt(0)
  store_out32(pend_v, pend_r, lane * 4, a);
  for (int64_t tile = u0, base = 0, slot = u0, tnext; tile < a.ntiles; tile = tnext) {
    slot += rot;
    if (slot >= ustep) slot -= ustep;
    base += ustep;
    tnext = base + slot;
    const int64_t b0 = tile * R;
    const int64_t nr = max((int64_t)0, min((int64_t)R, a.B - b0));
    if (a.prio) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int k = 0; k < NV; ++k) *reinterpret_cast<float4*>(lds + loff[k]) = buf[k];
    float z[DPL];
#pragma unroll
    for (int i = 0; i < DPL; ++i) z[i] = norm ? f_div<FAST>(ybuf[i] - ymean[i], yrstd[i]) : ybuf[i];
    wave_lds_sync();
    issue(tnext);
    store_out32(pend_v, pend_r, lane * 4, a);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    const float lp = eval_chain_gd<G, DPL, FAST, FULL, FWD>(z, tl + sl * S, a, j) - corr;
    wave_lds_sync();  // this tile's LDS reads done before the next writes
    if constexpr (FWD) {  // z_K: rows past B fall outside the descriptor
      const auto rz = tile_rsrc(a.z_out && nr > 0 ? a.z_out + b0 * a.d : a.z_out, a.z_out ? (int)nr * a.d * 4 : 0);
#pragma unroll
      for (int i = 0; i < DPL; ++i)
        if (FULL || j + G * i < a.d)
          store_out32(z[i], rz, (sl * a.d + j + G * i) * 4, a);
    } else if (j == 0 && sl < nr) {
      acc += (double)lp;
      nfc += nonfinite1(lp);
    }
    // lane i < R takes sample i's value (held by its group's lanes): one 64 B store
    // from 16 lanes instead of 4 identical copies per sample; lanes >= nr fall
    // outside the descriptor and are dropped
    pend_v = __shfl(lp, (lane * G) & 63);
    pend_r = tile_rsrc(a.out && nr > 0 ? a.out + b0 : a.out, a.out ? (int)nr * 4 : 0);
  }
  store_out32(pend_v, pend_r, lane * 4, a);
  if (a.partials) {
    write_partial(a.partials, acc, nfc, red, a.out_sum, a.epoch, a.pair_base);
  }
}

}  // namespace nfn

#pragma clang fp contract(fast)
