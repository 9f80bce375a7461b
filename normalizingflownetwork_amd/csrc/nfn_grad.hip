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
#include "nfn_launch.h"

namespace nfn {
namespace {

template <bool FAST>
__device__ __forceinline__ float f_sigmoid(float x) {
  if constexpr (FAST) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * kLog2e));
  } else {
    return 1.0f / (1.0f + expf(-x));
  }
}

__device__ __forceinline__ float sign0(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

// Adjoints.  `a` enters as d logp / d z_{k+1} and leaves as d logp / d z_k;
// `gl` is the adjoint of every log-det term (the upstream gradient g_b).
// Derivations: tests/analytic_grad.py (checked against autodiff in fp64).

// Planar: u_hat = u + c w / n, c = (-1 + softplus(w.u) + 1e-5) - w.u, n = |w|^2 + 1e-9,
// f = z + u_hat tanh(w.z + b), ldj = log|1 + (1 - tanh^2) w.u_hat|.
template <int DM, bool FAST>
__device__ __forceinline__ void planar_bwd(const float (&z)[DM], float (&a)[DM], float* p, int d, float gl) {
  float u[DM], w[DM];
  float wtu = 0.0f, nw2 = 0.0f, s = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      u[j] = p[j];
      w[j] = p[d + j] + 1.0f;
      wtu += w[j] * u[j];
      nw2 += w[j] * w[j];
      s += w[j] * z[j];
    } else {
      u[j] = 0.0f;
      w[j] = 0.0f;
    }
  }
  s += p[2 * d];
  nw2 += 1e-9f;
  const float m = (-1.0f + softplus_tf<FAST>(wtu)) + 1e-5f;  // = w . u_hat (the constraint)
  const float c = m - wtu;
  const float sg = f_sigmoid<FAST>(wtu);
  const float cn = f_div_acc<FAST>(c, nw2);
  // tanh and its derivative from E = e^{-2|s|}: 1 - tanh^2 = 4E / (1 + E)^2 keeps its
  // relative accuracy where tanh saturates (1 - h*h would cancel to 0 or 1 ulp).
  const float E = f_exp<FAST>(-2.0f * fabsf(s));
  const float rE = f_div<FAST>(1.0f, 1.0f + E);
  float h;
  if constexpr (FAST)
    h = copysignf((1.0f - E) * rE, s);
  else
    h = tanhf(s);
  const float hp = 4.0f * E * rE * rE;
  float uh[DM];
  float ua = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    uh[j] = fmaf(cn, w[j], u[j]);
    ua += uh[j] * a[j];
  }
  // w . u_hat = wtu + c |w|^2 / n = m - c * 1e-9 / n, without the d-term cancellation
  const float q = m - cn * 1e-9f;
  const float hpd = gl * f_div<FAST>(hp, 1.0f + hp * q);
  const float Ss = hp * ua - 2.0f * q * h * hpd;
  float G[DM];
  float wG = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    G[j] = h * a[j] + hpd * w[j];
    wG += w[j] * G[j];
  }
  const float wGn = f_div<FAST>(wG, nw2);
  const float k1 = (sg - 1.0f) * wGn;
  const float k2 = 2.0f * cn * wGn;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      // d = 1: G - (1 - sg) (wG/n) w = G (1e-9 + sg w^2) / n exactly (no cancellation
      // when sg -> 0); for d > 1 the along-w cancellation is the reference's own.
      p[j] = d == 1 ? G[j] * f_div<FAST>(fmaf(sg * w[j], w[j], 1e-9f), nw2) : G[j] + k1 * w[j];
      p[d + j] = z[j] * Ss + hpd * uh[j] + cn * G[j] - k2 * w[j] + k1 * u[j];
      a[j] = fmaf(w[j], Ss, a[j]);
    }
  }
  p[2 * d] = Ss;
}

// Radial: alpha = softplus(0.3 a0 - 2), beta = softplus(0.1 b0 + log(e-1)) - 1,
// h = 1/(alpha + |z-gamma|_1), f = z + alpha beta h (z - gamma),
// ldj = (d-1) log(1 + ab h) + log(1 + ab alpha h^2)   (= the reference's
// 1 + ab h + ab h' r with h' = -h^2).
template <int DM, bool FAST>
__device__ __forceinline__ void radial_bwd(const float (&z)[DM], float (&a)[DM], float* p, int d, float gl) {
  const float xa = 0.3f * p[0] - 2.0f;
  const float xb = 0.1f * p[1] + kLogExpm1One;
  const float al = softplus_tf<FAST>(xa);
  const float be = softplus_tf<FAST>(xb) - 1.0f;
  float dz[DM];
  float r = 0.0f, da = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    dz[j] = j < d ? z[j] - p[2 + j] : 0.0f;
    r += fabsf(dz[j]);
    da += dz[j] * a[j];
  }
  const float h = f_div<FAST>(1.0f, al + r);
  const float hh = h * h;
  const float ab = al * be;
  const float A = 1.0f + ab * h;
  const float rB = f_div<FAST>(1.0f, 1.0f + ab * al * hh);
  const float dm1 = (float)(d - 1);
  const float rA = d > 1 ? f_div<FAST>(dm1, A) : 0.0f;  // (d-1) / A
  const float H = ab * da + gl * (ab * rA + 2.0f * ab * al * h * rB);
  const float g_ab = h * da + gl * (h * rA + al * hh * rB);
  const float g_al = be * g_ab + gl * ab * hh * rB - hh * H;
  const float hH = hh * H;
  const float abh = ab * h;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      const float sg = sign0(dz[j]);
      p[2 + j] = hH * sg - abh * a[j];
      a[j] = A * a[j] - hH * sg;
    }
  }
  p[0] = 0.3f * f_sigmoid<FAST>(xa) * g_al;
  p[1] = 0.1f * f_sigmoid<FAST>(xb) * al * g_ab;
}

// Affine: f = z * (1 + s) + shift, ldj = sum log|1 + s|.
template <int DM, bool FAST>
__device__ __forceinline__ void affine_bwd(const float (&z)[DM], float (&a)[DM], float* p, int d, float gl) {
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      const float sc = 1.0f + p[d + j];
      p[j] = a[j];
      p[d + j] = z[j] * a[j] + gl * f_div<FAST>(1.0f, sc);
      a[j] *= sc;
    }
  }
}

// Base MVNDiag(loc = t[:d], scale = 1e-3 + softplus(log(e-1) + 0.1 t[d:2d])), or N(0, I).
template <int DM, bool FAST>
__device__ __forceinline__ void base_bwd(const float (&z)[DM], float (&a)[DM], float* p, int d, bool trainable,
                                         float gl) {
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) {
      if (trainable) {
        const float xs = kLogExpm1One + 0.1f * p[d + j];
        const float rs = f_div<FAST>(1.0f, 1e-3f + softplus_tf<FAST>(xs));
        const float zz = (z[j] - p[j]) * rs;
        const float gz = gl * zz * rs;
        a[j] = -gz;
        p[j] = gz;
        p[d + j] = 0.1f * f_sigmoid<FAST>(xs) * gl * fmaf(zz, zz, -1.0f) * rs;
      } else {
        a[j] = -gl * z[j];
      }
    } else {
      a[j] = 0.0f;
    }
  }
}

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
__global__ void __launch_bounds__(64) chain_grad_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  const int R = ga.rows;
  const int S = a.lds_stride;
  const int d = a.d;
  const int K = a.prog.K;
  float* tile = lds;          // R rows x S
  float* zh = lds + R * S;    // flow inputs: zh[(k * d + j) * R + lane]
  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, a.B - b0);
  const bool tb = a.t_rowstride == 0;
  if (a.P > 0) stage_rows(tile, a.t + (tb ? 0 : b0 * a.t_rowstride), a.t_rowstride, nr, a.P, S, a.vec4 != 0);
  __syncthreads();
  if (lane < nr) {
    const int64_t b = b0 + lane;
    float* row = tile + lane * S;
    float z[DM];
    const float corr = load_y<DM, FAST>(z, a, b);
    float lp;
    if constexpr (DM == 1 && FAST) {
      // the forward kernels' own d = 1 evaluator (same functions, same order)
      float l2 = 0.0f;
      for (int k = 0; k < K; ++k) {
        const int st = a.prog.step[k];
        zh[k * R + lane] = z[0];
        float pc[3];
        read3(pc, row, st);
        l2 += __builtin_amdgcn_logf(fabsf(flow1_fast(st & 3, z[0], pc)));
      }
      lp = base1_fast(z[0], row, a.trainable != 0) + l2 * kLn2 - corr;
    } else {
      float ildj = 0.0f;
      for (int k = 0; k < K; ++k) {
        const int st = a.prog.step[k];
#pragma unroll
        for (int j = 0; j < DM; ++j)
          if (j < d) zh[(k * d + j) * R + lane] = z[j];
        ildj = ildj + flow_step<DM, FAST>(st & 3, z, row + (st >> 2), d);
      }
      lp = base_log_prob<DM, FAST>(z, row, d, a.trainable != 0) + ildj - corr;
    }
    if (a.out) a.out[b] = lp;
    const float gl = ga.g_out ? ga.g_out[b] : 1.0f;
    float adj[DM];
    base_bwd<DM, FAST>(z, adj, row, d, a.trainable != 0, gl);
    for (int k = K - 1; k >= 0; --k) {
      const int st = a.prog.step[k];
      float zk[DM];
#pragma unroll
      for (int j = 0; j < DM; ++j) zk[j] = j < d ? zh[(k * d + j) * R + lane] : 0.0f;
      float* p = row + (st >> 2);
      const int id = st & 3;
      if (id == NFN_FLOW_PLANAR)
        planar_bwd<DM, FAST>(zk, adj, p, d, gl);
      else if (id == NFN_FLOW_RADIAL)
        radial_bwd<DM, FAST>(zk, adj, p, d, gl);
      else
        affine_bwd<DM, FAST>(zk, adj, p, d, gl);
    }
    if (ga.grad_y) {
#pragma unroll
      for (int j = 0; j < DM; ++j)
        if (j < d) ga.grad_y[b * d + j] = a.y_std ? f_div<FAST>(adj[j], a.y_std[j]) : adj[j];
    }
  }
  __syncthreads();
  if (ga.grad_t && a.P > 0) store_rows(tile, ga.grad_t + b0 * ga.gt_rowstride, ga.gt_rowstride, nr, a.P, S,
                                       ga.gt_vec4 != 0);
}

template <bool FAST>
void launch_grad_t(int dm, const GradArgs& ga, dim3 grid, size_t lds, hipStream_t s) {
  switch (dm) {
    case 1: chain_grad_kernel<1, FAST><<<grid, 64, lds, s>>>(ga); break;
    case 2: chain_grad_kernel<2, FAST><<<grid, 64, lds, s>>>(ga); break;
    case 4: chain_grad_kernel<4, FAST><<<grid, 64, lds, s>>>(ga); break;
    case 8: chain_grad_kernel<8, FAST><<<grid, 64, lds, s>>>(ga); break;
    case 16: chain_grad_kernel<16, FAST><<<grid, 64, lds, s>>>(ga); break;
    default: chain_grad_kernel<32, FAST><<<grid, 64, lds, s>>>(ga); break;
  }
}

}  // namespace

void launch_grad(bool fast, int dm, const GradArgs& ga, dim3 grid, size_t lds, hipStream_t s) {
  if (fast)
    launch_grad_t<true>(dm, ga, grid, lds, s);
  else
    launch_grad_t<false>(dm, ga, grid, lds, s);
}

}  // namespace nfn
