// nfn_sample.hip — sampling through the inverted flows.
// The reference cannot sample: its layer inverts the chain for fast densities and
// TFP would need each flow's _inverse, which PlanarFlow / RadialFlow do not define
// (DistributionLayers.py:223-226, 240).  Here the distribution's sampling map is
//   y = f_0^{-1}( f_1^{-1}( ... f_{K-1}^{-1}( loc + scale * eps ) ) )
// with the flows of the reversed layout (DistributionLayers.py:267-278):
//   * planar: z_out = z + u_hat tanh(w.z + b) is solved along w: c = w.z satisfies
//     c + q tanh(c + b) = w.z_out with q = w.u_hat >= -1 + 1e-5 (the constraint of
//     PlanarFlow._u_circ makes the left side strictly increasing), by Newton steps
//     safeguarded with bisection on the bracket [w.z_out - |q|, w.z_out + |q|]
//     (the rtsafe scheme);
//     then z = z_out - u_hat tanh(c + b);
//   * radial (L1 norm, RadialFlow._r): z - gamma keeps its direction, and
//     r' = r (1 + alpha beta / (alpha + r)) is a quadratic in r with one root >= 0;
//   * affine: z = (z_out - shift) / scale.
// The log-density of each sample, logp(y) = log N(z_K) + sum_k fldj_k(z_k), comes
// out of the same walk (every z_k is known once inverted).
#include "nfn_launch.h"

namespace nfn {
namespace {

template <int DM, bool FAST>
__device__ __forceinline__ void planar_inv(float (&z)[DM], const float* p, int d) {
  float u[DM], w[DM];
  float wtu = 0.0f, nw2 = 0.0f, wzo = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    u[j] = j < d ? p[j] : 0.0f;
    w[j] = j < d ? p[d + j] + 1.0f : 0.0f;
    wtu += w[j] * u[j];
    nw2 += w[j] * w[j];
    wzo += w[j] * z[j];
  }
  const float b = p[2 * d];
  const float m = (-1.0f + softplus_tf<FAST>(wtu)) + 1e-5f;
  const float cn = f_div_acc<FAST>(m - wtu, nw2 + 1e-9f);
  float uh[DM];
  float q = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    uh[j] = fmaf(cn, w[j], u[j]);
    q += w[j] * uh[j];
  }
  // solve g(c) = c + q tanh(c + b) - wzo = 0 (g increasing) by Newton steps kept
  // inside the bracket, falling back to bisection whenever a step leaves it or
  // does not halve the previous one (q > 1 gives g an inflection Newton would
  // oscillate across)
  float lo = wzo - fabsf(q), hi = wzo + fabsf(q);
  float c = fminf(fmaxf(wzo - q * tanhf(wzo + b), lo), hi);
  float dxold = hi - lo, dx = dxold;
  float th = tanhf(c + b);
  float g = c + q * th - wzo;
  float dg = 1.0f + q * (1.0f - th * th);
  for (int it = 0; it < 60; ++it) {
    if (((c - hi) * dg - g) * ((c - lo) * dg - g) > 0.0f || fabsf(2.0f * g) > fabsf(dxold * dg)) {
      dxold = dx;
      dx = 0.5f * (hi - lo);
      c = lo + dx;
    } else {
      dxold = dx;
      dx = g / dg;
      c = c - dx;
    }
    if (!(fabsf(dx) > 1e-7f * fmaxf(1.0f, fabsf(c)))) break;  // converged (or NaN input)
    th = tanhf(c + b);
    g = c + q * th - wzo;
    dg = 1.0f + q * (1.0f - th * th);
    if (g < 0.0f)
      lo = c;
    else
      hi = c;
  }
  th = tanhf(c + b);
#pragma unroll
  for (int j = 0; j < DM; ++j)
    if (j < d) z[j] = z[j] - uh[j] * th;
}

template <int DM, bool FAST>
__device__ __forceinline__ void radial_inv(float (&z)[DM], const float* p, int d) {
  const float al = softplus_alpha<FAST>(0.3f * p[0] - 2.0f);
  const float be = softplus_tf<FAST>(0.1f * p[1] + kLogExpm1One) - 1.0f;
  float ro = 0.0f;
#pragma unroll
  for (int j = 0; j < DM; ++j)
    if (j < d) ro += fabsf(z[j] - p[2 + j]);
  // r^2 + A r - al ro = 0 with A = al (1 + be) - ro; the stable root form
  const float A = al * (1.0f + be) - ro;
  const float disc = sqrtf(fmaf(A, A, 4.0f * al * ro));
  const float r = A > 0.0f ? (2.0f * al * ro) / (A + disc) : 0.5f * (disc - A);
  const float s = 1.0f + (al * be) / (al + r);
#pragma unroll
  for (int j = 0; j < DM; ++j)
    if (j < d) z[j] = p[2 + j] + (z[j] - p[2 + j]) / s;
}

template <int DM>
__device__ __forceinline__ void affine_inv(float (&z)[DM], const float* p, int d) {
#pragma unroll
  for (int j = 0; j < DM; ++j)
    if (j < d) z[j] = (z[j] - p[j]) / (1.0f + p[d + j]);
}

template <int DM, bool FAST>
__global__ void __launch_bounds__(kMaxBlock) chain_sample_kernel(SampleArgs sa) {
  const ChainArgs& a = sa.c;
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
  const float* row = lds + (tb ? 0 : tid * a.lds_stride);
  const float* e = sa.eps + b * sa.eps_bstride;
  float z[DM];
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    z[j] = 0.0f;
    if (j < d) {
      if (a.trainable) {
        const float sc = 1e-3f + softplus_tf<FAST>(kLogExpm1One + 0.1f * row[d + j]);
        z[j] = fmaf(sc, e[j], row[j]);
      } else {
        z[j] = e[j];
      }
    }
  }
  for (int k = a.prog.K - 1; k >= 0; --k) {
    const int st = a.prog.step[k];
    const float* p = row + (st >> 2);
    const int id = st & 3;
    if (id == NFN_FLOW_PLANAR)
      planar_inv<DM, FAST>(z, p, d);
    else if (id == NFN_FLOW_RADIAL)
      radial_inv<DM, FAST>(z, p, d);
    else
      affine_inv<DM>(z, p, d);
  }
  // z is now the sample in the flow's (normalised) y space
  if (sa.logp) {
    float zf[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) zf[j] = z[j];
    float ildj = 0.0f;
    for (int k = 0; k < a.prog.K; ++k) {
      const int st = a.prog.step[k];
      ildj = ildj + flow_step<DM, FAST>(st & 3, zf, row + (st >> 2), d);
    }
    float lp = base_log_prob<DM, FAST>(zf, row, d, a.trainable != 0) + ildj;
    if (a.y_mean) {
      for (int j = 0; j < d; ++j) lp -= f_log<FAST>(a.y_std[j]);
    }
    sa.logp[b] = lp;
  }
#pragma unroll
  for (int j = 0; j < DM; ++j) {
    if (j < d) sa.y_out[b * d + j] = a.y_mean ? fmaf(z[j], a.y_std[j], a.y_mean[j]) : z[j];
  }
}

template <bool FAST>
void launch_sample_t(int dm, const SampleArgs& sa, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  switch (dm) {
    case 1: nfn_launch((chain_sample_kernel<1, FAST>), grid, block, lds, s, sa); break;
    case 2: nfn_launch((chain_sample_kernel<2, FAST>), grid, block, lds, s, sa); break;
    case 4: nfn_launch((chain_sample_kernel<4, FAST>), grid, block, lds, s, sa); break;
    case 8: nfn_launch((chain_sample_kernel<8, FAST>), grid, block, lds, s, sa); break;
    case 16: nfn_launch((chain_sample_kernel<16, FAST>), grid, block, lds, s, sa); break;
    default: nfn_launch((chain_sample_kernel<32, FAST>), grid, block, lds, s, sa); break;
  }
}

}  // namespace

void launch_sample(bool fast, int dm, const SampleArgs& sa, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  if (fast)
    launch_sample_t<true>(dm, sa, grid, block, lds, s);
  else
    launch_sample_t<false>(dm, sa, grid, block, lds, s);
}

}  // namespace nfn
