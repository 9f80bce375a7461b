// nfn_grad_device.h — closed-form adjoints of the flow chain,
// shared by the backward kernels (nfn_grad.hip, nfn_grad_group.hip).
//
// `a` enters as d logp / d z_{k+1} and leaves as d logp / d z_k; `gl` is the
// adjoint of every log-det term (the upstream gradient g_b); each flow overwrites
// its own parameter block with d logp / d (its parameters).  What Keras autodiff
// computes through PlanarFlow.py:43-80, RadialFlow.py:44-84, AffineFlow.py:4-9 and
// DistributionLayers.py:280-294 when the reference trains.
// Derivations: tests/analytic_grad.py (checked against autodiff in fp64).
#pragma once

#include "nfn_device.h"

// Contraction of a * b + c into an fma only within one source expression (as written),
// never by the backend across expressions: the adjoints are then evaluated the same way
// in every kernel that inlines them (one or two samples per lane, any chain form), so the
// backward kernels agree bitwise.  (The build default, fast-honor-pragmas, lets the backend
// fuse across statements, and its choices follow the surrounding code.)  Restored at the
// end of this header.  Measured cost on the C2 backward: none (profiles/r04/r04c_*).
#pragma clang fp contract(on)

namespace nfn {

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
  const float sp = softplus_alpha<FAST>(wtu);  // relative accuracy as w.u -> -inf
  const float m = (-1.0f + sp) + 1e-5f;        // = w . u_hat (the constraint)
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
    // d = 1: (1e-9 u + m w) / n, the well-conditioned form of planar_step
    uh[j] = d == 1 ? f_div_acc<FAST>(fmaf(u[j], 1e-9f, m * w[j]), nw2) : fmaf(cn, w[j], u[j]);
    ua += uh[j] * a[j];
  }
  // w . u_hat = wtu + c |w|^2 / n = m - c * 1e-9 / n, without the d-term cancellation;
  // det = 1 + hp q = h^2 + hp (softplus + 1e-5 - c 1e-9 / n), without the q -> -1 one
  const float q = m - cn * 1e-9f;
  const float hpd = gl * f_div<FAST>(hp, fmaf(h, h, hp * ((sp + 1e-5f) - cn * 1e-9f)));
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
  const float al = softplus_alpha<FAST>(xa);
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

// ---------------------------------------------------------------------------
// d = 1, fast math: scalar forms of the same adjoints with the transcendentals
// shared (softplus and sigmoid from one exponential, one reciprocal of |w|^2).
// ---------------------------------------------------------------------------

// softplus(x) and sigmoid(x) from e = e^{-|x|}: sigmoid = 1/(1+e) (x >= 0) or e/(1+e).
template <bool ACC = false>
__device__ __forceinline__ void sp_sig1(float x, float& sp, float& sg) {
  const float e = __builtin_amdgcn_exp2f(-fabsf(x) * kLog2e);
  const float r = __builtin_amdgcn_rcpf(1.0f + e);
  if constexpr (ACC)
    sp = softplus_acc_fast(x, e);
  else
    sp = fmaf(__builtin_amdgcn_logf(1.0f + e), kLn2, fmaxf(x, 0.0f));
  sg = x >= 0.0f ? r : e * r;
}

// z-only forward steps (the backward needs each flow's input, not its log-det).
// (planar1_fast<false>'s z update, bitwise: the backward keeps round 5's m, see planar1_fast)
__device__ __forceinline__ void planar1_z(float& z, float u, float wraw, float b) {
  const float w = wraw + 1.0f;
  const float wtu = w * u;
  const float nw2 = fmaf(w, w, 1e-9f);
  const float m = softplus_alpha<true>(wtu) - (1.0f - 1e-5f);
  const float uh = planar1_uh(u, w, __builtin_amdgcn_rcpf(nw2), m);
  z = fmaf(uh, tanh_fast(fmaf(w, z, b)), z);
}

__device__ __forceinline__ void radial1_z(float& z, float a0, float b0, float g) {
  const float alpha = softplus_alpha<true>(fmaf(0.3f, a0, -2.0f));
  const float ab = fmaf(alpha, sp_fast1(fmaf(0.1f, b0, kLogExpm1One)), -alpha);
  const float dz = z - g;
  z = fmaf(ab * __builtin_amdgcn_rcpf(alpha + fabsf(dz)), dz, z);
}

// (p0, p1, p2): the flow's parameters (already read); `p`: where its gradient goes
// (ST floats between consecutive parameters: 1 = row-major tile, the fused Dense
// backward's column-major tile uses its padded column stride).
template <int ST = 1>
__device__ __forceinline__ void planar1_bwd(float z, float& a, float p0, float p1, float p2, float* p, float gl) {
  const float u = p0;
  const float w = p1 + 1.0f;
  const float wtu = w * u;
  float sp, sg;
  sp_sig1<true>(wtu, sp, sg);
  const float m = (sp - 1.0f) + 1e-5f;
  const float c = m - wtu;
  const float nw2 = fmaf(w, w, 1e-9f);
  const float rn = __builtin_amdgcn_rcpf(nw2);
  const float q0 = c * rn;
  const float cn = fmaf(fmaf(-nw2, q0, c), rn, q0);  // c / n, Newton-refined
  const float uh = planar1_uh(u, w, rn, m);  // (planar1_fast's well-conditioned form)
  const float s = fmaf(w, z, p2);
  const float E = __builtin_amdgcn_exp2f(fabsf(s) * (-2.0f * kLog2e));
  const float rE = __builtin_amdgcn_rcpf(1.0f + E);
  const float h = copysignf((1.0f - E) * rE, s);
  const float hp = 4.0f * E * rE * rE;
  const float q = fmaf(-cn, 1e-9f, m);
  // det = 1 + hp q = h^2 + hp (softplus + 1e-5 - cn 1e-9): no cancellation as q -> -1
  const float hpd = gl * hp * __builtin_amdgcn_rcpf(fmaf(h, h, hp * fmaf(-cn, 1e-9f, sp + 1e-5f)));
  const float Ss = fmaf(hp, uh * a, -2.0f * q * h * hpd);
  const float G = fmaf(h, a, hpd * w);
  const float wGn = w * G * rn;
  const float k1 = (sg - 1.0f) * wGn;
  p[0] = G * (fmaf(sg * w, w, 1e-9f) * rn);
  p[ST] = fmaf(z, Ss, fmaf(hpd, uh, fmaf(cn, G, fmaf(-2.0f * cn * wGn, w, k1 * u))));
  p[2 * ST] = Ss;
  a = fmaf(w, Ss, a);
}

template <int ST = 1>
__device__ __forceinline__ void radial1_bwd(float z, float& a, float p0, float p1, float p2, float* p, float gl) {
  const float xa = fmaf(0.3f, p0, -2.0f);
  const float xb = fmaf(0.1f, p1, kLogExpm1One);
  float al, sga, spb, sgb;
  sp_sig1<true>(xa, al, sga);  // relative accuracy as alpha -> 0 (softplus_alpha)
  sp_sig1(xb, spb, sgb);
  const float be = spb - 1.0f;
  const float dz = z - p2;
  const float h = __builtin_amdgcn_rcpf(al + fabsf(dz));
  const float hh = h * h;
  const float ab = fmaf(al, spb, -al);
  const float rB = __builtin_amdgcn_rcpf(fmaf(ab * al, hh, 1.0f));
  const float da = dz * a;
  const float glr = gl * rB;
  const float H = fmaf(ab, da, 2.0f * ab * al * h * glr);
  const float g_ab = fmaf(h, da, al * hh * glr);
  const float g_al = fmaf(be, g_ab, ab * hh * glr) - hh * H;
  const float hH = hh * H;
  const float sg = sign0(dz);
  p[0] = 0.3f * sga * g_al;
  p[ST] = 0.1f * sgb * al * g_ab;
  p[2 * ST] = fmaf(hH, sg, -ab * h * a);
  a = fmaf(fmaf(ab, h, 1.0f), a, -hH * sg);
}

template <int ST = 1>
__device__ __forceinline__ void affine1_bwd(float z, float& a, float p0, float p1, float* p, float gl) {
  (void)p0;
  const float sc = 1.0f + p1;
  p[0] = a;
  p[ST] = fmaf(z, a, gl * __builtin_amdgcn_rcpf(sc));
  a *= sc;
}

template <int ST = 1>
__device__ __forceinline__ void flow1_bwd(int id, float z, float& a, const float (&pv)[3], float* p, float gl) {
  if (id == NFN_FLOW_PLANAR)
    planar1_bwd<ST>(z, a, pv[0], pv[1], pv[2], p, gl);
  else if (id == NFN_FLOW_RADIAL)
    radial1_bwd<ST>(z, a, pv[0], pv[1], pv[2], p, gl);
  else
    affine1_bwd<ST>(z, a, pv[0], pv[1], p, gl);
}

// d = 1, fast math, chains of <= 16 flows with the packed program (types 2 bits
// per flow; offsets by scalar arithmetic: no scalar-memory loads inside the
// loops, whose lgkmcnt(0) waits would drain the pipelined LDS reads).  Both
// passes read the NEXT flow's parameters (and, in reverse, its input z) from LDS
// before evaluating the current flow.  ST: floats between a sample's consecutive
// parameters (see planar1_bwd).
// Called once between the forward and the reverse pass of grad1_packed / grad1_pairs
// (the streaming backward may issue part of its next-tile prefetch there).
struct NoMid {
  __device__ __forceinline__ void operator()() const {}
};

template <int ST = 1, class Mid = NoMid>
__device__ __forceinline__ float grad1_packed(float& z, float* row, float* zh, int zs, uint32_t types, int K, int P,
                                              bool trainable, float gl, bool want_lp, float& adj,
                                              const Mid& mid = Mid{}) {
  float l2 = 0.0f;
  int id = (int)(types & 3u);
  int off = max(P - size1(id), 0);
  float pc[3];
  if (K > 0) read3c<ST>(pc, row, off);
#pragma unroll 1
  for (int k = 0; k < 16; ++k) {
    if (k < K) {
      const int idn = (int)((types >> (2 * (k + 1) & 31)) & 3u);
      const int offn = max(off - size1(idn), 0);
      float pn[3];
      read3c<ST>(pn, row, offn);
      zh[k * zs] = z;
      if (want_lp) {
        l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(id, z, pc)));
      } else if (id == NFN_FLOW_PLANAR) {
        planar1_z(z, pc[0], pc[1], pc[2]);
      } else if (id == NFN_FLOW_RADIAL) {
        radial1_z(z, pc[0], pc[1], pc[2]);
      } else {
        z = fmaf(z, 1.0f + pc[1], pc[0]);
      }
      id = idn;
      off = offn;
      pc[0] = pn[0];
      pc[1] = pn[1];
      pc[2] = pn[2];
    }
  }
  const float lp = want_lp ? base1_fast<ST>(z, row, trainable) + l2 * kLn2 : 0.0f;
  mid();
  float a1;
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[ST], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    a1 = -gz;
    row[0] = gz;
    row[ST] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
  } else {
    a1 = -gl * z;
  }
  // reverse: flow K-1's block follows the base, flow k-1's follows flow k's
  int ob = trainable ? 2 : 0;
  int ib = (int)((types >> (2 * (K - 1) & 31)) & 3u);
  float pb[3] = {0.0f, 0.0f, 0.0f};
  float zb = 0.0f;
  if (K > 0) {
    read3c<ST>(pb, row, ob);
    zb = zh[(K - 1) * zs];
  }
#pragma unroll 1
  for (int k = 15; k >= 0; --k) {
    if (k < K) {
      const int ip = (int)((types >> (2 * (k - 1) & 31)) & 3u);
      const int op = min(ob + size1(ib), P - 1);  // k = 0: a harmless in-slot read
      float pp[3];
      read3c<ST>(pp, row, op);
      const float zp = zh[max(k - 1, 0) * zs];
      flow1_bwd<ST>(ib, zb, a1, pb, row + ob * ST, gl);
      ib = ip;
      ob = op;
      pb[0] = pp[0];
      pb[1] = pp[1];
      pb[2] = pp[2];
      zb = zp;
    }
  }
  adj = a1;
  return lp;
}


// The base density's adjoint (grad1_packed's, row-major tile): writes d/d(loc, scale
// param) into row[0..1] and returns d log_prob / d z_K.
__device__ __forceinline__ float base1_bwd(float z, float* row, bool trainable, float gl) {
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[1], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    row[0] = gz;
    row[1] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
    return -gz;
  }
  return -gl * z;
}

// grad1_packed for TWO samples per lane (the rows ra, rb of one wave tile, flow inputs at
// zha / zhb) under ONE walk of the program: the flow dispatch, the block offsets and the
// parameter-read schedule are shared, and the two samples' arithmetic forms two
// independent dependency chains for the scheduler to interleave — the streaming backward
// (chain_grad_wave2_kernel) then hides the chain's latency with half the resident waves.
// Per sample it is exactly grad1_packed's arithmetic in grad1_packed's order (bitwise).
template <class Mid = NoMid>
__device__ __forceinline__ void grad1_packed2(float& za, float& zb, float* ra, float* rb, float* zha, float* zhb,
                                              int zs, uint32_t types, int K, int P, bool trainable, float gla,
                                              float glb, bool want_lp, float& adja, float& adjb, float& lpa,
                                              float& lpb, const Mid& mid = Mid{}) {
  float l2a = 0.0f, l2b = 0.0f;
  int id = (int)(types & 3u);
  int off = max(P - size1(id), 0);
  float pa[3], pb[3];
  if (K > 0) {
    read3c(pa, ra, off);
    read3c(pb, rb, off);
  }
#pragma unroll 1
  for (int k = 0; k < 16; ++k) {
    if (k < K) {
      const int idn = (int)((types >> (2 * (k + 1) & 31)) & 3u);
      const int offn = max(off - size1(idn), 0);
      float na[3], nb[3];
      read3c(na, ra, offn);
      read3c(nb, rb, offn);
      zha[k * zs] = za;
      zhb[k * zs] = zb;
      if (id == NFN_FLOW_PLANAR) {
        if (want_lp) {
          l2a += __builtin_amdgcn_logf(fabsf(planar1_fast<false>(za, pa[0], pa[1], pa[2])));
          l2b += __builtin_amdgcn_logf(fabsf(planar1_fast<false>(zb, pb[0], pb[1], pb[2])));
        } else {
          planar1_z(za, pa[0], pa[1], pa[2]);
          planar1_z(zb, pb[0], pb[1], pb[2]);
        }
      } else if (id == NFN_FLOW_RADIAL) {
        if (want_lp) {
          l2a += __builtin_amdgcn_logf(fabsf(radial1_fast(za, pa[0], pa[1], pa[2])));
          l2b += __builtin_amdgcn_logf(fabsf(radial1_fast(zb, pb[0], pb[1], pb[2])));
        } else {
          radial1_z(za, pa[0], pa[1], pa[2]);
          radial1_z(zb, pb[0], pb[1], pb[2]);
        }
      } else {
        if (want_lp) {
          l2a += __builtin_amdgcn_logf(fabsf(affine1_fast(za, pa[0], pa[1])));
          l2b += __builtin_amdgcn_logf(fabsf(affine1_fast(zb, pb[0], pb[1])));
        } else {
          za = fmaf(za, 1.0f + pa[1], pa[0]);
          zb = fmaf(zb, 1.0f + pb[1], pb[0]);
        }
      }
      id = idn;
      off = offn;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pa[i] = na[i];
        pb[i] = nb[i];
      }
    }
  }
  lpa = want_lp ? base1_fast<1>(za, ra, trainable) + l2a * kLn2 : 0.0f;
  lpb = want_lp ? base1_fast<1>(zb, rb, trainable) + l2b * kLn2 : 0.0f;
  mid();
  float a1a = base1_bwd(za, ra, trainable, gla);
  float a1b = base1_bwd(zb, rb, trainable, glb);
  int ob = trainable ? 2 : 0;
  int ib = (int)((types >> (2 * (K - 1) & 31)) & 3u);
  float qa[3] = {0.0f, 0.0f, 0.0f}, qb[3] = {0.0f, 0.0f, 0.0f};
  float zba = 0.0f, zbb = 0.0f;
  if (K > 0) {
    read3c(qa, ra, ob);
    read3c(qb, rb, ob);
    zba = zha[(K - 1) * zs];
    zbb = zhb[(K - 1) * zs];
  }
#pragma unroll 1
  for (int k = 15; k >= 0; --k) {
    if (k < K) {
      const int ip = (int)((types >> (2 * (k - 1) & 31)) & 3u);
      const int op = min(ob + size1(ib), P - 1);  // k = 0: a harmless in-slot read
      float ppa[3], ppb[3];
      read3c(ppa, ra, op);
      read3c(ppb, rb, op);
      const float zpa = zha[max(k - 1, 0) * zs];
      const float zpb = zhb[max(k - 1, 0) * zs];
      if (ib == NFN_FLOW_PLANAR) {
        planar1_bwd(zba, a1a, qa[0], qa[1], qa[2], ra + ob, gla);
        planar1_bwd(zbb, a1b, qb[0], qb[1], qb[2], rb + ob, glb);
      } else if (ib == NFN_FLOW_RADIAL) {
        radial1_bwd(zba, a1a, qa[0], qa[1], qa[2], ra + ob, gla);
        radial1_bwd(zbb, a1b, qb[0], qb[1], qb[2], rb + ob, glb);
      } else {
        affine1_bwd(zba, a1a, qa[0], qa[1], ra + ob, gla);
        affine1_bwd(zbb, a1b, qb[0], qb[1], rb + ob, glb);
      }
      ib = ip;
      ob = op;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        qa[i] = ppa[i];
        qb[i] = ppb[i];
      }
      zba = zpa;
      zbb = zpb;
    }
  }
  adja = a1a;
  adjb = a1b;
}

// grad1_packed with two flows per dispatch in both passes (chain1_fast_pairs): each of
// the nine (type, type) bodies is straight-line code.  Same arithmetic in the same
// order as grad1_packed.
__device__ __forceinline__ void flow1_z(int id, float& z, const float (&p)[3]) {
  if (id == NFN_FLOW_PLANAR)
    planar1_z(z, p[0], p[1], p[2]);
  else if (id == NFN_FLOW_RADIAL)
    radial1_z(z, p[0], p[1], p[2]);
  else
    z = fmaf(z, 1.0f + p[1], p[0]);
}

template <int IA, int IB>
__device__ __forceinline__ void fwd_pair1(float& z, float& l2, float& za, float& zb, const float (&pa)[3],
                                          const float (&pb)[3], bool want_lp) {
  za = z;
  if (want_lp)
    l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(IA, z, pa)));
  else
    flow1_z(IA, z, pa);
  zb = z;
  if (want_lp)
    l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(IB, z, pb)));
  else
    flow1_z(IB, z, pb);
}

template <int IA, int IB, int ST>
__device__ __forceinline__ void bwd_pair1(float& a1, float* row, float za, float zb, const float (&pa)[3],
                                          const float (&pb)[3], int oba, int obb, float gl) {
  flow1_bwd<ST>(IA, za, a1, pa, row + oba * ST, gl);
  flow1_bwd<ST>(IB, zb, a1, pb, row + obb * ST, gl);
}

template <int ST = 1, class Mid = NoMid>
__device__ __forceinline__ float grad1_pairs(float& z, float* row, float* zh, int zs, uint32_t types, int K, int P,
                                             bool trainable, float gl, bool want_lp, float& adj,
                                             const Mid& mid = Mid{}) {
  float l2 = 0.0f;
  int ia = type1(types, 0), ib = type1(types, 1);
  int offa = max(P - size1(ia), 0), offb = max(offa - size1(ib), 0);
  float pa[3] = {0.0f, 0.0f, 0.0f}, pb[3] = {0.0f, 0.0f, 0.0f};
  if (K > 0) {
    read3c<ST>(pa, row, offa);
    read3c<ST>(pb, row, offb);
  }
  int k = 0;
#pragma unroll 1
  for (; k + 1 < K; k += 2) {
    const int ian = type1(types, k + 2), ibn = type1(types, k + 3);
    const int offan = max(offb - size1(ian), 0), offbn = max(offan - size1(ibn), 0);
    float pna[3], pnb[3];
    read3c<ST>(pna, row, offan);
    read3c<ST>(pnb, row, offbn);
    float za, zb;
#define NFN_FWD(A, B) fwd_pair1<A, B>(z, l2, za, zb, pa, pb, want_lp)
    NFN_PAIR_SWITCH(ia * 3 + ib, NFN_FWD)
#undef NFN_FWD
    zh[k * zs] = za;
    zh[(k + 1) * zs] = zb;
    ia = ian;
    ib = ibn;
    offb = offbn;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pa[i] = pna[i];
      pb[i] = pnb[i];
    }
  }
  if (K & 1) {  // the last flow: already read
    zh[(K - 1) * zs] = z;
    if (want_lp)
      l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(ia, z, pa)));
    else
      flow1_z(ia, z, pa);
  }
  const float lp = want_lp ? base1_fast<ST>(z, row, trainable) + l2 * kLn2 : 0.0f;
  mid();
  float a1;
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[ST], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    a1 = -gz;
    row[0] = gz;
    row[ST] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
  } else {
    a1 = -gl * z;
  }
  // reverse, flows K-1, K-2, ... in pairs: flow K-1's block follows the base, flow
  // k-1's follows flow k's; the next pair's parameters and inputs are read first
  k = K - 1;
  ia = type1(types, k);
  ib = type1(types, k - 1);
  int oba = min(trainable ? 2 : 0, P - 1);
  int obb = min(oba + size1(ia), P - 1);
  float za = 0.0f, zb = 0.0f;
  if (K > 0) {
    read3c<ST>(pa, row, oba);
    read3c<ST>(pb, row, obb);
    za = zh[k * zs];
    zb = zh[max(k - 1, 0) * zs];
  }
#pragma unroll 1
  for (; k >= 1; k -= 2) {
    const int ian = type1(types, k - 2), ibn = type1(types, k - 3);
    const int oban = min(obb + size1(ib), P - 1), obbn = min(oban + size1(ian), P - 1);
    float pna[3], pnb[3];
    read3c<ST>(pna, row, oban);
    read3c<ST>(pnb, row, obbn);
    const float zan = zh[max(k - 2, 0) * zs], zbn = zh[max(k - 3, 0) * zs];
#define NFN_BWD(A, B) bwd_pair1<A, B, ST>(a1, row, za, zb, pa, pb, oba, obb, gl)
    NFN_PAIR_SWITCH(ia * 3 + ib, NFN_BWD)
#undef NFN_BWD
    ia = ian;
    ib = ibn;
    oba = oban;
    obb = obbn;
    za = zan;
    zb = zbn;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pa[i] = pna[i];
      pb[i] = pnb[i];
    }
  }
  if (k == 0) flow1_bwd<ST>(ia, za, a1, pa, row + oba * ST, gl);  // flow 0: already read
  adj = a1;
  return lp;
}

// grad1_pairs for a program alternating two types (IA, IB, IA, ...: chain1_fast_hpairs):
// the pair bodies and block offsets are compile-time, no dispatch.  The same fwd_pair1 /
// bwd_pair1 calls on the same values as grad1_pairs.
template <int IA, int IB, int ST, bool ODD>
__device__ __forceinline__ float hpair_reverse(float* row, const float* zh, int zs, int K, int P, int ob0, float gl,
                                               float a1) {
  // flows K-1, K-2, ... in pairs; K even: (IB, IA) pairs, K odd: (IA, IB) then flow 0 (IA)
  constexpr int TA = ODD ? IA : IB, TB = ODD ? IB : IA;
  constexpr int SA = TA == NFN_FLOW_AFFINE ? 2 : 3, SP = SA + (TB == NFN_FLOW_AFFINE ? 2 : 3);
  int oba = ob0;
  int k = K - 1;
  float pa[3], pb[3];
  read3c<ST>(pa, row, min(oba, P - 1));
  read3c<ST>(pb, row, min(oba + SA, P - 1));
  float za = zh[k * zs], zb = zh[max(k - 1, 0) * zs];
#pragma unroll 1
  for (; k >= 1; k -= 2) {
    const int oban = oba + SP;
    float pna[3], pnb[3];
    read3c<ST>(pna, row, min(oban, P - 1));
    read3c<ST>(pnb, row, min(oban + SA, P - 1));
    const float zan = zh[max(k - 2, 0) * zs], zbn = zh[max(k - 3, 0) * zs];
    bwd_pair1<TA, TB, ST>(a1, row, za, zb, pa, pb, oba, oba + SA, gl);
    oba = oban;
    za = zan;
    zb = zbn;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pa[i] = pna[i];
      pb[i] = pnb[i];
    }
  }
  if constexpr (ODD) flow1_bwd<ST>(IA, za, a1, pa, row + oba * ST, gl);  // flow 0: already read
  return a1;
}

// grad1_hpairs with the flow inputs in registers: both passes unrolled over up to 8 pairs
// (each guarded by the runtime pair count), so z_k needs no LDS round trip; the per-flow
// adjoints run in the same order (K-1 .. 0) on the same values as grad1_pairs.
template <int IA, int IB, int ST = 1>
__device__ __forceinline__ float grad1_hpairs_regs(float& z, float* row, int K, int P, bool trainable, float gl,
                                                   bool want_lp, float& adj) {
  constexpr int SA = IA == NFN_FLOW_AFFINE ? 2 : 3, SB = IB == NFN_FLOW_AFFINE ? 2 : 3, SP = SA + SB;
  constexpr int kNP = 8;
  float zk[2 * kNP];
  float l2 = 0.0f;
  const int np = K >> 1;
#pragma unroll
  for (int p = 0; p < kNP; ++p) {
    zk[2 * p] = zk[2 * p + 1] = 0.0f;
    if (p < np) {
      float pa[3], pb[3];
      read3c<ST>(pa, row, P - p * SP - SA);
      read3c<ST>(pb, row, P - (p + 1) * SP);
      fwd_pair1<IA, IB>(z, l2, zk[2 * p], zk[2 * p + 1], pa, pb, want_lp);
    }
  }
  float zl = 0.0f;  // the input of flow K - 1 when K is odd
  if (K & 1) {
    float pa[3];
    read3c<ST>(pa, row, P - np * SP - SA);
    zl = z;
    if (want_lp)
      l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(IA, z, pa)));
    else
      flow1_z(IA, z, pa);
  }
  const float lp = want_lp ? base1_fast<ST>(z, row, trainable) + l2 * kLn2 : 0.0f;
  float a1;
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[ST], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    a1 = -gz;
    row[0] = gz;
    row[ST] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
  } else {
    a1 = -gl * z;
  }
  // reverse: flow K-1's block follows the base, flow k-1's follows flow k's
  int ob = trainable ? 2 : 0;
  if (K & 1) {
    float pa[3];
    read3c<ST>(pa, row, ob);
    flow1_bwd<ST>(IA, zl, a1, pa, row + ob * ST, gl);
    ob += SA;
  }
#pragma unroll
  for (int p = kNP - 1; p >= 0; --p) {
    if (p < np) {  // flows 2p + 1 (IB), then 2p (IA)
      float pa[3], pb[3];
      read3c<ST>(pb, row, ob);
      read3c<ST>(pa, row, ob + SB);
      flow1_bwd<ST>(IB, zk[2 * p + 1], a1, pb, row + ob * ST, gl);
      flow1_bwd<ST>(IA, zk[2 * p], a1, pa, row + (ob + SB) * ST, gl);
      ob += SP;
    }
  }
  adj = a1;
  return lp;
}

template <int IA, int IB, int ST = 1, class Mid = NoMid>
__device__ __forceinline__ float grad1_hpairs(float& z, float* row, float* zh, int zs, int K, int P, bool trainable,
                                              float gl, bool want_lp, float& adj, const Mid& mid = Mid{}) {
  constexpr int SA = IA == NFN_FLOW_AFFINE ? 2 : 3, SP = SA + (IB == NFN_FLOW_AFFINE ? 2 : 3);
  float l2 = 0.0f;
  int off = P;
  int k = 0;
  float pa[3], pb[3];
  read3c<ST>(pa, row, max(off - SA, 0));
  read3c<ST>(pb, row, max(off - SP, 0));
#pragma unroll 1
  for (; k + 1 < K; k += 2) {
    off -= SP;
    float pna[3], pnb[3];  // the next pair's parameters first (past flow 0: in-row reads)
    read3c<ST>(pna, row, max(off - SA, 0));
    read3c<ST>(pnb, row, max(off - SP, 0));
    float za, zb;
    fwd_pair1<IA, IB>(z, l2, za, zb, pa, pb, want_lp);
    zh[k * zs] = za;
    zh[(k + 1) * zs] = zb;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pa[i] = pna[i];
      pb[i] = pnb[i];
    }
  }
  if (K & 1) {  // the last flow: already read
    zh[(K - 1) * zs] = z;
    if (want_lp)
      l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(IA, z, pa)));
    else
      flow1_z(IA, z, pa);
  }
  const float lp = want_lp ? base1_fast<ST>(z, row, trainable) + l2 * kLn2 : 0.0f;
  mid();
  float a1;
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[ST], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    a1 = -gz;
    row[0] = gz;
    row[ST] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
  } else {
    a1 = -gl * z;
  }
  const int ob0 = trainable ? 2 : 0;
  adj = (K & 1) ? hpair_reverse<IA, IB, ST, true>(row, zh, zs, K, P, ob0, gl, a1)
                : hpair_reverse<IA, IB, ST, false>(row, zh, zs, K, P, ob0, gl, a1);
  return lp;
}


// Diagnostic experiment: grad1_packed for one program fixed at compile time (flow
// inputs in registers, straight-line code).
template <uint32_t TYPES, int K, int ST = 1>
__device__ __forceinline__ float grad1_static(float& z, float* row, float* zh, int zs, int P, bool trainable,
                                              float gl, bool want_lp, float& adj) {
  (void)zh;
  (void)zs;
  float l2 = 0.0f;
  float zk[K];
  int off = P;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int id = (int)((TYPES >> (2 * k)) & 3u);
    off -= size1(id);
    float pc[3];
    read3c<ST>(pc, row, off);
    zk[k] = z;
    if (want_lp)
      l2 += __builtin_amdgcn_logf(fabsf(flow1_fast<false>(id, z, pc)));
    else
      flow1_z(id, z, pc);
  }
  const float lp = want_lp ? base1_fast<ST>(z, row, trainable) + l2 * kLn2 : 0.0f;
  float a1;
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[ST], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    a1 = -gz;
    row[0] = gz;
    row[ST] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
  } else {
    a1 = -gl * z;
  }
  int ob = trainable ? 2 : 0;
#pragma unroll
  for (int k = K - 1; k >= 0; --k) {
    const int id = (int)((TYPES >> (2 * k)) & 3u);
    float pc[3];
    read3c<ST>(pc, row, ob);
    flow1_bwd<ST>(id, zk[k], a1, pc, row + ob * ST, gl);
    ob += size1(id);
  }
  adj = a1;
  return lp;
}

// grad1_static with a parameter-scalar cache (verdict r05 "Next" 2) — the fused Dense
// backward's form for a program fixed at compile time (C2's (planar, radial) x 5): the forward
// pass forms, per flow, every parameter-only scalar the reverse pass needs (planar: sigma(w u),
// 1 / |w|^2, c / |w|^2, u_hat, m and the det's parameter term; radial: alpha,
// sigma(0.3 a - 2), sigma(0.1 b + log(e - 1)), alpha beta, beta) once, from one exponential per
// softplus, and keeps them in registers (the program is a compile-time constant, so the cache is
// plain unrolled locals: 224 VGPRs, 2 waves per SIMD) instead of the reverse pass recomputing
// them (per planar flow an exp, two rcp and a log; per radial two of each).  Each radial flow
// also keeps h = 1 / (alpha + |z - z0|), the same rcp on the same operands in both passes.
// SHARE (the release form) goes one step further for the planar flows: the forward evaluates
// the reverse pass's e^{-2|s|} form of tanh(s) (s = w z + b) once and keeps tanh and tanh'
// for the reverse, taking tanh(s) from it for |s| >= 0.3 (tanh_poly03 below, as tanh_fast)
// instead of tanh_fast's e^{2|s|} form: one exp and one rcp fewer per planar flow, forward
// values within a few ulp of tanh_fast's.  !SHARE (diag NFN_CHAIN_FORM=5): bitwise
// grad1_static's values (the same expressions on the same operands; tests/test_gpu_diag.py).
template <uint32_t TYPES, int K, int ST = 1, bool SHARE = true>
__device__ __forceinline__ float grad1_static_cache(float& z, float* row, int P, bool trainable, float gl,
                                                    bool want_lp, float& adj) {
  float l2 = 0.0f;
  float zk[K], c0[K], c1[K], c2[K], c3[K], c4[K], c5[K], c6[K], c7[K];
  int off = P;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int id = (int)((TYPES >> (2 * k)) & 3u);
    off -= size1(id);
    float pc[3];
    read3c<ST>(pc, row, off);
    zk[k] = z;
    if (id == NFN_FLOW_PLANAR) {
      const float u = pc[0], w = pc[1] + 1.0f, b = pc[2];
      const float wtu = w * u;
      float sp, sg;
      sp_sig1<true>(wtu, sp, sg);  // sp: softplus_alpha's value bitwise
      const float nw2 = fmaf(w, w, 1e-9f);
      const float rn = __builtin_amdgcn_rcpf(nw2);
      // the forward: planar1_z / planar1_fast<false> bitwise
      const float mf = sp - (1.0f - 1e-5f);
      const float uhf = planar1_uh(u, w, rn, mf);
      const float sv = fmaf(w, z, b);
      float th;
      if constexpr (SHARE) {  // planar1_bwd's tanh and tanh' of s
        const float E = __builtin_amdgcn_exp2f(fabsf(sv) * (-2.0f * kLog2e));
        const float rE = __builtin_amdgcn_rcpf(1.0f + E);
        const float hE = copysignf((1.0f - E) * rE, sv);
        c6[k] = hE;
        c7[k] = 4.0f * E * rE * rE;
        th = fabsf(sv) < 0.3f ? tanh_poly03(sv) : hE;
      } else {
        th = tanh_fast(sv);
        c6[k] = c7[k] = 0.0f;
      }
      z = fmaf(uhf, th, z);
      if (want_lp) {
        const float qd = fmaf((wtu - mf) * 1e-9f, rn, sp + 1e-5f);
        l2 += __builtin_amdgcn_logf(fabsf(fmaf(th, th, fmaf(-th, th, 1.0f) * qd)));
      }
      // the reverse pass's parameter scalars (planar1_bwd's expressions)
      const float m = (sp - 1.0f) + 1e-5f;
      const float c = m - wtu;
      const float q0 = c * rn;
      const float cn = fmaf(fmaf(-nw2, q0, c), rn, q0);
      c0[k] = sg;
      c1[k] = rn;
      c2[k] = cn;
      c3[k] = planar1_uh(u, w, rn, m);
      c4[k] = m;
      c5[k] = fmaf(-cn, 1e-9f, sp + 1e-5f);
    } else if (id == NFN_FLOW_RADIAL) {
      const float xa = fmaf(0.3f, pc[0], -2.0f);
      const float xb = fmaf(0.1f, pc[1], kLogExpm1One);
      float al, sga, spb, sgb;
      sp_sig1<true>(xa, al, sga);  // al: softplus_alpha's value bitwise
      sp_sig1(xb, spb, sgb);       // spb: sp_fast1's value bitwise
      const float ab = fmaf(al, spb, -al);
      const float dz = z - pc[2];
      const float h = __builtin_amdgcn_rcpf(al + fabsf(dz));
      const float abh = ab * h;
      z = fmaf(abh, dz, z);  // radial1_z / radial1_fast bitwise
      if (want_lp) l2 += __builtin_amdgcn_logf(fabsf(fmaf(abh, al * h, 1.0f)));
      c6[k] = h;
      c7[k] = 0.0f;
      c0[k] = al;
      c1[k] = sga;
      c2[k] = sgb;
      c3[k] = ab;
      c4[k] = spb - 1.0f;
      c5[k] = 0.0f;
    } else {
      const float sc = 1.0f + pc[1];
      if (want_lp) l2 += __builtin_amdgcn_logf(fabsf(sc));
      z = fmaf(z, sc, pc[0]);
      c0[k] = c1[k] = c2[k] = c3[k] = c4[k] = c5[k] = c6[k] = c7[k] = 0.0f;
    }
  }
  const float lp = want_lp ? base1_fast<ST>(z, row, trainable) + l2 * kLn2 : 0.0f;
  float a;
  if (trainable) {
    float sps, sgs;
    sp_sig1(kLogExpm1One + 0.1f * row[ST], sps, sgs);
    const float rs = __builtin_amdgcn_rcpf(1e-3f + sps);
    const float zz = (z - row[0]) * rs;
    const float gz = gl * zz * rs;
    a = -gz;
    row[0] = gz;
    row[ST] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
  } else {
    a = -gl * z;
  }
  int ob = trainable ? 2 : 0;
#pragma unroll
  for (int k = K - 1; k >= 0; --k) {
    const int id = (int)((TYPES >> (2 * k)) & 3u);
    float pc[3];
    read3c<ST>(pc, row, ob);
    float* p = row + ob * ST;
    const float zz = zk[k];
    if (id == NFN_FLOW_PLANAR) {  // planar1_bwd with the cached scalars
      const float u = pc[0], w = pc[1] + 1.0f;
      const float sg = c0[k], rn = c1[k], cn = c2[k], uh = c3[k], m = c4[k], qd0 = c5[k];
      float h, hp;
      if constexpr (SHARE) {
        h = c6[k];
        hp = c7[k];
      } else {
        const float s = fmaf(w, zz, pc[2]);
        const float E = __builtin_amdgcn_exp2f(fabsf(s) * (-2.0f * kLog2e));
        const float rE = __builtin_amdgcn_rcpf(1.0f + E);
        h = copysignf((1.0f - E) * rE, s);
        hp = 4.0f * E * rE * rE;
      }
      const float q = fmaf(-cn, 1e-9f, m);
      const float hpd = gl * hp * __builtin_amdgcn_rcpf(fmaf(h, h, hp * qd0));
      const float Ss = fmaf(hp, uh * a, -2.0f * q * h * hpd);
      const float G = fmaf(h, a, hpd * w);
      const float wGn = w * G * rn;
      const float k1 = (sg - 1.0f) * wGn;
      p[0] = G * (fmaf(sg * w, w, 1e-9f) * rn);
      p[ST] = fmaf(zz, Ss, fmaf(hpd, uh, fmaf(cn, G, fmaf(-2.0f * cn * wGn, w, k1 * u))));
      p[2 * ST] = Ss;
      a = fmaf(w, Ss, a);
    } else if (id == NFN_FLOW_RADIAL) {  // radial1_bwd with the cached scalars
      const float al = c0[k], sga = c1[k], sgb = c2[k], ab = c3[k], be = c4[k];
      const float dz = zz - pc[2];
      const float h = c6[k];
      const float hh = h * h;
      const float rB = __builtin_amdgcn_rcpf(fmaf(ab * al, hh, 1.0f));
      const float da = dz * a;
      const float glr = gl * rB;
      const float H = fmaf(ab, da, 2.0f * ab * al * h * glr);
      const float g_ab = fmaf(h, da, al * hh * glr);
      const float g_al = fmaf(be, g_ab, ab * hh * glr) - hh * H;
      const float hH = hh * H;
      const float sgn = sign0(dz);
      p[0] = 0.3f * sga * g_al;
      p[ST] = 0.1f * sgb * al * g_ab;
      p[2 * ST] = fmaf(hH, sgn, -ab * h * a);
      a = fmaf(fmaf(ab, h, 1.0f), a, -hH * sgn);
    } else {
      affine1_bwd<ST>(zz, a, pc[0], pc[1], p, gl);
    }
    ob += size1(id);
  }
  adj = a;
  return lp;
}

// ---------------------------------------------------------------------------
// Lane-group forms (d >= 4): a G-lane group owns one sample, lane j holds the
// DPL dimensions j, j + G, ...; inner products are DPP group sums (gsum).
// ---------------------------------------------------------------------------

template <int G, int DPL, bool FAST, bool FULL = false>
__device__ __forceinline__ void planar_gd_bwd(const float (&z)[DPL], float (&a)[DPL], float* p, int d_, int j,
                                              float gl) {
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
  const float wtu = gsum<G>(swu);
  const float nw2 = gsum<G>(sww) + 1e-9f;
  const float s = gsum<G>(swz) + p[2 * d];
  float sp, sg;
  if constexpr (FAST) {
    sp_sig1<true>(wtu, sp, sg);  // softplus relative-accurate as w.u -> -inf
  } else {
    sp = softplus_tf<false>(wtu);
    sg = f_sigmoid<false>(wtu);
  }
  const float m = (-1.0f + sp) + 1e-5f;
  const float c = m - wtu;
  const float cn = f_div_acc<FAST>(c, nw2);
  const float E = f_exp<FAST>(-2.0f * fabsf(s));
  const float rE = f_div<FAST>(1.0f, 1.0f + E);
  float h;
  if constexpr (FAST)
    h = copysignf((1.0f - E) * rE, s);
  else
    h = tanhf(s);
  const float hp = 4.0f * E * rE * rE;
  float uh[DPL];
  float sua = 0.0f;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    uh[i] = fmaf(cn, w[i], u[i]);
    sua += uh[i] * a[i];
  }
  const float ua = gsum<G>(sua);
  const float q = m - cn * 1e-9f;
  // det = 1 + hp q = h^2 + hp (softplus + 1e-5 - cn 1e-9) (planar_bwd)
  const float hpd = gl * f_div<FAST>(hp, fmaf(h, h, hp * ((sp + 1e-5f) - cn * 1e-9f)));
  const float Ss = hp * ua - 2.0f * q * h * hpd;
  float Gv[DPL];
  float swG = 0.0f;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    Gv[i] = h * a[i] + hpd * w[i];
    swG += w[i] * Gv[i];
  }
  const float wGn = f_div<FAST>(gsum<G>(swG), nw2);
  const float k1 = (sg - 1.0f) * wGn;
  const float k2 = 2.0f * cn * wGn;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    if (FULL || jj < d) {
      p[jj] = Gv[i] + k1 * w[i];
      p[d + jj] = z[i] * Ss + hpd * uh[i] + cn * Gv[i] - k2 * w[i] + k1 * u[i];
      a[i] = fmaf(w[i], Ss, a[i]);
    }
  }
  if (j == 0) p[2 * d] = Ss;  // the group's lanes read p[2d] above, in lockstep
}

template <int G, int DPL, bool FAST, bool FULL = false>
__device__ __forceinline__ void radial_gd_bwd(const float (&z)[DPL], float (&a)[DPL], float* p, int d_, int j,
                                              float gl) {
  const int d = FULL ? G * DPL : d_;
  const float xa = 0.3f * p[0] - 2.0f;
  const float xb = 0.1f * p[1] + kLogExpm1One;
  float al, sga, spb, sgb;
  if constexpr (FAST) {
    sp_sig1<true>(xa, al, sga);  // relative accuracy as alpha -> 0 (softplus_alpha)
    sp_sig1(xb, spb, sgb);
  } else {
    al = softplus_tf<false>(xa);
    sga = f_sigmoid<false>(xa);
    spb = softplus_tf<false>(xb);
    sgb = f_sigmoid<false>(xb);
  }
  const float be = spb - 1.0f;
  float dz[DPL];
  float sr = 0.0f, sda = 0.0f;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    dz[i] = (FULL || j + G * i < d) ? z[i] - p[2 + j + G * i] : 0.0f;
    sr += fabsf(dz[i]);
    sda += dz[i] * a[i];
  }
  const float r = gsum<G>(sr);
  const float da = gsum<G>(sda);
  const float h = f_div<FAST>(1.0f, al + r);
  const float hh = h * h;
  const float ab = al * be;
  const float A = 1.0f + ab * h;
  const float rB = f_div<FAST>(1.0f, 1.0f + ab * al * hh);
  const float rA = d > 1 ? f_div<FAST>((float)(d - 1), A) : 0.0f;  // (d-1) / A
  const float H = ab * da + gl * (ab * rA + 2.0f * ab * al * h * rB);
  const float g_ab = h * da + gl * (h * rA + al * hh * rB);
  const float g_al = be * g_ab + gl * ab * hh * rB - hh * H;
  const float hH = hh * H;
  const float abh = ab * h;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    if (FULL || jj < d) {
      const float sgn = sign0(dz[i]);
      p[2 + jj] = hH * sgn - abh * a[i];
      a[i] = A * a[i] - hH * sgn;
    }
  }
  if (j == 0) {
    p[0] = 0.3f * sga * g_al;
    p[1] = 0.1f * sgb * al * g_ab;
  }
}

template <int G, int DPL, bool FAST, bool FULL = false>
__device__ __forceinline__ void affine_gd_bwd(const float (&z)[DPL], float (&a)[DPL], float* p, int d_, int j,
                                              float gl) {
  const int d = FULL ? G * DPL : d_;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    if (FULL || jj < d) {
      const float sc = 1.0f + p[d + jj];
      p[jj] = a[i];
      p[d + jj] = z[i] * a[i] + gl * f_div<FAST>(1.0f, sc);
      a[i] *= sc;
    }
  }
}

template <int G, int DPL, bool FAST, bool FULL = false>
__device__ __forceinline__ void base_gd_bwd(const float (&z)[DPL], float (&a)[DPL], float* row, int d_, int j,
                                            bool trainable, float gl) {
  const int d = FULL ? G * DPL : d_;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int jj = j + G * i;
    a[i] = 0.0f;
    if (FULL || jj < d) {
      if (trainable) {
        const float xs = kLogExpm1One + 0.1f * row[d + jj];
        float sps, sgs;
        if constexpr (FAST) {
          sp_sig1(xs, sps, sgs);
        } else {
          sps = softplus_tf<false>(xs);
          sgs = f_sigmoid<false>(xs);
        }
        const float rs = f_div<FAST>(1.0f, 1e-3f + sps);
        const float zz = (z[i] - row[jj]) * rs;
        const float gz = gl * zz * rs;
        a[i] = -gz;
        row[jj] = gz;
        row[d + jj] = 0.1f * sgs * gl * fmaf(zz, zz, -1.0f) * rs;
      } else {
        a[i] = -gl * z[i];
      }
    }
  }
}

// One sample: forward from z (already normalised), keeping each flow's input in
// zh[(k * d + j) * zs] (LDS), then the reverse pass; the parameter row `row` (LDS)
// is overwritten in place with d logp / d t.  Returns log_prob (without the
// -sum(log y_std) correction); `adj` receives d logp / d z_0.
template <int DM, bool FAST, int CM = kChainLoop>
__device__ __forceinline__ float grad_sample(float (&z)[DM], float* row, float* zh, int zs, const ChainArgs& a,
                                             float gl, float (&adj)[DM]) {
  const int d = a.d;
  const int K = a.prog.K;
  float lp;
  if constexpr (DM == 1 && FAST && CM == kStaticProg) {  // diagnostic: the C2 program at compile time
    float a1;
    const float lp1 = grad1_static<kStaticTypes[0], kStaticK[0]>(z[0], row, zh, zs, a.P, a.trainable != 0, gl,
                                                                 a.out != nullptr, a1);
    adj[0] = a1;
    return lp1;
  }
  if constexpr (DM == 1 && FAST && CM >= kChainHPair) {  // an alternating program (hpair_types)
    float a1;
    constexpr int c = CM - kChainHPair;
    const float lp1 = grad1_hpairs<(c % 9) / 3, c % 3>(z[0], row, zh, zs, K, a.P, a.trainable != 0, gl,
                                                       a.out != nullptr, a1);
    adj[0] = a1;
    return lp1;
  }
  if constexpr (DM == 1 && FAST) {
    if (K <= 16) {
      float a1;
      const float lp1 = CM == kChainPairs ? grad1_pairs(z[0], row, zh, zs, a.prog.types[0], K, a.P,
                                                        a.trainable != 0, gl, a.out != nullptr, a1)
                                          : grad1_packed(z[0], row, zh, zs, a.prog.types[0], K, a.P,
                                                         a.trainable != 0, gl, a.out != nullptr, a1);
      adj[0] = a1;
      return lp1;
    }
  }
  {
    float ildj = 0.0f;
    for (int k = 0; k < K; ++k) {
      const int st = a.prog.step[k];
#pragma unroll
      for (int j = 0; j < DM; ++j)
        if (j < d) zh[(k * d + j) * zs] = z[j];
      ildj = ildj + flow_step<DM, FAST>(st & 3, z, row + (st >> 2), d);
    }
    lp = base_log_prob<DM, FAST>(z, row, d, a.trainable != 0) + ildj;
  }
  base_bwd<DM, FAST>(z, adj, row, d, a.trainable != 0, gl);
  for (int k = K - 1; k >= 0; --k) {
    const int st = a.prog.step[k];
    float zk[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) zk[j] = j < d ? zh[(k * d + j) * zs] : 0.0f;
    float* p = row + (st >> 2);
    const int id = st & 3;
    if (id == NFN_FLOW_PLANAR)
      planar_bwd<DM, FAST>(zk, adj, p, d, gl);
    else if (id == NFN_FLOW_RADIAL)
      radial_bwd<DM, FAST>(zk, adj, p, d, gl);
    else
      affine_bwd<DM, FAST>(zk, adj, p, d, gl);
  }
  return lp;
}

}  // namespace nfn

#pragma clang fp contract(fast)
