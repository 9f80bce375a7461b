// nfn_grid.hip — density on a grid of y values:
// out[g, b] = log p(y_grid[g] | t_b) for every grid point g and parameter row b —
// the evaluation behind evaluation/visualization/flow_plotting.py:33-53
// (plot_model: dist.prob(y[i]) over a y-grid for a batch of x) without one launch
// per grid point.  Each workgroup stages a tile of parameter rows in LDS once and
// walks a chunk of the grid (blockIdx.y): every lane re-evaluates its own row for
// each grid value, which is read once per wave (uniform address); the (g, b)
// outputs of a wave are 256 contiguous bytes.  Compute-bound: t is read once per
// (tile, chunk), so HBM traffic is ~4 B per evaluation.
#include "nfn_launch.h"

// the d = 1 split form below must round as nfn_device.h's evaluators do (contraction only
// within an expression): it then equals them bit for bit
#pragma clang fp contract(on)

namespace nfn {
namespace {

// d = 1, fast math: each flow's parameter-only terms (planar w, b, u_hat and the det
// coefficient; radial alpha and alpha beta; affine scale and shift) and the base's loc /
// scale are formed ONCE per row, in registers, and every grid value then runs only the
// z-dependent remainder of planar1_fast / radial1_fast / affine1_fast (the same
// expressions: same results as eval_sample).  Per grid value that drops the softplus pair,
// the reciprocals and u_hat of every flow, about half of a planar step.
constexpr int kGridMaxK = 16;

struct GridRow1 {
  float c0[kGridMaxK], c1[kGridMaxK], c2[kGridMaxK], c3[kGridMaxK];
  float loc, rsc, lconst;
};

__device__ __forceinline__ void grid1_prepare(GridRow1& r, const float* row, const ChainArgs& a) {
  const int K = a.prog.K;
#pragma unroll
  for (int k = 0; k < kGridMaxK; ++k) {
    r.c0[k] = r.c1[k] = r.c2[k] = r.c3[k] = 0.0f;
    if (k < K) {
      const int st = a.prog.step[k];  // kernel argument: uniform
      const int id = st & 3;
      float p[3];
      read3(p, row, st);
      if (id == NFN_FLOW_PLANAR) {  // planar1_fast(z, u = p0, wraw = p1, b = p2)
        const float w = p[1] + 1.0f;
        const float wtu = w * p[0];
        const float nw2 = fmaf(w, w, 1e-9f);
        const float rn = __builtin_amdgcn_rcpf(nw2);
        const float sp = softplus_alpha<true>(wtu);
        const float m = planar1_m(w, p[0], sp);
        r.c0[k] = w;
        r.c1[k] = p[2];
        r.c2[k] = planar1_uh(p[0], w, rn, m);
        r.c3[k] = fmaf((wtu - m) * 1e-9f, rn, sp + 1e-5f);
      } else if (id == NFN_FLOW_RADIAL) {  // radial1_fast(z, a0 = p0, b0 = p1, g = p2)
        const float alpha = softplus_alpha<true>(fmaf(0.3f, p[0], -2.0f));
        r.c0[k] = alpha;
        r.c1[k] = fmaf(alpha, sp_fast1(fmaf(0.1f, p[1], kLogExpm1One)), -alpha);
        r.c2[k] = p[2];
      } else {  // affine1_fast(z, sh = p0, scraw = p1)
        r.c0[k] = 1.0f + p[1];
        r.c1[k] = p[0];
      }
    }
  }
  if (a.trainable) {  // base1_fast
    const float sc = 1e-3f + sp_fast1(kLogExpm1One + 0.1f * row[1]);
    r.loc = row[0];
    r.rsc = __builtin_amdgcn_rcpf(sc);
    r.lconst = kHalfLog2Pi + __builtin_amdgcn_logf(sc) * kLn2;
  } else {
    r.loc = 0.0f;
    r.rsc = 1.0f;
    r.lconst = kHalfLog2Pi;
  }
}

__device__ __forceinline__ float grid1_eval(float z, const GridRow1& r, const ChainArgs& a) {
  const int K = a.prog.K;
  float l2 = 0.0f;
#pragma unroll
  for (int k = 0; k < kGridMaxK; ++k) {
    if (k < K) {
      const int id = a.prog.step[k] & 3;
      float det;
      if (id == NFN_FLOW_PLANAR) {
        const float th = tanh_fast(fmaf(r.c0[k], z, r.c1[k]));
        z = fmaf(r.c2[k], th, z);
        det = fmaf(th, th, fmaf(-th, th, 1.0f) * r.c3[k]);
      } else if (id == NFN_FLOW_RADIAL) {
        const float dz = z - r.c2[k];
        const float h = __builtin_amdgcn_rcpf(r.c0[k] + fabsf(dz));
        const float abh = r.c1[k] * h;
        z = fmaf(abh, dz, z);
        det = fmaf(abh, r.c0[k] * h, 1.0f);
      } else {
        z = fmaf(z, r.c0[k], r.c1[k]);
        det = r.c0[k];
      }
      l2 += __builtin_amdgcn_logf(fabsf(det));
    }
  }
  const float zz = (z - r.loc) * r.rsc;
  return (-0.5f * (zz * zz) - r.lconst) + l2 * kLn2;
}

template <int DM, bool FAST, bool PRE = true>
__global__ void __launch_bounds__(kMaxBlock) chain_grid_kernel(GridArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  const int rows = a.tile_rows > 0 ? a.tile_rows : blockDim.x;
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * rows;
  const int nr = (int)min((int64_t)rows, a.B - b0);
  const int g0 = (int)blockIdx.y * ga.gchunk;
  const int g1 = min(ga.G, g0 + ga.gchunk);
  const bool tb = a.t_rowstride == 0;
  if (a.P > 0) {
    stage_rows(lds, a.t + (tb ? 0 : b0 * a.t_rowstride), a.t_rowstride, tb ? 1 : nr, a.P, a.lds_stride,
               a.vec4 != 0);
  }
  __syncthreads();
  if (tid >= nr) return;
  const float* row = lds + (tb ? 0 : tid * a.lds_stride);
  float corr = 0.0f;
  if (a.y_mean) {
    for (int j = 0; j < a.d; ++j) corr += f_log<FAST>(a.y_std[j]);
  }
  if constexpr (DM == 1 && FAST && PRE) {
    if (a.prog.K <= kGridMaxK) {
      GridRow1 r;
      grid1_prepare(r, row, a);
      for (int g = g0; g < g1; ++g) {
        float z = ga.y_grid[(int64_t)g * ga.y_gstride];
        if (a.y_mean) z = f_div<FAST>(z - a.y_mean[0], a.y_std[0]);
        ga.out[(int64_t)g * ga.out_gstride + b0 + tid] = grid1_eval(z, r, a) - corr;
      }
      return;
    }
  }
  for (int g = g0; g < g1; ++g) {
    const float* yg = ga.y_grid + (int64_t)g * ga.y_gstride;
    float z[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      z[j] = j < a.d ? yg[j] : 0.0f;
      if (a.y_mean && j < a.d) z[j] = f_div<FAST>(z[j] - a.y_mean[j], a.y_std[j]);
    }
    ga.out[(int64_t)g * ga.out_gstride + b0 + tid] = eval_sample<DM, FAST>(z, row, a) - corr;
  }
}

template <bool FAST>
void launch_grid_t(int dm, const GridArgs& ga, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  switch (dm) {
    case 1:
      // NFN_GRID_PRE=0 (diag A/B): every grid value re-derives the parameter-only terms
      if (env_int("NFN_GRID_PRE", 1) != 0)
        nfn_launch((chain_grid_kernel<1, FAST>), grid, block, lds, s, ga);
      else
        nfn_launch((chain_grid_kernel<1, FAST, false>), grid, block, lds, s, ga);
      break;
    case 2: nfn_launch((chain_grid_kernel<2, FAST>), grid, block, lds, s, ga); break;
    case 4: nfn_launch((chain_grid_kernel<4, FAST>), grid, block, lds, s, ga); break;
    case 8: nfn_launch((chain_grid_kernel<8, FAST>), grid, block, lds, s, ga); break;
    case 16: nfn_launch((chain_grid_kernel<16, FAST>), grid, block, lds, s, ga); break;
    default: nfn_launch((chain_grid_kernel<32, FAST>), grid, block, lds, s, ga); break;
  }
}

}  // namespace

void launch_grid(bool fast, int dm, const GridArgs& ga, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  if (fast)
    launch_grid_t<true>(dm, ga, grid, block, lds, s);
  else
    launch_grid_t<false>(dm, ga, grid, block, lds, s);
}

}  // namespace nfn
