// nfn_grad2.hip — DIAGNOSTIC A/B only (NFN_DIAG build; an empty object in the release
// library): the d = 1 fused backward with two samples per lane, in its own translation unit
// so that it can be compiled without the SLP vectorizer (build.py: -fno-slp-vectorize).
// With it, the compiler fused the two samples' scalar chains into packed v_pk_* fp32
// operations — one dependency chain of half-rate instructions instead of two independent
// ones — and the kernel lost the instruction-level parallelism it exists for (DESIGN.md
// "C2 backward: two samples per lane").
#include "nfn_grad_device.h"
#include "nfn_launch.h"

#ifdef NFN_DIAG
namespace nfn {
namespace {

// DIAGNOSTIC A/B (NFN_DIAG build, NFN_GRAD_WAVE2=1; measured and not adopted, DESIGN.md
// "C2 backward: two samples per lane"): bitwise the release kernel's results.
// d = 1, fast math, P = 4Q (Q in {2, 4, 8}: C1, C2): chain_grad_wave_kernel's walk over
// 128-sample wave tiles with TWO samples per lane (rows lane and lane + 64, grad1_packed2:
// one program walk, two interleaved dependency chains).  The chain needs >= 12 resident
// one-sample waves per CU to hide its latency while the backward's copy-shaped stream
// moves its bytes fastest from few waves (memory-only 0.79 of the spec at 4 waves per CU,
// 0.69-0.72 at 8-14, DESIGN.md "C2 backward"); two samples per lane give each wave the
// independent work of two at 6 waves per CU.  The LDS slot holds the 128 rows at the odd
// stride S and the K x 128 flow inputs (C2: 22 KiB); the next tile's 2Q float4 row pieces
// per lane, y and g are prefetched into registers.  Per sample the arithmetic is
// grad1_packed's: bitwise chain_grad_wave_kernel's results.
template <int Q>
__global__ void __launch_bounds__(128, 1) chain_grad_wave2_kernel(GradArgs ga) {
  const ChainArgs& a = ga.c;
  extern __shared__ float lds[];
  constexpr int NV = 2 * Q;       // float4 row pieces per lane per 128-row tile
  constexpr int RSTEP = 64 / Q;   // rows per wave instruction
  const int S = a.lds_stride;
  const int K = a.prog.K;
  const int P = a.P;
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float* tl = lds + wid * (128 * S + K * 128);
  float* zha = tl + 128 * S + lane;
  float* zhb = zha + 64;
  const int r0 = lane / Q;
  const int c4 = lane - r0 * Q;
  const int64_t rs = a.t_rowstride;
  const int64_t gts = ga.gt_rowstride;
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  const int64_t ustep = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool norm = a.y_mean != nullptr;
  const float ymean = norm ? a.y_mean[0] : 0.0f, ystd = norm ? a.y_std[0] : 1.0f;
  const float corr = norm ? f_log<true>(ystd) : 0.0f;
  const uint32_t types = a.prog.types[0];
  const bool want_lp = a.out != nullptr;

  float4 buf[NV];
  float ya = 0.0f, yb = 0.0f, ga_ = 1.0f, gb_ = 1.0f;
  bool issued_once = false;
  auto issue = [&](int64_t tile) {
    if (a.ablate_loads && issued_once) return;  // diagnostic: compute-only timing
    issued_once = true;
    const int64_t b0 = tile * 128;
    const int nr = (int)min((int64_t)128, a.B - b0);
    const float* base = a.t + b0 * rs + 4 * c4;
#pragma unroll
    for (int k = 0; k < NV; ++k)
      if (r0 + k * RSTEP < nr) buf[k] = load_row4<true>(base + (int64_t)(r0 + k * RSTEP) * rs);
    if (lane < nr) {
      ya = a.y[(b0 + lane) * a.y_bstride];
      if (ga.g_out) ga_ = __builtin_nontemporal_load(ga.g_out + b0 + lane);
    }
    if (lane + 64 < nr) {
      yb = a.y[(b0 + 64 + lane) * a.y_bstride];
      if (ga.g_out) gb_ = __builtin_nontemporal_load(ga.g_out + b0 + 64 + lane);
    }
  };

  int64_t tile = u0;
  const int64_t ntiles = a.ntiles;
  if (tile < ntiles) issue(tile);
  for (; tile < ntiles; tile += ustep) {
    const int64_t b0 = tile * 128;
    const int nr = (int)min((int64_t)128, a.B - b0);
    if (a.prio) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (r0 + k * RSTEP < nr) {
        float* dst = tl + (r0 + k * RSTEP) * S + 4 * c4;
        dst[0] = buf[k].x;
        dst[1] = buf[k].y;
        dst[2] = buf[k].z;
        dst[3] = buf[k].w;
      }
    }
    float za = norm ? f_div<true>(ya - ymean, ystd) : ya;
    float zb = norm ? f_div<true>(yb - ymean, ystd) : yb;
    const float gla = ga_, glb = gb_;
    wave_lds_sync();
    if (tile + ustep < ntiles) issue(tile + ustep);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    if (lane < nr) {  // lane + 64 >= nr: the second sample runs on a stale row, never stored
      float adja, adjb, lpa, lpb;
      grad1_packed2(za, zb, tl + lane * S, tl + (lane + 64) * S, zha, zhb, 128, types, K, P, a.trainable != 0,
                    gla, glb, want_lp, adja, adjb, lpa, lpb);
      const int64_t b = b0 + lane;
      if (want_lp) __builtin_nontemporal_store(lpa - corr, a.out + b);
      if (ga.grad_y) ga.grad_y[b] = norm ? f_div<true>(adja, ystd) : adja;
      if (lane + 64 < nr) {
        if (want_lp) __builtin_nontemporal_store(lpb - corr, a.out + b + 64);
        if (ga.grad_y) ga.grad_y[b + 64] = norm ? f_div<true>(adjb, ystd) : adjb;
      }
    }
    wave_lds_sync();
    if (ga.grad_t) {
      float* gbase = ga.grad_t + b0 * gts + 4 * c4;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int r = r0 + k * RSTEP;
        if (r < nr) {
          const float* src = tl + r * S + 4 * c4;
          const f32x4 v = {src[0], src[1], src[2], src[3]};
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(gbase + (int64_t)r * gts));
        }
      }
    }
  }
}

template <int Q>
bool launch_wave2_q(const GradArgs& ga, hipStream_t s, int64_t* grid) {
  auto k = chain_grad_wave2_kernel<Q>;
  const size_t lds = (size_t)2 * (128 * ga.c.lds_stride + ga.c.prog.K * 128) * sizeof(float);
  *grid = std::max<int64_t>(1, persistent_grid(k, 128, lds, (ga.c.ntiles + 1) / 2));
  nfn_launch((k), dim3((unsigned)*grid), dim3(128), lds, s, ga);
  return true;
}

}  // namespace

bool launch_grad_wave2(int Q, const GradArgs& ga, hipStream_t s, int64_t* grid) {
  switch (Q) {
    case 2: return launch_wave2_q<2>(ga, s, grid);
    case 4: return launch_wave2_q<4>(ga, s, grid);
    case 8: return launch_wave2_q<8>(ga, s, grid);
  }
  return false;
}

}  // namespace nfn
#endif  // NFN_DIAG
