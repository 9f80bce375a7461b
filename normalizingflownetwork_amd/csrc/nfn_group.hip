// nfn_group.hip — instantiations of chain_group_kernel (d >= 4).
// Compiled twice: -DNFN_FAST=1 and -DNFN_FAST=0.
#include "nfn_launch.h"

#ifndef NFN_FAST
#error "compile with -DNFN_FAST=0 or -DNFN_FAST=1"
#endif

namespace nfn {
namespace {

constexpr bool kFast = NFN_FAST != 0;

template <int G, int DPL, int NV, bool POST>
void launch_g(const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid_out) {
  // contiguous rows, plain chain: the branch-free buffer pipeline (chain_group1_kernel)
  const bool g1 = !POST && a.t_rowstride == a.P && a.y_bstride * 256 < ((int64_t)1 << 31) &&
                  (int64_t)(64 / G) * a.P * 4 < ((int64_t)1 << 31) && env_int("NFN_GROUP1", 1) != 0;
  if (g1) {
    auto kfn = a.d == G * DPL ? chain_group1_kernel<G, DPL, kFast, NV, true>
                              : chain_group1_kernel<G, DPL, kFast, NV, false>;
    // 2 resident workgroups per CU (C3: 0.419 vs 0.433 ms at the occupancy limit of
    // 4, as for the d = 1 kernel: fewer bytes in flight stream faster once the flow
    // math is short enough to hide); NFN_WG_PER_CU overrides
    int64_t grid = persistent_grid(kfn, kMaxBlock, lds, (a.ntiles + 3) / 4);
    if (env_int("NFN_WG_PER_CU", 0) <= 0) grid = std::min<int64_t>(grid, (int64_t)cu_count() * 2);
    grid = cap_grid(grid, a);
    *grid_out = grid;
    nfn_launch(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, a);
    return;
  }
  auto kfn = chain_group_kernel<G, DPL, kFast, NV, POST>;
  const int64_t grid = cap_grid(persistent_grid(kfn, kMaxBlock, lds, (a.ntiles + 3) / 4), a);  // 4 wave teams per WG
  *grid_out = grid;
  nfn_launch(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, a);
}

// float4 slots per thread: the exact count for the common widths (every slot is a
// live register), rounded up otherwise
template <int G, int DPL, bool POST>
bool launch_g_nv(int nv, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* g) {
  if (nv <= 4)
    launch_g<G, DPL, 4, POST>(a, lds, s, g);
  else if (nv <= 5)
    launch_g<G, DPL, 5, POST>(a, lds, s, g);
  else if (nv <= 6)
    launch_g<G, DPL, 6, POST>(a, lds, s, g);
  else if (nv <= 8)
    launch_g<G, DPL, 8, POST>(a, lds, s, g);
  else if (nv <= 9)
    launch_g<G, DPL, 9, POST>(a, lds, s, g);
  else if (nv <= 12)
    launch_g<G, DPL, 12, POST>(a, lds, s, g);
  else if (nv <= 16)
    launch_g<G, DPL, 16, POST>(a, lds, s, g);
  else if (G == 2 && nv <= 18)
    launch_g<G, DPL, 18, POST>(a, lds, s, g);
  else
    return false;
  return true;
}

template <bool POST>
bool launch_g_shape(int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* g) {
  // default shapes per event-size bound (see group_shape in nfn_api.hip)
  if (G == 4 && DPL == 1) return launch_g_nv<4, 1, POST>(nv, a, lds, s, g);
  if (G == 4 && DPL == 2) return launch_g_nv<4, 2, POST>(nv, a, lds, s, g);
  if (G == 4 && DPL == 4) return launch_g_nv<4, 4, POST>(nv, a, lds, s, g);
  if (G == 8 && DPL == 4) return launch_g_nv<8, 4, POST>(nv, a, lds, s, g);
  // alternates for tuning runs (fast math, plain chain)
  if constexpr (kFast && !POST) {
    if (G == 8 && DPL == 1) return launch_g_nv<8, 1, POST>(nv, a, lds, s, g);
    if (G == 8 && DPL == 2) return launch_g_nv<8, 2, POST>(nv, a, lds, s, g);
    if (G == 2 && DPL == 4) return launch_g_nv<2, 4, POST>(nv, a, lds, s, g);  // NFN_GROUP_LANES=2
  }
  return false;
}

#if NFN_FAST
template <int G, int DPL, int NV>
void launch_gf(const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid_out) {
  auto kfn = a.d == G * DPL ? chain_group1_kernel<G, DPL, true, NV, true, true>
                            : chain_group1_kernel<G, DPL, true, NV, false, true>;
  int64_t grid = std::min<int64_t>((a.ntiles + 3) / 4, (int64_t)cu_count() * 2);
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, a);
}

template <int G, int DPL>
bool launch_gf_nv(int nv, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* g) {
  if (nv <= 4) launch_gf<G, DPL, 4>(a, lds, s, g);
  else if (nv <= 8) launch_gf<G, DPL, 8>(a, lds, s, g);
  else if (nv <= 12) launch_gf<G, DPL, 12>(a, lds, s, g);
  else if (nv <= 16) launch_gf<G, DPL, 16>(a, lds, s, g);
  else if (G == 2 && nv <= 18) launch_gf<G, DPL, 18>(a, lds, s, g);
  else return false;
  return true;
}
#endif

}  // namespace

#if NFN_FAST
// the Chain bijector (forward + fldj, chain_group1_kernel<..., FWD>) for d >= 4, contiguous rows
bool launch_group1_fwd(int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid) {
  if (G == 4 && DPL == 1) return launch_gf_nv<4, 1>(nv, a, lds, s, grid);
  if (G == 4 && DPL == 2) return launch_gf_nv<4, 2>(nv, a, lds, s, grid);
  if (G == 2 && DPL == 4) return launch_gf_nv<2, 4>(nv, a, lds, s, grid);
  if (G == 4 && DPL == 4) return launch_gf_nv<4, 4>(nv, a, lds, s, grid);
  if (G == 8 && DPL == 4) return launch_gf_nv<8, 4>(nv, a, lds, s, grid);
  return false;
}

bool launch_group_fast(bool post, int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s,
                       int64_t* grid) {
#else
bool launch_group_precise(bool post, int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s,
                          int64_t* grid) {
#endif
  return post ? launch_g_shape<true>(G, DPL, nv, a, lds, s, grid) : launch_g_shape<false>(G, DPL, nv, a, lds, s, grid);
}

}  // namespace nfn
