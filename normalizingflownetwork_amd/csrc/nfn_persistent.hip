// nfn_persistent.hip — instantiations of chain_persistent_kernel (d <= 32, P <= 64).
// Compiled twice: -DNFN_FAST=1 (fast transcendentals) and -DNFN_FAST=0 (precise).
#include "nfn_launch.h"

#ifndef NFN_FAST
#error "compile with -DNFN_FAST=0 or -DNFN_FAST=1"
#endif

namespace nfn {
namespace {

constexpr bool kFast = NFN_FAST != 0;

#if NFN_FAST
// The compile-time pair bodies (chain1_fast_hpairs) of an alternating program, sel =
// hpair_types(a).
template <int Q, int U>
auto posterior_hpair_kernel(int sel) {
  switch (sel) {
    case 0: return posterior_wave1_kernel<Q, true, hpair_form(0, 0, U)>;
    case 1: return posterior_wave1_kernel<Q, true, hpair_form(0, 1, U)>;
    case 3: return posterior_wave1_kernel<Q, true, hpair_form(1, 0, U)>;
    default: return posterior_wave1_kernel<Q, true, hpair_form(1, 1, U)>;
  }
}

template <int Q, int U = 1>
auto wave1_hpair_kernel(int sel) {
  switch (sel) {
    case 0: return chain_wave1_kernel<true, Q, true, false, hpair_form(0, 0, U)>;
    case 1: return chain_wave1_kernel<true, Q, true, false, hpair_form(0, 1, U)>;
    case 3: return chain_wave1_kernel<true, Q, true, false, hpair_form(1, 0, U)>;
    default: return chain_wave1_kernel<true, Q, true, false, hpair_form(1, 1, U)>;
  }
}
#endif

// d = 1 wave-tile kernel (chain_wave1_kernel) for rows of exactly Q float4.
template <int Q>
void launch_w1(const ChainArgs& a, int T, size_t lds, hipStream_t s, int64_t* grid_out) {
  auto kfn = (kFast && a.prog.K <= 16 && env_int("NFN_PACKED", 1) == 1) ? chain_wave1_kernel<kFast, Q, kFast>
                                                                        : chain_wave1_kernel<kFast, Q, false>;
#if NFN_FAST
  if (a.prog.K <= kPairsMaxKStream && env_int("NFN_PACKED", 1) == 1)
    kfn = chain_wave1_kernel<true, Q, true, false, kChainPairs>;
  // an alternating program (hpair_types): compile-time pair bodies.  With the log_prob stores
  // write-through (kOutAux) they stream C2 at 0.378-0.380 ms against 0.395-0.400 for the packed
  // loop on three boxes (bench harness, profiles/r05/r05u / r05v / r05w_*; round 3's loop
  // library 0.380 on the same box); with non-temporal stores the two forms traded places box to
  // box (r05m vs r05u), which is why round 5 first moved C2 back to the loop
  if (hpair_types(a) >= 0 && env_int("NFN_PACKED", 1) == 1) kfn = wave1_hpair_kernel<Q>(hpair_types(a));
#ifdef NFN_DIAG
  // chain-form A/B (diag build): 0 = loop, 3 = pairs, 2 = the C2 program at compile time
  const int cm = env_int("NFN_CHAIN_FORM", -1);
  if (cm == kChainLoop && a.prog.K <= 16) kfn = chain_wave1_kernel<true, Q, true>;
  if (cm == kChainPairs && a.prog.K <= 16) kfn = chain_wave1_kernel<true, Q, true, false, kChainPairs>;
  if (cm == kStaticProg && a.prog.K == kStaticK[0] && a.prog.types[0] == kStaticTypes[0])
    kfn = chain_wave1_kernel<true, Q, true, false, kStaticProg>;
  if (cm == kChainHPair && hpair_types(a) >= 0)
    kfn = env_int("NFN_HPAIR_U", 1) == 0 ? wave1_hpair_kernel<Q, 0>(hpair_types(a)) : wave1_hpair_kernel<Q>(hpair_types(a));
#endif
#endif
  const int64_t units = a.ntiles;
  const int teams = T / 64;
  // Resident workgroups per CU: a long chain (C2: 10 flows) keeps each wave busy
  // long enough that 2 waves per SIMD hide the streamed rows and fewer bytes in
  // flight stream faster (C2: 0.365 ms at 2 vs 0.418 at 4 per CU); a short chain
  // (C1: 2 flows) in the loop form is latency-bound and wants all 4 (0.127 vs 0.173 ms); as
  // compile-time pair bodies it is stream-bound and streams faster at 3 (C1 0.131-0.132 vs
  // 0.142 ms, memory-only 0.131 vs 0.140; profiles/r04/r04v_c1occ.log, r04w_c1occ.log).
  int64_t grid;
  const int wgs = a.prog.K >= 4 ? 2 : (kFast && hpair_types(a) >= 0 ? 3 : 4);
  if (env_int("NFN_WG_PER_CU", 0) > 0)
    grid = persistent_grid(kfn, T, lds, (units + teams - 1) / teams);
  else
    grid = std::min<int64_t>((units + teams - 1) / teams, (int64_t)cu_count() * wgs);
  grid = cap_grid(grid, a);
  *grid_out = grid;
  nfn_launch(kfn, dim3((unsigned)grid), dim3(T), lds, s, a);
}

#if NFN_FAST
// the Bijector API's Chain (forward + fldj) on the same pipeline (chain_wave1_kernel<FWD>)
template <int Q>
void launch_fw1(const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid_out) {
  auto kfn = chain_wave1_kernel<true, Q, true, true>;
  const int teams = kMaxBlock / 64;
  const int64_t grid = std::min<int64_t>((a.ntiles + teams - 1) / teams, (int64_t)cu_count() * (a.prog.K >= 4 ? 2 : 4));
  *grid_out = std::max<int64_t>(1, grid);
  nfn_launch(kfn, dim3((unsigned)*grid_out), dim3(kMaxBlock), lds, s, a);
}
#endif

template <bool POST>
bool try_wave1(int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s, int64_t* g) {
  // the posterior (C5) stays on the generic kernel: measured 0.177 vs 0.181 ms there
  if (POST || a.d != 1 || a.ownrow != 2 || !a.nt || env_int("NFN_WAVE1", 1) == 0) return false;
  // 32-bit lane byte offsets: a tile's 64 rows (and y entries) must span < 2 GiB
  if (a.t_rowstride * 256 >= (int64_t)1 << 31 || a.y_bstride * 256 >= (int64_t)1 << 31) return false;
  switch (Q) {
    case 2: launch_w1<2>(a, T, lds, s, g); return true;
    case 4: launch_w1<4>(a, T, lds, s, g); return true;
    case 8: launch_w1<8>(a, T, lds, s, g); return true;
    case 16: launch_w1<16>(a, T, lds, s, g); return true;
    default: return false;
  }
}

template <int DM, int NV, bool POST>
void launch_p(const ChainArgs& a, int T, size_t lds, hipStream_t s, int64_t* grid_out) {
  // the packed-program fast path exists for d = 1 chains of <= 16 flows
  auto kfn = (DM == 1 && kFast && a.prog.K <= 16 && env_int("NFN_PACKED", 1) == 1)
                 ? chain_persistent_kernel<DM, kFast, NV, POST, DM == 1 && kFast>
                 : chain_persistent_kernel<DM, kFast, NV, POST, false>;
  // units = tiles x draw ranges; in wave mode a workgroup runs T/64 units at a time
  const int64_t units = a.ntiles * (POST ? a.nsplit : 1);
  const int teams = a.ownrow == 2 ? T / 64 : 1;
  const int64_t grid = cap_grid(persistent_grid(kfn, T, lds, (units + teams - 1) / teams), a);
  *grid_out = grid;
  nfn_launch(kfn, dim3((unsigned)grid), dim3(T), lds, s, a);
}

template <int DM, bool POST>
void launch_p_nv(int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s, int64_t* g) {
  if (Q <= 2)
    launch_p<DM, 2, POST>(a, T, lds, s, g);
  else if (Q <= 4)
    launch_p<DM, 4, POST>(a, T, lds, s, g);
  else if (Q <= 8)
    launch_p<DM, 8, POST>(a, T, lds, s, g);
  else
    launch_p<DM, 16, POST>(a, T, lds, s, g);
}

template <bool POST>
void launch_p_dm(int dm, int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s, int64_t* g) {
  switch (dm) {
    case 1: launch_p_nv<1, POST>(Q, a, T, lds, s, g); break;
    case 2: launch_p_nv<2, POST>(Q, a, T, lds, s, g); break;
    case 4: launch_p_nv<4, POST>(Q, a, T, lds, s, g); break;
    case 8: launch_p_nv<8, POST>(Q, a, T, lds, s, g); break;
    case 16: launch_p_nv<16, POST>(Q, a, T, lds, s, g); break;
    default: launch_p_nv<32, POST>(Q, a, T, lds, s, g); break;
  }
}

#if NFN_FAST
template <int Q>
void launch_pw1(const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid_out) {
  // two flows per dispatch (chain1_fast_pairs, bitwise the loop's values); an alternating
  // program (hpair_types: C5's) as compile-time pair bodies, C5 0.182-0.186 -> 0.169 ms
  // (profiles/r04/r04l_hpair*.log)
  auto kfn = (a.prog.K <= 16 && env_int("NFN_PACKED", 1) == 1) ? posterior_wave1_kernel<Q, true, kChainPairs>
                                                                : posterior_wave1_kernel<Q, false>;
  if (hpair_types(a) >= 0 && env_int("NFN_PACKED", 1) == 1) kfn = posterior_hpair_kernel<Q, 1>(hpair_types(a));
#ifdef NFN_DIAG
  const int cm = env_int("NFN_CHAIN_FORM", -1);
  if (cm == kChainLoop && a.prog.K <= 16) kfn = posterior_wave1_kernel<Q, true>;
  if (cm == kChainPairs && a.prog.K <= 16) kfn = posterior_wave1_kernel<Q, true, kChainPairs>;
  if (cm == kStaticProg && a.prog.K == kStaticK[0] && a.prog.types[0] == kStaticTypes[0])
    kfn = posterior_wave1_kernel<Q, true, kStaticProg>;
  if (cm == kChainHPair && hpair_types(a) >= 0) {  // NFN_HPAIR_U pairs per loop trip
    const int u = env_int("NFN_HPAIR_U", 5), sel = hpair_types(a);
    kfn = u == 0 ? posterior_hpair_kernel<Q, 0>(sel)
        : u == 1 ? posterior_hpair_kernel<Q, 1>(sel)
        : u == 2 ? posterior_hpair_kernel<Q, 2>(sel) : posterior_hpair_kernel<Q, 5>(sel);
  }
#endif
  const int64_t units = a.ntiles * a.nsplit;
  const int64_t grid = cap_grid(std::min<int64_t>((units + 3) / 4, (int64_t)cu_count() * posterior_wave1_wgs_per_cu()), a);
  *grid_out = grid;
#ifdef NFN_DIAG
  // experiment: two draws per step (posterior_wave1x2_kernel), whole-tile units only
  if (env_int("NFN_POST_X2", 0) == 1 && a.nsplit == 1 && a.prog.K <= 16) {
    nfn_launch(posterior_wave1x2_kernel<Q>, dim3((unsigned)grid), dim3(kMaxBlock), 2 * (lds - 16) + 16, s, a);
    return;
  }
#endif
  nfn_launch(kfn, dim3((unsigned)grid), dim3(kMaxBlock), lds, s, a);
}
#endif

}  // namespace

#if NFN_FAST
// Resident workgroups per CU of posterior_wave1_kernel (4 waves each).
int posterior_wave1_wgs_per_cu() {
  const int w = env_int("NFN_WG_PER_CU", 0);
  return w > 0 ? w : 2;
}

bool launch_fwd_ldj_wave1(int Q, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid) {
  switch (Q) {
    case 2: launch_fw1<2>(a, lds, s, grid); return true;
    case 4: launch_fw1<4>(a, lds, s, grid); return true;
    case 8: launch_fw1<8>(a, lds, s, grid); return true;
    case 16: launch_fw1<16>(a, lds, s, grid); return true;
  }
  return false;
}

void launch_posterior_wave1(int Q, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid) {
  switch (Q) {
    case 2: launch_pw1<2>(a, lds, s, grid); break;
    case 4: launch_pw1<4>(a, lds, s, grid); break;
    case 8: launch_pw1<8>(a, lds, s, grid); break;
    default: launch_pw1<16>(a, lds, s, grid); break;
  }
}

bool launch_persistent_fast(bool post, int dm, int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s,
                            int64_t* grid) {
#else
bool launch_persistent_precise(bool post, int dm, int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s,
                               int64_t* grid) {
#endif
  if (Q < 1 || Q > 16) return false;
  if (dm == 1 && (post ? try_wave1<true>(Q, a, T, lds, s, grid) : try_wave1<false>(Q, a, T, lds, s, grid)))
    return true;
  if (post)
    launch_p_dm<true>(dm, Q, a, T, lds, s, grid);
  else
    launch_p_dm<false>(dm, Q, a, T, lds, s, grid);
  return true;
}

}  // namespace nfn
