// nfn_tile.hip — one-tile-per-workgroup fallback kernels (unaligned / strided /
// broadcast parameter rows) and the single-bijector kernel of the Bijector API.
#include "nfn_launch.h"

namespace nfn {
namespace {

template <int DM, bool FAST>
void launch_t(const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s, bool posterior) {
  if (posterior)
    hipLaunchKernelGGL((posterior_lse_kernel<DM, FAST>), grid, block, lds, s, a);
  else
    hipLaunchKernelGGL((chain_logprob_kernel<DM, FAST>), grid, block, lds, s, a);
}

template <bool FAST>
void launch_t_dm(int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s, bool post) {
  switch (dm) {
    case 1: launch_t<1, FAST>(a, grid, block, lds, s, post); break;
    case 2: launch_t<2, FAST>(a, grid, block, lds, s, post); break;
    case 4: launch_t<4, FAST>(a, grid, block, lds, s, post); break;
    case 8: launch_t<8, FAST>(a, grid, block, lds, s, post); break;
    case 16: launch_t<16, FAST>(a, grid, block, lds, s, post); break;
    default: launch_t<32, FAST>(a, grid, block, lds, s, post); break;
  }
}

template <int DM, bool FAST>
void launch_f(int32_t flow_id, const float* z, int64_t zs, const float* tk, int64_t ts, int64_t B, int32_t d,
              float* z_out, float* ldj_out, hipStream_t s) {
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  hipLaunchKernelGGL((flow_fwd_ldj_kernel<DM, FAST>), dim3((unsigned)nblk), dim3(kMaxBlock), 0, s, flow_id, z, zs,
                     tk, ts, B, d, z_out, ldj_out);
}

template <bool FAST>
void launch_f_dm(int dm, int32_t flow_id, const float* z, int64_t zs, const float* tk, int64_t ts, int64_t B,
                 int32_t d, float* z_out, float* ldj_out, hipStream_t s) {
  switch (dm) {
    case 1: launch_f<1, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 2: launch_f<2, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 4: launch_f<4, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 8: launch_f<8, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    case 16: launch_f<16, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
    default: launch_f<32, FAST>(flow_id, z, zs, tk, ts, B, d, z_out, ldj_out, s); break;
  }
}

}  // namespace

void launch_tile(bool fast, bool post, int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  if (fast)
    launch_t_dm<true>(dm, a, grid, block, lds, s, post);
  else
    launch_t_dm<false>(dm, a, grid, block, lds, s, post);
}

void launch_flow(bool fast, int dm, int32_t flow_id, const float* z, int64_t z_bstride, const float* tk,
                 int64_t t_rowstride, int64_t B, int32_t d, float* z_out, float* ldj_out, hipStream_t s) {
  if (fast)
    launch_f_dm<true>(dm, flow_id, z, z_bstride, tk, t_rowstride, B, d, z_out, ldj_out, s);
  else
    launch_f_dm<false>(dm, flow_id, z, z_bstride, tk, t_rowstride, B, d, z_out, ldj_out, s);
}

}  // namespace nfn
