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

namespace nfn {
namespace {

template <int DM, bool FAST>
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
    case 1: chain_grid_kernel<1, FAST><<<grid, block, lds, s>>>(ga); break;
    case 2: chain_grid_kernel<2, FAST><<<grid, block, lds, s>>>(ga); break;
    case 4: chain_grid_kernel<4, FAST><<<grid, block, lds, s>>>(ga); break;
    case 8: chain_grid_kernel<8, FAST><<<grid, block, lds, s>>>(ga); break;
    case 16: chain_grid_kernel<16, FAST><<<grid, block, lds, s>>>(ga); break;
    default: chain_grid_kernel<32, FAST><<<grid, block, lds, s>>>(ga); break;
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
