// nfn_launch.h — host-side launch wrappers shared by the translation units.
// Each wrapper instantiates its kernel templates in exactly one .hip file so the
// instantiations compile in parallel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "nfn_device.h"

#include <hip/hip_ext.h>

namespace nfn {

// Record `msg` as this thread's nfn_last_error() and return `code` (nfn_api.hip).
int32_t set_error(int32_t code, const char* msg);

// nfn_set_launch_events: the calling thread's pending (start, stop) pair (nfn_api.hip).
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents& launch_events();

// The measurement hook belongs to the very next API call: that call's first launch takes
// it, and whatever the call does (a validation error, B == 0, a memset-only path) the hook
// is disarmed when it returns, so it never times an unrelated later call.  Every extern "C"
// entry point that can launch holds one.
struct HookScope {
  HookScope() = default;
  HookScope(const HookScope&) = delete;
  HookScope& operator=(const HookScope&) = delete;
  ~HookScope() { launch_events() = LaunchEvents{}; }
};

// Every kernel launch of the library: a plain launch, or — when the caller armed the
// measurement hook — hipExtLaunchKernel with the pending events (the dispatch's own
// timestamps), after which the hook clears.
template <typename... Args, typename F = void (*)(Args...)>
inline void nfn_launch(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t s, Args... args) {
  LaunchEvents& ev = launch_events();
  if (ev.start != nullptr || ev.stop != nullptr) {
    const LaunchEvents e = ev;
    ev = LaunchEvents{};
    hipExtLaunchKernelGGL(kernel, grid, block, lds, s, e.start, e.stop, 0u, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
  }
}

// Tuning / diagnostic knobs.  Only the NFN_DIAG build (libnfn_hip_diag.so, built for
// tools/microbench.py) reads them from the environment; in the release library every
// knob is its measured default, so no environment variable can change a result.
#ifdef NFN_DIAG
inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
#else
inline int env_int(const char*, int dflt) { return dflt; }
#endif

// 3 * IA + IB when the d = 1 program alternates two of (planar, radial) — IA, IB, IA, ...,
// IA == IB for a homogeneous chain — over 2 <= K <= 16 flows; -1 otherwise.  Such programs
// run the compile-time pair bodies (chain1_fast_hpairs / grad1_hpairs).
inline int hpair_types(const ChainArgs& a) {
  const int K = a.prog.K;
  if (a.d != 1 || K < 2 || K > 16) return -1;
  const uint32_t ty = a.prog.types[0];
  const int ia = (int)(ty & 3u), ib = (int)((ty >> 2) & 3u);
  if (ia > NFN_FLOW_RADIAL || ib > NFN_FLOW_RADIAL) return -1;
  for (int k = 0; k < K; ++k)
    if ((int)((ty >> (2 * k)) & 3u) != ((k & 1) ? ib : ia)) return -1;
  return 3 * ia + ib;
}

// A persistent grid never exceeds the workspace's partial slots (ChainArgs::grid_cap).
inline int64_t cap_grid(int64_t grid, const ChainArgs& a) {
  return a.grid_cap > 0 ? std::min(grid, a.grid_cap) : grid;
}

// CU count of the current device, queried once per device and process (a launch
// below 2^20 samples takes ~10 us, so no runtime query sits on the launch path).
inline int cu_count() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cached[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev >= 0 && dev < kMaxDev) {
    const int c = cached[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  if (dev >= 0 && dev < kMaxDev) cached[dev].store(n, std::memory_order_relaxed);
  return n;
}

// Resident workgroups per CU of (kernel, threads, LDS bytes): the occupancy query runs
// once per key and process.  (The answer depends on the kernel's resources only, which
// are the same on every MI355X of a node.)
inline int occupancy_cached(const void* kfn, int threads, size_t lds) {
  struct Key {
    const void* f;
    int threads;
    size_t lds;
    int occ;
  };
  static std::mutex mu;
  static std::vector<Key> table;
  {
    std::lock_guard<std::mutex> g(mu);
    for (const Key& k : table)
      if (k.f == kfn && k.threads == threads && k.lds == lds) return k.occ;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kfn, threads, lds) != hipSuccess || occ <= 0) return 1;
  std::lock_guard<std::mutex> g(mu);
  if (table.size() < 4096) table.push_back({kfn, threads, lds, occ});
  return occ;
}

// Persistent grid: CUs x resident workgroups (occupancy query, or NFN_WG_PER_CU).
template <typename K>
inline int64_t persistent_grid(K kfn, int threads, size_t lds, int64_t units) {
  int occ = env_int("NFN_WG_PER_CU", 0);
  if (occ <= 0) occ = occupancy_cached(reinterpret_cast<const void*>(kfn), threads, lds);
  return std::min<int64_t>(units, (int64_t)cu_count() * occ);
}

// nfn_persistent.hip (compiled once per math mode)
bool launch_persistent_fast(bool post, int dm, int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s,
                            int64_t* grid);
bool launch_persistent_precise(bool post, int dm, int Q, const ChainArgs& a, int T, size_t lds, hipStream_t s,
                               int64_t* grid);
// nfn_persistent.hip (fast-math unit): d = 1 posterior on the wave1 pipeline, Q in {2, 4, 8, 16}
void launch_posterior_wave1(int Q, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid);
int posterior_wave1_wgs_per_cu();
// nfn_persistent.hip (fast-math unit): the Chain bijector (forward + fldj) on the wave1
// pipeline for the layer's contiguous reversed blocks, Q in {2, 4, 8, 16}
bool launch_fwd_ldj_wave1(int Q, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid);
// nfn_group.hip (compiled once per math mode); false if (G, DPL, nv) has no instance
bool launch_group_fast(bool post, int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s,
                       int64_t* grid);
bool launch_group_precise(bool post, int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s,
                          int64_t* grid);
// nfn_group.hip (fast-math unit): the Chain bijector for d >= 4 over contiguous layer rows
bool launch_group1_fwd(int G, int DPL, int nv, const ChainArgs& a, size_t lds, hipStream_t s, int64_t* grid);
// nfn_tile.hip
void launch_tile(bool fast, bool post, int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s);
void launch_chain_fwd_ldj(bool fast, int dm, const ChainArgs& a, dim3 grid, dim3 block, size_t lds, float* z_out,
                          float* ldj_out, hipStream_t s);
void launch_flow(bool fast, int dm, int32_t flow_id, const float* z, int64_t z_bstride, const float* tk,
                 int64_t t_rowstride, int64_t B, int32_t d, float* z_out, float* ldj_out, hipStream_t s);
// nfn_grad.hip
void launch_grad(bool fast, int dm, const GradArgs& ga, dim3 grid, size_t lds, hipStream_t s);
// one bijector's vector-Jacobian product (nfn_flow_vjp_f32)
struct FlowVjpArgs {
  const float* z;
  int64_t z_bstride;
  const float* t;
  int64_t t_rowstride;
  int64_t B;
  const float* g_z;    // (B, d) contiguous or NULL (= 0)
  const float* g_ldj;  // (B,) or NULL (= 0)
  float* dz;           // (B, d) contiguous or NULL
  float* dt;           // (B, ps) contiguous or NULL
  int32_t flow_id;
  int32_t d;
  int32_t ps;
};
void launch_flow_vjp(bool fast, int dm, const FlowVjpArgs& v, hipStream_t s);
// wave-owned persistent form; false if (dm, nv) has no instance
bool launch_grad_wave(bool fast, int dm, int nv, const GradArgs& ga, size_t lds_block, int waves_per_block,
                      hipStream_t s, int64_t* grid);
// nfn_grad_group.hip (compiled once per math mode); false if (G, DPL, nv) has no instance
bool launch_grad_group_fast(int G, int DPL, int nv, const GradArgs& ga, size_t lds, hipStream_t s, int64_t* grid);
bool launch_grad_group_precise(int G, int DPL, int nv, const GradArgs& ga, size_t lds, hipStream_t s,
                               int64_t* grid);
// chain_dense1_kernel's t tile: column-major at this padded column stride (floats),
// overlaying the wave's h tile (dead once the A fragments are in registers): one
// wave's LDS region in floats
constexpr int kCS = 68;
__host__ __device__ inline int dense1_wave_floats(int P, int SH) { return std::max(64 * SH, (P + 1) * kCS); }
// chain_dense1_grad_kernel: the t tile ((P + 2) columns) + K x 64 flow inputs, the h
// rows (64 x SH) overlaying both (dead before either is written)
__host__ __device__ inline int dense1_grad_wave_floats(int P, int SH, int K) {
  return std::max(64 * SH, (P + 2) * kCS + K * 64);
}
// nfn_dense.hip; false if (dm, H) has no instance
bool launch_dense(bool fast, int dm, int nvh, const DenseArgs& da, size_t lds, hipStream_t s, int64_t* grid);
bool launch_posterior_dense(bool fast, int dm, const DenseArgs& da, hipStream_t s, int64_t* grid);
// d = 1 fused Dense forward (post = false) / posterior (post = true) for an alternating
// program, sel = hpair_types(da.c); each sel's kernels are their own unit (nfn_dense.hip
// built with -DNFN_DENSE_HP=sel).  False: no kernel for this H.
bool launch_dense1_hpair(int sel, bool post, const DenseArgs& da, hipStream_t s, int64_t* grid);
bool launch_dense1_hpair_0(bool post, const DenseArgs& da, hipStream_t s, int64_t* grid);
bool launch_dense1_hpair_1(bool post, const DenseArgs& da, hipStream_t s, int64_t* grid);
bool launch_dense1_hpair_3(bool post, const DenseArgs& da, hipStream_t s, int64_t* grid);
bool launch_dense1_hpair_4(bool post, const DenseArgs& da, hipStream_t s, int64_t* grid);
// nfn_dense_grad.hip: returns the number of per-workgroup partials written (0 = no instance)
int64_t launch_dense_grad(bool fast, int dm, const DenseGradArgs& g, size_t lds, int64_t max_parts, hipStream_t s);
void launch_sum_partials(const float* part, int64_t nparts, int n, float* gW, float* gb, int nW, hipStream_t s);
// nfn_sample.hip
void launch_sample(bool fast, int dm, const SampleArgs& sa, dim3 grid, dim3 block, size_t lds, hipStream_t s);
// nfn_grid.hip
void launch_grid(bool fast, int dm, const GridArgs& ga, dim3 grid, dim3 block, size_t lds, hipStream_t s);
// nfn_misc.hip
struct SplitArgs {
  const float* t;
  int64_t rs;  // row stride of t (floats)
  int64_t B;
  float* dst;
  int32_t W;  // sum of the widths
  int32_t nblocks;
  int32_t widths[NFN_MAX_FLOWS];
};
void launch_split_blocks(const SplitArgs& sa, hipStream_t s);
void launch_reduce_partials(const double* ws, double* out, hipStream_t s);
void launch_reduce_f64(const double* in, int64_t n, double* out, hipStream_t s);
void launch_posterior_merge(bool fast, const float2* parts, int nsplit, int S, int64_t B, float* out, double* partials,
                            double* out_sum, uint32_t epoch, hipStream_t s);

}  // namespace nfn
