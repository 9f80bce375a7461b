// nfn_api.hip — the extern "C" ABI of libnfn_hip.so (include/nfn.h): argument
// validation, the flow program (reversed parameter layout,
// estimators/DistributionLayers.py:270-277), kernel selection and launch.
#include <atomic>
#include <string>

#include "nfn_launch.h"

#define NFN_VERSION_NUM NFN_ABI_VERSION  // include/nfn.h: the version history

namespace nfn {

thread_local std::string g_last_error;
thread_local LaunchEvents g_launch_events;  // nfn_set_launch_events

LaunchEvents& launch_events() { return g_launch_events; }

int32_t set_error(int32_t code, const char* msg) {
  g_last_error = msg;
  return code;
}

namespace {

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------

int32_t fail(int32_t code, const std::string& msg) { return set_error(code, msg.c_str()); }

int32_t param_size(int32_t id, int32_t d) {
  switch (id) {
    case NFN_FLOW_PLANAR: return 2 * d + 1;
    case NFN_FLOW_RADIAL: return d + 2;
    case NFN_FLOW_AFFINE: return 2 * d;
    default: return -1;
  }
}

int g_math_mode = [] {
  const char* e = getenv("NFN_MATH");
  return (e && strcmp(e, "precise") == 0) ? 1 : 0;
}();

bool use_fast_math() { return g_math_mode == 0; }

// Validates the flow list and fills the program (parameter offsets of the
// reversed layout, DistributionLayers.py:270-277).  Returns P or < 0.
int32_t build_program(const int32_t* flow_ids, int32_t K, int32_t d, int32_t trainable, FlowProgram* prog) {
  if (d < 1 || d > NFN_MAX_DIMS) return fail(NFN_E_SHAPE, "n_dims must be in [1, " + std::to_string(NFN_MAX_DIMS) + "]");
  if (K < 0 || K > NFN_MAX_FLOWS) return fail(NFN_E_FLOW_ID, "number of flows must be in [0, " + std::to_string(NFN_MAX_FLOWS) + "]");
  if (K > 0 && !flow_ids) return fail(NFN_E_NULLPTR, "flow_ids is NULL");
  int32_t off = trainable ? 2 * d : 0;
  // blocks are laid out for flow_types[K-1], ..., flow_types[0]
  for (int32_t k = K - 1; k >= 0; --k) {
    const int32_t ps = param_size(flow_ids[k], d);
    if (ps < 0) return fail(NFN_E_FLOW_ID, "unknown flow id " + std::to_string(flow_ids[k]));
    if (prog) prog->step[k] = (off << 2) | flow_ids[k];
    off += ps;
  }
  if (prog) {
    prog->K = K;
    for (int q = 0; q < 4; ++q) prog->types[q] = 0;
    for (int32_t k = 0; k < K; ++k) prog->types[k >> 4] |= (uint32_t)flow_ids[k] << (2 * (k & 15));
  }
  return off;
}

int dm_for(int d) {
  if (d <= 1) return 1;
  if (d <= 2) return 2;
  if (d <= 4) return 4;
  if (d <= 8) return 8;
  if (d <= 16) return 16;
  return 32;
}

struct TileGeom {
  int rows;     // samples per tile
  int threads;  // workgroup size (>= 64: one full wave even for narrow tiles)
  int lds_stride;
  size_t lds_bytes;
};

TileGeom tile_geom(int P) {
  TileGeom g;
  g.lds_stride = P | 1;  // odd stride: conflict-free per-lane ds_read_b32
  const size_t row_bytes = (size_t)g.lds_stride * sizeof(float);
  int rows = kMaxBlock;
#ifdef NFN_DIAG
  if (const char* e = getenv("NFN_TILE_ROWS")) {  // tuning knob: 64, 128, 192 or 256
    const int r = atoi(e);
    if (r >= 64 && r <= kMaxBlock && r % 64 == 0) rows = r;
  }
#endif
  while (rows > 64 && (size_t)rows * row_bytes > (size_t)kLdsTileBudget) rows -= 64;
  // very wide rows (up to NFN_MAX_FLOWS x (2 NFN_MAX_DIMS + 1) floats): fewer samples
  // per tile so the tile fits the 160 KiB of LDS a workgroup may hold
  while (rows > 1 && (size_t)rows * row_bytes > (size_t)kLdsMaxBytes) rows >>= 1;
  g.rows = rows;
  g.threads = std::max(rows, 64);
  g.lds_bytes = P > 0 ? (size_t)rows * row_bytes : 0;
  return g;
}

// NFN_LOAD_MODE = auto|coop|ownrow|tile|wave selects the tile-streaming strategy
// (tuning / tests); auto = the measured default.
enum LoadMode { kAuto = 0, kCoop = 1, kOwnRow = 2, kTile = 3, kWave = 4 };

int load_mode_env() {
#ifndef NFN_DIAG
  return kAuto;  // release build: the measured default only
#endif
  const char* e = getenv("NFN_LOAD_MODE");
  if (!e) return kAuto;
  if (!strcmp(e, "coop")) return kCoop;
  if (!strcmp(e, "ownrow")) return kOwnRow;
  if (!strcmp(e, "tile")) return kTile;
  if (!strcmp(e, "wave")) return kWave;
  return kAuto;
}

int group_lds_stride(int P, int G) {
  int Sx = ((P + G - 1) / G) * G;
  if (((Sx / G) & 1) == 0) Sx += G;  // S / G odd
  if (G >= 4) {
    while (Sx % 4) Sx += 2 * G;  // float4 LDS writes (G >= 4: S = G * odd is a multiple of 4)
  }
  return Sx;
}

// Default (G, DPL) per event-size bound DM, and the alternates a tuning run may
// request with NFN_GROUP_LANES (fast math, plain chain only).
void group_shape(int dm, int want_g, int* G, int* DPL) {
  struct Shape { int dm, g, dpl; };
  static const Shape defaults[] = {{4, 4, 1}, {8, 4, 2}, {16, 4, 4}, {32, 8, 4}};
  static const Shape alts[] = {{8, 8, 1}, {16, 8, 2}, {8, 2, 4}};
  for (const Shape& x : defaults)
    if (x.dm == dm) { *G = x.g; *DPL = x.dpl; }
  for (const Shape& x : alts)
    if (x.dm == dm && x.g == want_g) { *G = x.g; *DPL = x.dpl; }
}

// Number of (sum, non-finite count) partial pairs the workspace holds: one per
// workgroup of the smallest tile any launch uses (64 rows, fewer for very wide
// rows).  Persistent launches whose grid could exceed it are capped at it
// (ChainArgs::grid_cap), so no launch writes past the workspace.
int64_t raw_partials(int64_t B, int P) {
  const int rows = std::min(64, tile_geom(P < 0 ? 0 : P).rows);
  return (B + rows - 1) / rows;
}

// The plain chain runs a batch longer than this as consecutive launches over its
// slices: the persistent grid's static tile stride drifts apart over a long launch
// (C2 at 2^27 as one launch 3.33 ms, as eight 2^24 launches 2.90-3.01 ms).
// Tuning knob NFN_CHUNK_LOG2 (0 = one launch), never below kMinChunkLog2.
constexpr int kChunkLog2 = 24, kMinChunkLog2 = 20;
int64_t chain_chunk_rows() {
  const int l = env_int("NFN_CHUNK_LOG2", kChunkLog2);
  return l <= 0 ? 0 : (int64_t)1 << std::max(l, kMinChunkLog2);
}

// Each chunk's grid is capped at raw_partials(chunk) slots, which exceed the slice's
// share of raw_partials(B) by at most one: one spare slot per smallest chunk.
int64_t partials_capacity(int64_t B, int P) {
  return raw_partials(B, P) + (B >> kMinChunkLog2) + 1;
}

// Doubles of the [count | ticket | (sum, count) pairs] block.
int64_t partials_doubles(int64_t B, int P) { return 2 + 2 * partials_capacity(B, P); }

// Draw ranges per tile for the posterior: enough (64-row tile, range) units for
// ~2 per resident wave (32 waves per CU on a 256-CU MI355X), at most 16 ranges.
// ONE function sizes the workspace's split region and bounds every launch's split.
int posterior_split(int64_t B) {
  constexpr int64_t kTarget = 2048 * 4;
  const int64_t ntiles = (B + 63) / 64;
  if (ntiles <= 0) return 1;
  return (int)std::max<int64_t>(1, std::min<int64_t>(16, (kTarget + ntiles - 1) / ntiles));
}

int32_t check_hip(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NFN_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return NFN_OK;
}

// The in-kernel finish counts workgroups on an epoch-tagged ticket at workspace[1]
// (write_partial in nfn_device.h): every summed call gets a fresh non-zero epoch, so the
// workspace needs no initialisation and no memset launch precedes the kernel (a ROCm
// memset is a fill-kernel launch: ~5 us per call, 1.3 % of the C2 step, 3 % of C5's).
uint32_t next_epoch() {
  static std::atomic<uint32_t> counter{0x9e3779b9u};
  uint32_t e;
  do {
    e = counter.fetch_add(1u, std::memory_order_relaxed);
  } while (e == 0u);
  return e;
}

// Every argument check of the plain chain / posterior entry points that does not depend
// on the launch shape: run before the first launch, so a rejected call has no side
// effect on the stream (also when a long batch runs as several chunk launches).
int32_t check_chain_args(const float* y, int64_t y_bstride, const float* t, int64_t t_drawstride,
                         int64_t t_rowstride, int32_t S, int64_t B, int32_t d, int32_t P, const float* y_mean,
                         const float* y_std, double* out_sum, double* workspace, bool posterior) {
  if (B < 0) return fail(NFN_E_SHAPE, "batch size must be >= 0");
  if (y_bstride < 0 || t_rowstride < 0 || t_drawstride < 0) return fail(NFN_E_SHAPE, "strides must be >= 0");
  if (y_bstride != 0 && y_bstride < d) return fail(NFN_E_SHAPE, "y batch stride < n_dims");
  if (t_rowstride != 0 && t_rowstride < P) return fail(NFN_E_SHAPE, "t row stride < total param size");
  if (posterior && S < 1) return fail(NFN_E_SHAPE, "number of draws must be >= 1");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  if (B == 0) return NFN_OK;
  if (!y) return fail(NFN_E_NULLPTR, "y is NULL");
  if (P > 0 && !t) return fail(NFN_E_NULLPTR, "t is NULL");
  if (out_sum && !workspace) return fail(NFN_E_NULLPTR, "workspace is NULL but out_sum requested");
  return NFN_OK;
}

// The forward streaming policy of the release library — measured defaults:
//  * t rows and log_prob are streamed once: non-temporal loads and stores (nt, nt_store);
//  * rotated tile slots in chain_wave1_kernel: each step a workgroup's waves take the slots
//    one workgroup further on; C2 -1.4 % and R10 -1.3 % against the plain walk in the bench
//    harness on two boxes (profiles/r05/r05zn, r05zq; two workgroups' shift gains nothing);
//  * wave priority raised around the tile hand-off (+1-2 % on C2, C5).
// Only the diagnostic build (libnfn_hip_diag.so) reads NFN_* overrides for A/B studies.
constexpr int kTileRot = 4;
void forward_stream_policy(ChainArgs& a) {
  a.nt = 1;
  a.nt_store = 1;
  a.tile_rot = kTileRot;
  a.prio = 1;
#ifdef NFN_DIAG
  // NFN_ABLATE_FLOWS=1: stream the same parameter rows but skip the flow math (memory only)
  if (env_int("NFN_ABLATE_FLOWS", 0) == 1) a.prog.K = 0;
  a.nt = env_int("NFN_NT_LOADS", 1) == 1 ? 1 : 0;
  a.nt_store = env_int("NFN_NT_STORES", 1) == 1 ? 1 : 0;
  a.ablate_loads = env_int("NFN_ABLATE_LOADS", 0) == 1 ? 1 : 0;
  a.tile_rot = std::max(0, env_int("NFN_TILE_ROT", kTileRot));  // >= 0: the kernel's slot walk only wraps upward
  a.tile_rot_g = std::max(0, env_int("NFN_TILE_ROT_G", 0));
  a.prio = std::min(std::max(env_int("NFN_PRIO", 1), 0), 2);  // 2 = + static split
#endif
}

// One launch over B samples.  A chunk of a longer batch (chunk_cap > 0) writes its
// partial pairs after the earlier chunks' (from slot pair_base, at most chunk_cap of
// them); only the last chunk finishes out_sum, over every chunk's pairs.
int32_t run_chain_launch(const float* y, int64_t y_bstride, const float* t, int64_t t_drawstride,
                         int64_t t_rowstride, int32_t S, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K,
                         int32_t trainable_base, const float* y_mean, const float* y_std, float* out,
                         double* out_sum, double* workspace, void* stream, bool posterior, int64_t pair_base,
                         int64_t chunk_cap, int64_t* grid_used) {
  ChainArgs a;
  memset(&a, 0, sizeof(a));
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
  if (P < 0) return P;
  forward_stream_policy(a);
  {
    const int32_t rc = check_chain_args(y, y_bstride, t, t_drawstride, t_rowstride, S, B, d, P, y_mean, y_std, out_sum,
                                        workspace, posterior);
    if (rc != NFN_OK) return rc;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (B == 0) {
    if (out_sum) {
      if (hipMemsetAsync(out_sum, 0, 2 * sizeof(double), s) != hipSuccess) return check_hip("hipMemsetAsync");
    }
    return NFN_OK;
  }
  if (!out && !workspace) return NFN_OK;
  const TileGeom g = tile_geom(P);
  a.y = y;
  a.t = t;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.out = out;
  a.partials = workspace ? workspace + 2 : nullptr;  // [count | ticket | pairs]
  a.out_sum = workspace ? out_sum : nullptr;         // finished in-kernel by the last workgroup
  a.epoch = a.out_sum ? next_epoch() : 0u;
  a.grid_cap = workspace ? (chunk_cap > 0 ? chunk_cap : partials_capacity(B, P)) : 0;
  a.pair_base = pair_base;
  a.y_bstride = y_bstride;
  a.t_rowstride = t_rowstride;
  a.t_drawstride = t_drawstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = g.lds_stride;
  a.trainable = trainable_base ? 1 : 0;
  a.S = posterior ? S : 1;
  a.vec4 = ((P & 3) == 0) && ((t_rowstride & 3) == 0) && ((t_drawstride & 3) == 0) &&
           ((reinterpret_cast<uintptr_t>(t) & 15) == 0);
  int64_t nblk = (B + g.rows - 1) / g.rows;
  if (nblk > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  const int dm = dm_for(d);
  const int Q = P >> 2;
  const int mode = load_mode_env();
  int G = 4, DPL = 1;
  // The plain forward with fast math and contiguous rows (chain_group1_kernel) runs
  // d in (4, 8] as 2 lanes x 4 dimensions per sample: half the per-sample scalar work
  // of 4 x 2 (C3 compute 0.40 -> 0.29 ms, kernel 0.400 -> 0.395 ms, now HBM-bound),
  // while the prefetch of its 32-row tiles still fits (<= 18 float4 per lane).
  const bool two_lane = !posterior && use_fast_math() && dm == 8 && t_rowstride == P && (Q + 1) / 2 <= 18;
  group_shape(dm, env_int("NFN_GROUP_LANES", two_lane ? 2 : 0), &G, &DPL);
  const int nv_group = (Q + G - 1) / G;  // float4 slots per lane: (64/G rows x Q) / 64
  const bool group_ok = a.vec4 && t_rowstride != 0 && d >= 4 && Q >= 1 && nv_group <= (G == 2 ? 18 : 16) &&
                        mode != kTile &&
                        mode != kCoop && mode != kOwnRow && mode != kWave && env_int("NFN_GROUP", 1) != 0;
  bool launched_group = false;
  if (group_ok) {
    const int R = 64 / G;  // samples per wave tile
    a.lds_stride = group_lds_stride(P, G);
    a.ntiles = (B + R - 1) / R;
    // four wave slots + pad: inactive lanes may read G * DPL floats past a row's block,
    // and the contiguous-row kernel parks out-of-tile float4 slots there (one per lane)
    const size_t lds = (size_t)(kMaxBlock / 64) * R * a.lds_stride * sizeof(float) +
                       std::max<size_t>((G * DPL + 4) * sizeof(float), 64 * 16);
    launched_group = use_fast_math() ? launch_group_fast(posterior, G, DPL, nv_group, a, lds, s, &nblk)
                                     : launch_group_precise(posterior, G, DPL, nv_group, a, lds, s, &nblk);
    if (!launched_group) a.lds_stride = g.lds_stride;
  }
  const bool persistent = !launched_group && a.vec4 && t_rowstride != 0 && Q >= 1 && Q <= 16 && mode != kTile;
  if (launched_group) {
    // launched above
  } else if (persistent) {
    const bool coop_ok = (Q & (Q - 1)) == 0 && g.rows % Q == 0;  // Q | 64 too (Q <= 16)
    // default: wave-tile streaming (measured fastest on C2/C5); coop / ownrow on request
    const bool wave = (mode == kWave || mode == kAuto) && coop_ok && g.rows % 64 == 0;
    a.ownrow = wave ? 2 : ((mode == kOwnRow || !coop_ok) ? 1 : 0);
    const int tile_rows = wave ? 64 : g.rows;
    const size_t lds_p = g.lds_bytes + 16;  // the packed d = 1 chain may read 3 floats past a row
    nblk = (B + tile_rows - 1) / tile_rows;
    a.ntiles = nblk;
    const bool fast = use_fast_math();
    if (posterior) {
      // draw split: more (tile, draw-range) units when the batch alone is too small
      // to fill the chip; needs the split region of the workspace
      // (the split region holds posterior_split(B) ranges; never more are used)
      int nsplit = workspace ? std::min(posterior_split(B), S) : 1;
      // d = 1, fast math, contiguous rows: posterior_wave1_kernel (draw-inner buffer
      // pipeline); it needs a split only when there are fewer tiles than resident waves
      const bool pw1 = fast && d == 1 && wave && a.nt && (Q == 2 || Q == 4 || Q == 8 || Q == 16) &&
                       t_rowstride * 256 < ((int64_t)1 << 31) && y_bstride * 256 < ((int64_t)1 << 31) &&
                       env_int("NFN_POST_WAVE1", 1) != 0;
      if (pw1) {
        const int64_t resident = (int64_t)cu_count() * posterior_wave1_wgs_per_cu() * (kMaxBlock / 64);
        nsplit = (int)std::min<int64_t>(nsplit, std::max<int64_t>(1, (resident + nblk - 1) / nblk));
      }
      if (env_int("NFN_POST_SPLIT", 0) > 0) nsplit = std::min(env_int("NFN_POST_SPLIT", 1), std::min(posterior_split(B), S));
      a.nsplit = nsplit;
      a.dps = (S + nsplit - 1) / nsplit;
      a.nsplit = (S + a.dps - 1) / a.dps;  // no empty ranges (<= nsplit)
      a.split_out = reinterpret_cast<float2*>(workspace + partials_doubles(B, P));
      if (a.nsplit > 1) a.grid_cap = 0;  // partials come from the merge kernel
      if (pw1)
        launch_posterior_wave1(Q, a, lds_p, s, &nblk);
      else if (fast)
        launch_persistent_fast(true, dm, Q, a, g.rows, lds_p, s, &nblk);
      else
        launch_persistent_precise(true, dm, Q, a, g.rows, lds_p, s, &nblk);
      if (a.nsplit > 1) {
        int32_t rc0 = check_hip("posterior kernel launch");
        if (rc0 != NFN_OK) return rc0;
        nblk = (B + kMaxBlock - 1) / kMaxBlock;
        launch_posterior_merge(fast, (const float2*)a.split_out, a.nsplit, S, B, out, workspace ? workspace + 2 : nullptr,
                               a.out_sum, a.epoch, s);
      }
    } else {
      if (fast) launch_persistent_fast(false, dm, Q, a, g.rows, lds_p, s, &nblk);
      else launch_persistent_precise(false, dm, Q, a, g.rows, lds_p, s, &nblk);
    }
  } else {
    if ((size_t)g.rows * ((size_t)g.lds_stride * sizeof(float)) > (size_t)kLdsMaxBytes)
      return fail(NFN_E_SHAPE, "parameter row too wide for LDS");
    a.tile_rows = g.rows;
    const dim3 grid((unsigned)nblk), block((unsigned)g.threads);
    launch_tile(use_fast_math(), posterior, dm, a, grid, block, g.lds_bytes, s);
  }
  if (grid_used) *grid_used = nblk;
  return check_hip(posterior ? "posterior kernel launch" : "chain kernel launch");
}

int32_t run_chain(const float* y, int64_t y_bstride, const float* t, int64_t t_drawstride, int64_t t_rowstride,
                  int32_t S, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                  const float* y_mean, const float* y_std, float* out, double* out_sum, double* workspace,
                  void* stream, bool posterior) {
  g_last_error.clear();
  const HookScope hook_scope;
  const int64_t chunk = posterior ? 0 : chain_chunk_rows();
  if (chunk <= 0 || B <= chunk || !y || (t == nullptr && t_rowstride != 0))
    return run_chain_launch(y, y_bstride, t, t_drawstride, t_rowstride, S, B, d, flow_ids, K, trainable_base, y_mean,
                            y_std, out, out_sum, workspace, stream, posterior, 0, 0, nullptr);
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, nullptr);
  if (P < 0) return P;
  {
    const int32_t rc = check_chain_args(y, y_bstride, t, t_drawstride, t_rowstride, S, B, d, P, y_mean, y_std, out_sum,
                                        workspace, posterior);
    if (rc != NFN_OK) return rc;
  }
  int64_t base = 0;
  for (int64_t b0 = 0; b0 < B; b0 += chunk) {
    const int64_t nb = std::min(chunk, B - b0);
    const bool last = b0 + nb >= B;
    int64_t used = 0;
    const int32_t rc = run_chain_launch(y + b0 * y_bstride, y_bstride, t ? t + b0 * t_rowstride : nullptr, t_drawstride,
                                        t_rowstride, S, nb, d, flow_ids, K, trainable_base, y_mean, y_std,
                                        out ? out + b0 : nullptr, last ? out_sum : nullptr, workspace, stream, false,
                                        base, raw_partials(nb, P), &used);
    if (rc != NFN_OK) return rc;
    base += used;
  }
  return NFN_OK;
}

int32_t run_grad(const float* y, int64_t y_bstride, const float* t, int64_t t_rowstride, int64_t B, int32_t d,
                 const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                 const float* y_std, const float* g_out, float* out_logp, float* grad_t, int64_t gt_rowstride,
                 float* grad_y, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  GradArgs ga;
  memset(&ga, 0, sizeof(ga));
  ChainArgs& a = ga.c;
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
  if (P < 0) return P;
  if (B < 0) return fail(NFN_E_SHAPE, "batch size must be >= 0");
  if (y_bstride < 0 || t_rowstride < 0) return fail(NFN_E_SHAPE, "strides must be >= 0");
  if (y_bstride != 0 && y_bstride < d) return fail(NFN_E_SHAPE, "y batch stride < n_dims");
  if (t_rowstride != 0 && t_rowstride < P) return fail(NFN_E_SHAPE, "t row stride < total param size");
  if (grad_t && gt_rowstride < P) return fail(NFN_E_SHAPE, "grad_t row stride < total param size");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  if (B == 0 || (!out_logp && !grad_t && !grad_y)) return NFN_OK;
  if (!y) return fail(NFN_E_NULLPTR, "y is NULL");
  if (P > 0 && !t) return fail(NFN_E_NULLPTR, "t is NULL");
  // Tile geometry: R samples per one-wave workgroup, each with a parameter row
  // (odd stride) and its K*d flow inputs in LDS.
  const int S = P | 1;
  const size_t row_bytes = (size_t)(S + K * d) * sizeof(float);
  int R = 64;
  while (R > 1 && (size_t)R * row_bytes > (size_t)64 * 1024) R >>= 1;
  if ((size_t)R * row_bytes > (size_t)160 * 1024) return fail(NFN_E_SHAPE, "parameter row + flow inputs exceed LDS");
  const int64_t nblk = (B + R - 1) / R;
  if (nblk > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  a.y = y;
  a.t = t;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.out = out_logp;
  a.y_bstride = y_bstride;
  a.t_rowstride = t_rowstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = S;
  a.trainable = trainable_base ? 1 : 0;
  a.S = 1;
  a.vec4 = ((P & 3) == 0) && ((t_rowstride & 3) == 0) && ((reinterpret_cast<uintptr_t>(t) & 15) == 0);
  ga.g_out = g_out;
  ga.grad_t = grad_t;
  ga.grad_y = grad_y;
  ga.gt_rowstride = grad_t ? gt_rowstride : 0;
  ga.gt_vec4 = ((P & 3) == 0) && ((gt_rowstride & 3) == 0) && ((reinterpret_cast<uintptr_t>(grad_t) & 15) == 0);
  ga.rows = R;
  // the backward's release policy: hand-off priority, z-only forward recompute when no
  // log_prob is wanted; the diagnostic build's overrides (memory-only / compute-only timing)
  a.prio = 1;
  a.zonly = 1;
#ifdef NFN_DIAG
  if (env_int("NFN_ABLATE_FLOWS", 0) == 1) a.prog.K = 0;
  a.prio = env_int("NFN_PRIO", 1) == 1 ? 1 : 0;
  a.ablate_loads = env_int("NFN_ABLATE_LOADS", 0) == 1 ? 1 : 0;
  a.zonly = env_int("NFN_GRAD_ZONLY", 1) != 0 ? 1 : 0;
  a.tile_rot_b = std::max(0, env_int("NFN_TILE_ROT_B", 0));  // chain_grad_wave_kernel's rotated slots (A/B)
#endif
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int Q = P >> 2;
  const int dm = dm_for(d);
  const size_t slot = (size_t)(64 * S + a.prog.K * d * 64) * sizeof(float);
  const bool wave_ok = a.vec4 && t_rowstride != 0 && P > 0 && (Q & (Q - 1)) == 0 && Q <= 16 && dm <= 2 &&
                       (!grad_t || ga.gt_vec4) && slot <= (size_t)40 * 1024 && env_int("NFN_GRAD_WAVE", 1) != 0;
  if (dm >= 4 && a.vec4 && t_rowstride != 0 && Q >= 1 && (!grad_t || ga.gt_vec4) &&
      env_int("NFN_GRAD_GROUP", 1) != 0) {
    int G = 4, DPL = 1;
    group_shape(dm, env_int("NFN_GROUP_LANES", 0), &G, &DPL);
    const int Rg = 64 / G;
    const int nv = (Q + G - 1) / G;  // float4 slots per lane: (R rows x Q) / 64
    a.lds_stride = group_lds_stride(P, G);
    const size_t gslot = (size_t)(Rg * a.lds_stride + a.prog.K * DPL * 64) * sizeof(float);
    if (nv <= 16 && gslot <= (size_t)40 * 1024) {
      a.ntiles = (B + Rg - 1) / Rg;
      int64_t grid = 0;
      const bool ok = use_fast_math() ? launch_grad_group_fast(G, DPL, nv, ga, 4 * gslot, s, &grid)
                                      : launch_grad_group_precise(G, DPL, nv, ga, 4 * gslot, s, &grid);
      if (ok) return check_hip("chain_grad_group_kernel launch");
    }
    a.lds_stride = S;
  }
  if (wave_ok) {
    a.ntiles = (B + 63) / 64;
    // two waves per workgroup measured fastest on C2 (finer LDS allocation granules
    // than 4-wave groups at ~11 KB of LDS per wave); NFN_GRAD_WPB overrides (1, 2, 4)
    int wpb = slot * 2 <= (size_t)80 * 1024 ? 2 : 1;
    const int want_wpb = env_int("NFN_GRAD_WPB", 0);
    if (want_wpb == 1 || want_wpb == 2 || want_wpb == 4)
      wpb = slot * want_wpb <= (size_t)80 * 1024 ? want_wpb : 1;
    int64_t grid = 0;
    if (launch_grad_wave(use_fast_math(), dm, Q, ga, slot * wpb, wpb, s, &grid))
      return check_hip("chain_grad_wave_kernel launch");
  }
  launch_grad(use_fast_math(), dm, ga, dim3((unsigned)nblk), (size_t)R * row_bytes, s);
  return check_hip("chain_grad_kernel launch");
}

int32_t run_dense(const float* y, int64_t y_bstride, const float* h, int64_t h_rowstride, int32_t H, const float* W,
                  const float* bias, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                  const float* y_mean, const float* y_std, float* out, double* out_sum, double* workspace,
                  void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  DenseArgs da;
  memset(&da, 0, sizeof(da));
  ChainArgs& a = da.c;
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
#ifdef NFN_DIAG
  if (env_int("NFN_ABLATE_FLOWS", 0) == 1) a.prog.K = 0;  // the Dense GEMM + streaming alone
  a.ablate_loads = env_int("NFN_ABLATE_LOADS", 0) == 1 ? 1 : 0;  // compute-only (first tile re-read)
#endif
  if (P < 0) return P;
  if (B < 0) return fail(NFN_E_SHAPE, "batch size must be >= 0");
  if (y_bstride < 0 || (y_bstride != 0 && y_bstride < d)) return fail(NFN_E_SHAPE, "bad y batch stride");
  // the fused kernel's shapes: H a power of two in [4, 64] (16-byte h pieces, 4-wide
  // MFMA k-steps), P <= 64 (per-wave t tile), d <= 8
  if (H < 4 || H > 64 || (H & (H - 1)) != 0) return fail(NFN_E_SHAPE, "hidden width H must be 4, 8, 16, 32 or 64");
  if (P < 1 || P > 64) return fail(NFN_E_SHAPE, "fused dense path needs 1 <= P <= 64");
  if (d > 8) return fail(NFN_E_SHAPE, "fused dense path needs n_dims <= 8");
  if (h_rowstride < H || (h_rowstride & 3) != 0) return fail(NFN_E_SHAPE, "h row stride must be >= H and a multiple of 4");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (B == 0) {
    if (out_sum && hipMemsetAsync(out_sum, 0, 2 * sizeof(double), s) != hipSuccess) return check_hip("hipMemsetAsync");
    return NFN_OK;
  }
  if (!y || !h || !W) return fail(NFN_E_NULLPTR, "y, h or W is NULL");
  if ((reinterpret_cast<uintptr_t>(h) & 15) != 0) return fail(NFN_E_SHAPE, "h must be 16-byte aligned");
  if (out_sum && !workspace) return fail(NFN_E_NULLPTR, "workspace is NULL but out_sum requested");
  if (!out && !workspace) return NFN_OK;
  a.y = y;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.out = out;
  a.partials = workspace ? workspace + 2 : nullptr;
  a.out_sum = workspace ? out_sum : nullptr;
  a.epoch = a.out_sum ? next_epoch() : 0u;
  a.y_bstride = y_bstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = P | 1;
  a.trainable = trainable_base ? 1 : 0;
  a.S = 1;
  a.ntiles = (B + 63) / 64;
  da.h = h;
  da.h_rowstride = h_rowstride;
  da.W = W;
  da.bias = bias;
  da.H = H;
  da.h_lds_stride = H | 1;
  const int NP = ((P + 15) / 16) * 16;
  // generic kernel: per wave the h tile + a row-major 64 x S t tile (chain_dense1_kernel
  // sizes its own, smaller, overlaid region)
  const size_t lds = (size_t)(H * NP + 4 * (64 * da.h_lds_stride + 64 * a.lds_stride) + 16) * sizeof(float);
  int64_t grid = 0;
  if (!launch_dense(use_fast_math(), dm_for(d), H / 4, da, lds, s, &grid))
    return fail(NFN_E_SHAPE, "no fused dense instance for this shape");
  return check_hip("chain_dense_kernel launch");
}

int32_t run_posterior_dense(const float* y, int64_t y_bstride, const float* h, int64_t h_drawstride,
                            int64_t h_rowstride, int32_t H, const float* W, int64_t w_drawstride, const float* bias,
                            int64_t b_drawstride, int32_t S, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K,
                            int32_t trainable_base, const float* y_mean, const float* y_std, float* out,
                            double* out_sum, double* workspace, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  DenseArgs da;
  memset(&da, 0, sizeof(da));
  ChainArgs& a = da.c;
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
#ifdef NFN_DIAG
  if (env_int("NFN_ABLATE_FLOWS", 0) == 1) a.prog.K = 0;  // the Dense GEMMs + streaming alone
  a.ablate_loads = env_int("NFN_ABLATE_LOADS", 0) == 1 ? 1 : 0;  // compute-only (first tile re-read)
#endif
  if (P < 0) return P;
  if (B < 0) return fail(NFN_E_SHAPE, "batch size must be >= 0");
  if (S < 1) return fail(NFN_E_SHAPE, "number of draws must be >= 1");
  if (y_bstride < 0 || (y_bstride != 0 && y_bstride < d)) return fail(NFN_E_SHAPE, "bad y batch stride");
  if (H < 4 || H > 64 || (H & (H - 1)) != 0) return fail(NFN_E_SHAPE, "hidden width H must be 4, 8, 16, 32 or 64");
  if (P < 1 || P > 64) return fail(NFN_E_SHAPE, "fused dense path needs 1 <= P <= 64");
  if (d > 8) return fail(NFN_E_SHAPE, "fused dense path needs n_dims <= 8");
  if (h_rowstride < H || (h_rowstride & 3) != 0) return fail(NFN_E_SHAPE, "h row stride must be >= H and a multiple of 4");
  if (h_drawstride < 0 || (h_drawstride & 3) != 0 || (h_drawstride != 0 && h_drawstride < B * h_rowstride))
    return fail(NFN_E_SHAPE, "h draw stride must be 0 (shared h) or >= B * h_rowstride, a multiple of 4");
  if (w_drawstride < 0 || (S > 1 && w_drawstride < (int64_t)H * P)) return fail(NFN_E_SHAPE, "W draw stride < H * P");
  if (bias && (b_drawstride < 0 || (S > 1 && b_drawstride < P))) return fail(NFN_E_SHAPE, "bias draw stride < P");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (B == 0) {
    if (out_sum && hipMemsetAsync(out_sum, 0, 2 * sizeof(double), s) != hipSuccess) return check_hip("hipMemsetAsync");
    return NFN_OK;
  }
  if (!y || !h || !W) return fail(NFN_E_NULLPTR, "y, h or W is NULL");
  if ((reinterpret_cast<uintptr_t>(h) & 15) != 0) return fail(NFN_E_SHAPE, "h must be 16-byte aligned");
  if (out_sum && !workspace) return fail(NFN_E_NULLPTR, "workspace is NULL but out_sum requested");
  if (!out && !workspace) return NFN_OK;
  a.y = y;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.out = out;
  a.partials = workspace ? workspace + 2 : nullptr;
  a.out_sum = workspace ? out_sum : nullptr;
  a.epoch = a.out_sum ? next_epoch() : 0u;
  a.y_bstride = y_bstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = P | 1;
  a.trainable = trainable_base ? 1 : 0;
  a.S = S;
  a.ntiles = (B + 63) / 64;
  da.h = h;
  da.h_rowstride = h_rowstride;
  da.h_drawstride = h_drawstride;
  da.W = W;
  da.w_drawstride = w_drawstride;
  da.bias = bias;
  da.b_drawstride = b_drawstride;
  da.H = H;
  da.h_lds_stride = H | 1;
  int64_t grid = 0;
  if (!launch_posterior_dense(use_fast_math(), dm_for(d), da, s, &grid))
    return fail(NFN_E_SHAPE, "no fused dense posterior instance for this shape");
  return check_hip("posterior_dense_kernel launch");
}

constexpr int64_t kDenseGradMaxParts = 2048;  // per-workgroup partials (>= CUs x resident workgroups)

int64_t dense_grad_parts(int64_t B) { return std::max<int64_t>(1, std::min<int64_t>(kDenseGradMaxParts, ((B + 63) / 64 + 3) / 4)); }

int32_t run_dense_grad(const float* y, int64_t y_bstride, const float* h, int64_t h_rowstride, int32_t H,
                       const float* W, const float* bias, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K,
                       int32_t trainable_base, const float* y_mean, const float* y_std, const float* g_out,
                       float* out_logp, float* grad_h, int64_t grad_h_rowstride, float* grad_W, float* grad_b,
                       float* grad_y, float* workspace, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  DenseGradArgs g;
  memset(&g, 0, sizeof(g));
  DenseArgs& da = g.da;
  ChainArgs& a = da.c;
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
#ifdef NFN_DIAG
  if (env_int("NFN_ABLATE_FLOWS", 0) == 1) a.prog.K = 0;  // the Dense GEMMs + streaming alone
  a.ablate_loads = env_int("NFN_ABLATE_LOADS", 0) == 1 ? 1 : 0;  // compute-only (first tile re-read)
#endif
  if (P < 0) return P;
  if (B < 0) return fail(NFN_E_SHAPE, "batch size must be >= 0");
  if (y_bstride < 0 || (y_bstride != 0 && y_bstride < d)) return fail(NFN_E_SHAPE, "bad y batch stride");
  if (H < 4 || H > 64 || (H & (H - 1)) != 0) return fail(NFN_E_SHAPE, "hidden width H must be 4, 8, 16, 32 or 64");
  if (P < 1 || P > 64) return fail(NFN_E_SHAPE, "fused dense path needs 1 <= P <= 64");
  if (d > 8) return fail(NFN_E_SHAPE, "fused dense path needs n_dims <= 8");
  if (h_rowstride < H || (h_rowstride & 3) != 0) return fail(NFN_E_SHAPE, "h row stride must be >= H and a multiple of 4");
  if (grad_h && grad_h_rowstride < H) return fail(NFN_E_SHAPE, "grad_h row stride < H");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nWb = H * P + P;
  if (B == 0) {
    if (grad_W && hipMemsetAsync(grad_W, 0, sizeof(float) * H * P, s) != hipSuccess) return check_hip("hipMemsetAsync");
    if (grad_b && hipMemsetAsync(grad_b, 0, sizeof(float) * P, s) != hipSuccess) return check_hip("hipMemsetAsync");
    return NFN_OK;
  }
  if (!y || !h || !W) return fail(NFN_E_NULLPTR, "y, h or W is NULL");
  if ((reinterpret_cast<uintptr_t>(h) & 15) != 0) return fail(NFN_E_SHAPE, "h must be 16-byte aligned");
  if ((grad_W || grad_b) && !workspace) return fail(NFN_E_NULLPTR, "workspace is NULL but grad_W / grad_b requested");
  const int S = P | 1;
  const int NP = ((P + 15) / 16) * 16;
  const size_t lds = (size_t)(H * NP + 4 * (64 * (H | 1) + 64 * S + K * d * 64) + nWb) * sizeof(float);
  if (lds > (size_t)160 * 1024) return fail(NFN_E_SHAPE, "fused dense backward: tile + flow inputs exceed LDS");
  a.y = y;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.out = out_logp;
  a.y_bstride = y_bstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = S;
  a.trainable = trainable_base ? 1 : 0;
  a.S = 1;
  a.ntiles = (B + 63) / 64;
  da.h = h;
  da.h_rowstride = h_rowstride;
  da.W = W;
  da.bias = bias;
  da.H = H;
  da.h_lds_stride = H | 1;
  g.g_out = g_out;
  g.grad_h = grad_h;
  g.gh_rowstride = grad_h ? grad_h_rowstride : 0;
  g.grad_y = grad_y;
  g.part = (grad_W || grad_b) ? workspace : nullptr;  // no partials without grad_W / grad_b
  const int64_t nparts = launch_dense_grad(use_fast_math(), dm_for(d), g, lds, dense_grad_parts(B), s);
  if (nparts == 0) return fail(NFN_E_SHAPE, "no fused dense backward instance for this shape");
  int32_t rc = check_hip("chain_dense_grad_kernel launch");
  if (rc == NFN_OK && (grad_W || grad_b)) {
    launch_sum_partials(g.part, nparts, nWb, grad_W, grad_b, H * P, s);
    rc = check_hip("sum_partials_kernel launch");
  }
  return rc;
}

int32_t run_sample(const float* eps, int64_t eps_bstride, const float* t, int64_t t_rowstride, int64_t B, int32_t d,
                   const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                   const float* y_std, float* y_out, float* logp_out, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  SampleArgs sa;
  memset(&sa, 0, sizeof(sa));
  ChainArgs& a = sa.c;
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
  if (P < 0) return P;
  if (B < 0) return fail(NFN_E_SHAPE, "batch size must be >= 0");
  if (eps_bstride < 0 || (eps_bstride != 0 && eps_bstride < d)) return fail(NFN_E_SHAPE, "bad eps batch stride");
  if (t_rowstride < 0 || (t_rowstride != 0 && t_rowstride < P)) return fail(NFN_E_SHAPE, "bad t row stride");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  if (B == 0) return NFN_OK;
  if (!eps || !y_out) return fail(NFN_E_NULLPTR, "eps or y_out is NULL");
  if (P > 0 && !t) return fail(NFN_E_NULLPTR, "t is NULL");
  const TileGeom g = tile_geom(P);
  if ((size_t)g.rows * ((size_t)g.lds_stride * sizeof(float)) > (size_t)kLdsMaxBytes)
    return fail(NFN_E_SHAPE, "parameter row too wide for LDS");
  a.t = t;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.t_rowstride = t_rowstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = g.lds_stride;
  a.trainable = trainable_base ? 1 : 0;
  a.S = 1;
  a.vec4 = ((P & 3) == 0) && ((t_rowstride & 3) == 0) && ((reinterpret_cast<uintptr_t>(t) & 15) == 0);
  a.tile_rows = g.rows;
  sa.eps = eps;
  sa.eps_bstride = eps_bstride;
  sa.y_out = y_out;
  sa.logp = logp_out;
  const int64_t nblk = (B + g.rows - 1) / g.rows;
  if (nblk > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  launch_sample(use_fast_math(), dm_for(d), sa, dim3((unsigned)nblk), dim3((unsigned)g.threads), g.lds_bytes,
                reinterpret_cast<hipStream_t>(stream));
  return check_hip("chain_sample_kernel launch");
}

int32_t run_grid(const float* y_grid, int64_t y_gstride, int32_t G, const float* t, int64_t t_rowstride, int64_t B,
                 int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                 const float* y_std, float* out, int64_t out_gstride, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  GridArgs ga;
  memset(&ga, 0, sizeof(ga));
  ChainArgs& a = ga.c;
  const int32_t P = build_program(flow_ids, K, d, trainable_base ? 1 : 0, &a.prog);
  if (P < 0) return P;
  if (B < 0 || G < 0) return fail(NFN_E_SHAPE, "batch and grid sizes must be >= 0");
  if (y_gstride < 0 || t_rowstride < 0) return fail(NFN_E_SHAPE, "strides must be >= 0");
  if (y_gstride != 0 && y_gstride < d) return fail(NFN_E_SHAPE, "y_grid stride < n_dims");
  if (t_rowstride != 0 && t_rowstride < P) return fail(NFN_E_SHAPE, "t row stride < total param size");
  if (out_gstride < B) return fail(NFN_E_SHAPE, "out grid stride < batch size");
  if ((y_mean == nullptr) != (y_std == nullptr)) return fail(NFN_E_NULLPTR, "y_mean and y_std must both be given or both NULL");
  if (B == 0 || G == 0) return NFN_OK;
  if (!y_grid || !out) return fail(NFN_E_NULLPTR, "y_grid or out is NULL");
  if (P > 0 && !t) return fail(NFN_E_NULLPTR, "t is NULL");
  const TileGeom g = tile_geom(P);
  if ((size_t)g.rows * ((size_t)g.lds_stride * sizeof(float)) > (size_t)kLdsMaxBytes)
    return fail(NFN_E_SHAPE, "parameter row too wide for LDS");
  a.t = t;
  a.y_mean = y_mean;
  a.y_std = y_std;
  a.t_rowstride = t_rowstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = g.lds_stride;
  a.trainable = trainable_base ? 1 : 0;
  a.S = 1;
  a.vec4 = ((P & 3) == 0) && ((t_rowstride & 3) == 0) && ((reinterpret_cast<uintptr_t>(t) & 15) == 0);
  a.tile_rows = g.rows;
  ga.y_grid = y_grid;
  ga.y_gstride = y_gstride;
  ga.out = out;
  ga.out_gstride = out_gstride;
  ga.G = G;
  const int64_t ntiles = (B + g.rows - 1) / g.rows;
  if (ntiles > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  // enough (tile, grid-chunk) workgroups to fill the chip: ~4 per CU
  const int64_t want = std::max<int64_t>(1, ((int64_t)cu_count() * 4 + ntiles - 1) / ntiles);
  int64_t nchunks = std::min<int64_t>({(int64_t)G, want, 65535});
  ga.gchunk = (int32_t)((G + nchunks - 1) / nchunks);
  nchunks = (G + ga.gchunk - 1) / ga.gchunk;
  launch_grid(use_fast_math(), dm_for(d), ga, dim3((unsigned)ntiles, (unsigned)nchunks), dim3((unsigned)g.threads),
              g.lds_bytes, reinterpret_cast<hipStream_t>(stream));
  return check_hip("chain_grid_kernel launch");
}

}  // namespace
}  // namespace nfn

using namespace nfn;

extern "C" {

int32_t nfn_version(void) { return NFN_VERSION_NUM; }

const char* nfn_last_error(void) { return g_last_error.c_str(); }

int32_t nfn_reduce_sum_f64(const double* in, int64_t n, double* out, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  if (n < 0) return fail(NFN_E_SHAPE, "n must be >= 0");
  if (!out || (n > 0 && !in)) return fail(NFN_E_NULLPTR, "in or out is NULL");
  launch_reduce_f64(in, n, out, reinterpret_cast<hipStream_t>(stream));
  return check_hip("reduce_f64_kernel launch");
}


int32_t nfn_set_launch_events(void* start_event, void* stop_event) {
  g_launch_events.start = reinterpret_cast<hipEvent_t>(start_event);
  g_launch_events.stop = reinterpret_cast<hipEvent_t>(stop_event);
  return NFN_OK;
}

int32_t nfn_set_math_mode(int32_t mode) {
  if (mode != 0 && mode != 1) return fail(NFN_E_SHAPE, "math mode must be 0 (fast) or 1 (precise)");
  const int32_t prev = g_math_mode;
  g_math_mode = mode;
  return prev;
}

int32_t nfn_param_size(int32_t flow_id, int32_t d) {
  if (d < 1 || d > NFN_MAX_DIMS) return fail(NFN_E_SHAPE, "n_dims out of range");
  const int32_t ps = param_size(flow_id, d);
  return ps < 0 ? fail(NFN_E_FLOW_ID, "unknown flow id " + std::to_string(flow_id)) : ps;
}

int32_t nfn_total_param_size(const int32_t* flow_ids, int32_t K, int32_t d, int32_t trainable_base) {
  return build_program(flow_ids, K, d, trainable_base ? 1 : 0, nullptr);
}

int64_t nfn_chain_workspace_doubles(int64_t B, int32_t d, int32_t P) {
  (void)d;
  (void)P;
  if (B <= 0) return 0;
  return partials_doubles(B, P);  // [count | ticket | (sum, count) pairs]
}

int64_t nfn_posterior_workspace_doubles(int64_t B, int32_t d, int32_t P) {
  if (B <= 0) return 0;
  // [count | ticket | pairs | draw-split region: (max, sum) float2 per (range, sample)]
  return partials_doubles(B, P) + (int64_t)posterior_split(B) * B;
}

int32_t nfn_reduce_partials_f64(const double* workspace, double* out_sum, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  if (!workspace || !out_sum) return fail(NFN_E_NULLPTR, "workspace or out_sum is NULL");
  launch_reduce_partials(workspace, out_sum, reinterpret_cast<hipStream_t>(stream));
  return check_hip("reduce_partials_kernel launch");
}

int32_t nfn_chain_logprob_f32(const float* y, int64_t y_bstride, const float* t, int64_t t_rowstride, int64_t B,
                              int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                              const float* y_mean, const float* y_std, float* out_logp, double* out_sum,
                              double* workspace, void* stream) {
  return run_chain(y, y_bstride, t, 0, t_rowstride, 1, B, d, flow_ids, K, trainable_base, y_mean, y_std, out_logp,
                   out_sum, workspace, stream, false);
}

int32_t nfn_posterior_lse_f32(const float* y, int64_t y_bstride, const float* t, int64_t t_drawstride,
                              int64_t t_rowstride, int32_t S, int64_t B, int32_t d, const int32_t* flow_ids,
                              int32_t K, int32_t trainable_base, const float* y_mean, const float* y_std,
                              float* out_lse, double* out_sum, double* workspace, void* stream) {
  return run_chain(y, y_bstride, t, t_drawstride, t_rowstride, S, B, d, flow_ids, K, trainable_base, y_mean, y_std,
                   out_lse, out_sum, workspace, stream, true);
}

int32_t nfn_chain_logprob_grad_f32(const float* y, int64_t y_bstride, const float* t, int64_t t_rowstride,
                                   int64_t B, int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                                   const float* y_mean, const float* y_std, const float* g_out, float* out_logp,
                                   float* grad_t, int64_t grad_t_rowstride, float* grad_y, void* stream) {
  return run_grad(y, y_bstride, t, t_rowstride, B, d, flow_ids, K, trainable_base, y_mean, y_std, g_out, out_logp,
                  grad_t, grad_t_rowstride, grad_y, stream);
}

int32_t nfn_chain_logprob_dense_f32(const float* y, int64_t y_bstride, const float* h, int64_t h_rowstride,
                                    int32_t H, const float* W, const float* bias, int64_t B, int32_t d,
                                    const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                                    const float* y_std, float* out_logp, double* out_sum, double* workspace,
                                    void* stream) {
  return run_dense(y, y_bstride, h, h_rowstride, H, W, bias, B, d, flow_ids, K, trainable_base, y_mean, y_std,
                   out_logp, out_sum, workspace, stream);
}

int64_t nfn_dense_grad_workspace_floats(int64_t B, int32_t H, int32_t P) {
  return (int64_t)(H * P + P) * dense_grad_parts(B < 0 ? 0 : B);
}

int32_t nfn_chain_logprob_dense_grad_f32(const float* y, int64_t y_bstride, const float* h, int64_t h_rowstride,
                                         int32_t H, const float* W, const float* bias, int64_t B, int32_t d,
                                         const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                                         const float* y_mean, const float* y_std, const float* g_out,
                                         float* out_logp, float* grad_h, int64_t grad_h_rowstride, float* grad_W,
                                         float* grad_b, float* grad_y, float* workspace, void* stream) {
  return run_dense_grad(y, y_bstride, h, h_rowstride, H, W, bias, B, d, flow_ids, K, trainable_base, y_mean, y_std,
                        g_out, out_logp, grad_h, grad_h_rowstride, grad_W, grad_b, grad_y, workspace, stream);
}

int32_t nfn_posterior_lse_dense_f32(const float* y, int64_t y_bstride, const float* h, int64_t h_drawstride,
                                    int64_t h_rowstride, int32_t H, const float* W, int64_t w_drawstride,
                                    const float* bias, int64_t bias_drawstride, int32_t S, int64_t B, int32_t d,
                                    const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                                    const float* y_std, float* out_lse, double* out_sum, double* workspace,
                                    void* stream) {
  return run_posterior_dense(y, y_bstride, h, h_drawstride, h_rowstride, H, W, w_drawstride, bias, bias_drawstride, S,
                             B, d, flow_ids, K, trainable_base, y_mean, y_std, out_lse, out_sum, workspace, stream);
}

int32_t nfn_chain_sample_f32(const float* eps, int64_t eps_bstride, const float* t, int64_t t_rowstride, int64_t B,
                             int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                             const float* y_mean, const float* y_std, float* y_out, float* logp_out, void* stream) {
  return run_sample(eps, eps_bstride, t, t_rowstride, B, d, flow_ids, K, trainable_base, y_mean, y_std, y_out,
                    logp_out, stream);
}

int32_t nfn_chain_logprob_grid_f32(const float* y_grid, int64_t y_gstride, int32_t G, const float* t,
                                   int64_t t_rowstride, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K,
                                   int32_t trainable_base, const float* y_mean, const float* y_std, float* out,
                                   int64_t out_gstride, void* stream) {
  return run_grid(y_grid, y_gstride, G, t, t_rowstride, B, d, flow_ids, K, trainable_base, y_mean, y_std, out,
                  out_gstride, stream);
}

int32_t nfn_flow_fwd_ldj_f32(int32_t flow_id, const float* z, int64_t z_bstride, const float* t_k,
                             int64_t t_rowstride, int64_t B, int32_t d, float* z_out, float* ldj_out, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  if (d < 1 || d > NFN_MAX_DIMS) return fail(NFN_E_SHAPE, "n_dims out of range");
  const int32_t ps = param_size(flow_id, d);
  if (ps < 0) return fail(NFN_E_FLOW_ID, "unknown flow id " + std::to_string(flow_id));
  if (B < 0 || z_bstride < 0 || t_rowstride < 0) return fail(NFN_E_SHAPE, "negative batch or stride");
  if (z_bstride != 0 && z_bstride < d) return fail(NFN_E_SHAPE, "z batch stride < n_dims");
  if (t_rowstride != 0 && t_rowstride < ps) return fail(NFN_E_SHAPE, "t row stride < flow param size");
  if (B == 0 || (!z_out && !ldj_out)) return NFN_OK;
  if (!z || !t_k) return fail(NFN_E_NULLPTR, "z or t_k is NULL");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  if (nblk > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  launch_flow(use_fast_math(), dm_for(d), flow_id, z, z_bstride, t_k, t_rowstride, B, d, z_out, ldj_out, s);
  return check_hip("flow_fwd_ldj_kernel launch");
}

int32_t nfn_flow_vjp_f32(int32_t flow_id, const float* z, int64_t z_bstride, const float* t_k, int64_t t_rowstride,
                         int64_t B, int32_t d, const float* g_z, const float* g_ldj, float* dz_out, float* dt_out,
                         void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  if (d < 1 || d > NFN_MAX_DIMS) return fail(NFN_E_SHAPE, "n_dims out of range");
  const int32_t ps = param_size(flow_id, d);
  if (ps < 0) return fail(NFN_E_FLOW_ID, "unknown flow id " + std::to_string(flow_id));
  if (B < 0 || z_bstride < 0 || t_rowstride < 0) return fail(NFN_E_SHAPE, "negative batch or stride");
  if (z_bstride != 0 && z_bstride < d) return fail(NFN_E_SHAPE, "z batch stride < n_dims");
  if (t_rowstride != 0 && t_rowstride < ps) return fail(NFN_E_SHAPE, "t row stride < flow param size");
  if (B == 0 || (!dz_out && !dt_out)) return NFN_OK;
  if (!z || !t_k) return fail(NFN_E_NULLPTR, "z or t_k is NULL");
  const int64_t nblk = (B + kMaxBlock - 1) / kMaxBlock;
  if (nblk > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  FlowVjpArgs v;
  memset(&v, 0, sizeof(v));
  v.z = z;
  v.z_bstride = z_bstride;
  v.t = t_k;
  v.t_rowstride = t_rowstride;
  v.B = B;
  v.g_z = g_z;
  v.g_ldj = g_ldj;
  v.dz = dz_out;
  v.dt = dt_out;
  v.flow_id = flow_id;
  v.d = d;
  v.ps = ps;
  launch_flow_vjp(use_fast_math(), dm_for(d), v, reinterpret_cast<hipStream_t>(stream));
  return check_hip("flow_vjp_kernel launch");
}

int32_t nfn_split_blocks_f32(const float* t, int64_t t_rowstride, int64_t B, const int32_t* widths, int32_t nblocks,
                             float* dst, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  if (nblocks < 1 || nblocks > NFN_MAX_FLOWS) return fail(NFN_E_SHAPE, "nblocks must be in [1, " + std::to_string(NFN_MAX_FLOWS) + "]");
  if (!widths) return fail(NFN_E_NULLPTR, "widths is NULL");
  if (B < 0 || t_rowstride < 0) return fail(NFN_E_SHAPE, "negative batch or stride");
  SplitArgs sa;
  memset(&sa, 0, sizeof(sa));
  int64_t W = 0;
  for (int32_t k = 0; k < nblocks; ++k) {
    if (widths[k] < 1) return fail(NFN_E_SHAPE, "block widths must be >= 1");
    sa.widths[k] = widths[k];
    W += widths[k];
  }
  if (W > 1024) return fail(NFN_E_SHAPE, "blocks wider than 1024 floats in total");
  if (B > 1 && t_rowstride < W) return fail(NFN_E_SHAPE, "t row stride < the blocks' total width");
  if (B == 0) return NFN_OK;
  if (!t || !dst) return fail(NFN_E_NULLPTR, "t or dst is NULL");
  if (B > (int64_t)0x7fffffff) return fail(NFN_E_SHAPE, "batch too large");
  sa.t = t;
  sa.rs = t_rowstride;
  sa.B = B;
  sa.dst = dst;
  sa.W = (int32_t)W;
  sa.nblocks = nblocks;
  launch_split_blocks(sa, reinterpret_cast<hipStream_t>(stream));
  return check_hip("split_blocks_kernel launch");
}

int32_t nfn_chain_fwd_ldj_f32(const float* z, int64_t z_bstride, const float* t, int64_t t_rowstride, int64_t B,
                              int32_t d, const int32_t* flow_ids, const int32_t* block_offsets, int32_t K,
                              float* z_out, float* ldj_out, void* stream) {
  g_last_error.clear();
  const HookScope hook_scope;
  if (d < 1 || d > NFN_MAX_DIMS) return fail(NFN_E_SHAPE, "n_dims out of range");
  if (K < 0 || K > NFN_MAX_FLOWS) return fail(NFN_E_FLOW_ID, "number of flows must be in [0, " + std::to_string(NFN_MAX_FLOWS) + "]");
  if (K > 0 && (!flow_ids || !block_offsets)) return fail(NFN_E_NULLPTR, "flow_ids or block_offsets is NULL");
  if (B < 0 || z_bstride < 0 || t_rowstride < 0) return fail(NFN_E_SHAPE, "negative batch or stride");
  if (z_bstride != 0 && z_bstride < d) return fail(NFN_E_SHAPE, "z batch stride < n_dims");
  ChainArgs a;
  memset(&a, 0, sizeof(a));
  int32_t lo = 0, hi = 0;  // the parameter span [lo, hi) of the row that the flows read
  for (int32_t k = 0; k < K; ++k) {
    const int32_t ps = param_size(flow_ids[k], d);
    if (ps < 0) return fail(NFN_E_FLOW_ID, "unknown flow id " + std::to_string(flow_ids[k]));
    if (block_offsets[k] < 0) return fail(NFN_E_SHAPE, "negative block offset");
    lo = k == 0 ? block_offsets[k] : std::min(lo, block_offsets[k]);
    hi = std::max(hi, block_offsets[k] + ps);
  }
  if (t_rowstride != 0 && t_rowstride < hi) return fail(NFN_E_SHAPE, "t row stride < the flows' parameter span");
  if (B == 0 || (!z_out && !ldj_out)) return NFN_OK;
  if (!z || (K > 0 && !t)) return fail(NFN_E_NULLPTR, "z or t is NULL");
  a.prog.K = K;
  for (int32_t k = 0; k < K; ++k) {
    a.prog.step[k] = ((block_offsets[k] - lo) << 2) | flow_ids[k];
    a.prog.types[k >> 4] |= (uint32_t)flow_ids[k] << (2 * (k & 15));
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // d = 1, fast math, the layer's contiguous reversed blocks (flow k ends where flow k-1's
  // begins, f_0 last): the packed program derives every offset from the row width, so
  // the kernel streams the 16-byte-aligned rows [lo & ~3, hi) on the wave1 pipeline
  {
    bool layer_layout = K >= 1;
    int32_t end = hi;
    for (int32_t k = 0; layer_layout && k < K; ++k) {
      end -= param_size(flow_ids[k], d);
      layer_layout = block_offsets[k] == end;
    }
    layer_layout = layer_layout && end == lo;
    // d >= 4, fast math, the layer's contiguous rows (the span ends the row and t points at
    // the row start): the lane-group pipeline of the C3 forward (chain_group1_kernel<FWD>)
    if (layer_layout && d >= 4 && use_fast_math() && t_rowstride == hi && (hi & 3) == 0 &&
        (reinterpret_cast<uintptr_t>(t) & 15) == 0 && z_bstride * 256 < ((int64_t)1 << 31) &&
        env_int("NFN_GROUP1", 1) != 0) {
      const int dm = dm_for(d);
      const int Qh = hi >> 2;
      int G = 4, DPL = 1;
      group_shape(dm, dm == 8 && (Qh + 1) / 2 <= 18 ? 2 : 0, &G, &DPL);
      const int R = 64 / G;
      const int nv = (Qh + G - 1) / G;
      if (G * DPL >= d && nv <= (G == 2 ? 18 : 16) && (int64_t)R * hi * 4 < ((int64_t)1 << 31)) {
        a.y = z;
        a.y_bstride = z_bstride;
        a.t = t;
        a.t_rowstride = t_rowstride;
        a.B = B;
        a.d = d;
        a.P = hi;
        a.lds_stride = group_lds_stride(hi, G);
        a.ntiles = (B + R - 1) / R;
        a.out = ldj_out;
        a.z_out = z_out;
        a.nt = 1;
        a.prio = 1;
        const size_t lds = (size_t)(kMaxBlock / 64) * R * a.lds_stride * sizeof(float) +
                           std::max<size_t>((G * DPL + 4) * sizeof(float), 64 * 16);
        int64_t grid = 0;
        if (launch_group1_fwd(G, DPL, nv, a, lds, s, &grid))
          return check_hip("chain_group1_kernel (Chain bijector) launch");
      }
    }
    layer_layout = layer_layout && K <= 16;  // the d = 1 packed program holds 16 flows
    const int32_t lo4 = lo & ~3;
    const int32_t Pw = hi - lo4;
    const int32_t Qw = Pw >> 2;
    const float* tw = t + lo4;
    if (layer_layout && d == 1 && use_fast_math() && (Pw & 3) == 0 && (Qw & (Qw - 1)) == 0 &&
        Qw >= 2 && Qw <= 16 && t_rowstride != 0 && (t_rowstride & 3) == 0 &&
        (reinterpret_cast<uintptr_t>(tw) & 15) == 0 && t_rowstride * 256 < ((int64_t)1 << 31) &&
        z_bstride * 256 < ((int64_t)1 << 31) && env_int("NFN_WAVE1", 1) != 0) {
      a.y = z;
      a.y_bstride = z_bstride;
      a.t = tw;
      a.t_rowstride = t_rowstride;
      a.B = B;
      a.d = 1;
      a.P = Pw;
      a.lds_stride = Pw | 1;
      a.ntiles = (B + 63) / 64;
      a.out = ldj_out;
      a.z_out = z_out;
      a.nt = 1;
      a.prio = 1;
      // (plain walk: rotated tile slots measured no faster here, 0.4159 vs 0.4145 ms, r05zv)
      int64_t grid = 0;
      if (launch_fwd_ldj_wave1(Qw, a, (size_t)kMaxBlock * a.lds_stride * sizeof(float), s, &grid))
        return check_hip("chain_wave1_kernel (Chain bijector) launch");
    }
  }
  const int32_t P = hi - lo;
  const TileGeom g = tile_geom(P);
  if ((size_t)g.rows * ((size_t)g.lds_stride * sizeof(float)) > (size_t)kLdsMaxBytes)
    return fail(NFN_E_SHAPE, "parameter span too wide for LDS");
  a.y = z;
  a.y_bstride = z_bstride;
  a.t = K > 0 ? t + lo : t;
  a.t_rowstride = t_rowstride;
  a.B = B;
  a.d = d;
  a.P = P;
  a.lds_stride = g.lds_stride;
  a.tile_rows = g.rows;
  a.vec4 = (P % 4 == 0 && t_rowstride % 4 == 0 && (reinterpret_cast<uintptr_t>(a.t) & 15) == 0) ? 1 : 0;
  const int64_t nblk = (B + g.rows - 1) / g.rows;
  if (nblk > 0x7fffffffLL) return fail(NFN_E_SHAPE, "batch too large");
  launch_chain_fwd_ldj(use_fast_math(), dm_for(d), a, dim3((unsigned)nblk), dim3((unsigned)g.threads), g.lds_bytes,
                       z_out, ldj_out, s);
  return check_hip("chain_fwd_ldj_kernel launch");
}

}  // extern "C"
