/*
 * nfn.h — C ABI of libnfn_hip.so, the MI355X (gfx950) implementation of the
 * conditional normalizing-flow log_prob hot path of siboehm/NormalizingFlowNetwork.
 *
 * Conventions
 *   - Every tensor pointer is DEVICE memory, caller-owned.  Nothing is allocated
 *     inside a compute call; scratch is passed in (`workspace`).
 *   - `flow_ids` is a HOST array (flow metadata, read while launching).
 *   - Calls are stream-ordered on `stream` (a hipStream_t; NULL = default stream)
 *     and return without synchronising.
 *   - Return value: 0 = ok; < 0 = error (see NFN_E_*); the message of the last
 *     error on the calling thread is returned by nfn_last_error().
 *   - Flow ids: 0 = planar, 1 = radial, 2 = affine (the reference's FLOWS
 *     registry, estimators/normalizing_flows/__init__.py:5).
 *   - `flow_ids[0..K-1]` is APPLICATION order, i.e. the reference's
 *     `flow_types` order.  The parameter row `t` is laid out exactly as the
 *     reference's Dense output: [base (2d if trainable_base) | block of
 *     flow_types[K-1] | ... | block of flow_types[0]]
 *     (estimators/DistributionLayers.py:252, 270-277).
 *   - Batch strides are in ELEMENTS (floats).  A stride of 0 broadcasts one row
 *     over the batch (tests/test_flows.py:22-29 feeds y of batch 1 against
 *     params of batch B).
 *
 * Reference interfaces replaced (file:line in the reference checkout):
 *   nfn_chain_logprob_f32  <- InverseNormalizingFlowLayer._get_distribution_fn(...)(t)
 *                             .log_prob(y)          estimators/DistributionLayers.py:245-255
 *                             incl. _get_bijector    estimators/DistributionLayers.py:267-278
 *                             and _get_base_dist     estimators/DistributionLayers.py:280-294;
 *                             with y_mean/y_std it is BaseEstimator.log_pdf's
 *                             "log_prob(y_circ) - sum(log y_std)"
 *                                                    estimators/BaseEstimator.py:77-86
 *                             and out_sum feeds score()/mle_log_likelihood_score
 *                                                    estimators/BaseEstimator.py:43-47,
 *                                                    evaluation/scorers.py:30-34
 *   nfn_chain_logprob_grad_f32
 *                          <- the gradient Keras autodiff takes through that log_prob when the
 *                             reference trains: model.compile(loss=NLL) / fit
 *                                                    estimators/BaseEstimator.py:19-31, 55-59,
 *                                                    estimators/MaximumLikelihoodNNEstimator.py:33-35
 *   nfn_chain_logprob_dense_f32
 *                          <- the estimator's output Dense layer (linear) followed by that
 *                             log_prob: MaximumLikelihoodNNEstimator.py:37-44 (Dense(P)) +
 *                             DistributionLayers.py:245-255, i.e. model(x).log_prob(y) given the
 *                             last hidden activations
 *   nfn_chain_sample_f32   <- new capability: the reference's layer cannot sample (its flows have
 *                             no _inverse; DistributionLayers.py:223-226, 240); this draws
 *                             y ~ p(y | t) through the inverted flows
 *   nfn_chain_logprob_grid_f32
 *                          <- the per-grid-point loop of dist.prob(y[i]) over a batch of x in
 *                             evaluation/visualization/flow_plotting.py:33-53 (plot_model)
 *   nfn_flow_fwd_ldj_f32   <- PlanarFlow._forward/_forward_log_det_jacobian
 *                                                    estimators/normalizing_flows/PlanarFlow.py:20-80
 *                             RadialFlow._forward/_forward_log_det_jacobian
 *                                                    estimators/normalizing_flows/RadialFlow.py:20-84
 *                             AffineFlow (tfp Affine) estimators/normalizing_flows/AffineFlow.py:4-9
 *   nfn_flow_vjp_f32       <- the gradient TF's tape takes through those three bijectors'
 *                             _forward / _forward_log_det_jacobian (PlanarFlow.py:68-80,
 *                             RadialFlow.py:50-70, AffineFlow.py:4-9) when a loss reads them
 *   nfn_split_blocks_f32   <- the tf slices t[:, o:o+size] (copies) that _get_bijector hands each
 *                             flow                   estimators/DistributionLayers.py:267-278
 *   nfn_chain_fwd_ldj_f32  <- tfp Chain(flows).forward / .forward_log_det_jacobian as composed by
 *                             InverseNormalizingFlowLayer._get_bijector
 *                                                    estimators/DistributionLayers.py:267-278
 *   nfn_posterior_lse_f32  <- BayesianNNEstimator.score per-sample logsumexp
 *                                                    estimators/BayesianNNEstimator.py:65-76,
 *                                                    evaluation/scorers.py:13-27
 *   nfn_comm_* /
 *   nfn_allreduce_mean     <- the mean of score()/mle_log_likelihood_score over a batch
 *                             sharded across GPUs (one RCCL all-reduce of {sum, count})
 *                                                    estimators/BaseEstimator.py:43-47,
 *                                                    evaluation/scorers.py:30-34
 *   nfn_param_size /
 *   nfn_total_param_size   <- Flow.get_param_size    PlanarFlow.py:35-41, RadialFlow.py:36-42,
 *                                                    AffineFlow.py:11-17
 *                             InverseNormalizingFlowLayer.get_total_param_size
 *                                                    estimators/DistributionLayers.py:257-265
 */
#ifndef NFN_H_
#define NFN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NFN_FLOW_PLANAR 0
#define NFN_FLOW_RADIAL 1
#define NFN_FLOW_AFFINE 2

#define NFN_MAX_FLOWS 64
#define NFN_MAX_DIMS 32

#define NFN_OK 0
#define NFN_E_SHAPE -1     /* bad batch / width / stride / dims            */
#define NFN_E_FLOW_ID -2   /* unknown flow id or too many flows            */
#define NFN_E_NULLPTR -3   /* required pointer is NULL                     */
#define NFN_E_HIP -4       /* HIP runtime error (launch, no device, ...)   */
#define NFN_E_COMM -5      /* RCCL error                                   */

#define NFN_COMM_ID_BYTES 128

/* Library version as MAJOR*10000 + MINOR*100 + PATCH.
 *   203 (0.2.3): + nfn_set_launch_events (additive, measurement hook).
 *   202 (0.2.2): + nfn_flow_vjp_f32 (additive).
 *   201 (0.2.1): + nfn_split_blocks_f32 (additive; every 200 entry point unchanged).
 *   200 (0.2.0): out_sum is a device double[2] {sum, non-finite count} (was double[1]);
 *                the workspace needs no initialisation (its finishing ticket carries a
 *                per-call epoch).
 *   100 (0.1.0): first release. */
#define NFN_ABI_VERSION 203
int32_t nfn_version(void);

/* Message of the last failing call on this thread ("" if none). */
const char* nfn_last_error(void);

/* Measurement hook (no reference counterpart: the reference has no device timing).  The
 * NEXT kernel launch made on the calling thread records start_event / stop_event (hipEvent_t,
 * created by the caller, e.g. torch.cuda.Event(enable_timing=True) after one record) from its
 * own dispatch (hipExtLaunchKernel: the dispatch packet's start / end timestamps), then the
 * hook clears; later launches of the same call go unrecorded.  Unlike hipEventRecord markers
 * around the call, nothing is queued between consecutive launches.  (NULL, NULL) clears a
 * pending pair.  Returns NFN_OK. */
int32_t nfn_set_launch_events(void* start_event, void* stop_event);

/* Transcendental implementation used by later launches in this process:
 * 0 = fast (gfx950 v_exp/v_log/v_rcp with stable rewrites; the default),
 * 1 = precise (OCML expf/logf/log1pf/tanhf, IEEE division).
 * The initial value comes from the environment variable NFN_MATH=fast|precise.
 * Returns the previous mode, or NFN_E_SHAPE for an unknown mode. */
int32_t nfn_set_math_mode(int32_t mode);

/* Width of one flow's parameter block for event dimension d; < 0 on bad id. */
int32_t nfn_param_size(int32_t flow_id, int32_t d);

/* Total width P of a parameter row: sum of blocks + 2d if trainable_base. */
int32_t nfn_total_param_size(const int32_t* flow_ids, int32_t K, int32_t d, int32_t trainable_base);

/* Number of doubles of device workspace nfn_chain_logprob_f32 needs when
 * out_sum != NULL (per-workgroup partial sums and non-finite counts). */
int64_t nfn_chain_workspace_doubles(int64_t B, int32_t d, int32_t P);

/*
 * Fused chain log-density.
 *   out_logp[b] = log N(z_K; base(t_b)) + sum_k fldj_k(z_k; theta_k(t_b)) [- sum_j log y_std_j]
 * with z_0 = y_b (or (y_b - y_mean)/y_std when y_mean/y_std are given).
 *   y          : (B or 1, d) rows at y_bstride floats (0 = broadcast)
 *   t          : (B or 1, P) rows at t_rowstride floats (0 = broadcast), P = nfn_total_param_size
 *   y_mean/y_std : (d,) device arrays or both NULL
 *   out_logp   : (B,) may be NULL when only the sum is wanted
 *   out_sum    : device double[2] or NULL — receives {sum_b out_logp[b] (fp64 accumulation;
 *                non-finite values propagate, as in the reference's .mean()), the number of
 *                non-finite out_logp values}, finished inside the kernel by its last
 *                workgroup (fixed summation order: bitwise deterministic; no extra launch)
 *   workspace  : device double[nfn_chain_workspace_doubles(B, d, P)] when out_sum != NULL.
 *                Needs no initialisation (e.g. a plain hipMalloc): the finishing ticket
 *                (workspace[1]) is tagged with a per-call epoch, so a stale or garbage
 *                ticket restarts the count (no memset launch precedes the kernel; only
 *                garbage whose upper 32 bits equal the call's epoch, 2^-32 for random
 *                bits, would be taken for this call's count).
 *                Layout: workspace[0] = number n of per-workgroup pairs written,
 *                workspace[1] = the finishing ticket, workspace[2 + 2i] /
 *                workspace[3 + 2i] = workgroup i's fp64 partial sum / non-finite count.
 *                With out_sum == NULL and workspace != NULL only the pairs are written
 *                (finish with nfn_reduce_partials_f64).  One workspace per call in
 *                flight: two calls in flight sharing one race.
 * A batch longer than 2^24 samples runs as consecutive launches over 2^24-sample slices
 * (a long persistent launch drifts): their pairs follow one another in the
 * workspace, n counts them all, and out_sum is one sum over every pair in fixed order.
 */
int32_t nfn_chain_logprob_f32(const float* y, int64_t y_bstride, const float* t, int64_t t_rowstride,
                              int64_t B, int32_t d, const int32_t* flow_ids, int32_t K,
                              int32_t trainable_base, const float* y_mean, const float* y_std,
                              float* out_logp, double* out_sum, double* workspace, void* stream);

/*
 * Fused backward (the training path).  With L = sum_b g_out[b] * logp[b]
 * (g_out NULL => all ones), per sample b:
 *   grad_t[b, :] = dL/dt[b, :]  — (B, P) rows at grad_t_rowstride (>= P), nullable
 *   grad_y[b, :] = dL/dy[b, :]  — (B, d) contiguous, nullable
 *   out_logp[b]  = logp[b]      — nullable
 * Inputs as for nfn_chain_logprob_f32.  A broadcast input (stride 0) still gets one
 * gradient row per sample; reducing over the batch is the caller's.  y_mean /
 * y_std are constants here (BaseEstimator.set_data_normalization, not trained).
 */
int32_t nfn_chain_logprob_grad_f32(const float* y, int64_t y_bstride, const float* t, int64_t t_rowstride,
                                   int64_t B, int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                                   const float* y_mean, const float* y_std, const float* g_out, float* out_logp,
                                   float* grad_t, int64_t grad_t_rowstride, float* grad_y, void* stream);

/*
 * Output Dense layer fused into the chain: t_b = h_b W + bias (never written to
 * memory), then the chain as nfn_chain_logprob_f32 evaluates it.  Numerics: at d = 1
 * (fast math) the chain keeps round 5's m = softplus(w u) - 1 + 1e-5 (the compute-bound
 * fused kernels do not take the cancellation-aware form), and at H = 16, P <= 32 t is formed
 * from exact 3-way bf16 splits of h and W on the bf16 matrix cores (six products per fp32
 * product, fp32 accumulation): fp32-level, not bitwise an fp32 GEMM.
 *   h    : (B, H) rows at h_rowstride floats (>= H, multiple of 4), 16-byte aligned;
 *          H in {4, 8, 16, 32, 64}
 *   W    : (H, P) row-major, P = nfn_total_param_size <= 64;  bias : (P,) or NULL
 *   d <= 8.  Other shapes return NFN_E_SHAPE (compute t = h W + b and call
 *   nfn_chain_logprob_f32 instead).  Workspace as for nfn_chain_logprob_f32.
 */
int32_t nfn_chain_logprob_dense_f32(const float* y, int64_t y_bstride, const float* h, int64_t h_rowstride,
                                    int32_t H, const float* W, const float* bias, int64_t B, int32_t d,
                                    const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                                    const float* y_std, float* out_logp, double* out_sum, double* workspace,
                                    void* stream);

/*
 * Sampling: y_b = f_0^{-1}(... f_{K-1}^{-1}(loc_b + scale_b * eps_b)) [* y_std + y_mean]
 * for caller-supplied standard-normal eps (B, d) at eps_bstride (0 = one row);
 * planar steps are inverted by safeguarded Newton iteration (the constraint
 * w.u_hat >= -1 + 1e-5 makes them invertible), radial steps in closed form.
 *   y_out    : (B, d) contiguous
 *   logp_out : (B,) log-density of each sample (incl. -sum log y_std), or NULL
 */
int32_t nfn_chain_sample_f32(const float* eps, int64_t eps_bstride, const float* t, int64_t t_rowstride, int64_t B,
                             int32_t d, const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                             const float* y_mean, const float* y_std, float* y_out, float* logp_out, void* stream);

/*
 * Density on a grid of y values shared by every parameter row:
 *   out[g * out_gstride + b] = logp(y_grid[g] | t_b) [- sum log y_std]
 *   y_grid : (G, d) rows at y_gstride floats (0 = one row);  t : as nfn_chain_logprob_f32
 *   out    : (G, B) with out_gstride >= B
 */
int32_t nfn_chain_logprob_grid_f32(const float* y_grid, int64_t y_gstride, int32_t G, const float* t,
                                   int64_t t_rowstride, int64_t B, int32_t d, const int32_t* flow_ids, int32_t K,
                                   int32_t trainable_base, const float* y_mean, const float* y_std, float* out,
                                   int64_t out_gstride, void* stream);

/*
 * One bijector, forward direction: z_out = f(z), ldj_out = log|det df/dz| (B,).
 *   z     : (B or 1, d) rows at z_bstride (0 = broadcast)
 *   t_k   : (B or 1, nfn_param_size(flow_id, d)) rows at t_rowstride (0 = broadcast);
 *           a column slice of a wider parameter row is passed as base pointer + stride
 *   z_out : (B, d) contiguous, may be NULL; ldj_out : (B,), may be NULL
 */
int32_t nfn_flow_fwd_ldj_f32(int32_t flow_id, const float* z, int64_t z_bstride, const float* t_k,
                             int64_t t_rowstride, int64_t B, int32_t d, float* z_out, float* ldj_out,
                             void* stream);

/*
 * One bijector's vector-Jacobian product (the backward of nfn_flow_fwd_ldj_f32): for
 * L = sum_b <g_z[b], f(z[b])> + g_ldj[b] * log|det df/dz|(z[b]),
 *   dz_out : (B, d) contiguous, dL/dz, may be NULL
 *   dt_out : (B, nfn_param_size(flow_id, d)) contiguous, dL/dt_k per sample (a broadcast
 *            t_k row still gets one gradient row per sample: the caller sums them), may be NULL
 *   g_z    : (B, d) contiguous, or NULL for zero; g_ldj : (B,), or NULL for zero
 *   z, t_k : as for nfn_flow_fwd_ldj_f32 (0 strides broadcast)
 */
int32_t nfn_flow_vjp_f32(int32_t flow_id, const float* z, int64_t z_bstride, const float* t_k, int64_t t_rowstride,
                         int64_t B, int32_t d, const float* g_z, const float* g_ldj, float* dz_out, float* dt_out,
                         void* stream);

/*
 * Column blocks of a parameter row, each made contiguous, in ONE pass over t:
 *   t      : (B, >= sum(widths)) rows at t_rowstride floats; block k is the widths[k]
 *            columns after blocks 0..k-1 (t points at block 0's first column)
 *   dst    : block k lands at dst + B * (widths[0] + ... + widths[k-1]) as a contiguous
 *            (B, widths[k]) array; dst must not overlap t
 * What InverseNormalizingFlowLayer._get_bijector's slices t[:, o:o+size] are in TF — copies
 * (estimators/DistributionLayers.py:267-278): the per-flow Bijector calls then read only their
 * own parameters (nfn_flow_fwd_ldj_f32 on a view of the wide row reads the whole 128-B lines).
 * 1 <= nblocks <= NFN_MAX_FLOWS, widths[k] >= 1.
 */
int32_t nfn_split_blocks_f32(const float* t, int64_t t_rowstride, int64_t B, const int32_t* widths, int32_t nblocks,
                             float* dst, void* stream);

/*
 * The Bijector API's Chain of flows in ONE launch (instead of one launch per flow):
 *   z_out[b]   = f_{K-1}( ... f_0(z[b]) )       (flow_ids in APPLICATION order, f_0 first)
 *   ldj_out[b] = sum_k log|det J_k|             (summed in application order, as tfp Chain)
 *   t : (B, >= span) rows at t_rowstride floats (0 = one row broadcast); flow k reads its
 *       param_size(flow_ids[k], d) floats at t + b*t_rowstride + block_offsets[k]
 *       (e.g. the layer's reversed layout: the views a Chain's flows hold into one t)
 *   z_out : (B, d) contiguous, may be NULL; ldj_out : (B,), may be NULL
 */
int32_t nfn_chain_fwd_ldj_f32(const float* z, int64_t z_bstride, const float* t, int64_t t_rowstride, int64_t B,
                              int32_t d, const int32_t* flow_ids, const int32_t* block_offsets, int32_t K,
                              float* z_out, float* ldj_out, void* stream);

/* out[0] = sum of the n doubles at `in` (device), one workgroup, fixed order
 * (deterministic). */
int32_t nfn_reduce_sum_f64(const double* in, int64_t n, double* out, void* stream);

/* Finishes a partials-only call: out_sum (device double[2]) := {sum of the partial sums,
 * number of non-finite values} a chain / posterior call left in `workspace`.  The same
 * fixed order as the in-kernel finish: bitwise identical to out_sum of the same call. */
int32_t nfn_reduce_partials_f64(const double* workspace, double* out_sum, void* stream);

/* Number of doubles of device workspace for nfn_posterior_lse_f32: the partials
 * block (as for the chain) followed by the draw-split region.  Passing a
 * workspace is optional without out_sum, but enables the draw split (more
 * parallelism when B is small relative to the GPU). */
int64_t nfn_posterior_workspace_doubles(int64_t B, int32_t d, int32_t P);

/*
 * Bayesian posterior score per sample:
 *   out_lse[b] = logsumexp_s( logp(y_b | t[s, b]) [- sum log y_std] ) - log(S)
 *   t : S draws; draw s, sample b at t + s*t_drawstride + b*t_rowstride
 *   out_sum (nullable), workspace: as nfn_chain_logprob_f32 — {sum_b out_lse[b], non-finite count}.
 */
int32_t nfn_posterior_lse_f32(const float* y, int64_t y_bstride, const float* t, int64_t t_drawstride,
                              int64_t t_rowstride, int32_t S, int64_t B, int32_t d,
                              const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                              const float* y_mean, const float* y_std, float* out_lse, double* out_sum,
                              double* workspace, void* stream);

/*
 * Backward of nfn_chain_logprob_dense_f32 (the training step through the output Dense
 * layer and the flow chain, MaximumLikelihoodNNEstimator.py:37-44 + BaseEstimator.py:19-31),
 * for L = sum_b g_out[b] * logp_b (g_out NULL = ones), t = h W + b never written:
 *   grad_h : (B, H) at grad_h_rowstride, dL/dh = dt W^T      (nullable)
 *   grad_W : (H, P) = sum_b h_b^T dt_b;  grad_b : (P,) = sum_b dt_b   (nullable; overwritten,
 *            fixed-order reduction: bitwise deterministic)
 *   grad_y : (B, d) contiguous (nullable);  out_logp : (B,) (nullable)
 *   workspace : device float[nfn_dense_grad_workspace_floats(B, H, P)] (needed with grad_W / grad_b)
 * Shapes as nfn_chain_logprob_dense_f32 (H in {4..64}, P <= 64, d <= 8), and the tile's
 * flow inputs must fit LDS; other shapes return NFN_E_SHAPE.  At d = 1, H = 16, P <= 32
 * (fast math) t stays an fp32 MFMA GEMM while dh and dW use exact 3-way bf16 splits.
 */
int64_t nfn_dense_grad_workspace_floats(int64_t B, int32_t H, int32_t P);
int32_t nfn_chain_logprob_dense_grad_f32(const float* y, int64_t y_bstride, const float* h, int64_t h_rowstride,
                                         int32_t H, const float* W, const float* bias, int64_t B, int32_t d,
                                         const int32_t* flow_ids, int32_t K, int32_t trainable_base,
                                         const float* y_mean, const float* y_std, const float* g_out,
                                         float* out_logp, float* grad_h, int64_t grad_h_rowstride, float* grad_W,
                                         float* grad_b, float* grad_y, float* workspace, void* stream);

/*
 * Bayesian posterior score with the output DenseVariational layer fused
 * (BayesianNNEstimator.py:65-76 score, :136-145 the variational output layer):
 *   out_lse[b] = logsumexp_s( logp(y_b | t_sb = h_sb W_s + bias_s) [- sum log y_std] ) - log(S)
 * with t_sb formed on chip (fp32 MFMA), never written to memory.
 *   h    : draw s, sample b at h + s*h_drawstride + b*h_rowstride (h_drawstride 0 = one h
 *          shared by every draw); H in {4, 8, 16, 32, 64}; 16-byte aligned, strides multiples of 4
 *   W    : draw s at W + s*w_drawstride, (H, P) row-major;  bias : draw s at
 *          bias + s*bias_drawstride, (P,), or NULL
 *   P <= 64, d <= 8 (else NFN_E_SHAPE).  out_sum / workspace as for nfn_chain_logprob_f32
 *   (nfn_chain_workspace_doubles).
 */
int32_t nfn_posterior_lse_dense_f32(const float* y, int64_t y_bstride, const float* h, int64_t h_drawstride,
                                    int64_t h_rowstride, int32_t H, const float* W, int64_t w_drawstride,
                                    const float* bias, int64_t bias_drawstride, int32_t S, int64_t B, int32_t d,
                                    const int32_t* flow_ids, int32_t K, int32_t trainable_base, const float* y_mean,
                                    const float* y_std, float* out_lse, double* out_sum, double* workspace,
                                    void* stream);

/*
 * Multi-GPU (one process per GPU, batch sharded over ranks).  The communicator
 * is RCCL over xGMI; its handle is opaque (`void*` = ncclComm_t).
 *   nfn_comm_unique_id : rank 0 creates the 128-byte rendezvous id, which the
 *                        caller distributes to every rank (any channel).
 *   nfn_comm_init      : collective over all ranks; binds the CURRENT HIP device.
 *   nfn_allreduce_mean : sum_count (device double[3]) := sum over ranks of
 *                        {local_sum[0], local_count, local_sum[1]}, where local_sum is a
 *                        {sum, non-finite count} pair as out_sum returns it; mean_out
 *                        (device double[1], nullable) := sum / count.  One 24-byte RCCL
 *                        all-reduce.  Stream-ordered, no host sync.
 */
int32_t nfn_comm_unique_id(uint8_t* id_out);
int32_t nfn_comm_init(void** comm_out, int32_t nranks, const uint8_t* id, int32_t rank);
int32_t nfn_comm_destroy(void* comm);
int32_t nfn_allreduce_mean(void* comm, const double* local_sum, int64_t local_count, double* sum_count,
                           double* mean_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NFN_H_ */
