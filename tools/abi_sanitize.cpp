// abi_sanitize.cpp — the C ABI's host code under AddressSanitizer + UBSan (SURVEY.md §5:
// host sanitizer build).  Links the library's objects with nfn_api.hip / nfn_comm.hip
// compiled for the host with -fsanitize=address,undefined (device code untouched) and
// drives every entry point's argument validation, the flow-program builder (through
// nfn_total_param_size and the rejection paths) and the workspace-size arithmetic — the
// host code that runs before any launch.  Every call here fails validation or is a pure
// host query, so nothing reaches the GPU (the program is safe with or without a device).
// Build + run: tests/test_host_sanitizer.py (or tools/build_abi_sanitize.sh).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "nfn.h"

static int g_fail = 0;
#define EXPECT(call, want)                                                                   \
  do {                                                                                       \
    const long long got_ = (long long)(call);                                                \
    if (got_ != (long long)(want)) {                                                         \
      fprintf(stderr, "%s:%d %s -> %lld, want %lld (%s)\n", __FILE__, __LINE__, #call, got_, \
              (long long)(want), nfn_last_error());                                          \
      ++g_fail;                                                                              \
    }                                                                                        \
  } while (0)

int main() {
  EXPECT(nfn_version(), NFN_ABI_VERSION);
  EXPECT(nfn_param_size(NFN_FLOW_PLANAR, 3), 7);
  EXPECT(nfn_param_size(NFN_FLOW_RADIAL, 3), 5);
  EXPECT(nfn_param_size(NFN_FLOW_AFFINE, 3), 6);
  EXPECT(nfn_param_size(7, 1), NFN_E_FLOW_ID);
  EXPECT(nfn_param_size(0, 0), NFN_E_SHAPE);
  EXPECT(nfn_param_size(0, NFN_MAX_DIMS + 1), NFN_E_SHAPE);
  const int32_t pr[2] = {NFN_FLOW_PLANAR, NFN_FLOW_RADIAL};
  int32_t many[NFN_MAX_FLOWS + 1];
  for (int i = 0; i <= NFN_MAX_FLOWS; ++i) many[i] = i % 3;
  EXPECT(nfn_total_param_size(pr, 2, 1, 1), 2 + 3 + 3);
  EXPECT(nfn_total_param_size(many, NFN_MAX_FLOWS, 8, 1) > 0, 1);
  EXPECT(nfn_total_param_size(many, NFN_MAX_FLOWS + 1, 1, 0), NFN_E_FLOW_ID);
  const int32_t bad[1] = {5};
  EXPECT(nfn_total_param_size(bad, 1, 1, 0), NFN_E_FLOW_ID);
  EXPECT(nfn_total_param_size(nullptr, 2, 1, 0) < 0, 1);
  for (int64_t B : {(int64_t)0, (int64_t)1, (int64_t)1000, (int64_t)1 << 24, (int64_t)1 << 27}) {
    EXPECT(nfn_chain_workspace_doubles(B, 1, 32) >= 0, 1);
    EXPECT(nfn_posterior_workspace_doubles(B, 1, 32) >= 0, 1);
    EXPECT(nfn_dense_grad_workspace_floats(B, 16, 32) >= 0, 1);
  }
  EXPECT(nfn_set_math_mode(3), NFN_E_SHAPE);

  float* f = reinterpret_cast<float*>(0x1000);  // never dereferenced: every call fails validation
  double* dd = reinterpret_cast<double*>(0x1000);
  const int64_t big = ((int64_t)1 << 24) + 1;
  // forward
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 8, -1, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 4, 10, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 8, 10, 1, pr, 2, 1, f, nullptr, f, nullptr, nullptr, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 8, 10, 1, pr, 2, 1, nullptr, nullptr, f, dd, nullptr, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_chain_logprob_f32(nullptr, 1, f, 8, 10, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 8, big, 1, pr, 2, 1, nullptr, nullptr, f, dd, nullptr, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 8, 10, 1, bad, 1, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_FLOW_ID);
  EXPECT(nfn_chain_logprob_f32(f, 1, f, 8, 0, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_OK);
  // posterior
  EXPECT(nfn_posterior_lse_f32(f, 1, f, 80, 8, 0, 10, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_SHAPE);
  // backward
  EXPECT(nfn_chain_logprob_grad_f32(f, 1, f, 4, 10, 1, pr, 2, 1, nullptr, nullptr, nullptr, nullptr, f, 8, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_logprob_grad_f32(f, 1, f, 8, 10, 1, pr, 2, 1, nullptr, nullptr, nullptr, nullptr, f, 4, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_logprob_grad_f32(nullptr, 1, f, 8, 10, 1, pr, 2, 1, nullptr, nullptr, nullptr, nullptr, f, 8, f, nullptr), NFN_E_NULLPTR);
  // fused Dense forward
  EXPECT(nfn_chain_logprob_dense_f32(f, 1, f, 16, 10, f, nullptr, 10, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_logprob_dense_f32(f, 1, f, 8, 16, f, nullptr, 10, 1, pr, 2, 1, nullptr, nullptr, f, nullptr, nullptr, nullptr), NFN_E_SHAPE);
  // per-flow, Chain, split, grid
  EXPECT(nfn_flow_fwd_ldj_f32(9, f, 1, f, 3, 10, 1, f, f, nullptr), NFN_E_FLOW_ID);
  EXPECT(nfn_flow_fwd_ldj_f32(0, f, 1, f, 2, 10, 1, f, f, nullptr), NFN_E_SHAPE);
  const int32_t offs[2] = {3, 0}, neg[2] = {3, -1}, badp[2] = {0, 9};
  EXPECT(nfn_chain_fwd_ldj_f32(f, 1, f, 6, 10, 1, badp, offs, 2, f, f, nullptr), NFN_E_FLOW_ID);
  EXPECT(nfn_chain_fwd_ldj_f32(f, 1, f, 5, 10, 1, pr, offs, 2, f, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_fwd_ldj_f32(f, 1, f, 6, 10, 1, pr, neg, 2, f, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_chain_fwd_ldj_f32(f, 1, f, 6, 10, 1, pr, nullptr, 2, f, f, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_chain_fwd_ldj_f32(f, 1, f, 6, 0, 1, pr, offs, 2, f, f, nullptr), NFN_OK);
  const int32_t w3[3] = {3, 3, 2}, w0[2] = {3, 0};
  EXPECT(nfn_split_blocks_f32(nullptr, 8, 10, w3, 3, nullptr, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_split_blocks_f32(f, 8, 10, nullptr, 3, f, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_split_blocks_f32(f, 8, 10, w3, 0, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_split_blocks_f32(f, 7, 10, w3, 3, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_split_blocks_f32(f, 8, 10, w0, 2, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_split_blocks_f32(f, 8, 10, w3, NFN_MAX_FLOWS + 1, f, nullptr), NFN_E_SHAPE);
  EXPECT(nfn_split_blocks_f32(f, 8, 0, w3, 3, f, nullptr), NFN_OK);
  EXPECT(nfn_chain_logprob_grid_f32(nullptr, 1, 4, nullptr, 8, 10, 1, pr, 2, 1, nullptr, nullptr, nullptr, 10, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_chain_logprob_grid_f32(nullptr, 1, -1, nullptr, 8, 10, 1, pr, 2, 1, nullptr, nullptr, nullptr, 10, nullptr), NFN_E_SHAPE);
  // communicator
  void* comm = nullptr;
  uint8_t uid[NFN_COMM_ID_BYTES];
  memset(uid, 0, sizeof(uid));
  EXPECT(nfn_comm_init(&comm, 0, uid, 0), NFN_E_SHAPE);
  EXPECT(nfn_comm_init(&comm, 2, uid, 2), NFN_E_SHAPE);
  EXPECT(nfn_comm_init(&comm, 2, nullptr, 0), NFN_E_NULLPTR);
  EXPECT(nfn_comm_unique_id(nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_allreduce_mean(nullptr, nullptr, 1, nullptr, nullptr, nullptr), NFN_E_NULLPTR);
  EXPECT(nfn_comm_destroy(nullptr), NFN_OK);
  EXPECT(strlen(nfn_last_error()) < 4096, 1);
  printf("abi_sanitize: %d mismatches\n", g_fail);
  return g_fail == 0 ? 0 : 1;
}
