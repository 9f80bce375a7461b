// nfn_comm.hip — multi-GPU reduction of the mean log-likelihood over RCCL
// (SURVEY.md §8(e)).  Samples are independent, so each rank evaluates its own
// batch slice; the only exchange is one 24-byte all-reduce of {sum, count,
// non-finite count} in fp64 — the distributed form of BaseEstimator.score's .mean()
// (estimators/BaseEstimator.py:43-47, evaluation/scorers.py:30-34).
// Everything is stream-ordered on the caller's stream: no host synchronisation.
#include <rccl/rccl.h>

#include <string>

#include "nfn_launch.h"

namespace nfn {
namespace {

static_assert(sizeof(ncclUniqueId) == NFN_COMM_ID_BYTES, "RCCL unique id size");

int32_t comm_fail(ncclResult_t r, const char* what) {
  return set_error(NFN_E_COMM, (std::string(what) + ": " + ncclGetErrorString(r)).c_str());
}

__global__ void pack_sum_count_kernel(const double* __restrict__ local_sum, double count,
                                      double* __restrict__ sum_count) {
  sum_count[0] = local_sum[0];
  sum_count[1] = count;
  sum_count[2] = local_sum[1];
}

__global__ void finish_mean_kernel(const double* __restrict__ sum_count, double* __restrict__ mean) {
  mean[0] = sum_count[0] / sum_count[1];
}

}  // namespace
}  // namespace nfn

using namespace nfn;

extern "C" {

int32_t nfn_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return set_error(NFN_E_NULLPTR, "nfn_comm_unique_id: id_out is NULL");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return comm_fail(r, "ncclGetUniqueId");
  memcpy(id_out, id.internal, NFN_COMM_ID_BYTES);
  return NFN_OK;
}

int32_t nfn_comm_init(void** comm_out, int32_t nranks, const uint8_t* id, int32_t rank) {
  if (!comm_out || !id) return set_error(NFN_E_NULLPTR, "nfn_comm_init: NULL comm_out or id");
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return set_error(NFN_E_SHAPE, "nfn_comm_init: need 0 <= rank < nranks");
  ncclUniqueId uid;
  memcpy(uid.internal, id, NFN_COMM_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, uid, rank);
  if (r != ncclSuccess) return comm_fail(r, "ncclCommInitRank");
  *comm_out = c;
  return NFN_OK;
}

int32_t nfn_comm_destroy(void* comm) {
  if (!comm) return NFN_OK;
  const ncclResult_t r = ncclCommDestroy(static_cast<ncclComm_t>(comm));
  return r == ncclSuccess ? NFN_OK : comm_fail(r, "ncclCommDestroy");
}

int32_t nfn_allreduce_mean(void* comm, const double* local_sum, int64_t local_count, double* sum_count,
                           double* mean_out, void* stream) {
  const HookScope hook_scope;
  if (!comm || !local_sum || !sum_count)
    return set_error(NFN_E_NULLPTR, "nfn_allreduce_mean: NULL comm, local_sum or sum_count");
  if (local_count < 0) return set_error(NFN_E_SHAPE, "nfn_allreduce_mean: negative local_count");
  hipStream_t s = static_cast<hipStream_t>(stream);
  nfn_launch((pack_sum_count_kernel), 1, 1, 0, s, local_sum, (double)local_count, sum_count);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NFN_E_HIP, hipGetErrorString(e));
  const ncclResult_t r = ncclAllReduce(sum_count, sum_count, 3, ncclFloat64, ncclSum,
                                       static_cast<ncclComm_t>(comm), s);
  if (r != ncclSuccess) return comm_fail(r, "ncclAllReduce");
  if (mean_out) {
    nfn_launch((finish_mean_kernel), 1, 1, 0, s, sum_count, mean_out);
    e = hipGetLastError();
    if (e != hipSuccess) return set_error(NFN_E_HIP, hipGetErrorString(e));
  }
  return NFN_OK;
}

}  // extern "C"
