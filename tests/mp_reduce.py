"""Rank body of tests/test_gpu_multiproc.py::test_two_rank_reduction_matches_one_rank
(run under torch.distributed.run, gloo, every rank on cuda:0): each rank evaluates its
contiguous shard of one dataset with the fused kernel and the (sum, count, non-finite)
all-reduce; rank 0 also evaluates the concatenated batch in one launch and prints both."""

import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from normalizingflownetwork_amd import ops  # noqa: E402
from normalizingflownetwork_amd.parallel import init_from_env, mean_log_prob_nonfinite, shard_bounds  # noqa: E402

C2 = ("planar", "radial") * 5


def main():
    rank, world, _ = init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    B = 1_000_003  # ragged over the ranks
    rng = np.random.default_rng(11)
    y = rng.standard_normal((B, 1)).astype(np.float32)
    t = rng.standard_normal((B, 32)).astype(np.float32)
    a, b = shard_bounds(B, rank, world)
    mean, nf = mean_log_prob_nonfinite(y[a:b], t[a:b], C2, 1, True)
    ypois = y.copy()
    ypois[[10, B // 2, B - 3]] = np.nan
    _, nf_p = mean_log_prob_nonfinite(ypois[a:b], t[a:b], C2, 1, True)
    res = {"rank": rank, "world": dist.get_world_size(), "mean": float(mean), "nonfinite": float(nf),
           "nonfinite_poisoned": float(nf_p)}
    if rank == 0:
        _, s1 = ops.chain_log_prob(y, t, C2, 1, True, want_values=False, want_sum=True)
        res["one_rank_mean"] = float(s1.item()) / B
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
