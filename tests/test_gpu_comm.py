"""The library's own RCCL path (nfn_comm_init / nfn_allreduce_mean, include/nfn.h)
on the one GPU of the test box: a single-rank communicator, so the all-reduce is
the identity and the mean must equal the local sum / count exactly.  The N-rank
form runs in the driver's 8-GPU bench (bench.py --allreduce native)."""

import numpy as np
import pytest
import torch

from oracle import nfn_oracle as O

pytestmark = pytest.mark.gpu


def test_native_comm_single_rank_mean(gpu):
    from normalizingflownetwork_amd.parallel import NativeComm

    comm = NativeComm()
    try:
        s = torch.tensor([12.5, 2.0], dtype=torch.float64, device=gpu)  # {sum, non-finite count}
        m = comm.allreduce_mean(s, 5)
        torch.cuda.synchronize()
        assert comm.sum_count.tolist() == [12.5, 5.0, 2.0]
        assert m.item() == 2.5
    finally:
        comm.close()


def test_native_comm_mean_log_prob_matches_oracle(gpu):
    from normalizingflownetwork_amd import ops
    from normalizingflownetwork_amd.parallel import NativeComm

    ft = ("planar", "radial") * 5
    B, d = 4096, 1
    P = O.total_param_size(ft, d, True)
    rng = np.random.default_rng(7)
    y = rng.standard_normal((B, d)).astype(np.float32)
    t = rng.standard_normal((B, P)).astype(np.float32)
    _, s, nf = ops.chain_log_prob(torch.from_numpy(y).to(gpu), torch.from_numpy(t).to(gpu), ft, d, True,
                                  want_values=False, want_nonfinite=True)
    comm = NativeComm()
    try:
        m = comm.allreduce_mean(torch.cat([s, nf]), B).item()
    finally:
        comm.close()
    ref = float(np.mean(O.chain_log_prob(y, t, ft, d, True)))
    assert abs(m - ref) <= 1e-5 * max(1.0, abs(ref))
