"""Host-side checks of round-2 items that need no GPU.

* The release library contains no tuning / ablation knob: the NFN_* names the NFN_DIAG
  build reads from the environment are absent from libnfn_hip.so (only NFN_MATH, the
  documented initial math mode, remains).
* Bayesian estimator: the DenseVariational mean-field posterior of the reference
  (BayesianNNEstimator.py:92-107, DistributionLayers.py:17-55) and its learning rate.
* The (sum, count, non-finite) all-reduce over a world-size-2 gloo group (CPU).
"""

import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import REPO

KNOBS = [b"NFN_ABLATE_FLOWS", b"NFN_ABLATE_LOADS", b"NFN_LOAD_MODE", b"NFN_POST_SPLIT", b"NFN_TILE_ROWS",
         b"NFN_WG_PER_CU", b"NFN_PRIO", b"NFN_GROUP_LANES"]


def test_release_library_has_no_knobs(native_lib):
    from normalizingflownetwork_amd import build

    blob = open(build.OUT, "rb").read()
    present = [k.decode() for k in KNOBS if k in blob]
    assert not present, f"knob names compiled into the release library: {present}"
    assert b"NFN_MATH" in blob
    if os.path.exists(build.DIAG_OUT):
        diag = open(build.DIAG_OUT, "rb").read()
        assert b"NFN_ABLATE_FLOWS" in diag and b"NFN_LOAD_MODE" in diag


def test_mean_field_scale_formula():
    from normalizingflownetwork_amd.estimators import mean_field_scale

    rho = torch.tensor([-50.0, -1.0, 0.0, 0.3, 10.0, 200.0])
    ref = [1e-3 + math.log1p(math.exp(math.log(math.expm1(1.0)) + 0.05 * r)) for r in rho.tolist()]
    np.testing.assert_allclose(mean_field_scale(rho).numpy(), ref, rtol=1e-6)
    assert mean_field_scale(torch.zeros(1)).item() == pytest.approx(1.001, rel=1e-6)  # softplus(log(e-1)) = 1


def test_bayes_posterior_variables_and_learning_rate():
    from normalizingflownetwork_amd.estimators import BayesNormalizingFlowNetwork

    m = BayesNormalizingFlowNetwork(n_dims=1, n_flows=2, hidden_sizes=(10,), n_dims_x=3)
    assert m.learning_rate == 2e-2  # BayesNormalizingFlowNetwork.build_function default, used by fit
    assert BayesNormalizingFlowNetwork(n_dims=1, learning_rate=0.5).learning_rate == 0.5
    P = m.dist_layer.get_total_param_size()
    assert [tuple(w.shape) for w in m._mlp.weights] == [(3, 10), (10, P)]
    # loc and rho ~ N(0, 0.05) (Keras "normal" initializer), one [loc | rho] vector per layer
    locs = torch.cat([torch.cat([w.reshape(-1), b]) for w, b in zip(m._mlp.weights, m._mlp.biases)])
    rhos = torch.cat([torch.cat([rw.reshape(-1), rb]) for rw, rb in m._post_rho])
    assert locs.numel() == rhos.numel() == 3 * 10 + 10 + 10 * P + P
    for v in (locs, rhos):
        assert abs(float(v.std()) - 0.05) < 0.01 and abs(float(v.mean())) < 0.01
    sc = m.posterior_scales()
    assert all(((s - 1.001).abs() < 0.01).all() for pair in sc for s in pair)
    mm = BayesNormalizingFlowNetwork(n_dims=1, n_flows=2, map_mode=True, n_dims_x=2)
    assert mm._post_rho is None and mm.posterior_scales() is None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from normalizingflownetwork_amd.parallel import allreduce_sum_count, init_from_env

    init_from_env(backend="gloo")
    buf = allreduce_sum_count(torch.tensor(1.5 + rank, dtype=torch.float64), 10 + rank,
                              local_nonfinite=torch.tensor(float(rank + 2), dtype=torch.float64))
    q.put((rank, buf.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_carries_nonfinite_count_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, buf in res:
        assert buf == [4.0, 21.0, 5.0]
