"""Multi-process (world_size 2, gloo, CPU) check of the batch-sharded mean
log-likelihood reduction: every rank sums its shard (here with the oracle, the
stand-in for the kernel's fp64 partial sum), all-reduces (sum, count), and the
mean equals the single-process mean (BaseEstimator.py:47)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, load_golden


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from normalizingflownetwork_amd.parallel import allreduce_sum_count, init_from_env, shard_bounds
    from oracle import nfn_oracle as O

    r, w, _ = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    g = load_golden("c2_pr5_d1")
    n = g["t"].shape[0]
    a, b = shard_bounds(n, rank, world)
    local = O.chain_log_prob(g["y"][a:b], g["t"][a:b], g["flow_types"], 1, True, np.float64)
    buf = allreduce_sum_count(torch.tensor(local.sum(), dtype=torch.float64), b - a)
    q.put((rank, float(buf[0]), float(buf[1])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_mean_allreduce_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = load_golden("c2_pr5_d1")
    total = g["ref64"].sum()
    for _, s, c in res:
        assert c == g["t"].shape[0]
        assert s == pytest.approx(total, rel=1e-12)
