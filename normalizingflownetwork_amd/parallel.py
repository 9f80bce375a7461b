"""Batch-axis data parallelism for the mean log-likelihood.

Samples are independent (``DistributionLayers.py:245-255`` has no cross-sample
op), so every rank owns a contiguous slice of the batch, evaluates it with the
fused kernel, and the ONLY collective is one all-reduce of ``(sum log_prob,
count)`` in fp64 (16 bytes) — the distributed form of ``score``'s ``.mean()``
(``BaseEstimator.py:47``, ``scorers.py:34``).  On MI355X the process group is
``nccl`` (= RCCL over xGMI); ``gloo`` works for CPU-side tests.
"""

from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import ops


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced ``[start, stop)`` slice of ``n`` samples for ``rank``."""
    assert world >= 1 and 0 <= rank < world
    base, rem = divmod(int(n), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def allreduce_sum_count(local_sum: torch.Tensor, local_count: int, group=None) -> torch.Tensor:
    """All-reduce ``[sum, count]`` (fp64) across the group; returns the reduced pair.

    The buffer lives where the backend needs it (device for nccl/RCCL, host for gloo)."""
    backend = dist.get_backend(group) if dist.is_initialized() else None
    dev = local_sum.device if backend == "nccl" else torch.device("cpu")
    buf = torch.empty((2,), dtype=torch.float64, device=dev)
    buf[0] = local_sum.reshape(()).to(device=dev, dtype=torch.float64)
    buf[1] = float(local_count)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def mean_log_prob(
    y_shard, t_shard, flow_types: Sequence[str], n_dims: int, trainable_base: bool,
    y_mean=None, y_std=None, group=None,
) -> torch.Tensor:
    """Mean of ``log_prob`` over the union of all ranks' shards (fp64, on every rank)."""
    _, s = ops.chain_log_prob(y_shard, t_shard, flow_types, n_dims, trainable_base, y_mean, y_std,
                              want_values=False, want_sum=True)
    count = max(int(ops.as_device_f32(y_shard).reshape(-1, n_dims).shape[0]),
                int(ops.as_device_f32(t_shard).shape[0]) if ops.total_param_size(flow_types, n_dims,
                                                                                  trainable_base) else 0)
    buf = allreduce_sum_count(s, count, group)
    return buf[0] / buf[1]


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun's env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Returns ``(rank, world, local_rank)``."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend)
    return rank, world, local_rank
