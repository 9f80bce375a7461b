"""Batch-axis data parallelism for the mean log-likelihood.

Samples are independent (``DistributionLayers.py:245-255`` has no cross-sample
op), so every rank owns a contiguous slice of the batch, evaluates it with the
fused kernel, and the ONLY collective is one all-reduce of ``(sum log_prob,
count, non-finite count)`` in fp64 (24 bytes) — the distributed form of ``score``'s ``.mean()``
(``BaseEstimator.py:47``, ``scorers.py:34``).  On MI355X the process group is
``nccl`` (= RCCL over xGMI); ``gloo`` works for CPU-side tests.

Two interchangeable forms of that all-reduce: ``allreduce_sum_count`` through
``torch.distributed``, and ``NativeComm`` — the library's own RCCL communicator
behind the C ABI (``nfn_comm_init`` / ``nfn_allreduce_mean``, include/nfn.h),
stream-ordered on the device with no host round trip.
"""

from __future__ import annotations

import ctypes
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


def allreduce_sum_count(local_sum: torch.Tensor, local_count: int, group=None,
                        local_nonfinite: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-reduce ``[sum, count, non-finite count]`` (fp64) across the group; returns the
    reduced triple.  The buffer lives where the backend needs it (device for nccl/RCCL,
    host for gloo)."""
    backend = dist.get_backend(group) if dist.is_initialized() else None
    dev = local_sum.device if backend == "nccl" else torch.device("cpu")
    buf = torch.zeros((3,), dtype=torch.float64, device=dev)
    buf[0] = local_sum.reshape(()).to(device=dev, dtype=torch.float64)
    buf[1] = float(local_count)
    if local_nonfinite is not None:
        buf[2] = local_nonfinite.reshape(()).to(device=dev, dtype=torch.float64)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def mean_log_prob(
    y_shard, t_shard, flow_types: Sequence[str], n_dims: int, trainable_base: bool,
    y_mean=None, y_std=None, group=None,
) -> torch.Tensor:
    """Mean of ``log_prob`` over the union of all ranks' shards (fp64, on every rank).
    Non-finite log-densities propagate into the mean as in the reference's ``.mean()``;
    :func:`mean_log_prob_nonfinite` also returns their global count."""
    return mean_log_prob_nonfinite(y_shard, t_shard, flow_types, n_dims, trainable_base, y_mean, y_std, group)[0]


def mean_log_prob_nonfinite(
    y_shard, t_shard, flow_types: Sequence[str], n_dims: int, trainable_base: bool,
    y_mean=None, y_std=None, group=None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(mean log_prob, global non-finite count)`` over the union of all ranks' shards."""
    _, s, nf = ops.chain_log_prob(y_shard, t_shard, flow_types, n_dims, trainable_base, y_mean, y_std,
                                  want_values=False, want_sum=True, want_nonfinite=True)
    count = max(int(ops.as_device_f32(y_shard).reshape(-1, n_dims).shape[0]),
                int(ops.as_device_f32(t_shard).shape[0]) if ops.total_param_size(flow_types, n_dims,
                                                                                  trainable_base) else 0)
    buf = allreduce_sum_count(s, count, group, local_nonfinite=nf)
    return buf[0] / buf[1], buf[2]


class NativeComm:
    """RCCL communicator owned by ``libnfn_hip.so`` (one per process / GPU).

    The 128-byte rendezvous id is made on rank 0 and distributed over the
    existing ``torch.distributed`` group (any backend); without an initialised
    group the communicator has one rank.  Binds the current HIP device."""

    def __init__(self, group=None):
        from . import _lib

        self._lib = _lib.load()
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = (ctypes.c_uint8 * _lib.NFN_COMM_ID_BYTES)()
        if self.rank == 0:
            _lib.check(self._lib.nfn_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)), "nfn_comm_unique_id")
        if self.world > 1:
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0, group=group)
            uid = (ctypes.c_uint8 * _lib.NFN_COMM_ID_BYTES).from_buffer_copy(box[0])
        handle = ctypes.c_void_p()
        _lib.check(self._lib.nfn_comm_init(ctypes.byref(handle), self.world, ctypes.cast(uid, ctypes.c_void_p),
                                           self.rank), "nfn_comm_init")
        self.handle = handle
        dev = torch.device("cuda", torch.cuda.current_device())
        self.sum_count = torch.zeros((3,), dtype=torch.float64, device=dev)  # sum, count, non-finite
        self.mean = torch.zeros((1,), dtype=torch.float64, device=dev)

    def allreduce_mean(self, local_sum: torch.Tensor, local_count: int, stream=None) -> torch.Tensor:
        """``local_sum`` = the kernel's (2,) fp64 {sum, non-finite count} (``out_sum``);
        ``{sum, count, non-finite}`` summed over ranks into ``self.sum_count``; returns the
        device scalar ``sum / count`` (``self.mean``).  Stream-ordered."""
        from . import _lib

        assert local_sum.dtype == torch.float64 and local_sum.is_cuda and local_sum.numel() == 2
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        _lib.check(self._lib.nfn_allreduce_mean(self.handle, local_sum.data_ptr(), int(local_count),
                                                self.sum_count.data_ptr(), self.mean.data_ptr(), int(stream)),
                   "nfn_allreduce_mean")
        return self.mean

    def close(self) -> None:
        from . import _lib

        if self.handle:
            _lib.check(self._lib.nfn_comm_destroy(self.handle), "nfn_comm_destroy")
            self.handle = ctypes.c_void_p()


def init_from_env(backend: Optional[str] = None, force: bool = False) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun's env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT) when there is more than one rank (or ``force``).
    Returns ``(rank, world, local_rank)``."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if force and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend)
    return rank, world, local_rank
