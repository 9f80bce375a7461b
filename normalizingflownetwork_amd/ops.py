"""Device-side entry points: torch device tensors in, HIP kernels via the C ABI.

Every function here launches a kernel from ``libnfn_hip.so`` on torch's
current HIP stream; torch provides only device memory and the stream handle.
There is no CPU fallback — without a GPU these raise ``RuntimeError``.
"""

from __future__ import annotations

import collections
import ctypes
import threading
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib

FLOW_IDS = {"planar": 0, "radial": 1, "affine": 2}

def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("normalizingflownetwork_amd needs a HIP device (MI355X); none is visible")
    return torch.device("cuda", torch.cuda.current_device())


def as_device_f32(x, device: Optional[torch.device] = None) -> torch.Tensor:
    """Convert array-likes / tensors to a float32 device tensor whose last dim is contiguous."""
    dev = device or _device()
    if isinstance(x, torch.Tensor):
        t = x.to(device=dev, dtype=torch.float32)
    else:
        t = torch.as_tensor(np.asarray(x, dtype=np.float32), device=dev)
    if t.dim() >= 1 and t.shape[-1] > 1 and t.stride(-1) != 1:
        t = t.contiguous()
    return t


def _row_stride(x: torch.Tensor) -> int:
    """Batch stride in elements of a (N, W) tensor; 0 broadcasts a single row."""
    return 0 if x.shape[0] == 1 else int(x.stride(0))


def _stream() -> int:
    return int(torch.cuda.current_stream().cuda_stream)


def _ptr(x: Optional[torch.Tensor]) -> Optional[int]:
    return None if x is None else int(x.data_ptr())


def flow_ids(flow_types: Sequence[str]):
    for f in flow_types:
        assert f in FLOW_IDS, f"unknown flow type {f!r}"  # DistributionLayers.py:231
    ids = (ctypes.c_int32 * max(1, len(flow_types)))(*[FLOW_IDS[f] for f in flow_types])
    return ids, len(flow_types)


def param_size(flow_type: str, n_dims: int) -> int:
    """Host metadata, same as the C ABI's ``nfn_param_size``: ``PlanarFlow.py:35-41`` (2d+1),
    ``RadialFlow.py:36-42`` (d+2), ``AffineFlow.py:11-17`` (2d)."""
    assert flow_type in FLOW_IDS, f"unknown flow type {flow_type!r}"
    return {"planar": 2 * n_dims + 1, "radial": n_dims + 2, "affine": 2 * n_dims}[flow_type]


def total_param_size(flow_types: Sequence[str], n_dims: int, trainable_base: bool) -> int:
    """``InverseNormalizingFlowLayer.get_total_param_size`` (``DistributionLayers.py:257-265``)."""
    return sum(param_size(f, n_dims) for f in flow_types) + (2 * n_dims if trainable_base else 0)


_workspaces: "collections.OrderedDict" = collections.OrderedDict()
_ws_lock = threading.Lock()
# (device, stream) workspaces kept at once; the least recently used is dropped beyond
# this (pooled / side streams come and go: fit's capture stream, the bench's ring).
WORKSPACE_CACHE_ENTRIES = 8
# Workspaces a captured HIP graph may hold the address of: handed out while their stream
# was capturing, as (pin sequence number, (device, stream) key, workspace).  A graph's replays
# write partials and the ticket there, so the block must not go back to the allocator while
# the graph lives.  Graphs do not tell when they die: an entry stays pinned for the life of
# the process unless the capturing code takes it over (``graph_pin_mark`` before the capture,
# ``take_graph_workspaces`` after it) and keeps it next to its graph, as ``estimators.fit``
# does.  Stream handles are pooled and reused, so a take is scoped by the mark, not only by
# the stream: pins made before the mark (another live graph's) stay where they are.
_graph_workspaces: list = []
_pin_seq = 0


def graph_pin_mark() -> int:
    """The pin sequence number before a capture: ``take_graph_workspaces(stream, mark)`` then
    hands back exactly the workspaces that capture pinned."""
    with _ws_lock:
        return _pin_seq


def take_graph_workspaces(stream, since: int) -> list:
    """Unpin and return the workspaces pinned on ``stream`` (a torch stream) since ``since``
    (a ``graph_pin_mark()``): the caller keeps them alive exactly as long as the graph
    captured there.  Pins made before the mark, on this stream handle or any other, stay."""
    key = (stream.device.index, int(stream.cuda_stream))
    with _ws_lock:
        return _take_pins(key, since)


def _take_pins(key, since: int) -> list:
    mine = [ws for seq, k, ws in _graph_workspaces if k == key and seq >= since]
    _graph_workspaces[:] = [(seq, k, ws) for seq, k, ws in _graph_workspaces if not (k == key and seq >= since)]
    return mine


def _pin(key, ws) -> None:
    """Pin ``ws`` for a capture on ``key`` (caller holds ``_ws_lock``).  A block already pinned
    by an earlier capture that nobody took stays pinned for the process: not pinned again."""
    global _pin_seq
    if not any(p is ws for _, _, p in _graph_workspaces):
        _graph_workspaces.append((_pin_seq, key, ws))
        _pin_seq += 1


def _workspace(n_doubles: int, device: torch.device) -> torch.Tensor:
    """The workspace of the current (device, stream): calls are ordered on their stream,
    so calls in flight on different streams never share partials, the posterior's split
    region or the finishing ticket.  No initialisation is needed (ABI 200: the ticket
    carries a per-call epoch).  Dropping (or outgrowing) an entry that no graph captured
    is safe: its memory returns to the caching allocator's pool of the SAME stream, so a
    later allocation that reuses it is ordered after the calls that used it.  An entry
    used during a capture is pinned instead (``_graph_workspaces``): the graph keeps its
    address, and eager warm-up calls on the capture stream commonly allocate it first."""
    stream = torch.cuda.current_stream(device)
    key = (device.index, int(stream.cuda_stream))
    capturing = torch.cuda.is_current_stream_capturing()
    with _ws_lock:
        ws = _workspaces.get(key)
        if ws is None or ws.numel() < n_doubles:
            ws = torch.empty(max(2, n_doubles), dtype=torch.float64, device=device)
        if capturing:
            _pin(key, ws)
        _workspaces[key] = ws
        _workspaces.move_to_end(key)
        while len(_workspaces) > WORKSPACE_CACHE_ENTRIES:
            _workspaces.popitem(last=False)
        return ws


def _with_nonfinite(out, osum, want_nonfinite: bool):
    """``(out, sum)`` or, with ``want_nonfinite``, ``(out, sum, nonfinite)``: ``osum`` is the
    kernel's (2,) fp64 {sum, non-finite count}; ``nonfinite`` counts the inf / NaN values
    among the summed log-densities (next to the partial sums in the kernel; SURVEY.md §5,
    the reference's ``TerminateOnNaN``, ``BaseEstimator.py:29``)."""
    s = None if osum is None else osum[0:1]
    if not want_nonfinite:
        return out, s
    return out, s, osum[1:2]


def _prep_2d(x, width: int, name: str, device) -> torch.Tensor:
    x = as_device_f32(x, device)
    if x.dim() == 1:
        x = x.unsqueeze(0)
    assert x.dim() == 2, f"{name} must be 2-D (batch, {width}), got shape {tuple(x.shape)}"
    assert x.shape[-1] == width, f"{name} last dimension must be {width}, got {x.shape[-1]}"
    return x


def chain_log_prob(
    y,
    t,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
    want_values: bool = True,
    want_sum: bool = False,
    want_nonfinite: bool = False,
):
    """Fused ``log_prob(y | t)`` over the whole flow chain (one kernel launch).

    Returns ``(log_prob (B,) float32 | None, sum (1,) float64 | None)``, plus the
    non-finite count (1,) fp64 when ``want_nonfinite`` (implies ``want_sum``).
    With ``y_mean``/``y_std`` it is ``BaseEstimator.log_pdf``'s
    ``log_prob((y-mu)/sigma) - sum(log sigma)`` (``BaseEstimator.py:77-86``).
    """
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    y = _prep_2d(y, n_dims, "y", dev)
    t = _prep_2d(t, P, "t", dev) if P > 0 else torch.zeros((1, 1), dtype=torch.float32, device=dev)
    B = max(y.shape[0], t.shape[0] if P > 0 else 1)
    assert y.shape[0] in (1, B) and (P == 0 or t.shape[0] in (1, B)), "incompatible batch sizes"
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
        assert ym.numel() == n_dims and ys.numel() == n_dims
    want_sum = want_sum or want_nonfinite
    out = torch.empty((B,), dtype=torch.float32, device=dev) if want_values else None
    osum = torch.empty((2,), dtype=torch.float64, device=dev) if want_sum else None
    lib = _lib.load()
    ws = _workspace(int(lib.nfn_chain_workspace_doubles(B, n_dims, P)), dev) if want_sum else None
    ids, k = flow_ids(flow_types)
    rc = lib.nfn_chain_logprob_f32(
        _ptr(y), _row_stride(y), _ptr(t), _row_stride(t) if P > 0 else 0, B, int(n_dims),
        ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys),
        _ptr(out), _ptr(osum), _ptr(ws), _stream(),
    )
    _lib.check(rc, "nfn_chain_logprob_f32")
    return _with_nonfinite(out, osum, want_nonfinite)


def chain_log_prob_grad(
    y,
    t,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
    g_out=None,
    want_logp: bool = False,
    want_grad_t: bool = True,
    want_grad_y: bool = True,
):
    """Fused backward (one kernel): per sample ``dL/dt`` (B, P) and ``dL/dy`` (B, d) for
    ``L = sum_b g_out[b] * log_prob_b`` (``g_out`` None => ones), optionally ``log_prob``.

    What Keras autodiff computes through the reference's log_prob when it trains
    (``BaseEstimator.py:19-31, 55-59``).  A broadcast input (batch 1) still gets
    one gradient row per sample.  Returns ``(log_prob | None, grad_t | None, grad_y | None)``."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    y = _prep_2d(y, n_dims, "y", dev)
    t = _prep_2d(t, P, "t", dev) if P > 0 else torch.zeros((1, 1), dtype=torch.float32, device=dev)
    B = max(y.shape[0], t.shape[0] if P > 0 else 1)
    assert y.shape[0] in (1, B) and (P == 0 or t.shape[0] in (1, B)), "incompatible batch sizes"
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
        assert ym.numel() == n_dims and ys.numel() == n_dims
    g = None
    if g_out is not None:
        g = as_device_f32(g_out, dev).reshape(-1).contiguous()
        assert g.numel() == B, f"g_out must have {B} elements"
    lp = torch.empty((B,), dtype=torch.float32, device=dev) if want_logp else None
    gt = torch.empty((B, P), dtype=torch.float32, device=dev) if (want_grad_t and P > 0) else None
    gy = torch.empty((B, n_dims), dtype=torch.float32, device=dev) if want_grad_y else None
    ids, k = flow_ids(flow_types)
    rc = _lib.load().nfn_chain_logprob_grad_f32(
        _ptr(y), _row_stride(y), _ptr(t), _row_stride(t) if P > 0 else 0, B, int(n_dims),
        ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys), _ptr(g),
        _ptr(lp), _ptr(gt), P if gt is not None else 0, _ptr(gy), _stream(),
    )
    _lib.check(rc, "nfn_chain_logprob_grad_f32")
    if want_grad_t and gt is None:
        gt = torch.empty((B, 0), dtype=torch.float32, device=dev)
    return lp, gt, gy


class _ChainLogProb(torch.autograd.Function):
    """``log_prob`` as a differentiable op: forward = the fused forward kernel,
    backward = the fused backward kernel (the chain is recomputed there, nothing
    but the inputs is saved)."""

    @staticmethod
    def forward(ctx, y, t, flow_types, n_dims, trainable_base, y_mean, y_std):
        out, _ = chain_log_prob(y, t, flow_types, n_dims, trainable_base, y_mean, y_std)
        ctx.save_for_backward(y, t)
        ctx.meta = (tuple(flow_types), int(n_dims), bool(trainable_base), y_mean, y_std)
        return out

    @staticmethod
    def backward(ctx, g):
        y, t = ctx.saved_tensors
        flow_types, n_dims, trainable_base, y_mean, y_std = ctx.meta
        need_y, need_t = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        _, gt, gy = chain_log_prob_grad(y, t, flow_types, n_dims, trainable_base, y_mean, y_std,
                                        g_out=g.contiguous(), want_grad_t=need_t, want_grad_y=need_y)
        B = g.shape[0]
        if need_y and y.shape[0] == 1 and B > 1:
            gy = gy.sum(0, keepdim=True)
        if need_t and t.shape[0] == 1 and B > 1:
            gt = gt.sum(0, keepdim=True)
        return (gy if need_y else None), (gt if need_t else None), None, None, None, None, None


def log_prob(y, t, flow_types: Sequence[str], n_dims: int, trainable_base: bool, y_mean=None, y_std=None):
    """Differentiable fused ``log_prob`` (B,): gradients w.r.t. ``t`` and ``y`` flow
    through ``torch.autograd`` via the fused backward kernel."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    y = _prep_2d(y, n_dims, "y", dev)
    t = _prep_2d(t, P, "t", dev) if P > 0 else torch.zeros((1, 1), dtype=torch.float32, device=dev)
    if y_mean is not None:
        y_mean = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        y_std = as_device_f32(y_std, dev).reshape(-1).contiguous()
    return _ChainLogProb.apply(y, t, tuple(flow_types), int(n_dims), bool(trainable_base), y_mean, y_std)


class _DenseLogProb(torch.autograd.Function):
    """``log_prob(y | t = h W + b)`` as a differentiable op with the output Dense layer
    fused both ways: forward = ``nfn_chain_logprob_dense_f32``, backward =
    ``nfn_chain_logprob_dense_grad_f32`` (t is never materialised)."""

    @staticmethod
    def forward(ctx, y, h, W, b, flow_types, n_dims, trainable_base):
        out, _ = chain_log_prob_dense(y, h, W, b, flow_types, n_dims, trainable_base)
        ctx.save_for_backward(y, h, W, b)
        ctx.meta = (tuple(flow_types), int(n_dims), bool(trainable_base))
        return out

    @staticmethod
    def backward(ctx, g):
        y, h, W, b = ctx.saved_tensors
        flow_types, n_dims, trainable_base = ctx.meta
        _, gh, gW, gb, gy = chain_log_prob_dense_grad(y, h, W, b, flow_types, n_dims, trainable_base,
                                                      g_out=g.contiguous())
        if y.shape[0] == 1 and gh.shape[0] > 1:
            gy = gy.sum(0, keepdim=True)
        return gy, gh, gW, gb, None, None, None


def log_prob_dense(y, h, W, b, flow_types: Sequence[str], n_dims: int, trainable_base: bool):
    """Differentiable ``log_prob(y | h W + b)`` (B,) through the fused Dense layer: the
    gradients w.r.t. ``h``, ``W``, ``b`` (and ``y``) come from the fused backward kernel."""
    dev = _device()
    y = _prep_2d(y, n_dims, "y", dev)
    h = as_device_f32(h, dev).contiguous()
    return _DenseLogProb.apply(y, h, as_device_f32(W, dev), as_device_f32(b, dev), tuple(flow_types), int(n_dims),
                               bool(trainable_base))


DENSE_HIDDEN_WIDTHS = (4, 8, 16, 32, 64)


def dense_fusable(H: int, P: int, n_dims: int) -> bool:
    """Shapes the fused Dense->chain kernel takes (include/nfn.h, nfn_chain_logprob_dense_f32)."""
    return H in DENSE_HIDDEN_WIDTHS and 1 <= P <= 64 and n_dims <= 8


def chain_log_prob_dense(
    y,
    h,
    W,
    b,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
    want_values: bool = True,
    want_sum: bool = False,
    want_nonfinite: bool = False,
):
    """``log_prob(y | t = h W + b)`` with the estimator's output Dense layer
    (``MaximumLikelihoodNNEstimator.py:37-44``) fused into the chain kernel: ``h`` (B, H) last
    hidden activations, ``W`` (H, P), ``b`` (P,).  Shapes the fused kernel does not take run
    as a library GEMM (torch) followed by the chain kernel."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    h = as_device_f32(h, dev)
    assert h.dim() == 2, "h must be (B, H)"
    H = int(h.shape[1])
    W = as_device_f32(W, dev).contiguous()
    assert tuple(W.shape) == (H, P), f"W must be ({H}, {P})"
    bb = None if b is None else as_device_f32(b, dev).reshape(-1).contiguous()
    if not dense_fusable(H, P, n_dims) or h.stride(0) % 4 or h.data_ptr() % 16:
        t = h @ W + (bb if bb is not None else 0.0)
        return chain_log_prob(y, t, flow_types, n_dims, trainable_base, y_mean, y_std, want_values, want_sum,
                              want_nonfinite)
    y = _prep_2d(y, n_dims, "y", dev)
    B = int(h.shape[0])
    assert y.shape[0] in (1, B), "incompatible batch sizes"
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
    want_sum = want_sum or want_nonfinite
    out = torch.empty((B,), dtype=torch.float32, device=dev) if want_values else None
    osum = torch.empty((2,), dtype=torch.float64, device=dev) if want_sum else None
    lib = _lib.load()
    ws = _workspace(int(lib.nfn_chain_workspace_doubles(B, n_dims, P)), dev) if want_sum else None
    ids, k = flow_ids(flow_types)
    rc = lib.nfn_chain_logprob_dense_f32(
        _ptr(y), _row_stride(y), _ptr(h), int(h.stride(0)), H, _ptr(W), _ptr(bb), B, int(n_dims),
        ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys), _ptr(out), _ptr(osum),
        _ptr(ws), _stream(),
    )
    _lib.check(rc, "nfn_chain_logprob_dense_f32")
    return _with_nonfinite(out, osum, want_nonfinite)


def chain_log_prob_dense_grad(
    y,
    h,
    W,
    b,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
    g_out=None,
    want_logp: bool = False,
):
    """Backward of :func:`chain_log_prob_dense` (one fused kernel + a fixed-order reduction):
    for ``L = sum_b g_out[b] * log_prob_b`` returns ``(log_prob | None, dL/dh (B, H),
    dL/dW (H, P), dL/db (P,), dL/dy (B, d))`` — what Keras autodiff takes through the output
    ``Dense(P)`` and the layer's ``log_prob`` when the reference trains
    (``MaximumLikelihoodNNEstimator.py:37-44``, ``BaseEstimator.py:19-31``), with ``t`` never
    materialised.  Shapes the fused kernel does not take run as library GEMMs around
    :func:`chain_log_prob_grad`."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    h = as_device_f32(h, dev)
    assert h.dim() == 2, "h must be (B, H)"
    B, H = int(h.shape[0]), int(h.shape[1])
    W = as_device_f32(W, dev).contiguous()
    assert tuple(W.shape) == (H, P), f"W must be ({H}, {P})"
    bb = None if b is None else as_device_f32(b, dev).reshape(-1).contiguous()
    y = _prep_2d(y, n_dims, "y", dev)
    assert y.shape[0] in (1, B), "incompatible batch sizes"
    g = None
    if g_out is not None:
        g = as_device_f32(g_out, dev).reshape(-1).contiguous()
        assert g.numel() == B, f"g_out must have {B} elements"
    lib = _lib.load()
    rc = _lib.NFN_E_SHAPE
    if dense_fusable(H, P, n_dims) and h.stride(0) % 4 == 0 and h.data_ptr() % 16 == 0:
        ym = ys = None
        if y_mean is not None:
            ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
            ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
        lp = torch.empty((B,), dtype=torch.float32, device=dev) if want_logp else None
        gh = torch.empty((B, H), dtype=torch.float32, device=dev)
        gW = torch.empty((H, P), dtype=torch.float32, device=dev)
        gb = torch.empty((P,), dtype=torch.float32, device=dev)
        gy = torch.empty((B, n_dims), dtype=torch.float32, device=dev)
        ws = torch.empty((max(1, int(lib.nfn_dense_grad_workspace_floats(B, H, P))),), dtype=torch.float32,
                         device=dev)
        ids, k = flow_ids(flow_types)
        rc = lib.nfn_chain_logprob_dense_grad_f32(
            _ptr(y), _row_stride(y), _ptr(h), int(h.stride(0)), H, _ptr(W), _ptr(bb), B, int(n_dims),
            ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys), _ptr(g), _ptr(lp),
            _ptr(gh), H, _ptr(gW), _ptr(gb), _ptr(gy), _ptr(ws), _stream(),
        )
        if rc == 0:
            return lp, gh, gW, gb, gy
        if rc != _lib.NFN_E_SHAPE:
            _lib.check(rc, "nfn_chain_logprob_dense_grad_f32")
    # unfused: t by the library GEMM, the chain backward kernel, library GEMMs for dh / dW / db
    t = h @ W + (bb if bb is not None else 0.0)
    lp, gt, gy = chain_log_prob_grad(y, t, flow_types, n_dims, trainable_base, y_mean, y_std, g, want_logp)
    return lp, gt @ W.t(), h.t() @ gt, gt.sum(0), gy


def posterior_lse_dense(
    y,
    h,
    W,
    b,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
    want_values: bool = True,
    want_sum: bool = False,
    want_nonfinite: bool = False,
):
    """Bayesian posterior score per sample with the output DenseVariational layer fused
    (``BayesianNNEstimator.py:65-76`` score over draws, ``:136-145`` the variational output
    layer): ``logsumexp_s log_prob(y | h_s W_s + b_s) - log S``.  ``h``: (S, B, H) per-draw
    last hidden activations, or (B, H) shared by every draw; ``W``: (S, H, P); ``b``: (S, P)
    or None.  Shapes the fused kernel does not take run as a library GEMM (torch) followed
    by :func:`posterior_lse`."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    h = as_device_f32(h, dev)
    W = as_device_f32(W, dev).contiguous()
    assert W.dim() == 3 and W.shape[2] == P, f"W must be (S, H, {P})"
    S, H = int(W.shape[0]), int(W.shape[1])
    assert h.dim() in (2, 3) and h.shape[-1] == H, f"h must be (S, B, {H}) or (B, {H})"
    if h.dim() == 3:
        assert h.shape[0] == S, "h and W disagree on the number of draws"
    bb = None
    if b is not None:
        bb = as_device_f32(b, dev).reshape(S, P).contiguous()
    B = int(h.shape[-2])
    hrow = int(h.stride(-2))
    hdraw = int(h.stride(0)) if h.dim() == 3 else 0
    aligned = h.stride(-1) == 1 and hrow % 4 == 0 and hdraw % 4 == 0 and h.data_ptr() % 16 == 0
    if h.dim() == 3 and S > 1 and hdraw < B * hrow:
        aligned = False
    if not dense_fusable(H, P, n_dims) or not aligned:
        hd = h if h.dim() == 3 else h.unsqueeze(0).expand(S, B, H)
        t = torch.matmul(hd, W) + (bb.unsqueeze(1) if bb is not None else 0.0)
        return posterior_lse(y, t, flow_types, n_dims, trainable_base, y_mean, y_std, want_values, want_sum,
                             want_nonfinite)
    y = _prep_2d(y, n_dims, "y", dev)
    assert y.shape[0] in (1, B), "incompatible batch sizes"
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
    want_sum = want_sum or want_nonfinite
    out = torch.empty((B,), dtype=torch.float32, device=dev) if want_values else None
    osum = torch.empty((2,), dtype=torch.float64, device=dev) if want_sum else None
    lib = _lib.load()
    ws = _workspace(int(lib.nfn_chain_workspace_doubles(B, n_dims, P)), dev) if want_sum else None
    ids, k = flow_ids(flow_types)
    rc = lib.nfn_posterior_lse_dense_f32(
        _ptr(y), _row_stride(y), _ptr(h), hdraw, hrow, H, _ptr(W), H * P, _ptr(bb), P, S, B, int(n_dims),
        ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys), _ptr(out), _ptr(osum),
        _ptr(ws), _stream(),
    )
    _lib.check(rc, "nfn_posterior_lse_dense_f32")
    return _with_nonfinite(out, osum, want_nonfinite)


class DenseLauncher:
    """Pre-bound fused Dense->chain launch over fixed device buffers (benchmark loop)."""

    def __init__(self, y: torch.Tensor, h: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor],
                 flow_types: Sequence[str], n_dims: int, trainable_base: bool, write_values: bool = True):
        self.lib = _lib.load()
        dev = y.device
        self.n_dims = int(n_dims)
        self.P = total_param_size(flow_types, n_dims, trainable_base)
        self.B, self.H = int(h.shape[0]), int(h.shape[1])
        assert dense_fusable(self.H, self.P, self.n_dims) and h.stride(1) == 1 and tuple(W.shape) == (self.H, self.P)
        self.y, self.h, self.W, self.b = y, h, W.contiguous(), b
        self.out = torch.empty((self.B,), dtype=torch.float32, device=dev) if write_values else None
        self.sum2 = torch.zeros((2,), dtype=torch.float64, device=dev)  # {sum, non-finite}
        self.sum = self.sum2[0:1]
        self.partials = torch.zeros((max(2, int(self.lib.nfn_chain_workspace_doubles(self.B, self.n_dims, self.P))),),
                                    dtype=torch.float64, device=dev)
        self._ids, self._k = flow_ids(flow_types)
        self._args = (
            _ptr(y), _row_stride(y), _ptr(h), int(h.stride(0)), self.H, _ptr(self.W), _ptr(b), self.B, self.n_dims,
            ctypes.cast(self._ids, ctypes.c_void_p), self._k, int(bool(trainable_base)), None, None, _ptr(self.out),
            _ptr(self.sum2), _ptr(self.partials),
        )

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self.lib.nfn_chain_logprob_dense_f32(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "nfn_chain_logprob_dense_f32")

    def finish_sum(self, stream: Optional[int] = None) -> torch.Tensor:
        """The launch's fp64 sum (finished inside the kernel: nothing to launch)."""
        return self.sum

    @property
    def nonfinite(self) -> torch.Tensor:
        """(1,) fp64: non-finite values among the last launch's log-densities."""
        return self.sum2[1:2]


class PosteriorDenseLauncher(DenseLauncher):
    """Pre-bound fused DenseVariational->posterior launch (``nfn_posterior_lse_dense_f32``):
    ``h`` (S, B, H), ``W`` (S, H, P), ``b`` (S, P) or None."""

    def __init__(self, y: torch.Tensor, h: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor],
                 flow_types: Sequence[str], n_dims: int, trainable_base: bool, write_values: bool = True):
        self.lib = _lib.load()
        dev = y.device
        self.n_dims = int(n_dims)
        self.P = total_param_size(flow_types, n_dims, trainable_base)
        self.S, self.B, self.H = (int(v) for v in h.shape)
        assert dense_fusable(self.H, self.P, self.n_dims) and h.is_contiguous()
        assert tuple(W.shape) == (self.S, self.H, self.P) and (b is None or tuple(b.shape) == (self.S, self.P))
        self.y, self.h, self.W = y, h, W.contiguous()
        self.b = None if b is None else b.contiguous()
        self.out = torch.empty((self.B,), dtype=torch.float32, device=dev) if write_values else None
        self.sum2 = torch.zeros((2,), dtype=torch.float64, device=dev)  # {sum, non-finite}
        self.sum = self.sum2[0:1]
        self.partials = torch.zeros((max(2, int(self.lib.nfn_chain_workspace_doubles(self.B, self.n_dims, self.P))),),
                                    dtype=torch.float64, device=dev)
        self._ids, self._k = flow_ids(flow_types)
        self._args = (
            _ptr(y), _row_stride(y), _ptr(h), int(h.stride(0)), int(h.stride(1)), self.H, _ptr(self.W),
            self.H * self.P, _ptr(self.b), self.P, self.S, self.B, self.n_dims, ctypes.cast(self._ids, ctypes.c_void_p),
            self._k, int(bool(trainable_base)), None, None, _ptr(self.out), _ptr(self.sum2), _ptr(self.partials),
        )

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self.lib.nfn_posterior_lse_dense_f32(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "nfn_posterior_lse_dense_f32")


def chain_sample(eps, t, flow_types: Sequence[str], n_dims: int, trainable_base: bool, y_mean=None, y_std=None,
                 want_log_prob: bool = True):
    """Draw ``y ~ p(y | t)`` through the inverted flows for given standard-normal ``eps``
    (B or 1, d): returns ``(y (B, d), log_prob (B,) | None)`` (``nfn_chain_sample_f32``).
    A capability the reference lacks (its flows define no inverse)."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    e = _prep_2d(eps, n_dims, "eps", dev)
    t = _prep_2d(t, P, "t", dev) if P > 0 else torch.zeros((1, 1), dtype=torch.float32, device=dev)
    B = max(int(e.shape[0]), int(t.shape[0]) if P > 0 else 1)
    assert e.shape[0] in (1, B) and (P == 0 or t.shape[0] in (1, B)), "incompatible batch sizes"
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
    y = torch.empty((B, n_dims), dtype=torch.float32, device=dev)
    lp = torch.empty((B,), dtype=torch.float32, device=dev) if want_log_prob else None
    ids, k = flow_ids(flow_types)
    rc = _lib.load().nfn_chain_sample_f32(
        _ptr(e), _row_stride(e), _ptr(t), _row_stride(t) if P > 0 else 0, B, int(n_dims),
        ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys), _ptr(y), _ptr(lp),
        _stream(),
    )
    _lib.check(rc, "nfn_chain_sample_f32")
    return y, lp


def chain_log_prob_grid(
    y_grid,
    t,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
) -> torch.Tensor:
    """``log_prob`` of every grid value ``y_grid[g]`` (G, d) under every parameter row
    ``t[b]`` (B, P): returns (G, B) — the density-grid evaluation of
    ``flow_plotting.plot_model`` (``evaluation/visualization/flow_plotting.py:33-53``) in
    one kernel."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    yg = _prep_2d(y_grid, n_dims, "y_grid", dev)
    t = _prep_2d(t, P, "t", dev) if P > 0 else torch.zeros((1, 1), dtype=torch.float32, device=dev)
    G = int(yg.shape[0])
    B = int(t.shape[0]) if P > 0 else 1
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
        assert ym.numel() == n_dims and ys.numel() == n_dims
    out = torch.empty((G, B), dtype=torch.float32, device=dev)
    ids, k = flow_ids(flow_types)
    rc = _lib.load().nfn_chain_logprob_grid_f32(
        _ptr(yg), int(yg.stride(0)) if G > 1 else 0, G, _ptr(t), _row_stride(t) if P > 0 else 0, B, int(n_dims),
        ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys), _ptr(out), B,
        _stream(),
    )
    _lib.check(rc, "nfn_chain_logprob_grid_f32")
    return out


def flow_forward_ldj(flow_type: str, z, t_k, n_dims: int, want_z: bool = True, want_ldj: bool = True):
    """One bijector: ``(forward(z), forward_log_det_jacobian(z))`` (either may be None)."""
    dev = _device()
    ps = param_size(flow_type, n_dims)
    z = _prep_2d(z, n_dims, "z", dev)
    t_k = as_device_f32(t_k, dev)
    if t_k.dim() == 1:
        t_k = t_k.unsqueeze(0)
    assert t_k.shape[-1] == ps, f"{flow_type} flow needs {ps} params, got {t_k.shape[-1]}"
    B = max(z.shape[0], t_k.shape[0])
    assert z.shape[0] in (1, B) and t_k.shape[0] in (1, B), "incompatible batch sizes"
    z_out = torch.empty((B, n_dims), dtype=torch.float32, device=dev) if want_z else None
    ldj = torch.empty((B,), dtype=torch.float32, device=dev) if want_ldj else None
    lib = _lib.load()
    rc = lib.nfn_flow_fwd_ldj_f32(
        FLOW_IDS[flow_type], _ptr(z), _row_stride(z), _ptr(t_k), _row_stride(t_k), B, int(n_dims),
        _ptr(z_out), _ptr(ldj), _stream(),
    )
    _lib.check(rc, "nfn_flow_fwd_ldj_f32")
    return z_out, ldj


def flow_vjp(flow_type: str, z: torch.Tensor, t_k: torch.Tensor, n_dims: int, g_z=None, g_ldj=None,
             want_dz: bool = True, want_dt: bool = True):
    """One bijector's vector-Jacobian product (``nfn_flow_vjp_f32``): ``(dL/dz, dL/dt_k)``
    per sample, (B, d) and (B, p), for ``L = sum_b <g_z[b], f(z_b)> + g_ldj[b] fldj(z_b)``
    (``g_z`` / ``g_ldj`` None => zero).  ``z`` / ``t_k`` as ``flow_forward_ldj`` takes them."""
    dev = _device()
    ps = param_size(flow_type, n_dims)
    z = _prep_2d(z, n_dims, "z", dev)
    t_k = as_device_f32(t_k, dev)
    if t_k.dim() == 1:
        t_k = t_k.unsqueeze(0)
    assert t_k.shape[-1] == ps, f"{flow_type} flow needs {ps} params, got {t_k.shape[-1]}"
    B = max(z.shape[0], t_k.shape[0])
    assert z.shape[0] in (1, B) and t_k.shape[0] in (1, B), "incompatible batch sizes"
    gz = gl = None
    if g_z is not None:
        gz = as_device_f32(g_z, dev).expand(B, n_dims).contiguous()
    if g_ldj is not None:
        gl = as_device_f32(g_ldj, dev).reshape(-1).expand(B).contiguous()
    dz = torch.empty((B, n_dims), dtype=torch.float32, device=dev) if want_dz else None
    dt = torch.empty((B, ps), dtype=torch.float32, device=dev) if want_dt else None
    rc = _lib.load().nfn_flow_vjp_f32(
        FLOW_IDS[flow_type], _ptr(z), _row_stride(z), _ptr(t_k), _row_stride(t_k), B, int(n_dims), _ptr(gz), _ptr(gl),
        _ptr(dz), _ptr(dt), _stream(),
    )
    _lib.check(rc, "nfn_flow_vjp_f32")
    return dz, dt


class _FlowForwardLdj(torch.autograd.Function):
    """One bijector's ``(forward(z), forward_log_det_jacobian(z))`` as a differentiable op:
    forward = ``nfn_flow_fwd_ldj_f32``, backward = ``nfn_flow_vjp_f32`` (the flow is
    recomputed there from the saved inputs).  What TF's tape differentiates through
    ``PlanarFlow._forward`` / ``_forward_log_det_jacobian`` (``PlanarFlow.py:68-80``),
    ``RadialFlow.py:50-70`` and tfp ``Affine``."""

    @staticmethod
    def forward(ctx, z, t_k, flow_type, n_dims):
        ctx.set_materialize_grads(False)
        z_out, ldj = flow_forward_ldj(flow_type, z, t_k, n_dims)
        ctx.save_for_backward(z, t_k)
        ctx.meta = (flow_type, int(n_dims))
        return z_out, ldj

    @staticmethod
    def backward(ctx, g_z, g_ldj):
        z, t_k = ctx.saved_tensors
        flow_type, n_dims = ctx.meta
        need_z, need_t = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if (g_z is None and g_ldj is None) or not (need_z or need_t):
            return None, None, None, None
        dz, dt = flow_vjp(flow_type, z, t_k, n_dims, g_z, g_ldj, want_dz=need_z, want_dt=need_t)
        B = max(z.shape[0], t_k.shape[0])
        if need_z and z.shape[0] == 1 and B > 1:
            dz = dz.sum(0, keepdim=True)
        if need_t and t_k.shape[0] == 1 and B > 1:
            dt = dt.sum(0, keepdim=True)
        return dz, dt, None, None


def flow_forward_ldj_diff(flow_type: str, z, t_k, n_dims: int):
    """Differentiable ``(forward(z), forward_log_det_jacobian(z))`` of one bijector: gradients
    w.r.t. ``z`` and ``t_k`` flow through ``torch.autograd`` via ``nfn_flow_vjp_f32``."""
    dev = _device()
    z = _prep_2d(z, n_dims, "z", dev)
    t_k = as_device_f32(t_k, dev)
    if t_k.dim() == 1:
        t_k = t_k.unsqueeze(0)
    return _FlowForwardLdj.apply(z, t_k, flow_type, int(n_dims))


def split_pays(widths: Sequence[int], row_stride: int) -> bool:
    """Whether the flows' single launches should read one-pass contiguous copies of their
    blocks (``split_blocks``) rather than their strided views, by expected HBM bytes per
    sample: a view launch fetches the whole 128-B lines its block touches (about
    ``128 + 4 (w - 1)`` bytes for a block of w floats at a random offset), the split reads the
    row once and writes and re-reads the blocks (``4 row_stride + 8 sum(w)``).  The split must
    win by 30 % to pay for its own pass: C2's 3-float blocks of 32-float rows (368 vs 1360 B)
    take it, C3's 10-17-float blocks of 140-float rows (1552 vs 1612 B) do not (measured:
    1.43 vs 4.32 ms and 2.60 vs 2.02 ms, profiles/r03/r03s2_*, r03c3g_*; C3 reading the
    rows is 1.82 ms since, r03j_*)."""
    strided = sum(128 + 4 * (int(w) - 1) for w in widths)
    split = 4 * int(row_stride) + 8 * sum(int(w) for w in widths)
    return split < 0.7 * strided


def split_blocks(t: torch.Tensor, widths: Sequence[int]):
    """``[t[:, o_k:o_k + w_k].contiguous() for each block]`` in ONE pass over ``t``
    (``nfn_split_blocks_f32``): ``t`` (B, >= sum(widths)) device rows with unit column
    stride, the blocks consecutive from column 0.  The blocks are views of one allocation.
    What the TF slices of ``_get_bijector`` are (``DistributionLayers.py:267-278``: copies)."""
    assert isinstance(t, torch.Tensor) and t.dim() == 2 and t.stride(1) == 1, "t must be (B, W), unit column stride"
    widths = [int(w) for w in widths]
    B, W = int(t.shape[0]), sum(widths)
    assert t.shape[1] >= W, "t narrower than its blocks"
    buf = torch.empty((B * W,), dtype=torch.float32, device=t.device)
    arr = (ctypes.c_int32 * max(1, len(widths)))(*widths)
    rc = _lib.load().nfn_split_blocks_f32(_ptr(t), _row_stride(t), B, arr, len(widths), _ptr(buf), _stream())
    _lib.check(rc, "nfn_split_blocks_f32")
    out, off = [], 0
    for w in widths:
        out.append(buf[off:off + B * w].view(B, w))
        off += B * w
    return out


def chain_forward_ldj(flow_types: Sequence[str], z, t, block_offsets: Sequence[int], n_dims: int,
                      want_z: bool = True, want_ldj: bool = True):
    """A Chain of flows as ONE kernel launch (``nfn_chain_fwd_ldj_f32``): ``(z_K, sum_k
    log|det J_k|)`` for flows applied in ``flow_types`` order, flow k reading its block at
    column ``block_offsets[k]`` of each row of ``t`` (B or 1, >= span).  What tfp's
    ``Chain.forward`` / ``forward_log_det_jacobian`` compute over the layer's flows
    (``DistributionLayers.py:267-278``)."""
    dev = _device()
    z = _prep_2d(z, n_dims, "z", dev)
    t = as_device_f32(t, dev)
    if t.dim() == 1:
        t = t.unsqueeze(0)
    assert t.dim() == 2 and t.stride(1) == 1, "t must be (B, W) with unit column stride"
    ids, K = flow_ids(flow_types)
    assert len(block_offsets) == K, "one block offset per flow"
    offs = (ctypes.c_int32 * max(1, K))(*[int(o) for o in block_offsets])
    B = max(z.shape[0], t.shape[0])
    assert z.shape[0] in (1, B) and t.shape[0] in (1, B), "incompatible batch sizes"
    z_out = torch.empty((B, n_dims), dtype=torch.float32, device=dev) if want_z else None
    ldj = torch.empty((B,), dtype=torch.float32, device=dev) if want_ldj else None
    lib = _lib.load()
    rc = lib.nfn_chain_fwd_ldj_f32(_ptr(z), _row_stride(z), _ptr(t), _row_stride(t), B, int(n_dims), ids, offs, K,
                                   _ptr(z_out), _ptr(ldj), _stream())
    _lib.check(rc, "nfn_chain_fwd_ldj_f32")
    return z_out, ldj


def posterior_lse(
    y,
    t_draws,
    flow_types: Sequence[str],
    n_dims: int,
    trainable_base: bool,
    y_mean=None,
    y_std=None,
    want_values: bool = True,
    want_sum: bool = False,
    want_nonfinite: bool = False,
):
    """``logsumexp_s(log_pdf(y_b | t[s, b])) - log S`` per sample (``BayesianNNEstimator.py:65-76``).

    ``t_draws``: (S, B, P) device tensor (rows contiguous)."""
    dev = _device()
    P = total_param_size(flow_types, n_dims, trainable_base)
    y = _prep_2d(y, n_dims, "y", dev)
    t_draws = as_device_f32(t_draws, dev)
    assert t_draws.dim() == 3 and t_draws.shape[-1] == P, f"t_draws must be (S, B, {P})"
    S, Bt = int(t_draws.shape[0]), int(t_draws.shape[1])
    B = max(y.shape[0], Bt)
    assert y.shape[0] in (1, B) and Bt in (1, B)
    ym = ys = None
    if y_mean is not None:
        ym = as_device_f32(y_mean, dev).reshape(-1).contiguous()
        ys = as_device_f32(y_std, dev).reshape(-1).contiguous()
    want_sum = want_sum or want_nonfinite
    out = torch.empty((B,), dtype=torch.float32, device=dev) if want_values else None
    osum = torch.empty((2,), dtype=torch.float64, device=dev) if want_sum else None
    lib = _lib.load()
    # the workspace also enables the draw split (more parallelism for small B)
    ws = _workspace(int(lib.nfn_posterior_workspace_doubles(B, n_dims, P)), dev)
    ids, k = flow_ids(flow_types)
    rc = lib.nfn_posterior_lse_f32(
        _ptr(y), _row_stride(y), _ptr(t_draws), int(t_draws.stride(0)), 0 if Bt == 1 else int(t_draws.stride(1)),
        S, B, int(n_dims), ctypes.cast(ids, ctypes.c_void_p), k, int(bool(trainable_base)), _ptr(ym), _ptr(ys),
        _ptr(out), _ptr(osum), _ptr(ws), _stream(),
    )
    _lib.check(rc, "nfn_posterior_lse_f32")
    return _with_nonfinite(out, osum, want_nonfinite)


def set_math_mode(mode: str) -> str:
    """Select the kernels' transcendental implementation for later launches:
    ``"fast"`` (default) or ``"precise"``.  Returns the previous mode."""
    assert mode in ("fast", "precise")
    prev = _lib.load().nfn_set_math_mode(1 if mode == "precise" else 0)
    _lib.check(prev if prev < 0 else 0, "nfn_set_math_mode")
    return "precise" if prev == 1 else "fast"


class BijectorLauncher:
    """Pre-bound one-launch Chain bijector (``nfn_chain_fwd_ldj_f32``) over the layer's
    flow blocks of ``t`` — the Bijector API path (``Chain.forward`` +
    ``forward_log_det_jacobian``) for the benchmark: ``launch()`` writes ``z_out`` (B, d)
    and ``ldj`` (B,)."""

    def __init__(self, z: torch.Tensor, t: torch.Tensor, flow_types: Sequence[str], n_dims: int,
                 trainable_base: bool):
        self.lib = _lib.load()
        dev = z.device
        d = int(n_dims)
        P = total_param_size(flow_types, d, trainable_base)
        assert z.dim() == 2 and z.shape[1] == d and z.stride(1) == 1
        assert t.dim() == 2 and t.shape[1] == P and t.stride(1) == 1
        self.B = max(int(z.shape[0]), int(t.shape[0]))
        # the layer's reversed layout: flow k's block offset within the row (_get_bijector)
        off, offs = 2 * d if trainable_base else 0, [0] * len(flow_types)
        for k in reversed(range(len(flow_types))):
            offs[k] = off
            off += param_size(flow_types[k], d)
        self.z, self.t = z, t
        self.z_out = torch.empty((self.B, d), dtype=torch.float32, device=dev)
        self.ldj = torch.empty((self.B,), dtype=torch.float32, device=dev)
        self._ids, self._k = flow_ids(flow_types)
        self._offs = (ctypes.c_int32 * max(1, len(offs)))(*offs)
        self._args = (_ptr(z), _row_stride(z), _ptr(t), _row_stride(t), self.B, d,
                      ctypes.cast(self._ids, ctypes.c_void_p), ctypes.cast(self._offs, ctypes.c_void_p), self._k,
                      _ptr(self.z_out), _ptr(self.ldj))

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self.lib.nfn_chain_fwd_ldj_f32(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "nfn_chain_fwd_ldj_f32")


class GridLauncher:
    """Pre-bound density grid (``nfn_chain_logprob_grid_f32``) for the benchmark: the
    ``log_prob`` of each of G grid values under each of B parameter rows, (G, B) out — the
    evaluation ``flow_plotting.plot_model`` makes (``evaluation/visualization/flow_plotting.py:33-53``)."""

    def __init__(self, y_grid: torch.Tensor, t: torch.Tensor, flow_types: Sequence[str], n_dims: int,
                 trainable_base: bool):
        self.lib = _lib.load()
        d = int(n_dims)
        P = total_param_size(flow_types, d, trainable_base)
        assert y_grid.dim() == 2 and y_grid.shape[1] == d and y_grid.stride(1) == 1
        assert t.dim() == 2 and t.shape[1] == P and t.stride(1) == 1
        self.G, self.B = int(y_grid.shape[0]), int(t.shape[0])
        self.y_grid, self.t = y_grid, t
        self.out = torch.empty((self.G, self.B), dtype=torch.float32, device=t.device)
        self._ids, self._k = flow_ids(flow_types)
        self._args = (_ptr(y_grid), int(y_grid.stride(0)) if self.G > 1 else 0, self.G, _ptr(t), _row_stride(t),
                      self.B, d, ctypes.cast(self._ids, ctypes.c_void_p), self._k, int(bool(trainable_base)),
                      None, None, _ptr(self.out), self.B)

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self.lib.nfn_chain_logprob_grid_f32(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "nfn_chain_logprob_grid_f32")


class FlowsLauncher:
    """Pre-bound flow-by-flow Bijector path for the benchmark: the Chain's K flows as K
    single-flow launches (``nfn_flow_fwd_ldj_f32``, PlanarFlow.py:68-80 / RadialFlow.py:50-70 /
    AffineFlow.py called one bijector at a time), flow k reading its own parameters and the
    previous flow's z, writing z and its own log|det J| (``ldj`` (K, B)).  ``z_out`` holds
    z_K after ``launch()``.  ``params`` says where the parameters come from:

    * ``"views"`` (what ``normalizing_flows`` does for the flows of one layer's ``t``): when
      ``split_pays`` (narrow blocks in wide rows, e.g. C2) each ``launch()`` first makes the
      flows' blocks contiguous in ONE pass over ``t`` (``nfn_split_blocks_f32``, as TF's slices
      copy them), then runs the K launches on the contiguous blocks; otherwise (C3) the
      launches read their blocks from the rows (``mode`` becomes ``"strided"``);
    * ``"separate"``: the flows were built individually, each over its own contiguous
      (B, param_size) tensor (copied here, once, outside the timed launches);
    * ``"strided"``: each launch reads its block straight from the wide rows of ``t``
      (every launch then fetches the whole 128-B lines: the pre-split path, for the record)."""

    def __init__(self, z: torch.Tensor, t: torch.Tensor, flow_types: Sequence[str], n_dims: int,
                 trainable_base: bool, separate: bool = False, params: Optional[str] = None):
        self.lib = _lib.load()
        dev = z.device
        d = int(n_dims)
        self.mode = params or ("separate" if separate else "views")
        assert self.mode in ("views", "separate", "strided")
        P = total_param_size(flow_types, d, trainable_base)
        assert z.dim() == 2 and z.shape[1] == d and z.stride(1) == 1
        assert t.dim() == 2 and t.shape[1] == P and t.stride(1) == 1
        B = max(int(z.shape[0]), int(t.shape[0]))
        self.B, K = B, len(flow_types)
        base = 2 * d if trainable_base else 0
        off, offs = base, [0] * K
        for k in reversed(range(K)):
            offs[k] = off
            off += param_size(flow_types[k], d)
        zs = [torch.empty((B, d), dtype=torch.float32, device=dev) for _ in range(2)]
        self.ldj = torch.empty((max(1, K), B), dtype=torch.float32, device=dev)
        self.z_out = zs[(K - 1) % 2] if K else z
        self._calls = []
        self._split = None
        self.params = []  # the flows' contiguous parameter tensors (kept alive here)
        if self.mode == "views" and not split_pays([param_size(f, d) for f in flow_types], _row_stride(t) or P):
            self.mode = "strided"  # the package's flows read such blocks straight from the rows
        if self.mode != "strided" and K:
            # blocks in row order: flow K-1 first (the layer's reversed layout)
            order = sorted(range(K), key=lambda k: offs[k])
            widths = [param_size(flow_types[k], d) for k in order]
            tb = t[:, base:]
            blocks = split_blocks(tb, widths)
            if self.mode == "views":
                self._split = (_ptr(tb), _row_stride(tb), B, (ctypes.c_int32 * len(widths))(*widths), len(widths),
                               _ptr(blocks[0]))
            by_flow = {k: blocks[i] for i, k in enumerate(order)}
            self.params = [by_flow[k] for k in range(K)]
        zin = z
        for k, f in enumerate(flow_types):
            zo = zs[k % 2]
            if self.mode == "strided":
                pptr, pstride = _ptr(t) + 4 * offs[k], _row_stride(t)
            else:
                pptr, pstride = _ptr(self.params[k]), param_size(f, d)
            self._calls.append((FLOW_IDS[f], _ptr(zin), _row_stride(zin), pptr, pstride, B, d, _ptr(zo),
                                _ptr(self.ldj[k])))
            zin = zo
        self.bytes_per_launch = float(B) * sum(4 * d + 4 * param_size(f, d) + 4 * d + 4 for f in flow_types)

    def launch(self, stream: Optional[int] = None) -> None:
        st = stream if stream is not None else _stream()
        if self._split is not None:
            rc = self.lib.nfn_split_blocks_f32(*self._split, st)
            if rc != 0:
                _lib.check(rc, "nfn_split_blocks_f32")
        for args in self._calls:
            rc = self.lib.nfn_flow_fwd_ldj_f32(*args, st)
            if rc != 0:
                _lib.check(rc, "nfn_flow_fwd_ldj_f32")


class ChainLauncher:
    """Pre-bound fused-chain launch for repeated evaluation of fixed device
    buffers (the benchmark / serving loop): all validation and pointer
    marshalling happens once; ``launch()`` is a single C-ABI call.

    ``launch()`` writes ``out`` (B,) and ``sum2`` = {fp64 sum, non-finite count}, finished
    in the kernel by its last workgroup (``sum`` is ``sum2[0:1]``)."""

    def __init__(self, y: torch.Tensor, t: torch.Tensor, flow_types: Sequence[str], n_dims: int,
                 trainable_base: bool, write_values: bool = True, draws: Optional[int] = None,
                 fused_sum: bool = True):
        self.lib = _lib.load()
        dev = y.device
        self.n_dims = int(n_dims)
        self.P = total_param_size(flow_types, n_dims, trainable_base)
        self.posterior = draws is not None
        assert y.dim() == 2 and y.shape[1] == n_dims and y.stride(1) == 1
        if self.posterior:
            assert t.dim() == 3 and t.shape[0] == draws and t.shape[2] == self.P and t.stride(2) == 1
            self.B = max(int(y.shape[0]), int(t.shape[1]))
        else:
            assert t.dim() == 2 and t.shape[1] == self.P and t.stride(1) == 1
            self.B = max(int(y.shape[0]), int(t.shape[0]))
        self.y, self.t = y, t
        self.out = torch.empty((self.B,), dtype=torch.float32, device=dev) if write_values else None
        self.sum2 = torch.zeros((2,), dtype=torch.float64, device=dev)  # {sum, non-finite}
        self.sum = self.sum2[0:1]
        fn_ws = self.lib.nfn_posterior_workspace_doubles if self.posterior else self.lib.nfn_chain_workspace_doubles
        self.n_partials = int(fn_ws(self.B, self.n_dims, self.P))
        self.partials = torch.zeros((max(2, self.n_partials),), dtype=torch.float64, device=dev)
        self.fused_sum = fused_sum
        self._ids, self._k = flow_ids(flow_types)
        self._ids_p = ctypes.cast(self._ids, ctypes.c_void_p)
        self._trainable = int(bool(trainable_base))
        if self.posterior:
            self._args = (
                _ptr(y), _row_stride(y), _ptr(t), int(t.stride(0)), 0 if t.shape[1] == 1 else int(t.stride(1)),
                int(draws), self.B, self.n_dims, self._ids_p, self._k, self._trainable, None, None,
                _ptr(self.out), _ptr(self.sum2) if fused_sum else None, _ptr(self.partials),
            )
            self._fn = self.lib.nfn_posterior_lse_f32
        else:
            self._args = (
                _ptr(y), _row_stride(y), _ptr(t), _row_stride(t), self.B, self.n_dims, self._ids_p, self._k,
                self._trainable, None, None, _ptr(self.out), _ptr(self.sum2) if fused_sum else None,
                _ptr(self.partials),
            )
            self._fn = self.lib.nfn_chain_logprob_f32
        self._sum_args = (_ptr(self.partials), _ptr(self.sum2))

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self._fn(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "fused chain launch")

    def bind_sum(self, target: torch.Tensor) -> None:
        """Make later launches finish their ``{sum, non-finite count}`` into ``target[0:2]``
        (fp64, device) — e.g. straight into an all-reduce buffer, so a multi-GPU step needs
        no copy kernels between the chain kernel and the collective."""
        assert self.fused_sum, "bind_sum needs the in-kernel finish"
        assert target.dtype == torch.float64 and target.is_contiguous() and target.numel() >= 2
        i = 14 if self.posterior else 12
        self._args = self._args[:i] + (_ptr(target),) + self._args[i + 1:]
        self.sum2, self.sum = target[0:2], target[0:1]

    def finish_sum(self, stream: Optional[int] = None) -> torch.Tensor:
        """``sum`` (1,) fp64 of the last launch: finished inside the kernel by default; with
        ``fused_sum=False`` the launch writes only the partials and this reduces them
        (``nfn_reduce_partials_f64``, the same summation order and bits)."""
        if not self.fused_sum:
            rc = self.lib.nfn_reduce_partials_f64(*self._sum_args, stream if stream is not None else _stream())
            if rc != 0:
                _lib.check(rc, "nfn_reduce_partials_f64")
        return self.sum

    @property
    def nonfinite(self) -> torch.Tensor:
        """(1,) fp64: non-finite values among the last launch's log-densities."""
        return self.sum2[1:2]


class GradLauncher:
    """Pre-bound fused-backward launch over fixed device buffers (the training-step
    benchmark): ``launch()`` writes ``grad_t`` (B, P) and ``grad_y`` (B, d) for the
    upstream gradient ``g_out`` (B,) — one C-ABI call."""

    def __init__(self, y: torch.Tensor, t: torch.Tensor, flow_types: Sequence[str], n_dims: int,
                 trainable_base: bool, g_out: Optional[torch.Tensor] = None, write_logp: bool = False):
        self.lib = _lib.load()
        dev = y.device
        self.n_dims = int(n_dims)
        self.P = total_param_size(flow_types, n_dims, trainable_base)
        assert y.dim() == 2 and y.shape[1] == n_dims and y.stride(1) == 1
        assert t.dim() == 2 and t.shape[1] == self.P and t.stride(1) == 1
        self.B = max(int(y.shape[0]), int(t.shape[0]))
        assert g_out is None or (g_out.numel() == self.B and g_out.is_contiguous())
        self.y, self.t, self.g_out = y, t, g_out
        self.logp = torch.empty((self.B,), dtype=torch.float32, device=dev) if write_logp else None
        self.grad_t = torch.empty((self.B, self.P), dtype=torch.float32, device=dev)
        self.grad_y = torch.empty((self.B, self.n_dims), dtype=torch.float32, device=dev)
        self._ids, self._k = flow_ids(flow_types)
        self._args = (
            _ptr(y), _row_stride(y), _ptr(t), _row_stride(t), self.B, self.n_dims,
            ctypes.cast(self._ids, ctypes.c_void_p), self._k, int(bool(trainable_base)), None, None,
            _ptr(g_out), _ptr(self.logp), _ptr(self.grad_t), self.P, _ptr(self.grad_y),
        )

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self.lib.nfn_chain_logprob_grad_f32(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "nfn_chain_logprob_grad_f32")


class DenseGradLauncher:
    """Pre-bound fused backward through the output Dense layer
    (``nfn_chain_logprob_dense_grad_f32``) over fixed device buffers (the training-step
    benchmark): ``launch()`` writes ``grad_h`` (B, H), ``grad_W`` (H, P), ``grad_b`` (P,)
    and ``grad_y`` (B, d) for the upstream gradient ``g_out`` — one C-ABI call (the
    fused kernel + the fixed-order partials sum)."""

    def __init__(self, y: torch.Tensor, h: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor],
                 flow_types: Sequence[str], n_dims: int, trainable_base: bool, g_out: Optional[torch.Tensor] = None):
        self.lib = _lib.load()
        dev = y.device
        self.n_dims = int(n_dims)
        self.P = total_param_size(flow_types, n_dims, trainable_base)
        self.B, self.H = int(h.shape[0]), int(h.shape[1])
        assert dense_fusable(self.H, self.P, self.n_dims) and h.stride(1) == 1 and h.stride(0) % 4 == 0
        assert tuple(W.shape) == (self.H, self.P) and y.dim() == 2 and y.shape[1] == n_dims
        assert g_out is None or (g_out.numel() == self.B and g_out.is_contiguous())
        self.y, self.h, self.W, self.b, self.g_out = y, h, W.contiguous(), b, g_out
        self.grad_h = torch.empty((self.B, self.H), dtype=torch.float32, device=dev)
        self.grad_W = torch.empty((self.H, self.P), dtype=torch.float32, device=dev)
        self.grad_b = torch.empty((self.P,), dtype=torch.float32, device=dev)
        self.grad_y = torch.empty((self.B, self.n_dims), dtype=torch.float32, device=dev)
        self.ws = torch.empty((max(1, int(self.lib.nfn_dense_grad_workspace_floats(self.B, self.H, self.P))),),
                              dtype=torch.float32, device=dev)
        self._ids, self._k = flow_ids(flow_types)
        self._args = (
            _ptr(y), _row_stride(y), _ptr(h), int(h.stride(0)), self.H, _ptr(self.W), _ptr(b), self.B, self.n_dims,
            ctypes.cast(self._ids, ctypes.c_void_p), self._k, int(bool(trainable_base)), None, None, _ptr(g_out),
            None, _ptr(self.grad_h), self.H, _ptr(self.grad_W), _ptr(self.grad_b), _ptr(self.grad_y), _ptr(self.ws),
        )

    def launch(self, stream: Optional[int] = None) -> None:
        rc = self.lib.nfn_chain_logprob_dense_grad_f32(*self._args, stream if stream is not None else _stream())
        if rc != 0:
            _lib.check(rc, "nfn_chain_logprob_dense_grad_f32")
