"""``InverseNormalizingFlowLayer`` and the flow distribution it produces.

Drop-in for ``estimators/DistributionLayers.py:215-294``.  The reference builds
``tfd.TransformedDistribution(MVNDiag(base(t)), Invert(Chain(reversed flows)))``
per call and TF evaluates its ``log_prob`` as ~40 eager element-wise ops per
flow.  Here the same object graph exists for API compatibility (``.bijector``,
``.distribution``, ``event_shape``, ``batch_shape``, the reversed-order
``_get_bijector``), but ``log_prob`` / ``prob`` go straight to ONE fused HIP
kernel (``nfn_chain_logprob_f32``) that walks the whole chain per sample in
registers.
"""

from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from . import ops
from .normalizing_flows import FLOWS, Chain, Invert
from .normalizing_flows.flows import SplitBlocks, snapshot_rows


class TensorShape(tuple):
    """Shape tuple that compares equal to lists / tuples / torch.Size (as TF's
    ``TensorShape`` does in the reference tests, e.g. ``dist.event_shape == [1]``)."""

    def __eq__(self, other):
        if isinstance(other, (list, tuple)):
            return tuple(self) == tuple(other)
        if isinstance(other, (int, np.integer)):
            return len(self) == 1 and self[0] == int(other)
        return NotImplemented

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    __hash__ = tuple.__hash__


def _shape(x):
    s = getattr(x, "shape", None)
    return tuple(np.shape(x)) if s is None else tuple(s)


def _cols(t, begin: int, end: int):
    """``t[..., begin:end]`` for torch tensors (a view: no copy), numpy arrays and lists."""
    if isinstance(t, torch.Tensor):
        return t[..., begin:end]
    return np.asarray(t, dtype=np.float32)[..., begin:end]


def _needs_grad(*xs) -> bool:
    return torch.is_grad_enabled() and any(isinstance(x, torch.Tensor) and x.requires_grad for x in xs)


def _broadcast_rows(y, t, event: int, width: int):
    """Bring ``y (..., event)`` and ``t (..., width)`` to 2-D row form for the kernel.

    The 2-D case (including batch-1 broadcast either way) passes through with
    stride-0 broadcasting inside the kernel; other batch ranks are expanded."""
    y = ops.as_device_f32(y)
    t = ops.as_device_f32(t) if width > 0 else None
    if y.dim() == 1:
        y = y.unsqueeze(0)
    bt = tuple(t.shape[:-1]) if t is not None else ()
    if t is not None and t.dim() == 1:
        t = t.unsqueeze(0)
    if y.dim() == 2 and (t is None or t.dim() == 2):
        return y, t, None
    bshape = torch.broadcast_shapes(tuple(y.shape[:-1]), bt)
    y2 = y.expand(*bshape, event).reshape(-1, event)
    t2 = t.expand(*bshape, width).reshape(-1, width) if t is not None else None
    return y2, t2, bshape


class MultivariateNormalDiag:
    """Base distribution of the layer (``DistributionLayers.py:280-294``).

    ``log_prob`` runs the fused kernel with an empty flow chain."""

    def __init__(self, t, n_dims: int, trainable: bool):
        self._t = t
        self._n_dims = int(n_dims)
        self._trainable = bool(trainable)
        if trainable:
            assert _shape(t)[-1] >= 2 * n_dims

    @property
    def event_shape(self):
        return TensorShape([self._n_dims])

    @property
    def batch_shape(self):
        return TensorShape(_shape(self._t)[:-1])

    def log_prob(self, x):
        d = self._n_dims
        base = _cols(self._t, 0, 2 * d) if self._trainable else None
        y, t, bshape = _broadcast_rows(x, base if base is not None else np.zeros((1, 0), np.float32), d,
                                       2 * d if self._trainable else 0)
        if not self._trainable:
            B = max(y.shape[0], int(np.prod(self.batch_shape)) if len(self.batch_shape) else 1)
            y = y.expand(B, d) if y.shape[0] == 1 and B > 1 else y
        if _needs_grad(y, t):
            lp = ops.log_prob(y, t, (), d, self._trainable)
        else:
            lp, _ = ops.chain_log_prob(y, t, (), d, self._trainable)
        return lp if bshape is None else lp.reshape(bshape)

    def prob(self, x):
        return torch.exp(self.log_prob(x))


class FlowDistribution:
    """``TransformedDistribution(base, Invert(Chain(...)))`` of the reference,
    evaluated by the fused kernel."""

    def __init__(self, t, n_dims: int, flow_types: Sequence[str], trainable_base_dist: bool):
        self._n_dims = int(n_dims)
        self._flow_types = tuple(flow_types)
        self._trainable = bool(trainable_base_dist)
        self._t = t
        self.distribution = InverseNormalizingFlowLayer._get_base_dist(t, n_dims, trainable_base_dist)
        # A wrong width raises AssertionError at construction, as in the reference
        # (DistributionLayers.py:272); the Chain itself (and the parameter snapshot its flows
        # own) is built on first use of ``bijector``: log_prob never needs it.
        flow_w = _shape(t)[-1] - (2 * n_dims if trainable_base_dist else 0)
        assert sum(FLOWS[f].get_param_size(n_dims) for f in self._flow_types) == flow_w
        self._bijector = None

    @property
    def bijector(self):
        """``Invert(Chain(flows))`` over a snapshot of ``t``'s flow columns taken on FIRST
        ACCESS (``_get_bijector``), not at construction: ``log_prob`` never pays for the copy.
        The distribution itself reads ``t`` live — ``log_prob`` / ``prob`` evaluate ``t`` as it
        is at the call, and so does the snapshot when it is taken — so a write into ``t``
        between construction and that first access reaches both (TF's tensors are immutable,
        so the reference has no such window).  From then on the Chain keeps its snapshot."""
        if self._bijector is None:
            d = self._n_dims
            # built under grad mode whenever t requires grad: a Chain first touched under
            # torch.no_grad() (sampling) is cached, and later forward / fldj calls must still
            # differentiate into t
            with torch.set_grad_enabled(isinstance(self._t, torch.Tensor) and self._t.requires_grad):
                flow_t = _cols(self._t, 2 * d, _shape(self._t)[-1]) if self._trainable else self._t
                self._bijector = Invert(InverseNormalizingFlowLayer._get_bijector(flow_t, self._flow_types, d))
        return self._bijector

    @property
    def event_shape(self):
        return TensorShape([self._n_dims])

    @property
    def batch_shape(self):
        return TensorShape(_shape(self._t)[:-1])

    @property
    def params(self):
        return self._t

    def log_prob(self, y, y_mean=None, y_std=None):
        """``log_prob(y)``; optional fused normalisation ``(y-mean)/std`` with the
        ``-sum(log std)`` Jacobian correction (``BaseEstimator.py:85-86``)."""
        P = _shape(self._t)[-1]
        yy, tt, bshape = _broadcast_rows(y, self._t, self._n_dims, P)
        if _needs_grad(yy, tt):  # training: differentiable through the fused backward kernel
            lp = ops.log_prob(yy, tt, self._flow_types, self._n_dims, self._trainable, y_mean, y_std)
        else:
            lp, _ = ops.chain_log_prob(yy, tt, self._flow_types, self._n_dims, self._trainable, y_mean, y_std)
        if bshape is not None:
            return lp.reshape(bshape)
        if len(self.batch_shape) == 0 and _shape(y) and len(_shape(y)) == 1:
            return lp.reshape(())
        return lp

    def log_prob_sum(self, y, y_mean=None, y_std=None, want_nonfinite: bool = False):
        """``sum_b log_prob(y_b)`` in fp64, reduced on the device (no (B,) output written);
        with ``want_nonfinite`` also the number of non-finite log-densities (fp64 scalar)."""
        P = _shape(self._t)[-1]
        yy, tt, _ = _broadcast_rows(y, self._t, self._n_dims, P)
        _, s, nf = ops.chain_log_prob(yy, tt, self._flow_types, self._n_dims, self._trainable, y_mean, y_std,
                                      want_values=False, want_nonfinite=True)
        return (s[0], nf[0]) if want_nonfinite else s[0]

    def prob(self, y, y_mean=None, y_std=None):
        return torch.exp(self.log_prob(y, y_mean, y_std))

    def log_prob_grid(self, y_grid, y_mean=None, y_std=None) -> torch.Tensor:
        """``log_prob`` of each grid value (G, d) under every batch member: (G, *batch_shape)."""
        P = _shape(self._t)[-1]
        t = ops.as_device_f32(self._t)
        bshape = tuple(t.shape[:-1])
        t2 = t.reshape(-1, P) if t.dim() != 2 else t
        yg = ops.as_device_f32(y_grid).reshape(-1, self._n_dims)
        out = ops.chain_log_prob_grid(yg, t2, self._flow_types, self._n_dims, self._trainable, y_mean, y_std)
        return out.reshape((yg.shape[0],) + bshape)

    def prob_grid(self, y_grid, y_mean=None, y_std=None) -> torch.Tensor:
        return torch.exp(self.log_prob_grid(y_grid, y_mean, y_std))

    def sample(self, sample_shape=(), seed=None) -> torch.Tensor:
        """Draws of shape ``sample_shape + batch_shape + [d]`` through the inverted flows
        (``nfn_chain_sample_f32``).  An extension: the reference's layer cannot sample
        (``DistributionLayers.py:223-226, 240``) because its flows define no inverse."""
        return self.sample_and_log_prob(sample_shape, seed)[0]

    def sample_and_log_prob(self, sample_shape=(), seed=None):
        d = self._n_dims
        P = _shape(self._t)[-1]
        t = ops.as_device_f32(self._t) if P > 0 else None
        bshape = tuple(self.batch_shape)
        sshape = (sample_shape,) if isinstance(sample_shape, int) else tuple(sample_shape)
        n_s = int(np.prod(sshape)) if sshape else 1
        nb = int(np.prod(bshape)) if bshape else 1
        dev = ops._device()
        gen = torch.Generator(device=dev)
        gen.manual_seed(int(seed) if seed is not None else int(torch.randint(0, 2**62, (1,)).item()))
        eps = torch.randn((n_s * nb, d), generator=gen, device=dev)
        if t is not None:
            t2 = t.reshape(nb, P)
            t2 = t2.repeat(n_s, 1) if n_s > 1 else t2
        else:
            t2 = torch.zeros((1, 0), dtype=torch.float32, device=dev)
        y, lp = ops.chain_sample(eps, t2, self._flow_types, d, self._trainable)
        return y.reshape(sshape + bshape + (d,)), lp.reshape(sshape + bshape)


class InverseNormalizingFlowLayer:
    """Turns a parameter tensor ``t`` into a flow distribution.

    ``flow_types`` are applied base -> transformed distribution; the layer
    evaluates ``log_prob`` of externally provided data by inverting the chain.
    Mirrors ``estimators/DistributionLayers.py:215-265`` (a Keras
    ``DistributionLambda`` there; a plain callable here)."""

    _flow_types = None
    _trainable_base_dist = None
    _n_dims = None

    def __init__(self, flow_types, n_dims, trainable_base_dist=False):
        assert all([flow_type in FLOWS for flow_type in flow_types])
        self._flow_types = tuple(flow_types)
        self._trainable_base_dist = bool(trainable_base_dist)
        self._n_dims = int(n_dims)
        self._make_distribution = self._get_distribution_fn(n_dims, self._flow_types, trainable_base_dist)

    def __call__(self, t) -> FlowDistribution:
        return self._make_distribution(t)

    @property
    def flow_types(self):
        return self._flow_types

    @property
    def n_dims(self):
        return self._n_dims

    @property
    def trainable_base_dist(self):
        return self._trainable_base_dist

    @staticmethod
    def _get_distribution_fn(n_dims, flow_types, trainable_base_dist):
        return lambda t: FlowDistribution(t, n_dims, flow_types, trainable_base_dist)

    def get_total_param_size(self):
        """Width of ``t``: flow blocks + ``2*n_dims`` for a trainable base."""
        return ops.total_param_size(self._flow_types, self._n_dims, self._trainable_base_dist)

    @staticmethod
    def _get_bijector(t, flow_types, n_dims):
        """Chain of flows; blocks are split in REVERSED ``flow_types`` order and
        ``bijectors[0]`` is the last flow type (``DistributionLayers.py:267-278``).  As TF's
        slices are copies, the flows own a snapshot of ``t`` taken here (one device pass,
        ``flows.snapshot_rows``): later writes to ``t`` do not reach them."""
        flow_types = list(reversed(list(flow_types)))
        param_sizes = [FLOWS[flow_type].get_param_size(n_dims) for flow_type in flow_types]
        assert sum(param_sizes) == _shape(t)[-1]
        t = snapshot_rows(t)
        chain = []
        begin = 0
        for size, flow_type in zip(param_sizes, flow_types):
            chain.append(FLOWS[flow_type](_cols(t, begin, begin + size), n_dims))
            begin += size
        if isinstance(t, torch.Tensor) and t.dim() == 2 and t.stride(-1) == 1 and len(chain) > 1:
            # the flows' own launches read contiguous copies of their blocks of the snapshot,
            # made in one pass on the first such call (normalizing_flows.SplitBlocks)
            group = SplitBlocks(t, param_sizes)
            for k, f in enumerate(chain):
                f._split = (group, k)
        return Chain(chain)

    @staticmethod
    def _get_base_dist(t, n_dims, trainable) -> MultivariateNormalDiag:
        return MultivariateNormalDiag(t, n_dims, trainable)
