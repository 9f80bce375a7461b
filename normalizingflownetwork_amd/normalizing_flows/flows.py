"""Planar, radial and affine flows — per-sample conditioned bijectors.

Drop-in for ``estimators/normalizing_flows/{PlanarFlow,RadialFlow,AffineFlow}.py``:
same class names, constructor ``(t, n_dims, name)``, ``AssertionError`` on a
wrong parameter width, static ``get_param_size(n_dims)``, and the bijector
methods ``forward`` / ``_forward`` / ``forward_log_det_jacobian`` /
``_forward_log_det_jacobian``.  The parameter constraints (``_u_circ``,
``_alpha_circ``, ``_beta_circ``) are applied inside the HIP kernel
(``csrc/nfn_device.h``: ``planar_step`` / ``radial_step`` / ``affine_step``, launched by
``csrc/nfn_tile.hip``'s ``flow_fwd_ldj_kernel``),
so a flow object only holds its raw parameter tensor ``t`` on the device.

Inputs may be torch tensors (any device), numpy arrays or nested lists; they
are moved to the HIP device.  Outputs are float32 device tensors.
"""

from __future__ import annotations

import torch

from .. import ops
from .bijector import Bijector


def _width(t) -> int:
    shape = getattr(t, "shape", None)
    if shape is None:
        import numpy as np

        shape = np.shape(t)
    return int(shape[-1])


def snapshot_rows(t):
    """A private copy of the (B, W) parameter tensor ``t`` for the flows ``_get_bijector``
    builds: TF's ``t[:, o:o+size]`` slices there (``DistributionLayers.py:267-278``) are copies
    of an immutable tensor, so a Chain keeps evaluating the parameters it was built from
    whatever later happens to ``t`` — including writes torch cannot see (HIP-graph replays
    into ``t``, raw-pointer / DLPack producers).  ONE pass on the device.  Layout: the copy
    sits in a (B, W + lead) buffer with ``lead = (-W) mod 4`` unread columns in front of
    each row, so the row stride is a multiple of 4 floats and every PADDED row start (the
    view the one-launch Chain kernel streams, lead columns included) is 16-byte aligned —
    as the layer's base columns pad the wide ``t`` (C2: 2 + 30 = 32 floats); a row's first
    flow column itself sits ``lead`` floats after that boundary.  A broadcast row (stride 0)
    stays one row.  Numpy / list inputs pass through (each flow moves its own slice:
    already a copy).  When ``t`` requires grad the copy is an autograd op WHATEVER the grad
    mode at the time (a bijector first built under ``torch.no_grad()``, e.g. while sampling,
    is cached and later differentiated), so gradients of the flows' outputs reach ``t`` as
    TF's tape reaches the Dense output.
    Memory: the snapshot holds B x (W + lead) floats (C2's 2^24 x 32: 2 GiB) until the flows
    built on it are dropped."""
    if not isinstance(t, torch.Tensor) or t.dim() != 2:
        return t
    with torch.set_grad_enabled(t.requires_grad):
        return _snapshot(t)


def _snapshot(t: torch.Tensor) -> torch.Tensor:
    B, W = int(t.shape[0]), int(t.shape[1])
    if B > 1 and t.stride(0) == 0:
        return t[:1].clone().expand(B, W)
    lead = (-W) % 4
    buf = torch.empty((B, W + lead), dtype=t.dtype, device=t.device)
    buf[:, lead:].copy_(t)
    return buf[:, lead:]


class SplitBlocks:
    """The contiguous copies of consecutive column blocks of the flows' private parameter
    snapshot (:func:`snapshot_rows`), made in ONE pass (``ops.split_blocks`` ->
    ``nfn_split_blocks_f32``) on the first single-flow call and shared by the flows that
    hold views of those blocks (the one-launch Chain reads the snapshot's rows directly).
    Why: a single-flow launch over a view of the wide rows fetches each row's whole 128-B
    lines for its few parameters (per-flow Bijector).  Used only where that costs
    more than the split's own pass (``ops.split_pays``: narrow blocks in wide rows) and only
    over real rows (a broadcast stride-0 row is already read once per line).
    The snapshot belongs to the flows, so the copies can only go stale through a write into
    a flow's own ``params``: torch in-place ops on them bump the version counter checked
    here; a raw-pointer writer into ``params`` must call :meth:`release`.  :meth:`release`
    also frees the copies' memory (B x sum(widths) floats) when the flows are done."""

    def __init__(self, base, widths):
        self.base = base
        self.widths = [int(w) for w in widths]
        self._blocks = None
        self._version = None
        rs = int(base.stride(0)) if base.dim() == 2 else sum(self.widths)
        # else the flows read their views directly
        self.pays = rs >= sum(self.widths) and ops.split_pays(self.widths, rs)

    def release(self):
        """Drop the copies (remade on the next single-flow call)."""
        self._blocks = None
        self._version = None

    def version(self):
        """The base tensor's in-place version counter, or None for a tensor that has none
        (made under ``torch.inference_mode()``): its copies could not be validated, so
        the flows then read the wide rows directly."""
        try:
            return self.base._version
        except RuntimeError:
            return None

    def blocks(self):
        ver = self.version()
        if self._blocks is None or self._version != ver:
            self._blocks = ops.split_blocks(self.base, self.widths)
            self._version = ver
        return self._blocks


class _ConditionedFlow(Bijector):
    flow_type: str = ""

    def __init__(self, t, n_dims: int, name: str):
        super().__init__(validate_args=False, name=name, inverse_min_event_ndims=1)
        assert _width(t) == self.get_param_size(n_dims)
        self.n_dims = int(n_dims)
        self._t = t  # raw Dense output block; moved to the device on first use
        self._split = None  # (SplitBlocks, index): set by InverseNormalizingFlowLayer._get_bijector

    @property
    def params(self):
        """The raw (unconstrained) parameter block as a device tensor."""
        if not hasattr(self._t, "is_cuda") or not self._t.is_cuda:
            self._t = ops.as_device_f32(self._t)
        return self._t

    def _kernel_params(self):
        """The block this flow's own launch reads: its contiguous copy when the flow holds a
        strided view of a wider row that belongs to a split group, else ``params``."""
        t = self.params
        if (self._split is not None and t.dim() == 2 and t.shape[0] > 1 and t.stride(0) != t.shape[1]
                and not (torch.is_grad_enabled() and t.requires_grad)):
            group, k = self._split
            if group.pays and group.version() is not None:
                return group.blocks()[k]
        return t

    def _differentiable(self, z) -> bool:
        """A loss may read this flow's outputs: TF's tape would differentiate through the
        flow (``PlanarFlow.py:68-80``, ``RadialFlow.py:50-70``), so the call goes through the
        autograd op (forward kernel + ``nfn_flow_vjp_f32`` backward)."""
        return torch.is_grad_enabled() and any(
            isinstance(x, torch.Tensor) and x.requires_grad for x in (z, self.params))

    def _forward(self, z):
        if self._differentiable(z):
            return ops.flow_forward_ldj_diff(self.flow_type, z, self.params, self.n_dims)[0]
        z_out, _ = ops.flow_forward_ldj(self.flow_type, z, self._kernel_params(), self.n_dims, want_ldj=False)
        return z_out

    def _forward_log_det_jacobian(self, z):
        if self._differentiable(z):
            return ops.flow_forward_ldj_diff(self.flow_type, z, self.params, self.n_dims)[1]
        _, ldj = ops.flow_forward_ldj(self.flow_type, z, self._kernel_params(), self.n_dims, want_z=False)
        return ldj

    def forward_and_log_det_jacobian(self, z):
        """Both results from one kernel launch (differentiable when ``z`` or the parameters
        require grad)."""
        if self._differentiable(z):
            return ops.flow_forward_ldj_diff(self.flow_type, z, self.params, self.n_dims)
        return ops.flow_forward_ldj(self.flow_type, z, self._kernel_params(), self.n_dims)


class PlanarFlow(_ConditionedFlow):
    """``x = z + u_hat * tanh(w^T z + b)``; ``t`` splits into ``u (d), w-1 (d), b (1)``
    and ``u`` is constrained so that ``w^T u_hat >= -1 + 1e-5``
    (``PlanarFlow.py:20-80``)."""

    flow_type = "planar"

    def __init__(self, t, n_dims, name="Inverted_Planar_Flow"):
        super().__init__(t, n_dims, name)

    @staticmethod
    def get_param_size(n_dims):
        return 2 * n_dims + 1


class RadialFlow(_ConditionedFlow):
    """``x = z + alpha*beta*(z - gamma) / (alpha + |z - gamma|_1)`` with
    ``alpha = softplus(0.3 a - 2)``, ``beta = softplus(0.1 b + log(e-1)) - 1``
    (``RadialFlow.py:20-84``)."""

    flow_type = "radial"

    def __init__(self, t, n_dims, name="RadialFlow"):
        super().__init__(t, n_dims, name)

    @staticmethod
    def get_param_size(n_dims):
        return n_dims + 2


class AffineFlow(_ConditionedFlow):
    """``x = z * (1 + t[d:2d]) + t[:d]`` — the reference's ``tfp.bijectors.Affine``
    subclass (``AffineFlow.py:4-17``)."""

    flow_type = "affine"

    def __init__(self, t, n_dims, name="AffineFlow"):
        super().__init__(t, n_dims, name)

    @staticmethod
    def get_param_size(n_dims):
        return 2 * n_dims
