"""Minimal ``tfp.bijectors`` surface the reference's flows rely on.

The reference subclasses ``tfp.bijectors.Bijector`` (``PlanarFlow.py:5``,
``RadialFlow.py:5``), ``tfp.bijectors.Affine`` (``AffineFlow.py:4``) and composes
them with ``tfp.bijectors.Chain`` / ``Invert`` (``DistributionLayers.py:250-278``).
TFP is not part of this framework, so this module restates the parts of that
contract the flow path uses:

* ``forward(x)`` / ``forward_log_det_jacobian(x, event_ndims)`` and the
  subclass hooks ``_forward`` / ``_forward_log_det_jacobian``;
* ``forward_min_event_ndims`` / ``inverse_min_event_ndims`` (one given => both);
* ``Chain([b0, ..., bn]).forward(x) == b0(b1(...bn(x)))`` with the fldj summed
  in that application order;
* ``Invert(b)``: ``inverse <-> forward`` swapped.

The flows are forward-only, exactly like the reference (no ``_inverse``;
sampling is impossible, ``DistributionLayers.py:223-226``).
"""

from __future__ import annotations

from typing import List, Optional, Sequence

import torch


class Bijector:
    """Base class (subset of ``tfp.bijectors.Bijector``)."""

    def __init__(
        self,
        validate_args: bool = False,
        name: Optional[str] = None,
        forward_min_event_ndims: Optional[int] = None,
        inverse_min_event_ndims: Optional[int] = None,
    ):
        if forward_min_event_ndims is None:
            forward_min_event_ndims = inverse_min_event_ndims
        if inverse_min_event_ndims is None:
            inverse_min_event_ndims = forward_min_event_ndims
        if forward_min_event_ndims is None:
            raise ValueError("must specify forward_min_event_ndims or inverse_min_event_ndims")
        self._forward_min_event_ndims = int(forward_min_event_ndims)
        self._inverse_min_event_ndims = int(inverse_min_event_ndims)
        self.validate_args = validate_args
        self.name = name or type(self).__name__

    @property
    def forward_min_event_ndims(self) -> int:
        return self._forward_min_event_ndims

    @property
    def inverse_min_event_ndims(self) -> int:
        return self._inverse_min_event_ndims

    # public API -----------------------------------------------------------
    def forward(self, x, name: Optional[str] = None):
        return self._forward(x)

    def inverse(self, y, name: Optional[str] = None):
        return self._inverse(y)

    def forward_log_det_jacobian(self, x, event_ndims: int = 1, name: Optional[str] = None):
        self._check_event_ndims(event_ndims, self.forward_min_event_ndims)
        return self._forward_log_det_jacobian(x)

    def inverse_log_det_jacobian(self, y, event_ndims: int = 1, name: Optional[str] = None):
        self._check_event_ndims(event_ndims, self.inverse_min_event_ndims)
        return self._inverse_log_det_jacobian(y)

    def __call__(self, x):
        return self.forward(x)

    # hooks ----------------------------------------------------------------
    def _forward(self, x):
        raise NotImplementedError(f"{self.name}: forward is not implemented")

    def _inverse(self, y):
        raise NotImplementedError(
            f"{self.name}: inverse is not implemented (the reference flows are forward-only)"
        )

    def _forward_log_det_jacobian(self, x):
        raise NotImplementedError(f"{self.name}: forward_log_det_jacobian is not implemented")

    def _inverse_log_det_jacobian(self, y):
        raise NotImplementedError(
            f"{self.name}: inverse_log_det_jacobian is not implemented (forward-only flow)"
        )

    @staticmethod
    def _check_event_ndims(event_ndims: int, min_event_ndims: int) -> None:
        # The flows reduce over exactly one event dimension (the reference always
        # uses event_ndims=1, DistributionLayers.py:250 via TransformedDistribution).
        if event_ndims != min_event_ndims:
            raise NotImplementedError(
                f"event_ndims={event_ndims} unsupported; this bijector reduces over {min_event_ndims} dim(s)"
            )


class Chain(Bijector):
    """``tfp.bijectors.Chain``: applies ``bijectors[-1]`` first."""

    def __init__(self, bijectors: Sequence[Bijector], validate_args: bool = False, name: Optional[str] = None):
        self._bijectors: List[Bijector] = list(bijectors)
        fmin = max([b.forward_min_event_ndims for b in self._bijectors], default=0)
        super().__init__(validate_args=validate_args, name=name or "chain_of_" + "_of_".join(
            b.name for b in self._bijectors), forward_min_event_ndims=fmin, inverse_min_event_ndims=fmin)

    @property
    def bijectors(self) -> List[Bijector]:
        return self._bijectors

    def _fused(self, x=None):
        """(flow_types in application order, base tensor, column offsets) when every
        bijector is one of the conditioned flows and their parameter blocks are column
        views of ONE device tensor (as InverseNormalizingFlowLayer._get_bijector slices
        t): the whole chain then runs as one kernel launch.  None otherwise — and None
        when gradients are wanted (``x`` or a parameter block requires grad): the chain then
        runs flow by flow through the flows' autograd op, whose backward is
        ``nfn_flow_vjp_f32``, as TF's tape differentiates the Chain op by op."""
        from .. import ops

        flows = list(reversed(self._bijectors))  # application order
        if not flows or not all(hasattr(b, "flow_type") and hasattr(b, "params") for b in flows):
            return None
        if torch.is_grad_enabled() and (
                (isinstance(x, torch.Tensor) and x.requires_grad) or any(b.params.requires_grad for b in flows)):
            return None
        if len({b.n_dims for b in flows}) != 1:
            return None
        ps = [b.params for b in flows]
        p0 = ps[0]
        if any(p.dim() != 2 or p.stride(1) != 1 or p.dtype != torch.float32 or p.device != p0.device
               or p.untyped_storage().data_ptr() != p0.untyped_storage().data_ptr()
               or p.shape[0] != p0.shape[0] or (p.shape[0] > 1 and p.stride(0) != p0.stride(0)) for p in ps):
            return None
        storage0 = p0.untyped_storage().data_ptr()
        base = min(p.data_ptr() for p in ps)
        if any((p.data_ptr() - base) % 4 for p in ps):
            return None
        # start the view at the row start when the blocks are column views of whole rows
        # (the layer's t: the kernels then stream contiguous rows), else at the 16-byte
        # boundary at or before the leftmost block (aligned float4 rows); the columns left
        # of the first block are staged, never read
        rs = p0.stride(0) if p0.shape[0] > 1 else None
        col = ((base - storage0) // 4) % rs if rs else None
        if rs and base - 4 * col >= storage0:
            base -= 4 * col
        else:
            base = max(storage0, base - base % 16)
        offs = [(p.data_ptr() - base) // 4 for p in ps]
        width = max(o + p.shape[1] for o, p in zip(offs, ps))
        if rs is None:
            rs = width
        elif width > rs:
            return None
        t = p0.as_strided((p0.shape[0], width), (rs, 1), (base - storage0) // 4)
        return [b.flow_type for b in flows], t, offs, flows[0].n_dims, ops

    def forward_and_log_det_jacobian(self, x):
        """``(forward(x), forward_log_det_jacobian(x))``: one kernel launch for a chain of
        the conditioned flows (``nfn_chain_fwd_ldj_f32``), else one launch per flow."""
        fz = self._fused(x)
        if fz is not None:
            ft, t, offs, d, ops = fz
            return ops.chain_forward_ldj(ft, x, t, offs, d)
        fldj = None
        for b in reversed(self._bijectors):
            if hasattr(b, "forward_and_log_det_jacobian"):
                x, ld = b.forward_and_log_det_jacobian(x)
            else:
                ld = b.forward_log_det_jacobian(x, event_ndims=self.forward_min_event_ndims)
                x = b.forward(x)
            fldj = ld if fldj is None else fldj + ld
        if fldj is None:
            x = torch.as_tensor(x)
            fldj = torch.zeros(x.shape[:-1], dtype=torch.float32, device=x.device)
        return x, fldj

    def _forward(self, x):
        fz = self._fused(x)
        if fz is not None:
            ft, t, offs, d, ops = fz
            return ops.chain_forward_ldj(ft, x, t, offs, d, want_ldj=False)[0]
        for b in reversed(self._bijectors):
            x = b.forward(x)
        return x

    def _forward_log_det_jacobian(self, x):
        fz = self._fused(x)
        if fz is not None:
            ft, t, offs, d, ops = fz
            return ops.chain_forward_ldj(ft, x, t, offs, d, want_z=False)[1]
        return self.forward_and_log_det_jacobian(x)[1]

    def _inverse(self, y):
        for b in self._bijectors:
            y = b.inverse(y)
        return y


class Invert(Bijector):
    """``tfp.bijectors.Invert``: swaps forward and inverse."""

    def __init__(self, bijector: Bijector, validate_args: bool = False, name: Optional[str] = None):
        self._bijector = bijector
        super().__init__(
            validate_args=validate_args,
            name=name or "invert_" + bijector.name,
            forward_min_event_ndims=bijector.inverse_min_event_ndims,
            inverse_min_event_ndims=bijector.forward_min_event_ndims,
        )

    @property
    def bijector(self) -> Bijector:
        return self._bijector

    def _forward(self, x):
        return self._bijector.inverse(x)

    def _inverse(self, y):
        return self._bijector.forward(y)

    def _forward_log_det_jacobian(self, x):
        return self._bijector.inverse_log_det_jacobian(x, event_ndims=self.forward_min_event_ndims)

    def _inverse_log_det_jacobian(self, y):
        return self._bijector.forward_log_det_jacobian(y, event_ndims=self.inverse_min_event_ndims)
