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

    def _forward(self, x):
        for b in reversed(self._bijectors):
            x = b.forward(x)
        return x

    def _forward_log_det_jacobian(self, x):
        fldj = None
        for b in reversed(self._bijectors):
            ld = b.forward_log_det_jacobian(x, event_ndims=self.forward_min_event_ndims)
            fldj = ld if fldj is None else fldj + ld
            x = b.forward(x)
        if fldj is None:
            x = torch.as_tensor(x)
            return torch.zeros(x.shape[:-1], dtype=torch.float32, device=x.device)
        return fldj

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
