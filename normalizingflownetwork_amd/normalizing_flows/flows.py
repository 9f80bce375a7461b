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

from .. import ops
from .bijector import Bijector


def _width(t) -> int:
    shape = getattr(t, "shape", None)
    if shape is None:
        import numpy as np

        shape = np.shape(t)
    return int(shape[-1])


class _ConditionedFlow(Bijector):
    flow_type: str = ""

    def __init__(self, t, n_dims: int, name: str):
        super().__init__(validate_args=False, name=name, inverse_min_event_ndims=1)
        assert _width(t) == self.get_param_size(n_dims)
        self.n_dims = int(n_dims)
        self._t = t  # raw Dense output block; moved to the device on first use

    @property
    def params(self):
        """The raw (unconstrained) parameter block as a device tensor."""
        if not hasattr(self._t, "is_cuda") or not self._t.is_cuda:
            self._t = ops.as_device_f32(self._t)
        return self._t

    def _forward(self, z):
        z_out, _ = ops.flow_forward_ldj(self.flow_type, z, self.params, self.n_dims, want_ldj=False)
        return z_out

    def _forward_log_det_jacobian(self, z):
        _, ldj = ops.flow_forward_ldj(self.flow_type, z, self.params, self.n_dims, want_z=False)
        return ldj

    def forward_and_log_det_jacobian(self, z):
        """Both results from one kernel launch."""
        return ops.flow_forward_ldj(self.flow_type, z, self.params, self.n_dims)


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
