"""CPU oracle for the BACKWARD of the conditional-flow ``log_prob``.

TEST INFRASTRUCTURE ONLY (same rules as ``nfn_oracle.py``): imported by ``tests/``
and ``__graft_entry__.smoke()`` as the checker, never by the product package.

The reference trains by Keras autodiff through the eager TF ops of the forward
path (``estimators/BaseEstimator.py:19-31`` compiles the model with the NLL loss
``:55-59``; ``MaximumLikelihoodNNEstimator.py:33-35``).  Restating that here means:
the SAME forward ops as ``nfn_oracle.chain_log_prob`` (reversed parameter layout
``DistributionLayers.py:267-278``, planar ``PlanarFlow.py:43-80``, radial
``RadialFlow.py:44-84`` incl. the ``GradientTape`` ``der_h``, affine, trainable MVNDiag
base ``DistributionLayers.py:280-294``, y normalisation ``BaseEstimator.py:85``),
written in torch so reverse-mode autodiff produces ``d log_prob / d t`` and
``d log_prob / d y`` per sample.  TF's gradient conventions that matter are the
ones torch shares: ``Abs`` -> ``sign(x)`` (0 at 0), ``Softplus`` -> ``sigmoid(x)``
for every x (``SoftplusGrad``), ``Log`` of ``Abs`` -> ``1/x``, ``Tanh`` -> ``1-tanh^2``.

Pinned by central finite differences of the numpy fp64 forward oracle
(``tests/test_grad_oracle.py``).
"""

from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch

from .nfn_oracle import param_size, total_param_size  # noqa: F401  (re-export)


class _SoftplusTF(torch.autograd.Function):
    """Value max(x, 0) + log1p(exp(-|x|)) (TF's SoftplusOp up to its +-13.94 cut-offs:
    differences < 1 ulp at fp32 there), gradient sigmoid(x) everywhere (TF SoftplusGrad).
    Autodiff through the max / abs form itself would give 1 instead of sigmoid(0) = 0.5 at
    x = 0 exactly (clamp passes the gradient at its boundary, |x|' = sign(0) = 0) — reached
    when a parameter product is exactly 0 (e.g. planar u = 0 on dyadic inputs)."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.clamp(x, min=0) + torch.log1p(torch.exp(-torch.abs(x)))

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.sigmoid(x)


def _softplus(x: torch.Tensor) -> torch.Tensor:
    return _SoftplusTF.apply(x)


def _planar(z, tk, d):
    u = tk[:, 0:d]
    w = tk[:, d:2 * d] + 1.0
    b = tk[:, 2 * d:2 * d + 1]
    wtu = (w * u).sum(-1, keepdim=True)
    m_wtu = (-1.0 + _softplus(wtu)) + 1e-5
    nw2 = (w ** 2).sum(-1, keepdim=True) + 1e-9
    u_hat = u + (m_wtu - wtu) * (w / nw2)
    th = torch.tanh((w * z).sum(-1, keepdim=True) + b)
    z_new = z + u_hat * th
    psi = (1.0 - th ** 2) * w
    ldj = torch.log(torch.abs(1.0 + (u_hat * psi).sum(-1)))
    return z_new, ldj


def _radial(z, tk, d):
    alpha = _softplus(0.3 * tk[:, 0:1] - 2.0)
    beta = _softplus(0.1 * tk[:, 1:2] + math.log(math.expm1(1.0))) - 1.0
    gamma = tk[:, 2:d + 2]
    r = torch.abs(z - gamma).sum(-1, keepdim=True)
    y = alpha + r
    h = 1.0 / y
    der_h = (-1.0 / y) / y  # GradientTape of h = 1/(alpha + r) w.r.t. r (RadialFlow.py:63-66)
    ab = alpha * beta
    z_new = z + (ab * h) * (z - gamma)
    det = (1.0 + ab * h) ** (d - 1) * (1.0 + ab * h + ab * der_h * r)
    return z_new, torch.log(det[:, 0])


def _affine(z, tk, d):
    scale = 1.0 + tk[:, d:2 * d]
    return z * scale + tk[:, 0:d], torch.log(torch.abs(scale)).sum(-1)


_FLOW = {"planar": _planar, "radial": _radial, "affine": _affine}


def chain_log_prob_torch(y: torch.Tensor, t: torch.Tensor, flow_types: Sequence[str], d: int,
                         trainable_base: bool, y_mean=None, y_std=None) -> torch.Tensor:
    """Differentiable restatement of ``nfn_oracle.log_pdf`` (same op order)."""
    B = max(y.shape[0], t.shape[0])
    z = y.expand(B, d)
    if y_mean is not None:
        z = (z - y_mean) / y_std
    o = 2 * d if trainable_base else 0
    rev = list(reversed(list(flow_types)))
    sizes = [param_size(f, d) for f in rev]
    assert o + sum(sizes) == t.shape[-1], "param width mismatch"
    starts, begin = [], o
    for s in sizes:
        starts.append(begin)
        begin += s
    starts = list(reversed(starts))  # application order
    tt = t.expand(B, t.shape[-1])
    ildj = torch.zeros((B,), dtype=t.dtype)
    for f, st in zip(flow_types, starts):
        z, l = _FLOW[f](z, tt[:, st:st + param_size(f, d)], d)
        ildj = ildj + l
    if trainable_base:
        loc = tt[:, 0:d]
        scale = 1e-3 + _softplus(math.log(math.expm1(1.0)) + 0.1 * tt[:, d:2 * d])
        zz = (z - loc) / scale
        base = -0.5 * (zz ** 2).sum(-1) - (0.5 * d * math.log(2 * math.pi) + torch.log(torch.abs(scale)).sum(-1))
    else:
        base = -0.5 * (z ** 2).sum(-1) - 0.5 * d * math.log(2 * math.pi)
    lp = base + ildj
    if y_mean is not None:
        lp = lp - torch.log(y_std).sum()
    return lp


def chain_log_prob_grad(y, t, flow_types, d, trainable_base, y_mean=None, y_std=None, g_out=None,
                        dtype=np.float64):
    """Return ``(log_prob (B,), dL/dt (B,P), dL/dy (B,d))`` with ``L = sum_b g_b log_prob_b``
    (``g_out`` None => ones, i.e. the per-sample gradients of log_prob).

    ``y`` (B or 1, d) and ``t`` (B or 1, P) are broadcast as the forward does; the
    returned gradients are per sample (B rows) — a caller that broadcast an input
    sums them over the batch itself."""
    tdt = torch.float64 if np.dtype(dtype) == np.float64 else torch.float32
    B = max(np.shape(y)[0], np.shape(t)[0])
    P = np.shape(t)[-1]
    yt = torch.tensor(np.broadcast_to(np.asarray(y, dtype=dtype), (B, d)).copy(), dtype=tdt, requires_grad=True)
    tt = torch.tensor(np.broadcast_to(np.asarray(t, dtype=dtype), (B, P)).copy(), dtype=tdt, requires_grad=True)
    ym = None if y_mean is None else torch.tensor(np.asarray(y_mean, dtype=dtype), dtype=tdt)
    ys = None if y_std is None else torch.tensor(np.asarray(y_std, dtype=dtype), dtype=tdt)
    lp = chain_log_prob_torch(yt, tt, flow_types, d, trainable_base, ym, ys)
    g = torch.ones_like(lp) if g_out is None else torch.tensor(np.asarray(g_out, dtype=dtype), dtype=tdt)
    gt, gy = torch.autograd.grad(lp, (tt, yt), grad_outputs=g, allow_unused=True)
    gt = torch.zeros_like(tt) if gt is None else gt
    gy = torch.zeros_like(yt) if gy is None else gy
    return lp.detach().numpy(), gt.numpy(), gy.numpy()


def fp32_spread(y, t, flow_types, d, trainable_base, y_mean=None, y_std=None, g_out=None, n_perturbed=3,
                seed=0):
    """The reference's own fp32 sensitivity per gradient element: the largest
    deviation from the fp64 truth over the fp32 autodiff evaluation at the given
    inputs and at ``n_perturbed`` copies whose inputs are moved by one random ulp
    (+-2^-23 relative).  Rounding inside an ill-conditioned chain (e.g. a planar
    determinant near 0) moves an fp32 result by about as much as such a
    perturbation does, so this — not a single fp32 run, which can be lucky —
    is what an fp32 implementation with a different op order must be held to.
    Returns ``(g64_t, g64_y, dev_t, dev_y)``."""
    _, gt64, gy64 = chain_log_prob_grad(y, t, flow_types, d, trainable_base, y_mean, y_std, g_out, np.float64)
    rng = np.random.default_rng(seed)
    dev_t = np.zeros_like(gt64)
    dev_y = np.zeros_like(gy64)
    y32 = np.asarray(y, np.float32)
    t32 = np.asarray(t, np.float32)
    for k in range(n_perturbed + 1):
        if k == 0:
            yk, tk = y32, t32
        else:
            yk = (y32 * (1 + rng.integers(-1, 2, y32.shape) * 2.0 ** -23)).astype(np.float32)
            tk = (t32 * (1 + rng.integers(-1, 2, t32.shape) * 2.0 ** -23)).astype(np.float32)
        _, gt32, gy32 = chain_log_prob_grad(yk, tk, flow_types, d, trainable_base, y_mean, y_std, g_out, np.float32)
        dev_t = np.maximum(dev_t, np.abs(gt32.astype(np.float64) - gt64))
        dev_y = np.maximum(dev_y, np.abs(gy32.astype(np.float64) - gy64))
    return gt64, gy64, dev_t, dev_y


def flow_vjp(flow_type, z, tk, d, g_z=None, g_ldj=None, dtype=np.float64):
    """One bijector's vector-Jacobian product: ``(dL/dz (B,d), dL/dt_k (B,p))`` for
    ``L = sum_b <g_z[b], f(z_b)> + g_ldj[b] * fldj(z_b)`` (None => zero), through the same
    per-flow ops as the chain (``PlanarFlow.py:43-80``, ``RadialFlow.py:44-84``, affine).
    What TF's tape gives for a loss on ``flow.forward`` / ``forward_log_det_jacobian``.
    Broadcast inputs (batch 1) get one gradient row per sample."""
    tdt = torch.float64 if np.dtype(dtype) == np.float64 else torch.float32
    B = max(np.shape(z)[0], np.shape(tk)[0])
    p = np.shape(tk)[-1]
    zt = torch.tensor(np.broadcast_to(np.asarray(z, dtype=dtype), (B, d)).copy(), dtype=tdt, requires_grad=True)
    tt = torch.tensor(np.broadcast_to(np.asarray(tk, dtype=dtype), (B, p)).copy(), dtype=tdt, requires_grad=True)
    z_new, ldj = _FLOW[flow_type](zt, tt, d)
    L = torch.zeros((), dtype=tdt)
    if g_z is not None:
        L = L + (z_new * torch.tensor(np.asarray(g_z, dtype=dtype), dtype=tdt)).sum()
    if g_ldj is not None:
        L = L + (ldj * torch.tensor(np.asarray(g_ldj, dtype=dtype), dtype=tdt)).sum()
    gz, gt = torch.autograd.grad(L, (zt, tt), allow_unused=True)
    gz = torch.zeros_like(zt) if gz is None else gz
    gt = torch.zeros_like(tt) if gt is None else gt
    return gz.detach().numpy(), gt.detach().numpy()


def flow_vjp_spread(flow_type, z, tk, d, g_z=None, g_ldj=None, n_perturbed=3, seed=0):
    """``flow_vjp`` in fp64 and the fp32 restatement's largest deviation from it over the
    inputs and ``n_perturbed`` one-ulp perturbations of them (as ``fp32_spread``).
    Returns ``(gz64, gt64, dev_z, dev_t)``."""
    gz64, gt64 = flow_vjp(flow_type, z, tk, d, g_z, g_ldj, np.float64)
    rng = np.random.default_rng(seed)
    dev_z, dev_t = np.zeros_like(gz64), np.zeros_like(gt64)
    z32, t32 = np.asarray(z, np.float32), np.asarray(tk, np.float32)
    for k in range(n_perturbed + 1):
        if k == 0:
            zk, tkk = z32, t32
        else:
            zk = (z32 * (1 + rng.integers(-1, 2, z32.shape) * 2.0 ** -23)).astype(np.float32)
            tkk = (t32 * (1 + rng.integers(-1, 2, t32.shape) * 2.0 ** -23)).astype(np.float32)
        gz32, gt32 = flow_vjp(flow_type, zk, tkk, d, g_z, g_ldj, np.float32)
        dev_z = np.maximum(dev_z, np.abs(gz32.astype(np.float64) - gz64))
        dev_t = np.maximum(dev_t, np.abs(gt32.astype(np.float64) - gt64))
    return gz64, gt64, dev_z, dev_t


def grad_tolerance(ref64: np.ndarray, dev32: np.ndarray, rel: float = 2e-5, cond_factor: float = 8.0,
                   row_scale: bool = True) -> np.ndarray:
    """Per-element bound for an fp32 gradient: ``max(rel * max(1, |ref64|, rowmax|ref64|/64),
    cond_factor * dev32)`` with ``dev32`` the reference's fp32 deviation (``fp32_spread``).
    The row term admits the absolute error an fp32 backward accumulates across a
    chain whose largest gradient entry is large (reverse mode sums products of
    per-flow Jacobians)."""
    a = np.abs(ref64)
    scale = np.maximum(1.0, a)
    if row_scale and a.ndim == 2 and a.shape[-1] > 0:
        scale = np.maximum(scale, a.max(axis=-1, keepdims=True) / 64.0)
    return np.maximum(rel * scale, cond_factor * dev32)
