"""Sampling through the inverted flows (nfn_chain_sample_f32).

Size-independent properties: the fp64 oracle's forward chain maps each sample back
onto loc + scale * eps (inverse then forward is the identity); the sample's
log-density equals the forward kernel's log_prob of the sample; and a 2^20-draw
sample from one fixed parameter row matches the CDF integrated from the density
(density-grid kernel)."""

import numpy as np
import pytest
import torch

from oracle import nfn_oracle as O

pytestmark = pytest.mark.gpu

CASES = [(("planar", "radial") * 5, 1), (("radial", "radial"), 1), (("affine", "planar", "radial"), 3),
         (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8), (("planar",) * 6, 2)]


def _base(t, d, dt=np.float64):
    loc = t[:, :d].astype(dt)
    scale = dt(1e-3) + O.softplus(dt(np.log(np.expm1(1.0))) + dt(0.1) * t[:, d:2 * d].astype(dt))
    return loc, scale


@pytest.mark.parametrize("ft,d", CASES)
def test_inverse_then_forward_is_identity(ft, d, gpu):
    from normalizingflownetwork_amd import ops

    rng = np.random.default_rng(len(ft) * 10 + d)
    B = 4099
    P = O.total_param_size(ft, d, True)
    t = (0.5 * rng.standard_normal((B, P))).astype(np.float32)
    eps = rng.standard_normal((B, d)).astype(np.float32)
    y, lp = ops.chain_sample(torch.from_numpy(eps).cuda(), torch.from_numpy(t).cuda(), ft, d, True)
    y = y.cpu().numpy().astype(np.float64)
    # forward chain of the sample in fp64 (the oracle) lands on loc + scale * eps
    base, blocks = O.split_params(t.astype(np.float64), ft, d, True)
    z = y.copy()
    zs, ls = [np.abs(y).max(1)], []
    for f, tk in zip(ft, blocks):
        z, l = O.flow_forward_fldj(f, z, tk, d)
        zs.append(np.abs(z).max(1))
        ls.append(l)
    loc, scale = _base(t, d)
    target = loc + scale * eps
    # per-sample bound from the inverse walk's own rounding: each step rounds its z_k
    # once (half an ulp per coordinate), and the forward map from z_k to z_K scales that
    # by |J_{k->K}| (per coordinate exp(sum_{j>=k} fldj_j / d)); summed over the steps.
    # Measured (tools/sample_err.py, 2^16 samples per case): max err / bound 2.4-5.5,
    # 99.9 % quantile <= 1.8 — a step stopped short of convergence lands far above it.
    tail, gain = np.zeros(B), np.maximum(1.0, zs[-1])
    for k in range(len(ls) - 1, -1, -1):
        tail = tail + ls[k]
        gain = gain + np.exp(tail / d) * np.maximum(1.0, zs[k])
    err = np.abs(z - target).max(1)
    bound = 16.0 * 2.0 ** -24 * gain  # 3x the largest measured ratio
    assert (err <= bound).all(), float((err / bound).max())
    # the sample's log-density is the forward kernel's log_prob of the sample
    lp_fwd, _ = ops.chain_log_prob(torch.from_numpy(y.astype(np.float32)).cuda(), torch.from_numpy(t).cuda(), ft, d,
                                   True)
    diff = (lp.cpu() - lp_fwd.cpu()).abs() / lp_fwd.cpu().abs().clamp(min=1.0)
    assert torch.quantile(diff, 0.999) < 1e-4


def test_samples_follow_the_density(gpu):
    """One fixed parameter row of the C2 chain: the empirical CDF of 2^20 samples vs
    the CDF integrated from the density on a fine grid (KS distance)."""
    from normalizingflownetwork_amd import ops

    ft, d = ("planar", "radial") * 5, 1
    P = O.total_param_size(ft, d, True)
    t1 = (0.8 * np.random.default_rng(3).standard_normal((1, P))).astype(np.float32)
    n = 1 << 20
    eps = torch.randn((n, 1), generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
    y, _ = ops.chain_sample(eps, torch.from_numpy(t1).cuda(), ft, d, True, want_log_prob=False)
    ys = np.sort(y.cpu().numpy().reshape(-1).astype(np.float64))
    lo, hi = ys[0] - 1.0, ys[-1] + 1.0
    grid = np.linspace(lo, hi, 200001)
    dens = np.exp(ops.chain_log_prob_grid(torch.from_numpy(grid.astype(np.float32)[:, None]).cuda(),
                                          torch.from_numpy(t1).cuda(), ft, d, True).cpu().numpy()[:, 0].astype(np.float64))
    cdf = np.concatenate([[0.0], np.cumsum(0.5 * (dens[1:] + dens[:-1]) * np.diff(grid))])
    assert abs(cdf[-1] - 1.0) < 2e-3  # the density integrates to one
    ecdf_at = np.searchsorted(ys, grid, side="right") / n
    ks = np.max(np.abs(ecdf_at - cdf / cdf[-1]))
    assert ks < 3e-3, ks


def test_distribution_sample_shapes(gpu):
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer

    layer = InverseNormalizingFlowLayer(("planar", "radial"), 2, True)
    t = np.random.default_rng(0).standard_normal((7, layer.get_total_param_size())).astype(np.float32)
    dist = layer(t)
    assert tuple(dist.sample().shape) == (7, 2)
    s, lp = dist.sample_and_log_prob((3,), seed=11)
    assert tuple(s.shape) == (3, 7, 2) and tuple(lp.shape) == (3, 7)
    again, _ = dist.sample_and_log_prob((3,), seed=11)
    assert torch.equal(s, again)
    np.testing.assert_allclose(lp.cpu().numpy(), dist.log_prob(s.reshape(3, 7, 2)).cpu().numpy(), rtol=1e-4, atol=1e-4)
