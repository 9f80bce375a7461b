"""Parity of the HIP path (through the C ABI) against the oracle.

Tolerance (written once, used everywhere): ``oracle.tolerance_bound`` —
``|gpu - ref64| <= max(1e-5 * max(1, |ref64|), 8 * |ref32 - ref64|)`` per sample:
the north-star 1e-5 relative bound (denominator floored at 1 because log_prob
crosses 0), widened only where the reference's own fp32 op order is
ill-conditioned (measured by the fp32 mirror, one run), and a widened sample must
stay within 2x that fp32 deviation (``tests/parity.py``).  Both transcendental modes
(fast = default, precise) must pass.
"""

import math

import numpy as np
import pytest
import torch

from conftest import CHAIN_FIXTURES, FLOW_FIXTURES, load_golden
from parity import check_forward, fp32_sensitivity
from oracle import nfn_oracle as O

pytestmark = pytest.mark.gpu

MODES = ["fast", "precise"]


@pytest.fixture(params=MODES)
def math_mode(request, gpu):
    from normalizingflownetwork_amd import ops

    prev = ops.set_math_mode(request.param)
    yield request.param
    ops.set_math_mode(prev)


assert_within = check_forward


@pytest.mark.parametrize("name", CHAIN_FIXTURES)
def test_chain_fixture(name, math_mode):
    from normalizingflownetwork_amd import ops

    g = load_golden(name)
    lp, s = ops.chain_log_prob(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"]), want_sum=True)
    lp = lp.cpu().numpy()
    assert lp.shape == g["ref64"].shape
    assert_within(lp, g["ref64"], g["ref32"], f"{name}/{math_mode}",
                  sensitivity=fp32_sensitivity(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"])))
    # the fused fp64 sum equals the sum of the returned values
    assert float(s.item()) == pytest.approx(lp.astype(np.float64).sum(), rel=1e-12, abs=1e-9)


def test_c1_log_pdf_with_fused_normalisation(math_mode):
    """BaseEstimator.log_pdf (BaseEstimator.py:77-86) on the reference's own data
    (simulation/dummy_data_gen.py cosine data, captured in the fixture)."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer

    g = load_golden("c1_nfn_radial2_d1")
    dist = InverseNormalizingFlowLayer(("radial", "radial"), 1, True)(g["t"])
    lp = dist.log_prob(g["y_raw"], g["y_mean"], g["y_std"]).cpu().numpy()
    assert_within(lp, g["logpdf64"], g["logpdf32"], "c1 log_pdf")


@pytest.mark.parametrize("name", FLOW_FIXTURES)
def test_single_flow_fixture(name, math_mode):
    from normalizingflownetwork_amd import FLOWS

    g = load_golden(name)
    ftype = name.split("_")[1]
    flow = FLOWS[ftype](g["t"], g["d"])
    z_out, ldj = flow.forward_and_log_det_jacobian(g["z"])
    z_out, ldj = z_out.cpu().numpy(), ldj.cpu().numpy()
    for j in range(g["d"]):
        assert_within(z_out[:, j], g["fwd64"][:, j], g["fwd32"][:, j], f"{name} forward[{j}]")
    assert_within(ldj, g["ldj64"], g["ldj32"], f"{name} fldj")
    # the separate entry points agree with the combined one
    np.testing.assert_array_equal(flow.forward(g["z"]).cpu().numpy(), z_out)
    np.testing.assert_array_equal(flow._forward_log_det_jacobian(g["z"]).cpu().numpy(), ldj)


@pytest.mark.parametrize("name", ["planar", "radial"])
def test_reference_flow_dimension_testing(name, gpu):
    """tests/test_flows.py:10-41 on the HIP path."""
    from normalizingflownetwork_amd import FLOWS, AffineFlow

    batch_size = 10
    for dim in (1, 4):
        cls = FLOWS[name]
        flow = cls(torch.ones((batch_size, cls.get_param_size(dim))), dim)
        reference = AffineFlow(torch.ones((batch_size, AffineFlow.get_param_size(dim))), dim)
        for tensor in ([[0.0] * dim], [[1.0] * dim] * batch_size):
            assert flow.forward(tensor).shape == reference.forward(tensor).shape
            assert flow._forward_log_det_jacobian(tensor).shape == reference._forward_log_det_jacobian(tensor).shape
        tensor = [[1.0] * dim] + ([[0.0] * dim] * (batch_size - 2)) + [[1.0] * dim]
        res = flow.forward(tensor).cpu().numpy()
        assert res[0] == pytest.approx(res[-1], rel=1e-5)
        assert res[1] == pytest.approx(res[-2], rel=1e-5)
        assert not all(res[0] == res[1])
        res = flow._forward_log_det_jacobian(tensor).cpu().numpy()
        assert res[0] == pytest.approx(res[-1], rel=1e-5)
        assert res[1] == pytest.approx(res[-2], rel=1e-5)
        assert not res[0] == pytest.approx(res[1])
        # and the values themselves against the oracle
        g = load_golden(f"flow_{name}_d{dim}")
        np.testing.assert_allclose(flow.forward(tensor).cpu().numpy(), g["sym_fwd64"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(res, g["sym_ldj64"], rtol=1e-5, atol=1e-6)


def test_posterior_fixture(math_mode):
    from normalizingflownetwork_amd import ops

    g = load_golden("posterior_s8_pr5_d1")
    out, s = ops.posterior_lse(g["y"], g["t"], g["flow_types"], 1, True, g["y_mean"], g["y_std"], want_sum=True)
    out = out.cpu().numpy()
    assert_within(out, g["ref64"], g["ref32"], "posterior",
                  sensitivity=fp32_sensitivity(g["y"], g["t"], g["flow_types"], 1, True, g["y_mean"], g["y_std"],
                                               posterior=True))
    assert float(s.item()) == pytest.approx(out.astype(np.float64).sum(), rel=1e-12)


def test_posterior_single_draw_equals_log_pdf(gpu):
    from normalizingflownetwork_amd import ops

    g = load_golden("posterior_s8_pr5_d1")
    t1 = g["t"][:1]
    out, _ = ops.posterior_lse(g["y"], t1, g["flow_types"], 1, True, g["y_mean"], g["y_std"])
    lp, _ = ops.chain_log_prob(g["y"], t1[0], g["flow_types"], 1, True, g["y_mean"], g["y_std"])
    np.testing.assert_allclose(out.cpu().numpy(), lp.cpu().numpy(), rtol=0, atol=2e-6)


def test_chain_bijector_api_matches_fused_kernel(gpu):
    """Invert(Chain) built by _get_bijector, driven flow by flow through the
    single-flow kernel, gives the same log_prob as the fused kernel."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer

    g = load_golden("asym_pra_d3")
    dist = InverseNormalizingFlowLayer(g["flow_types"], 3, True)(torch.as_tensor(g["t"]).cuda())
    chain = dist.bijector.bijector
    x = chain.forward(g["y"])
    ildj = dist.bijector.inverse_log_det_jacobian(g["y"], event_ndims=1)
    lp_steps = (dist.distribution.log_prob(x) + ildj).cpu().numpy()
    lp_fused = dist.log_prob(g["y"]).cpu().numpy()
    np.testing.assert_allclose(lp_steps, lp_fused, rtol=2e-5, atol=2e-5)
    assert_within(lp_fused, g["ref64"], g["ref32"], "fused")


def test_broadcast_and_strided_views(gpu):
    from normalizingflownetwork_amd import ops

    g = load_golden("c2_pr5_d1")
    ft, B = g["flow_types"], 1024
    y, t = torch.as_tensor(g["y"][:B]).cuda(), torch.as_tensor(g["t"][:B]).cuda()
    ref, _ = ops.chain_log_prob(y, t, ft, 1, True)
    # t as a column slice of a wider row buffer (non-contiguous rows, stride 40)
    wide = torch.zeros((B, 40), device="cuda")
    wide[:, 5:37] = t
    got, _ = ops.chain_log_prob(y, wide[:, 5:37], ft, 1, True)
    np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy())
    # y of batch 1 against t of batch B, and t of batch 1 against y of batch B
    got, _ = ops.chain_log_prob(y[:1], t, ft, 1, True)
    full, _ = ops.chain_log_prob(y[:1].expand(B, 1).contiguous(), t, ft, 1, True)
    np.testing.assert_array_equal(got.cpu().numpy(), full.cpu().numpy())
    got, _ = ops.chain_log_prob(y, t[:1], ft, 1, True)
    full, _ = ops.chain_log_prob(y, t[:1].expand(B, 32).contiguous(), ft, 1, True)
    np.testing.assert_array_equal(got.cpu().numpy(), full.cpu().numpy())


@pytest.mark.parametrize("B", [0, 1, 63, 255, 257, 1000])
def test_ragged_and_empty_batches(B, gpu):
    from normalizingflownetwork_amd import ops

    g = load_golden("c2_pr5_d1")
    ft = g["flow_types"]
    lp, s = ops.chain_log_prob(g["y"][:B].reshape(B, 1), g["t"][:B].reshape(B, 32), ft, 1, True, want_sum=True)
    assert lp.shape == (B,)
    assert_within(lp.cpu().numpy(), g["ref64"][:B], g["ref32"][:B], f"B={B}")
    assert float(s.item()) == pytest.approx(float(lp.double().sum().item()), rel=1e-12, abs=1e-12)


def test_radial_identity_known_answer(gpu):
    from normalizingflownetwork_amd import RadialFlow

    rng = np.random.default_rng(3)
    tk = rng.standard_normal((300, 5)).astype(np.float32)
    tk[:, 1] = 0.0
    z = rng.standard_normal((300, 3)).astype(np.float32)
    zo, ldj = RadialFlow(tk, 3).forward_and_log_det_jacobian(z)
    np.testing.assert_allclose(zo.cpu().numpy(), z, atol=1e-6)
    np.testing.assert_allclose(ldj.cpu().numpy(), 0.0, atol=1e-6)


def test_estimators_end_to_end(gpu):
    from normalizingflownetwork_amd.estimators import BayesNormalizingFlowNetwork, NormalizingFlowNetwork
    from normalizingflownetwork_amd.scorers import DummySklearWrapper, mle_log_likelihood_score

    g = load_golden("c1_nfn_radial2_d1")
    x, y = g["x"], g["y_raw"]
    nfn = NormalizingFlowNetwork(n_dims=1, n_flows=2, hidden_sizes=(16, 16), activation="tanh")
    nfn.set_data_normalization(x, y)
    lp = nfn.log_pdf(x, y).cpu().numpy()
    t = nfn.params(x).cpu().numpy()
    ref64 = O.log_pdf(y, t, ("radial", "radial"), 1, True, nfn.y_mean, nfn.y_std)
    ref32 = O.log_pdf(y, t, ("radial", "radial"), 1, True, nfn.y_mean, nfn.y_std, np.float32)
    assert_within(lp, ref64, ref32, "NFN.log_pdf")
    np.testing.assert_allclose(nfn.pdf(x, y).cpu().numpy(), np.exp(lp), rtol=1e-6)
    score = nfn.score(x, y)
    assert score == pytest.approx(ref64.mean(), rel=1e-5)
    assert mle_log_likelihood_score(DummySklearWrapper(nfn), x, y) == pytest.approx(score, rel=1e-12)

    bnn = BayesNormalizingFlowNetwork(n_dims=1, n_flows=2)
    bnn.set_data_normalization(x, y)
    bs = bnn.score(x[:512], y[:512], n_draws=4)
    assert np.isfinite(bs)
    # H = 16: the score runs the fused DenseVariational posterior kernel; the same
    # posterior draws (re-seeded) through the oracle on t = h W + b
    bnn16 = BayesNormalizingFlowNetwork(n_dims=1, n_flows=2, hidden_sizes=(16,))
    bnn16.set_data_normalization(x, y)
    bnn16._draw_gen = None
    s16 = bnn16.score(x[:512], y[:512], n_draws=4)
    bnn16._draw_gen = None
    td = bnn16.params_draws(x[:512], 4).cpu().numpy()
    r64 = O.posterior_lse(y[:512], td, ("radial", "radial"), 1, True, bnn16.y_mean, bnn16.y_std)
    r32 = O.posterior_lse(y[:512], td, ("radial", "radial"), 1, True, bnn16.y_mean, bnn16.y_std, np.float32)
    assert abs(s16 - r64.mean()) <= O.tolerance_bound(r64, r32).mean() + 1e-6


# ---------------------------------------------------------------------------
# Full BASELINE sizes: size-independent properties + an oracle-checked sample.
# ---------------------------------------------------------------------------

FULL = {
    "C2": (("planar", "radial") * 5, 1, 1 << 24),
    "C3": (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8, 1 << 22),
}


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_full_size_properties(cfg, gpu):
    from normalizingflownetwork_amd import ops

    ft, d, B = FULL[cfg]
    P = O.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(22)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = torch.randn((B, P), generator=gen, device="cuda")
    lp1, s1 = ops.chain_log_prob(y, t, ft, d, True, want_sum=True)
    lp2, s2 = ops.chain_log_prob(y, t, ft, d, True, want_sum=True)
    # deterministic, bitwise (no atomics, fixed reduction order)
    assert torch.equal(lp1, lp2) and torch.equal(s1, s2)
    # non-finite values only where the oracle has them too (a log|det| of 0 is a
    # legitimate -inf of the reference math)
    bad = torch.nonzero(~torch.isfinite(lp1)).flatten()
    assert bad.numel() <= 16
    if bad.numel():
        with np.errstate(all="ignore"):
            r64 = O.chain_log_prob(y[bad].cpu().numpy(), t[bad].cpu().numpy(), ft, d, True, np.float64)
        np.testing.assert_array_equal(lp1[bad].cpu().numpy(), r64.astype(np.float32))
    # fused fp64 sum == sum of outputs
    if bad.numel() == 0:
        assert float(s1.item()) == pytest.approx(float(lp1.double().sum().item()), rel=1e-12)
    # sum-only launch gives the same sum
    _, s3 = ops.chain_log_prob(y, t, ft, d, True, want_values=False, want_sum=True)
    assert torch.equal(s1, s3)
    # samples are independent: a permutation of the batch permutes the outputs bitwise
    perm = torch.randperm(B, generator=gen, device="cuda")
    lpp, _ = ops.chain_log_prob(y[perm], t[perm], ft, d, True)
    assert torch.equal(lpp, lp1[perm])
    # the partials-only launch + nfn_reduce_partials_f64 gives the same sum
    L = ops.ChainLauncher(y, t, ft, d, True, write_values=False, fused_sum=False)
    L.launch()
    assert torch.equal(L.finish_sum(), s1)
    # 4096 random samples (spread over the whole batch) against the oracle
    for what, idx in (("sample", torch.randint(0, B, (4096,), generator=gen, device="cuda")),
                      ("tail", torch.arange(B - 300, B, device="cuda"))):
        yn, tn = y[idx].cpu().numpy(), t[idx].cpu().numpy()
        ref64 = O.chain_log_prob(yn, tn, ft, d, True, np.float64)
        ref32 = O.chain_log_prob(yn, tn, ft, d, True, np.float32)
        assert_within(lp1[idx].cpu().numpy(), ref64, ref32, f"{cfg} {what}",
                      sensitivity=fp32_sensitivity(yn, tn, ft, d, True))


def test_full_size_posterior_properties(gpu):
    """C5 shape per GPU (S=64, B=2^17): lse of identical draws == single-draw log_prob."""
    from normalizingflownetwork_amd import ops

    ft = ("planar", "radial") * 5
    S, B = 64, 1 << 17
    gen = torch.Generator(device="cuda").manual_seed(5)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((S, B, 32), generator=gen, device="cuda")
    out, s = ops.posterior_lse(y, t, ft, 1, True, want_sum=True)
    assert torch.isfinite(out).all()
    assert float(s.item()) == pytest.approx(float(out.double().sum().item()), rel=1e-12)
    idx = torch.randint(0, B, (256,), generator=gen, device="cuda")
    tn, yn = t[:, idx].cpu().numpy(), y[idx].cpu().numpy()
    ref64 = O.posterior_lse(yn, tn, ft, 1, True)
    ref32 = O.posterior_lse(yn, tn, ft, 1, True, dtype=np.float32)
    assert_within(out[idx].cpu().numpy(), ref64, ref32, "C5 sample")
    # (the draw-split path vs the single-range path: tests/test_gpu_diag.py, NFN_DIAG build)
    # S copies of one draw: lse - log S == log_prob
    rep = t[:1].expand(S, B, 32).contiguous()
    out_rep, _ = ops.posterior_lse(y, rep, ft, 1, True)
    lp, _ = ops.chain_log_prob(y, t[0], ft, 1, True)
    np.testing.assert_allclose(out_rep.cpu().numpy(), lp.cpu().numpy(), rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("d,K", [(32, 64), (1, 64), (16, 40), (5, 64)])
def test_maximum_sizes(d, K, math_mode):
    """NFN_MAX_DIMS / NFN_MAX_FLOWS (include/nfn.h): the widest parameter rows
    (d=32, 64 flows: P = 4224 floats) run on narrow tiles; forward, posterior and
    backward against the oracle on a ragged batch."""
    from normalizingflownetwork_amd import ops
    from oracle import nfn_grad_oracle as G

    rng = np.random.default_rng(d * 100 + K)
    ft = tuple(rng.choice(["planar", "radial", "affine"], size=K))
    P = O.total_param_size(ft, d, True)
    B = 37
    y = rng.standard_normal((B, d)).astype(np.float32)
    t = (0.3 * rng.standard_normal((B, P))).astype(np.float32)
    lp, s = ops.chain_log_prob(torch.from_numpy(y).cuda(), torch.from_numpy(t).cuda(), ft, d, True,
                               want_sum=True)
    ref64 = O.chain_log_prob(y, t, ft, d, True, np.float64)
    ref32 = O.chain_log_prob(y, t, ft, d, True, np.float32)
    assert_within(lp.cpu().numpy(), ref64, ref32, f"max d={d} K={K}")
    assert abs(s.item() - ref64.sum()) <= 1e-4 * max(1.0, abs(ref64.sum()))
    td = torch.from_numpy(np.stack([t, t[::-1].copy()])).cuda()
    post, _ = ops.posterior_lse(torch.from_numpy(y).cuda(), td, ft, d, True)
    r64 = O.posterior_lse(y, np.stack([t, t[::-1]]), ft, d, True, dtype=np.float64)
    r32 = O.posterior_lse(y, np.stack([t, t[::-1]]), ft, d, True, dtype=np.float32)
    assert_within(post.cpu().numpy(), r64, r32, f"max posterior d={d} K={K}")
    _, gt, gy = ops.chain_log_prob_grad(torch.from_numpy(y).cuda(), torch.from_numpy(t).cuda(), ft, d, True)
    # the gradient gate's standard spread (the fp32 autodiff at the inputs and at three 1-ulp
    # perturbations, nfn_grad_oracle.fp32_spread's default, as in every other gradient check)
    gt64, gy64, dev_t, dev_y = G.fp32_spread(y, t, ft, d, True)
    for got, ref, dev in ((gt.cpu().numpy(), gt64, dev_t), (gy.cpu().numpy(), gy64, dev_y)):
        ok = np.isfinite(ref)
        ratio = np.abs(got - ref)[ok] / G.grad_tolerance(ref, dev)[ok]
        assert ratio.size == 0 or ratio.max() <= 1.0, f"grad d={d} K={K}: max err/bound {ratio.max():.3g}"
    # the margin on the one-perturbation spread this check used before round 4, kept as a
    # regression guard: the round-4 tanh moved d = 32, K = 64 from 0.93 to 1.25
    # of it; a further loss of backward accuracy at the largest sizes must not go unseen
    gt64, gy64, dev_t1, dev_y1 = G.fp32_spread(y, t, ft, d, True, n_perturbed=1)
    for got, ref, dev, what in ((gt.cpu().numpy(), gt64, dev_t1, "d/dt"), (gy.cpu().numpy(), gy64, dev_y1, "d/dy")):
        ok = np.isfinite(ref)
        r1 = np.abs(got - ref)[ok] / G.grad_tolerance(ref, dev)[ok]
        r1max = float(r1.max()) if r1.size else 0.0
        print(f"grad {what} d={d} K={K} [{math_mode}]: max err / one-perturbation bound {r1max:.3f}")
        assert r1max <= 1.3, f"grad {what} d={d} K={K}: {r1max:.3g} of the one-perturbation bound (> 1.3)"


@pytest.mark.parametrize("d", [1, 3, 8])
def test_radial_tiny_alpha_at_center(d, math_mode):
    """alpha = softplus(0.3 a - 2) underflowing in the fast form made
    h = 1 / (alpha + r) infinite at z == gamma; TF's softplus returns exp(x) there and the
    log-density stays finite (RadialFlow.py:24-27, 44-70).  Parity unpinned by the
    reference (no fixture of its own covers it): checked against the oracle."""
    from normalizingflownetwork_amd import ops

    rng = np.random.default_rng(d)
    B = 256
    ft = ("radial", "radial")
    P = O.total_param_size(ft, d, True)
    y = rng.standard_normal((B, d)).astype(np.float32)
    t = (0.3 * rng.standard_normal((B, P))).astype(np.float32)
    # block of flow_types[0] is last (reversed layout): [a, b, gamma(d)]
    a_col, g0 = P - (d + 2), P - d
    # x = 0.3 a - 2 in [-42.8, -8]: the plain fast softplus rounded alpha to 0 below
    # x = -16.6; below x = -44 the reference's own fp32 h' = (-1/y)/y overflows at r = 0
    # (RadialFlow.py:63-66) and its log-density is NaN there too
    t[:, a_col] = np.linspace(-136.0, -20.0, B, dtype=np.float32)
    t[:, g0:] = y  # z_0 == gamma: r = 0
    ref64 = O.chain_log_prob(y, t, ft, d, True, np.float64)
    ref32 = O.chain_log_prob(y, t, ft, d, True, np.float32)
    assert np.isfinite(ref64).all() and np.isfinite(ref32).all()
    lp, _ = ops.chain_log_prob(y, t, ft, d, True)
    lp = lp.cpu().numpy()
    assert np.isfinite(lp).all(), f"{int((~np.isfinite(lp)).sum())} non-finite"
    assert_within(lp, ref64, ref32, f"tiny alpha d={d}")


@pytest.mark.parametrize("name,d", [("c2_pr5_d1", 1), ("asym_pra_d3", 3), ("c3_apr_d8", 8), ("planar_radial_d16", 16)])
def test_chain_bijector_one_launch(name, d, gpu):
    """The Bijector API's Chain over views of one t runs as ONE launch
    (nfn_chain_fwd_ldj_f32): bitwise the flow-by-flow path (same per-flow math, ldj summed
    in application order), and its forward + fldj agree with the fp64 oracle's bijectors
    (DistributionLayers.py:267-278; PlanarFlow.py / RadialFlow.py / AffineFlow.py)."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer, ops
    from normalizingflownetwork_amd.normalizing_flows import Chain

    g = load_golden(name)
    ft, n = g["flow_types"], 777
    t = torch.as_tensor(g["t"][:n]).cuda()
    y = torch.as_tensor(g["y"][:n]).cuda()
    chain = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d)
    fz = chain._fused()
    assert fz is not None
    # the flows own a snapshot of t's flow columns (TF's slices are copies), whose rows start
    # (-W) mod 4 lead columns left of the first block on a 16-byte boundary; the fused view
    # starts at that row start, so the rows stream whole (d = 1: the wave1 pipeline; d = 8:
    # the lane-group one)
    W = t.shape[1] - 2 * d
    lead = (-W) % 4
    assert fz[1].data_ptr() == chain.bijectors[0].params.data_ptr() - 4 * lead and min(fz[2]) == lead
    assert fz[1].stride(0) == W + lead and fz[1].data_ptr() % 16 == 0
    launches = []
    real = ops.chain_forward_ldj

    def counting(*a, **k):
        launches.append(1)
        return real(*a, **k)

    ops.chain_forward_ldj = counting
    try:
        z, ldj = chain.forward_and_log_det_jacobian(y)
        assert torch.equal(chain.forward(y), z) and torch.equal(chain.forward_log_det_jacobian(y, event_ndims=1), ldj)
    finally:
        ops.chain_forward_ldj = real
    assert len(launches) == 3
    # flow by flow through the single-flow kernel (a Chain of copies: no shared storage);
    # bitwise the one-launch result where both run the generic per-flow math (the tile
    # kernel: d = 3); d = 1 (wave1) and d = 8, 16 (lane groups over the snapshot's float4
    # rows) run the fast-math chain forms — all are held to the oracle below
    steps = Chain([type(b)(b.params.clone(), d) for b in chain.bijectors])
    assert steps._fused() is None
    z1, ldj1 = steps.forward_and_log_det_jacobian(y)
    if d == 3:
        assert torch.equal(z, z1) and torch.equal(ldj, ldj1)
    # against the oracle's flows applied in the same order (fp64 truth, fp32 op-by-op mirror
    # for the conditioning term), through the forward tolerance
    def oracle(t_, y_, dt):
        _, blocks = O.split_params(t_.astype(dt), ft, d, True)
        zr, lr = y_.astype(dt), np.zeros(len(y_), dt)
        for f, tk in zip(ft, blocks):
            zr, l = O.flow_forward_fldj(f, zr, tk, d)
            lr = lr + l
        return zr.astype(np.float64), lr.astype(np.float64)

    t0, y0 = g["t"][:n], g["y"][:n]
    z64, l64 = oracle(t0, y0, np.float64)
    z32, l32 = oracle(t0, y0, np.float32)
    for tag, zz, ll in (("one launch", z, ldj), ("flow by flow", z1, ldj1)):
        check_forward(ll.cpu().numpy(), l64, l32, f"bijector {name} {tag} ldj", kind="bijector")
        check_forward(zz.cpu().numpy(), z64, z32, f"bijector {name} {tag} z", kind="bijector")


@pytest.mark.parametrize("ft,d,B", [(("planar", "radial"), 1, 65), (("radial",) * 14, 1, 1000),
                                    (("affine", "planar"), 1, 1), (("planar", "radial") * 2, 4, 63),
                                    (("radial", "planar", "affine"), 8, 257), (("planar",) * 20, 1, 130)])
def test_chain_bijector_shapes(ft, d, B, gpu):
    """The one-launch Chain over ragged batches and every kernel form it takes (d = 1 wave1
    with Q = 2 / 16, a 16+-flow chain on the tile kernel, the d >= 4 lane groups): against the
    flow-by-flow path, both against the oracle at the forward tolerance."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer
    from normalizingflownetwork_amd.normalizing_flows import Chain

    rng = np.random.default_rng(B + d)
    P = O.total_param_size(ft, d, True)
    t = torch.from_numpy((0.5 * rng.standard_normal((B, P))).astype(np.float32)).cuda()
    y = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).cuda()
    chain = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d)
    assert chain._fused() is not None
    z, ldj = chain.forward_and_log_det_jacobian(y)
    steps = Chain([type(b)(b.params.clone(), d) for b in chain.bijectors])
    z1, ldj1 = steps.forward_and_log_det_jacobian(y)

    def oracle(dt):
        _, blocks = O.split_params(t.cpu().numpy().astype(dt), ft, d, True)
        zr, lr = y.cpu().numpy().astype(dt), np.zeros(B, dt)
        for f, tk in zip(ft, blocks):
            zr, l = O.flow_forward_fldj(f, zr, tk, d)
            lr = lr + l
        return zr.astype(np.float64), lr.astype(np.float64)

    z64, l64 = oracle(np.float64)
    z32, l32 = oracle(np.float32)
    for tag, zz, ll in (("one launch", z, ldj), ("flow by flow", z1, ldj1)):
        assert zz.shape == (B, d) and ll.shape == (B,)
        check_forward(ll.cpu().numpy(), l64, l32, f"bijector shapes {ft[:3]} d={d} B={B} {tag} ldj", kind="bijector")
        check_forward(zz.cpu().numpy(), z64, z32, f"bijector shapes {ft[:3]} d={d} B={B} {tag} z", kind="bijector")
