"""Pins the CPU oracle (oracle/nfn_oracle.py) before it is trusted as the checker.

The reference's own tests hold no numeric log_prob values, so
the oracle is pinned by:
  * an independent torch-fp64 restatement of each bijector's FORWARD map whose
    log|det J| comes from autodiff (torch.func.jacrev), for d in {1, 3, 8};
  * analytic known-answer cases;
  * the reference tests' relational properties (tests/test_flows.py:31-41,
    tests/test_distribution_layers.py:16-24, 234-249);
  * re-deriving every committed golden fixture.
"""

import math

import numpy as np
import pytest
import torch

from conftest import CHAIN_FIXTURES, FLOW_FIXTURES, load_golden
from oracle import nfn_oracle as O

F64 = torch.float64


# ---- independent torch restatement of the forward maps (fp64) -------------------

def t_softplus(x):
    return torch.nn.functional.softplus(x)


def t_planar(z, tk, d):
    u, w, b = tk[:d], tk[d:2 * d] + 1, tk[2 * d]
    wtu = (w * u).sum()
    m = -1 + t_softplus(wtu) + 1e-5
    uh = u + (m - wtu) * w / ((w * w).sum() + 1e-9)
    return z + uh * torch.tanh((w * z).sum() + b)


def t_radial(z, tk, d):
    a = t_softplus(0.3 * tk[0] - 2)
    be = t_softplus(0.1 * tk[1] + math.log(math.e - 1)) - 1
    g = tk[2:2 + d]
    r = (z - g).abs().sum()
    return z + a * be / (a + r) * (z - g)


def t_affine(z, tk, d):
    return z * (1 + tk[d:2 * d]) + tk[:d]


T_FWD = {"planar": t_planar, "radial": t_radial, "affine": t_affine}


def autodiff_fldj(ftype, z, tk, d):
    out = []
    for zi, ti in zip(torch.as_tensor(z, dtype=F64), torch.as_tensor(tk, dtype=F64)):
        J = torch.func.jacrev(lambda v: T_FWD[ftype](v, ti, d))(zi)
        out.append(torch.linalg.slogdet(J)[1].item())
    return np.array(out)


@pytest.mark.parametrize("ftype", ["planar", "radial", "affine"])
@pytest.mark.parametrize("d", [1, 3, 8])
def test_fldj_matches_autodiff_jacobian(ftype, d):
    rng = np.random.default_rng(1000 + d)
    ps = O.param_size(ftype, d)
    tk = rng.standard_normal((64, ps))
    z = rng.standard_normal((64, d)) * 1.5
    fwd, fldj = O.flow_forward_fldj(ftype, z, tk, d)
    ref_fwd = np.stack([T_FWD[ftype](torch.as_tensor(zi, dtype=F64), torch.as_tensor(ti, dtype=F64), d).numpy()
                        for zi, ti in zip(z, tk)])
    np.testing.assert_allclose(fwd, ref_fwd, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(fldj, autodiff_fldj(ftype, z, tk, d), rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("d", [1, 3, 8])
def test_chain_log_prob_matches_autodiff(d):
    """Whole chain incl. the reversed param layout and the base density."""
    flows = ("planar", "radial", "affine", "radial")
    rng = np.random.default_rng(77 + d)
    P = O.total_param_size(flows, d, True)
    t = rng.standard_normal((32, P))
    y = rng.standard_normal((32, d))
    lp = O.chain_log_prob(y, t, flows, d, True, np.float64)
    ref = []
    for yi, ti in zip(y, t):
        # reversed layout: after the 2d base params come blocks of flows[-1], ..., flows[0]
        off = 2 * d
        blocks = {}
        for k in reversed(range(len(flows))):
            ps = O.param_size(flows[k], d)
            blocks[k] = torch.as_tensor(ti[off:off + ps], dtype=F64)
            off += ps
        z = torch.as_tensor(yi, dtype=F64)
        ldj = 0.0
        for k, f in enumerate(flows):
            J = torch.func.jacrev(lambda v: T_FWD[f](v, blocks[k], d))(z)
            ldj += torch.linalg.slogdet(J)[1].item()
            z = T_FWD[f](z, blocks[k], d)
        loc = torch.as_tensor(ti[:d], dtype=F64)
        s = 1e-3 + t_softplus(math.log(math.e - 1) + 0.1 * torch.as_tensor(ti[d:2 * d], dtype=F64))
        base = torch.distributions.Normal(loc, s).log_prob(z).sum().item()
        ref.append(base + ldj)
    np.testing.assert_allclose(lp, np.array(ref), rtol=1e-9, atol=1e-9)


def test_known_answers():
    d = 3
    rng = np.random.default_rng(5)
    z = rng.standard_normal((16, d))
    # radial with t[1] = 0 -> beta = softplus(log(e-1)) - 1 = 0 -> identity, fldj = 0
    tk = rng.standard_normal((16, d + 2))
    tk[:, 1] = 0.0
    f, l = O.flow_forward_fldj("radial", z, tk, d)
    np.testing.assert_allclose(f, z, atol=1e-15)
    np.testing.assert_allclose(l, 0.0, atol=1e-15)
    # affine with t = 0 -> identity, fldj = 0
    f, l = O.flow_forward_fldj("affine", z, np.zeros((16, 2 * d)), d)
    np.testing.assert_allclose(f, z)
    np.testing.assert_allclose(l, 0.0)
    # affine-only chain with a fixed base: log_prob = log N(y; 0, I)
    lp = O.chain_log_prob(z, np.zeros((16, 2 * d)), ("affine",), d, False)
    np.testing.assert_allclose(lp, -0.5 * (z ** 2).sum(1) - 0.5 * d * math.log(2 * math.pi), rtol=1e-14)
    # planar, d=1, u=0, w=1 (t_w=0), b=0, z=0: wtu=0, m=log2-1+1e-5,
    # u_hat=m/(1+1e-9), f(0)=0, fldj=log(1+u_hat)
    f, l = O.flow_forward_fldj("planar", np.zeros((1, 1)), np.zeros((1, 3)), 1)
    m = math.log(2.0) - 1 + 1e-5
    assert f[0, 0] == 0.0
    assert l[0] == pytest.approx(math.log(1 + m / (1 + 1e-9)), rel=1e-13)


def test_reference_param_sizes():
    # tests/test_distribution_layers.py:65-73
    assert O.total_param_size(("planar", "radial", "affine"), 1, False) == 3 + 3 + 2
    assert O.total_param_size(("planar", "radial", "affine"), 3, True) == (3 + 3 + 1) + (3 + 1 + 1) + (3 + 3) + (3 + 3)
    with pytest.raises(AssertionError):
        O.split_params(np.zeros((10, 8)), ("planar", "radial"), 2, False)  # :248-249


def test_reversed_layout_is_observable():
    """Asymmetric chain: swapping the block order must change the result
    (a symmetric chain would hide a wrong layout, SURVEY.md §7 'Hard parts')."""
    g = load_golden("asym_pra_d3")
    ft = g["flow_types"]
    t = g["t"].astype(np.float64)
    d = g["d"]
    good = O.chain_log_prob(g["y"], t, ft, d, True)
    # interpret the same row with forward-order blocks: must differ
    wrong = O.chain_log_prob(g["y"], t, tuple(reversed(ft)), d, True)
    assert np.abs(good - wrong).max() > 1e-2


@pytest.mark.parametrize("ftype", ["planar", "radial"])
def test_reference_symmetry_properties(ftype):
    """tests/test_flows.py:31-41 — t = ones, batch [1, 0 x 8, 1]."""
    for d in (1, 4):
        g = load_golden(f"flow_{ftype}_d{d}")
        res, ldj = g["sym_fwd64"], g["sym_ldj64"]
        np.testing.assert_allclose(res[0], res[-1], rtol=1e-5)
        np.testing.assert_allclose(res[1], res[-2], rtol=1e-5)
        assert not np.all(res[0] == res[1])
        assert ldj[0] == pytest.approx(ldj[-1], rel=1e-5)
        assert ldj[1] == pytest.approx(ldj[-2], rel=1e-5)
        assert not ldj[0] == pytest.approx(ldj[1])


@pytest.mark.parametrize("name", CHAIN_FIXTURES)
def test_golden_chain_fixtures_rederive(name):
    g = load_golden(name)
    r64 = O.chain_log_prob(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"]), np.float64)
    np.testing.assert_array_equal(r64, g["ref64"])
    r32 = O.chain_log_prob(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"]), np.float32)
    np.testing.assert_array_equal(r32, g["ref32"])
    # the fp32 op-order mirror stays within the north-star bound on well-conditioned samples
    bound = O.tolerance_bound(g["ref64"], g["ref32"])
    assert np.all(np.abs(g["ref32"] - g["ref64"]) <= bound)


def test_golden_c1_logpdf():
    g = load_golden("c1_nfn_radial2_d1")
    lp = O.log_pdf(g["y_raw"], g["t"], g["flow_types"], 1, True, g["y_mean"], g["y_std"])
    np.testing.assert_array_equal(lp, g["logpdf64"])
    # log_pdf = log_prob(y_circ) - log(y_std)
    np.testing.assert_allclose(lp, g["ref64"] - np.log(np.float64(g["y_std"][0])), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", FLOW_FIXTURES)
def test_golden_flow_fixtures_rederive(name):
    g = load_golden(name)
    ftype = name.split("_")[1]
    f, l = O.flow_forward_fldj(ftype, g["z"].astype(np.float64), g["t"].astype(np.float64), g["d"])
    np.testing.assert_array_equal(f, g["fwd64"])
    np.testing.assert_array_equal(l, g["ldj64"])


def test_golden_posterior_rederive():
    g = load_golden("posterior_s8_pr5_d1")
    r = O.posterior_lse(g["y"], g["t"], g["flow_types"], 1, True, g["y_mean"], g["y_std"])
    np.testing.assert_array_equal(r, g["ref64"])
    # scipy's logsumexp (scorers.py:25) agrees
    from scipy.special import logsumexp

    scores = np.stack([O.log_pdf(g["y"], g["t"][s], g["flow_types"], 1, True, g["y_mean"], g["y_std"])
                       for s in range(g["t"].shape[0])])
    np.testing.assert_allclose(r, logsumexp(scores, axis=0) - np.log(scores.shape[0]), rtol=1e-12)


def test_broadcast_y_batch1():
    """tests/test_flows.py:22-29: y of batch 1 against params of batch B."""
    g = load_golden("bcast_y1_pr_d2")
    assert g["y"].shape[0] == 1 and g["t"].shape[0] == 256
    full = O.chain_log_prob(np.repeat(g["y"], 256, 0), g["t"], g["flow_types"], 2, True)
    np.testing.assert_array_equal(full, g["ref64"])
