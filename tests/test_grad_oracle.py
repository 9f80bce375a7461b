"""Pin the backward oracle (oracle/nfn_grad_oracle.py): its forward equals the
numpy fp64 restatement, and its autodiff gradients equal central finite
differences of that numpy forward (the training path)."""

import numpy as np
import pytest

from conftest import CHAIN_FIXTURES, load_golden
from oracle import nfn_grad_oracle as G
from oracle import nfn_oracle as O

CASES = [
    (("planar", "radial") * 5, 1, True),
    (("radial", "radial"), 1, True),
    (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8, True),
    (("planar", "radial", "affine"), 3, False),
    (("radial", "planar"), 2, True),
    ((), 2, True),
]


def _inputs(ft, d, tr, B=6, seed=3):
    rng = np.random.default_rng(seed)
    P = O.total_param_size(ft, d, tr)
    return rng.standard_normal((B, d)), rng.standard_normal((B, P))


@pytest.mark.parametrize("ft,d,tr", CASES)
def test_forward_matches_numpy_oracle(ft, d, tr):
    y, t = _inputs(ft, d, tr)
    lp, _, _ = G.chain_log_prob_grad(y, t, ft, d, tr)
    np.testing.assert_allclose(lp, O.chain_log_prob(y, t, ft, d, tr), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("ft,d,tr", CASES)
@pytest.mark.parametrize("norm", [False, True])
def test_gradients_match_finite_differences(ft, d, tr, norm):
    y, t = _inputs(ft, d, tr, B=4)
    ym = np.linspace(-0.3, 0.2, d) if norm else None
    ys = np.linspace(0.7, 1.6, d) if norm else None
    _, gt, gy = G.chain_log_prob_grad(y, t, ft, d, tr, ym, ys)
    f = (lambda yy, tt: O.log_pdf(yy, tt, ft, d, tr, ym, ys))
    h = 1e-6
    for j in range(t.shape[1]):
        tp, tm = t.copy(), t.copy()
        tp[:, j] += h
        tm[:, j] -= h
        fd = (f(y, tp) - f(y, tm)) / (2 * h)
        np.testing.assert_allclose(gt[:, j], fd, rtol=1e-6, atol=1e-6, err_msg=f"dt[{j}]")
    for j in range(d):
        yp, ym_ = y.copy(), y.copy()
        yp[:, j] += h
        ym_[:, j] -= h
        fd = (f(yp, t) - f(ym_, t)) / (2 * h)
        np.testing.assert_allclose(gy[:, j], fd, rtol=1e-6, atol=1e-6, err_msg=f"dy[{j}]")


def test_upstream_gradient_scales_rows():
    ft, d, tr = ("planar", "radial"), 1, True
    y, t = _inputs(ft, d, tr)
    g = np.linspace(-2, 3, y.shape[0])
    _, gt1, gy1 = G.chain_log_prob_grad(y, t, ft, d, tr)
    _, gtg, gyg = G.chain_log_prob_grad(y, t, ft, d, tr, g_out=g)
    np.testing.assert_allclose(gtg, gt1 * g[:, None], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(gyg, gy1 * g[:, None], rtol=1e-12, atol=1e-14)


def test_broadcast_y_gives_per_sample_rows():
    ft, d, tr = ("planar", "radial"), 2, True
    y, t = _inputs(ft, d, tr)
    _, gt_b, gy_b = G.chain_log_prob_grad(y[:1], t, ft, d, tr)
    _, gt_f, gy_f = G.chain_log_prob_grad(np.repeat(y[:1], len(t), 0), t, ft, d, tr)
    np.testing.assert_array_equal(gt_b, gt_f)
    np.testing.assert_array_equal(gy_b, gy_f)


@pytest.mark.parametrize("name", ["c2_pr5_d1", "asym_pra_d8"])
def test_fixture_forward_consistent(name):
    fx = load_golden(name)
    lp, _, _ = G.chain_log_prob_grad(fx["y"][:64], fx["t"][:64], fx["flow_types"], fx["d"], bool(fx["trainable"]))
    np.testing.assert_allclose(lp, fx["ref64"][:64], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("ft,d,tr", CASES)
def test_closed_form_backward(ft, d, tr):
    """The closed-form reverse pass the HIP kernels implement (tests/analytic_grad.py)
    equals the autodiff oracle in fp64."""
    from analytic_grad import chain_grad

    y, t = _inputs(ft, d, tr, B=32, seed=11)
    ym, ys = np.linspace(-0.3, 0.2, d), np.linspace(0.7, 1.6, d)
    for args in ((None, None), (ym, ys)):
        lp, gt, gy = chain_grad(y, t, ft, d, tr, *args)
        lp0, gt0, gy0 = G.chain_log_prob_grad(y, t, ft, d, tr, *args)
        np.testing.assert_allclose(lp, lp0, rtol=1e-11, atol=1e-11)
        np.testing.assert_allclose(gt, gt0, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(gy, gy0, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("name", CHAIN_FIXTURES)
def test_closed_form_backward_fp32_within_tolerance(name):
    """The kernels' closed-form reverse pass evaluated in fp32 (numpy emulation, same
    accuracy-preserving forms: 1 - tanh^2 = 4E/(1+E)^2, w.u_hat = m - c 1e-9/n)
    stays inside the gradient tolerance the GPU tests use — with margin."""
    from analytic_grad import chain_grad

    fx = load_golden(name)
    ft, d, tr = fx["flow_types"], fx["d"], bool(fx["trainable"])
    y, t = fx["y"][:512], fx["t"][:512]
    gt64, gy64, dev_t, dev_y = G.fp32_spread(y, t, ft, d, tr)
    with np.errstate(all="ignore"):
        _, gt, gy = chain_grad(y, t, ft, d, tr, dtype=np.float32)
    for got, ref, dev in ((gt, gt64, dev_t), (gy, gy64, dev_y)):
        ok = np.isfinite(ref)
        ratio = np.abs(got - ref)[ok] / G.grad_tolerance(ref, dev)[ok]
        assert ratio.size == 0 or ratio.max() < 0.6, (name, float(ratio.max()))


def test_autodiff_oracle_at_exact_zero_arguments():
    """Softplus arguments that are exactly 0 (planar u = 0, w.u = 0; reached on dyadic
    inputs such as the full-size Dense backward test's): the autodiff oracle's softplus
    gradient is TF's SoftplusGrad = sigmoid(0) = 0.5 there (its max / abs value form alone
    would autodiff to 1), so it equals the closed form at every row, exact zeros included."""
    from analytic_grad import chain_grad

    ft = ("planar", "radial") * 5
    rng = np.random.default_rng(3)
    h = (rng.integers(-8, 9, (2048, 16)) / 8).astype(np.float32)
    W = (rng.integers(-16, 17, (16, 32)) / 64).astype(np.float32)
    b = (rng.integers(-8, 9, 32) / 64).astype(np.float32)
    t = (h @ W + b).astype(np.float32)
    assert (t == 0).sum() > 50
    y = rng.standard_normal((2048, 1)).astype(np.float32)
    _, gt0, gy0 = G.chain_log_prob_grad(y, t, ft, 1, True)
    _, gt, gy = chain_grad(y, t, ft, 1, True)
    np.testing.assert_allclose(gt0, gt, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(gy0, gy, rtol=1e-9, atol=1e-9)
