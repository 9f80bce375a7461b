"""Training on the GPU through the fused backward: the
reference's estimator tests that call ``fit`` (tests/test_ml_estimator.py,
tests/test_noise_reg.py), restated with numpy data of the same distributions, and
an end-to-end check of the MLP weight gradients against the autodiff oracle."""

import numpy as np
import pytest
import torch

from oracle import nfn_grad_oracle as G

pytestmark = pytest.mark.gpu


def _nfn(*args, **kw):
    from normalizingflownetwork_amd import NormalizingFlowNetwork

    return NormalizingFlowNetwork(*args, **kw)


def test_ml_dims_after_fit(gpu):
    """tests/test_ml_estimator.py:19-40, 86-101 (NFN rows)."""
    x = np.linspace(-1, 1, 10).reshape((10, 1))
    m = _nfn(1, n_flows=1, hidden_sizes=(2, 2), trainable_base_dist=False)
    m.fit(x, x, epochs=1, verbose=0)
    out = m(x)
    assert out.event_shape == [1] and out.batch_shape == [10]
    assert tuple(out.log_prob([[0.0]]).shape) == (10,)
    x3 = np.linspace([[-1]] * 3, [[1]] * 3, 10).reshape((10, 3))
    m3 = _nfn(3, n_flows=1, hidden_sizes=(2, 2), trainable_base_dist=True)
    m3.fit(x3, x3, epochs=1, verbose=0)
    out3 = m3(x3)
    assert out3.event_shape == [3] and out3.batch_shape == [10]
    assert tuple(out3.log_prob([[0.0] * 3]).shape) == (10,)


def test_fit_rejects_vectors(gpu):
    m = _nfn(1, n_flows=1)
    with pytest.raises(AssertionError):
        m.fit(np.zeros(10), np.zeros(10))


def test_weight_gradients_match_autodiff_oracle(gpu):
    """One training loss: MLP weight gradients with the fused backward kernel vs
    fp64 autodiff of the oracle's op sequence through the same MLP."""
    from normalizingflownetwork_amd import ops

    ft, d = ("planar", "radial", "radial"), 1
    m = _nfn(d, flow_types=ft, hidden_sizes=(10, 10), trainable_base_dist=True, n_dims_x=1)
    rng = np.random.default_rng(4)
    x = rng.standard_normal((256, 1)).astype(np.float32)
    y = (np.sin(2 * x) + 0.3 * rng.standard_normal((256, 1))).astype(np.float32)
    m._mlp.to(gpu)
    ws = [w.detach().requires_grad_(True) for w in m._mlp.weights + m._mlp.biases]
    nw = len(m._mlp.weights)

    def mlp(xx, params):
        h = xx
        for i in range(nw):
            h = h @ params[i] + params[nw + i]
            if i < nw - 1:
                h = torch.relu(h)
        return h

    t = mlp(torch.from_numpy(x).to(gpu), ws)
    loss = -ops.log_prob(torch.from_numpy(y).to(gpu), t, ft, d, True).mean()
    loss.backward()
    got = [w.grad.double().cpu() for w in ws]
    ws64 = [w.detach().double().cpu().requires_grad_(True) for w in ws]
    t64 = mlp(torch.from_numpy(x).double(), ws64)
    lp64 = G.chain_log_prob_torch(torch.from_numpy(y).double(), t64, ft, d, True)
    (-lp64.mean()).backward()
    for g, w in zip(got, ws64):
        torch.testing.assert_close(g, w.grad, rtol=2e-4, atol=2e-5)


def _sinusoid(n, rng):
    x = np.linspace(-3, 3, n, dtype=np.float32).reshape((n, 1))
    y = (5 * np.sin(2 * x) + np.abs(x) * rng.standard_normal((n, 1))).astype(np.float32)
    return x, y


def _sinusoid_pdf(x, y):
    s = np.abs(x)
    return np.exp(-0.5 * ((y - 5 * np.sin(2 * x)) / s) ** 2) / (np.sqrt(2 * np.pi) * s)


def test_ml_nf_fitting_sinusoid(gpu):
    """tests/test_ml_estimator.py:43-59, 104-107: NFN(1, n_flows=3, (10, 10)) fitted
    800 epochs on 400 heteroscedastic sinusoid points; mean |pdf - true pdf| < 0.45."""
    rng = np.random.default_rng(22)
    m = _nfn(1, n_flows=3, hidden_sizes=(10, 10), trainable_base_dist=True)
    x, y = _sinusoid(400, rng)
    hist = m.fit(x, y, epochs=800, verbose=0)
    assert hist["loss"][-1] < hist["loss"][0]
    xt, yt = _sinusoid(1000, rng)
    pdf = m.pdf(xt, yt).cpu().numpy().reshape(-1)
    score = np.sum(np.abs(pdf - _sinusoid_pdf(xt, yt).reshape(-1))) / 1000.0
    assert score < 0.45, score


def test_ml_nf_fitting_bimodal(gpu):
    """tests/test_ml_estimator.py:62-83, 108: equal mixture of N(3, 0.5) and N(-3, 0.5)
    independent of x; mean |pdf - true pdf| < 0.1012."""
    rng = np.random.default_rng(22)

    def data(n):
        x = np.linspace(-3, 3, n, dtype=np.float32).reshape((n, 1))
        c = rng.integers(0, 2, (n, 1))
        y = (np.where(c == 0, 3.0, -3.0) + 0.5 * rng.standard_normal((n, 1))).astype(np.float32)
        return x, y

    def true_pdf(y):
        n = lambda mu: np.exp(-0.5 * ((y - mu) / 0.5) ** 2) / (np.sqrt(2 * np.pi) * 0.5)  # noqa: E731
        return 0.5 * n(3.0) + 0.5 * n(-3.0)

    m = _nfn(1, n_flows=3, hidden_sizes=(10, 10), trainable_base_dist=True)
    x, y = data(400)
    m.fit(x, y, epochs=800, verbose=0)
    xt, yt = data(1000)
    score = np.sum(np.abs(m.pdf(xt, yt).cpu().numpy().reshape(-1) - true_pdf(yt).reshape(-1))) / 1000.0
    assert score < 0.1012, score


def test_noise_off_at_evaluation(gpu):
    """tests/test_noise_reg.py:13-33: with heavy noise regularisation the fitted
    model's pdf is deterministic at evaluation (noise only while training), and a
    lightly regularised model scores higher than the over-regularised one."""
    rng = np.random.default_rng(22)
    x, y = _sinusoid(300, rng)
    heavy = _nfn(1, n_flows=2, hidden_sizes=(16, 16), noise_reg=("fixed_rate", 3.0), trainable_base_dist=True)
    heavy.fit(x, y, epochs=700, verbose=0)
    xt, yt = _sinusoid(300, rng)
    p1 = heavy.pdf(xt, yt).cpu().numpy()
    p2 = heavy.pdf(xt, yt).cpu().numpy()
    assert np.array_equal(p1, p2)
    light = _nfn(1, n_flows=2, hidden_sizes=(16, 16), noise_reg=("rule_of_thumb", 0.1), trainable_base_dist=True)
    light.fit(x, y, epochs=700, verbose=0)
    assert light.pdf(xt, yt).sum().item() / 700.0 > p1.sum() / 700.0


def test_weight_gradients_fused_dense_match_autodiff_oracle(gpu):
    """The same training loss through ops.log_prob_dense (output Dense layer fused into
    the chain forward and backward, t never materialised) with H = 16: every MLP weight
    gradient against fp64 autodiff of the oracle's op sequence."""
    from normalizingflownetwork_amd import ops

    ft, d = ("planar", "radial", "radial"), 1
    m = _nfn(d, flow_types=ft, hidden_sizes=(10, 16), trainable_base_dist=True, n_dims_x=1)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((300, 1)).astype(np.float32)
    y = (np.sin(2 * x) + 0.3 * rng.standard_normal((300, 1))).astype(np.float32)
    m._mlp.to(gpu)
    ws = [w.detach().requires_grad_(True) for w in m._mlp.weights + m._mlp.biases]
    nw = len(m._mlp.weights)

    def hidden(xx, params):
        h = xx
        for i in range(nw - 1):
            h = torch.relu(h @ params[i] + params[nw + i])
        return h

    h = hidden(torch.from_numpy(x).to(gpu), ws)
    loss = -ops.log_prob_dense(torch.from_numpy(y).to(gpu), h, ws[nw - 1], ws[2 * nw - 1], ft, d, True).mean()
    loss.backward()
    got = [w.grad.double().cpu() for w in ws]
    ws64 = [w.detach().double().cpu().requires_grad_(True) for w in ws]
    t64 = hidden(torch.from_numpy(x).double(), ws64) @ ws64[nw - 1] + ws64[2 * nw - 1]
    lp64 = G.chain_log_prob_torch(torch.from_numpy(y).double(), t64, ft, d, True)
    (-lp64.mean()).backward()
    for g, w in zip(got, ws64):
        torch.testing.assert_close(g, w.grad, rtol=2e-4, atol=2e-5)


def test_fit_fused_dense_matches_unfused(gpu):
    """fit with the fused Dense path (hidden width 16) and with the materialised t give
    the same training trajectory up to fp32 rounding, and the fused model fits."""
    rng = np.random.default_rng(22)
    x, y = _sinusoid(400, rng)
    losses = {}
    for fused in (True, False):
        m = _nfn(1, n_flows=3, hidden_sizes=(16, 16), trainable_base_dist=True)
        m.fused_dense = fused
        losses[fused] = m.fit(x, y, epochs=50, verbose=0)["loss"]
    assert losses[True][-1] < losses[True][0]
    # the first steps agree to fp32 rounding; afterwards the two paths' different GEMM
    # summation orders (MFMA k-order in the fused kernel vs the library GEMMs) are
    # amplified by Adam's normalised steps: a few 1e-4 by epoch 10
    np.testing.assert_allclose(losses[True][:5], losses[False][:5], rtol=1e-5)
    np.testing.assert_allclose(losses[True][:10], losses[False][:10], rtol=5e-4)
    np.testing.assert_allclose(losses[True][-1], losses[False][-1], rtol=2e-2)


@pytest.mark.parametrize("fused,noise", [(True, False), (False, True)])
def test_fit_graph_replay_matches_eager(gpu, fused, noise):
    """fit's HIP-graph path (the full-batch step captured once and replayed; a partial last
    batch eager) trains exactly as the eager loop: same generator calls in the same order,
    same kernels — the per-epoch losses and the final weights are bitwise equal."""
    rng = np.random.default_rng(5)
    x, y = _sinusoid(203, rng)  # 6 full batches of 32 + a partial one per epoch
    out = {}
    for use_graph in (True, False):
        m = _nfn(1, n_flows=3, hidden_sizes=(16, 16), trainable_base_dist=True,
                 noise_reg=("fixed_rate", 0.1 if noise else 0.0))
        m.fused_dense = fused
        hist = m.fit(x, y, epochs=4, verbose=0, use_graph=use_graph)["loss"]
        out[use_graph] = (hist, [w.detach().cpu().numpy() for w in m._mlp.weights + m._mlp.biases])
    assert out[True][0] == out[False][0]
    for a, b in zip(out[True][1], out[False][1]):
        np.testing.assert_array_equal(a, b)


class _Wrapper:
    def __init__(self, model):
        self.model = model


def test_mle_score_equals_minus_evaluate(gpu):
    """tests/test_evaluation.py:47-55: after fitting, ``mle_log_likelihood_score`` equals
    ``-evaluate`` (the compiled loss with noise off).  Here the two run different kernel
    paths: the score through the fused Dense -> chain kernel with an fp64 device sum, the
    loss through the MLP's materialised t and the chain kernel."""
    from normalizingflownetwork_amd.scorers import mle_log_likelihood_score

    x = np.linspace(-1, 1, 10).reshape((10, 1))
    y = np.linspace(-1, 1, 10).reshape((10, 1))
    mle = _nfn(1, n_flows=0, hidden_sizes=(6, 6), trainable_base_dist=True)
    mle.fit(x, y, epochs=10, verbose=0)
    assert mle_log_likelihood_score(_Wrapper(mle), x, y) == pytest.approx(-mle.evaluate(x, y), rel=1e-5)
    # with flows, and a hidden width the fused Dense path takes (16)
    m2 = _nfn(1, n_flows=3, hidden_sizes=(16, 16), trainable_base_dist=True)
    m2.fit(x, y, epochs=10, verbose=0)
    assert mle_log_likelihood_score(_Wrapper(m2), x, y) == pytest.approx(-m2.evaluate(x, y), rel=1e-5)


def test_bayesian_score(gpu):
    """tests/test_evaluation.py:16-44: the Bayesian scorer on a deterministic (MLE) model
    equals ``-evaluate``; on a Bayesian model the posterior log-mean-exp score exceeds the
    negated mean loss over 50 draws (here the loss has no KL term — SURVEY.md §2 — and the
    inequality is Jensen's: log E[p] >= E[log p], strict while the draws differ)."""
    from normalizingflownetwork_amd import BayesNormalizingFlowNetwork
    from normalizingflownetwork_amd.scorers import bayesian_log_likelihood_score

    rng = np.random.default_rng(22)
    x = np.linspace(-3, 3, 300, dtype=np.float32).reshape((300, 1))
    y = (5 * np.sin(2 * x) + np.abs(x) * rng.standard_normal((300, 1))).astype(np.float32)
    mle = _nfn(1, n_flows=0, hidden_sizes=(6, 6), trainable_base_dist=True)
    mle.fit(x, y, epochs=20, verbose=0)
    mle.map_mode = False
    assert bayesian_log_likelihood_score(_Wrapper(mle), x, y) == pytest.approx(-mle.evaluate(x, y), rel=1e-5)
    be = BayesNormalizingFlowNetwork(n_dims=1, kl_weight_scale=1.0 / x.shape[0], n_flows=0, hidden_sizes=(6, 6),
                                     trainable_base_dist=True)
    be.fit(x, y, epochs=30, verbose=0)
    score = bayesian_log_likelihood_score(_Wrapper(be), x, y)
    loss = sum(be.evaluate(x, y) for _ in range(50)) / 50
    assert np.isfinite(score) and score > -loss


def test_y_noise_input_model(gpu):
    """tests/test_noise_reg.py:50-70: with ``fixed_rate`` noise the y input model is
    deterministic at evaluation and random while training (Keras GaussianNoise)."""
    x = np.linspace([[-1]] * 3, [[1]] * 3, 10, dtype=np.float32).reshape((10, 3))
    y = np.linspace([[-1]] * 3, [[1]] * 3, 10, dtype=np.float32).reshape((10, 3))
    m = _nfn(3, n_flows=3, hidden_sizes=(16, 16), trainable_base_dist=True, noise_reg=("fixed_rate", 1.0))
    m.fit(x, y, epochs=10, verbose=0)
    input_model = m._get_input_model()
    y1 = input_model(y, training=False).cpu().numpy()
    y2 = input_model(y, training=False).cpu().numpy()
    assert np.all(y1 == y2)
    np.testing.assert_allclose(y1, (y - m.y_mean) / m.y_std, rtol=1e-6, atol=1e-7)
    y1 = input_model(y, training=True).cpu().numpy()
    y2 = input_model(y, training=True).cpu().numpy()
    assert not np.all(y1 == y2)


@pytest.mark.parametrize("d,n_flows,trainable", [(1, 3, False), (1, 0, True), (3, 3, True)])
def test_bayes_model_output_dims(gpu, d, n_flows, trainable):
    """tests/test_bayesian_estimator.py:23-80: after one epoch of ``fit`` the Bayesian
    estimator's distribution has event shape [d] and batch shape [10], ``log_prob`` of a
    broadcast row has shape [10], ``pdf`` too (1-d case), and the posterior score is finite."""
    from normalizingflownetwork_amd import BayesNormalizingFlowNetwork

    x = np.linspace([[-1]] * d, [[1]] * d, 10, dtype=np.float32).reshape((10, d))
    m = BayesNormalizingFlowNetwork(d, kl_weight_scale=1.0 / x.shape[0], n_flows=n_flows, hidden_sizes=(16, 16),
                                    trainable_base_dist=trainable)
    m.fit(x, x, epochs=1, verbose=0)
    out = m(x)
    assert out.event_shape == [d] and out.batch_shape == [10]
    assert tuple(out.log_prob([[0.0] * d]).shape) == (10,)
    if d == 1:
        assert tuple(m.pdf(x, x).shape) == (10,)
    assert np.isfinite(m.score(x, x))


def test_bayes_y_noise_input_model(gpu):
    """tests/test_bayesian_estimator.py:83-106: ``rule_of_thumb`` noise on the Bayesian
    estimator: the y input model is deterministic at evaluation, random while training."""
    from normalizingflownetwork_amd import BayesNormalizingFlowNetwork

    x = np.linspace([[-1]] * 3, [[1]] * 3, 10, dtype=np.float32).reshape((10, 3))
    m = BayesNormalizingFlowNetwork(3, kl_weight_scale=1.0 / x.shape[0], n_flows=3, hidden_sizes=(16, 16),
                                    trainable_base_dist=True, noise_reg=("rule_of_thumb", 1.0))
    m.fit(x, x, epochs=10, verbose=0)
    assert m.y_noise_std == pytest.approx(1.0 * (10 + 1) ** (-1 / (4 + 6)))
    im = m._get_input_model()
    assert np.all(im(x, training=False).cpu().numpy() == im(x, training=False).cpu().numpy())
    assert not np.all(im(x, training=True).cpu().numpy() == im(x, training=True).cpu().numpy())
