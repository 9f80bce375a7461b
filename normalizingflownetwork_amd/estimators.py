"""Estimator surface around the flow hot path.

Mirrors ``estimators/BaseEstimator.py:43-86``, ``MaximumLikelihoodNNEstimator.py``,
``NormalizingFlowNetwork.py`` and ``BayesNormalizingFlowNetwork.py`` /
``BayesianNNEstimator.py:65-76`` for EVALUATION: ``log_pdf``, ``pdf``, ``score``.

The x -> t network (the reference's Keras Dense stack) is not on the hot path
(out of scope); it is a small torch MLP here, used only to
produce ``t``.  Everything from ``t`` to the density / score runs in the fused
HIP kernels: the y normalisation ``(y - mu)/sigma``, the whole flow chain, the
base density, the ``-sum(log sigma)`` correction and (for ``score``) the fp64
batch sum.  ``fit`` trains on the GPU: torch autograd through the MLP and the
fused backward kernel through the flow chain; the Bayesian
estimator's variational training (KL term) is not mirrored.
"""

from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from . import ops
from .distribution_layers import InverseNormalizingFlowLayer

_ACTIVATIONS = {
    "tanh": torch.tanh,
    "relu": torch.relu,
    "linear": lambda v: v,
    "sigmoid": torch.sigmoid,
    "elu": torch.nn.functional.elu,
}


class _MLP:
    """Dense stack x -> t (``MaximumLikelihoodNNEstimator.py:37-44``), Glorot-uniform
    weights and zero biases like Keras' ``Dense`` defaults."""

    def __init__(self, n_in: int, hidden_sizes: Sequence[int], n_out: int, activation: str, seed: int):
        assert type(hidden_sizes) in (tuple, list)
        assert activation in _ACTIVATIONS, f"unknown activation {activation!r}"
        g = torch.Generator().manual_seed(seed)
        sizes = [n_in] + list(hidden_sizes) + [n_out]
        self.weights, self.biases = [], []
        for a, b in zip(sizes[:-1], sizes[1:]):
            lim = float(np.sqrt(6.0 / (a + b)))
            self.weights.append((torch.rand((a, b), generator=g, dtype=torch.float32) * 2 - 1) * lim)
            self.biases.append(torch.zeros((b,), dtype=torch.float32))
        self.activation = activation
        self._device = None

    def to(self, device):
        if self._device != device:
            self.weights = [w.to(device) for w in self.weights]
            self.biases = [b.to(device) for b in self.biases]
            self._device = device
        return self

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        act = _ACTIVATIONS[self.activation]
        h = x
        n = len(self.weights)
        for i, (w, b) in enumerate(zip(self.weights, self.biases)):
            h = h @ w + b
            if i < n - 1:
                h = act(h)
        return h

    def hidden(self, x: torch.Tensor) -> torch.Tensor:
        """Activations entering the linear output layer (the fused Dense path's input)."""
        act = _ACTIVATIONS[self.activation]
        h = x
        for w, b in zip(self.weights[:-1], self.biases[:-1]):
            h = act(h @ w + b)
        return h.contiguous()


class BaseEstimator:
    """Evaluation half of ``estimators/BaseEstimator.py``."""

    def __init__(self, dist_layer: InverseNormalizingFlowLayer, n_dims_x: Optional[int] = None,
                 hidden_sizes=(16, 16), activation="relu", random_seed=22, noise_reg=("fixed_rate", 0.0)):
        assert len(noise_reg) == 2
        self.dist_layer = dist_layer
        self.n_dims = dist_layer.n_dims
        self.hidden_sizes = tuple(hidden_sizes)
        self.activation = activation
        self.random_seed = random_seed
        self.noise_fn_type, self.noise_scale_factor = noise_reg
        self.x_noise_std = self.y_noise_std = 0.0  # set by fit (BaseEstimator.py:9-10, 33-41)
        self.x_mean = self.x_std = None
        self.y_mean = np.zeros((self.n_dims,), np.float32)
        self.y_std = np.ones((self.n_dims,), np.float32)
        self._mlp = None
        # fit: the output Dense layer fused into the chain kernels (forward + backward)
        # when its shapes allow; False trains through the materialised t instead
        self.fused_dense = True
        self.last_score_nonfinite = 0
        if n_dims_x is not None:
            self._build(n_dims_x)

    # --- x -> t -----------------------------------------------------------------
    def _build(self, n_dims_x: int):
        self._mlp = _MLP(n_dims_x, self.hidden_sizes, self.dist_layer.get_total_param_size(), self.activation,
                         self.random_seed)
        if self.x_mean is None:
            self.x_mean = np.zeros((n_dims_x,), np.float32)
            self.x_std = np.ones((n_dims_x,), np.float32)

    def _assign_data_normalization(self, x, y):
        """``BaseEstimator.py:49-53``."""
        x = np.asarray(x, np.float32)
        y = np.asarray(y, np.float32)
        self.x_mean = np.mean(x, axis=0, dtype=np.float32)
        self.y_mean = np.mean(y, axis=0, dtype=np.float32)
        self.x_std = np.std(x, axis=0, dtype=np.float32)
        self.y_std = np.std(y, axis=0, dtype=np.float32)

    def set_data_normalization(self, x, y):
        self._assign_data_normalization(x, y)

    def params(self, x) -> torch.Tensor:
        """``t = MLP((x - mu_x)/(sigma_x + 1e-8))`` (``MaximumLikelihoodNNEstimator.py:40-43``)."""
        x = ops.as_device_f32(x)
        if x.dim() == 1:
            x = x.unsqueeze(-1)
        if self._mlp is None:
            self._build(int(x.shape[-1]))
        dev = x.device
        self._mlp.to(dev)
        xm = torch.as_tensor(self.x_mean, dtype=torch.float32, device=dev)
        xs = torch.as_tensor(self.x_std, dtype=torch.float32, device=dev)
        return self._mlp((x - xm) / (xs + 1e-8)).contiguous()

    def __call__(self, x):
        return self.dist_layer(self.params(x))

    def _fused_dense_inputs(self, x):
        """``(h, W, b)`` of the output Dense layer when the fused Dense->chain kernel takes
        the shapes (evaluation only: no autograd through it), else None."""
        if torch.is_grad_enabled() and any(w.requires_grad for w in (self._mlp.weights if self._mlp else [])):
            return None
        x = ops.as_device_f32(x)
        if x.dim() == 1:
            x = x.unsqueeze(-1)
        if self._mlp is None:
            self._build(int(x.shape[-1]))
        self._mlp.to(x.device)
        W, b = self._mlp.weights[-1], self._mlp.biases[-1]
        if not ops.dense_fusable(int(W.shape[0]), int(W.shape[1]), self.n_dims) or len(self._mlp.weights) < 2:
            return None
        xm = torch.as_tensor(self.x_mean, dtype=torch.float32, device=x.device)
        xs = torch.as_tensor(self.x_std, dtype=torch.float32, device=x.device)
        return self._mlp.hidden((x - xm) / (xs + 1e-8)), W, b

    def call(self, x, training=False):
        return self(x)

    # --- evaluation ---------------------------------------------------------------
    def log_pdf(self, x, y):
        """``BaseEstimator.py:77-86``: ``log_prob((y-mu)/sigma) - sum(log sigma)``."""
        x = np.asarray(x, np.float32) if not isinstance(x, torch.Tensor) else x
        y = np.asarray(y, np.float32) if not isinstance(y, torch.Tensor) else y
        assert tuple(x.shape) == tuple(y.shape)
        fused = self._fused_dense_inputs(x)
        if fused is not None:  # output Dense layer fused into the chain kernel
            dl = self.dist_layer
            lp, _ = ops.chain_log_prob_dense(y, *fused, dl.flow_types, self.n_dims, dl.trainable_base_dist,
                                             self.y_mean, self.y_std)
            return lp
        output = self(x)
        assert output.event_shape == y.shape[-1]
        return output.log_prob(y, self.y_mean, self.y_std)

    def pdf(self, x, y):
        """``BaseEstimator.py:71-75``: ``prob(y_circ) / prod(sigma)`` = ``exp(log_pdf)``."""
        return torch.exp(self.log_pdf(x, y))

    def score(self, x_data, y_data) -> float:
        """``BaseEstimator.py:43-47``: mean log-likelihood, reduced on the device in fp64."""
        x_data = np.asarray(x_data, np.float32) if not isinstance(x_data, torch.Tensor) else x_data
        y_data = np.asarray(y_data, np.float32) if not isinstance(y_data, torch.Tensor) else y_data
        fused = self._fused_dense_inputs(x_data)
        if fused is not None:  # output Dense layer fused into the chain kernel
            dl = self.dist_layer
            _, s, nf = ops.chain_log_prob_dense(y_data, *fused, dl.flow_types, self.n_dims, dl.trainable_base_dist,
                                                self.y_mean, self.y_std, want_values=False, want_nonfinite=True)
        else:
            output = self(x_data)
            s, nf = output.log_prob_sum(y_data, self.y_mean, self.y_std, want_nonfinite=True)
        return self._finish_score(s, nf, int(y_data.shape[0]))

    def _finish_score(self, s: torch.Tensor, nf: torch.Tensor, n: int) -> float:
        """Mean from the device fp64 sum.  Non-finite log-densities propagate into the
        mean exactly as in the reference's ``.mean()`` (``BaseEstimator.py:47``); their
        count (kept as ``last_score_nonfinite``) is reported with a ``RuntimeWarning``
        instead of passing silently."""
        vals = torch.cat([s.reshape(1), nf.reshape(1)]).cpu().tolist()
        self.last_score_nonfinite = int(vals[1])
        if self.last_score_nonfinite:
            import warnings

            warnings.warn(f"score: {self.last_score_nonfinite} of {n} log-densities are not finite",
                          RuntimeWarning, stacklevel=3)
        return vals[0] / n

    def _get_input_model(self):
        """``BaseEstimator.py:61-69``: ``y -> (y - mu_y) / sigma_y`` followed by Keras
        ``GaussianNoise(y_noise_std)``, which adds noise only when called with
        ``training=True``.  Returns ``input_model(y, training=False)`` (a device tensor)."""
        gen = {}

        def input_model(y, training=False):
            y = ops.as_device_f32(y)
            ym = torch.as_tensor(self.y_mean, dtype=torch.float32, device=y.device)
            ys = torch.as_tensor(self.y_std, dtype=torch.float32, device=y.device)
            yc = (y - ym) / ys
            if training and self.y_noise_std > 0.0:
                if "g" not in gen:
                    gen["g"] = torch.Generator(device=y.device)
                    gen["g"].manual_seed(int(self.random_seed) + 7)
                yc = yc + self.y_noise_std * torch.randn(yc.shape, generator=gen["g"], device=y.device,
                                                         dtype=yc.dtype)
            return yc

        return input_model

    def _get_neg_log_likelihood(self):
        """``BaseEstimator.py:55-59``: the compiled loss, ``nll(y, p_y) = -p_y.log_prob(
        input_model(y)) + sum(log sigma_y)`` per sample (noise off: evaluation)."""
        input_model = self._get_input_model()
        log_sy = float(np.sum(np.log(np.asarray(self.y_std, np.float64))))
        return lambda y, p_y: -p_y.log_prob(input_model(y)) + log_sy

    def evaluate(self, x, y, batch_size=None, verbose=0, **kwargs) -> float:
        """Keras ``Model.evaluate`` of the compiled loss (``MaximumLikelihoodNNEstimator.py:33-35``):
        the sample mean of ``_get_neg_log_likelihood()(y, self(x))`` with noise off.  The
        per-batch means Keras averages (weighted by batch size) equal this one mean, so the
        data runs as one batch: the MLP in torch, ``log_prob`` in the fused chain kernel on
        the materialised ``t`` (``score`` takes the fused Dense -> chain path: the reference's
        ``score == -evaluate`` tests compare the two)."""
        x = np.asarray(x, np.float32) if not isinstance(x, torch.Tensor) else x
        y = np.asarray(y, np.float32) if not isinstance(y, torch.Tensor) else y
        with torch.no_grad():
            nll = self._get_neg_log_likelihood()(y, self.call(x, training=False))
        return float(nll.double().mean().item())

    def _assign_noise_regularisation(self, n_dims: int, n_datapoints: int):
        """``BaseEstimator.py:33-41``."""
        assert self.noise_fn_type in ["rule_of_thumb", "fixed_rate"]
        if self.noise_fn_type == "rule_of_thumb":
            std = self.noise_scale_factor * (n_datapoints + 1) ** (-1 / (4 + n_dims))
        else:
            std = self.noise_scale_factor
        self.x_noise_std = self.y_noise_std = float(std)

    def fit(self, x, y, batch_size=None, epochs=None, verbose=1, shuffle=True, use_graph=True, **kwargs):
        """Maximum-likelihood training on the GPU: ``BaseEstimator.fit`` (``BaseEstimator.py:19-31``)
        with the model compiled as in ``MaximumLikelihoodNNEstimator.py:33-35`` —
        Adam(learning_rate), loss = mean over the batch of ``-log_prob(y_circ + noise | t)
        + sum(log y_std)`` (``BaseEstimator.py:55-67``), Keras defaults ``batch_size=32``,
        ``epochs=1``, per-epoch shuffling, GaussianNoise on the normalised x and y while
        training, and TerminateOnNaN.  ``t = MLP(x)`` runs in torch; ``log_prob`` and its
        gradient w.r.t. ``t`` run in the fused HIP kernels (``nfn_chain_logprob_f32`` /
        ``nfn_chain_logprob_grad_f32``).

        At the reference's batch sizes a training step is a few dozen tiny launches, so with
        ``use_graph`` the full-batch step (gather, normalisation, MLP, fused log_prob forward
        and backward, Adam) is captured once into a HIP graph and replayed: per step only the
        batch indices and the noise draws (if any) are written into the graph's static inputs
        — the same generator calls in the same order as the eager loop, so both paths train
        identically.  A final partial batch runs eagerly.  Returns ``{"loss": [per-epoch
        mean loss]}``."""
        x = np.asarray(x, np.float32)
        y = np.asarray(y, np.float32)
        assert len(x.shape) == len(y.shape) == 2, "Please pass a matrix not a vector"
        self._assign_data_normalization(x, y)
        self._assign_noise_regularisation(n_dims=x.shape[1] + y.shape[1], n_datapoints=x.shape[0])
        if self._mlp is None:
            self._build(int(x.shape[1]))
        dev = ops._device()
        self._mlp.to(dev)
        params = [p.detach().requires_grad_(True) for p in self._mlp.weights + self._mlp.biases]
        nw = len(self._mlp.weights)
        self._mlp.weights, self._mlp.biases = params[:nw], params[nw:]
        lr = getattr(self, "learning_rate", 3e-3)
        # Keras Adam defaults; capturable: the step counts and bias corrections live on the
        # device, so the same optimizer runs eagerly and inside the graph
        opt = torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), eps=1e-7, capturable=True)
        dl = self.dist_layer
        P = ops.total_param_size(dl.flow_types, self.n_dims, dl.trainable_base_dist)
        fused_dense = (len(self._mlp.weights) > 1 and self.fused_dense
                       and ops.dense_fusable(int(self._mlp.weights[-1].shape[0]), P, self.n_dims))
        batch_size = 32 if batch_size is None else int(batch_size)
        epochs = 1 if epochs is None else int(epochs)
        X = torch.from_numpy(x).to(dev)
        Y = torch.from_numpy(y).to(dev)
        xm, xs = (torch.as_tensor(v, dtype=torch.float32, device=dev) for v in (self.x_mean, self.x_std))
        ym, ys = (torch.as_tensor(v, dtype=torch.float32, device=dev) for v in (self.y_mean, self.y_std))
        sum_log_ys = torch.log(ys).sum()
        gen = torch.Generator(device=dev).manual_seed(int(self.random_seed))
        n = X.shape[0]
        acc = torch.zeros((), dtype=torch.float64, device=dev)

        def step(idx, nx, ny):
            """One training step on the rows ``idx`` with the noise draws ``nx`` / ``ny``."""
            xn = (X[idx] - xm) / (xs + 1e-8)
            if nx is not None:
                xn = xn + self.x_noise_std * nx
            yc = (Y[idx] - ym) / ys
            if ny is not None:
                yc = yc + self.y_noise_std * ny
            if fused_dense:  # output layer fused into the chain, forward and backward
                lp = ops.log_prob_dense(yc, self._mlp.hidden(xn), self._mlp.weights[-1], self._mlp.biases[-1],
                                        dl.flow_types, self.n_dims, dl.trainable_base_dist)
            else:
                t = self._mlp(xn)
                lp = ops.log_prob(yc, t, dl.flow_types, self.n_dims, dl.trainable_base_dist)
            loss = -lp.mean() + sum_log_ys
            loss.backward()
            opt.step()
            acc.add_(loss.detach().double() * idx.numel())

        def draws(rows):
            nx = torch.randn((rows, X.shape[1]), generator=gen, device=dev) if self.x_noise_std > 0 else None
            ny = torch.randn((rows, Y.shape[1]), generator=gen, device=dev) if self.y_noise_std > 0 else None
            return nx, ny

        graph = None  # (graph, static idx, static x noise, static y noise, its pinned workspaces)
        warm = 3  # eager steps before the capture (optimizer state, allocator pools)
        steps_done = 0
        history = {"loss": []}
        try:
            for _ in range(epochs):
                perm = torch.randperm(n, generator=gen, device=dev) if shuffle else torch.arange(n, device=dev)
                acc.zero_()
                for i in range(0, n, batch_size):
                    idx = perm[i:i + batch_size]
                    full = idx.numel() == batch_size
                    if use_graph and full and graph is not None:
                        g_, sidx, snx, sny, _ = graph
                        sidx.copy_(idx)
                        if snx is not None:
                            snx.normal_(generator=gen)
                        if sny is not None:
                            sny.normal_(generator=gen)
                        g_.replay()
                        continue
                    nx, ny = draws(idx.numel())
                    if use_graph and full and steps_done >= warm:
                        # capture the full-batch step (the capture itself executes nothing:
                        # this batch then runs as the graph's first replay)
                        sidx = idx.clone()
                        snx, sny = nx, ny
                        opt.zero_grad(set_to_none=True)
                        side = torch.cuda.Stream(device=dev)
                        side.wait_stream(torch.cuda.current_stream(dev))
                        g_ = torch.cuda.CUDAGraph()
                        mark = ops.graph_pin_mark()
                        with torch.cuda.stream(side):
                            with torch.cuda.graph(g_, stream=side):
                                step(sidx, snx, sny)
                        torch.cuda.current_stream(dev).wait_stream(side)
                        # the workspaces the capture pinned live exactly as long as this graph
                        graph = (g_, sidx, snx, sny, ops.take_graph_workspaces(side, mark))
                        g_.replay()
                        continue
                    opt.zero_grad(set_to_none=True)
                    if use_graph and steps_done < warm:
                        side = torch.cuda.Stream(device=dev)  # warm-up on a side stream (capture rules)
                        side.wait_stream(torch.cuda.current_stream(dev))
                        with torch.cuda.stream(side):
                            step(idx, nx, ny)
                        torch.cuda.current_stream(dev).wait_stream(side)
                    else:
                        step(idx, nx, ny)
                    steps_done += 1
                ep_loss = float(acc.item()) / n
                history["loss"].append(ep_loss)
                if verbose:
                    print(f"epoch {len(history['loss'])}/{epochs} loss {ep_loss:.6f}", flush=True)
                if not np.isfinite(ep_loss):  # tf.keras.callbacks.TerminateOnNaN
                    break
        finally:
            self._mlp.weights = [p.detach() for p in self._mlp.weights]
            self._mlp.biases = [p.detach() for p in self._mlp.biases]
        return history


class NormalizingFlowNetwork(BaseEstimator):
    """``estimators/NormalizingFlowNetwork.py:9-19``: ``n_flows`` radial flows by
    default.  ``flow_types`` (a compatible superset) picks any chain, e.g. the
    planar/radial chains of the benchmark configs."""

    def __init__(self, n_dims, n_flows=10, trainable_base_dist=True, flow_types=None, hidden_sizes=(16, 16),
                 noise_reg=("fixed_rate", 0.0), learning_rate=3e-3, activation="relu", random_seed=22,
                 n_dims_x=None):
        flow_types = tuple(flow_types) if flow_types is not None else ("radial",) * n_flows
        dist_layer = InverseNormalizingFlowLayer(flow_types=flow_types, n_dims=n_dims,
                                                 trainable_base_dist=trainable_base_dist)
        self.learning_rate = learning_rate
        super().__init__(dist_layer, n_dims_x=n_dims_x, hidden_sizes=hidden_sizes, activation=activation,
                         random_seed=random_seed, noise_reg=noise_reg)

    @staticmethod
    def build_function(n_dims=1, n_flows=3, hidden_sizes=(16, 16), trainable_base_dist=True,
                       noise_reg=("fixed_rate", 0.0), learning_rate=3e-3, activation="tanh"):
        return NormalizingFlowNetwork(n_dims=n_dims, n_flows=n_flows, hidden_sizes=hidden_sizes,
                                      trainable_base_dist=trainable_base_dist, noise_reg=noise_reg,
                                      learning_rate=learning_rate, activation=activation)


def mean_field_scale(rho: torch.Tensor) -> torch.Tensor:
    """Scale of the mean-field posterior over every DenseVariational weight:
    ``1e-3 + softplus(log(expm1(1)) + 0.05 * rho)`` (``MeanFieldLayer``,
    ``DistributionLayers.py:45-55``)."""
    return 1e-3 + torch.nn.functional.softplus(float(np.log(np.expm1(1.0))) + 0.05 * rho)


class BayesNormalizingFlowNetwork(BaseEstimator):
    """Posterior-scoring half of ``estimators/BayesNormalizingFlowNetwork.py`` /
    ``BayesianNNEstimator.py``.  Every layer is a ``DenseVariational`` whose weights
    (kernel and bias) have a mean-field Gaussian posterior held as one variable vector
    ``[loc | rho]`` initialised N(0, 0.05) (Keras ``"normal"``; ``BayesianNNEstimator.py:92-107``,
    ``DistributionLayers.py:17-55``): a draw is ``loc + (1e-3 + softplus(log(e-1) + 0.05 rho))
    * eps``, one weight sample per layer per draw shared by the batch (``:122-145``); in
    ``map_mode`` the variable holds ``loc`` only and the weights ARE ``loc``.  ``score``
    stacks the S draws' last hidden activations and output-layer weights and evaluates
    ``logsumexp_s(log_pdf) - log S`` per sample in ONE fused kernel
    (``nfn_posterior_lse_dense_f32``, the output DenseVariational layer fused; or
    ``nfn_posterior_lse_f32`` over a library-GEMM ``t``) instead of S model re-runs.
    ``fit`` trains the posterior means by maximum likelihood; the KL(q || p) term and
    the scales' training are not mirrored (out of scope)."""

    def __init__(self, n_dims, kl_weight_scale=1.0, n_flows=2, trainable_base_dist=True, flow_types=None,
                 hidden_sizes=(10,), activation="tanh", noise_reg=("fixed_rate", 0.0), learning_rate=2e-2,
                 map_mode=False, prior_scale=1.0, trainable_prior=False, kl_use_exact=True, random_seed=22,
                 n_dims_x=None):
        assert kl_weight_scale <= 1.0  # BayesianNNEstimator.py:120
        flow_types = tuple(flow_types) if flow_types is not None else ("radial",) * n_flows
        dist_layer = InverseNormalizingFlowLayer(flow_types=flow_types, n_dims=n_dims,
                                                 trainable_base_dist=trainable_base_dist)
        self.map_mode = map_mode
        self.prior_scale = prior_scale
        self.trainable_prior = trainable_prior
        self.kl_use_exact = kl_use_exact
        self.kl_weight_scale = kl_weight_scale
        self.learning_rate = learning_rate  # BayesianNNEstimator.py:61-63 (Adam(learning_rate))
        self._post_rho = None
        super().__init__(dist_layer, n_dims_x=n_dims_x, hidden_sizes=hidden_sizes, activation=activation,
                         random_seed=random_seed, noise_reg=noise_reg)
        self._draw_gen = None

    def _build(self, n_dims_x: int):
        """Shapes from the Dense stack; the posterior variables replace its weights: the
        means ``loc`` live in ``self._mlp`` (so ``params`` is the posterior-mean network),
        the ``rho`` in ``self._post_rho`` (None in map mode)."""
        super()._build(n_dims_x)
        g = torch.Generator().manual_seed(int(self.random_seed) + 1)
        rhos = []
        for w, b in zip(self._mlp.weights, self._mlp.biases):
            size = w.numel() + b.numel()  # DenseVariational: kernel (in x units) then bias
            v = 0.05 * torch.randn((size if self.map_mode else 2 * size,), generator=g, dtype=torch.float32)
            w.copy_(v[:w.numel()].reshape(w.shape))
            b.copy_(v[w.numel():size])
            if not self.map_mode:
                rhos.append((v[size:size + w.numel()].reshape(w.shape).clone(), v[size + w.numel():].clone()))
        self._post_rho = None if self.map_mode else rhos

    def posterior_scales(self, device=None):
        """Per layer ``(scale_W, scale_b)`` of the mean-field posterior (None in map mode)."""
        if self._post_rho is None:
            return None
        return [(mean_field_scale(rw).to(device), mean_field_scale(rb).to(device)) for rw, rb in self._post_rho]

    def _last_layer_draws(self, x, n_draws: int):
        """Per posterior draw: the last hidden activations and the sampled output layer,
        ``h (S, B, H)``, ``W (S, H, P)``, ``b (S, P)`` (every layer re-sampled per draw,
        ``BayesianNNEstimator.py:122-145``)."""
        x = ops.as_device_f32(x)
        if x.dim() == 1:
            x = x.unsqueeze(-1)
        if self._mlp is None:
            self._build(int(x.shape[-1]))
        dev = x.device
        self._mlp.to(dev)
        if self._draw_gen is None:
            self._draw_gen = torch.Generator(device=dev).manual_seed(self.random_seed)
        xm = torch.as_tensor(self.x_mean, dtype=torch.float32, device=dev)
        xs = torch.as_tensor(self.x_std, dtype=torch.float32, device=dev)
        xn = (x - xm) / (xs + 1e-8)
        act = _ACTIVATIONS[self.activation]
        scales = self.posterior_scales(dev)
        hs, ws, bs = [], [], []
        n = len(self._mlp.weights)
        for _ in range(n_draws):
            h = xn
            for i, (w, b) in enumerate(zip(self._mlp.weights, self._mlp.biases)):
                if scales is not None:  # a sample of q(w) = N(loc, scale^2), map mode: the mean
                    sw, sb = scales[i]
                    w = w + sw * torch.randn(w.shape, generator=self._draw_gen, device=dev, dtype=torch.float32)
                    b = b + sb * torch.randn(b.shape, generator=self._draw_gen, device=dev, dtype=torch.float32)
                if i < n - 1:
                    h = act(h @ w + b)
                else:
                    hs.append(h)
                    ws.append(w)
                    bs.append(b)
        return torch.stack(hs).contiguous(), torch.stack(ws).contiguous(), torch.stack(bs).contiguous()

    def evaluate(self, x, y, batch_size=None, verbose=0, **kwargs) -> float:
        """Keras ``evaluate`` of ``BayesianNNEstimator``'s compiled loss for ONE posterior
        draw (every ``DenseVariational`` re-samples its weights per call,
        ``BayesianNNEstimator.py:122-145``): the mean NLL of (x, y) under ``t`` of a fresh
        draw.  The KL(q || p) regularisation term the reference adds is not mirrored
        (SURVEY.md §2), so this is the NLL part of its loss."""
        x = np.asarray(x, np.float32) if not isinstance(x, torch.Tensor) else x
        y = np.asarray(y, np.float32) if not isinstance(y, torch.Tensor) else y
        with torch.no_grad():
            t = self.params_draws(x, 1)[0]
            nll = self._get_neg_log_likelihood()(y, self.dist_layer(t))
        return float(nll.double().mean().item())

    def params_draws(self, x, n_draws: int) -> torch.Tensor:
        """``t`` for ``n_draws`` posterior weight samples: (S, B, P)."""
        h, W, b = self._last_layer_draws(x, n_draws)
        return torch.matmul(h, W) + b[:, None, :]

    def score(self, x_data, y_data, n_draws: Optional[int] = None) -> float:
        """``BayesianNNEstimator.py:65-76``: 50 draws (1 in map mode).  The output layer is
        fused into the posterior kernel (``nfn_posterior_lse_dense_f32``: t_s = h_s W_s + b_s
        never written to memory) when its width allows, else t is formed by the library GEMM."""
        S = n_draws if n_draws is not None else (1 if self.map_mode else 50)
        h, W, b = self._last_layer_draws(np.asarray(x_data, np.float32), S)
        _, s, nf = ops.posterior_lse_dense(np.asarray(y_data, np.float32), h, W, b, self.dist_layer.flow_types,
                                           self.n_dims, self.dist_layer.trainable_base_dist, self.y_mean,
                                           self.y_std, want_values=False, want_sum=True, want_nonfinite=True)
        return self._finish_score(s, nf, int(np.shape(y_data)[0]))
