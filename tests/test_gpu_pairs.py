"""The d = 1 chain two flows per dispatch (`chain1_fast_pairs` / `grad1_pairs`,
DESIGN.md "The d = 1 chain is instruction-issue-bound").

The pair form runs in the posterior, the fused Dense kernels and, for chains of at most
4 flows, the streaming forward / backward. These programs reach those kernels (rows of
P = 8, 16 or 32 floats: P/4 a power of two), with odd and even flow counts, affine
blocks of 2 parameters between the 3-parameter ones, and the longest packed chains.
Forward, posterior and backward are held to the oracles at the tolerances the other GPU
tests use: `tolerance_bound` for log-densities and `grad_tolerance` for gradients."""

import numpy as np
import pytest
import torch

from oracle import nfn_grad_oracle as G
from oracle import nfn_oracle as O
from parity import check_forward, check_grad, fp32_sensitivity

pytestmark = pytest.mark.gpu

PROGRAMS = [
    ("affine",) * 3,                                              # K = 3, P = 8
    ("radial", "radial"),                                         # K = 2, P = 8 (C1)
    ("planar", "affine", "radial"),                               # K = 3, P = 10: generic kernels
    ("planar", "radial", "planar", "affine", "radial"),           # K = 5, P = 16
    ("planar", "affine", "radial", "affine", "affine", "affine"),  # K = 6, P = 16
    ("affine",) * 15,                                             # K = 15, P = 32
    ("radial", "planar") * 5,                                     # K = 10, P = 32
    # K = 2, P = 8: every alternating (planar, radial) program of the compile-time pair
    # bodies (hpair_types) the wave kernels take
    ("planar", "planar"),
    ("planar", "radial"),
    ("radial", "planar"),
]


def _ids(ft):
    return "-".join(f[0] for f in ft)


@pytest.mark.parametrize("ft", PROGRAMS, ids=_ids)
def test_pair_form_forward_and_posterior(ft, gpu):
    from normalizingflownetwork_amd import ops

    rng = np.random.default_rng(len(ft) * 31 + len(ft[0]))
    P = O.total_param_size(ft, 1, True)
    B = 1000
    y = rng.standard_normal((B, 1)).astype(np.float32)
    t = (0.7 * rng.standard_normal((B, P))).astype(np.float32)
    lp, _ = ops.chain_log_prob(y, t, ft, 1, True)
    with np.errstate(all="ignore"):
        r64 = O.chain_log_prob(y, t, ft, 1, True, np.float64)
        r32 = O.chain_log_prob(y, t, ft, 1, True, np.float32)
    check_forward(lp.cpu().numpy(), r64, r32, f"pairs {_ids(ft)} forward", nonfinite="match",
                  sensitivity=fp32_sensitivity(y, t, ft, 1, True))
    # posterior: S draws of t per sample
    S, Bp = 3, 333
    tp = (0.7 * rng.standard_normal((S, Bp, P))).astype(np.float32)
    out, _ = ops.posterior_lse(y[:Bp], tp, ft, 1, True)
    with np.errstate(all="ignore"):
        p64 = O.posterior_lse(y[:Bp], tp, ft, 1, True)
        p32 = O.posterior_lse(y[:Bp], tp, ft, 1, True, dtype=np.float32)
    check_forward(out.cpu().numpy(), p64, p32, f"pairs {_ids(ft)} posterior", nonfinite="match")


@pytest.mark.parametrize("ft", [p for p in PROGRAMS if len(p) <= 6], ids=_ids)
def test_pair_form_backward(ft, gpu):
    from normalizingflownetwork_amd import ops

    rng = np.random.default_rng(7 * len(ft))
    P = O.total_param_size(ft, 1, True)
    B = 64 * 5 + 17
    y = rng.standard_normal((B, 1)).astype(np.float32)
    t = (0.7 * rng.standard_normal((B, P))).astype(np.float32)
    g = rng.standard_normal(B).astype(np.float32)
    gt64, gy64, dev_t, dev_y = G.fp32_spread(y, t, ft, 1, True, g_out=g)
    lp, gt, gy = ops.chain_log_prob_grad(torch.from_numpy(y).to(gpu), torch.from_numpy(t).to(gpu), ft, 1, True,
                                         g_out=torch.from_numpy(g).to(gpu), want_logp=True)
    for got, ref, dev, what in ((gt, gt64, dev_t, "d/dt"), (gy, gy64, dev_y, "d/dy")):
        check_grad(got.cpu().numpy().reshape(ref.shape), ref, dev, f"pairs {_ids(ft)} {what}")
    with np.errstate(all="ignore"):
        r64 = O.chain_log_prob(y, t, ft, 1, True, np.float64)
        r32 = O.chain_log_prob(y, t, ft, 1, True, np.float32)
    check_forward(lp.cpu().numpy(), r64, r32, f"pairs {_ids(ft)} backward's log_prob", nonfinite="match",
                  sensitivity=fp32_sensitivity(y, t, ft, 1, True))


@pytest.mark.parametrize("ft", [("planar", "radial") * 5, ("affine",) * 15, ("planar", "radial", "planar", "affine", "radial")],
                         ids=_ids)
def test_pair_form_bitwise_the_loop(ft, gpu):
    """At K > 4 the streaming forward keeps the one-flow loop while the posterior runs the
    pair form; with one draw the posterior's log-sum-exp is the log-density itself
    (m + log 1 - log 1), so the two kernels must agree bit for bit."""
    from normalizingflownetwork_amd import ops

    prev = ops.set_math_mode("fast")
    try:
        gen = torch.Generator(device="cuda").manual_seed(len(ft))
        P = O.total_param_size(ft, 1, True)
        B = 64 * 70 + 9
        y = torch.randn((B, 1), generator=gen, device="cuda")
        t = 0.7 * torch.randn((B, P), generator=gen, device="cuda")
        lp, _ = ops.chain_log_prob(y, t, ft, 1, True)
        post, _ = ops.posterior_lse(y, t.unsqueeze(0).contiguous(), ft, 1, True)
        assert torch.equal(lp, post)
    finally:
        ops.set_math_mode(prev)
