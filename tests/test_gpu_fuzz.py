"""Randomised parity sweep (fixed seeds): random event sizes, chains, base
trainability, batch sizes, strides and broadcasting, through every kernel family
the dispatcher can pick (persistent, lane-group, tile fallback, posterior split,
backward wave / group / tile) against the oracles."""

import numpy as np
import pytest
import torch

from oracle import nfn_grad_oracle as G
from oracle import nfn_oracle as O
from parity import check_forward, check_grad, fp32_sensitivity

pytestmark = pytest.mark.gpu

FLOWS = ("planar", "radial", "affine")


def _config(seed):
    rng = np.random.default_rng(1000 + seed)
    d = int(rng.choice([1, 1, 1, 2, 3, 4, 5, 8, 8, 16]))
    K = int(rng.integers(0, 13))
    ft = tuple(rng.choice(FLOWS, size=K))
    tr = bool(rng.integers(0, 2)) or K == 0
    B = int(rng.choice([1, 37, 64, 255, 1000, 3001]))
    pad = int(rng.choice([0, 0, 1, 4]))  # extra columns: strided (and unaligned when 1) parameter rows
    ybc = bool(rng.random() < 0.15)
    return rng, d, ft, tr, B, pad, ybc


@pytest.mark.parametrize("seed", range(64))
def test_random_chain(seed, gpu):
    from normalizingflownetwork_amd import ops

    rng, d, ft, tr, B, pad, ybc = _config(seed)
    P = O.total_param_size(ft, d, tr)
    if P == 0:
        pytest.skip("empty parameter row")
    wide = (0.7 * rng.standard_normal((B, P + pad))).astype(np.float32)
    t = wide[:, :P]
    y = rng.standard_normal((1 if ybc else B, d)).astype(np.float32)
    tw = torch.from_numpy(wide).cuda()
    lp, s = ops.chain_log_prob(torch.from_numpy(y).cuda(), tw[:, :P], ft, d, tr, want_sum=True)
    ref64 = O.chain_log_prob(y, t, ft, d, tr, np.float64)
    ref32 = O.chain_log_prob(y, t, ft, d, tr, np.float32)
    bound = O.tolerance_bound(ref64, ref32)
    ok = np.isfinite(ref64)
    check_forward(lp.cpu().numpy(), ref64, ref32, f"fuzz {seed} forward d={d} K={len(ft)} B={B}", nonfinite="match",
                  kind="fuzz", sensitivity=fp32_sensitivity(y, t, ft, d, tr))
    assert abs(s.item() - ref64[ok].sum()) <= bound[ok].sum() + 1e-6 * abs(ref64[ok].sum()) or not ok.all()
    # backward
    nb = min(B, 300)
    _, gt, gy = ops.chain_log_prob_grad(torch.from_numpy(y[:nb] if not ybc else y).cuda(), tw[:nb, :P], ft, d, tr)
    gt64, gy64, dt, dy = G.fp32_spread(y[:nb] if not ybc else y, t[:nb], ft, d, tr, n_perturbed=2)
    for got_g, ref, dev, what in ((gt.cpu().numpy(), gt64, dt, "d/dt"), (gy.cpu().numpy(), gy64, dy, "d/dy")):
        check_grad(got_g, ref, dev, f"fuzz {seed} {what} d={d} K={len(ft)}", nonfinite="ignore")
    # posterior over a few draws
    S = int(rng.integers(1, 5))
    td = (0.7 * rng.standard_normal((S, nb, P))).astype(np.float32)
    post, _ = ops.posterior_lse(torch.from_numpy(y[:nb] if not ybc else y).cuda(), torch.from_numpy(td).cuda(), ft,
                                d, tr)
    r64 = O.posterior_lse(y[:nb] if not ybc else y, td, ft, d, tr, dtype=np.float64)
    r32 = O.posterior_lse(y[:nb] if not ybc else y, td, ft, d, tr, dtype=np.float32)
    check_forward(post.cpu().numpy(), r64, r32, f"fuzz {seed} posterior S={S}", nonfinite="match", kind="fuzz")
