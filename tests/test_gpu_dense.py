"""Output Dense layer fused into the chain: t = h W + b on
chip (fp32 MFMA), then the chain — against the oracle on t computed in fp64 / fp32."""

import numpy as np
import pytest
import torch

from oracle import nfn_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fast", "precise"])
def math_mode(request, gpu):
    from normalizingflownetwork_amd import ops

    prev = ops.set_math_mode(request.param)
    yield request.param
    ops.set_math_mode(prev)


def _case(ft, d, H, B, seed, bias=True):
    rng = np.random.default_rng(seed)
    P = O.total_param_size(ft, d, True)
    h = rng.standard_normal((B, H)).astype(np.float32)
    W = (rng.standard_normal((H, P)) / np.sqrt(H)).astype(np.float32)
    b = (0.1 * rng.standard_normal(P)).astype(np.float32) if bias else None
    y = rng.standard_normal((B, d)).astype(np.float32)
    t64 = h.astype(np.float64) @ W.astype(np.float64) + (0 if b is None else b.astype(np.float64))
    t32 = (h @ W + (0 if b is None else b)).astype(np.float32)
    return h, W, b, y, t64, t32


@pytest.mark.parametrize("ft,d,H,B", [(("planar", "radial") * 5, 1, 16, 1000), (("radial", "radial"), 1, 4, 333),
                                      (("planar", "radial") * 5, 1, 64, 777), (("affine", "planar", "radial"), 3, 8, 300),
                                      (("radial",) * 10, 1, 32, 64), (("planar", "affine"), 8, 16, 129),
                                      # d = 1 with 3 and 4 sixteen-column N tiles (P = 44, 50), H = 8 / 32
                                      (("radial",) * 14, 1, 8, 1001), (("planar", "radial") * 8, 1, 32, 700)])
def test_dense_matches_oracle(math_mode, ft, d, H, B):
    from normalizingflownetwork_amd import ops

    h, W, b, y, t64, t32 = _case(ft, d, H, B, seed=H + B)
    out, s = ops.chain_log_prob_dense(torch.from_numpy(y).cuda(), torch.from_numpy(h).cuda(), torch.from_numpy(W).cuda(),
                                      torch.from_numpy(b).cuda(), ft, d, True, want_sum=True)
    ref64 = O.chain_log_prob(y, t64, ft, d, True, np.float64)
    ref32 = O.chain_log_prob(y, t32, ft, d, True, np.float32)
    got = out.cpu().numpy()
    bound = O.tolerance_bound(ref64, ref32)
    bad = ~(np.abs(got - ref64) <= bound)
    assert not bad.any(), (int(bad.sum()), got[bad][:4], ref64[bad][:4])
    assert abs(s.item() - ref64.sum()) <= bound.sum() + 1e-6 * abs(ref64.sum())


def test_dense_with_normalisation_and_fallback(gpu):
    """With and without bias, with the fused y normalisation, and through the
    unsupported-shape fallback (H = 10: library GEMM + chain kernel), against the
    oracle's log_pdf on t = h W + b."""
    from normalizingflownetwork_amd import ops

    ft, d = ("planar", "radial") * 3, 1
    ym, ys = np.array([0.3], np.float32), np.array([1.4], np.float32)
    for H, bias in ((16, True), (8, False), (10, True)):
        h, W, b, y, t64, t32 = _case(ft, d, H, 513, seed=H, bias=bias)
        bb = None if b is None else torch.from_numpy(b).cuda()
        out, _ = ops.chain_log_prob_dense(torch.from_numpy(y).cuda(), torch.from_numpy(h).cuda(),
                                          torch.from_numpy(W).cuda(), bb, ft, d, True, ym, ys)
        ref64 = O.log_pdf(y, t64, ft, d, True, ym, ys, np.float64)
        ref32 = O.log_pdf(y, t32, ft, d, True, ym, ys, np.float32)
        assert np.all(np.abs(out.cpu().numpy() - ref64) <= O.tolerance_bound(ref64, ref32)), H
