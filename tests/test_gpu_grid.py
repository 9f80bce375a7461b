"""Density-grid evaluation (flow_plotting.py:33-53) against
the oracle: every (grid value, parameter row) pair, with and without the fused y
normalisation, broadcast parameter rows and ragged sizes; and the heatmap helper
against a per-row loop of ``dist.prob``."""

import numpy as np
import pytest
import torch

from oracle import nfn_oracle as O
from parity import check_forward

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fast", "precise"])
def math_mode(request, gpu):
    from normalizingflownetwork_amd import ops

    prev = ops.set_math_mode(request.param)
    yield request.param
    ops.set_math_mode(prev)


def _ref(yg, t, ft, d, tr, ym=None, ys=None):
    r64 = np.stack([O.log_pdf(np.broadcast_to(g, (1, d)), t, ft, d, tr, ym, ys, np.float64) for g in yg])
    r32 = np.stack([O.log_pdf(np.broadcast_to(g, (1, d)), t, ft, d, tr, ym, ys, np.float32) for g in yg])
    return r64, r32


@pytest.mark.parametrize("ft,d,B,G", [(("planar", "radial") * 5, 1, 300, 17), (("radial",) * 3, 1, 1, 101),
                                      (("affine", "planar", "radial"), 3, 129, 9),
                                      (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8, 70, 33)])
def test_grid_matches_oracle(math_mode, ft, d, B, G):
    from normalizingflownetwork_amd import ops

    rng = np.random.default_rng(B + G)
    P = O.total_param_size(ft, d, True)
    t = rng.standard_normal((B, P)).astype(np.float32)
    yg = rng.standard_normal((G, d)).astype(np.float32) * 2
    out = ops.chain_log_prob_grid(torch.from_numpy(yg).cuda(), torch.from_numpy(t).cuda(), ft, d, True)
    r64, r32 = _ref(yg, t, ft, d, True)
    assert out.shape == (G, B)
    check_forward(out.cpu().numpy(), r64, r32, f"grid {ft[:2]}x{len(ft)} d={d} B={B} G={G} [{math_mode}]", kind="grid")
    ym, ys = np.linspace(-0.2, 0.3, d).astype(np.float32), np.linspace(0.5, 2.0, d).astype(np.float32)
    outn = ops.chain_log_prob_grid(torch.from_numpy(yg).cuda(), torch.from_numpy(t).cuda(), ft, d, True, ym, ys)
    r64, r32 = _ref(yg, t, ft, d, True, ym, ys)
    check_forward(outn.cpu().numpy(), r64, r32, f"grid normalised {ft[:2]}x{len(ft)} d={d} [{math_mode}]", kind="grid")
    # a broadcast parameter row gives the same column for every b
    out1 = ops.chain_log_prob_grid(torch.from_numpy(yg).cuda(), torch.from_numpy(t[:1]).cuda(), ft, d, True)
    assert torch.equal(out1[:, 0], out[:, 0])


def test_grid_equals_per_row_prob(gpu):
    """flow_plotting.plot_model's loop (dist.prob(y[i]) per grid row) == the grid kernel."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer
    from normalizingflownetwork_amd.flow_plotting import model_density_heatmap

    class _Model:  # the surface plot_model uses: __call__(x) -> dist, y_mean, y_std
        def __init__(self):
            self.layer = InverseNormalizingFlowLayer(("radial", "planar"), 1, True)
            rng = np.random.default_rng(3)
            self.W = rng.standard_normal((1, self.layer.get_total_param_size())).astype(np.float32)
            self.y_mean = np.array([0.4], np.float32)
            self.y_std = np.array([1.7], np.float32)

        def __call__(self, x):
            return self.layer(torch.from_numpy(np.asarray(x, np.float32) @ self.W).cuda())

    m = _Model()
    x = np.linspace(-2, 2, 50, dtype=np.float32).reshape(-1, 1)
    heat = model_density_heatmap(x, m, (-3, 3), y_num=40)
    dist = m(x)
    y = (np.linspace(3, -3, 40).reshape(40, 1) - m.y_mean) / m.y_std
    loop = np.stack([dist.prob(y[i].astype(np.float32)).cpu().numpy() for i in range(40)]) / np.sum(m.y_std)
    np.testing.assert_allclose(heat, loop, rtol=1e-5, atol=1e-30)  # exp of log_prob < -87 is denormal


def test_grid_launcher_equals_op(gpu):
    """bench.py --mode grid's pre-bound launcher computes what ops.chain_log_prob_grid does,
    at the bench's shape (G = 256 grid values x 2^16 C2 parameter rows), and matches the
    oracle on a random subset of (g, b) pairs."""
    from normalizingflownetwork_amd import ops

    ft, d = ("planar", "radial") * 5, 1
    P = O.total_param_size(ft, d, True)
    G, B = 256, 1 << 16
    gen = torch.Generator(device="cuda").manual_seed(5)
    t = torch.randn((B, P), generator=gen, device="cuda")
    yg = torch.linspace(-4.0, 4.0, G, device="cuda").reshape(G, 1).contiguous()
    lz = ops.GridLauncher(yg, t, ft, d, True)
    lz.launch()
    ref = ops.chain_log_prob_grid(yg, t, ft, d, True)
    torch.cuda.synchronize()
    assert torch.equal(lz.out, ref)
    rng = np.random.default_rng(0)
    gi, bi = rng.integers(0, G, 2048), rng.integers(0, B, 2048)
    tn, ygn = t.cpu().numpy(), yg.cpu().numpy()
    r64 = O.log_pdf(ygn[gi], tn[bi], ft, d, True, None, None, np.float64)
    r32 = O.log_pdf(ygn[gi], tn[bi], ft, d, True, None, None, np.float32)
    check_forward(lz.out.cpu().numpy()[gi, bi], r64, r32, "grid bench shape G=256 B=2^16 (2048 pairs)", kind="grid")


@pytest.mark.parametrize("ft", [("planar", "radial") * 5, ("affine", "radial", "planar"), ("radial",) * 3])
def test_grid_d1_equals_fused_log_prob_bitwise(gpu, ft):
    """At d = 1 (fast math) the grid forms each flow's parameter-only terms once per row
    and runs only the z-dependent part per grid value: the same expressions as the fused
    log_prob kernels, so every (g, b) equals log_prob(y_g | t_b) of ops.chain_log_prob
    bit for bit (normalised y included)."""
    from normalizingflownetwork_amd import ops

    prev = ops.set_math_mode("fast")
    try:
        d = 1
        P = O.total_param_size(ft, d, True)
        rng = np.random.default_rng(len(ft))
        B, G = 1000, 7
        t = torch.from_numpy(rng.standard_normal((B, P)).astype(np.float32)).cuda()
        yg = torch.from_numpy((rng.standard_normal((G, 1)) * 2).astype(np.float32)).cuda()
        for ym, ys in ((None, None), (np.array([0.3], np.float32), np.array([1.7], np.float32))):
            grid = ops.chain_log_prob_grid(yg, t, ft, d, True, ym, ys)
            for g in range(G):
                lp, _ = ops.chain_log_prob(yg[g:g + 1].expand(B, 1).contiguous(), t, ft, d, True, ym, ys)
                assert torch.equal(grid[g], lp), (ft, g, ym is not None)
    finally:
        ops.set_math_mode(prev)
