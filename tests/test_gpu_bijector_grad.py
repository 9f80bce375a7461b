"""The per-flow Bijector API is differentiable (verdict r04, Missing 1): gradients of a loss on
``flow.forward`` / ``forward_log_det_jacobian`` reach ``z`` and the flow's parameters through
the HIP backward ``nfn_flow_vjp_f32``, as TF's tape reaches them through
``PlanarFlow._forward`` / ``_forward_log_det_jacobian`` (``PlanarFlow.py:68-80``),
``RadialFlow.py:50-70`` (its own ``GradientTape`` included) and tfp ``Affine``.

Checked against the per-flow autodiff oracle (``oracle.nfn_grad_oracle.flow_vjp``) at the
gradient gate ``grad_tolerance`` = max(2e-5 max(1, |g64|, rowmax|g64| / 64), 8 dev32), dev32 the
fp32 restatement's largest deviation over the inputs and three one-ulp perturbations."""

import numpy as np
import pytest
import torch

from conftest import FLOW_FIXTURES, load_golden
from parity import check_grad
from oracle import nfn_grad_oracle as G

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fast", "precise"])
def math_mode(request, gpu):
    from normalizingflownetwork_amd import ops

    prev = ops.set_math_mode(request.param)
    yield request.param
    ops.set_math_mode(prev)


def _cot(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


@pytest.mark.parametrize("name", FLOW_FIXTURES)
def test_flow_forward_and_fldj_gradients_vs_oracle(gpu, math_mode, name):
    from normalizingflownetwork_amd import FLOWS

    g = load_golden(name)
    ftype, d = name.split("_")[1], g["d"]
    z, t = g["z"].astype(np.float32), g["t"].astype(np.float32)
    gz, gl = _cot(z.shape, 1), _cot((z.shape[0],), 2)
    zt = torch.tensor(z, device=gpu, requires_grad=True)
    tt = torch.tensor(t, device=gpu, requires_grad=True)
    flow = FLOWS[ftype](tt, d)
    z_out, ldj = flow.forward_and_log_det_jacobian(zt)
    assert z_out.grad_fn is not None and ldj.grad_fn is not None
    loss = (z_out * torch.tensor(gz, device=gpu)).sum() + (ldj * torch.tensor(gl, device=gpu)).sum()
    loss.backward()
    gz64, gt64, dz32, dt32 = G.flow_vjp_spread(ftype, z, t, d, gz, gl)
    check_grad(zt.grad.cpu().numpy(), gz64, dz32, f"{name} d/dz [{math_mode}]")
    check_grad(tt.grad.cpu().numpy(), gt64, dt32, f"{name} d/dt [{math_mode}]")


@pytest.mark.parametrize("name", ["flow_planar_d1", "flow_radial_d4", "flow_affine_d4"])
def test_separate_entry_points_are_differentiable(gpu, name):
    """``forward`` alone and ``forward_log_det_jacobian`` alone each carry their own gradient."""
    from normalizingflownetwork_amd import FLOWS

    g = load_golden(name)
    ftype, d = name.split("_")[1], g["d"]
    z, t = g["z"].astype(np.float32), g["t"].astype(np.float32)
    gz = _cot(z.shape, 3)
    for which in ("forward", "fldj"):
        zt = torch.tensor(z, device=gpu, requires_grad=True)
        tt = torch.tensor(t, device=gpu, requires_grad=True)
        flow = FLOWS[ftype](tt, d)
        if which == "forward":
            (flow.forward(zt) * torch.tensor(gz, device=gpu)).sum().backward()
            ref = G.flow_vjp_spread(ftype, z, t, d, g_z=gz)
        else:
            flow.forward_log_det_jacobian(zt, event_ndims=1).sum().backward()
            ref = G.flow_vjp_spread(ftype, z, t, d, g_ldj=np.ones(z.shape[0], np.float32))
        check_grad(zt.grad.cpu().numpy(), ref[0], ref[2], f"{name} {which} d/dz")
        check_grad(tt.grad.cpu().numpy(), ref[1], ref[3], f"{name} {which} d/dt")


def test_broadcast_rows_sum_their_gradients(gpu):
    """A batch-1 ``z`` against B parameter rows (tests/test_flows.py:22-29) gets the summed
    gradient, and a batch-1 parameter row against B inputs likewise."""
    from normalizingflownetwork_amd import FLOWS

    g = load_golden("flow_radial_d4")
    d = g["d"]
    z, t = g["z"].astype(np.float32), g["t"].astype(np.float32)
    gl = np.ones(len(t), np.float32)
    zt = torch.tensor(z[:1], device=gpu, requires_grad=True)
    tt = torch.tensor(t, device=gpu, requires_grad=True)
    FLOWS["radial"](tt, d).forward_log_det_jacobian(zt, event_ndims=1).sum().backward()
    gz64, gt64, dz32, dt32 = G.flow_vjp_spread("radial", z[:1], t, d, g_ldj=gl)
    assert zt.grad.shape == (1, d)
    check_grad(zt.grad.cpu().numpy(), gz64.sum(0, keepdims=True), dz32.sum(0, keepdims=True), "bcast z d/dz")
    check_grad(tt.grad.cpu().numpy(), gt64, dt32, "bcast z d/dt")
    zt = torch.tensor(z, device=gpu, requires_grad=True)
    t1 = torch.tensor(t[:1], device=gpu, requires_grad=True)
    FLOWS["radial"](t1, d).forward_log_det_jacobian(zt, event_ndims=1).sum().backward()
    gz64, gt64, dz32, dt32 = G.flow_vjp_spread("radial", z, t[:1], d, g_ldj=gl)
    assert t1.grad.shape == (1, d + 2)
    check_grad(t1.grad.cpu().numpy(), gt64.sum(0, keepdims=True), dt32.sum(0, keepdims=True), "bcast t d/dt")
    check_grad(zt.grad.cpu().numpy(), gz64, dz32, "bcast t d/dz")


@pytest.mark.parametrize("name", ["asym_pra_d3", "c2_pr5_d1"])
def test_layer_bijector_gradients_reach_t(gpu, name):
    """The layer's ``dist.bijector`` (``Invert(Chain(flows))`` over a snapshot of t) is
    differentiable end to end: d/dt and d/dy of ``sum(bijector.forward(y)) +
    sum(bijector.forward_log_det_jacobian(y))`` — here ``Invert``'s forward is the Chain's
    inverse, so the Chain is used directly, as ``log_prob`` does — against the chain of
    per-flow oracles, and the gradient of ``log_prob`` through the Chain's pieces equals the
    fused backward's."""
    from conftest import load_golden as lg
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer, ops

    fx = lg(name)
    ft, d, tr = fx["flow_types"], fx["d"], bool(fx["trainable"])
    y, t = fx["y"][:512].astype(np.float32), fx["t"][:512].astype(np.float32)
    layer = InverseNormalizingFlowLayer(ft, d, tr)
    tt = torch.tensor(t, device=gpu, requires_grad=True)
    yt = torch.tensor(y, device=gpu, requires_grad=True)
    dist = layer(tt)
    chain = dist.bijector.bijector
    assert chain._fused(yt) is None  # gradients wanted: flow by flow through the autograd op
    x, ldj = chain.forward_and_log_det_jacobian(yt)
    # base log-density of the trainable MVNDiag on top (DistributionLayers.py:280-294)
    base = dist.distribution.log_prob(x)
    (base + ldj).sum().backward()
    g_t, g_y = tt.grad.cpu().numpy(), yt.grad.cpu().numpy()
    _, gt_f, gy_f = ops.chain_log_prob_grad(torch.tensor(y, device=gpu), torch.tensor(t, device=gpu), ft, d, tr)
    gt64, gy64, dt32, dy32 = G.fp32_spread(y, t, ft, d, tr)
    check_grad(g_t, gt64, dt32, f"{name} bijector pieces d/dt")
    check_grad(g_y, gy64, dy32, f"{name} bijector pieces d/dy")
    check_grad(gt_f.cpu().numpy(), gt64, dt32, f"{name} fused d/dt")


def test_no_grad_keeps_the_one_launch_chain(gpu):
    """Without a gradient request the Chain still runs as ONE launch, and the results equal
    the differentiable path's values."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer

    fx = load_golden("c2_pr5_d1")
    ft, d, tr = fx["flow_types"], fx["d"], bool(fx["trainable"])
    y, t = fx["y"][:256], fx["t"][:256]
    layer = InverseNormalizingFlowLayer(ft, d, tr)
    t_dev = torch.tensor(t, device=gpu)
    chain = layer(t_dev).bijector.bijector
    y_dev = torch.tensor(y, device=gpu)
    assert chain._fused(y_dev) is not None
    x0, l0 = chain.forward_and_log_det_jacobian(y_dev)
    y_req = y_dev.clone().requires_grad_(True)
    x1, l1 = chain.forward_and_log_det_jacobian(y_req)
    assert x1.grad_fn is not None
    np.testing.assert_allclose(x1.detach().cpu().numpy(), x0.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(l1.detach().cpu().numpy(), l0.cpu().numpy(), rtol=1e-5, atol=1e-5)
    with torch.no_grad():
        assert chain._fused(y_req) is not None


def test_bijector_first_built_under_no_grad_still_differentiates(gpu):
    """``dist.bijector`` caches its Chain (and the parameter snapshot) on FIRST access.  When
    that access happens under ``torch.no_grad()`` (e.g. while sampling), later grad-enabled
    forward / fldj calls must still reach ``t`` — as TF's tape would: the same
    gradients as a bijector built with grad mode on."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer

    fx = load_golden("asym_pra_d3")
    ft, d, tr = fx["flow_types"], fx["d"], bool(fx["trainable"])
    y, t = fx["y"][:256].astype(np.float32), fx["t"][:256].astype(np.float32)
    layer = InverseNormalizingFlowLayer(ft, d, tr)
    grads = []
    for first_no_grad in (False, True):
        tt = torch.tensor(t, device=gpu, requires_grad=True)
        dist = layer(tt)
        if first_no_grad:
            with torch.no_grad():
                chain = dist.bijector.bijector
                chain.forward_and_log_det_jacobian(torch.tensor(y, device=gpu))  # sampling-like use
        else:
            chain = dist.bijector.bijector
        x, ldj = chain.forward_and_log_det_jacobian(torch.tensor(y, device=gpu))
        assert ldj.requires_grad, "the cached Chain lost its graph to t"
        (x.sum() + ldj.sum()).backward()
        grads.append(tt.grad.cpu().numpy())
    np.testing.assert_array_equal(grads[1], grads[0])
