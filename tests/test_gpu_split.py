"""The per-flow Bijector path over the views ``InverseNormalizingFlowLayer._get_bijector``
hands each flow (``estimators/DistributionLayers.py:267-278``): the flows' blocks are made
contiguous in ONE pass (``nfn_split_blocks_f32``; TF's slices are copies) on the first
single-flow call, and every flow's launch reads its own copy.  Checked bitwise against the
same launches on torch-made contiguous copies and on the strided views, with the cache
remade after an in-place change of ``t``."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("widths,B,extra,col0", [([3] * 10, 4099, 0, 2), ([16] + [17] * 4 + [10] * 4, 1000, 0, 16),
                                                 ([65] * 5, 333, 0, 0), ([3, 3], 1, 0, 2), ([2, 5, 1], 257, 7, 1),
                                                 ([3, 3], 300, 100, 3), ([3] * 10, (1 << 20) + 3, 0, 2)])
def test_split_blocks_equals_slices(gpu, widths, B, extra, col0):
    """Dense rows (the 16-byte span loads, 0-3 floats of misalignment) and sparse rows
    (stride > W + 32: row-by-row loads), ragged batches, one row."""
    from normalizingflownetwork_amd import ops

    W = sum(widths)
    gen = torch.Generator(device=gpu).manual_seed(B + W)
    wide = torch.randn((B, W + extra + col0), generator=gen, device=gpu)
    t = wide[:, col0:col0 + W]  # a column view of a wider row (stride W + extra + col0)
    got = ops.split_blocks(t, widths)
    off = 0
    for w, blk in zip(widths, got):
        assert blk.shape == (B, w) and blk.is_contiguous()
        assert torch.equal(blk, t[:, off:off + w].contiguous())
        off += w


def _layer_flows(ft, d, t):
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer

    return InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d).bijectors


@pytest.mark.parametrize("ft,d,B", [(("planar", "radial") * 5, 1, 5000), (("affine", "planar", "radial"), 3, 777)])
def test_per_flow_calls_read_split_copies(gpu, ft, d, B):
    from normalizingflownetwork_amd import ops
    from normalizingflownetwork_amd.normalizing_flows import FLOWS

    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device=gpu).manual_seed(B)
    t = torch.randn((B, P), generator=gen, device=gpu)
    z0 = torch.randn((B, d), generator=gen, device=gpu)
    flows = _layer_flows(ft, d, t)
    group = flows[0]._split[0]
    assert all(f._split[0] is group for f in flows)

    def run(fs):
        z, out = z0, []
        for f in reversed(fs):  # bijectors[-1] applies first (tfp Chain)
            z, l = f.forward_and_log_det_jacobian(z)
            out.append((z.clone(), l.clone()))
        return out

    got = run(flows)
    blocks = group.blocks()
    assert all(f._kernel_params().data_ptr() == blocks[k].data_ptr() for k, f in enumerate(flows))
    ref_copy = run([FLOWS[type(f).flow_type](f.params.contiguous(), d) for f in flows])
    ref_view = run([FLOWS[type(f).flow_type](f.params, d) for f in flows])
    for (zg, lg), (zc, lc), (zv, lv) in zip(got, ref_copy, ref_view):
        assert torch.equal(zg, zc) and torch.equal(lg, lc)
        assert torch.equal(zg, zv) and torch.equal(lg, lv)
    # the split is made once and reused while the flows' parameters are unchanged
    assert group.blocks()[0] is blocks[0]
    # the flows own a snapshot of t (TF's slices are copies): a write to t does not reach them
    t.mul_(0.5)
    again = run(flows)
    assert group.blocks()[0] is blocks[0]
    for (zg, lg), (za, la) in zip(got, again):
        assert torch.equal(zg, za) and torch.equal(lg, la)
    # an in-place change of a flow's own parameters is seen: the copies are remade
    flows[-1].params.mul_(0.5)
    got2 = run(flows)
    assert group.blocks()[0] is not blocks[0]
    ref2 = run([FLOWS[type(f).flow_type](f.params.contiguous(), d) for f in flows])
    for (zg, lg), (zc, lc) in zip(got2, ref2):
        assert torch.equal(zg, zc) and torch.equal(lg, lc)
    assert not torch.equal(got2[0][0], got[0][0])
    group.release()
    assert group._blocks is None
    got3 = run(flows)
    for (zg, lg), (zc, lc) in zip(got3, ref2):
        assert torch.equal(zg, zc) and torch.equal(lg, lc)


def test_one_launch_chain_makes_no_copies(gpu):
    """The Chain's one-launch path reads the wide rows directly: calling it leaves the
    layer's split group empty (no 2 B-per-parameter copy is made unless a flow is called
    on its own)."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer, ops

    ft, d, B = ("planar", "radial") * 3, 1, 3000
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device=gpu).manual_seed(7)
    t = torch.randn((B, P), generator=gen, device=gpu)
    z = torch.randn((B, d), generator=gen, device=gpu)
    chain = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d)
    assert chain._fused() is not None
    chain.forward(z)
    chain.forward_log_det_jacobian(z, event_ndims=1)
    assert chain.bijectors[0]._split[0]._blocks is None
    chain.bijectors[-1].forward(z)  # a single flow on its own: now the copies exist
    assert chain.bijectors[0]._split[0]._blocks is not None


def test_inference_mode_tensor_reads_wide_rows(gpu):
    """A ``t`` made under ``torch.inference_mode()`` has no version counter, so its copies
    could not be checked against in-place changes: the flows then read the wide rows
    directly (the same values, no copies)."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer, ops
    from normalizingflownetwork_amd.normalizing_flows import FLOWS

    ft, d, B = ("planar", "radial") * 2, 1, 2000
    P = ops.total_param_size(ft, d, True)
    with torch.inference_mode():
        gen = torch.Generator(device=gpu).manual_seed(8)
        t = torch.randn((B, P), generator=gen, device=gpu)
        z = torch.randn((B, d), generator=gen, device=gpu)
        flows = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d).bijectors
        f = flows[0]
        zg, lg = f.forward_and_log_det_jacobian(z)
        assert f._split[0]._blocks is None and f._kernel_params().data_ptr() == f.params.data_ptr()
        zc, lc = FLOWS[type(f).flow_type](f.params.contiguous(), d).forward_and_log_det_jacobian(z)
        assert torch.equal(zg, zc) and torch.equal(lg, lc)


def test_graph_replay_into_t_does_not_reach_built_flows(gpu):
    """A HIP-graph replay whose static output is t changes t without torch's version
    counter.  Flows built by _get_bijector before the replay keep evaluating the
    parameters they were built from (their snapshot, also through the split copies); a
    Chain built after it sees the new values."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer, ops
    from normalizingflownetwork_amd.normalizing_flows import FLOWS

    ft, d, B = ("planar", "radial") * 5, 1, 4099
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device=gpu).manual_seed(11)
    t = torch.randn((B, P), generator=gen, device=gpu)
    src = torch.randn((B, P), generator=gen, device=gpu)
    z0 = torch.randn((B, d), generator=gen, device=gpu)
    chain = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d)

    def run(fs):
        z, out = z0, []
        for f in reversed(fs):
            z, l = f.forward_and_log_det_jacobian(z)
            out.append((z.clone(), l.clone()))
        return out

    ref_old = run([FLOWS[type(f).flow_type](f.params.contiguous(), d) for f in chain.bijectors])
    first = run(chain.bijectors)  # makes the split copies
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            t.copy_(src)
    t.zero_()  # the capture did not run the copy
    ver = t._version
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(t, src) and t._version == ver
    after = run(chain.bijectors)
    for (za, la), (zr, lr), (zf, lf) in zip(after, ref_old, first):
        assert torch.equal(za, zr) and torch.equal(la, lr) and torch.equal(za, zf)
    z1, l1 = chain.forward_and_log_det_jacobian(z0)  # the one-launch Chain reads the snapshot too
    new = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d)
    ref_new = run([FLOWS[type(f).flow_type](src[:, 2 * d:][:, o:o + f.get_param_size(d)].contiguous(), d)
                   for f, o in zip(new.bijectors, _offsets(new, d))])
    got_new = run(new.bijectors)
    for (zg, lg), (zr, lr) in zip(got_new, ref_new):
        assert torch.equal(zg, zr) and torch.equal(lg, lr)
    zo, lo = chain.forward_and_log_det_jacobian(z0)
    zn, ln = new.forward_and_log_det_jacobian(z0)
    assert torch.equal(zo, z1) and not torch.equal(zo, zn)


def _offsets(chain, d):
    offs, o = [], 0
    for f in chain.bijectors:
        offs.append(o)
        o += f.get_param_size(d)
    return offs


@pytest.mark.parametrize("ft,d", [(("planar", "radial") * 5, 1), (("affine", "planar", "radial"), 3)])
def test_per_flow_over_broadcast_row(gpu, ft, d):
    """t = one row expanded to B rows (stride 0): the flows read the broadcast row (no
    split: nfn_split_blocks_f32 needs real rows) and match flows over materialised rows."""
    from normalizingflownetwork_amd import InverseNormalizingFlowLayer, ops
    from normalizingflownetwork_amd.normalizing_flows import FLOWS

    B = 3001
    P = ops.total_param_size(ft, d, False)
    gen = torch.Generator(device=gpu).manual_seed(5)
    row = torch.randn((1, P), generator=gen, device=gpu)
    z = torch.randn((B, d), generator=gen, device=gpu)
    chain = InverseNormalizingFlowLayer._get_bijector(row.expand(B, P), ft, d)
    assert chain.bijectors[0]._split[0].pays is False
    full = InverseNormalizingFlowLayer._get_bijector(row.expand(B, P).contiguous(), ft, d)
    for f, g in zip(reversed(chain.bijectors), reversed(full.bijectors)):
        za, la = f.forward_and_log_det_jacobian(z)
        zb, lb = FLOWS[type(g).flow_type](g.params.contiguous(), d).forward_and_log_det_jacobian(z)
        assert torch.equal(za, zb) and torch.equal(la, lb)
        z = za
