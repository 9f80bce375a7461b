"""Host-side API mirror of the reference (no compute): the shape / size / order /
assertion checks of tests/test_flows.py and tests/test_distribution_layers.py,
re-expressed against normalizingflownetwork_amd."""

import numpy as np
import torch
import pytest

from normalizingflownetwork_amd import FLOWS, AffineFlow, InverseNormalizingFlowLayer, PlanarFlow, RadialFlow
from normalizingflownetwork_amd.distribution_layers import TensorShape
from normalizingflownetwork_amd.parallel import shard_bounds


def test_registry():
    assert FLOWS == {"planar": PlanarFlow, "radial": RadialFlow, "affine": AffineFlow}


@pytest.mark.parametrize("name", ["planar", "radial", "affine"])
def test_param_width_assertion_and_event_ndims(name):
    # tests/test_flows.py:13-23
    for dim in (1, 4):
        cls = FLOWS[name]
        with pytest.raises(AssertionError):
            cls(np.ones((10, cls.get_param_size(dim) + 1), np.float32), dim)
        flow = cls(np.ones((10, cls.get_param_size(dim)), np.float32), dim)
        ref = AffineFlow(np.ones((10, AffineFlow.get_param_size(dim)), np.float32), dim)
        assert flow.forward_min_event_ndims == ref.forward_min_event_ndims == 1
        assert flow.inverse_min_event_ndims == 1


def test_total_param_size_nf():
    # tests/test_distribution_layers.py:65-73
    layer1 = InverseNormalizingFlowLayer(("planar", "radial", "affine"), n_dims=1, trainable_base_dist=False)
    layer2 = InverseNormalizingFlowLayer(("planar", "radial", "affine"), n_dims=3, trainable_base_dist=True)
    assert layer1.get_total_param_size() == 3 + 3 + 2
    assert layer2.get_total_param_size() == (3 + 3 + 1) + (3 + 1 + 1) + (3 + 3) + (3 + 3)


def test_unknown_flow_type():
    with pytest.raises(AssertionError):
        InverseNormalizingFlowLayer(("planar", "banana"), n_dims=1)


def test_nf_dist_fn_shapes():
    # tests/test_distribution_layers.py:203-231
    dist_fn = InverseNormalizingFlowLayer._get_distribution_fn(n_dims=1, flow_types=("radial", "planar"),
                                                               trainable_base_dist=False)
    dist = dist_fn(np.ones((1, 6), np.float32))
    assert dist.event_shape == [1]
    assert dist.batch_shape == [1]
    dist = dist_fn(np.ones((3, 6), np.float32))
    assert dist.event_shape == [1]
    assert dist.batch_shape == [3]
    with pytest.raises(AssertionError):
        dist_fn(np.ones((10, 7), np.float32))
    dist_fn = InverseNormalizingFlowLayer._get_distribution_fn(n_dims=2, flow_types=("radial", "planar"),
                                                               trainable_base_dist=True)
    dist = dist_fn(np.ones((1, 13), np.float32))
    assert dist.event_shape == [2]
    assert dist.batch_shape == [1]
    dist = dist_fn(np.ones((3, 13), np.float32))
    assert dist.event_shape == [2]
    assert dist.batch_shape == [3]
    with pytest.raises(AssertionError):
        dist_fn(np.ones((10, 12), np.float32))


def test_get_bijector_order():
    # tests/test_distribution_layers.py:234-249
    out = InverseNormalizingFlowLayer._get_bijector(np.zeros((10, 8), np.float32), ("planar", "radial", "affine"), 1)
    assert len(out.bijectors) == 3
    assert out.inverse_min_event_ndims == 1
    assert type(out.bijectors[0]) == FLOWS["affine"]
    assert type(out.bijectors[1]) == FLOWS["radial"]
    assert type(out.bijectors[2]) == FLOWS["planar"]
    out = InverseNormalizingFlowLayer._get_bijector(np.zeros((10, 9), np.float32), ("planar", "radial"), 2)
    assert len(out.bijectors) == 2
    assert out.inverse_min_event_ndims == 1
    with pytest.raises(AssertionError):
        InverseNormalizingFlowLayer._get_bijector(np.zeros((10, 8), np.float32), ("planar", "radial"), 2)


def test_get_bijector_blocks_are_reversed():
    """bijectors[0] (last flow type) owns the FIRST block after the base."""
    t = np.arange(8, dtype=np.float32)[None, :]
    chain = InverseNormalizingFlowLayer._get_bijector(t, ("planar", "radial", "affine"), 1)
    np.testing.assert_array_equal(chain.bijectors[0]._t, [[0, 1]])  # affine (2)
    np.testing.assert_array_equal(chain.bijectors[1]._t, [[2, 3, 4]])  # radial (3)
    np.testing.assert_array_equal(chain.bijectors[2]._t, [[5, 6, 7]])  # planar (3)


def test_bijector_inverse_is_not_defined():
    """The reference's flows define no _inverse (DistributionLayers.py:223-226); the
    host mirror keeps that.  Sampling the distribution is this build's extension
    (nfn_chain_sample_f32) and, like every compute path, needs the GPU."""
    with pytest.raises(NotImplementedError):
        RadialFlow(np.ones((2, 3), np.float32), 1).inverse([[0.0]])
    dist = InverseNormalizingFlowLayer(("radial",), 1, False)(np.ones((2, 3), np.float32))
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):
            dist.sample()


def test_tensorshape_semantics():
    assert TensorShape([3]) == [3]
    assert TensorShape([3]) == (3,)
    assert TensorShape([3]) == 3
    assert TensorShape([3]) != [2]
    assert hash(TensorShape([1, 2])) == hash((1, 2))


@pytest.mark.parametrize("n,world", [(10, 3), (1 << 24, 8), (7, 8), (0, 2)])
def test_shard_bounds_partition(n, world):
    spans = [shard_bounds(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, _) in zip(spans, spans[1:]):
        assert b == c and b >= a
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_noise_regularisation_values():
    """BaseEstimator._assign_noise_regularisation (BaseEstimator.py:33-41)."""
    from normalizingflownetwork_amd import NormalizingFlowNetwork

    m = NormalizingFlowNetwork(1, n_flows=1, noise_reg=("rule_of_thumb", 0.1))
    m._assign_noise_regularisation(n_dims=2, n_datapoints=300)
    assert m.x_noise_std == m.y_noise_std == pytest.approx(0.1 * 301 ** (-1 / 6))
    m = NormalizingFlowNetwork(1, n_flows=1, noise_reg=("fixed_rate", 3.0))
    m._assign_noise_regularisation(n_dims=2, n_datapoints=300)
    assert m.x_noise_std == 3.0
    m = NormalizingFlowNetwork(1, n_flows=1, noise_reg=("bogus", 3.0))
    with pytest.raises(AssertionError):
        m._assign_noise_regularisation(n_dims=2, n_datapoints=300)


def test_split_pays_rule():
    # ops.split_pays: the per-flow calls read one-pass copies of their blocks only where the
    # expected bytes say so (C2: 10 blocks of 3 floats in 32-float rows; C3: affine + 4 planar
    # + 4 radial at d = 8 in 140-float rows)
    from normalizingflownetwork_amd import ops
    assert ops.split_pays([3] * 10, 32)
    assert not ops.split_pays([16] + [17] * 4 + [10] * 4, 140)
    # a wide row holding one narrow block: the split would read the whole row for 12 B
    assert not ops.split_pays([3], 1024)


def test_get_bijector_snapshots_t():
    """TF's slices in _get_bijector are copies (DistributionLayers.py:267-278): the flows own
    a snapshot of t taken when the Chain is built, so a later write to t — in place, through
    a raw pointer or a graph replay — does not reach them.  The snapshot keeps t's values,
    puts each row start on a 16-byte boundary (C2: 2 lead + 30 columns) and keeps a
    broadcast (stride-0) row a single row."""
    from normalizingflownetwork_amd.normalizing_flows.flows import snapshot_rows

    ft = ("planar", "radial") * 5
    t = torch.randn(64, 32)
    chain = InverseNormalizingFlowLayer._get_bijector(t[:, 2:], ft, 1)
    before = [f._t.clone() for f in chain.bijectors]
    t.mul_(3.0)
    for f, b in zip(chain.bijectors, before):
        assert torch.equal(f._t, b)
    snap = chain.bijectors[0]._t
    assert snap.stride(0) == 32 and snap.storage_offset() == 2
    s = snapshot_rows(t[:, 1:])  # W = 31: 1 lead column
    assert torch.equal(s, t[:, 1:]) and s.stride(0) == 32 and s.storage_offset() == 1
    row = torch.randn(1, 30).expand(1000, 30)
    s = snapshot_rows(row)
    assert s.stride(0) == 0 and torch.equal(s, row) and s.data_ptr() != row.data_ptr()


def test_split_group_skips_broadcast_rows():
    """A stride-0 (broadcast) parameter row is read once per cache line by the flows'
    own launches already: no split (nfn_split_blocks_f32 needs real rows)."""
    ft = ("planar", "radial") * 5
    chain = InverseNormalizingFlowLayer._get_bijector(torch.randn(1, 30).expand(4096, 30), ft, 1)
    assert chain.bijectors[0]._split[0].pays is False
    chain = InverseNormalizingFlowLayer._get_bijector(torch.randn(4096, 32)[:, 2:], ft, 1)
    assert chain.bijectors[0]._split[0].pays is True


def test_distribution_builds_its_bijector_on_first_use():
    """FlowDistribution checks the width at construction (AssertionError, as the reference)
    but builds the Chain — and the flows' parameter snapshot — only when ``bijector`` is
    first read: log_prob never pays for the copy."""
    layer = InverseNormalizingFlowLayer(("planar", "radial"), 1, True)
    dist = layer(torch.zeros(8, 8))
    assert dist._bijector is None
    b = dist.bijector
    assert b is dist.bijector and len(b.bijector.bijectors) == 2
    with pytest.raises(AssertionError):
        layer(torch.zeros(8, 9))
