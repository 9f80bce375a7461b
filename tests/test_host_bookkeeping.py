"""Host bookkeeping.  The graph-pinned workspaces (``ops._pin`` / ``take_graph_workspaces``):
a take hands back only the pins made since its mark, so a capture on a pooled stream
handle that another live graph captured on never takes over that graph's workspace
(ADVICE r05).  CPU tensors stand in for the device blocks: only the bookkeeping runs."""

import torch

from normalizingflownetwork_amd import ops


class _FakeStream:
    def __init__(self, handle):
        self.device = type("D", (), {"index": 0})()
        self.cuda_stream = handle


def test_take_is_scoped_by_mark():
    saved = list(ops._graph_workspaces)
    try:
        key = (0, 1234)
        a, b = torch.empty(2), torch.empty(4)
        with ops._ws_lock:
            ops._pin(key, a)  # an earlier graph on this handle, never taken
        mark = ops.graph_pin_mark()
        with ops._ws_lock:
            ops._pin(key, b)  # this capture's block
            ops._pin(key, a)  # reused block already pinned: not pinned twice
        mine = ops.take_graph_workspaces(_FakeStream(1234), mark)
        assert len(mine) == 1 and mine[0] is b
        assert any(p is a for _, _, p in ops._graph_workspaces), "the earlier graph's pin was taken"
        assert not any(p is b for _, _, p in ops._graph_workspaces)
        # a second take with the same mark finds nothing more
        assert ops.take_graph_workspaces(_FakeStream(1234), mark) == []
        # another handle's pins made after the mark are not this stream's
        with ops._ws_lock:
            ops._pin((0, 99), b)
        assert ops.take_graph_workspaces(_FakeStream(1234), mark) == []
        assert len(ops.take_graph_workspaces(_FakeStream(99), mark)) == 1
    finally:
        ops._graph_workspaces[:] = saved


def test_taken_block_is_pinned_again_by_a_later_capture():
    saved = list(ops._graph_workspaces)
    try:
        key, ws = (0, 77), torch.empty(2)
        m0 = ops.graph_pin_mark()
        with ops._ws_lock:
            ops._pin(key, ws)
        assert ops.take_graph_workspaces(_FakeStream(77), m0) == [ws]
        m1 = ops.graph_pin_mark()  # the first graph's owner holds ws; a new capture reuses it
        with ops._ws_lock:
            ops._pin(key, ws)
        assert ops.take_graph_workspaces(_FakeStream(77), m1) == [ws]
    finally:
        ops._graph_workspaces[:] = saved


def test_snapshot_keeps_graph_under_no_grad():
    """``flows.snapshot_rows`` takes an autograd copy whenever ``t`` requires grad, whatever the
    grad mode at the time: a snapshot taken under ``torch.no_grad()`` still sends
    gradients to ``t``; a ``t`` that needs no grad gives a plain copy."""
    from normalizingflownetwork_amd.normalizing_flows.flows import snapshot_rows

    t = torch.randn(8, 30, requires_grad=True)
    with torch.no_grad():
        s = snapshot_rows(t)
    assert s.requires_grad and s.stride(0) == 32 and torch.equal(s.detach(), t.detach())
    (s * 2.0).sum().backward()
    assert torch.equal(t.grad, torch.full_like(t, 2.0))
    tb = torch.randn(1, 30, requires_grad=True).expand(8, 30)
    with torch.no_grad():
        sb = snapshot_rows(tb)
    assert sb.requires_grad and sb.stride(0) == 0
    assert not snapshot_rows(torch.randn(4, 6)).requires_grad
