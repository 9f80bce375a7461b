"""Workspace, reduction and multi-stream correctness of the C ABI (round-2 review items).

* No launch writes past the workspace the library asks for: the posterior's draw-split
  region (sized and bounded by ONE split function) and the per-workgroup partials of the
  lane-group kernels (grids capped at the workspace's slots) — checked with a canary
  after the region, through the C ABI.
* The non-finite count the partials kernels keep next to the fp64 sum
  equals the number of inf / NaN log-densities, on every kernel family.
* Two streams in flight with their own workspaces give the single-stream results bitwise.
* C4's per-GPU form at the full 8-GPU global batch: B = 2^27 on ONE device (t = 16 GiB,
  offsets past 2^31 elements), against the oracle on samples spread over the batch.
"""

import ctypes

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import nfn_oracle as O
from parity import check_forward

pytestmark = pytest.mark.gpu
C2 = ("planar", "radial") * 5
SENTINEL = 12345.678


def _ids(ft):
    from normalizingflownetwork_amd import ops

    return ops.flow_ids(ft)


def _canary_ws(n):
    """The workspace the library asks for (zero-initialised: the finishing ticket) followed
    by 64 sentinel doubles."""
    ws = torch.full((n + 64,), SENTINEL, dtype=torch.float64, device="cuda")
    ws[:n] = 0.0
    return ws


def _check_canary(ws, n, what):
    tail = ws[n:].cpu().numpy()
    assert (tail == SENTINEL).all(), f"{what}: workspace overrun ({int((tail != SENTINEL).sum())} doubles past the end)"


@pytest.mark.parametrize("S,B", [(16, 34817), (32, 34817), (16, 40000), (50, 34817), (3, 1000)])
def test_posterior_split_stays_in_workspace(S, B, gpu):
    """the split region was sized with 256-row tiles but launched with
    64-row ones; B = 34817 with S = 16 or 32 overran it by one range."""
    from normalizingflownetwork_amd import _lib

    lib = _lib.load()
    rng = np.random.default_rng(S * 7 + B)
    y = rng.standard_normal((B, 1)).astype(np.float32)
    t = rng.standard_normal((S, B, 32)).astype(np.float32)
    yd, td = torch.from_numpy(y).cuda(), torch.from_numpy(t).cuda()
    n = int(lib.nfn_posterior_workspace_doubles(B, 1, 32))
    ws = _canary_ws(n)
    out = torch.empty((B,), dtype=torch.float32, device="cuda")
    osum = torch.empty((2,), dtype=torch.float64, device="cuda")
    ids, k = _ids(C2)
    rc = lib.nfn_posterior_lse_f32(yd.data_ptr(), 1, td.data_ptr(), B * 32, 32, S, B, 1, ctypes.cast(ids, ctypes.c_void_p),
                                   k, 1, None, None, out.data_ptr(), osum.data_ptr(), ws.data_ptr(), None)
    _lib.check(rc, "posterior")
    torch.cuda.synchronize()
    _check_canary(ws, n, f"posterior S={S} B={B}")
    got = out.cpu().numpy()
    assert float(osum[0].item()) == pytest.approx(got.astype(np.float64).sum(), rel=1e-12)
    assert int(ws[1].item()) == 0  # the finishing ticket is left at zero
    idx = np.r_[0:64, rng.integers(0, B, 192), B - 64:B]
    r64 = O.posterior_lse(y[idx], t[:, idx], C2, 1, True)
    r32 = O.posterior_lse(y[idx], t[:, idx], C2, 1, True, dtype=np.float32)
    check_forward(got[idx], r64, r32, f"posterior split S={S} B={B}")


@pytest.mark.parametrize("d,ft", [(20, ("radial", "radial", "affine")), (24, ("radial", "radial", "affine")),
                                  (32, ("radial", "radial", "affine")), (17, ("affine", "affine", "affine")),
                                  (8, ("affine",) + ("planar",) * 4 + ("radial",) * 4)])
@pytest.mark.parametrize("B", [10000, 777])
def test_group_partials_stay_in_workspace(d, ft, B, gpu):
    """with 17 <= d <= 32 the 8-lane-group kernel's grid (B/32
    workgroups) outgrew the partial slots (B/64)."""
    from normalizingflownetwork_amd import _lib

    lib = _lib.load()
    P = O.total_param_size(ft, d, True)
    assert P % 4 == 0
    rng = np.random.default_rng(d * 1000 + B)
    y = rng.standard_normal((B, d)).astype(np.float32)
    t = (0.5 * rng.standard_normal((B, P))).astype(np.float32)
    yd, td = torch.from_numpy(y).cuda(), torch.from_numpy(t).cuda()
    n = int(lib.nfn_chain_workspace_doubles(B, d, P))
    ws = _canary_ws(n)
    out = torch.empty((B,), dtype=torch.float32, device="cuda")
    osum = torch.empty((2,), dtype=torch.float64, device="cuda")
    ids, k = _ids(ft)
    rc = lib.nfn_chain_logprob_f32(yd.data_ptr(), d, td.data_ptr(), P, B, d, ctypes.cast(ids, ctypes.c_void_p), k, 1,
                                   None, None, out.data_ptr(), osum.data_ptr(), ws.data_ptr(), None)
    _lib.check(rc, "chain")
    torch.cuda.synchronize()
    _check_canary(ws, n, f"chain d={d} B={B}")
    got = out.cpu().numpy()
    with np.errstate(all="ignore"):
        r64 = O.chain_log_prob(y, t, ft, d, True, np.float64)
        r32 = O.chain_log_prob(y, t, ft, d, True, np.float32)
    fin = np.isfinite(r64)  # an affine scale 1 + t of 0 is a legitimate -inf log-density
    check_forward(got, r64, r32, f"group partials d={d} B={B}", nonfinite="match")
    assert (~np.isfinite(got[~fin])).all()
    assert osum[1].item() == float((~np.isfinite(got)).sum())  # the non-finite count
    assert int(ws[1].item()) == 0  # the finishing ticket is left at zero
    if fin.all():
        assert float(osum[0].item()) == pytest.approx(got.astype(np.float64).sum(), rel=1e-12)


def _poison(y, rows_nan, rows_inf):
    y = y.copy()
    y[rows_nan, 0] = np.nan
    y[rows_inf, 0] = np.inf
    return y


@pytest.mark.parametrize("name", ["c2_pr5_d1", "c3_apr_d8", "asym_pra_d3", "c1_nfn_radial2_d1"])
def test_nonfinite_count_chain(name, gpu):
    from normalizingflownetwork_amd import ops

    g = load_golden(name)
    B = g["y"].shape[0]
    y = _poison(g["y"], [0, 5, B - 1], [7, B // 2])
    lp, s, nf = ops.chain_log_prob(y, g["t"], g["flow_types"], g["d"], bool(g["trainable"]), want_nonfinite=True)
    with np.errstate(all="ignore"):
        ref = O.chain_log_prob(y, g["t"], g["flow_types"], g["d"], bool(g["trainable"]), np.float64)
    n_ref = int((~np.isfinite(ref)).sum())
    assert n_ref >= 5
    assert int(nf.item()) == n_ref == int((~torch.isfinite(lp)).sum().item())
    assert not np.isfinite(s.item())  # propagates, as the reference's .mean() does
    # sum-only launch, and the pre-bound launcher's reduction
    _, _, nf2 = ops.chain_log_prob(y, g["t"], g["flow_types"], g["d"], bool(g["trainable"]), want_values=False,
                                   want_nonfinite=True)
    assert int(nf2.item()) == n_ref
    # clean input: zero
    _, _, nf0 = ops.chain_log_prob(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"]), want_nonfinite=True)
    assert int(nf0.item()) == int((~np.isfinite(g["ref64"])).sum())


def test_nonfinite_count_posterior_dense_launcher(gpu):
    from normalizingflownetwork_amd import ops

    gp = load_golden("posterior_s8_pr5_d1")
    B = gp["y"].shape[0]
    y = _poison(gp["y"], [1, 2], [3])
    out, s, nf = ops.posterior_lse(y, gp["t"], gp["flow_types"], 1, True, gp["y_mean"], gp["y_std"],
                                   want_nonfinite=True)
    assert int(nf.item()) == 3 == int((~torch.isfinite(out)).sum().item())
    # fused Dense path (chain) and fused DenseVariational path (posterior)
    rng = np.random.default_rng(3)
    H, P = 16, 32
    h = torch.from_numpy(rng.standard_normal((B, H)).astype(np.float32)).cuda()
    W = torch.from_numpy((rng.standard_normal((H, P)) / 4).astype(np.float32)).cuda()
    b = torch.zeros((P,), device="cuda")
    yd = torch.from_numpy(y).cuda()
    _, _, nfd = ops.chain_log_prob_dense(yd, h, W, b, C2, 1, True, want_nonfinite=True)
    assert int(nfd.item()) == 3
    hs = h.unsqueeze(0).expand(4, B, H).contiguous()
    _, _, nfp = ops.posterior_lse_dense(yd, hs, W.unsqueeze(0).expand(4, H, P).contiguous(),
                                        b.unsqueeze(0).expand(4, P).contiguous(), C2, 1, True, want_nonfinite=True)
    assert int(nfp.item()) == 3
    L = ops.ChainLauncher(yd, torch.from_numpy(load_golden("c2_pr5_d1")["t"][:B]).cuda(), C2, 1, True)
    L.launch()
    L.finish_sum()
    assert int(L.nonfinite.item()) == 3


def test_concurrent_streams_match_single_stream(gpu):
    """calls in flight on two streams (each with its own workspace)
    give the single-stream results bitwise."""
    from normalizingflownetwork_amd import ops

    gen = torch.Generator(device="cuda").manual_seed(9)
    B = 1 << 20
    ys = [torch.randn((B, 1), generator=gen, device="cuda") for _ in range(2)]
    ts = [torch.randn((B, 32), generator=gen, device="cuda") for _ in range(2)]
    tp = [torch.randn((16, B // 16, 32), generator=gen, device="cuda") for _ in range(2)]
    ref = [ops.chain_log_prob(ys[i], ts[i], C2, 1, True, want_sum=True) for i in range(2)]
    pref = [ops.posterior_lse(ys[i][: B // 16], tp[i], C2, 1, True, want_sum=True) for i in range(2)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got, pgot = [None, None], [None, None]
    for rep in range(3):
        for i in range(2):
            with torch.cuda.stream(streams[i]):
                got[i] = ops.chain_log_prob(ys[i], ts[i], C2, 1, True, want_sum=True)
                pgot[i] = ops.posterior_lse(ys[i][: B // 16], tp[i], C2, 1, True, want_sum=True)
        torch.cuda.synchronize()
        for i in range(2):
            assert torch.equal(got[i][0], ref[i][0]) and torch.equal(got[i][1], ref[i][1])
            assert torch.equal(pgot[i][0], pref[i][0]) and torch.equal(pgot[i][1], pref[i][1])


def test_c4_global_batch_on_one_device(gpu):
    """2^27 samples (C4's global batch) in one call (eight 2^24-sample launches): t is
    16 GiB, element offsets pass 2^31.  Samples spread over the whole batch (and the last rows) against the oracle;
    the fused sum and the non-finite count against the returned values."""
    from normalizingflownetwork_amd import ops

    B, P = 1 << 27, 32
    gen = torch.Generator(device="cuda").manual_seed(27)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((B, P), generator=gen, device="cuda")
    lp, s, nf = ops.chain_log_prob(y, t, C2, 1, True, want_nonfinite=True)
    torch.cuda.synchronize()
    fin = torch.isfinite(lp)
    assert int(nf.item()) == int((~fin).sum().item())
    if bool(fin.all()):
        assert float(s.item()) == pytest.approx(float(lp.double().sum().item()), rel=1e-12)
    idx = torch.cat([torch.randint(0, B, (3000,), generator=gen, device="cuda"),
                     torch.arange((1 << 26) - 500, (1 << 26) + 500, device="cuda"),
                     torch.arange(B - 600, B, device="cuda")])
    yn, tn = y[idx].cpu().numpy(), t[idx].cpu().numpy()
    r64 = O.chain_log_prob(yn, tn, C2, 1, True, np.float64)
    r32 = O.chain_log_prob(yn, tn, C2, 1, True, np.float32)
    check_forward(lp[idx].cpu().numpy(), r64, r32, "C4 global batch on one device, sample", nonfinite="match")
    del t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("ft,d,B", [(C2, 1, (1 << 24) + 4097), (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8,
                                                                 (1 << 24) + 999)])
def test_chunked_batch(ft, d, B, gpu):
    """A batch past 2^24 samples runs as consecutive launches over its slices (the
    static tile stride drifts over one long launch).  Values bitwise those of
    separate calls on the slices; one fused sum over every chunk's partials (the same
    bits as the partials-only call + nfn_reduce_partials_f64), the workspace not overrun,
    the ticket left at zero, the header = the total number of pairs."""
    from normalizingflownetwork_amd import _lib

    lib = _lib.load()
    P = O.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(B)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = 0.5 * torch.randn((B, P), generator=gen, device="cuda")
    ids, k = _ids(ft)
    n = int(lib.nfn_chain_workspace_doubles(B, d, P))
    ws = _canary_ws(n)
    out = torch.empty((B,), dtype=torch.float32, device="cuda")
    osum = torch.empty((2,), dtype=torch.float64, device="cuda")

    def call(yv, tv, nb, o, s, w):
        rc = lib.nfn_chain_logprob_f32(yv.data_ptr(), d, tv.data_ptr(), P, nb, d, ctypes.cast(ids, ctypes.c_void_p), k,
                                       1, None, None, o.data_ptr() if o is not None else None,
                                       s.data_ptr() if s is not None else None, w.data_ptr() if w is not None else None,
                                       None)
        _lib.check(rc, "chain")

    call(y, t, B, out, osum, ws)
    torch.cuda.synchronize()
    _check_canary(ws, n, f"chunked d={d} B={B}")
    assert int(ws[1].item()) == 0
    npairs = int(ws[0].item())
    assert 2 <= npairs <= (n - 2) // 2
    assert float(osum[0].item()) == pytest.approx(out.double().sum().item(), rel=1e-12)
    assert osum[1].item() == float((~torch.isfinite(out)).sum().item())
    # partials-only call, then the reduction: the same bits
    ws2 = torch.zeros((n,), dtype=torch.float64, device="cuda")
    call(y, t, B, None, None, ws2)
    osum2 = torch.empty((2,), dtype=torch.float64, device="cuda")
    _lib.check(lib.nfn_reduce_partials_f64(ws2.data_ptr(), osum2.data_ptr(), None), "reduce")
    torch.cuda.synchronize()
    assert int(ws2[0].item()) == npairs
    assert torch.equal(osum2, osum)
    # each slice on its own: bitwise the same values
    c = 1 << 24
    for b0 in (0, c):
        nb = min(c, B - b0)
        o = torch.empty((nb,), dtype=torch.float32, device="cuda")
        call(y[b0:], t[b0:], nb, o, None, None)
        assert torch.equal(o, out[b0:b0 + nb])
    idx = torch.cat([torch.arange(c - 300, c + 300, device="cuda"), torch.arange(B - 200, B, device="cuda"),
                     torch.randint(0, B, (1000,), generator=gen, device="cuda")])
    yn, tn = y[idx].cpu().numpy(), t[idx].cpu().numpy()
    r64 = O.chain_log_prob(yn, tn, ft, d, True, np.float64)
    r32 = O.chain_log_prob(yn, tn, ft, d, True, np.float32)
    check_forward(out[idx].cpu().numpy(), r64, r32, f"chunked d={d} B={B} sample", nonfinite="match")
    del t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", ["chain", "chain_chunked", "posterior", "dense"])
def test_uninitialised_workspace(kind, gpu):
    """ABI 200: a workspace from plain allocation — here filled with garbage,
    the finishing ticket included — gives the same fp64 sum as a zeroed one: the ticket
    carries a per-call epoch that the garbage does not (write_partial, nfn_device.h)."""
    from normalizingflownetwork_amd import _lib

    lib = _lib.load()
    gen = torch.Generator(device="cuda").manual_seed(7)
    B = {"chain": 100_000, "chain_chunked": (1 << 24) + 77, "posterior": 30_000, "dense": 50_000}[kind]
    y = torch.randn((B, 1), generator=gen, device="cuda")
    ids, k = _ids(C2)
    p_ids = ctypes.cast(ids, ctypes.c_void_p)
    res = []
    for garbage in (False, True):
        t = None
        if kind == "posterior":
            n = int(lib.nfn_posterior_workspace_doubles(B, 1, 32))
        else:
            n = int(lib.nfn_chain_workspace_doubles(B, 1, 32))
        ws = torch.zeros((n,), dtype=torch.float64, device="cuda")
        if garbage:
            ws.view(torch.int32).fill_(0x5A5A5A5A)  # a non-zero ticket (workspace[1]), garbage pairs
        osum = torch.full((2,), -1.0, dtype=torch.float64, device="cuda")
        out = torch.empty((B,), dtype=torch.float32, device="cuda")
        if kind in ("chain", "chain_chunked"):
            t = torch.randn((B, 32), generator=torch.Generator(device="cuda").manual_seed(1), device="cuda")
            rc = lib.nfn_chain_logprob_f32(y.data_ptr(), 1, t.data_ptr(), 32, B, 1, p_ids, k, 1, None, None,
                                           out.data_ptr(), osum.data_ptr(), ws.data_ptr(), None)
        elif kind == "posterior":
            S = 4
            t = torch.randn((S, B, 32), generator=torch.Generator(device="cuda").manual_seed(1), device="cuda")
            rc = lib.nfn_posterior_lse_f32(y.data_ptr(), 1, t.data_ptr(), B * 32, 32, S, B, 1, p_ids, k, 1, None,
                                           None, out.data_ptr(), osum.data_ptr(), ws.data_ptr(), None)
        else:
            H = 16
            g1 = torch.Generator(device="cuda").manual_seed(1)
            h = torch.randn((B, H), generator=g1, device="cuda")
            W = 0.3 * torch.randn((H, 32), generator=g1, device="cuda")
            rc = lib.nfn_chain_logprob_dense_f32(y.data_ptr(), 1, h.data_ptr(), H, H, W.data_ptr(), None, B, 1, p_ids,
                                                 k, 1, None, None, out.data_ptr(), osum.data_ptr(), ws.data_ptr(),
                                                 None)
        _lib.check(rc, kind)
        torch.cuda.synchronize()
        assert int(ws[1].item()) == 0, "the ticket is left at zero"
        res.append((osum.clone(), out.clone()))
        del t
    assert torch.equal(res[0][1], res[1][1])
    assert torch.equal(res[0][0], res[1][0]), (res[0][0], res[1][0])
    fin = torch.isfinite(res[0][1])
    if fin.all():
        assert float(res[0][0][0].item()) == pytest.approx(float(res[0][1].double().sum().item()), rel=1e-12)
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", ["chain", "posterior_split"])
def test_graph_replay_repeats_epoch(kind, gpu):
    """A summed call captured in a HIP graph replays with the SAME ticket epoch every time
    (write_partial, nfn_device.h): the last workgroup's clear of the ticket is what makes
    the next replay count from one.  Three replays over changing inputs (written into the
    graph's static t between replays), each sum against its own values, and the first
    against an eager call."""
    from normalizingflownetwork_amd import _lib

    lib = _lib.load()
    ids, k = _ids(C2)
    p_ids = ctypes.cast(ids, ctypes.c_void_p)
    B, S = (200_000, 1) if kind == "chain" else (30_000, 8)
    gen = torch.Generator(device="cuda").manual_seed(3)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((S, B, 32), generator=gen, device="cuda")
    n = int(lib.nfn_chain_workspace_doubles(B, 1, 32) if kind == "chain" else lib.nfn_posterior_workspace_doubles(B, 1, 32))
    ws = torch.empty((n,), dtype=torch.float64, device="cuda")
    ws.view(torch.int32).fill_(0x5A5A5A5A)
    osum = torch.empty((2,), dtype=torch.float64, device="cuda")
    out = torch.empty((B,), dtype=torch.float32, device="cuda")

    def call(stream):
        if kind == "chain":
            rc = lib.nfn_chain_logprob_f32(y.data_ptr(), 1, t.data_ptr(), 32, B, 1, p_ids, k, 1, None, None,
                                           out.data_ptr(), osum.data_ptr(), ws.data_ptr(), stream)
        else:
            rc = lib.nfn_posterior_lse_f32(y.data_ptr(), 1, t.data_ptr(), B * 32, 32, S, B, 1, p_ids, k, 1, None,
                                           None, out.data_ptr(), osum.data_ptr(), ws.data_ptr(), stream)
        _lib.check(rc, kind)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        call(ctypes.c_void_p(side.cuda_stream))  # eager, on the capture stream
    torch.cuda.synchronize()
    eager = (osum.clone(), out.clone())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        call(ctypes.c_void_p(side.cuda_stream))
    torch.cuda.synchronize()
    for r in range(3):
        if r:
            t.copy_(torch.randn((S, B, 32), generator=gen, device="cuda"))
        osum.fill_(-1.0)
        g.replay()
        torch.cuda.synchronize()
        if r == 0:
            assert torch.equal(out, eager[1]) and torch.equal(osum, eager[0])
        assert torch.isfinite(out).all()
        assert float(osum[0].item()) == pytest.approx(float(out.double().sum().item()), rel=1e-12), r
        assert float(osum[1].item()) == 0.0
        assert int(ws[1].item()) == 0, "the ticket is left at zero"


def test_graph_workspace_survives_cache_eviction(gpu):
    """ops._workspace hands a stream its cached workspace; an entry used while the stream
    captures a graph is pinned, so pushing more than WORKSPACE_CACHE_ENTRIES other streams
    through the cache (which evicts its least recently used entries) cannot return the
    graph's workspace to the allocator: replays after the eviction still sum correctly
    while other tensors are allocated and written on the capture stream's pool."""
    from normalizingflownetwork_amd import ops

    ft, d, B = ("planar", "radial") * 5, 1, 100_000
    gen = torch.Generator(device="cuda").manual_seed(21)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((B, 32), generator=gen, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        _, s_eager = ops.chain_log_prob(y, t, ft, d, True, want_values=False, want_sum=True)  # warm-up
    torch.cuda.synchronize()
    ref = float(s_eager[0].item())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        _, s_graph = ops.chain_log_prob(y, t, ft, d, True, want_values=False, want_sum=True)
    (key,) = [k for k in ops._workspaces if k[1] == int(side.cuda_stream)]
    ws = ops._workspaces[key]
    assert any(p is ws for _, _, p in ops._graph_workspaces)
    streams = [torch.cuda.Stream() for _ in range(ops.WORKSPACE_CACHE_ENTRIES + 2)]
    for st in streams:
        with torch.cuda.stream(st):
            ops.chain_log_prob(y[:1000], t[:1000], ft, d, True, want_values=False, want_sum=True)
    torch.cuda.synchronize()
    assert key not in ops._workspaces  # evicted from the cache, still alive for the graph
    with torch.cuda.stream(side):
        junk = [torch.full((ws.numel(),), 7.0, dtype=torch.float64, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert float(s_graph[0].item()) == pytest.approx(ref, rel=1e-12)
    assert all(float(j[0].item()) == 7.0 for j in junk)


def test_taken_graph_workspaces_are_unpinned(gpu):
    """A capturing caller that takes over its pinned workspaces (``ops.take_graph_workspaces``,
    as ``fit`` keeps them next to its graph) leaves nothing pinned for that stream: repeated
    captures on fresh streams do not grow the process-wide pin list."""
    from normalizingflownetwork_amd import ops

    ft, d, B = ("planar", "radial") * 5, 1, 10_000
    y = torch.randn((B, 1), device="cuda")
    t = torch.randn((B, 32), device="cuda")
    n0 = len(ops._graph_workspaces)
    kept = []
    for _ in range(3):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ops.chain_log_prob(y, t, ft, d, True, want_values=False, want_sum=True)
        g = torch.cuda.CUDAGraph()
        mark = ops.graph_pin_mark()
        with torch.cuda.graph(g, stream=side):
            _, s_graph = ops.chain_log_prob(y, t, ft, d, True, want_values=False, want_sum=True)
        mine = ops.take_graph_workspaces(side, mark)
        assert len(mine) == 1
        kept.append((g, s_graph, mine))
        assert len(ops._graph_workspaces) == n0
    for g, s_graph, _ in kept:
        g.replay()
    torch.cuda.synchronize()
    ref = float(ops.chain_log_prob(y, t, ft, d, True, want_values=False, want_sum=True)[1][0].item())
    for _, s_graph, _ in kept:
        assert float(s_graph[0].item()) == pytest.approx(ref, rel=1e-12)


def test_take_leaves_another_graphs_pin_on_the_same_stream(gpu):
    """Two graphs captured on ONE stream handle (torch pools and reuses stream handles):
    the first is left pinned process-wide, the second is captured between a pin mark and a
    take.  The take hands back only what the second capture pinned (here a larger block,
    since it outgrew the first's), the first graph's block stays pinned, and both graphs
    still replay correctly after the cache has evicted the stream's entry."""
    from normalizingflownetwork_amd import ops

    ft, d = ("planar", "radial") * 5, 1
    gen = torch.Generator(device="cuda").manual_seed(5)
    y = torch.randn((1 << 20, 1), generator=gen, device="cuda")
    t = torch.randn((1 << 20, 32), generator=gen, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graphs = []
    for B in (10_000, 1 << 20):  # the second needs more partials: a new, larger workspace
        with torch.cuda.stream(side):
            ops.chain_log_prob(y[:B], t[:B], ft, d, True, want_values=False, want_sum=True)
        g = torch.cuda.CUDAGraph()
        mark = ops.graph_pin_mark()
        with torch.cuda.graph(g, stream=side):
            _, s_graph = ops.chain_log_prob(y[:B], t[:B], ft, d, True, want_values=False, want_sum=True)
        key = (side.device.index, int(side.cuda_stream))
        graphs.append((B, g, s_graph, ops._workspaces[key], mark))
    (_, _, _, ws_a, _), (_, _, _, ws_b, mark_b) = graphs
    assert ws_a is not ws_b
    mine = ops.take_graph_workspaces(side, mark_b)
    assert len(mine) == 1 and mine[0] is ws_b
    assert any(p is ws_a for _, _, p in ops._graph_workspaces), "the first graph's block was unpinned"
    for st in [torch.cuda.Stream() for _ in range(ops.WORKSPACE_CACHE_ENTRIES + 2)]:
        with torch.cuda.stream(st):
            ops.chain_log_prob(y[:1000], t[:1000], ft, d, True, want_values=False, want_sum=True)
    torch.cuda.synchronize()
    for B, g, s_graph, _, _ in graphs:
        g.replay()
        torch.cuda.synchronize()
        ref = float(ops.chain_log_prob(y[:B], t[:B], ft, d, True, want_values=False, want_sum=True)[1][0].item())
        assert float(s_graph[0].item()) == pytest.approx(ref, rel=1e-12)
