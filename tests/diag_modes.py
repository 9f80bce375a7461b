"""Subprocess body of tests/test_gpu_diag.py (one process, one GPU context).

  python tests/diag_modes.py strategies   -- NFN_DIAG build: every tile-streaming strategy
      (NFN_LOAD_MODE) gives bitwise-identical per-sample log_prob, and the draw-split
      posterior agrees with the single-range one (NFN_POST_SPLIT=1)
  python tests/diag_modes.py grad_stream  -- NFN_DIAG build: the d = 1 straight-line
      backward (NFN_GRAD_WAVE1=1) equals the release's generic wave kernel bitwise
  python tests/diag_modes.py flow_tile    -- NFN_DIAG build: the LDS-staged per-flow kernel (d > 1)
      equals the per-lane global-read one bitwise (NFN_FLOW_VARIANT=0)
  python tests/diag_modes.py densep       -- NFN_DIAG build: the prefetching d >= 2 posterior Dense
      kernel equals the synchronous one bitwise (NFN_DENSEP=0)
  python tests/diag_modes.py release      -- release build under ablation / tuning knobs in
      the environment: results are the oracle's (the knobs are compiled out)
Prints one JSON line; exits non-zero on a mismatch."""

import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import load_golden  # noqa: E402
from oracle import nfn_oracle as O  # noqa: E402  (checker)


def strategies():
    import torch

    from normalizingflownetwork_amd import _lib

    _lib.use_diagnostic_build()
    from normalizingflownetwork_amd import ops

    g = load_golden("stress_pr5_d1")
    gp = load_golden("posterior_s8_pr5_d1")
    ref, _ = ops.chain_log_prob(g["y"], g["t"], g["flow_types"], 1, True)
    pref, _ = ops.posterior_lse(gp["y"], gp["t"], gp["flow_types"], 1, True, gp["y_mean"], gp["y_std"])
    res = {}
    for mode in ("coop", "wave", "ownrow", "tile"):
        os.environ["NFN_LOAD_MODE"] = mode
        try:
            got, s = ops.chain_log_prob(g["y"], g["t"], g["flow_types"], 1, True, want_sum=True)
            pgot, _ = ops.posterior_lse(gp["y"], gp["t"], gp["flow_types"], 1, True, gp["y_mean"], gp["y_std"])
        finally:
            os.environ.pop("NFN_LOAD_MODE")
        assert torch.equal(got, ref), mode
        assert abs(float(s.item()) - float(got.double().sum().item())) <= 1e-12 * abs(float(s.item())), mode
        np.testing.assert_allclose(pgot.cpu().numpy(), pref.cpu().numpy(), rtol=2e-6, atol=2e-6)
        res[mode] = "bitwise"
    # C5 shape: draw split (default) vs one range
    ft = ("planar", "radial") * 5
    S, B = 64, 1 << 17
    gen = torch.Generator(device="cuda").manual_seed(5)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((S, B, 32), generator=gen, device="cuda")
    out, _ = ops.posterior_lse(y, t, ft, 1, True)
    os.environ["NFN_POST_SPLIT"] = "1"
    try:
        out1, _ = ops.posterior_lse(y, t, ft, 1, True)
    finally:
        os.environ.pop("NFN_POST_SPLIT")
    np.testing.assert_allclose(out.cpu().numpy(), out1.cpu().numpy(), rtol=2e-6, atol=2e-6)
    res["post_split_vs_single"] = "allclose 2e-6"
    # C2 shape on chain_wave1_kernel (ragged tail): the plain tile walk (diag NFN_TILE_ROT=0)
    # gives the rotated walk's per-sample values bitwise (the same math on the same rows) and
    # the same fixed-order fp64 sum
    B2 = (1 << 20) + 37
    y2 = torch.randn((B2, 1), generator=gen, device="cuda")
    t2 = torch.randn((B2, 32), generator=gen, device="cuda")
    base, s2 = ops.chain_log_prob(y2, t2, ft, 1, True, want_sum=True)
    os.environ["NFN_TILE_ROT"] = "0"
    try:
        got, g2 = ops.chain_log_prob(y2, t2, ft, 1, True, want_sum=True)
    finally:
        os.environ.pop("NFN_TILE_ROT")
    assert torch.equal(got, base), "NFN_TILE_ROT=0"
    assert abs(float(g2.item()) - float(s2.item())) <= 1e-12 * abs(float(s2.item()))
    res["nfn_tile_rot_0"] = "bitwise"
    res["library"] = os.path.basename(_lib.LIB_PATH)
    return res


def grad_stream():
    """d = 1 backward: the straight-line buffer pipeline (chain_grad_wave1_kernel, diag
    NFN_GRAD_WAVE1=1, in one or two prefetch pieces) and the producer / consumer workgroup
    (chain_grad_pc_kernel, NFN_GRAD_PC=1) against the release's wave kernel
    (chain_grad_wave_kernel): the same per-sample math, so log_prob, d/dt and d/dy must be
    bitwise equal (NaN where both are)."""
    import torch

    from normalizingflownetwork_amd import _lib

    _lib.use_diagnostic_build()
    from normalizingflownetwork_amd import ops

    res = {"library": os.path.basename(_lib.LIB_PATH)}
    cases = [(("planar", "radial") * 5, 1 << 20, None), (("planar", "radial") * 5, 4099, (0.3, 1.6)),
             (("radial", "radial"), 777, None), (("planar", "radial", "planar", "radial", "affine"), 5000, None)]
    for ft, B, norm in cases:
        P = ops.total_param_size(ft, 1, True)
        gen = torch.Generator(device="cuda").manual_seed(B)
        y = torch.randn((B, 1), generator=gen, device="cuda")
        t = torch.randn((B, P), generator=gen, device="cuda")
        g = torch.randn((B,), generator=gen, device="cuda")
        ym, ys = (np.float32([norm[0]]), np.float32([norm[1]])) if norm else (None, None)
        outs = {}
        for v, split, pc, rot in (("0", "1", "0", "0"), ("1", "1", "0", "0"), ("1", "2", "0", "0"),
                                  ("0", "1", "1", "0"), ("0", "1", "0", "4")):
            os.environ["NFN_GRAD_WAVE1"], os.environ["NFN_GRAD_SPLIT"], os.environ["NFN_GRAD_PC"] = v, split, pc
            os.environ["NFN_TILE_ROT_B"] = rot
            try:
                outs[v + split + pc + rot] = ops.chain_log_prob_grad(y, t, ft, 1, True, ym, ys, g_out=g, want_logp=True)
            finally:
                for k in ("NFN_GRAD_WAVE1", "NFN_GRAD_SPLIT", "NFN_GRAD_PC", "NFN_TILE_ROT_B"):
                    os.environ.pop(k)
        outs["01"] = outs["0100"]
        for alt in ("1100", "1200", "0110", "0104"):
            for a, b, what in zip(outs[alt], outs["01"], ("log_prob", "grad_t", "grad_y")):
                same = (a == b) | (torch.isnan(a) & torch.isnan(b))
                assert bool(same.all()), f"{ft} B={B} {alt} {what}: {int((~same).sum())} values differ"
        res[f"P{P}_B{B}"] = "bitwise"
    return res


def densep():
    """Posterior with the output DenseVariational layer fused, d >= 2, fast math: the
    prefetching pipeline (posterior_densep_kernel, default) against the synchronous kernel
    (posterior_dense_kernel, NFN_DENSEP=0) — the same MFMA accumulation order, chain and
    logsumexp, so the scores must be bitwise equal; per-draw and shared h, y normalisation,
    no bias, ragged batches."""
    import torch

    from normalizingflownetwork_amd import _lib

    _lib.use_diagnostic_build()
    from normalizingflownetwork_amd import ops

    res = {"library": os.path.basename(_lib.LIB_PATH)}
    c3 = ("affine",) + ("planar",) * 4 + ("radial",) * 4
    cases = [(c3, 3, 16, 4099, 5, False, True, False), (("radial", "planar"), 2, 4, 65, 3, True, True, True),
             (("planar", "radial", "affine"), 8, 8, 300, 2, False, False, True), (c3, 3, 16, 1, 64, True, True, False)]
    for ft, d, H, B, S, shared, bias, normed in cases:
        P = ops.total_param_size(ft, d, True)
        gen = torch.Generator(device="cuda").manual_seed(B + d)
        y = torch.randn((B, d), generator=gen, device="cuda")
        h = torch.randn((B, H) if shared else (S, B, H), generator=gen, device="cuda")
        W = torch.randn((S, H, P), generator=gen, device="cuda") / float(np.sqrt(H))
        b = 0.1 * torch.randn((S, P), generator=gen, device="cuda") if bias else None
        ym, ys = (np.full(d, 0.3, np.float32), np.full(d, 1.7, np.float32)) if normed else (None, None)
        outs = []
        for v in ("1", "0"):
            os.environ["NFN_DENSEP"] = v
            try:
                outs.append(ops.posterior_lse_dense(y, h, W, b, ft, d, True, ym, ys, want_sum=True))
            finally:
                os.environ.pop("NFN_DENSEP")
        (o1, s1), (o0, s0) = outs
        same = (o1 == o0) | (torch.isnan(o1) & torch.isnan(o0))
        assert bool(same.all()), f"d={d} H={H} B={B} S={S}: {int((~same).sum())} scores differ"
        assert torch.equal(s1, s0), f"d={d} H={H} B={B} S={S}: sums differ"
        res[f"d{d}_H{H}_B{B}_S{S}"] = "bitwise"
    return res


def flow_tile():
    """Per-flow bijector at d > 1: the LDS-staged kernel (default) against the per-lane
    global-read kernel (NFN_FLOW_VARIANT=0) — the same flow_step on the same values, so z
    and log|det J| must be bitwise equal; ragged batches, strided / broadcast rows."""
    import torch

    from normalizingflownetwork_amd import _lib

    _lib.use_diagnostic_build()
    from normalizingflownetwork_amd import ops

    res = {"library": os.path.basename(_lib.LIB_PATH)}
    n = 0
    for d in (2, 3, 8, 16):
        for ft in ("planar", "radial", "affine"):
            ps = ops.param_size(ft, d)
            for B, bz, bt in ((777, False, False), (256, False, False), (1000, True, False), (300, False, True)):
                gen = torch.Generator(device="cuda").manual_seed(B + d)
                wide = torch.randn((B, ps + 5), generator=gen, device="cuda")
                tk = wide[:1, 2:2 + ps] if bt else wide[:, 2:2 + ps]
                z = torch.randn((1 if bz else B, d), generator=gen, device="cuda")
                outs = []
                for v in ("1", "0"):
                    os.environ["NFN_FLOW_VARIANT"] = v
                    try:
                        outs.append(ops.flow_forward_ldj(ft, z, tk, d))
                    finally:
                        os.environ.pop("NFN_FLOW_VARIANT")
                (z1, l1), (z0, l0) = outs
                for a, b, what in ((z1, z0, "z"), (l1, l0, "ldj")):
                    same = (a == b) | (torch.isnan(a) & torch.isnan(b))
                    assert bool(same.all()), f"{ft} d={d} B={B} bz={bz} bt={bt} {what}: {int((~same).sum())} differ"
                n += 1
    res["cases"] = n
    return res


def dense_cache():
    """The fused Dense backward's parameter-scalar cache for C2's compile-time program.  The
    exact cache (diag NFN_CHAIN_FORM=5: the reverse pass takes the scalars the forward formed
    with the same expressions) against the uncached program (diag NFN_CHAIN_FORM=2,
    grad1_static): log_prob, dh, dW, db and dy bitwise equal.  The release form (=4, which also
    shares planar tanh / tanh' between the passes, tanh(s) from the e^{-2|s|} form for
    |s| >= 0.3): log_prob within 1e-5 of the uncached program's on the well-conditioned entries,
    and the gradients' relative differences recorded (test_gpu_dense gates them on the oracle);
    the pair form of the runtime program (=3) within 1e-5 likewise."""
    import torch

    from normalizingflownetwork_amd import _lib

    _lib.use_diagnostic_build()
    from normalizingflownetwork_amd import ops

    res = {"library": os.path.basename(_lib.LIB_PATH)}
    ft = ("planar", "radial") * 5
    names = ("log_prob", "dh", "dW", "db", "dy")
    for B in (64 * 37 + 5, 1 << 16):
        gen = torch.Generator(device="cuda").manual_seed(B)
        y = torch.randn((B, 1), generator=gen, device="cuda")
        h = torch.randn((B, 16), generator=gen, device="cuda")
        W = torch.randn((16, 32), generator=gen, device="cuda") / 4.0
        b = 0.1 * torch.randn((32,), generator=gen, device="cuda")
        g = torch.randn((B,), generator=gen, device="cuda")
        outs = {}
        for cm in ("3", "2", "4", "5"):
            os.environ["NFN_CHAIN_FORM"] = cm
            try:
                outs[cm] = ops.chain_log_prob_dense_grad(y, h, W, b, ft, 1, True, g_out=g, want_logp=True)
            finally:
                os.environ.pop("NFN_CHAIN_FORM")
        for x2, x5, what in zip(outs["2"], outs["5"], names):
            same = (x2 == x5) | (torch.isnan(x2) & torch.isnan(x5))
            assert bool(same.all()), f"B={B} {what}: {int((~same).sum())} values differ (exact cache vs static)"
        lp2 = outs["2"][0]
        ok = torch.isfinite(lp2) & (lp2.abs() < 1e4)
        for cm in ("3", "4"):
            assert torch.allclose(outs[cm][0][ok], lp2[ok], rtol=1e-5, atol=1e-5), f"B={B}: form {cm} vs static log_prob"
        rel = {}
        for x2, x4, what in zip(outs["2"], outs["4"], names):
            fin = torch.isfinite(x2) & torch.isfinite(x4)
            r = ((x4 - x2).abs() / x2.abs().clamp_min(1.0))[fin].double()
            rel[what] = {"max": float(r.max()), "p999": float(torch.quantile(r[:1 << 20], 0.999)),
                         "n_beyond_1e-5": int((r > 1e-5).sum()), "n": int(r.numel())}
        res[f"B{B}"] = {"exact_cache": "bitwise", "shared_vs_static": rel}
        # the estimator's default program, radial x 10 (no planar flow: the release form is the
        # exact cache), against the runtime program's pair form
        W10 = torch.randn((16, 32), generator=gen, device="cuda") / 4.0
        outs = {}
        for cm in ("3", "4", "5"):
            os.environ["NFN_CHAIN_FORM"] = cm
            try:
                outs[cm] = ops.chain_log_prob_dense_grad(y, h, W10, b, ("radial",) * 10, 1, True, g_out=g,
                                                         want_logp=True)
            finally:
                os.environ.pop("NFN_CHAIN_FORM")
        for x4, x5, what in zip(outs["4"], outs["5"], names):
            same = (x4 == x5) | (torch.isnan(x4) & torch.isnan(x5))
            assert bool(same.all()), f"radial x 10 B={B} {what}: {int((~same).sum())} values differ (release vs exact)"
        lp3, lp4 = outs["3"][0], outs["4"][0]
        ok = torch.isfinite(lp3) & (lp3.abs() < 1e4)
        assert torch.allclose(lp4[ok], lp3[ok], rtol=1e-5, atol=1e-5), f"radial x 10 B={B}: cache vs pairs log_prob"
        res[f"R10_B{B}"] = "bitwise"
    return res


def tanh():
    """tanh_fast (the planar flows' tanh in every fast-math kernel) on the device against fp64
    over a dense sweep of [-1, 1] (where the two branches meet, at |a| = 0.3) and a coarser one
    of [-12, 12]: the largest error in fp32 ulps of the correctly rounded result.  The bound
    is pinned by test_gpu_diag, so a change cannot loosen it silently."""
    import ctypes

    import torch

    from normalizingflownetwork_amd import build

    lib = ctypes.CDLL(build.DIAG_OUT)
    fn = lib.nfn_diag_tanh_fast
    fn.restype, fn.argtypes = ctypes.c_int32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    res = {"library": os.path.basename(build.DIAG_OUT)}
    for name, lo, hi, n in (("sweep_1", -1.0, 1.0, 1 << 22), ("sweep_12", -12.0, 12.0, 1 << 22)):
        x = np.linspace(lo, hi, n, dtype=np.float32)
        x = x[x != 0.0]
        xd = torch.from_numpy(x).cuda()
        yd = torch.empty_like(xd)
        assert fn(xd.data_ptr(), yd.data_ptr(), xd.numel(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        got = yd.cpu().numpy()
        ref = np.tanh(x.astype(np.float64))
        ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
        err = np.abs(got.astype(np.float64) - ref) / ulp
        k = int(np.argmax(err))
        res[name] = {"max_ulp": float(err.max()), "at": float(x[k]), "mean_ulp": float(err.mean())}
    return res


def release():
    from normalizingflownetwork_amd import _lib, ops

    knobs = {k: v for k, v in os.environ.items() if k.startswith("NFN_")}
    assert knobs.get("NFN_ABLATE_FLOWS") == "1", "run with the knobs set"
    res = {"library": os.path.basename(_lib.LIB_PATH), "knobs": knobs}
    from parity import check_forward, fp32_sensitivity

    for name in ("c2_pr5_d1", "c3_apr_d8", "stress_pr5_d1"):
        g = load_golden(name)
        lp, _ = ops.chain_log_prob(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"]))
        # the suite's forward gate (tests/parity.py), as in test_gpu_parity's fixture checks
        check_forward(lp.cpu().numpy(), g["ref64"], g["ref32"], f"{name} under the knobs",
                      sensitivity=fp32_sensitivity(g["y"], g["t"], g["flow_types"], g["d"], bool(g["trainable"])))
        res[name] = "oracle parity"
    gp = load_golden("posterior_s8_pr5_d1")
    out, _ = ops.posterior_lse(gp["y"], gp["t"], gp["flow_types"], 1, True, gp["y_mean"], gp["y_std"])
    ok = np.abs(out.cpu().numpy() - gp["ref64"]) <= O.tolerance_bound(gp["ref64"], gp["ref32"])
    assert ok.all()
    res["posterior"] = "oracle parity"
    return res


if __name__ == "__main__":
    which = sys.argv[1]
    print(json.dumps({which: {"strategies": strategies, "release": release, "grad_stream": grad_stream, "flow_tile": flow_tile,
                             "densep": densep, "tanh": tanh, "dense_cache": dense_cache}[which]()}), flush=True)
