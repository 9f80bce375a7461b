#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (cdna guide §5.4 rule 24).

Variants are selected through the library's tuning environment variables
(NFN_LOAD_MODE, NFN_WG_PER_CU) and the math mode; each round times every variant
back to back with HIP events on the launch stream.  Outputs are also checked
against the first variant (max |diff|)."""

import json
import time
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflownetwork_amd import _lib, ops  # noqa: E402

_lib.use_diagnostic_build()  # the NFN_* tuning / ablation knobs live only in the NFN_DIAG build

CFG = {
    "C2": (("planar", "radial") * 5, 1, 1 << 24, None),
    "C3": (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8, 1 << 22, None),
    "C5": (("planar", "radial") * 5, 1, 1 << 17, 64),
    "R2": (("radial", "radial"), 1, 1 << 24, None),
    "K4": (("planar", "radial") * 2, 1, 1 << 24, None),
    "K6": (("planar", "radial") * 3, 1, 1 << 24, None),
    "K8": (("planar", "radial") * 4, 1, 1 << 24, None),
    "R10": (("radial",) * 10, 1, 1 << 24, None),
}


def bytes_per_launch(d, P, B, S):
    return B * (4 * d + 4 * P + 4) if S is None else B * (S * 4 * P + 4 * d + 4)


def maxdiff(x, ref):
    """max |x - ref| where the two differ; equal values (incl. equal infinities) and NaN in
    both count as 0, a NaN in only one of them as inf."""
    same = (x == ref) | (torch.isnan(x) & torch.isnan(ref))
    d = torch.where(same, torch.zeros_like(x), (x - ref).abs())
    return float(d.nan_to_num(nan=float("inf")).max().item())


def prewarm(fn, ms=400.0):
    """Untimed launches for >= `ms` of device time (the clocks ramp over the first tens of ms)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    for _ in range(int(ms / max(e0.elapsed_time(e1), 1e-3)) + 1):
        fn()
    torch.cuda.synchronize()


def run(cfg, variants, reps=20, rounds=3):
    ft, d, B, S = CFG[cfg]
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = torch.randn((B, P) if S is None else (S, B, P), generator=gen, device="cuda")
    L = ops.ChainLauncher(y, t, ft, d, True, draws=S)
    L_noout = ops.ChainLauncher(y, t, ft, d, True, write_values=False, draws=S)
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    prewarm(lambda: L.launch(sh))
    times = {v["name"]: [] for v in variants}
    outs = {}
    for r in range(rounds):
        for v in variants:
            for k, val in v.get("env", {}).items():
                os.environ[k] = str(val)
            ops.set_math_mode(v.get("math", "fast"))
            LL = L_noout if v.get("noout") else L
            for _ in range(3):
                LL.launch(sh)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                LL.launch(sh)
                e1.record(stream)
            torch.cuda.synchronize()
            times[v["name"]].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
            if r == 0:
                outs[v["name"]] = L.out.clone()
            for k in v.get("env", {}):
                os.environ.pop(k, None)
    ref = outs[variants[0]["name"]]
    if variants[0].get("noout"):
        raise SystemExit("first variant must write outputs")
    res = []
    bpl = bytes_per_launch(d, P, B, S)
    for v in variants:
        ms = float(np.median(times[v["name"]]))
        diff = maxdiff(outs[v["name"]], ref)
        res.append({"cfg": cfg, "variant": v["name"], "ms": ms, "GBps": bpl / ms / 1e6, "frac8TBs": bpl / ms / 1e6 / 8000,
                    "evals_per_s": B * (S or 1) / ms * 1e3, "maxdiff_vs_first": diff, "rounds_ms": times[v["name"]]})
        print(json.dumps(res[-1]), flush=True)
    return res


def run_grad(cfg, variants, reps=10, rounds=3):
    """Fused backward variants (GradLauncher), same interleaving."""
    ft, d, B, S = CFG[cfg]
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = torch.randn((B, P), generator=gen, device="cuda")
    g = torch.full((B,), -1.0 / B, device="cuda")
    L = ops.GradLauncher(y, t, ft, d, True, g_out=g)
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    prewarm(lambda: L.launch(sh))
    times = {v["name"]: [] for v in variants}
    outs = {}
    for r in range(rounds):
        for v in variants:
            for k, val in v.get("env", {}).items():
                os.environ[k] = str(val)
            ops.set_math_mode(v.get("math", "fast"))
            for _ in range(2):
                L.launch(sh)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                L.launch(sh)
                e1.record(stream)
            torch.cuda.synchronize()
            times[v["name"]].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
            if r == 0:
                outs[v["name"]] = L.grad_t.clone()
            for k in v.get("env", {}):
                os.environ.pop(k, None)
    ref = outs[variants[0]["name"]]
    bpl = B * (8 * d + 8 * P + 4)
    for v in variants:
        ms = float(np.median(times[v["name"]]))
        diff = maxdiff(outs[v["name"]], ref)
        print(json.dumps({"cfg": cfg, "mode": "grad", "variant": v["name"], "ms": ms, "GBps": bpl / ms / 1e6,
                          "frac8TBs": bpl / ms / 1e6 / 8000, "maxdiff_vs_first": diff,
                          "rounds_ms": times[v["name"]]}), flush=True)


def run_dense(variants, H=16, reps=20, rounds=3):
    """Fused Dense -> chain (C2 flows, d = 1) variants, same interleaving."""
    ft, d, B, _ = CFG["C2"]
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    h = torch.randn((B, H), generator=gen, device="cuda")
    W = torch.randn((H, P), generator=gen, device="cuda") / float(np.sqrt(H))
    b = 0.1 * torch.randn((P,), generator=gen, device="cuda")
    L = ops.DenseLauncher(y, h, W, b, ft, d, True)
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    prewarm(lambda: L.launch(sh))
    times = {v["name"]: [] for v in variants}
    outs = {}
    for r in range(rounds):
        for v in variants:
            for k, val in v.get("env", {}).items():
                os.environ[k] = str(val)
            for _ in range(3):
                L.launch(sh)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                L.launch(sh)
                e1.record(stream)
            torch.cuda.synchronize()
            times[v["name"]].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
            if r == 0:
                outs[v["name"]] = L.out.clone()
            for k in v.get("env", {}):
                os.environ.pop(k, None)
    ref = outs[variants[0]["name"]]
    for v in variants:
        ms = float(np.median(times[v["name"]]))
        print(json.dumps({"cfg": "C2", "mode": "dense", "H": H, "variant": v["name"], "ms": ms,
                          "evals_per_s": B / ms * 1e3,
                          "maxdiff_vs_first": float((outs[v["name"]] - ref).abs().max().item()),
                          "rounds_ms": times[v["name"]]}), flush=True)


def run_posterior_dense(H=16, S=64, B=1 << 17, reps=20, rounds=3, ft=("planar", "radial") * 5, d=1, cfg="C5"):
    """C5 per-GPU shape (or another flow stack / d) with the output DenseVariational layer:
    fused posterior (t_s formed on chip) vs the unfused path (library GEMM writes t, then
    the posterior kernel) vs the posterior kernel alone on a resident t; for d >= 2 also the
    fused form on the synchronous kernel (NFN_DENSEP=0)."""
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    h = torch.randn((S, B, H), generator=gen, device="cuda")
    W = torch.randn((S, H, P), generator=gen, device="cuda") / float(np.sqrt(H))
    b = 0.1 * torch.randn((S, P), generator=gen, device="cuda")
    t = torch.matmul(h, W) + b[:, None]
    fns = {
        "fused": lambda: ops.posterior_lse_dense(y, h, W, b, ft, d, True),
        "unfused_gemm_plus_posterior": lambda: ops.posterior_lse(y, torch.matmul(h, W) + b[:, None], ft, d, True),
        "posterior_on_resident_t": lambda: ops.posterior_lse(y, t, ft, d, True),
    }

    def loopform():
        os.environ["NFN_CHAIN_FORM"] = "0"
        r_ = ops.posterior_lse_dense(y, h, W, b, ft, d, True)
        del os.environ["NFN_CHAIN_FORM"]
        return r_

    def hpair():
        os.environ["NFN_CHAIN_FORM"] = "8"
        r_ = ops.posterior_lse_dense(y, h, W, b, ft, d, True)
        del os.environ["NFN_CHAIN_FORM"]
        return r_

    if d == 1:
        fns["fused_loopform"] = loopform
        fns["fused_hpair"] = hpair
    else:
        def sync_kernel():
            os.environ["NFN_DENSEP"] = "0"
            r_ = ops.posterior_lse_dense(y, h, W, b, ft, d, True)
            del os.environ["NFN_DENSEP"]
            return r_

        fns["fused_synchronous_kernel"] = sync_kernel
    stream = torch.cuda.current_stream()
    prewarm(fns["fused"])
    times = {k: [] for k in fns}
    outs = {}
    for r in range(rounds):
        for k, fn in fns.items():
            for _ in range(3):
                fn()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                fn()
                e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
            if r == 0:
                outs[k] = fn()[0].clone()
    ref = outs["unfused_gemm_plus_posterior"]
    for k in fns:
        ms = float(np.median(times[k]))
        print(json.dumps({"cfg": cfg, "mode": "posterior_dense", "H": H, "S": S, "B": B, "variant": k, "ms": ms,
                          "pairs_per_s": S * B / ms * 1e3,
                          "maxdiff_vs_unfused": float((outs[k] - ref).abs().max().item()),
                          "rounds_ms": times[k]}), flush=True)


def run_dense_grad(H=16, B=1 << 24, reps=20, rounds=3, static=False, gemm_ceiling=False, forms=None):
    """C2 training step through the output Dense layer: the fused backward (t never
    written) vs the unfused path (library GEMM t, chain backward kernel, GEMMs for
    dh / dW and the db sum) vs the chain backward alone on a resident t."""
    ft, d = ("planar", "radial") * 5, 1
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(1)
    y = torch.randn((B, d), generator=gen, device="cuda")
    h = torch.randn((B, H), generator=gen, device="cuda")
    W = torch.randn((H, P), generator=gen, device="cuda") / float(np.sqrt(H))
    b = 0.1 * torch.randn((P,), generator=gen, device="cuda")
    g = torch.full((B,), -1.0 / B, device="cuda")
    t = torch.addmm(b, h, W)

    def unfused():
        tt = torch.addmm(b, h, W)
        _, gt, gy = ops.chain_log_prob_grad(y, tt, ft, d, True, g_out=g)
        return gt @ W.t(), h.t() @ gt, gt.sum(0), gy

    fused = lambda: ops.chain_log_prob_dense_grad(y, h, W, b, ft, d, True, g_out=g)
    fns = {
        "fused": fused,
        "fused_generic": fused,
        "fused_gemms_only": fused,
        "fused_loopform": fused,
        "unfused": unfused,
        "chain_backward_on_resident_t": lambda: ops.chain_log_prob_grad(y, t, ft, d, True, g_out=g),
    }
    envs = {"fused_generic": {"NFN_DENSE1_GRAD": "0"}, "fused_gemms_only": {"NFN_ABLATE_FLOWS": "1"},
            "fused_loopform": {"NFN_CHAIN_FORM": "0"}}
    if static:
        fns = {"fused": fused, "fused_static": fused, "fused_loopform": fused}
        envs["fused_static"] = {"NFN_CHAIN_FORM": "2"}
    if forms:  # {name: NFN_CHAIN_FORM}; "_regs" names also set NFN_HPAIR_U=2
        fns = {"fused": fused, **{k: fused for k in forms}, "fused_b": fused}
        envs.update({k: {"NFN_CHAIN_FORM": str(v), **({"NFN_HPAIR_U": "2"} if k.endswith("_regs") else {})}
                     for k, v in forms.items()})
    if gemm_ceiling:  # dh / dW MFMAs replaced by VALU touches of the same operands (NFN_DGRAD_ABLATE)
        fns = {"fused": fused, "no_dh_mfma": fused, "no_dW_mfma": fused, "no_dh_dW_mfma": fused,
               "fused_gemms_only": fused}
        envs.update({"no_dh_mfma": {"NFN_DGRAD_ABLATE": "1"}, "no_dW_mfma": {"NFN_DGRAD_ABLATE": "2"},
                     "no_dh_dW_mfma": {"NFN_DGRAD_ABLATE": "3"}})
    os.environ["NFN_CHAIN_FORM"] = "0"
    loop_out = [x for x in fused()]
    del os.environ["NFN_CHAIN_FORM"]
    for name, a_, b_ in zip(("lp", "dh", "dW", "db", "dy"), [x for x in fused()], loop_out):
        if a_ is None:
            continue
        print(json.dumps({"check": "pairs vs loop chain form", "what": name,
                          "max_abs": float((a_ - b_).abs().max().item())}), flush=True)
    for k in (forms or {}):
        os.environ.update(envs[k])
        alt = [x for x in fused()]
        for e in envs[k]:
            del os.environ[e]
        for name, a_, b_ in zip(("lp", "dh", "dW", "db", "dy"), alt, [x for x in fused()]):
            if a_ is not None:
                print(json.dumps({"check": f"{k} vs release", "what": name,
                                  "max_abs": float((a_ - b_).abs().max().item())}), flush=True)
    ref = [x for x in fused()[1:]]
    os.environ["NFN_DENSE1_GRAD"] = "0"
    gen_out = [x for x in fused()[1:]]
    del os.environ["NFN_DENSE1_GRAD"]
    for name, a_, b_ in zip(("dh", "dW", "db", "dy"), ref, gen_out):
        print(json.dumps({"check": "dense1_grad vs generic", "what": name,
                          "max_rel": float(((a_ - b_).abs() / (b_.abs() + 1e-30)).max().item()),
                          "max_abs": float((a_ - b_).abs().max().item())}), flush=True)
    stream = torch.cuda.current_stream()
    prewarm(fns["fused"])
    times = {k: [] for k in fns}
    for r in range(rounds):
        for k, fn in fns.items():
            saved = {e: os.environ.get(e) for e in envs.get(k, {})}
            os.environ.update(envs.get(k, {}))
            for _ in range(3):
                fn()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                fn()
                e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
            for e, v in saved.items():
                if v is None:
                    os.environ.pop(e, None)
                else:
                    os.environ[e] = v
    for k in fns:
        ms = float(np.median(times[k]))
        print(json.dumps({"cfg": "C2", "mode": "dense_grad", "H": H, "B": B, "variant": k, "ms": ms,
                          "evals_per_s": B / ms * 1e3, "rounds_ms": times[k]}), flush=True)


def run_finish(cfgs=("C2", "C5", "C3"), reps=30, rounds=4):
    """In-kernel finish of the fp64 sum (last-workgroup ticket) vs partials + the separate
    reduce kernel, whole step (launch + finish) timed with events on the launch stream."""
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    for cfg in cfgs:
        ft, d, B, S = CFG[cfg]
        P = ops.total_param_size(ft, d, True)
        gen = torch.Generator(device="cuda").manual_seed(1)
        y = torch.randn((B, d), generator=gen, device="cuda")
        t = torch.randn((B, P) if S is None else (S, B, P), generator=gen, device="cuda")
        Ls = {"fused": ops.ChainLauncher(y, t, ft, d, True, draws=S, fused_sum=True),
              "partials+reduce": ops.ChainLauncher(y, t, ft, d, True, draws=S, fused_sum=False)}
        steps = {k: (lambda L=L: (L.launch(sh), L.finish_sum(sh))) for k, L in Ls.items()}
        prewarm(steps["fused"])
        times = {k: [] for k in steps}
        for _ in range(rounds):
            for k, fn in steps.items():
                for _ in range(3):
                    fn()
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for e0, e1 in evs:
                    e0.record(stream)
                    fn()
                    e1.record(stream)
                torch.cuda.synchronize()
                times[k].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
        sums = {k: L.sum2.tolist() for k, L in Ls.items()}
        for k in steps:
            print(json.dumps({"cfg": cfg, "mode": "finish", "variant": k, "ms": float(np.median(times[k])),
                              "rounds_ms": times[k], "sum_nonfinite": sums[k]}), flush=True)


def run_pcie(reps=5):
    """The drop-in path with HOST inputs (the reference hands numpy arrays to TF on the CPU):
    C2 log_prob end to end — y, t host -> device, the fused kernel, log_prob device -> host —
    from pageable numpy arrays (what ops.chain_log_prob(numpy, numpy) does) and from pinned
    host tensors with async copies; the device-resident kernel alone for comparison."""
    ft, d, B, _ = CFG["C2"]
    P = ops.total_param_size(ft, d, True)
    rng = np.random.default_rng(0)
    y_np = rng.standard_normal((B, d)).astype(np.float32)
    t_np = rng.standard_normal((B, P)).astype(np.float32)
    y_pin, t_pin = torch.from_numpy(y_np).pin_memory(), torch.from_numpy(t_np).pin_memory()
    out_pin = torch.empty((B,), dtype=torch.float32).pin_memory()
    yd, td = y_pin.cuda(), t_pin.cuda()

    def pageable():
        lp, _ = ops.chain_log_prob(y_np, t_np, ft, d, True)
        return lp.cpu()

    def pinned():
        yd.copy_(y_pin, non_blocking=True)
        td.copy_(t_pin, non_blocking=True)
        lp, _ = ops.chain_log_prob(yd, td, ft, d, True)
        out_pin.copy_(lp, non_blocking=True)
        torch.cuda.synchronize()
        return out_pin

    def resident():
        lp, _ = ops.chain_log_prob(yd, td, ft, d, True)
        torch.cuda.synchronize()
        return lp

    for name, fn in (("host_pageable", pageable), ("host_pinned", pinned), ("device_resident", resident)):
        fn()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ms = float(np.median(ts)) * 1e3
        print(json.dumps({"cfg": "C2", "mode": "pcie", "variant": name, "ms": ms, "evals_per_s": B / ms * 1e3,
                          "h2d_bytes": B * (d + P) * 4 if name != "device_resident" else 0}), flush=True)


def run_sweep(reps=30):
    """Batch-size sweep of the C2 forward (fused log_prob + in-kernel fp64 sum): kernel time
    with HIP events on the launch stream and the fraction of the 8 TB/s peak, B = 2^10..2^27
    — where the chip saturates (small batches are launch / latency bound)."""
    ft, d, _, _ = CFG["C2"]
    P = ops.total_param_size(ft, d, True)
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    gen = torch.Generator(device="cuda").manual_seed(1)
    ymax = torch.randn((1 << 27, d), generator=gen, device="cuda")
    tmax = torch.randn((1 << 27, P), generator=gen, device="cuda")
    order = [int(v) for v in os.environ.get("NFN_SWEEP_ORDER", "").split(",") if v] or list(range(10, 28))
    for e in order:
        B = 1 << e
        L = ops.ChainLauncher(ymax[:B], tmax[:B], ft, d, True)
        prewarm(lambda: L.launch(sh), ms=100.0)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in evs:
            e0.record(stream)
            L.launch(sh)
            e1.record(stream)
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
        byts = B * (4 * d + 4 * P + 4)
        print(json.dumps({"cfg": "C2", "mode": "sweep", "log2_batch": e, "ms": ms, "evals_per_s": B / ms * 1e3,
                          "frac8TBs": byts / ms / 1e6 / 8000}), flush=True)


def run_slices(reps=10):
    """Footprint vs launch length: the 2^27-sample C2 batch as ONE launch, as eight 2^24
    launches over its eight consecutive slices (the same 17 GB, shorter launches), and one
    2^24 launch repeated eight times over the first slice (2 GB footprint)."""
    ft, d, _, _ = CFG["C2"]
    P = ops.total_param_size(ft, d, True)
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    gen = torch.Generator(device="cuda").manual_seed(1)
    ymax = torch.randn((1 << 27, d), generator=gen, device="cuda")
    tmax = torch.randn((1 << 27, P), generator=gen, device="cuda")
    big = ops.ChainLauncher(ymax, tmax, ft, d, True)
    s24 = 1 << 24
    parts = [ops.ChainLauncher(ymax[k * s24:(k + 1) * s24], tmax[k * s24:(k + 1) * s24], ft, d, True) for k in range(8)]
    def unchunked():
        os.environ["NFN_CHUNK_LOG2"] = "0"  # one launch over the whole batch (diag build)
        big.launch(sh)
        os.environ.pop("NFN_CHUNK_LOG2")

    variants = {"one_2^27_call_chunked": lambda: big.launch(sh),
                "one_2^27_launch_unchunked": unchunked,
                "eight_2^24_slices": lambda: [p_.launch(sh) for p_ in parts],
                "eight_2^24_same_slice": lambda: [parts[0].launch(sh) for _ in range(8)]}
    prewarm(variants["one_2^27_call_chunked"], ms=300.0)
    for r in range(2):
        for name, fn in variants.items():
            fn()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                fn()
                e1.record(stream)
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
            print(json.dumps({"cfg": "C2", "mode": "slices", "round": r, "variant": name, "ms": ms,
                              "frac8TBs": (1 << 27) * (4 * d + 4 * P + 4) / ms / 1e6 / 8000}), flush=True)


def main():
    which = sys.argv[1:] or ["C2"]
    if which[0] == "slices":
        run_slices()
        return
    if which[0] == "sweep":
        run_sweep()
        return
    if which[0] == "pcie":
        run_pcie()
        return
    if which[0] == "finish":
        run_finish()
        return
    if which[0] == "dgrad":
        run_dense_grad()
        return
    if which[0] == "dgradceil":  # what any faster dh / dW GEMM form could win at most
        run_dense_grad(gemm_ceiling=True, rounds=4)
        return
    if which[0] == "pdense":
        run_posterior_dense()
        return
    if which[0] == "pdensep":  # C3P: the d >= 2 posterior Dense kernel, prefetching vs synchronous
        run_posterior_dense(ft=("affine",) + ("planar",) * 4 + ("radial",) * 4, d=3, cfg="C3P", rounds=4)
        return
    if which[0] == "flows":  # the per-flow Bijector path at C2: d = 1 fast-path kernel vs the generic one
        ft, d, B, _ = CFG["C2"]
        P = ops.total_param_size(ft, d, True)
        gen = torch.Generator(device="cuda").manual_seed(1)
        y = torch.randn((B, d), generator=gen, device="cuda")
        t = torch.randn((B, P), generator=gen, device="cuda")
        L = ops.FlowsLauncher(y, t, ft, d, True)
        stream = torch.cuda.current_stream()
        sh = int(stream.cuda_stream)
        prewarm(lambda: L.launch(sh))
        names = (("d1", {}), ("generic", {"NFN_FLOW_VARIANT": "0"}))
        times, outs = {n: [] for n, _ in names}, {}
        for r in range(4):
            for name, env in names:
                os.environ.update(env)
                for _ in range(2):
                    L.launch(sh)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
                for e0, e1 in evs:
                    e0.record(stream)
                    L.launch(sh)
                    e1.record(stream)
                torch.cuda.synchronize()
                times[name].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
                outs[name] = (L.z_out.clone(), L.ldj.clone())
                for k in env:
                    os.environ.pop(k)
        ref_ldj = outs["d1"][1]
        for name in times:
            bad = (outs[name][1] != ref_ldj)
            per_flow = bad.sum(dim=1).tolist()
            first = torch.nonzero(bad[0]).flatten()[:8].tolist() if bad[0].any() else []
            print(json.dumps({"variant": name, "mismatching_rows_per_flow": per_flow, "first_rows_flow0": first,
                              "ldj_flow0_first": outs[name][1][0][first].tolist() if first else [],
                              "ref_flow0_first": ref_ldj[0][first].tolist() if first else []}), flush=True)
        for name in times:
            print(json.dumps({"variant": name, "ms_10_flows": float(np.median(times[name])), "rounds": times[name],
                              "maxdiff_z_vs_d1": maxdiff(outs[name][0], outs["d1"][0]),
                              "maxdiff_ldj_vs_d1": maxdiff(outs[name][1], outs["d1"][1])}), flush=True)
        return
    if which[0] == "occ":  # resident workgroups per CU for the d = 1 streaming kernels (C5 posterior, C2)
        for cfg in ("C5", "C2"):
            run(cfg, [{"name": "default", "env": {}}, {"name": "wg3", "env": {"NFN_WG_PER_CU": 3}},
                      {"name": "wg4", "env": {"NFN_WG_PER_CU": 4}}], rounds=4)
        return
    if which[0] == "evcost":  # what per-launch timing events cost the step loop (C2, C5)
        for cfg in ("C2", "C5"):
            ft, d, B, S = CFG[cfg]
            P = ops.total_param_size(ft, d, True)
            gen = torch.Generator(device="cuda").manual_seed(1)
            y = torch.randn((B, d), generator=gen, device="cuda")
            t = torch.randn((B, P) if S is None else (S, B, P), generator=gen, device="cuda")
            L = ops.ChainLauncher(y, t, ft, d, True, draws=S)
            stream = torch.cuda.current_stream()
            sh = int(stream.cuda_stream)
            prewarm(lambda: L.launch(sh))
            K = 200
            res = {"none": [], "per_launch": [], "region": []}
            for r in range(4):
                for mode in res:
                    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    if mode == "region":
                        evs[0][0].record(stream)
                    for e0, e1 in evs:
                        if mode == "per_launch":
                            e0.record(stream)
                        L.launch(sh)
                        if mode == "per_launch":
                            e1.record(stream)
                    if mode == "region":
                        evs[0][1].record(stream)
                    torch.cuda.synchronize()
                    wall = (time.perf_counter() - t0) * 1e3 / K
                    kern = (float(np.mean([a.elapsed_time(b) for a, b in evs])) if mode == "per_launch"
                            else evs[0][0].elapsed_time(evs[0][1]) / K if mode == "region" else None)
                    res[mode].append((wall, kern))
            for mode, v in res.items():
                print(json.dumps({"cfg": cfg, "events": mode, "wall_ms_per_launch": float(np.median([w for w, _ in v])),
                                  "event_ms_per_launch": (float(np.median([k for _, k in v])) if v[0][1] is not None else None),
                                  "rounds": v}), flush=True)
        return
    if which[0] == "postx2":  # C5 posterior: two draws per step (NFN_POST_X2) vs one
        run("C5", [{"name": "one_draw", "env": {}}, {"name": "two_draws", "env": {"NFN_POST_X2": 1}},
                   {"name": "two_draws_wg1", "env": {"NFN_POST_X2": 1, "NFN_WG_PER_CU": 1}},
                   {"name": "one_draw_b", "env": {}}], rounds=4)
        return
    if which[0] == "fwdab":  # forward kernels: full vs memory-only (flows skipped) vs compute-only (one tile)
        for cfg in ("C5", "C2", "C3"):
            run(cfg, [{"name": "full", "env": {}}, {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                      {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}}], rounds=4)
        return
    if which[0] == "gradab":  # the fused backward: full vs memory-only (flows skipped) vs compute-only (one tile)
        for cfg in ("C2", "C3"):
            run_grad(cfg, [{"name": "full", "env": {}}, {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                           {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}}], rounds=4)
        return
    if which[0] == "gradw1":  # d = 1 backward: straight-line buffer pipeline vs the generic wave kernel
        for cfg in ("C2", "R2"):
            G = {"NFN_GRAD_WAVE1": 0}
            run_grad(cfg, [{"name": "wave1", "env": {"NFN_GRAD_WAVE1": 1}}, {"name": "generic", "env": dict(G)},
                           {"name": "wave1_memory_only", "env": {"NFN_GRAD_WAVE1": 1, "NFN_ABLATE_FLOWS": 1}},
                           {"name": "generic_memory_only", "env": dict(G, NFN_ABLATE_FLOWS=1)},
                           {"name": "wave1_compute_only", "env": {"NFN_GRAD_WAVE1": 1, "NFN_ABLATE_LOADS": 1}},
                           {"name": "wave1_wpb1", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": 1}},
                           {"name": "wave1_wpb4", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": 4}},
                           {"name": "wave1_wg3", "env": {"NFN_GRAD_WAVE1": 1, "NFN_WG_PER_CU": 3}},
                           {"name": "wave1_wg4", "env": {"NFN_GRAD_WAVE1": 1, "NFN_WG_PER_CU": 4}},
                           {"name": "wave1_noprio", "env": {"NFN_GRAD_WAVE1": 1, "NFN_PRIO": 0}},
                           {"name": "wave1_b", "env": {"NFN_GRAD_WAVE1": 1}}, {"name": "generic_b", "env": dict(G)}], rounds=4)
        return
    if which[0] == "gradpolicy":  # C2 backward: cache policy of the row loads / gradient stores
        A = {"NFN_ABLATE_FLOWS": 1}
        v = [{"name": "nt_nt", "env": {}}, {"name": "plainload_nt", "env": {"NFN_GRAD_NTL": 0}},
             {"name": "nt_plainstore", "env": {"NFN_GRAD_NTS": 0}},
             {"name": "plain_plain", "env": {"NFN_GRAD_NTL": 0, "NFN_GRAD_NTS": 0}},
             {"name": "mem_nt_nt", "env": dict(A)}, {"name": "mem_nt_plainstore", "env": dict(A, NFN_GRAD_NTS=0)},
             {"name": "mem_plain_plain", "env": dict(A, NFN_GRAD_NTL=0, NFN_GRAD_NTS=0)},
             {"name": "nt_nt_b", "env": {}}, {"name": "nt_plainstore_b", "env": {"NFN_GRAD_NTS": 0}}]
        run_grad("C2", v, rounds=4)
        return
    if which[0] == "gradpc":  # d = 1 backward: producer / consumer workgroup vs the release kernel
        PC = {"NFN_GRAD_PC": 1}
        for cfg in ("C2", "R2"):
            run_grad(cfg, [{"name": "release", "env": {}}, {"name": "pc", "env": dict(PC)},
                           {"name": "pc_memory_only", "env": dict(PC, NFN_ABLATE_FLOWS=1)},
                           {"name": "pc_compute_only", "env": dict(PC, NFN_ABLATE_LOADS=1)},
                           {"name": "pc_wg3", "env": dict(PC, NFN_WG_PER_CU=3)},
                           {"name": "pc_wg2", "env": dict(PC, NFN_WG_PER_CU=2)},
                           {"name": "pc_pairs", "env": dict(PC, NFN_CHAIN_FORM=3)},
                           {"name": "release_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                           {"name": "release_b", "env": {}}, {"name": "pc_b", "env": dict(PC)}], rounds=4)
        return
    if which[0] == "gradstatic":  # C2 backward: the chain program at compile time (diag) vs the runtime program
        S = {"NFN_CHAIN_FORM": 2}
        W = {"NFN_GRAD_WAVE1": 1}
        v = [{"name": "loop", "env": {}}, {"name": "static", "env": dict(S)},
             {"name": "loop_compute", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "static_compute", "env": dict(S, NFN_ABLATE_LOADS=1)},
             {"name": "static_wave1", "env": dict(S, **W)},
             {"name": "static_wave1_wpb4", "env": dict(S, **W, NFN_GRAD_WPB=4)},
             {"name": "static_wave1_wpb1_wg12", "env": dict(S, **W, NFN_GRAD_WPB=1, NFN_WG_PER_CU=12)},
             {"name": "static_wave1_compute", "env": dict(S, **W, NFN_ABLATE_LOADS=1)},
             {"name": "static_wg4", "env": dict(S, NFN_WG_PER_CU=4)},
             {"name": "loop_b", "env": {}}, {"name": "static_b", "env": dict(S)}]
        run_grad("C2", v, rounds=4)
        return
    if which[0] == "gradsplit":  # d = 1 backward: next-tile rows in one piece vs two (second half mid-chain)
        G = {"NFN_GRAD_WAVE1": 0}
        v = [{"name": "generic", "env": dict(G)}]
        for wpb, wg in ((2, 0), (4, 3), (1, 12), (2, 4), (4, 2), (1, 8)):
            e = {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": wpb, "NFN_WG_PER_CU": wg} if wg else {"NFN_GRAD_WAVE1": 1}
            v.append({"name": f"split1_wpb{wpb}_wg{wg}", "env": dict(e)})
            v.append({"name": f"split2_wpb{wpb}_wg{wg}", "env": dict(e, NFN_GRAD_SPLIT=2)})
        v += [{"name": "generic_b", "env": dict(G)}]
        for cfg in ("C2", "R2"):
            run_grad(cfg, v, rounds=4)
        return
    if which[0] == "gradw1mem":  # d = 1 backward: memory-only stream vs resident waves; full at the best shapes
        G = {"NFN_GRAD_WAVE1": 0}
        A = {"NFN_ABLATE_FLOWS": 1}
        v = [{"name": "generic", "env": dict(G)}, {"name": "wave1_wpb4_wg3", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": 4, "NFN_WG_PER_CU": 3}},
             {"name": "wave1_wpb1_wg12", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": 1, "NFN_WG_PER_CU": 12}},
             {"name": "wave1_wpb4_wg3_noprio", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": 4, "NFN_WG_PER_CU": 3, "NFN_PRIO": 0}}]
        for wpb, wg in ((4, 1), (4, 2), (4, 3), (2, 3), (2, 5), (2, 7), (1, 12)):
            v.append({"name": f"mem_wave1_wpb{wpb}_wg{wg}", "env": dict(A, NFN_GRAD_WAVE1=1, NFN_GRAD_WPB=wpb, NFN_WG_PER_CU=wg)})
        for wg in (2, 3, 4, 6):
            v.append({"name": f"mem_generic_wg{wg}", "env": dict(A, **G, NFN_WG_PER_CU=wg)})
        v += [{"name": "generic_b", "env": dict(G)}, {"name": "wave1_wpb4_wg3_b", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": 4, "NFN_WG_PER_CU": 3}}]
        run_grad("C2", v, rounds=4)
        return
    if which[0] == "gradw1occ":  # d = 1 backward: resident waves per CU, both pipelines
        G = {"NFN_GRAD_WAVE1": 0}
        v = [{"name": "generic", "env": dict(G)}, {"name": "generic_compute_only", "env": dict(G, NFN_ABLATE_LOADS=1)},
             {"name": "wave1_compute_only", "env": {"NFN_GRAD_WAVE1": 1, "NFN_ABLATE_LOADS": 1}}]
        for wpb, wgs in ((2, (4, 5, 6, 7)), (4, (2, 3)), (1, (8, 10, 12))):
            for wg in wgs:
                v.append({"name": f"wave1_wpb{wpb}_wg{wg}", "env": {"NFN_GRAD_WAVE1": 1, "NFN_GRAD_WPB": wpb, "NFN_WG_PER_CU": wg}})
        for wg in (4, 5, 6):
            v.append({"name": f"generic_wg{wg}", "env": dict(G, NFN_WG_PER_CU=wg)})
        v.append({"name": "generic_b", "env": dict(G)})
        run_grad("C2", v, rounds=3)
        return
    if which[0] == "gradshape":  # the fused backward: persistent wave tiles vs one tile per workgroup
        for cfg in ("C2",):
            run_grad(cfg, [{"name": "wave_persistent", "env": {}},
                           {"name": "tile_per_workgroup", "env": {"NFN_GRAD_WAVE": 0}},
                           {"name": "wave_wpb1", "env": {"NFN_GRAD_WPB": 1}},
                           {"name": "wave_wpb4", "env": {"NFN_GRAD_WPB": 4}}])
        return
    if which[0] == "ceiling":  # HBM ceilings of plain torch streams over the C2 parameter buffer
        B, P = 1 << 24, 32
        t = torch.randn((B, P), device="cuda")
        out = torch.empty_like(t)
        stream = torch.cuda.current_stream()
        for name, fn, nbytes in (("sum_read", lambda: t.sum(), t.numel() * 4),
                                 ("copy", lambda: out.copy_(t), 2 * t.numel() * 4),
                                 ("fill_write", lambda: out.fill_(1.0), t.numel() * 4)):
            for _ in range(3):
                fn()
            ms = []
            for _ in range(3):
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
                for e0, e1 in evs:
                    e0.record(stream)
                    fn()
                    e1.record(stream)
                torch.cuda.synchronize()
                ms.append(float(np.median([a.elapsed_time(b) for a, b in evs])))
            m = float(np.median(ms))
            print(json.dumps({"variant": name, "ms": m, "GBps": nbytes / m / 1e6, "frac8TBs": nbytes / m / 1e6 / 8000}),
                  flush=True)
        return
    if which[0] == "kthresh":  # chain length at which the pair form stops paying in the streaming kernels
        for cfg in ("K4", "K6", "K8", "R10"):
            run(cfg, [{"name": "loop", "env": {}}, {"name": "pairs", "env": {"NFN_CHAIN_FORM": 3}}], rounds=2)
            run_grad(cfg, [{"name": "loop", "env": {}}, {"name": "pairs", "env": {"NFN_CHAIN_FORM": 3}}],
                     reps=10, rounds=2)
        return
    if which[0] == "gradform":  # pair form in the plain fused backward (C2, C1)
        for cfg in ("C2", "R2"):
            run_grad(cfg, [{"name": "loop", "env": {}}, {"name": "pairs", "env": {"NFN_CHAIN_FORM": 3}},
                           {"name": "loop_compute", "env": {"NFN_ABLATE_LOADS": 1}},
                           {"name": "pairs_compute", "env": {"NFN_CHAIN_FORM": 3, "NFN_ABLATE_LOADS": 1}}],
                     reps=10, rounds=2)
        run(cfg="R2", variants=[{"name": "loop", "env": {}}, {"name": "pairs", "env": {"NFN_CHAIN_FORM": 3}}])
        return
    if which[0] == "dgradcmp":  # pair vs loop chain form in the fused Dense backward: where do dh / dW differ
        ft, d, H = ("planar", "radial") * 5, 1, 16
        P = ops.total_param_size(ft, d, True)
        for B in (4096, 1 << 20):
            gen = torch.Generator(device="cuda").manual_seed(5)
            y = torch.randn((B, d), generator=gen, device="cuda")
            h = torch.randn((B, H), generator=gen, device="cuda")
            W = torch.randn((H, P), generator=gen, device="cuda") / 4.0
            b = 0.1 * torch.randn((P,), generator=gen, device="cuda")
            g = torch.full((B,), -1.0 / B, device="cuda")
            outs = {}
            for form in ("3", "0"):
                os.environ["NFN_CHAIN_FORM"] = form
                outs[form] = ops.chain_log_prob_dense_grad(y, h, W, b, ft, d, True, g_out=g)
                del os.environ["NFN_CHAIN_FORM"]
            (_, dh3, dW3, db3, dy3), (_, dh0, dW0, db0, dy0) = outs["3"], outs["0"]
            rowdiff = (dh3 - dh0).abs().amax(1)
            bad = torch.nonzero(rowdiff > 0).flatten()
            print(json.dumps({"B": B, "dh_rows_differing": int(bad.numel()),
                              "dh_max_abs": float(rowdiff.max().item()),
                              "dh_max_rel_row": float((rowdiff / (dh0.abs().amax(1) + 1e-30)).max().item()),
                              "first_bad_rows": bad[:8].tolist(),
                              "dW_max_rel": float(((dW3 - dW0).abs() / (dW0.abs() + 1e-30)).max().item()),
                              "db_equal": bool(torch.equal(db3, db0)), "dy_equal": bool(torch.equal(dy3, dy0))}),
                  flush=True)
        return
    if which[0] == "staticdense":  # how much a compile-time program would add in the fused Dense kernels
        run_dense([{"name": "dense1_pairs", "env": {}}, {"name": "dense1_static", "env": {"NFN_CHAIN_FORM": 2}}])
        run_dense_grad(static=True)
        return
    if which[0] == "chainform_dense":  # the pair form in the fused Dense kernels
        run_dense([{"name": "dense1_pairs", "env": {}}, {"name": "dense1_loop", "env": {"NFN_CHAIN_FORM": 0}}])
        run_posterior_dense()
        run_dense_grad()
        return
    if which[0] == "hpair":  # posterior: alternating-type pair form (U pairs per trip) vs pairs / static
        v = [{"name": "pairs", "env": {"NFN_CHAIN_FORM": 3}}, {"name": "static", "env": {"NFN_CHAIN_FORM": 2}}]
        for u in (1, 2, 5):
            v.append({"name": f"hpair_u{u}", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": u}})
        v.append({"name": "pairs_b", "env": {"NFN_CHAIN_FORM": 3}})
        run("C5", v, reps=20, rounds=4)
        return
    if which[0] == "hpair_pf":  # one pair per trip: next pair's parameters read first (U = 0) or not (U = 1)
        for cfg in ("C5", "C2"):
            run(cfg, [{"name": "hpair_u1", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 1}},
                      {"name": "hpair_u0", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 0}},
                      {"name": "hpair_u1_compute", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 1, "NFN_ABLATE_LOADS": 1}},
                      {"name": "hpair_u0_compute", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 0, "NFN_ABLATE_LOADS": 1}},
                      {"name": "hpair_u1_b", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 1}},
                      {"name": "hpair_u0_b", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 0}}], reps=20, rounds=3)
        run_dense_grad(rounds=3, forms={"fused_hpair_prefetch": 8, "fused_static": 2})
        run_grad("C2", [{"name": "loop", "env": {}}, {"name": "hpair_prefetch", "env": {"NFN_CHAIN_FORM": 8}},
                        {"name": "loop_b", "env": {}}, {"name": "hpair_prefetch_b", "env": {"NFN_CHAIN_FORM": 8}}],
                 reps=8, rounds=3)
        return
    if which[0] == "hpair_all":  # alternating-type pair form in the compute-bound d = 1 kernels
        run("C2", [{"name": "loop", "env": {}}, {"name": "hpair", "env": {"NFN_CHAIN_FORM": 8}},
                   {"name": "loop_compute", "env": {"NFN_ABLATE_LOADS": 1}},
                   {"name": "hpair_compute", "env": {"NFN_CHAIN_FORM": 8, "NFN_ABLATE_LOADS": 1}},
                   {"name": "loop_b", "env": {}}, {"name": "hpair_b", "env": {"NFN_CHAIN_FORM": 8}}], reps=20, rounds=3)
        run_dense([{"name": "dense1_pairs", "env": {}}, {"name": "dense1_hpair", "env": {"NFN_CHAIN_FORM": 8}},
                   {"name": "dense1_static", "env": {"NFN_CHAIN_FORM": 2}},
                   {"name": "dense1_pairs_b", "env": {}}], rounds=4)
        run_posterior_dense(rounds=4)
        run_dense_grad(rounds=3, forms={"fused_hpair": 8, "fused_static": 2})
        run_grad("C2", [{"name": "loop", "env": {}}, {"name": "hpair", "env": {"NFN_CHAIN_FORM": 8}},
                        {"name": "static", "env": {"NFN_CHAIN_FORM": 2}},
                        {"name": "hpair_compute", "env": {"NFN_CHAIN_FORM": 8, "NFN_ABLATE_LOADS": 1}},
                        {"name": "loop_compute", "env": {"NFN_ABLATE_LOADS": 1}},
                        {"name": "loop_b", "env": {}}, {"name": "hpair_b", "env": {"NFN_CHAIN_FORM": 8}}],
                 reps=8, rounds=3)
        return
    if which[0] == "c2form5":  # round 5: C2 / R10 streaming forward, pair bodies vs loop, occupancy
        for cfg in which[1:] or ["C2", "R10"]:
            v = [{"name": "auto_hpair", "env": {}},
                 {"name": "hpair_wg3", "env": {"NFN_WG_PER_CU": 3}},
                 {"name": "hpair_wg4", "env": {"NFN_WG_PER_CU": 4}},
                 {"name": "hpair_u0", "env": {"NFN_CHAIN_FORM": 8, "NFN_HPAIR_U": 0}},
                 {"name": "loop", "env": {"NFN_CHAIN_FORM": 0}},
                 {"name": "loop_wg3", "env": {"NFN_CHAIN_FORM": 0, "NFN_WG_PER_CU": 3}},
                 {"name": "pairs", "env": {"NFN_CHAIN_FORM": 3}},
                 {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                 {"name": "memory_only_wg3", "env": {"NFN_ABLATE_FLOWS": 1, "NFN_WG_PER_CU": 3}},
                 {"name": "hpair_compute", "env": {"NFN_ABLATE_LOADS": 1}},
                 {"name": "loop_compute", "env": {"NFN_CHAIN_FORM": 0, "NFN_ABLATE_LOADS": 1}},
                 {"name": "auto_hpair_b", "env": {}}]
            run(cfg, v, reps=20, rounds=3)
        return
    if which[0] == "chainform":  # d = 1 chain as a packed loop, two flows per dispatch, or a compile-time program
        forms = [("loop", 0), ("pairs", 3), ("static", 2)]
        for cfg in ("C2", "C5"):
            v = []
            for name, cm in forms:
                v.append({"name": name, "env": {"NFN_CHAIN_FORM": cm}})
                v.append({"name": name + "_compute", "env": {"NFN_CHAIN_FORM": cm, "NFN_ABLATE_LOADS": 1}})
                for wg in (3, 4):
                    v.append({"name": f"{name}_wg{wg}", "env": {"NFN_CHAIN_FORM": cm, "NFN_WG_PER_CU": wg}})
            run(cfg, v, reps=20, rounds=2)
        return
    if which[0] == "c1occ":  # C1 (radial x 2, 32-byte rows): stream vs chain, resident workgroups
        v = [{"name": "auto", "env": {}}, {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}}]
        v += [{"name": f"wg{w}", "env": {"NFN_WG_PER_CU": w}} for w in (2, 3, 6, 8)]
        v += [{"name": f"memory_only_wg{w}", "env": {"NFN_ABLATE_FLOWS": 1, "NFN_WG_PER_CU": w}} for w in (2, 6, 8)]
        v.append({"name": "auto_b", "env": {}})
        run("R2", v, reps=20, rounds=3)
        return
    if which[0] == "dense_occ":  # fused Dense forward with the pair bodies: resident workgroups per CU
        v = [{"name": "dense1_auto", "env": {}}]
        v += [{"name": f"dense1_wg{w}", "env": {"NFN_WG_PER_CU": w}} for w in (1, 2, 3, 4)]
        v += [{"name": "dense1_nochain", "env": {"NFN_ABLATE_FLOWS": 1}},
              {"name": "dense1_pairs", "env": {"NFN_CHAIN_FORM": 3}}, {"name": "dense1_auto_b", "env": {}}]
        run_dense(v, rounds=3)
        return
    if which[0] == "dense":  # fused Dense -> chain: wave1-style pipeline vs generic, occupancy
        run_dense([{"name": "dense1", "env": {}}, {"name": "generic", "env": {"NFN_DENSE1": 0}},
                   {"name": "dense1_wg2", "env": {"NFN_WG_PER_CU": 2}},
                   {"name": "dense1_wg3", "env": {"NFN_WG_PER_CU": 3}},
                   {"name": "dense1_nochain", "env": {"NFN_ABLATE_FLOWS": 1}},
                   {"name": "dense1_b", "env": {}}, {"name": "generic_b", "env": {"NFN_DENSE1": 0}}])
        return
    if which[0] == "dgrad_regs":  # fused Dense backward: compile-time pair bodies with the flow inputs in registers
        run_dense_grad(rounds=4, forms={"fused_hpair_regs": 8, "fused_static": 2})
        return
    if which[0] == "gradc1":  # C1 backward (radial x 2): waves per workgroup x resident workgroups
        v = [{"name": "auto", "env": {}}, {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}}]
        for wpb in (2, 4):
            for wg in (1, 2, 3, 4):
                v.append({"name": f"wpb{wpb}_wg{wg}", "env": {"NFN_GRAD_WPB": wpb, "NFN_WG_PER_CU": wg}})
        v.append({"name": "auto_b", "env": {}})
        run_grad("R2", v, reps=10, rounds=2)
        return
    if which[0] == "gradc2hp":  # C2 backward with the compile-time pair bodies: fewer resident waves?
        v = [{"name": "loop_auto", "env": {}}, {"name": "hpair_auto", "env": {"NFN_CHAIN_FORM": 8}}]
        for wpb, wgs in ((4, (1, 2)), (2, (3, 4, 5))):
            for wg in wgs:
                v.append({"name": f"hpair_wpb{wpb}_wg{wg}",
                          "env": {"NFN_CHAIN_FORM": 8, "NFN_GRAD_WPB": wpb, "NFN_WG_PER_CU": wg}})
        v += [{"name": "loop_auto_b", "env": {}}, {"name": "hpair_auto_b", "env": {"NFN_CHAIN_FORM": 8}}]
        run_grad("C2", v, reps=8, rounds=2)
        return
    if which[0] == "gradc2":  # C2 backward occupancy: waves per workgroup x resident workgroups
        v = [{"name": "auto", "env": {}}]
        for wpb in (2, 4):
            for wg in (1, 2, 3, 4, 6):
                v.append({"name": f"wpb{wpb}_wg{wg}", "env": {"NFN_GRAD_WPB": wpb, "NFN_WG_PER_CU": wg}})
        v.append({"name": "auto_b", "env": {}})
        run_grad("C2", v, reps=8, rounds=2)
        return
    if which[0] == "gradc3":  # C3 backward occupancy: waves per workgroup x register cap
        run_grad("C3", [{"name": "wpb4", "env": {}},
                        {"name": "generic_walk", "env": {"NFN_GRAD_GROUP1": 0}},
                        {"name": "wpb2", "env": {"NFN_GRAD_GROUP_WPB": 2}},
                        {"name": "wg_cap3", "env": {"NFN_WG_PER_CU": 3}},
                        {"name": "wpb2_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
                        {"name": "wpb2_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                        {"name": "wpb4_b", "env": {}}, {"name": "generic_walk_b", "env": {"NFN_GRAD_GROUP1": 0}},
                        {"name": "wpb2_b", "env": {"NFN_GRAD_GROUP_WPB": 2}}])
        return
    if which[0] == "gradc3z":  # C3 backward: z-only forward recompute vs full flow steps
        run_grad("C3", [{"name": "zonly", "env": {}}, {"name": "with_ldj", "env": {"NFN_GRAD_ZONLY": 0}},
                        {"name": "zonly_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
                        {"name": "with_ldj_compute_only", "env": {"NFN_GRAD_ZONLY": 0, "NFN_ABLATE_LOADS": 1}},
                        {"name": "zonly_b", "env": {}}, {"name": "with_ldj_b", "env": {"NFN_GRAD_ZONLY": 0}}])
        return
    if which[0] == "gradc3b128":  # C3 backward: b128 LDS tile accesses vs the split ds_*2_b32 pairs
        run_grad("C3", [{"name": "b128", "env": {}}, {"name": "split", "env": {"NFN_LDS_SPLIT": 1}},
                        {"name": "b128_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
                        {"name": "split_compute_only", "env": {"NFN_LDS_SPLIT": 1, "NFN_ABLATE_LOADS": 1}},
                        {"name": "b128_b", "env": {}}, {"name": "split_b", "env": {"NFN_LDS_SPLIT": 1}}],
                 rounds=4)
        return
    if which[0] == "c3mem":  # C3 forward: full vs compute-only vs memory-only (is the hand-off on the critical path?)
        run("C3", [{"name": "full", "env": {}}, {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
                   {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}}, {"name": "full_b", "env": {}}], rounds=4)
        return
    if which[0] == "gradc3tape":  # C3 backward: per-flow scalars taped in LDS vs recomputed in the reverse pass
        run_grad("C3", [{"name": "tape", "env": {}}, {"name": "recompute", "env": {"NFN_GRAD_TAPE": 0}},
                        {"name": "tape_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
                        {"name": "recompute_compute_only", "env": {"NFN_GRAD_TAPE": 0, "NFN_ABLATE_LOADS": 1}},
                        {"name": "tape_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                        {"name": "tape_b", "env": {}}, {"name": "recompute_b", "env": {"NFN_GRAD_TAPE": 0}}])
        return
    if which[0] == "grad":
        v = [{"name": "wave", "env": {}},
             {"name": "wpb4", "env": {"NFN_GRAD_WPB": 4}},
             {"name": "wpb1", "env": {"NFN_GRAD_WPB": 1}},
             {"name": "tile_v1", "env": {"NFN_GRAD_WAVE": 0}},
             {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "v1_memory_only", "env": {"NFN_ABLATE_FLOWS": 1, "NFN_GRAD_WAVE": 0}},
             {"name": "v1_compute_only", "env": {"NFN_ABLATE_LOADS": 1, "NFN_GRAD_WAVE": 0}}]
        run_grad("C2", v)
        run_grad("C3", [{"name": "group", "env": {}}, {"name": "g8x1", "env": {"NFN_GROUP_LANES": 8}},
                        {"name": "tile_v1", "env": {"NFN_GRAD_GROUP": 0}},
                        {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
                        {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}}])
        return
    if which[0] == "c5":  # posterior: posterior_wave1_kernel (default) vs the generic persistent kernel
        G = {"NFN_POST_WAVE1": 0}
        v = [{"name": "pw1", "env": {}},
             {"name": "generic", "env": dict(G)},
             {"name": "pw1_wg3", "env": {"NFN_WG_PER_CU": 3}}, {"name": "pw1_wg4", "env": {"NFN_WG_PER_CU": 4}},
             {"name": "pw1_wg1", "env": {"NFN_WG_PER_CU": 1}},
             {"name": "pw1_split2", "env": {"NFN_POST_SPLIT": 2}},
             {"name": "pw1_split4_wg4", "env": {"NFN_POST_SPLIT": 4, "NFN_WG_PER_CU": 4}},
             {"name": "pw1_noprio", "env": {"NFN_PRIO": 0}},
             {"name": "pw1_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "generic_split2", "env": dict(G, NFN_POST_SPLIT=2)},
             {"name": "pw1_b", "env": {}}, {"name": "generic_b", "env": dict(G)}]
        run("C5", v)
        return
    if which[0] == "group1":  # C3: branch-free buffer pipeline vs the generic group kernel
        v = [{"name": "group1", "env": {}}, {"name": "group", "env": {"NFN_GROUP1": 0}},
             {"name": "g4x2", "env": {"NFN_GROUP_LANES": 4}},
             {"name": "g4x2_compute_only", "env": {"NFN_GROUP_LANES": 4, "NFN_ABLATE_LOADS": 1}},
             {"name": "group1_wg4", "env": {"NFN_WG_PER_CU": 4}},
             {"name": "group1_wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "group1_noprio", "env": {"NFN_PRIO": 0}},
             {"name": "group1_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "group1_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "group1_noout", "env": {}, "noout": True},
             {"name": "group1_b", "env": {}}, {"name": "group_b", "env": {"NFN_GROUP1": 0}}]
        run("C3", v)
        run("C2", [{"name": "wave1", "env": {}}, {"name": "generic", "env": {"NFN_WAVE1": 0}},
                   {"name": "wave1_b", "env": {}}])
        return
    if which[0] == "c3":  # wide-event group kernel
        v = [{"name": "auto_g4x2", "env": {}},
             {"name": "g8x1", "env": {"NFN_GROUP_LANES": 8}},
             {"name": "g2x4", "env": {"NFN_GROUP_LANES": 2}},
             {"name": "tile", "env": {"NFN_LOAD_MODE": "tile"}},
             {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "g8_compute_only", "env": {"NFN_GROUP_LANES": 8, "NFN_ABLATE_LOADS": 1}},
             {"name": "g2_compute_only", "env": {"NFN_GROUP_LANES": 2, "NFN_ABLATE_LOADS": 1}},
             {"name": "wg2", "env": {"NFN_WG_PER_CU": 2}},
             {"name": "wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "precise", "env": {}, "math": "precise"}]
        run("C3", v)
        return
    if which[0] == "prio":  # wave priority around the tile hand-off
        v = [{"name": "prio", "env": {"NFN_PRIO": 1}}, {"name": "noprio", "env": {"NFN_PRIO": 0}},
             {"name": "prio_b", "env": {"NFN_PRIO": 1}}, {"name": "noprio_b", "env": {"NFN_PRIO": 0}}]
        for cfg in ("C2", "C5"):
            run(cfg, v, reps=30, rounds=4)
        return
    if which[0] == "valu":  # compute vs memory floors
        for cfg in ("C2", "C5"):
            W = {"NFN_LOAD_MODE": "wave", "NFN_NT_STORES": 1}
            v = [{"name": "wave", "env": dict(W)},
                 {"name": "compute_only", "env": dict(W, NFN_ABLATE_LOADS=1)},
                 {"name": "memory_only", "env": dict(W, NFN_ABLATE_FLOWS=1)},
                 {"name": "precise", "env": dict(W), "math": "precise"},
                 {"name": "precise_compute_only", "env": dict(W, NFN_ABLATE_LOADS=1), "math": "precise"}]
            run(cfg, v)
        return
    if which[0] == "mode":  # load-mode study, C2 and C5
        for cfg in ("C2", "C5"):
            v = [{"name": "coop", "env": {"NFN_LOAD_MODE": "coop"}},
                 {"name": "wave", "env": {"NFN_LOAD_MODE": "wave"}},
                 {"name": "coop_ntst", "env": {"NFN_LOAD_MODE": "coop", "NFN_NT_STORES": 1}},
                 {"name": "wave_ntst", "env": {"NFN_LOAD_MODE": "wave", "NFN_NT_STORES": 1}},
                 {"name": "coop_wg3", "env": {"NFN_LOAD_MODE": "coop", "NFN_WG_PER_CU": 3}},
                 {"name": "wave_wg3", "env": {"NFN_LOAD_MODE": "wave", "NFN_WG_PER_CU": 3}},
                 {"name": "wave_wg2", "env": {"NFN_LOAD_MODE": "wave", "NFN_WG_PER_CU": 2}},
                 {"name": "coop_nont", "env": {"NFN_LOAD_MODE": "coop", "NFN_NT_LOADS": 0}},
                 {"name": "wave_ablate", "env": {"NFN_LOAD_MODE": "wave", "NFN_ABLATE_FLOWS": 1}},
                 {"name": "coop_ablate", "env": {"NFN_LOAD_MODE": "coop", "NFN_ABLATE_FLOWS": 1}}]
            if cfg == "C5":
                v += [{"name": "coop_nosplit", "env": {"NFN_LOAD_MODE": "coop", "NFN_POST_SPLIT": 1}},
                      {"name": "wave_nosplit", "env": {"NFN_LOAD_MODE": "wave", "NFN_POST_SPLIT": 1}}]
            run(cfg, v)
        return
    if which[0] == "wave1":  # straight-line d = 1 wave kernel: occupancy, output, ablations
        v = [{"name": "wave1", "env": {}}, {"name": "generic", "env": {"NFN_WAVE1": 0}},
             {"name": "wave1_wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "wave1_wg4", "env": {"NFN_WG_PER_CU": 4}},
             {"name": "wave1_noout", "env": {}, "noout": True},
             {"name": "wave1_noprio", "env": {"NFN_PRIO": 0}},
             {"name": "wave1_memory_only", "env": {"NFN_ABLATE_FLOWS": 1, "NFN_WG_PER_CU": 2}},
             {"name": "wave1_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "wave1_b", "env": {}}]
        for cfg in which[1:] or ["C2", "R2"]:
            run(cfg, v)
        return
    if which[0] == "c5":  # posterior: posterior_wave1_kernel (default) vs the generic persistent kernel
        G = {"NFN_POST_WAVE1": 0}
        v = [{"name": "pw1", "env": {}},
             {"name": "generic", "env": dict(G)},
             {"name": "pw1_wg3", "env": {"NFN_WG_PER_CU": 3}}, {"name": "pw1_wg4", "env": {"NFN_WG_PER_CU": 4}},
             {"name": "pw1_wg1", "env": {"NFN_WG_PER_CU": 1}},
             {"name": "pw1_split2", "env": {"NFN_POST_SPLIT": 2}},
             {"name": "pw1_split4_wg4", "env": {"NFN_POST_SPLIT": 4, "NFN_WG_PER_CU": 4}},
             {"name": "pw1_noprio", "env": {"NFN_PRIO": 0}},
             {"name": "pw1_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "generic_split2", "env": dict(G, NFN_POST_SPLIT=2)},
             {"name": "pw1_b", "env": {}}, {"name": "generic_b", "env": dict(G)}]
        run("C5", v)
        return
    if which[0] == "group1":  # C3: branch-free buffer pipeline vs the generic group kernel
        v = [{"name": "group1", "env": {}}, {"name": "group", "env": {"NFN_GROUP1": 0}},
             {"name": "g4x2", "env": {"NFN_GROUP_LANES": 4}},
             {"name": "g4x2_compute_only", "env": {"NFN_GROUP_LANES": 4, "NFN_ABLATE_LOADS": 1}},
             {"name": "group1_wg4", "env": {"NFN_WG_PER_CU": 4}},
             {"name": "group1_wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "group1_noprio", "env": {"NFN_PRIO": 0}},
             {"name": "group1_memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "group1_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "group1_noout", "env": {}, "noout": True},
             {"name": "group1_b", "env": {}}, {"name": "group_b", "env": {"NFN_GROUP1": 0}}]
        run("C3", v)
        run("C2", [{"name": "wave1", "env": {}}, {"name": "generic", "env": {"NFN_WAVE1": 0}},
                   {"name": "wave1_b", "env": {}}])
        return
    if which[0] == "c3":  # wide-event group kernel
        v = [{"name": "auto_g4x2", "env": {}},
             {"name": "g8x1", "env": {"NFN_GROUP_LANES": 8}},
             {"name": "g2x4", "env": {"NFN_GROUP_LANES": 2}},
             {"name": "tile", "env": {"NFN_LOAD_MODE": "tile"}},
             {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "memory_only", "env": {"NFN_ABLATE_FLOWS": 1}},
             {"name": "g8_compute_only", "env": {"NFN_GROUP_LANES": 8, "NFN_ABLATE_LOADS": 1}},
             {"name": "g2_compute_only", "env": {"NFN_GROUP_LANES": 2, "NFN_ABLATE_LOADS": 1}},
             {"name": "wg2", "env": {"NFN_WG_PER_CU": 2}},
             {"name": "wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "precise", "env": {}, "math": "precise"}]
        run("C3", v)
        return
    if which[0] == "prio":  # wave priority around the tile hand-off
        v = [{"name": "prio", "env": {"NFN_PRIO": 1}}, {"name": "noprio", "env": {"NFN_PRIO": 0}},
             {"name": "prio_b", "env": {"NFN_PRIO": 1}}, {"name": "noprio_b", "env": {"NFN_PRIO": 0}}]
        for cfg in ("C2", "C5"):
            run(cfg, v, reps=30, rounds=4)
        return
    if which[0] == "valu":  # compute vs memory floors
        for cfg in ("C2", "C5"):
            W = {"NFN_LOAD_MODE": "wave", "NFN_NT_STORES": 1}
            v = [{"name": "wave", "env": dict(W)},
                 {"name": "compute_only", "env": dict(W, NFN_ABLATE_LOADS=1)},
                 {"name": "memory_only", "env": dict(W, NFN_ABLATE_FLOWS=1)},
                 {"name": "precise", "env": dict(W), "math": "precise"},
                 {"name": "precise_compute_only", "env": dict(W, NFN_ABLATE_LOADS=1), "math": "precise"}]
            run(cfg, v)
        return
    if which[0] == "mode":  # load-mode study, C2 and C5
        for cfg in ("C2", "C5"):
            v = [{"name": "coop", "env": {"NFN_LOAD_MODE": "coop"}},
                 {"name": "wave", "env": {"NFN_LOAD_MODE": "wave"}},
                 {"name": "coop_ntst", "env": {"NFN_LOAD_MODE": "coop", "NFN_NT_STORES": 1}},
                 {"name": "wave_ntst", "env": {"NFN_LOAD_MODE": "wave", "NFN_NT_STORES": 1}},
                 {"name": "coop_wg3", "env": {"NFN_LOAD_MODE": "coop", "NFN_WG_PER_CU": 3}},
                 {"name": "wave_wg3", "env": {"NFN_LOAD_MODE": "wave", "NFN_WG_PER_CU": 3}},
                 {"name": "wave_wg2", "env": {"NFN_LOAD_MODE": "wave", "NFN_WG_PER_CU": 2}},
                 {"name": "coop_nont", "env": {"NFN_LOAD_MODE": "coop", "NFN_NT_LOADS": 0}},
                 {"name": "wave_ablate", "env": {"NFN_LOAD_MODE": "wave", "NFN_ABLATE_FLOWS": 1}},
                 {"name": "coop_ablate", "env": {"NFN_LOAD_MODE": "coop", "NFN_ABLATE_FLOWS": 1}}]
            if cfg == "C5":
                v += [{"name": "coop_nosplit", "env": {"NFN_LOAD_MODE": "coop", "NFN_POST_SPLIT": 1}},
                      {"name": "wave_nosplit", "env": {"NFN_LOAD_MODE": "wave", "NFN_POST_SPLIT": 1}}]
            run(cfg, v)
        return
    if which[0] == "wave1":  # straight-line d = 1 wave kernel: unit size x occupancy
        v = [{"name": "g4", "env": {}}, {"name": "generic", "env": {"NFN_WAVE1": 0}},
             {"name": "g1", "env": {"NFN_UNIT_TILES": 1}},
             {"name": "g4_wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "g4_wg4", "env": {"NFN_WG_PER_CU": 4}},
             {"name": "g4_wg2", "env": {"NFN_WG_PER_CU": 2}},
             {"name": "g4_noout", "env": {}, "noout": True},
             {"name": "g1_noout", "env": {"NFN_UNIT_TILES": 1}, "noout": True},
             {"name": "g4_noprio", "env": {"NFN_PRIO": 0}},
             {"name": "g4_memory_only", "env": {"NFN_ABLATE_FLOWS": 1, "NFN_WG_PER_CU": 2}},
             {"name": "g4_compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "g4_b", "env": {}}, {"name": "g1_b", "env": {"NFN_UNIT_TILES": 1}}]
        for cfg in which[1:] or ["C2", "R2"]:
            run(cfg, v)
        return
    if which[0] == "mem":  # memory-path study on C2
        A = {"NFN_ABLATE_FLOWS": 1}
        v = [{"name": "auto", "env": {}},
             {"name": "nt", "env": {"NFN_NT_LOADS": 1}},
             {"name": "wg3", "env": {"NFN_WG_PER_CU": 3}},
             {"name": "wg3_nt", "env": {"NFN_WG_PER_CU": 3, "NFN_NT_LOADS": 1}},
             {"name": "noout", "env": {}, "noout": True},
             {"name": "ablate", "env": dict(A)},
             {"name": "ablate_nt", "env": dict(A, NFN_NT_LOADS=1)},
             {"name": "ablate_noout", "env": dict(A), "noout": True},
             {"name": "ablate_wg1", "env": dict(A, NFN_WG_PER_CU=1)},
             {"name": "ablate_wg2", "env": dict(A, NFN_WG_PER_CU=2)},
             {"name": "ablate_wg3", "env": dict(A, NFN_WG_PER_CU=3)},
             {"name": "ablate_ownrow_wg2", "env": dict(A, NFN_WG_PER_CU=2, NFN_LOAD_MODE="ownrow")},
             {"name": "wg1", "env": {"NFN_WG_PER_CU": 1}},
             {"name": "wg2", "env": {"NFN_WG_PER_CU": 2}},
             {"name": "compute_only", "env": {"NFN_ABLATE_LOADS": 1}},
             {"name": "noprio", "env": {"NFN_PRIO": 0}},
             {"name": "ablate_noprio", "env": dict(A, NFN_PRIO=0)}]
        run("C2", v)
        return
    base = [
        {"name": "auto", "env": {}},
        {"name": "coop", "env": {"NFN_LOAD_MODE": "coop"}},
        {"name": "ownrow", "env": {"NFN_LOAD_MODE": "ownrow"}},
        {"name": "tile", "env": {"NFN_LOAD_MODE": "tile"}},
        {"name": "coop_wg2", "env": {"NFN_LOAD_MODE": "coop", "NFN_WG_PER_CU": 2}},
        {"name": "coop_wg3", "env": {"NFN_LOAD_MODE": "coop", "NFN_WG_PER_CU": 3}},
        {"name": "ownrow_wg2", "env": {"NFN_LOAD_MODE": "ownrow", "NFN_WG_PER_CU": 2}},
        {"name": "precise", "math": "precise"},
        {"name": "ablate_flows", "env": {"NFN_ABLATE_FLOWS": 1}},
        {"name": "coop_rows128", "env": {"NFN_LOAD_MODE": "coop", "NFN_TILE_ROWS": 128}},
        {"name": "coop_rows192", "env": {"NFN_LOAD_MODE": "coop", "NFN_TILE_ROWS": 192}},
        {"name": "rows128_ablate", "env": {"NFN_TILE_ROWS": 128, "NFN_ABLATE_FLOWS": 1}},
    ]
    for cfg in which:
        run(cfg, base if cfg in ("C2", "R2") else [b for b in base if b["name"] in ("auto", "tile", "precise", "ablate_flows")])


if __name__ == "__main__":
    main()
