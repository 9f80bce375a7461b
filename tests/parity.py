"""The parity checks every GPU test uses (one place for the tolerances and the records).

* Forward values (log-densities, posterior scores, z and log|det J| of the bijectors):
  ``|gpu - ref64| <= max(1e-5 * max(1, |ref64|), WIDEN_CAP * S32)`` per sample: the
  north-star 1e-5 relative bound (denominator floored at 1 because a log-density crosses
  0), widened only where the reference's own fp32 evaluation (the oracle's op-by-op fp32
  mirror) deviates more than that from the fp64 truth — S32, see :func:`check_forward`.
* Gradients: ``nfn_grad_oracle.grad_tolerance`` — ``max(2e-5 * max(1, |g64|, rowmax|g64| / 64),
  8 * dev32)`` with ``dev32`` the fp32 autodiff restatement's spread at the inputs and at
  1-ulp perturbations of them (``nfn_grad_oracle.fp32_spread``).

Every check is recorded (``conftest.record_parity``) and written to
``gpurun_out/parity.json`` at the end of the session: the margins committed under
``profiles/``."""

from __future__ import annotations

import numpy as np

from conftest import WIDEN_CAP, record_parity
from oracle import nfn_grad_oracle as G
from oracle import nfn_oracle as O


def fp32_sensitivity(y, t, flow_types, d, trainable, y_mean=None, y_std=None, n_perturbed=64, posterior=False):
    """``idx -> S32[idx]``: the reference's own fp32 sensitivity on those samples, the
    largest deviation from the fp64 truth of the oracle's op-by-op fp32 mirror evaluated
    at the inputs and at ``n_perturbed`` copies moved by one random ulp
    (``oracle.fp32_spread``).  Evaluated lazily, only for the samples a check needs it for
    (those beyond the 1e-5 base bound).  ``posterior``: t is (S, B, P)."""
    y = np.asarray(y)
    t = np.asarray(t)

    def sens(idx):
        yi = y if len(y) == 1 else y[idx]
        if posterior:
            return _posterior_spread(yi, t[:, idx], flow_types, d, trainable, y_mean, y_std, n_perturbed)
        ti = t if len(t) == 1 else t[idx]
        with np.errstate(all="ignore"):
            _, s32 = O.fp32_spread(yi, ti, flow_types, d, trainable, y_mean, y_std, n_perturbed=n_perturbed)
        return s32

    return sens


def _posterior_spread(y, t, flow_types, d, trainable, y_mean, y_std, n_perturbed, seed=0):
    rng = np.random.default_rng(seed)
    with np.errstate(all="ignore"):
        r64 = O.posterior_lse(y, t, flow_types, d, trainable, y_mean, y_std, np.float64)
        out = np.zeros_like(r64)
        y32, t32 = np.asarray(y, np.float32), np.asarray(t, np.float32)
        for k in range(n_perturbed + 1):
            yk, tk = y32, t32
            if k:
                yk = (y32 * (1 + rng.integers(-1, 2, y32.shape) * 2.0 ** -23)).astype(np.float32)
                tk = (t32 * (1 + rng.integers(-1, 2, t32.shape) * 2.0 ** -23)).astype(np.float32)
            r32 = O.posterior_lse(yk, tk, flow_types, d, trainable, y_mean, y_std, np.float32)
            out = np.maximum(out, np.abs(r32.astype(np.float64) - r64))
    return out


def check_forward(got, ref64, ref32, what, extra_rel: float = 0.0, nonfinite: str = "fail", kind="forward",
                  sensitivity=None):
    """Per-sample forward parity:
        |gpu - ref64| <= max(1e-5 * max(1, |ref64|), WIDEN_CAP * S32)
    with S32 the reference's own fp32 deviation on the sample: |ref32 - ref64| of the
    oracle's op-by-op fp32 run, or — when the check has its inputs (``sensitivity``, from
    :func:`fp32_sensitivity`) — the largest such deviation over that run and 64 runs at
    1-ulp perturbations of the inputs (one fp32 evaluation order can be luckily accurate
    on an ill-conditioned sample; the OCML-precise build of these kernels misses the
    single-run form on the same samples, DESIGN.md "Tolerances").
    ``nonfinite``: "fail" (every reference value must be finite and matched), "match" (a
    non-finite reference value — e.g. log|0| of an affine scale 1 + t = 0 — must be
    non-finite on the GPU too; the finite ones are checked).
    S32 is measured wherever the error reaches half the base bound, so the recorded margin
    of the check is the exact max |gpu - ref64| / bound.
    Returns max |gpu - ref64| / max(1, |ref64|) over the finite samples."""
    got = np.asarray(got, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    ref32 = np.broadcast_to(np.asarray(ref32, np.float64), ref64.shape)
    assert got.shape == ref64.shape, f"{what}: shape {got.shape} != {ref64.shape}"
    if got.size == 0:
        return 0.0
    fin = np.isfinite(ref64)
    if nonfinite == "match":
        assert (~np.isfinite(got[~fin])).all(), f"{what}: {int(np.isfinite(got[~fin]).sum())} finite where ref64 is not"
    else:
        assert fin.all(), f"{what}: {int((~fin).sum())} non-finite reference values"
    with np.errstate(invalid="ignore"):
        err = np.where(fin, np.abs(got - ref64), 0.0)
        s32 = np.where(fin, np.abs(ref32 - ref64), 0.0)
    base = (O.REL_TOL + extra_rel) * np.maximum(1.0, np.where(fin, np.abs(ref64), 0.0))
    # The sensitivity is measured on every sample whose error reaches half the base bound:
    # the pass / fail decision needs it only beyond the base, but the recorded margin
    # (max |gpu - ref64| / bound) is then the exact one of the bound as defined, for every
    # sample that could hold the maximum (below half the base a sample is at <= 0.5 of it).
    over = fin & ~(err <= 0.5 * base)
    n_sens = 0
    if over.any() and sensitivity is not None and got.ndim == 1:
        idx = np.flatnonzero(over)
        s32[idx] = np.maximum(s32[idx], np.asarray(sensitivity(idx), np.float64))
        n_sens = int(idx.size)
    bound = np.maximum(base, WIDEN_CAP * s32)
    record_parity(what, got, ref64, ref32, err, np.where(fin, bound, 1.0), kind=kind, sens32=s32, n_sens=n_sens)
    bad = fin & ~(err <= bound)
    if bad.any():
        i = int(np.argmax(np.where(bad, err / bound, -1.0)))
        raise AssertionError(f"{what}: {int(bad.sum())} / {int(fin.sum())} samples outside tolerance; worst: "
                             f"got {got.flat[i]!r} ref64 {ref64.flat[i]!r} ref32 {ref32.flat[i]!r} "
                             f"S32 {s32.flat[i]!r} bound {bound.flat[i]!r}")
    return float((err[fin] / np.maximum(1.0, np.abs(ref64[fin]))).max())


def check_grad(got, ref64, dev32, what, row_scale: bool = True, nonfinite: str = "match"):
    """Per-element gradient parity against the autodiff oracle on the finite reference
    elements; ``nonfinite="match"``: the non-finite patterns must be equal too."""
    got = np.asarray(got, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    assert got.shape == ref64.shape, (what, got.shape, ref64.shape)
    if got.size == 0:
        return 0.0
    bound = G.grad_tolerance(ref64, dev32, row_scale=row_scale)
    finite = np.isfinite(ref64)
    if nonfinite == "match":
        assert np.array_equal(np.isfinite(got), finite), f"{what}: non-finite pattern differs"
    err = np.abs(got - ref64)
    record_parity(what, got, ref64, ref64 + np.asarray(dev32, np.float64), np.where(finite, err, 0.0),
                  np.where(finite, bound, 1.0), kind="grad")
    bad = finite & ~(err <= bound)
    if bad.any():
        i = np.argwhere(bad)[0]
        raise AssertionError(f"{what}: {bad.sum()} elements out of tolerance; first {tuple(i)}: "
                             f"got {got[tuple(i)]!r} ref64 {ref64[tuple(i)]!r} bound {bound[tuple(i)]!r}; "
                             f"max err/bound {np.max(err[finite] / bound[finite]):.3g}")
    return float(np.max(err[finite] / bound[finite])) if finite.any() else 0.0


def check_bound(got, ref64, bound, what, kind):
    """Parity against a check-specific per-element bound (e.g. the fused Dense backward's
    dh / dW / db: the dt tolerance carried through the products), recorded like the others."""
    got = np.asarray(got, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    bound = np.broadcast_to(np.asarray(bound, np.float64), ref64.shape)
    assert got.shape == ref64.shape, (what, got.shape, ref64.shape)
    err = np.abs(got - ref64)
    record_parity(what, got, ref64, ref64, err, bound, kind=kind)
    ok = err <= bound
    assert ok.all(), f"{what}: {int((~ok).sum())} elements out of tolerance; max err/bound {np.max(err / bound):.3g}"
    return float(np.max(err / bound)) if err.size else 0.0
