"""The parity checks every GPU test uses (one place for the tolerances and the records).

* Forward values (log-densities, posterior scores, z and log|det J| of the bijectors):
  ``oracle.tolerance_bound`` — ``|gpu - ref64| <= max(1e-5 * max(1, |ref64|), 8 * |ref32 - ref64|)``
  per sample: the north-star 1e-5 relative bound (denominator floored at 1 because a
  log-density crosses 0), widened only where the reference's own fp32 op order (the
  oracle's op-by-op fp32 mirror, one run) is ill-conditioned.  A sample admitted only
  through the widening must stay within ``WIDEN_CAP`` x that fp32 deviation.
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


def check_forward(got, ref64, ref32, what, extra_rel: float = 0.0, nonfinite: str = "fail", kind="forward"):
    """Per-sample forward parity.  ``nonfinite``: "fail" (every reference value must be
    finite and matched), "match" (a non-finite reference value — e.g. log|0| of an affine
    scale 1 + t = 0 — must be non-finite on the GPU too; the finite ones are checked).
    Returns max |gpu - ref64| / max(1, |ref64|) over the finite samples."""
    got = np.asarray(got, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    ref32 = np.asarray(ref32, np.float64)
    assert got.shape == ref64.shape, f"{what}: shape {got.shape} != {ref64.shape}"
    if got.size == 0:
        return 0.0
    fin = np.isfinite(ref64)
    if nonfinite == "match":
        assert (~np.isfinite(got[~fin])).all(), f"{what}: {int(np.isfinite(got[~fin]).sum())} finite where ref64 is not"
    else:
        assert fin.all(), f"{what}: {int((~fin).sum())} non-finite reference values"
    with np.errstate(invalid="ignore"):
        bound = O.tolerance_bound(ref64, ref32)
    if extra_rel:
        bound = bound + extra_rel * np.maximum(1.0, np.abs(ref64))
    err = np.abs(got - ref64)
    record_parity(what, got, ref64, ref32, np.where(fin, err, 0.0), np.where(fin, bound, 1.0), kind=kind)
    g, r, e, b, r32 = got[fin], ref64[fin], err[fin], bound[fin], ref32[fin]
    bad = ~(e <= b)
    if bad.any():
        i = int(np.argmax(np.where(np.isfinite(e), e - b, np.inf)))
        raise AssertionError(f"{what}: {int(bad.sum())} / {bad.size} samples outside tolerance; worst: got {g[i]!r} "
                             f"ref64 {r[i]!r} ref32 {r32[i]!r} bound {b[i]!r}")
    base = O.REL_TOL * np.maximum(1.0, np.abs(r))
    dev32 = np.abs(r32 - r)
    widened = e > base
    if widened.any():
        ratio = e[widened] / dev32[widened]
        assert (ratio <= WIDEN_CAP).all(), (
            f"{what}: {int((ratio > WIDEN_CAP).sum())} widened samples exceed {WIDEN_CAP} x |ref32 - ref64| "
            f"(max ratio {float(ratio.max()):.3g})")
    return float((e / np.maximum(1.0, np.abs(r))).max())


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
