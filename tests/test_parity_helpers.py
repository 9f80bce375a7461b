"""The parity helpers every GPU test uses (tests/parity.py, conftest.record_parity), on
synthetic arrays: no GPU needed."""

import numpy as np
import pytest

import conftest
from parity import check_bound, check_forward, check_grad, fp32_sensitivity


@pytest.fixture(autouse=True)
def _isolated_records(monkeypatch):
    monkeypatch.setattr(conftest, "PARITY", [])
    yield


def test_check_forward_records_and_passes():
    rng = np.random.default_rng(0)
    ref64 = rng.standard_normal(1000) * 10
    ref32 = (ref64 + 1e-7 * rng.standard_normal(1000)).astype(np.float32)
    got = ref64 + 1e-6 * rng.standard_normal(1000)
    m = check_forward(got, ref64, ref32, "synthetic")
    assert 0 < m < 1e-5
    rec = conftest.PARITY[-1]
    assert rec["n"] == 1000 and rec["check"] == "synthetic" and rec["max_err_over_bound"] < 1
    assert rec["n_small_ref"] == int((np.abs(ref64) < 1).sum())


def test_check_forward_2d_and_nonfinite():
    ref64 = np.array([[1.0, -np.inf], [3.0, 0.5]])
    ref32 = ref64.copy()
    got = np.array([[1.0, -np.inf], [3.0, 0.5 + 1e-6]])
    check_forward(got, ref64, ref32, "2d", nonfinite="match")
    with pytest.raises(AssertionError):
        check_forward(got, ref64, ref32, "2d strict")  # non-finite reference not allowed by default
    with pytest.raises(AssertionError):
        check_forward(np.array([[1.0, 0.0], [3.0, 0.5]]), ref64, ref32, "finite where ref is not", nonfinite="match")


def test_check_forward_widening_cap():
    ref64 = np.array([10.0])
    ref32 = np.array([10.0 + 1e-3])   # the reference's own fp32 is ill-conditioned here
    check_forward(np.array([10.0 + 1.5e-3]), ref64, ref32, "within 2x")
    with pytest.raises(AssertionError):
        check_forward(np.array([10.0 + 3e-3]), ref64, ref32, "beyond 2x")
    with pytest.raises(AssertionError):
        check_forward(np.array([10.0 + 1e-3]), ref64, ref64, "no widening without fp32 deviation")


def test_check_grad_and_bound_2d():
    rng = np.random.default_rng(1)
    ref = rng.standard_normal((50, 7))
    dev = np.full_like(ref, 1e-7)
    check_grad(ref + 1e-6, ref, dev, "grad")
    assert conftest.PARITY[-1]["kind"] == "grad" and conftest.PARITY[-1]["n"] == 350
    with pytest.raises(AssertionError):
        check_grad(ref + 1e-3, ref, dev, "grad too far")
    bound = np.full((50, 7), 1e-5)
    check_bound(ref + 5e-6, ref, bound, "bounded", kind="dense_grad")
    check_bound(ref[0] + 5e-6, ref[0], 1e-5, "scalar bound", kind="dense_grad")
    with pytest.raises(AssertionError):
        check_bound(ref + 2e-5, ref, bound, "out of bound", kind="dense_grad")


def test_check_forward_with_measured_sensitivity():
    """A sample beyond the base bound is judged against the reference's fp32 sensitivity
    measured with input perturbations (only for the samples that need it)."""
    ft = ("planar", "radial") * 5
    g = conftest.load_golden("stress_pr5_d1")
    y, t, r64, r32 = g["y"][:512], g["t"][:512], g["ref64"][:512], g["ref32"][:512]
    calls = []
    sens = fp32_sensitivity(y, t, ft, 1, True)

    def counting(idx):
        calls.append(len(idx))
        return sens(idx)

    check_forward(r64.copy(), r64, r32, "exact", sensitivity=counting)
    assert calls == []  # nothing beyond the base bound: no oracle re-runs
    dev = np.abs(r32 - r64) / np.maximum(1.0, np.abs(r64))
    i = int(np.argmax(dev))
    s_i = float(sens(np.array([i]))[0])  # the same perturbations check_forward draws for this one sample
    got = r64.copy()
    got[i] += 1.5 * s_i  # within 2x the measured sensitivity
    if 1.5 * s_i > 1e-5 * max(1.0, abs(r64[i])):
        check_forward(got, r64, r32, "within sensitivity", sensitivity=counting)
        assert calls == [1]
        assert conftest.PARITY[-1]["n_sens_measured"] == 1
