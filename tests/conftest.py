import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


def load_golden(name):
    """Committed fixture (tests/golden/make_golden.py) as a dict of arrays."""
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    if "flow_types" in out:
        out["flow_types"] = tuple(str(s) for s in out["flow_types"])
    for k in ("d", "trainable"):
        if k in out:
            out[k] = int(out[k])
    return out


CHAIN_FIXTURES = [
    "c1_nfn_radial2_d1",
    "c2_pr5_d1",
    "c3_apr_d8",
    "asym_pra_d1",
    "asym_pra_d3",
    "asym_pra_d8",
    "asym_pra_d3_fixedbase",
    "noflows_d2",
    "bcast_y1_pr_d2",
    "stress_pr5_d1",
    "radial10_d5",
    "planar_radial_d16",
]
FLOW_FIXTURES = [f"flow_{f}_d{d}" for f in ("planar", "radial", "affine") for d in (1, 4)]

# Parity margins measured by the GPU tests (written at session end when non-empty).
PARITY = []
# A sample admitted only through the fp32-conditioning term of oracle.tolerance_bound
# (|gpu - ref64| > 1e-5 max(1, |ref64|)) must still be within WIDEN_CAP x the reference's
# own fp32 deviation on that sample, |ref32 - ref64| (the single op-by-op fp32 run).
WIDEN_CAP = 2.0


def record_parity(what, got, ref64, ref32, err, bound, kind="forward", sens32=None, n_sens=0):
    """Per check: the max of |gpu - ref64| / max(1, |ref64|); the max of |gpu - ref64| / |ref64|
    over |ref64| < 1 and how many samples there pass only through the max(1, |ref|) floor
    (err > 1e-5 |ref| but <= 1e-5); the samples admitted only through the fp32-conditioning
    widening, their count and max |gpu - ref64| / |ref32 - ref64|; the worst sample
    relative to its bound; the reference fp32 mirror's own error statistics on the same
    samples (how many exceed 1e-5, its largest relative error).  ``bound`` is the check's
    own per-element tolerance (tests/parity.py); ``sens32`` the fp32 sensitivity it used
    (``n_sens`` samples measured with input perturbations)."""
    err = np.asarray(err, np.float64)
    shape = err.shape
    bound = np.broadcast_to(np.asarray(bound, np.float64), shape).ravel()
    got = np.broadcast_to(np.asarray(got, np.float64), shape).ravel()
    ref64 = np.broadcast_to(np.asarray(ref64, np.float64), shape).ravel()
    ref32 = np.broadcast_to(np.asarray(ref32, np.float64), shape).ravel()
    err = err.ravel()
    sens = None if sens32 is None else np.broadcast_to(np.asarray(sens32, np.float64), shape).ravel()
    with np.errstate(invalid="ignore"):
        dev32 = np.abs(ref32 - ref64)
    base = 1e-5 * np.maximum(1.0, np.abs(ref64))
    fin = np.isfinite(ref64) & np.isfinite(got)
    small = fin & (np.abs(ref64) < 1.0) & (ref64 != 0.0)
    widened = fin & (err > base)
    floor_only = small & (err > 1e-5 * np.abs(ref64)) & (err <= base)
    # beyond both the 1e-5 base and the single-run gate WIDEN_CAP x |ref32 - ref64|: admitted
    # only by the perturbed runs' fp32 sensitivity (tests/parity.py)
    with np.errstate(invalid="ignore"):
        by_pert = widened & (err > WIDEN_CAP * dev32) & (err <= bound)
    w = int(np.argmax(np.where(fin, err / np.maximum(bound, 1e-300), -1.0))) if err.size else 0
    PARITY.append({
        "check": what,
        "kind": kind,
        "n": int(ref64.size),
        "nonfinite_ref": int((~np.isfinite(ref64)).sum()),
        "nonfinite_match": bool(np.array_equal(~np.isfinite(ref64), ~np.isfinite(got))),
        "max_err_over_bound": float((err[fin] / np.maximum(bound[fin], 1e-300)).max()) if fin.any() else None,
        "max_err_over_max1ref": float((err[fin] / np.maximum(1.0, np.abs(ref64[fin]))).max()) if fin.any() else None,
        "max_rel_err_small_ref": float((err[small] / np.abs(ref64[small])).max()) if small.any() else None,
        "n_small_ref": int(small.sum()),
        "n_floor_only": int(floor_only.sum()),
        "n_widened": int(widened.sum()),
        "n_pass_only_by_perturbation": int(by_pert.sum()),
        "max_err_over_base_unwidened": float((err[fin & ~widened] / base[fin & ~widened]).max())
        if (fin & ~widened).any() else None,
        "widened_max_err_over_dev32": float((err[widened] / np.maximum(dev32[widened], 1e-300)).max())
        if widened.any() else None,
        "widened_max_err_over_base": float((err[widened] / base[widened]).max()) if widened.any() else None,
        "widened_max_err_over_sens32": float((err[widened] / np.maximum(sens[widened], 1e-300)).max())
        if (widened.any() and sens is not None) else None,
        "n_sens_measured": int(n_sens),
        "ref32_n_over_base": int((fin & (dev32 > base)).sum()),
        "ref32_max_err_over_max1ref": float((dev32[fin] / np.maximum(1.0, np.abs(ref64[fin]))).max())
        if fin.any() else None,
        "worst": {"idx": w, "got": float(got[w]), "ref64": float(ref64[w]), "ref32": float(ref32[w]),
                  "err_over_bound": float(err[w] / bound[w])} if err.size else None,
    })


def pytest_sessionfinish(session, exitstatus):
    if not PARITY:
        return
    import json

    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity.json"), "w") as f:
        json.dump({"widen_cap": WIDEN_CAP, "checks": PARITY}, f, indent=1)


@pytest.fixture(scope="session")
def native_lib():
    """The built C-ABI library (built in-tree on demand; hipcc cross-compiles without a GPU)."""
    from normalizingflownetwork_amd import _lib, build

    build.build(verbose=False)
    return _lib.load()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test requested but no HIP device is visible")
    from normalizingflownetwork_amd import _lib

    _lib.load()  # loud failure if the extension is missing
    return torch.device("cuda", 0)
