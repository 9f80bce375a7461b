"""Tuning / ablation knobs live only in the NFN_DIAG build (libnfn_hip_diag.so).

* The release library ignores them: with NFN_ABLATE_FLOWS=1 (which would zero the flow
  count), NFN_ABLATE_LOADS, NFN_LOAD_MODE, NFN_POST_SPLIT ... in the environment, the
  results still match the oracle (VERDICT r1 "Next" 8).
* The diagnostic build's alternative tile-streaming strategies all compute each sample
  with the same math (bitwise-identical outputs), and its single-range posterior agrees
  with the draw-split default.
Each runs in one child process (a fresh library binding; one GPU context)."""

import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
SCRIPT = os.path.join(REPO, "tests", "diag_modes.py")


def _run(which, extra_env=None):
    env = dict(os.environ)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, SCRIPT, which], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])[which]


def test_release_library_ignores_knobs(gpu):
    res = _run("release", {"NFN_ABLATE_FLOWS": "1", "NFN_ABLATE_LOADS": "1", "NFN_LOAD_MODE": "tile",
                           "NFN_POST_SPLIT": "3", "NFN_TILE_ROWS": "64", "NFN_WG_PER_CU": "1",
                           "NFN_GROUP": "0", "NFN_WAVE1": "0"})
    assert res["library"] == "libnfn_hip.so"
    assert res["posterior"] == "oracle parity"


def test_diag_strategies_bitwise_equal(gpu):
    from normalizingflownetwork_amd import build

    assert os.path.exists(build.DIAG_OUT), "libnfn_hip_diag.so is built by __graft_entry__.build()"
    res = _run("strategies")
    assert res["library"] == "libnfn_hip_diag.so"
    assert all(res[m] == "bitwise" for m in ("coop", "wave", "ownrow", "tile", "nfn_tile_rot_0"))


def test_diag_grad_stream_bitwise_equal(gpu):
    res = _run("grad_stream")
    assert res["library"] == "libnfn_hip_diag.so"
    assert sum(v == "bitwise" for v in res.values()) == 4


def test_diag_flow_tile_bitwise_equal(gpu):
    res = _run("flow_tile")
    assert res["library"] == "libnfn_hip_diag.so" and res["cases"] == 48


def test_diag_posterior_densep_bitwise_equal(gpu):
    res = _run("densep")
    assert res["library"] == "libnfn_hip_diag.so"
    assert sum(v == "bitwise" for v in res.values()) == 4


def test_diag_tanh_fast_ulp_bound(gpu):
    """tanh_fast on the device against fp64, in ulps of the correctly rounded tanh,
    on [-1, 1] (the polynomial below |a| = 0.3, the exp form above it) and on [-12, 12].
    Measured on MI355X (profiles/r06/r06a_pytest_gpu.log): 3.19 ulp at a = -0.346 and 3.09,
    mean 0.42 / 0.22 — the exp form with the hardware v_exp / v_rcp (its comment's 2.9 ulp
    assumes correctly rounded ones).  Pinned at 3.25 so a future change cannot loosen it
    silently; test_gpu_fullbatch's outlier counts stay the parity gate."""
    res = _run("tanh")
    print(res)
    assert res["library"] == "libnfn_hip_diag.so"
    assert res["sweep_1"]["max_ulp"] <= 3.25, res["sweep_1"]
    assert res["sweep_12"]["max_ulp"] <= 3.25, res["sweep_12"]


def test_diag_dense_grad_scalar_cache_bitwise(gpu):
    """The fused Dense backward's parameter-scalar cache (verdict r05): the exact cache gives the
    uncached compile-time program's values bitwise; the release form (shared planar tanh) is
    within 1e-5 on log_prob (its gradients are gated on the oracle by test_gpu_dense)."""
    res = _run("dense_cache")
    print(res)
    assert res["library"] == "libnfn_hip_diag.so"
    assert sum(isinstance(v, dict) and v["exact_cache"] == "bitwise" for v in res.values()) == 2
    assert sum(v == "bitwise" for k, v in res.items() if k.startswith("R10_")) == 2
