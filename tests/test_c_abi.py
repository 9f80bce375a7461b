"""The C-ABI library loads and exports every symbol include/nfn.h declares; host-side
validation (no GPU needed: every case here fails before any HIP call)."""

import ctypes
import os
import re

import pytest

from conftest import REPO
from oracle import nfn_oracle as O


def header_symbols():
    src = open(os.path.join(REPO, "include", "nfn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nfn_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ("nfn_chain_logprob_f32", "nfn_flow_fwd_ldj_f32", "nfn_posterior_lse_f32", "nfn_version",
              "nfn_last_error", "nfn_param_size", "nfn_total_param_size", "nfn_set_math_mode"):
        assert s in syms


def test_library_exports_every_header_symbol(native_lib):
    from normalizingflownetwork_amd import _lib

    for s in header_symbols():
        assert hasattr(native_lib, s), f"{s} not exported by {_lib.LIB_NAME}"
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    # and nothing the binding expects is missing from the header
    assert set(_lib.SIGNATURES) == set(header_symbols())


def test_exported_symbols_are_c_linkage(native_lib):
    from normalizingflownetwork_amd import _lib
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (nfn_[a-z0-9_]+)$", out, flags=re.M))
    assert set(header_symbols()) <= exported


def test_version(native_lib):
    # 200: out_sum is double[2] and the workspace needs no initialisation; 201: + the
    # additive nfn_split_blocks_f32; 202: + the additive nfn_flow_vjp_f32; 203: + the
    # measurement hook nfn_set_launch_events (include/nfn.h)
    from normalizingflownetwork_amd import _lib

    assert native_lib.nfn_version() == _lib.ABI_VERSION == 203
    hdr = open(os.path.join(REPO, "include", "nfn.h")).read()
    assert re.search(r"#define NFN_ABI_VERSION 203\b", hdr)


def test_launch_events_hook_arms_and_clears(native_lib):
    # host-only: arming and clearing the pending pair launches nothing (no GPU needed)
    assert native_lib.nfn_set_launch_events(None, None) == 0


def _ids(*names):
    return (ctypes.c_int32 * max(1, len(names)))(*[O.FLOW_IDS[n] for n in names])


@pytest.mark.parametrize("d", [1, 2, 3, 8, 16, 32])
def test_param_sizes_match_python(native_lib, d):
    for f in ("planar", "radial", "affine"):
        assert native_lib.nfn_param_size(O.FLOW_IDS[f], d) == O.param_size(f, d)
    ft = ("planar", "radial", "affine", "radial")
    for tr in (0, 1):
        assert native_lib.nfn_total_param_size(ctypes.cast(_ids(*ft), ctypes.c_void_p), len(ft), d, tr) == \
            O.total_param_size(ft, d, bool(tr))


def test_bad_arguments_are_rejected_before_launch(native_lib):
    lib = native_lib
    assert lib.nfn_param_size(7, 1) == -2
    assert lib.nfn_param_size(0, 0) == -1
    assert lib.nfn_param_size(0, 33) == -1
    assert b"n_dims" in lib.nfn_last_error()
    bad = (ctypes.c_int32 * 1)(5)
    assert lib.nfn_total_param_size(ctypes.cast(bad, ctypes.c_void_p), 1, 1, 0) == -2
    # too many flows
    many = (ctypes.c_int32 * 65)(*([1] * 65))
    assert lib.nfn_total_param_size(ctypes.cast(many, ctypes.c_void_p), 65, 1, 0) == -2
    ids = ctypes.cast(_ids("planar", "radial"), ctypes.c_void_p)
    fake = 0x1000  # never dereferenced: every call below fails validation first
    # negative batch
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 8, -1, 1, ids, 2, 1, None, None, fake, None, None, None) == -1
    # row stride smaller than P
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 4, 10, 1, ids, 2, 1, None, None, fake, None, None, None) == -1
    # y_mean without y_std
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 8, 10, 1, ids, 2, 1, fake, None, fake, None, None, None) == -3
    # sum requested without workspace
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 8, 10, 1, ids, 2, 1, None, None, fake, fake, None, None) == -3
    # NULL y
    assert lib.nfn_chain_logprob_f32(None, 1, fake, 8, 10, 1, ids, 2, 1, None, None, fake, None, None, None) == -3
    # a batch longer than one chunk (2^24 + 1 samples runs as two launches) is validated as a
    # whole before the first launch: no chunk may run before the call is rejected
    big = (1 << 24) + 1
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 8, big, 1, ids, 2, 1, None, None, fake, fake, None, None) == -3
    assert b"workspace" in lib.nfn_last_error()
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 8, big, 1, ids, 2, 1, fake, None, fake, None, None, None) == -3
    assert lib.nfn_chain_logprob_f32(fake, 1, fake, 4, big, 1, ids, 2, 1, None, None, fake, None, None, None) == -1
    # bad flow id in the single-flow entry point
    assert lib.nfn_flow_fwd_ldj_f32(9, fake, 1, fake, 3, 10, 1, fake, fake, None) == -2
    assert lib.nfn_flow_fwd_ldj_f32(0, fake, 1, fake, 2, 10, 1, fake, fake, None) == -1  # stride < 2d+1
    # the one-launch Chain: unknown flow id, row stride shorter than the blocks' span,
    # negative offset, NULL offsets; B = 0 is a no-op
    offs = (ctypes.c_int32 * 2)(3, 0)
    bad = (ctypes.c_int32 * 2)(0, 9)
    assert lib.nfn_chain_fwd_ldj_f32(fake, 1, fake, 6, 10, 1, bad, offs, 2, fake, fake, None) == -2
    assert lib.nfn_chain_fwd_ldj_f32(fake, 1, fake, 5, 10, 1, ids, offs, 2, fake, fake, None) == -1
    neg = (ctypes.c_int32 * 2)(3, -1)
    assert lib.nfn_chain_fwd_ldj_f32(fake, 1, fake, 6, 10, 1, ids, neg, 2, fake, fake, None) == -1
    assert lib.nfn_chain_fwd_ldj_f32(fake, 1, fake, 6, 10, 1, ids, None, 2, fake, fake, None) == -3
    assert lib.nfn_chain_fwd_ldj_f32(fake, 1, fake, 6, 0, 1, ids, offs, 2, fake, fake, None) == 0
    # posterior with zero draws
    assert lib.nfn_posterior_lse_f32(fake, 1, fake, 80, 8, 0, 10, 1, ids, 2, 1, None, None, fake, None, None,
                                     None) == -1
    assert lib.nfn_set_math_mode(3) == -1


def test_workspace_size(native_lib):
    assert native_lib.nfn_chain_workspace_doubles(0, 1, 32) == 0
    # one partial per workgroup at any tile size (>= 64 rows per tile)
    for B in (1, 1000, 1 << 22, 1 << 24):
        for d, P in ((1, 32), (8, 140)):
            assert native_lib.nfn_chain_workspace_doubles(B, d, P) >= -(-B // 64)


def test_python_binding_fails_loudly_without_device(native_lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    from normalizingflownetwork_amd import ops

    with pytest.raises(RuntimeError):
        ops.chain_log_prob([[0.0]], [[0.0] * 8], ("radial", "radial"), 1, True)


def test_comm_entry_points_validate_before_rccl(native_lib):
    """nfn_comm_init / nfn_allreduce_mean reject bad arguments without touching
    RCCL or the device (multi-GPU boundary, include/nfn.h)."""
    from normalizingflownetwork_amd import _lib

    h = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * _lib.NFN_COMM_ID_BYTES)()
    p_uid = ctypes.cast(uid, ctypes.c_void_p)
    assert native_lib.nfn_comm_init(ctypes.byref(h), 0, p_uid, 0) == _lib.NFN_E_SHAPE
    assert native_lib.nfn_comm_init(ctypes.byref(h), 2, p_uid, 2) == _lib.NFN_E_SHAPE
    assert native_lib.nfn_comm_init(ctypes.byref(h), 2, None, 0) == _lib.NFN_E_NULLPTR
    assert native_lib.nfn_comm_unique_id(None) == _lib.NFN_E_NULLPTR
    assert native_lib.nfn_allreduce_mean(None, None, 1, None, None, None) == _lib.NFN_E_NULLPTR
    assert "allreduce" in _lib.last_error()
    assert native_lib.nfn_comm_destroy(None) == _lib.NFN_OK


def test_grid_entry_point_validates(native_lib):
    from normalizingflownetwork_amd import _lib

    ids = _ids("planar", "radial")
    p_ids = ctypes.cast(ids, ctypes.c_void_p)
    f = native_lib.nfn_chain_logprob_grid_f32
    assert f(None, 1, 4, None, 8, 10, 1, p_ids, 2, 1, None, None, None, 10, None) == _lib.NFN_E_NULLPTR
    assert f(None, 1, -1, None, 8, 10, 1, p_ids, 2, 1, None, None, None, 10, None) == _lib.NFN_E_SHAPE
    assert f(None, 1, 4, None, 8, 10, 1, p_ids, 2, 1, None, None, None, 9, None) == _lib.NFN_E_SHAPE
    assert f(None, 1, 0, None, 8, 10, 1, p_ids, 2, 1, None, None, None, 10, None) == _lib.NFN_OK


def test_dense_entry_point_validates(native_lib):
    from normalizingflownetwork_amd import _lib

    ids = _ids("planar", "radial")
    p_ids = ctypes.cast(ids, ctypes.c_void_p)
    f = native_lib.nfn_chain_logprob_dense_f32
    args = lambda H, hs, d=1: (None, 1, None, hs, H, None, None, 10, d, p_ids, 2, 1, None, None, None, None,  # noqa: E731
                               None, None)
    assert f(*args(16, 16)) == _lib.NFN_E_NULLPTR
    assert f(*args(10, 12)) == _lib.NFN_E_SHAPE       # H not a power of two
    assert f(*args(16, 8)) == _lib.NFN_E_SHAPE        # row stride < H
    assert f(*args(16, 18)) == _lib.NFN_E_SHAPE       # row stride not a multiple of 4
    assert "dense" in _lib.last_error() or "stride" in _lib.last_error()


def test_split_blocks_entry_point_validates(native_lib):
    from normalizingflownetwork_amd import _lib

    f = native_lib.nfn_split_blocks_f32
    w3 = (ctypes.c_int32 * 3)(3, 3, 2)
    p_w = ctypes.cast(w3, ctypes.c_void_p)
    assert f(None, 8, 10, p_w, 3, None, None) == _lib.NFN_E_NULLPTR      # t / dst NULL
    assert f(None, 8, 10, None, 3, None, None) == _lib.NFN_E_NULLPTR     # widths NULL
    assert f(None, 8, 10, p_w, 0, None, None) == _lib.NFN_E_SHAPE        # no blocks
    assert f(None, 7, 10, p_w, 3, None, None) == _lib.NFN_E_SHAPE        # row stride < 8
    assert "stride" in _lib.last_error()
    w0 = (ctypes.c_int32 * 2)(3, 0)
    assert f(None, 8, 10, ctypes.cast(w0, ctypes.c_void_p), 2, None, None) == _lib.NFN_E_SHAPE
    assert f(None, 8, 0, p_w, 3, None, None) == _lib.NFN_OK              # empty batch: nothing to do


def test_flow_vjp_entry_point_validates(native_lib):
    from normalizingflownetwork_amd import _lib

    f = native_lib.nfn_flow_vjp_f32
    fake = 0x1000  # never dereferenced
    assert f(9, fake, 1, fake, 3, 10, 1, None, None, fake, fake, None) == _lib.NFN_E_FLOW_ID
    assert f(0, fake, 1, fake, 2, 10, 1, None, None, fake, fake, None) == _lib.NFN_E_SHAPE    # stride < 2d+1
    assert f(1, fake, 1, fake, 3, 10, 0, None, None, fake, fake, None) == _lib.NFN_E_SHAPE    # n_dims 0
    assert f(1, fake, 1, fake, 3, -1, 1, None, None, fake, fake, None) == _lib.NFN_E_SHAPE    # negative batch
    assert f(1, None, 1, fake, 3, 10, 1, None, None, fake, fake, None) == _lib.NFN_E_NULLPTR  # NULL z
    assert "NULL" in _lib.last_error()
    assert f(1, fake, 1, fake, 3, 10, 1, None, None, None, None, None) == _lib.NFN_OK         # nothing requested
    assert f(1, fake, 1, fake, 3, 0, 1, None, None, fake, fake, None) == _lib.NFN_OK          # empty batch
