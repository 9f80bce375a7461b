"""ctypes binding of ``libnfn_hip.so`` (C ABI declared in ``include/nfn.h``).

There is no CPU fallback: if the library is missing every compute entry point
raises ``RuntimeError``.  The library is built in-tree by
``python -m normalizingflownetwork_amd.build`` (or ``__graft_entry__.build()``).
"""

from __future__ import annotations

import ctypes
import os

LIB_NAME = "libnfn_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
DIAG_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnfn_hip_diag.so")

# Symbols declared in include/nfn.h, with their ctypes signatures.
_c_int32 = ctypes.c_int32
_c_int64 = ctypes.c_int64
_vp = ctypes.c_void_p

SIGNATURES = {
    "nfn_version": (_c_int32, []),
    "nfn_last_error": (ctypes.c_char_p, []),
    "nfn_set_math_mode": (_c_int32, [_c_int32]),
    "nfn_set_launch_events": (_c_int32, [_vp, _vp]),
    "nfn_reduce_sum_f64": (_c_int32, [_vp, _c_int64, _vp, _vp]),
    "nfn_reduce_partials_f64": (_c_int32, [_vp, _vp, _vp]),
    "nfn_param_size": (_c_int32, [_c_int32, _c_int32]),
    "nfn_total_param_size": (_c_int32, [_vp, _c_int32, _c_int32, _c_int32]),
    "nfn_chain_workspace_doubles": (_c_int64, [_c_int64, _c_int32, _c_int32]),
    "nfn_posterior_workspace_doubles": (_c_int64, [_c_int64, _c_int32, _c_int32]),
    "nfn_chain_logprob_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _c_int32, _c_int32, _vp, _vp, _vp, _vp, _vp, _vp],
    ),
    "nfn_flow_fwd_ldj_f32": (
        _c_int32,
        [_c_int32, _vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _vp, _vp],
    ),
    "nfn_flow_vjp_f32": (
        _c_int32,
        [_c_int32, _vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _vp, _vp, _vp, _vp],
    ),
    "nfn_split_blocks_f32": (_c_int32, [_vp, _c_int64, _c_int64, _vp, _c_int32, _vp, _vp]),
    "nfn_chain_fwd_ldj_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _vp, _c_int32, _vp, _vp, _vp],
    ),
    "nfn_posterior_lse_f32": (
        _c_int32,
        [
            _vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _c_int64, _c_int32, _vp, _c_int32, _c_int32,
            _vp, _vp, _vp, _vp, _vp, _vp,
        ],
    ),
    "nfn_chain_logprob_grad_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _c_int32, _c_int32, _vp, _vp, _vp, _vp, _vp,
         _c_int64, _vp, _vp],
    ),
    "nfn_chain_logprob_dense_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int32, _vp, _vp, _c_int64, _c_int32, _vp, _c_int32, _c_int32, _vp, _vp,
         _vp, _vp, _vp, _vp],
    ),
    "nfn_dense_grad_workspace_floats": (_c_int64, [_c_int64, _c_int32, _c_int32]),
    "nfn_chain_logprob_dense_grad_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int32, _vp, _vp, _c_int64, _c_int32, _vp, _c_int32, _c_int32, _vp, _vp,
         _vp, _vp, _vp, _c_int64, _vp, _vp, _vp, _vp, _vp],
    ),
    "nfn_posterior_lse_dense_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _c_int64, _vp, _c_int64, _c_int32, _c_int64,
         _c_int32, _vp, _c_int32, _c_int32, _vp, _vp, _vp, _vp, _vp, _vp],
    ),
    "nfn_chain_sample_f32": (
        _c_int32,
        [_vp, _c_int64, _vp, _c_int64, _c_int64, _c_int32, _vp, _c_int32, _c_int32, _vp, _vp, _vp, _vp, _vp],
    ),
    "nfn_chain_logprob_grid_f32": (
        _c_int32,
        [_vp, _c_int64, _c_int32, _vp, _c_int64, _c_int64, _c_int32, _vp, _c_int32, _c_int32, _vp, _vp, _vp,
         _c_int64, _vp],
    ),
    "nfn_comm_unique_id": (_c_int32, [_vp]),
    "nfn_comm_init": (_c_int32, [ctypes.POINTER(_vp), _c_int32, _vp, _c_int32]),
    "nfn_comm_destroy": (_c_int32, [_vp]),
    "nfn_allreduce_mean": (_c_int32, [_vp, _vp, _c_int64, _vp, _vp, _vp]),
}

# Status codes (include/nfn.h)
NFN_OK = 0
NFN_E_SHAPE = -1
NFN_E_FLOW_ID = -2
NFN_E_NULLPTR = -3
NFN_E_HIP = -4
NFN_E_COMM = -5
NFN_COMM_ID_BYTES = 128
# include/nfn.h NFN_ABI_VERSION: the binding's argument conventions (out_sum double[2],
# uninitialised workspaces) and its symbol table (nfn_split_blocks_f32 since 201,
# nfn_flow_vjp_f32 since 202)
ABI_VERSION = 203

_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_NAME} is not built (expected at {LIB_PATH}); run "
            "`python -m normalizingflownetwork_amd.build`. There is no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nfn_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_NAME} has ABI version {lib.nfn_version()}, this binding needs {ABI_VERSION}; "
                           "rebuild with `python -m normalizingflownetwork_amd.build --force`")
    _lib = lib
    return lib


def use_diagnostic_build() -> None:
    """Bind ``libnfn_hip_diag.so`` (built with ``-DNFN_DIAG``: tuning / ablation knobs read
    from ``NFN_*`` environment variables) instead of the release library.  For
    ``tools/microbench.py`` only; must run before the first :func:`load`."""
    global LIB_PATH, LIB_NAME
    assert _lib is None, "the release library is already loaded"
    LIB_PATH, LIB_NAME = DIAG_LIB_PATH, os.path.basename(DIAG_LIB_PATH)


def last_error() -> str:
    return load().nfn_last_error().decode("utf-8", "replace")


def check(rc: int, what: str) -> None:
    """Map a C-ABI status to the reference's exception types: shape / width /
    flow-name problems are ``AssertionError`` (the reference asserts,
    ``PlanarFlow.py:22``, ``DistributionLayers.py:231,272``); HIP failures are
    ``RuntimeError``."""
    if rc == NFN_OK:
        return
    msg = f"{what}: {last_error()} (status {rc})"
    if rc in (NFN_E_SHAPE, NFN_E_FLOW_ID, NFN_E_NULLPTR):
        raise AssertionError(msg)
    raise RuntimeError(msg)
