"""Build ``libnfn_hip.so`` in-tree for gfx950 (``python -m normalizingflownetwork_amd.build``).

The kernels are split over several translation units (fast / precise math
instantiations compile as separate objects) that are compiled in parallel and
linked into one shared library.

``--diag`` (``build(diag=True)``) builds ``libnfn_hip_diag.so`` with ``-DNFN_DIAG``:
the same kernels plus the tuning / ablation knobs read from ``NFN_*`` environment
variables, for ``tools/microbench.py`` only.  The release library reads none of them
(only ``NFN_MATH``, the documented initial math mode)."""

from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
OBJ_DIR = os.path.join(PKG_DIR, "_obj")
OUT = os.path.join(PKG_DIR, "libnfn_hip.so")
DIAG_OBJ_DIR = os.path.join(PKG_DIR, "_obj_diag")
DIAG_OUT = os.path.join(PKG_DIR, "libnfn_hip_diag.so")
ARCH = os.environ.get("NFN_OFFLOAD_ARCH", "gfx950")
HEADERS = [os.path.join(CSRC, "nfn_device.h"), os.path.join(CSRC, "nfn_launch.h"),
           os.path.join(CSRC, "nfn_grad_device.h"),
           os.path.join(REPO_DIR, "include", "nfn.h")]
# (object name, source, extra flags)
UNITS = [
    ("api", "nfn_api.hip", []),
    ("persistent_fast", "nfn_persistent.hip", ["-DNFN_FAST=1"]),
    ("persistent_precise", "nfn_persistent.hip", ["-DNFN_FAST=0"]),
    ("group_fast", "nfn_group.hip", ["-DNFN_FAST=1"]),
    ("group_precise", "nfn_group.hip", ["-DNFN_FAST=0"]),
    ("tile", "nfn_tile.hip", []),
    ("misc", "nfn_misc.hip", []),
    ("grad", "nfn_grad.hip", []),
    ("grad_group_fast", "nfn_grad_group.hip", ["-DNFN_FAST=1"]),
    ("grad_group_precise", "nfn_grad_group.hip", ["-DNFN_FAST=0"]),
    ("grid", "nfn_grid.hip", []),
    ("dense", "nfn_dense.hip", []),
    # the d = 1 fused Dense kernels with the compile-time pair bodies, one unit per
    # alternating program (hpair_types: 3 * IA + IB over planar = 0, radial = 1)
    ("dense_hp0", "nfn_dense.hip", ["-DNFN_DENSE_HP=0"]),
    ("dense_hp1", "nfn_dense.hip", ["-DNFN_DENSE_HP=1"]),
    ("dense_hp3", "nfn_dense.hip", ["-DNFN_DENSE_HP=3"]),
    ("dense_hp4", "nfn_dense.hip", ["-DNFN_DENSE_HP=4"]),
    ("dense_grad", "nfn_dense_grad.hip", []),
    ("sample", "nfn_sample.hip", []),
    ("comm", "nfn_comm.hip", []),
]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LINK_LIBS = ["-L" + os.path.join(ROCM, "lib"), "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-lrccl"]
SOURCES = sorted({os.path.join(CSRC, u[1]) for u in UNITS})


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _common() -> list:
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I", os.path.join(REPO_DIR, "include")]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(unit, verbose: bool, obj_dir: str, extra) -> str:
    name, src, flags = unit
    obj = os.path.join(obj_dir, name + ".o")
    srcp = os.path.join(CSRC, src)
    if _stale(obj, [srcp] + HEADERS):
        cmd = [hipcc()] + _common() + list(extra) + flags + ["-c", srcp, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = True, jobs: int = 0, diag: bool = False) -> str:
    """Compile (in parallel) the translation units that are out of date and link."""
    obj_dir, out, extra = (DIAG_OBJ_DIR, DIAG_OUT, ["-DNFN_DIAG"]) if diag else (OBJ_DIR, OUT, [])
    os.makedirs(obj_dir, exist_ok=True)
    if force:
        for u in UNITS:
            p = os.path.join(obj_dir, u[0] + ".o")
            if os.path.exists(p):
                os.remove(p)
    jobs = jobs or min(len(UNITS), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda u: _compile(u, verbose, obj_dir, extra), UNITS))
    if force or _stale(out, objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs + LINK_LIBS
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, diag="--diag" in sys.argv)
