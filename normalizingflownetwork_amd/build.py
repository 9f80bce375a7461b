"""Build ``libnfn_hip.so`` in-tree for gfx950 (``python -m normalizingflownetwork_amd.build``)."""

from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
SRC = os.path.join(PKG_DIR, "csrc", "nfn_kernels.hip")
OUT = os.path.join(PKG_DIR, "libnfn_hip.so")
ARCH = os.environ.get("NFN_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def command(out: str = OUT) -> list:
    return [
        hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-Wall",
        "-I",
        os.path.join(REPO_DIR, "include"),
        "-o",
        out,
        SRC,
    ]


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile the HIP library unless it is newer than its sources."""
    deps = [SRC, os.path.join(REPO_DIR, "include", "nfn.h")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(p) for p in deps):
        return OUT
    cmd = command(OUT + ".tmp")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
