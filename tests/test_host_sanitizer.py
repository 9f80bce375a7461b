"""Host sanitizer build: the C ABI's host code — argument validation, the
flow-program builder, workspace sizing, the communicator's checks — compiled with
AddressSanitizer + UndefinedBehaviorSanitizer for the HOST only (``-Xarch_host``; device
code untouched) and driven by ``tools/abi_sanitize.cpp`` through every entry point's
rejection paths.  Every call there fails validation or is a host query, so nothing reaches
a GPU: the test runs on the CPU (it builds the two sanitized units and links them with the
release objects; about a minute)."""

import os
import shutil
import subprocess

import pytest

from conftest import REPO

OBJ = os.path.join(REPO, "normalizingflownetwork_amd", "_obj")
OUT = os.path.join(REPO, "normalizingflownetwork_amd", "_obj_asan")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=all"]


def test_abi_host_code_under_asan_ubsan():
    from normalizingflownetwork_amd import build

    if not os.path.exists(os.path.join(OBJ, "tile.o")):
        pytest.skip("release objects not built (python -m normalizingflownetwork_amd.build)")
    hipcc = build.hipcc()
    os.makedirs(OUT, exist_ok=True)
    common = [hipcc, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-I", os.path.join(REPO, "include")]
    units = [("api.o", os.path.join(REPO, "normalizingflownetwork_amd", "csrc", "nfn_api.hip")),
             ("comm.o", os.path.join(REPO, "normalizingflownetwork_amd", "csrc", "nfn_comm.hip")),
             ("drv.o", os.path.join(REPO, "tools", "abi_sanitize.cpp"))]
    for obj, src in units:
        subprocess.run(common + SAN + ["-c", src, "-o", os.path.join(OUT, obj)], check=True, capture_output=True)
    rel = [os.path.join(OBJ, f) for f in sorted(os.listdir(OBJ)) if f.endswith(".o") and f not in ("api.o", "comm.o")]
    exe = os.path.join(OUT, "abi_sanitize")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-fsanitize=address", "-fsanitize=undefined", "-fno-gpu-sanitize"]
                   + [os.path.join(OUT, u[0]) for u in units] + rel
                   + ["-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrccl", "-o", exe], check=True, capture_output=True)
    nm = subprocess.run(["nm", exe], capture_output=True, text=True).stdout
    assert "__asan_init" in nm and "__ubsan_handle" in nm, "the driver is not instrumented"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 mismatches" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    shutil.rmtree(OUT, ignore_errors=True)
