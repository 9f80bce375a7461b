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
