"""Multi-process bench path on one GPU: two ranks (both on cuda:0) run bench.py's
N > 1 step — fused kernel on each rank's own shard + the (sum, count) all-reduce —
over gloo (RCCL needs one GPU per rank; the 8-GPU nccl run is the driver's)."""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo(gpu):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--backend", "gloo", "--batch", str(1 << 18)]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 * (1 << 18)
    assert out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["scaling"] == "weak"
    # the all-reduced mean covers both ranks' shards (different seeds => finite mean)
    assert out["mean_log_prob"] == out["mean_log_prob"]


@pytest.mark.parametrize("allreduce,config", [("torch", "C2"), ("native", "C2"), ("torch", "C5")])
def test_bench_nccl_step_path_one_rank(gpu, allreduce, config):
    """The N > 1 step path over RCCL (async all-reduce ring / the library's own
    communicator) exercised with one rank on the one GPU of the test box; C5 = the
    posterior's 8-GPU form (each rank its own 2^17 samples x 64 draws)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    batch = str(1 << 18) if config == "C2" else str(1 << 14)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "5", "--warmup", "2", "--backend", "nccl", "--force-pg",
           "--allreduce", allreduce, "--config", config, "--batch", batch, "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["pg_world_size"] == 1 and np.isfinite(out["mean_log_prob"])
    # the kernel interval comes from events the chain launch records itself (nfn_set_launch_events)
    assert out["roofline"]["kernel_events"] == "dispatch" and out["roofline"]["kernel_ms"] > 0
    # the RCCL step path (the kernel finishing its sum straight into the all-reduce ring for
    # torch, the library communicator for native) gives exactly the plain N = 1 mean
    plain = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "5", "--warmup", "2",
             "--config", config, "--batch", batch, "--no-cpu-baseline"]
    r1 = subprocess.run(plain, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    ref = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][0])
    assert out["mean_log_prob"] == ref["mean_log_prob"] and out["nonfinite_log_prob"] == ref["nonfinite_log_prob"]


def test_bench_spawns_its_ranks(gpu):
    """`python bench.py --gpus 2` (no launcher): bench.py starts torch.distributed.run as a
    child and the JSON line proves the process group's size (VERDICT r1 "Next" 1)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--backend", "gloo", "--batch", str(1 << 18), "--prewarm-ms", "20"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["pg_world_size"] == 2 and out["rank_devices"] == [0, 0]
    assert out["config"]["global_batch"] == 2 * (1 << 18)
    assert out["cpu_baseline"] is None  # rank 0 at N = 1 only
    assert np.isfinite(out["mean_log_prob"]) and out["nonfinite_log_prob"] == 0


def test_two_rank_reduction_matches_one_rank(gpu):
    """The all-reduced mean over two ranks' shards equals one launch over the concatenated
    batch (fp64, rel 1e-12), and the non-finite counts add up across ranks."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "tests", "mp_reduce.py")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = {d["rank"]: d for d in (json.loads(l) for l in r.stdout.splitlines() if l.startswith("{"))}
    assert sorted(res) == [0, 1] and res[0]["world"] == 2
    assert res[0]["mean"] == res[1]["mean"]
    assert res[0]["mean"] == pytest.approx(res[0]["one_rank_mean"], rel=1e-12)
    assert res[0]["nonfinite"] == 0 and res[0]["nonfinite_poisoned"] == res[1]["nonfinite_poisoned"] == 3
