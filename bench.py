#!/usr/bin/env python3
"""Benchmark: fused conditional-flow log_prob on MI355X.

Metric (BASELINE.json): "log_prob evals/sec (whole node), 10-flow planar+radial
chain, y_dim=1".  Default workload = config C2 per GPU: B = 2^24 samples,
y_dim = 1, flows ("planar","radial") x 5, trainable base => P = 32 floats of
per-sample parameters.  Multi-GPU (C4 form): every rank owns its own 2^24 batch
(weak scaling) and the step ends with ONE RCCL all-reduce of (sum log_prob,
count) — the mean log-likelihood.

One step = the fused chain kernel over the rank's batch (writes log_prob (B,)
and per-workgroup fp64 partial sums) + the partials reduce + (N > 1) the
all-reduce.  Inputs are synthetic N(0,1) float32 generated on the device and
resident in HBM before the timed region.  The dominant kernel's duration (`roofline`) comes
from HIP events that the step's launch records from its own dispatch (the library's
nfn_set_launch_events hook, hipExtLaunchKernel): no marker packets sit between the timed
steps, so the wall clock (`value`) carries no timing overhead (`--event-mode marker`: the
older hipEventRecord pair around every step).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C5|C3P]
                  [--mode forward|grad|dense|dense_grad|bijector|flows [--flow-params views|separate|strided]]
  N > 1: either under a launcher (python -m torch.distributed.run --nproc-per-node N ...
  bench.py --gpus N), or plain `python bench.py --gpus N`, which starts that launcher as a
  child process itself (before touching the GPU) and exits with its status.

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from normalizingflownetwork_amd import _lib, ops  # noqa: E402
from normalizingflownetwork_amd.parallel import init_from_env  # noqa: E402

C2_FLOWS = ("planar", "radial") * 5
CONFIGS = {
    # name: (flow_types, d, batch per GPU, draws or None)
    "C2": (C2_FLOWS, 1, 1 << 24, None),
    "C3": (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8, 1 << 22, None),
    "C5": (C2_FLOWS, 1, 1 << 17, 64),
    # C5's posterior over C3's flow stack at y_dim 3 (P = 60: inside the fused Dense path's
    # P <= 64; C3's own d = 8, P = 140 is not) — the d >= 2 posterior Dense kernel's line
    "C3P": (("affine",) + ("planar",) * 4 + ("radial",) * 4, 3, 1 << 17, 64),
    # configs[0]'s flow stack (radial, radial) at C2's batch, and the estimator's default
    # NormalizingFlowNetwork(n_flows=10): radial x 10 (NormalizingFlowNetwork.py:10-17)
    "R2": (("radial", "radial"), 1, 1 << 24, None),
    "R10": (("radial",) * 10, 1, 1 << 24, None),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes_per_launch(d: int, P: int, B: int, S) -> float:
    """4*d (y) + 4*P (t) + 4 (log_prob) per eval; the posterior
    reads t once per (draw, sample) and y / writes out once per sample."""
    if S is None:
        return float(B) * (4 * d + 4 * P + 4)
    return float(B) * (S * 4 * P + 4 * d + 4)


def algorithmic_bytes_grad(d: int, P: int, B: int) -> float:
    """Fused backward: y (4d) + t (4P) + upstream gradient (4) in, d/dt (4P) + d/dy (4d) out."""
    return float(B) * (8 * d + 8 * P + 4)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_workers() -> int:
    """Host cores this process may use: its affinity mask, bounded by the job's thread
    share (OMP_NUM_THREADS is the box's CPU share on the GPU pool, 16 per GPU)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def _cpu_job(kind: str, cfg: str, rows: int, seed: int, H: int):
    """(run, evals per run) for one CPU-baseline worker: the oracle's op-by-op restatement of
    the reference's eager path on `rows` samples (test infrastructure, timed only here)."""
    from oracle import nfn_oracle as O

    ft, d, _, S = CONFIGS[cfg]
    P = O.total_param_size(ft, d, True)
    rng = np.random.default_rng(seed)
    y = rng.standard_normal((rows, d)).astype(np.float32)
    if kind == "forward":
        if S is None:
            t = rng.standard_normal((rows, P)).astype(np.float32)
            return (lambda: O.chain_log_prob(y, t, ft, d, True, np.float32)), rows
        t = rng.standard_normal((S, rows, P)).astype(np.float32)
        return (lambda: O.posterior_lse(y, t, ft, d, True, dtype=np.float32)), rows * S
    if kind == "bijector":
        t = rng.standard_normal((rows, P)).astype(np.float32)
        _, blocks = O.split_params(t, ft, d, True)

        def chain():
            z, ldj = y, np.zeros(rows, np.float32)
            for f, tk in zip(ft, blocks):
                z, l = O.flow_forward_fldj(f, z, tk, d)
                ldj = ldj + l
            return z, ldj

        return chain, rows
    if kind == "grad":
        from oracle import nfn_grad_oracle as G

        t = rng.standard_normal((rows, P)).astype(np.float32)
        g = np.full((rows,), -1.0 / rows, np.float32)
        return (lambda: G.chain_log_prob_grad(y, t, ft, d, True, g_out=g, dtype=np.float32)), rows
    lead = () if S is None else (S,)
    h = rng.standard_normal(lead + (rows, H)).astype(np.float32)
    W = (rng.standard_normal(lead + (H, P)) / np.sqrt(H)).astype(np.float32)
    b = (0.1 * rng.standard_normal(lead + (P,))).astype(np.float32)
    if kind == "dense":
        if S is None:
            return (lambda: O.chain_log_prob(y, h @ W + b, ft, d, True, np.float32)), rows
        return (lambda: O.posterior_lse(y, np.matmul(h, W) + b[:, None], ft, d, True, dtype=np.float32)), rows * S
    # dense_grad: Keras autodiff through Dense(P) and the chain = t by GEMM, the chain's
    # autodiff (torch fp32 over the eager op sequence), then dh = dt W^T, dW = h^T dt, db
    from oracle import nfn_grad_oracle as G

    g = np.full((rows,), -1.0 / rows, np.float32)

    def run():
        t = h @ W + b
        _, gt, gy = G.chain_log_prob_grad(y, t, ft, d, True, g_out=g, dtype=np.float32)
        return gt @ W.T, h.T @ gt, gt.sum(0), gy

    return run, rows


def _cpu_worker(job):
    """One process of the pooled baseline: single-threaded numerics on its own row slice,
    timed until `seconds` have passed; returns (evals, elapsed)."""
    kind, cfg, rows, seed, H, seconds = job
    from threadpoolctl import threadpool_limits

    torch.set_num_threads(1)
    with threadpool_limits(limits=1):
        run, per = _cpu_job(kind, cfg, rows, seed, H)
        run()  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            run()
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds or reps >= 200:
                break
    return reps * per, el


def _cpu_pool(n: int, kind: str, cfg: str, rows: int, H: int, seconds: float) -> float:
    """n concurrent single-threaded workers on their own `rows`-row slices: summed evals/s."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this process's HIP state is inherited
    pool = ctx.Pool(n)
    try:
        res = pool.map(_cpu_worker, [(kind, cfg, rows, 22 + i, H, seconds) for i in range(n)])
        pool.close()  # workers exit on their own (the context manager's terminate() SIGTERMs them)
        pool.join()
    except BaseException:
        pool.terminate()
        raise
    return sum(e / el for e, el in res)


def cpu_baseline(kind: str, cfg: str, H: int = 16, seconds: float = 8.0) -> dict:
    """The reference-path stand-in timed on this host's cores (rank 0, N = 1 only): the
    oracle's fp32 op-by-op restatement of TF eager's per-op evaluation
    (`BaseEstimator.py:77-86` / `:19-31` for the backward).  TF runs each Eigen op over its
    intra-op pool on every core, streaming the op's whole batch; so the headline `value` runs
    one single-threaded worker per core, each over a WHOLE bounded batch (its arrays stream
    from DRAM per op, as TF's do), concurrently in a process pool.  `cache_resident_value` is
    the same pool over one row slice of that batch per core (arrays that stay in the core's
    caches: ~2.6x faster per core, which no per-op evaluation of the reference's batch gets);
    `single_thread` is the whole batch on one core."""
    ft, d, _, S = CONFIGS[cfg]
    total = {"forward": 1 << 20, "dense": 1 << 20, "grad": 1 << 16, "dense_grad": 1 << 16, "bijector": 1 << 20}[kind]
    if S is not None:
        total = max(64, total // S)
    n = cpu_workers()
    if kind in ("grad", "dense_grad"):
        # torch's autograd engine initialises the HIP runtime in every worker that runs a
        # backward (device threads), so those workers hold the GPU open: parent + workers
        # stay within the 16 processes a leased GPU allows
        n = min(n, 15)
    one_evals, one_el = _cpu_worker((kind, cfg, total, 22, H, seconds))
    streamed = _cpu_pool(n, kind, cfg, total, H, seconds)
    rows = max(64, total // n)
    cached = _cpu_pool(n, kind, cfg, rows, H, seconds)
    unit_rows = "(draw, sample) pairs" if S is not None else "samples"
    per = S or 1
    what = {"forward": "numpy fp32 op-by-op chain", "dense": "numpy fp32 GEMM + op-by-op chain",
            "grad": "torch fp32 autodiff of the eager op sequence",
            "bijector": "numpy fp32 flow-by-flow forward + fldj",
            "dense_grad": "numpy GEMM + torch fp32 autodiff of the eager op sequence + weight-gradient GEMMs"}[kind]
    return {
        "value": streamed,
        "unit": "evals/s",
        "cores": n,
        "kind": "port",
        "sample": f"{cfg} {kind}: {n} concurrent single-threaded workers, each over a whole {total}-row batch "
                  f"({total * per} {unit_rows}; every op's arrays stream from DRAM, as TF's intra-op pool streams "
                  f"each op over the batch), {what} (oracle/), ~{seconds:.0f} s each",
        "cache_resident_value": cached,
        "cache_resident_sample": f"the same {n} workers over {rows}-row slices of one {rows * n}-row batch "
                                 f"(cache-resident arrays, faster per core than any per-op pass over the batch)",
        "single_thread": one_evals / one_el,
        "single_thread_sample": f"{total} rows on 1 core ({unit_rows})",
        "host_cpus": os.cpu_count(),
        "cpu_model": cpu_model(),
    }


def load_traffic(cfg: str, B: int):
    """Per-launch HBM bytes of the chain kernel from committed rocprofv3 PMC passes
    (`tools/prof_summary.py pmc` -> profiles/*pmc_<cfg>.json, the latest round's file), or None."""
    import glob

    cands = sorted(glob.glob(os.path.join(REPO, "profiles", f"*pmc_{cfg}.json")))
    if not cands:
        return None, None
    with open(cands[-1]) as f:
        rec = json.load(f)
    if int(rec.get("batch", -1)) != B:
        return None, None
    return float(rec["hbm_bytes_per_launch"]), os.path.relpath(cands[-1], REPO)


def spawn_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: run N ranks as a CHILD
    `torch.distributed.run` (one process per GPU, 127.0.0.1 rendezvous) with the same
    arguments, stream its output and return its exit code.  Runs before anything here
    touches the GPU; nothing is exec'd in place."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def nfn_environment(allow_ablation: bool = False) -> dict:
    """Every NFN_* variable in the environment (recorded in the JSON line).  The release
    library reads only NFN_MATH (overridden by --math); the tuning / ablation knobs exist
    only in the NFN_DIAG build, and an ablation knob in the environment aborts the bench
    (unless --diag: an A/B study with the diagnostic library, never a reported line)."""
    env = {k: v for k, v in os.environ.items() if k.startswith("NFN_")}
    bad = [k for k in env if k.startswith("NFN_ABLATE")]
    if bad and not allow_ablation:
        raise SystemExit(f"refusing to benchmark with ablation knobs set: {bad}")
    return env


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--prewarm-ms", type=float, default=300.0,
                    help="untimed launches before the W warmup steps until this much device time has "
                         "run: the MI355X raises its clocks over the first tens of ms of sustained load, "
                         "so a short warmup would time the ramp, not the steady state (0 disables)")
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="override the per-GPU batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--diag", action="store_true",
                    help="bind libnfn_hip_diag.so (NFN_* knobs, e.g. NFN_ABLATE_FLOWS=1): A/B studies only, "
                         "never a reported line")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--math", default="fast", choices=["fast", "precise"])
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only for tests)")
    ap.add_argument("--mode", default="forward", choices=["forward", "grad", "dense", "dense_grad", "bijector", "flows", "grid"],
                    help="forward = fused log_prob (the headline); grad = the fused backward of the "
                         "mean-NLL training step (d/dt, d/dy for a uniform upstream gradient); dense = the "
                         "output Dense layer (H -> P) fused into the chain, streaming h instead of t; "
                         "dense_grad = the training step's backward through that fused layer (dh, dW, db, dy); "
                         "bijector = the Bijector API's Chain.forward + forward_log_det_jacobian over the "
                         "layer's flows in one launch (no base density); flows = the same Chain flow by flow, "
                         "one single-flow launch per flow (nfn_flow_fwd_ldj_f32)")
    ap.add_argument("--grid", type=int, default=256,
                    help="--mode grid: grid values G (each evaluated under every one of the B parameter rows; "
                         "B defaults to 2^16, so G x B = 2^24 evals as at C2)")
    ap.add_argument("--hidden", type=int, default=16, help="--mode dense / dense_grad: hidden width H")
    ap.add_argument("--event-every", type=int, default=None,
                    help="time the dominant kernel on every E-th timed step (default 4 with dispatch-recorded "
                         "events: each timed launch still costs ~3 us of wall clock, but its interval is the "
                         "kernel's own, profiles/r05/r05zi_*; 1 with markers, whose sampled intervals would "
                         "include the dispatch gap: +1 %% at C2, profiles/r03/r03u_event_sampling_ab.log)")
    ap.add_argument("--event-mode", default="auto", choices=["auto", "dispatch", "marker"],
                    help="how the timed steps' kernel events are recorded: 'dispatch' arms "
                         "nfn_set_launch_events so the step's first (dominant) launch records them from its own "
                         "dispatch (hipExtLaunchKernel: no marker packets between steps); 'marker' records "
                         "them with hipEventRecord around the whole step; 'auto' = dispatch for every mode "
                         "whose step is one dominant launch, marker for --mode flows (ten launches)")
    ap.add_argument("--flow-params", default="views", choices=["views", "separate", "strided"],
                    help="--mode flows: the flows' parameters as views of the layer's one wide t (each step "
                         "first makes the blocks contiguous in one pass, nfn_split_blocks_f32, as the "
                         "package's flows do), built individually over their own contiguous (B, param_size) "
                         "tensors, or read straight from the wide rows by every launch (strided: each launch "
                         "fetches whole 128-B lines)")
    ap.add_argument("--force-pg", action="store_true",
                    help="initialise the process group and run the all-reduce even at N = 1 (tests)")
    ap.add_argument("--allreduce", default="torch", choices=["torch", "native"],
                    help="N > 1 mean all-reduce: torch.distributed, or the library's own RCCL "
                         "communicator (nfn_allreduce_mean, stream-ordered; needs --backend nccl)")
    args = ap.parse_args()
    if args.diag:  # measurement tool only: the NFN_DIAG library reads NFN_* ablation / tuning knobs
        _lib.use_diagnostic_build()
    nfn_env = nfn_environment(allow_ablation=args.diag)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))

    rank, world, local_rank = init_from_env(backend=args.backend, force=args.force_pg)
    dist_on = dist.is_initialized()  # world > 1, or --force-pg (test hook: the N > 1 step path at N = 1)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    ops.set_math_mode(args.math)
    pg_world = dist.get_world_size() if dist_on else 1
    rank_devices = [dev_index]
    if dist_on:
        rank_devices = [None] * pg_world
        dist.all_gather_object(rank_devices, dev_index)

    ft, d, B, S = CONFIGS[args.config]
    if args.batch:
        B = args.batch
    P = ops.total_param_size(ft, d, True)
    gen = torch.Generator(device=dev).manual_seed(22 + rank)
    y = torch.randn((B, d), generator=gen, device=dev)
    grad_mode = args.mode in ("grad", "dense_grad")
    dense_mode = args.mode in ("dense", "dense_grad")
    H = args.hidden
    if dense_mode:
        # the output Dense layer fused: per sample h (B, H) instead of t (B, P); C5: the
        # posterior with the output DenseVariational layer fused (per draw h_s, W_s, b_s)
        hgen = torch.Generator(device=dev).manual_seed(122 + rank)
        lead = () if S is None else (S,)
        h = torch.randn(lead + (B, H), generator=hgen, device=dev)
        Wd = torch.randn(lead + (H, P), generator=hgen, device=dev) / float(np.sqrt(H))
        bd = 0.1 * torch.randn(lead + (P,), generator=hgen, device=dev)
        if grad_mode:
            assert S is None, "--mode dense_grad covers the plain chain configs (C2, C3)"
            g_up = torch.full((B,), -1.0 / B, dtype=torch.float32, device=dev)  # d(mean NLL)/d log_prob
            launcher = ops.DenseGradLauncher(y, h, Wd, bd, ft, d, True, g_out=g_up)
        else:
            launcher = (ops.DenseLauncher if S is None else ops.PosteriorDenseLauncher)(y, h, Wd, bd, ft, d, True)
    elif args.mode == "grid":
        # the density grid of flow_plotting.plot_model: G y values x B parameter rows
        assert S is None, "--mode grid covers the plain chain configs (C2, C3)"
        if not args.batch:
            B = 1 << 16
        G = args.grid
        yg = (torch.linspace(-4.0, 4.0, G, device=dev).reshape(G, 1).repeat(1, d).contiguous() if d == 1 else
              torch.randn((G, d), generator=gen, device=dev))
        t = torch.randn((B, P), generator=gen, device=dev)
        launcher = ops.GridLauncher(yg, t, ft, d, True)
    elif args.mode in ("bijector", "flows"):
        assert S is None, "--mode bijector / flows cover the plain chain configs (C2, C3)"
        t = torch.randn((B, P), generator=gen, device=dev)
        if args.mode == "bijector":
            launcher = ops.BijectorLauncher(y, t, ft, d, True)
        else:
            launcher = ops.FlowsLauncher(y, t, ft, d, True, params=args.flow_params)
    else:
        t = torch.randn((B, P) if S is None else (S, B, P), generator=gen, device=dev)
        if grad_mode:
            assert S is None, "--mode grad covers the plain chain configs (C2, C3)"
            g_up = torch.full((B,), -1.0 / B, dtype=torch.float32, device=dev)  # d(mean NLL)/d log_prob
            launcher = ops.GradLauncher(y, t, ft, d, True, g_out=g_up)
        else:
            launcher = ops.ChainLauncher(y, t, ft, d, True, write_values=True, draws=S)
    # the steps run on a stream of their own (back-to-back launches cost the same there as on
    # the legacy default stream: tools/graph_gap.py, profiles/r05/r05zh); inputs and launchers
    # above were made on the default stream, so it is drained first
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = int(stream.cuda_stream)
    # (sum, non-finite) all-reduce buffers (the count is B per rank): a ring of two, so step i's all-reduce
    # (async, on the process group's stream) overlaps step i+1's chain kernel; a buffer
    # is reused only after the stream has waited for its previous all-reduce.  Over RCCL
    # the chain kernel finishes its {sum, non-finite} straight into the ring slot
    # (ChainLauncher.bind_sum): no copy kernels between the chain and the collective.
    reds = [torch.zeros((2,), dtype=torch.float64, device=dev) for _ in range(2)]
    direct = dist_on and args.backend == "nccl" and args.allreduce == "torch" and hasattr(launcher, "bind_sum") \
        and getattr(launcher, "fused_sum", False)
    works = [None, None]
    nstep = [0]
    evals_per_step = B * (1 if S is None else S) * (args.grid if args.mode == "grid" else 1)
    native = None
    if dist_on and args.allreduce == "native":
        from normalizingflownetwork_amd.parallel import NativeComm

        native = NativeComm()

    ev_dispatch = args.event_mode == "dispatch" or (args.event_mode == "auto" and args.mode != "flows")
    set_events = _lib.load().nfn_set_launch_events

    def step(ev0=None, ev1=None):
        if direct:
            i = nstep[0] % 2
            nstep[0] += 1
            if works[i] is not None:
                works[i].wait()  # stream-side wait: the slot's previous all-reduce is done
            launcher.bind_sum(reds[i])
        if ev0 is not None and ev_dispatch:
            set_events(ctypes.c_void_p(ev0.cuda_event), ctypes.c_void_p(ev1.cuda_event))
        elif ev0 is not None:
            ev0.record(stream)
        launcher.launch(sh)
        if ev1 is not None and not ev_dispatch:
            ev1.record(stream)
        if grad_mode or args.mode in ("bijector", "flows", "grid"):  # per-sample outputs stay on their rank
            return
        if direct:
            works[i] = dist.all_reduce(reds[i], async_op=True)
            last_red[0] = reds[i]
            return
        s = launcher.finish_sum(sh)
        if native is not None:
            native.allreduce_mean(launcher.sum2, B, sh)
        elif dist_on:
            i = nstep[0] % 2
            nstep[0] += 1
            buf = reds[i]
            if args.backend == "nccl":
                if works[i] is not None:
                    works[i].wait()  # stream-side wait: the buffer's previous all-reduce is done
                buf[0:1].copy_(s)
                buf[1:2].copy_(launcher.nonfinite)
                works[i] = dist.all_reduce(buf, async_op=True)
            else:  # gloo reduces host tensors
                buf[0:1].copy_(s)
                buf[1:2].copy_(launcher.nonfinite)
                hb = buf.cpu()
                dist.all_reduce(hb)
                buf.copy_(hb)
            last_red[0] = buf

    last_red = [reds[0]]

    def drain():
        for w in works:
            if w is not None:
                w.wait()

    # clock ramp: keep the device busy with untimed steps for >= --prewarm-ms of device time
    prewarm_steps = 0
    if args.prewarm_ms > 0:
        # the step time is taken AFTER a first untimed step: the first launch carries the
        # module load and first-touch costs (milliseconds), which would cut the prewarm short
        step()
        drain()
        torch.cuda.synchronize()
        pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        pe0.record(stream)
        for _ in range(4):
            step()
        pe1.record(stream)
        drain()
        torch.cuda.synchronize()
        per = max(pe0.elapsed_time(pe1) / 4, 1e-3)
        prewarm_steps = int(min(20000, np.ceil(args.prewarm_ms / per)))
        if dist_on:  # every rank must issue the same number of step all-reduces
            drain()
            cnt = torch.tensor([prewarm_steps], dtype=torch.int64,
                               device=dev if args.backend == "nccl" else torch.device("cpu"))
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX)
            prewarm_steps = int(cnt.item())
        for _ in range(prewarm_steps):
            step()
        drain()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    # the dominant kernel's duration: HIP events recorded by its own dispatch (default), or
    # hipEventRecord markers on its stream around the launches of the timed steps (every step
    # by default; the marker pairs add ~4 us per step to the wall clock, which `value` keeps)
    ev_every = max(1, args.event_every if args.event_every is not None else (4 if ev_dispatch else 1))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(0, args.steps, ev_every)]
    if ev_dispatch:  # torch creates an event's HIP handle at its first record: create them now
        for e0, e1 in evs:
            e0.record(stream)
            e1.record(stream)
        torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i % ev_every == 0:
            step(*evs[i // ev_every])
        else:
            step()
    drain()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")
    if dist_on:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if dist_on:
        kt = torch.tensor([kern_ms], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
        kern_ms = float(kt.item())
    unfused_ms = None
    if args.mode == "dense" and rank == 0:
        # the same x->density work unfused: t = h W + b by the library GEMM (t written to
        # HBM), then the chain kernel over t (read back) — what the fusion replaces
        t_buf = torch.empty((B, P) if S is None else (S, B, P), dtype=torch.float32, device=dev)
        plain = ops.ChainLauncher(y, t_buf, ft, d, True, write_values=True, draws=S)

        def unfused():
            if S is None:
                torch.addmm(bd, h, Wd, out=t_buf)
            else:
                torch.baddbmm(bd[:, None, :], h, Wd, out=t_buf)
            plain.launch(sh)
    elif args.mode == "dense_grad" and rank == 0:
        # unfused: t by the library GEMM, the chain backward kernel, library GEMMs for dh / dW, db
        t_buf = torch.empty((B, P), dtype=torch.float32, device=dev)
        plain = ops.GradLauncher(y, t_buf, ft, d, True, g_out=g_up)

        def unfused():
            torch.addmm(bd, h, Wd, out=t_buf)
            plain.launch(sh)
            gt = plain.grad_t
            return gt @ Wd.t(), h.t() @ gt, gt.sum(0)
    elif args.mode == "bijector" and rank == 0:
        # the same Chain through the flow-by-flow Bijector path (one single-flow launch per
        # flow: each reads its block's cache lines of t again)
        from normalizingflownetwork_amd import InverseNormalizingFlowLayer
        from normalizingflownetwork_amd.normalizing_flows import Chain

        flows = InverseNormalizingFlowLayer._get_bijector(t[:, 2 * d:], ft, d).bijectors
        steps = Chain([type(f)(f.params, d) for f in flows])
        steps._fused = lambda x=None: None

        def unfused():
            steps.forward_and_log_det_jacobian(y)
    if (dense_mode or args.mode == "bijector") and rank == 0:
        for _ in range(3):
            unfused()
        pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for e0, e1 in pairs:
            e0.record(stream)
            unfused()
            e1.record(stream)
        torch.cuda.synchronize()
        unfused_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in pairs]))
        if dense_mode:
            del t_buf, plain
    nonfinite = None
    if grad_mode or args.mode in ("bijector", "flows", "grid"):
        mean_ll = None
    elif native is not None:
        mean_ll = float(native.mean.item())
        nonfinite = int(native.sum_count[2].item())
    elif dist_on:
        red = last_red[0]
        mean_ll = float(red[0].item()) / float(B * world)
        nonfinite = int(red[1].item())
    else:
        mean_ll = float(launcher.sum.item()) / B
        nonfinite = int(launcher.nonfinite.item())

    if rank == 0:
        total_evals = evals_per_step * world * args.steps
        value = total_evals / elapsed
        if args.mode == "grad":
            bytes_launch = algorithmic_bytes_grad(d, P, B)
        elif args.mode == "dense":
            nd = 1 if S is None else S
            bytes_launch = float(B) * (4 * H * nd + 4 * d + 4) + nd * (4.0 * H * P + 4.0 * P)
        elif args.mode == "bijector":
            # z in, the flows' blocks of t (P - 2d floats), z_K and ldj out
            bytes_launch = float(B) * (4 * d + 4 * (P - 2 * d) + 4 * d + 4)
        elif args.mode == "flows":
            # per flow: z in, its block of t, z and its ldj out (the K launches of one step)
            bytes_launch = launcher.bytes_per_launch
        elif args.mode == "grid":
            # the B parameter rows and G grid values once, the (G, B) log-densities out
            bytes_launch = float(B) * 4 * P + float(args.grid) * 4 * d + float(args.grid) * B * 4
        elif args.mode == "dense_grad":
            # h, y, upstream g in; dh, dy out; W, b read and dW, db written once per launch
            bytes_launch = float(B) * (8 * H + 8 * d + 4) + 2 * (4.0 * H * P + 4.0 * P)
        else:
            bytes_launch = algorithmic_bytes_per_launch(d, P, B, S)
        achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = load_traffic(args.config + {"grad": "_grad", "dense": "_dense", "dense_grad": "_dense_grad",
                                                           "bijector": "_bijector", "grid": "_grid",
                                                           "flows": "_flows" if args.flow_params == "views" else "_flows_" + args.flow_params
                                                           }.get(args.mode, ""), B)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline({"flows": "bijector", "grid": "forward"}.get(args.mode, args.mode), args.config, H=H,
                               seconds=args.cpu_seconds)
        wl = {
            "C2": "C2: y_dim=1, (planar,radial)x5 chain, batch 2^24 per GPU" + (" (C4 form: RCCL mean-NLL all-reduce)" if world > 1 else ""),
            "C3": "C3: y_dim=8, affine+planar x4+radial x4, batch 2^22 per GPU",
            "C5": "C5: Bayes posterior, 64 draws x 2^17 samples per GPU, y_dim=1, (planar,radial)x5",
            "C3P": "C3P: Bayes posterior, 64 draws x 2^17 samples per GPU, y_dim=3, affine+planar x4+radial x4 (P = 60)",
            "R2": "R2: y_dim=1, (radial,radial) chain (configs[0]'s flows at C2's batch; not SURVEY's C1, which is B = 4096 CPU plumbing), batch 2^24 per GPU",
            "R10": "R10: y_dim=1, radial x 10 (NormalizingFlowNetwork's default), batch 2^24 per GPU",
        }[args.config]
        if args.mode == "grad":
            kernel_name = "chain_grad_wave_kernel" if d <= 2 else "chain_grad_group1_kernel"
            metric = f"log_prob backward evals/sec (whole node), {args.config}"
        elif args.mode == "dense_grad":
            # dispatch-recorded events time the step's first launch; markers bracket both
            kernel_name = ("chain_dense1_grad_sb_kernel" if d == 1 and H == 16 and P <= 32 and args.math == "fast"
                           else "chain_dense1_grad_kernel" if d == 1 and H in (16, 32) and args.math == "fast"
                           else "chain_dense_grad_kernel") + \
                ("" if ev_dispatch else " + sum_partials_kernel")
            metric = f"Dense(H={H})->log_prob backward evals/sec (whole node), {args.config}"
        elif args.mode == "bijector":
            kernel_name = "chain_wave1_kernel (Chain bijector form)" if d == 1 else "chain_fwd_ldj_kernel"
            metric = f"Chain bijector forward+fldj evals/sec (whole node), {args.config}"
        elif args.mode == "flows":
            kernel_name = (f"flow_fwd_ldj_kernel x {len(ft)} launches"
                           + (" after split_blocks_kernel" if getattr(launcher, "_split", None) is not None else ""))
            metric = f"flow-by-flow bijector forward+fldj chain evals/sec (whole node), {args.config}"
        elif args.mode == "grid":
            kernel_name = "chain_grid_kernel"
            metric = f"density-grid log_prob evals/sec (whole node), {args.config} (G={args.grid} grid values x B rows)"
        elif args.mode == "dense":
            if S is None:
                kernel_name = "chain_dense1_kernel" if d == 1 else "chain_dense_kernel"
                metric = f"Dense(H={H})->log_prob evals/sec (whole node), {args.config}"
            else:
                kernel_name = ("posterior_dense1_kernel" if d == 1 else
                               "posterior_densep_kernel" if (H <= 16 and args.math == "fast") else "posterior_dense_kernel")
                metric = f"DenseVariational(H={H})->posterior (draw, sample) evals/sec (whole node), {args.config}"
        else:
            kernel_name = {"C2": "chain_wave1_kernel", "C3": "chain_group1_kernel", "R2": "chain_wave1_kernel",
                           "R10": "chain_wave1_kernel", "C5": "posterior_wave1_kernel",
                           "C3P": "chain_persistent_kernel (posterior)"}[args.config]
            metric = ("log_prob evals/sec (whole node), 10-flow planar+radial chain, y_dim=1"
                      if args.config == "C2" else f"log_prob evals/sec (whole node), {args.config}")
        line = {
            "metric": metric,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "pg_world_size": pg_world,
            "rank_devices": rank_devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm": {"ms": args.prewarm_ms, "steps": prewarm_steps},
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic N(0,1) y and per-sample flow params t, generated on device (seed 22+rank)",
            "config": {
                "workload": wl,
                "batch_per_gpu": B,
                "global_batch": B * world,
                "draws": S,
                "y_dim": d,
                "flows": list(ft),
                "param_width": P,
                "hidden": H if dense_mode else None,
                "trainable_base": True,
                "math": args.math,
                "parallelism": f"dp{world}",
                "allreduce": None if (world == 1 or grad_mode) else args.allreduce,
                "mode": args.mode,
                **({"flow_params": args.flow_params} if args.mode == "flows" else {}),
                **({"grid": args.grid} if args.mode == "grid" else {}),
            },
            "roofline": {
                **({"note": "compute-bound: the parameter rows are read once for all G grid values, so the "
                            "HBM fraction is small by construction; DESIGN.md compares the evals/s with the "
                            "C2 forward's compute-only rate"} if args.mode == "grid" else {}),
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kernel_name,
                "kernel_ms": kern_ms,
                "kernel_ms_launches": len(evs),
                "kernel_events": "dispatch" if ev_dispatch else "marker",
                "algorithmic_bytes_per_launch": bytes_launch,
                "traffic_source": traffic_src,
            },
            "cpu_baseline": cpu,
            # fused Dense modes: the fp32 GEMM work per launch (t = hW, and for the backward
            # dh = dt W^T, dW = h^T dt) in algorithmic fp32 FLOPs against the 157.3 TF/s fp32
            # matrix peak; at H = 16, P <= 32 (d = 1, fast math) the kernels run t (forward) and
            # dh, dW (backward) as exact 3-way split-bf16 products on v_mfma_f32_16x16x32_bf16
            "mfma": None if not dense_mode else {
                "tflops": (3 if grad_mode else 1) * 2.0 * B * H * P * (1 if S is None else S) / (kern_ms * 1e-3) / 1e12,
                "peak": 157.3,
                "gemm_form": ("split-bf16 (t f32 MFMA in the backward)" if grad_mode else "split-bf16 t")
                if (H == 16 and P <= 32 and d == 1 and S is None and args.math == "fast") else "f32 MFMA"},
            "mean_log_prob": mean_ll,
            "nonfinite_log_prob": nonfinite,
            "unfused_ms": unfused_ms,
            "nfn_env": nfn_env,
            **({"library": "libnfn_hip_diag.so (--diag: A/B study, not a reported line)"} if args.diag else {}),
        }
        print(json.dumps(line), flush=True)
    if native is not None:
        native.close()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
