"""Parity over EVERY sample at the BASELINE sizes (BASELINE.json configs C2, C3, C5).

The fp64 oracle (and its op-by-op fp32 mirror for the conditioning term of the bound) runs
over the whole batch in 2^20-row chunks on the host, on threads (numpy releases the GIL
inside its array loops); every finite sample must be within ``oracle.tolerance_bound`` and
every non-finite one must be non-finite on the GPU too (``tests/parity.py``).  The records
(``n`` = the full batch, max err / bound) go to ``gpurun_out/parity.json``.

* C2: d = 1, (planar, radial) x 5, B = 2^24 (``DistributionLayers.py:245-255``)
* C3: d = 8, affine + planar x 4 + radial x 4, B = 2^22
* C4: C2's chain at the 8-GPU global batch, B = 2^27, on one device
* C5: the Bayesian posterior score at its GLOBAL size, S = 64 draws x B = 2^20 samples on
  one GPU (t is 8.6 GB) (``BayesianNNEstimator.py:65-76``, ``scorers.py:13-27``)
"""

import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import nfn_oracle as O
from parity import check_forward, fp32_sensitivity

pytestmark = pytest.mark.gpu

CHUNK = 1 << 20
THREADS = 8
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dump_worst(name, got, r64, r32, rows, n=256):
    """The n samples with the largest error / bound, with their input rows (the evidence
    for profiles/ and for tools/eval_rows.py, which replays them through any library build)."""
    with np.errstate(all="ignore"):
        ratio = np.abs(got - r64) / O.tolerance_bound(r64, r32)
    ratio = np.where(np.isfinite(ratio), ratio, -1.0)
    idx = np.argsort(ratio)[::-1][:n]
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    np.savez_compressed(os.path.join(out, f"fullbatch_{name}_worst.npz"), idx=idx, got=got[idx], ref64=r64[idx],
                        ref32=r32[idx], ratio=ratio[idx], **{k: v(idx) for k, v in rows.items()})


def _chunked(fn, n, chunk=CHUNK):
    """fn(lo, hi) -> (ref64, ref32) over [0, n) in chunks on a thread pool."""
    spans = [(lo, min(n, lo + chunk)) for lo in range(0, n, chunk)]
    t0 = time.time()
    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        parts = list(ex.map(lambda s: fn(*s), spans))
    print(f"  oracle over {n} samples in {len(spans)} chunks: {time.time() - t0:.1f} s", flush=True)
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4"])
def test_full_batch_parity(cfg, gpu):
    """C4 is C2's chain at the 8-GPU global batch (2^27) on ONE device: t is 16 GiB, the call
    runs as eight 2^24-sample chunk launches with one fused sum (include/nfn.h)."""
    from normalizingflownetwork_amd import ops

    ft, d, B = {"C2": (("planar", "radial") * 5, 1, 1 << 24),
                "C3": (("affine",) + ("planar",) * 4 + ("radial",) * 4, 8, 1 << 22),
                "C4": (("planar", "radial") * 5, 1, 1 << 27)}[cfg]
    P = O.total_param_size(ft, d, True)
    gen = torch.Generator(device="cuda").manual_seed(22)
    y = torch.randn((B, d), generator=gen, device="cuda")
    t = torch.randn((B, P), generator=gen, device="cuda")
    lp, s = ops.chain_log_prob(y, t, ft, d, True, want_sum=True)
    got = lp.cpu().numpy()
    yh, th = y.cpu().numpy(), t.cpu().numpy()
    del y, t

    def ref(lo, hi):
        with np.errstate(all="ignore"):
            return (O.chain_log_prob(yh[lo:hi], th[lo:hi], ft, d, True, np.float64),
                    O.chain_log_prob(yh[lo:hi], th[lo:hi], ft, d, True, np.float32))

    r64, r32 = _chunked(ref, B)
    _dump_worst(cfg, got, r64, r32, {"y": lambda i: yh[i], "t": lambda i: th[i]})
    m = check_forward(got, r64, r32, f"{cfg} full batch (B={B})", nonfinite="match", kind="full_batch",
                      sensitivity=fp32_sensitivity(yh, th, ft, d, True))
    print(f"  {cfg}: max |err| / max(1, |ref|) = {m:.3g}", flush=True)
    fin = np.isfinite(got)
    if fin.all():
        assert float(s.item()) == pytest.approx(got.astype(np.float64).sum(), rel=1e-12)
    torch.cuda.empty_cache()


def test_c5_global_posterior_parity(gpu):
    """C5 at its global size on ONE device: S = 64 draws x B = 2^20, every sample's
    logsumexp score against the oracle."""
    from normalizingflownetwork_amd import ops

    ft, S, B = ("planar", "radial") * 5, 64, 1 << 20
    P = O.total_param_size(ft, 1, True)
    gen = torch.Generator(device="cuda").manual_seed(5)
    y = torch.randn((B, 1), generator=gen, device="cuda")
    t = torch.randn((S, B, P), generator=gen, device="cuda")
    out, s = ops.posterior_lse(y, t, ft, 1, True, want_sum=True)
    got = out.cpu().numpy()
    yh = y.cpu().numpy()
    chunk = 1 << 16
    # host copies per sample chunk (all draws of those samples), 8 MB x S each
    th = [t[:, lo:lo + chunk].cpu().numpy() for lo in range(0, B, chunk)]
    del t
    torch.cuda.empty_cache()

    def ref(lo, hi):
        tc = th[lo // chunk]
        with np.errstate(all="ignore"):
            return (O.posterior_lse(yh[lo:hi], tc, ft, 1, True, dtype=np.float64),
                    O.posterior_lse(yh[lo:hi], tc, ft, 1, True, dtype=np.float32))

    r64, r32 = _chunked(ref, B, chunk)
    _dump_worst("C5", got, r64, r32, {"y": lambda i: yh[i],
                                      "t": lambda i: np.stack([th[j // chunk][:, j % chunk] for j in i], axis=1)})
    def sens(idx):
        tt = np.stack([th[j // chunk][:, j % chunk] for j in idx], axis=1)
        return fp32_sensitivity(yh[idx], tt, ft, 1, True, posterior=True)(np.arange(len(idx)))

    m = check_forward(got, r64, r32, f"C5 global posterior (S={S}, B={B})", nonfinite="match", kind="full_batch",
                      sensitivity=sens)
    print(f"  C5: max |err| / max(1, |ref|) = {m:.3g}", flush=True)
    if np.isfinite(got).all():
        assert float(s.item()) == pytest.approx(got.astype(np.float64).sum(), rel=1e-12)
