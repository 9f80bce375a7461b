"""How many 1-ulp input perturbations the parity gate's fp32 sensitivity needs (oracle only).

The forward parity gate (``tests/parity.py``) widens a sample's bound past 1e-5 relative
only to ``WIDEN_CAP x S32``, where S32 is the largest deviation from the fp64 truth of the
oracle's op-by-op fp32 mirror of the reference (TF eager's order) over the run at the inputs
and ``n`` runs at random 1-ulp perturbations of them (``oracle.fp32_spread``).  This study
takes the samples a full-batch GPU run put beyond 1e-5 (the dumps of
``tests/test_gpu_fullbatch.py``: ``profiles/r03/r03n_fullbatch_C{2,4}_worst.npz`` hold the
256 worst samples by error / 1e-5 bound, with the kernel's value) and evaluates S32 as a
function of ``n`` over one fixed random sequence (a running max, so S32(n) is monotone):

* ``S32(n) / S32(n_max)``: how far the estimate has converged at ``n``;
* how many of the samples would pass ``err <= 2 S32(n)``.

The gate's count is chosen from where the curve flattens, never from the kernel's error.

  python tools/perturbation_study.py profiles/r03/r03n_fullbatch_C2_worst.npz [...]
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import nfn_oracle as O  # noqa: E402

NS = [0, 4, 16, 64, 256, 1024]
FLOWS = ("planar", "radial") * 5


def spread_curve(y, t, ns, seed=0):
    """S32 after each n in ``ns`` (one random sequence): (len(ns), n_samples)."""
    ref64 = O.log_pdf(y, t, FLOWS, 1, True, None, None, np.float64)
    rng = np.random.default_rng(seed)
    y32, t32 = np.asarray(y, np.float32), np.asarray(t, np.float32)
    spread = np.zeros_like(ref64)
    out = []
    for k in range(max(ns) + 1):
        if k == 0:
            yk, tk = y32, t32
        else:
            yk = (y32 * (1 + rng.integers(-1, 2, y32.shape) * 2.0 ** -23)).astype(np.float32)
            tk = (t32 * (1 + rng.integers(-1, 2, t32.shape) * 2.0 ** -23)).astype(np.float32)
        with np.errstate(all="ignore"):
            r32 = O.log_pdf(yk, tk, FLOWS, 1, True, None, None, np.float32)
        spread = np.maximum(spread, np.abs(r32.astype(np.float64) - ref64))
        if k in ns:
            out.append(spread.copy())
    return ref64, np.array(out)


def main():
    for path in sys.argv[1:]:
        dump = np.load(path)
        got, r64 = dump["got"].astype(np.float64), dump["ref64"].astype(np.float64)
        base = 1e-5 * np.maximum(1.0, np.abs(r64))
        err = np.abs(got - r64)
        sel = err > base
        y, t = dump["y"][sel], dump["t"][sel]
        ref64, curve = spread_curve(y, t, NS)
        assert np.allclose(ref64, r64[sel], rtol=0, atol=1e-12)
        e = err[sel]
        print(f"{path}: {int(sel.sum())} samples beyond 1e-5 relative (of the {sel.size} dumped)")
        print("   n   median S32(n)/S32(1024)  min S32(n)/S32(1024)  pass err<=2*S32(n)  max err/(2*S32(n))")
        for n, s in zip(NS, curve):
            r = s / curve[-1]
            print(f"{n:5d}   {np.median(r):22.3f}  {np.min(r):20.3f}  {int((e <= 2 * s).sum()):10d} / {e.size:<5d}"
                  f"  {np.max(e / (2 * s)):16.3f}")
        for seed in (1, 2):
            _, c2 = spread_curve(y, t, [64, 1024], seed=seed)
            print(f"  seed {seed}: S32(64)/S32(1024) median {np.median(c2[0] / c2[1]):.3f}, "
                  f"S32(1024, seed {seed}) / S32(1024, seed 0) median {np.median(c2[1] / curve[-1]):.3f}; "
                  f"pass at 64: {int((e <= 2 * c2[0]).sum())}, at 1024: {int((e <= 2 * c2[1]).sum())}")


if __name__ == "__main__":
    main()
