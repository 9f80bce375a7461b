"""Where the fused d = 1 kernel's error on its worst full-batch samples comes from.

Replays the worst samples of a full-batch parity run (``tests/test_gpu_fullbatch.py``
dumps, e.g. ``profiles/r03/r03n_fullbatch_C4_worst.npz``) through an fp64 evaluation of
the kernel's own forms (``planar1_fast`` / ``radial1_fast`` / ``base1_fast`` in
``csrc/nfn_device.h``), with fp32-sized rounding noise injected at one group of
intermediates at a time: x -> x (1 + k eps u), eps = 2^-24, u ~ U(-1, 1), k = 1 for a
rounded arithmetic result, 2 for v_exp/v_log/v_rcp, 3 for tanh_fast.  The max over 64
noise draws per sample is printed beside the kernel's measured error
(|got - ref64| / max(1, |ref64|)).  Groups:

  pw   w = 1 + w_raw          pwtu  w u                psp  softplus(w u)
  pm   m = sp - (1 - 1e-5)    prn   w^2 + 1e-9, 1/.    puh  u_hat
  ts   s = w z + b            tt    tanh(s)            z    the z update
  det  the planar / radial det terms   log  log|det|   sum  the running sum
  rad  radial |z - g|, h      base  the base density   all  every group at once

  python tools/error_attribution.py profiles/r03/r03n_fullbatch_C4_worst.npz [n]
"""

import sys

import numpy as np

EPS = 2.0 ** -24
GROUPS = ["pw", "pwtu", "psp", "pm", "prn", "puh", "ts", "tt", "z", "det", "log", "sum", "rad", "base"]
_active = set()
_rng = np.random.default_rng(0)


def _n(x, g, k=1.0):
    if g not in _active:
        return x
    return x * (1 + k * EPS * _rng.uniform(-1, 1, size=np.shape(x)))


def _sp(x):
    return np.logaddexp(0.0, x)


def chain1(y, t, flow_types):
    """d = 1, trainable base, the layer's reversed layout [base 2 | f_{K-1} .. f_0]."""
    z = y[:, 0].astype(np.float64)
    il = np.zeros_like(z)
    off = t.shape[1]
    for f in flow_types:
        off -= 3
        p = t[:, off:off + 3].astype(np.float64)
        if f == "planar":
            u, w, b = p[:, 0], _n(p[:, 1] + 1, "pw"), p[:, 2]
            wtu = _n(w * u, "pwtu")
            sp = _n(_sp(wtu), "psp", 2)
            m = _n(sp - (1 - 1e-5), "pm")
            nw2 = _n(w * w + 1e-9, "prn")
            rn = _n(1 / nw2, "prn", 2)
            uh = _n(_n(u * 1e-9 + m * w, "puh") * rn, "puh")
            th = _n(np.tanh(_n(w * z + b, "ts")), "tt", 3)
            qd = _n(_n(sp + 1e-5, "det") - _n((m - wtu) * 1e-9 * rn, "det"), "det")
            det = _n(th * th + _n(1 - th * th, "det") * qd, "det")
            il = _n(il + _n(np.log(np.abs(det)), "log", 2), "sum")
            z = _n(z + _n(uh * th, "z"), "z")
        elif f == "radial":
            al = _n(_sp(0.3 * p[:, 0] - 2), "rad", 2)
            ab = _n(al * _sp(0.1 * p[:, 1] + np.log(np.e - 1)) - al, "rad")
            dz = _n(z - p[:, 2], "rad")
            h = _n(1 / _n(al + np.abs(dz), "rad"), "rad", 2)
            det = _n(1 + _n(_n(ab * h, "det") * _n(al * h, "det"), "det"), "det")
            il = _n(il + _n(np.log(det), "log", 2), "sum")
            z = _n(z + _n(_n(ab * h, "z") * dz, "z"), "z")
        else:
            raise ValueError("d = 1 planar / radial chains only")
    loc = t[:, 0].astype(np.float64)
    scale = 1e-3 + _sp(0.1 * t[:, 1].astype(np.float64) + np.log(np.e - 1))
    zz = _n(_n(z - loc, "base") / scale, "base")
    return -0.5 * zz * zz - 0.5 * np.log(2 * np.pi) - np.log(scale) + il


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dump = np.load(path)
    y, t, r64, got = dump["y"][:n], dump["t"][:n], dump["ref64"][:n], dump["got"][:n]
    flow_types = ("planar", "radial") * 5
    den = np.maximum(1.0, np.abs(r64))
    _active.clear()
    print(f"{path}: noise-free fp64 kernel forms vs the oracle's ref64: "
          f"{np.max(np.abs(chain1(y, t, flow_types) - r64) / den):.2e}")
    res = {}
    for g in GROUPS + ["all"]:
        _active.clear()
        _active.update(GROUPS if g == "all" else [g])
        res[g] = np.max([np.abs(chain1(y, t, flow_types) - r64) / den for _ in range(64)], axis=0)
    ref32 = np.abs(dump["ref32"][:n] - r64) / den
    print("kernel    ref32     " + "".join(f"{g:>9}" for g in GROUPS + ["all"]))
    for i in range(n):
        print(f"{abs(got[i] - r64[i]) / den[i]:.2e}  {ref32[i]:.2e}  " + "".join(f"{res[g][i]:9.1e}" for g in GROUPS + ["all"]))
    print("median over the samples of (group max / kernel error):")
    kerr = np.abs(got - r64) / den
    print("  " + "  ".join(f"{g} {np.median(res[g] / kerr):.2f}" for g in GROUPS + ["all"]))


if __name__ == "__main__":
    main()
