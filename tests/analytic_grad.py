"""Closed-form backward of the flow chain in numpy — the derivation the HIP
gradient kernels implement, checked on the CPU against the autodiff oracle
(tests/test_grad_oracle.py::test_closed_form_backward).  Test helper."""

import math

import numpy as np

from oracle import nfn_oracle as O

C_BASE = math.log(math.expm1(1.0))


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def _sp(x):
    return np.maximum(x, 0) + np.log1p(np.exp(-np.abs(x)))


def chain_grad(y, t, ft, d, tr, y_mean=None, y_std=None, dtype=np.float64):
    y = np.asarray(y, dtype)
    t = np.asarray(t, dtype)
    B = max(len(y), len(t))
    z = np.broadcast_to(y, (B, d)).copy()
    t = np.broadcast_to(t, (B, t.shape[1]))
    if y_mean is not None:
        z = (z - y_mean) / y_std
    o = 2 * d if tr else 0
    offs, off = [], t.shape[1]
    for f in ft:  # blocks in reverse application order: off_0 = P - size(f_0)
        off -= O.param_size(f, d)
        offs.append(off)
    assert off == o
    zs, lp = [], np.zeros(B)
    for f, of in zip(ft, offs):
        zs.append(z.copy())
        z, l = O.flow_forward_fldj(f, z, t[:, of:of + O.param_size(f, d)], d)
        lp += l
    gt = np.zeros_like(t)
    if tr:
        loc, ts = t[:, :d], t[:, d:2 * d]
        scale = 1e-3 + _sp(C_BASE + 0.1 * ts)
        zz = (z - loc) / scale
        lp += -0.5 * (zz ** 2).sum(1) - 0.5 * d * math.log(2 * math.pi) - np.log(scale).sum(1)
        a = -zz / scale
        gt[:, :d] = zz / scale
        gt[:, d:2 * d] = 0.1 * _sig(C_BASE + 0.1 * ts) * (zz ** 2 - 1) / scale
    else:
        lp += -0.5 * (z ** 2).sum(1) - 0.5 * d * math.log(2 * math.pi)
        a = -z
    for f, of, z in reversed(list(zip(ft, offs, zs))):
        p = t[:, of:of + O.param_size(f, d)]
        if f == "planar":
            u, w, b = p[:, :d], p[:, d:2 * d] + 1.0, p[:, 2 * d]
            wtu = (w * u).sum(1)
            sg = _sig(wtu)
            m = -1.0 + _sp(wtu) + 1e-5
            c = m - wtu
            n = (w * w).sum(1) + 1e-9
            uh = u + (c / n)[:, None] * w
            s = (w * z).sum(1) + b
            h = np.tanh(s)
            E = np.exp(-2 * np.abs(s))
            hp = 4 * E / ((1 + E) * (1 + E))  # 1 - tanh^2 without cancellation
            q = m - c * (1e-9 / n)  # = w.u_hat exactly, without the d-term cancellation
            det = 1 + hp * q
            Ss = hp * (uh * a).sum(1) + q * (-2 * h * hp) / det
            G = h[:, None] * a + (hp / det)[:, None] * w
            wG = (w * G).sum(1)
            k1 = (sg - 1) * wG / n
            if d == 1:  # G - (1 - sg) (wG/n) w = G (1e-9 + sg w^2) / n exactly: no cancellation
                gt[:, of:of + d] = G * ((1e-9 + sg * w[:, 0] ** 2) / n)[:, None]
            else:
                gt[:, of:of + d] = G + k1[:, None] * w
            gt[:, of + d:of + 2 * d] = (z * Ss[:, None] + (hp / det)[:, None] * uh + (c / n)[:, None] * G
                                        - (2 * c * wG / n ** 2)[:, None] * w + k1[:, None] * u)
            gt[:, of + 2 * d] = Ss
            a = a + w * Ss[:, None]
        elif f == "radial":
            x_a, x_b = 0.3 * p[:, 0] - 2.0, 0.1 * p[:, 1] + C_BASE
            al, be = _sp(x_a), _sp(x_b) - 1.0
            g = p[:, 2:2 + d]
            dz = z - g
            r = np.abs(dz).sum(1)
            sgn = np.sign(dz)
            h = 1.0 / (al + r)
            ab = al * be
            A = 1 + ab * h
            Bv = 1 + ab * al * h * h
            da = (dz * a).sum(1)
            H = ab * da + (d - 1) * ab / A + 2 * ab * al * h / Bv
            g_ab = h * da + (d - 1) * h / A + al * h * h / Bv
            g_al = be * g_ab + ab * h * h / Bv - h * h * H
            gt[:, of] = 0.3 * _sig(x_a) * g_al
            gt[:, of + 1] = 0.1 * _sig(x_b) * al * g_ab
            gt[:, of + 2:of + 2 + d] = -(ab * h)[:, None] * a + (h * h * H)[:, None] * sgn
            a = A[:, None] * a - (h * h * H)[:, None] * sgn
        else:
            sc = 1.0 + p[:, d:2 * d]
            gt[:, of:of + d] = a
            gt[:, of + d:of + 2 * d] = z * a + 1.0 / sc
            a = sc * a
    gy = a / y_std if y_mean is not None else a
    if y_mean is not None:
        lp -= np.log(y_std).sum()
    return lp, gt, gy
