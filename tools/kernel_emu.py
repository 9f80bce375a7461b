"""fp32 emulation of the fused d = 1 chain kernel's arithmetic (``csrc/nfn_device.h``:
``planar1_fast``, ``radial1_fast``, ``base1_fast``, the log2-domain sum), op by op in
numpy float32 (fma: one rounding of the exact fp64 product-sum; ``v_exp_f32`` /
``v_log_f32`` / ``v_rcp_f32``: the correctly rounded fp32 value, optionally moved by
up to ``hw_ulp`` ulp at random — the hardware's documented ~1-ulp accuracy).

A design tool (not test infrastructure): candidate forms of the planar / radial steps are
compared here by their error against the fp64 oracle on the samples a GPU run found worst
(``tests/test_gpu_fullbatch.py`` dumps) and on random batches, before they are written as
HIP.  ``FORMS`` names the variants; ``python tools/kernel_emu.py <dump.npz> ...`` prints the
error statistics of each.
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

F = np.float32
LOG2E = F(1.4426950408889634)
LN2 = F(0.6931471805599453)
LOGEXPM1ONE = F(np.log(np.expm1(1.0)))
HALFLOG2PI = F(0.5 * np.log(2 * np.pi))
_rng = np.random.default_rng(0)
HW_ULP = [0.0]


def r32(x):
    return np.asarray(x, np.float64).astype(F)


def fma(a, b, c):
    return r32(np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64))


def _hw(x64):
    x = r32(x64)
    if HW_ULP[0]:
        k = np.rint(_rng.uniform(-HW_ULP[0], HW_ULP[0], np.shape(x))).astype(np.int32)
        x = np.nextafter(x, np.where(k > 0, F(np.inf), F(-np.inf))) if True else x
        x = np.where(k == 0, r32(x64), x)
    return x


def exp2(x):
    return _hw(np.exp2(np.asarray(x, np.float64)))


def log2(x):
    with np.errstate(divide="ignore", invalid="ignore"):
        return _hw(np.log2(np.asarray(x, np.float64)))


def rcp(x):
    with np.errstate(divide="ignore"):
        return _hw(1.0 / np.asarray(x, np.float64))


# ----------------------------------------------------------------------------- round-3 forms
def softplus_alpha(x):
    e = exp2(F(-np.abs(x)) * LOG2E)
    u = F(1) + e
    c = e - (u - F(1))
    return fma(log2(u), LN2, np.maximum(x, F(0)) + c)


def sp_fast1(x):
    e = exp2(F(-np.abs(x)) * LOG2E)
    return fma(log2(F(1) + e), LN2, np.maximum(x, F(0)))


def tanh_r3(a):
    E = exp2(a * F(2 * 1.4426950408889634))
    te = F(1) - rcp(fma(E, F(0.5), F(0.5)))
    a2 = a * a
    p = fma(a2, F(62 / 2835), F(-17 / 315))
    p = fma(a2, p, F(2 / 15))
    p = fma(a2, p, F(-1 / 3))
    tp = fma(a * a2, p, a)
    return np.where(np.abs(a) < F(0.3), tp, te)


ONE_M = F(1) - F(1e-5)


def planar_r3(z, u, wraw, b, tanh=tanh_r3):
    w = wraw + F(1)
    wtu = w * u
    nw2 = fma(w, w, F(1e-9))
    rn = rcp(nw2)
    sp = softplus_alpha(wtu)
    m = sp - ONE_M
    uh = fma(u, F(1e-9), m * w) * rn
    qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
    th = tanh(fma(w, z, b))
    z = fma(uh, th, z)
    return z, fma(th, th, fma(-th, th, F(1)) * qd)


def radial_r3(z, a0, b0, g):
    alpha = softplus_alpha(fma(F(0.3), a0, F(-2)))
    ab = fma(alpha, sp_fast1(fma(F(0.1), b0, LOGEXPM1ONE)), -alpha)
    dz = z - g
    h = rcp(alpha + np.abs(dz))
    abh = ab * h
    z = fma(abh, dz, z)
    return z, fma(abh, alpha * h, F(1))


def base_r3(z, t):
    sc = F(1e-3) + sp_fast1(LOGEXPM1ONE + F(0.1) * t[:, 1])
    zz = (z - t[:, 0]) * rcp(sc)
    return F(-0.5) * (zz * zz) - (HALFLOG2PI + log2(sc) * LN2)


FORMS = {"r3": (planar_r3, radial_r3, base_r3)}


def chain(y, t, flow_types=("planar", "radial") * 5, form="r3"):
    planar, radial, base = FORMS[form]
    t = np.asarray(t, F)
    z = np.asarray(y, F)[:, 0].copy()
    l2 = np.zeros_like(z)
    off = t.shape[1]
    for f in flow_types:
        off -= 3
        p = t[:, off:off + 3]
        z, det = (planar if f == "planar" else radial)(z, p[:, 0], p[:, 1], p[:, 2])
        l2 = l2 + log2(np.abs(det))
    return base(z, t) + l2 * LN2


def main():
    from oracle import nfn_oracle as O

    forms = [f for f in sys.argv[1:] if f in FORMS] or list(FORMS)
    paths = [p for p in sys.argv[1:] if p not in FORMS]
    for path in paths:
        d = np.load(path)
        y, t, r64, got = d["y"], d["t"], d["ref64"].astype(np.float64), d["got"].astype(np.float64)
        den = np.maximum(1.0, np.abs(r64))
        print(f"{path}: {len(r64)} samples; GPU max rel {np.max(np.abs(got - r64) / den):.3e}, "
              f"beyond 1e-5: {int((np.abs(got - r64) > 1e-5 * den).sum())}")
        for form in forms:
            for hw in (0.0, 1.0):
                HW_ULP[0] = hw
                e = np.abs(chain(y, t, form=form).astype(np.float64) - r64) / den
                extra = ""
                if form == "r3" and hw == 0.0:
                    g = chain(y, t, form=form).astype(np.float64)
                    extra = f"  (emu vs GPU: bitwise {int((g == got).sum())}, max |d|/den {np.max(np.abs(g - got) / den):.2e})"
                print(f"  {form:10s} hw_ulp={hw:.0f}: max {e.max():.3e} median {np.median(e):.3e} "
                      f"beyond 1e-5 {int((e > 1e-5).sum())}{extra}")
    HW_ULP[0] = 0.0
    rng = np.random.default_rng(22)
    B = 1 << 20
    y = rng.standard_normal((B, 1)).astype(F)
    t = rng.standard_normal((B, 32)).astype(F)
    r64 = O.log_pdf(y, t, ("planar", "radial") * 5, 1, True, None, None, np.float64)
    den = np.maximum(1.0, np.abs(r64))
    with np.errstate(all="ignore"):
        r32_ = O.log_pdf(y, t, ("planar", "radial") * 5, 1, True, None, None, np.float32).astype(np.float64)
    e32 = np.abs(r32_ - r64) / den
    print(f"random C2-shaped batch (2^20, seed 22): reference fp32 mirror max {e32.max():.3e}, "
          f"beyond 1e-5 {int((e32 > 1e-5).sum())}, beyond 3e-6 {int((e32 > 3e-6).sum())}")
    for form in forms:
        for hw in (0.0, 1.0):
            HW_ULP[0] = hw
            e = np.abs(chain(y, t, form=form).astype(np.float64) - r64) / den
            print(f"  {form:10s} hw_ulp={hw:.0f}: max {e.max():.3e} beyond 1e-5 {int((e > 1e-5).sum())} "
                  f"beyond 3e-6 {int((e > 3e-6).sum())} beyond 1e-6 {int((e > 1e-6).sum())}")



# ----------------------------------------------------------------------------- candidates
def tanh_exact(a):
    return r32(np.tanh(np.asarray(a, np.float64)))


def make_planar(m_direct=False, rn_newton=False, tanh=tanh_r3, w_comp=False, uh_div=False):
    def planar(z, u, wraw, b):
        w = wraw + F(1)
        if w_comp:  # w's rounding error, exact (|wraw| < 2: Fast2Sum with 1 the larger; else with wraw)
            wl = np.where(np.abs(wraw) < F(2), (F(1) - w) + wraw, (wraw - w) + F(1))
            wtu = fma(w, u, wl * u)
        else:
            wl = F(0)
            wtu = w * u
        nw2 = fma(w, w, F(1e-9))
        rn = rcp(nw2)
        if rn_newton:
            rn = fma(fma(-nw2, rn, F(1)), rn, rn)
        x = wtu
        e = exp2(F(-np.abs(x)) * LOG2E)
        uu = F(1) + e
        c = e - (uu - F(1))
        L = log2(uu)
        sp = fma(L, LN2, np.maximum(x, F(0)) + c)
        if m_direct:
            m = fma(L, LN2, (np.maximum(x, F(0)) - F(1)) + c) + F(1e-5)
        else:
            m = sp - ONE_M
        num = fma(u, F(1e-9), m * w)
        uh = num * rn
        if uh_div:
            uh = fma(fma(-nw2, uh, num), rn, uh)
        qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
        s = fma(w, z, b)
        if w_comp:
            s = fma(wl, z, s)
        th = tanh(s)
        z = fma(uh, th, z)
        return z, fma(th, th, fma(-th, th, F(1)) * qd)
    return planar


FORMS["m"] = (make_planar(m_direct=True), radial_r3, base_r3)
FORMS["rn"] = (make_planar(rn_newton=True), radial_r3, base_r3)
FORMS["uhdiv"] = (make_planar(uh_div=True), radial_r3, base_r3)
FORMS["tanhx"] = (make_planar(tanh=tanh_exact), radial_r3, base_r3)
FORMS["wc"] = (make_planar(w_comp=True), radial_r3, base_r3)
FORMS["m+rn"] = (make_planar(m_direct=True, rn_newton=True), radial_r3, base_r3)
FORMS["m+uhdiv"] = (make_planar(m_direct=True, uh_div=True), radial_r3, base_r3)
FORMS["m+uhdiv+tx"] = (make_planar(m_direct=True, uh_div=True, tanh=tanh_exact), radial_r3, base_r3)
FORMS["all"] = (make_planar(m_direct=True, uh_div=True, tanh=tanh_exact, w_comp=True), radial_r3, base_r3)



def tanh_acc(a):
    """poly below |a| = 0.3; above it (1 - E) / (1 + E), E = e^{-2|a|} (no overflow), the
    quotient Newton-refined, the sign copied back."""
    x = np.abs(a)
    E = exp2(x * F(-2 * 1.4426950408889634))
    n = F(1) - E
    d = F(1) + E
    r = rcp(d)
    q = n * r
    q = fma(fma(-d, q, n), r, q)
    te = np.copysign(q, a)
    a2 = a * a
    p = fma(a2, F(62 / 2835), F(-17 / 315))
    p = fma(a2, p, F(2 / 15))
    p = fma(a2, p, F(-1 / 3))
    tp = fma(a * a2, p, a)
    return np.where(x < F(0.3), tp, te)


def radial_beta(z, a0, b0, g):
    alpha = softplus_alpha(fma(F(0.3), a0, F(-2)))
    x = fma(F(0.1), b0, LOGEXPM1ONE)
    e = exp2(F(-np.abs(x)) * LOG2E)
    uu = F(1) + e
    c = e - (uu - F(1))
    beta = fma(log2(uu), LN2, (np.maximum(x, F(0)) - F(1)) + c)
    ab = alpha * beta
    dz = z - g
    h = rcp(alpha + np.abs(dz))
    abh = ab * h
    z = fma(abh, dz, z)
    return z, fma(abh, alpha * h, F(1))


def base_acc(z, t):
    sc = F(1e-3) + sp_fast1(LOGEXPM1ONE + F(0.1) * t[:, 1])
    num = z - t[:, 0]
    r = rcp(sc)
    zz = num * r
    zz = fma(fma(-sc, zz, num), r, zz)
    return F(-0.5) * (zz * zz) - (HALFLOG2PI + log2(sc) * LN2)


FORMS["tacc"] = (make_planar(tanh=tanh_acc), radial_r3, base_r3)
FORMS["beta"] = (planar_r3, radial_beta, base_r3)
FORMS["base"] = (planar_r3, radial_r3, base_acc)
FORMS["m+tacc"] = (make_planar(m_direct=True, tanh=tanh_acc), radial_r3, base_r3)
FORMS["m+ud+tacc"] = (make_planar(m_direct=True, uh_div=True, tanh=tanh_acc), radial_r3, base_r3)
FORMS["m+ud+tacc+beta"] = (make_planar(m_direct=True, uh_div=True, tanh=tanh_acc), radial_beta, base_r3)
FORMS["m+ud+tacc+b+b"] = (make_planar(m_direct=True, uh_div=True, tanh=tanh_acc), radial_beta, base_acc)
FORMS["m+ud+tx+b+b"] = (make_planar(m_direct=True, uh_div=True, tanh=tanh_exact), radial_beta, base_acc)


# candidate measured on the GPU and not shipped: the accurate m with the Newton-refined
# (1 - E) / (1 + E) tanh (profiles/r04/r04abc_accuracy_cost_ab.log: C2 +4.2 %)
FORMS["m+acc"] = (make_planar(m_direct=True, tanh=tanh_acc), radial_r3, base_r3)


# cheaper accurate tanh candidate: a minimax odd polynomial (tanh(a) / a - 1 in a^2, five
# terms, fitted on |a| <= 0.55) and, above, the round-3 exp form evaluated at |a| (its
# error is 2x larger on the negative side, where 2 / (1 + e^{2a}) > 1) with the sign
# copied back
TANH_P5 = [F(-0.3333332), F(0.13332602), F(-0.053853896), F(0.021077914), F(-0.0062827035)]


def tanh_t2(a):
    x = np.abs(a)
    E = exp2(x * F(2 * 1.4426950408889634))
    te = np.copysign(F(1) - rcp(fma(E, F(0.5), F(0.5))), a)
    a2 = a * a
    p = TANH_P5[4]
    for c in TANH_P5[3::-1]:
        p = fma(a2, p, c)
    tp = fma(a * a2, p, a)
    return np.where(x < F(0.55), tp, te)


FORMS["t2"] = (make_planar(tanh=tanh_t2), radial_r3, base_r3)
FORMS["r4"] = FORMS["t2"]  # round 4's shipped form (csrc/nfn_device.h tanh_fast)
FORMS["m+t2"] = (make_planar(m_direct=True, tanh=tanh_t2), radial_r3, base_r3)


# round 5's shipped form (csrc/nfn_device.h tanh_fast): round 4's exp form at |a| with the sign
# copied back, and a three-term polynomial on [0, 0.3] (two fma fewer than round 4's five terms)
TANH_P3 = [F(-0.33333063), F(0.13314915), F(-0.050372913)]


def tanh_t3(a):
    x = np.abs(a)
    E = exp2(x * F(2 * 1.4426950408889634))
    te = np.copysign(F(1) - rcp(fma(E, F(0.5), F(0.5))), a)
    a2 = a * a
    p = fma(a2, TANH_P3[2], TANH_P3[1])
    p = fma(a2, p, TANH_P3[0])
    tp = fma(a * a2, p, a)
    return np.where(x < F(0.3), tp, te)


FORMS["r5"] = (make_planar(tanh=tanh_t3), radial_r3, base_r3)


def make_planar_m_exact(tanh=tanh_t3):
    """Attribution experiment (not a kernel form): m = softplus(w u) - 1 + 1e-5 correctly rounded
    from the fp32 w u (fp64 evaluation), everything else as the kernel.  Round 5: 2^21 random C2
    samples beyond 3e-6 relative 206 -> 56, beyond 1e-5 5 -> 1; a one-ulp error on that m
    already gives 170 — the z-path error floor is the fp32 softplus, which only an evaluation
    beyond fp32 (double-float exp / log) could lower."""
    base = make_planar(tanh=tanh)

    def planar(z, u, wraw, b):
        w = wraw + F(1)
        wtu = w * u
        sp64 = np.logaddexp(0.0, np.asarray(wtu, np.float64))
        m = r32(sp64 - (1.0 - 1e-5))
        sp = r32(sp64)
        nw2 = fma(w, w, F(1e-9))
        rn = rcp(nw2)
        uh = fma(u, F(1e-9), m * w) * rn
        qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
        th = tanh(fma(w, z, b))
        z = fma(uh, th, z)
        return z, fma(th, th, fma(-th, th, F(1)) * qd)
    del base
    return planar


FORMS["m_exact"] = (make_planar_m_exact(), radial_r3, base_r3)


# Round 6 (verdict r05 "Next" 3): a cancellation-aware m near w u = log(e - 1), where
# softplus(w u) - 1 cancels.  With delta = w u - log(e - 1) formed by one fma against the
# two-float constant X0H + X0L (the product w u is exact inside the fma: no rounding of w u
# enters delta), m = log1p((1 - 1/e) expm1(delta)) + 1e-5 = delta P(delta) + 1e-5 with a
# degree-5 polynomial fitted for relative error on |delta| <= 0.25 (<= 2 ulp in fp32 Horner);
# outside that range the existing form (softplus - (1 - 1e-5)) is not cancellation-limited.
X0H, X0L = F(0.54132485), F(7.158233e-10)
M_POLY = [F(0.63212055), F(0.11627208), F(-0.010241115), F(-0.0038298753), F(0.0009094632), F(0.00016557719)]
M_RANGE = F(0.25)


def m_delta(w, u, sp):
    d = fma(w, u, -X0H) - X0L
    p = M_POLY[5]
    for c in M_POLY[4::-1]:
        p = fma(d, p, c)
    md = fma(d, p, F(1e-5))
    return np.where(np.abs(d) <= M_RANGE, md, sp - ONE_M)


def make_planar_mdelta(tanh=tanh_t3):
    def planar(z, u, wraw, b):
        w = wraw + F(1)
        wtu = w * u
        nw2 = fma(w, w, F(1e-9))
        rn = rcp(nw2)
        sp = softplus_alpha(wtu)
        m = m_delta(w, u, sp)
        uh = fma(u, F(1e-9), m * w) * rn
        qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
        th = tanh(fma(w, z, b))
        z = fma(uh, th, z)
        return z, fma(th, th, fma(-th, th, F(1)) * qd)
    return planar


def make_planar_dfsp(tanh=tanh_t3):
    """The double-float alternative, emulated at its best: m from a correctly rounded softplus of
    the EXACT w u (fp64 evaluation) — the floor any double-float softplus could reach."""
    def planar(z, u, wraw, b):
        w = wraw + F(1)
        wtu = w * u
        wtu64 = np.asarray(w, np.float64) * np.asarray(u, np.float64)
        sp64 = np.logaddexp(0.0, wtu64)
        m = r32(sp64 - (1.0 - 1e-5))
        sp = r32(sp64)
        nw2 = fma(w, w, F(1e-9))
        rn = rcp(nw2)
        uh = fma(u, F(1e-9), m * w) * rn
        qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
        th = tanh(fma(w, z, b))
        z = fma(uh, th, z)
        return z, fma(th, th, fma(-th, th, F(1)) * qd)
    return planar


FORMS["mdelta"] = (make_planar_mdelta(), radial_r3, base_r3)
FORMS["dfsp"] = (make_planar_dfsp(), radial_r3, base_r3)


def fit_m_poly(R, deg):
    """fp32 coefficients of P with log1p((1 - 1/e) expm1(d)) ~= d P(d) on |d| <= R (relative
    least squares on Chebyshev nodes)."""
    c = 1 - 1 / np.e
    d = np.cos(np.linspace(0, np.pi, 8001)) * R
    d = d[np.abs(d) > 1e-12]
    g = np.log1p(c * np.expm1(d)) / d
    V = np.vander(d, deg + 1, increasing=True)
    coef, *_ = np.linalg.lstsq(V / g[:, None], np.ones_like(g), rcond=None)
    return [F(x) for x in coef]


def make_planar_mdelta_r(R, deg, tanh=tanh_t3):
    cf, RR = fit_m_poly(R, deg), F(R)

    def planar(z, u, wraw, b):
        w = wraw + F(1)
        wtu = w * u
        nw2 = fma(w, w, F(1e-9))
        rn = rcp(nw2)
        sp = softplus_alpha(wtu)
        d = fma(w, u, -X0H) - X0L
        p = cf[-1]
        for c in cf[-2::-1]:
            p = fma(d, p, c)
        m = np.where(np.abs(d) <= RR, fma(d, p, F(1e-5)), sp - ONE_M)
        uh = fma(u, F(1e-9), m * w) * rn
        qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
        th = tanh(fma(w, z, b))
        z = fma(uh, th, z)
        return z, fma(th, th, fma(-th, th, F(1)) * qd)
    return planar


for _R, _deg in ((0.75, 7), (1.5, 11), (2.0, 13), (3.0, 17)):
    FORMS[f"md{_R}"] = (make_planar_mdelta_r(_R, _deg), radial_r3, base_r3)
# round 6's shipped form (csrc/nfn_device.h planar1_m): |d| <= 0.75, degree 7
FORMS["r6"] = FORMS["md0.75"]
# attribution: the round-6 m with an exact tanh / a wider polynomial range with an exact tanh
FORMS["r6+tx"] = (make_planar_mdelta_r(0.75, 7, tanh=tanh_exact), radial_r3, base_r3)
FORMS["md2.0+tx"] = (make_planar_mdelta_r(2.0, 13, tanh=tanh_exact), radial_r3, base_r3)


def make_planar_r6x(tanh=tanh_t3, rn_newton=False, uh_div=False):
    """Round 6's shipped planar form (planar1_m, |d| <= 0.75) with the attribution's next
    candidates: a Newton-refined 1 / (w^2 + 1e-9) (two fma) and a corrected u_hat quotient."""
    cf, RR = fit_m_poly(0.75, 7), F(0.75)

    def planar(z, u, wraw, b):
        w = wraw + F(1)
        wtu = w * u
        nw2 = fma(w, w, F(1e-9))
        rn = rcp(nw2)
        if rn_newton:
            rn = fma(fma(-nw2, rn, F(1)), rn, rn)
        sp = softplus_alpha(wtu)
        d = fma(w, u, -X0H) - X0L
        p = cf[-1]
        for c in cf[-2::-1]:
            p = fma(d, p, c)
        m = np.where(np.abs(d) <= RR, fma(d, p, F(1e-5)), sp - ONE_M)
        num = fma(u, F(1e-9), m * w)
        uh = num * rn
        if uh_div:
            uh = fma(fma(-nw2, uh, num), rn, uh)
        qd = fma((wtu - m) * F(1e-9), rn, sp + F(1e-5))
        th = tanh(fma(w, z, b))
        z = fma(uh, th, z)
        return z, fma(th, th, fma(-th, th, F(1)) * qd)
    return planar


FORMS["r6+rn"] = (make_planar_r6x(rn_newton=True), radial_r3, base_r3)
FORMS["r6+ud"] = (make_planar_r6x(uh_div=True), radial_r3, base_r3)
FORMS["r6+rn+ud"] = (make_planar_r6x(rn_newton=True, uh_div=True), radial_r3, base_r3)
FORMS["r6+tacc"] = (make_planar_r6x(tanh=tanh_acc), radial_r3, base_r3)
FORMS["r6+tx+ud"] = (make_planar_r6x(tanh=tanh_exact, uh_div=True), radial_r3, base_r3)
FORMS["r6+tacc+ud"] = (make_planar_r6x(tanh=tanh_acc, uh_div=True), radial_r3, base_r3)


if __name__ == "__main__":
    main()
