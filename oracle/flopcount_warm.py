"""Instrumented op count of the weakly relativistic warm alpha (absorption
model 2, iwarm 1) as the GPU evaluates it (torj.jl_amd/csrc/torj_warm.hpp:
larmornumber, fsup_s, dieltens_wr, warmdisp_n2, alpha_core / alpha_warm_v).

TEST INFRASTRUCTURE: a pure-Python restatement of that arithmetic on the
counting float of oracle/flopcount.py (same convention: add/sub/mul/div/sqrt 1,
fma 2, exp 26; compares, negations, and integer work free).  It produces the
FLOPS_WARM_* constants committed in torj_hip/flops.py (`python
oracle/flopcount_warm.py`), and tests/test_warm_flops.py checks that the
per-trip model of flops.py, fed with this restatement's trip counts, equals its
instrumented count from below (lower bound, within a few %), and that the
restatement computes the same N_perp^2 as the C oracle (so its branches and
trip counts are the real ones).

Algorithmic conventions (what is NOT counted): the factorial tables asl, bsl,
0.5^l (2l)!/l! (integer-only constants); loop-invariant per-call quantities
(psi, 1/psi^2, amu anpl, 1/yg, ...) once per call, not per use.  Branch-
dependent parts are counted at their cheapest branch (a lower bound):
  fsup side: alpha < 0 (no shifted arguments), large |psi| (cf32 from czp, czm);
  recursion step: the small-|psi| form (1 + phi2 cf1) / (l + 1/2);
  warmdisp: every pass but the last of each call sums the tensor and updates
  N_perp^2 (the last one breaks before its sum); unconverged calls (100
  updates) are counted with 99.
The Faddeeva value comes from scipy; its op count is that of the branch the
kernel runs (torj_warm.hpp faddeeva_upper): the asymptotic series (10 terms)
where |x| >= 16 or Im z >= 16, else Weideman's N = 36 sum (both by the
real-coefficient recurrence since round 6, complex Horner before).  The
model prices larmornumber's resonance tests at one per call (their least).
"""
from __future__ import annotations

import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from flopcount import CF, Counter, exp, sqrt  # noqa: E402

KC, KE, KME = 2.99792458e8, 1.602176634e-19, 9.1093837015e-31
KWEID_N = 36
I_MAX = 5


def _n(fn, *a):
    """op count of fn(*a)"""
    c0 = Counter.n
    fn(*a)
    return Counter.n - c0


class CC:
    """complex of counting floats: (a+bi)(c+di) = 4 mul + 2 add, Smith division"""
    __slots__ = ("re", "im")

    def __init__(self, re, im=0.0):
        self.re = re if isinstance(re, CF) else CF(re)
        self.im = im if isinstance(im, CF) else CF(im)

    @staticmethod
    def _c(o):
        return o if isinstance(o, CC) else None

    def __add__(self, o):
        c = self._c(o)
        return CC(self.re + c.re, self.im + c.im) if c else CC(self.re + o, self.im)

    __radd__ = __add__

    def __sub__(self, o):
        c = self._c(o)
        return CC(self.re - c.re, self.im - c.im) if c else CC(self.re - o, self.im)

    def __rsub__(self, o):  # real - complex
        return CC(o - self.re, -self.im)

    def __neg__(self):
        return CC(-self.re, -self.im)

    def __mul__(self, o):
        c = self._c(o)
        if c:
            return CC(self.re * c.re - self.im * c.im, self.re * c.im + self.im * c.re)
        return CC(o * self.re, o * self.im)

    __rmul__ = __mul__

    def __truediv__(self, o):
        c = self._c(o)
        if not c:
            r = 1.0 / o
            return CC(self.re * r, self.im * r)
        if abs(c.re.v) >= abs(c.im.v):  # Smith's algorithm (torj_warm.hpp operator/)
            r = c.im / c.re
            d = 1.0 / (c.re + c.im * r)
            return CC((self.re + self.im * r) * d, (self.im - self.re * r) * d)
        r = c.re / c.im
        d = 1.0 / (c.re * r + c.im)
        return CC((self.re * r + self.im) * d, (self.im * r - self.re) * d)

    def itimes(self):
        return CC(-self.im, self.re)

    def value(self):
        return complex(self.re.v, self.im.v)


def cabs(a):  # hypot: x^2 + y^2 and a sqrt (scaling not counted)
    return sqrt(a.re * a.re + a.im * a.im)


def cnorm(a):  # |a|^2
    return a.re * a.re + a.im * a.im


def csqrt(z):  # torj_warm.hpp csqrt_: |z| from the norm, one reciprocal
    if z.re.v == 0.0 and z.im.v == 0.0:
        return CC(0.0, z.im)
    r = sqrt(cnorm(z))
    t = sqrt(0.5 * (r + CF(abs(z.re.v))))
    h = 0.5 * (1.0 / t)
    if z.re.v >= 0.0:
        return CC(t, z.im * h)
    return CC(CF(abs(z.im.v)) * h, CF(math.copysign(t.v, z.im.v)))


def root_update(cc2, sg, rr, cc4, na):
    """warmdisp's root and convergence test as the kernel forms them: the
    division by 2 cc4 as a product with conj(cc4) / (2 |cc4|^2), the moduli
    from their squares (na = |anpr2a|^2, carried from the previous pass)"""
    ic = 0.5 * (1.0 / cnorm(cc4))
    anpr2 = (-cc2 + sg * csqrt(rr)) * CC(cc4.re * ic, -cc4.im * ic)
    n2 = cnorm(anpr2)
    errnpr = abs((1.0 - sqrt(n2 * (1.0 / na))).v)
    return anpr2, n2, errnpr


def faddeeva_weideman_count():
    """the kernel's faddeeva_upper + zetac_upper on counting floats (fixed cost)"""
    c0 = Counter.n
    x, y, L = CF(0.3), CF(0.2), 5.0
    dr, di = L + y, -x
    idn = 1.0 / (dr * dr + di * di)
    ir, ii = dr * idn, -di * idn
    nr, ni = L - y, x
    zr, zi = nr * ir - ni * ii, nr * ii + ni * ir
    # weid_poly (round 6): the real-coefficient recurrence b_k = a_k + r b_(k+1) - s b_(k+2)
    r, s = 2.0 * zr, zr * zr + zi * zi
    b2 = CF(0.1)
    b1 = r * b2 + 0.01
    for k in range(2, KWEID_N - 1):
        b1, b2 = r * b1 + (-s * b2 + 0.01 * k), b1
    pr = zr * b1 + (-s * b2 + 0.02)
    pim = zi * b1
    i2r, i2i = ir * ir - ii * ii, 2.0 * ir * ii
    wr = 2.0 * (pr * i2r - pim * i2i) + 0.5 * ir
    wi = 2.0 * (pr * i2i + pim * i2r) + 0.5 * ii
    _ = (-1.77 * wi, 1.77 * wr)
    return Counter.n - c0


FAD = faddeeva_weideman_count()
KFAD_ASYM, KFAD_ASYM_K = 16.0, 10


def faddeeva_asym_count():
    """the kernel's faddeeva_asym + zetac_upper on counting floats (fixed cost)"""
    c0 = Counter.n
    x, y = CF(20.0), CF(3.0)
    ir2 = 1.0 / (x * x + y * y)
    a, b = x * ir2, -y * ir2
    ur, ui = 0.5 * (a * a - b * b), a * b
    # the (2k - 1)!! series in u by Knuth's real-coefficient recurrence (torj_warm.hpp
    # asym_horner, TORJ_ASYM_KNUTH, round 6; complex Horner before)
    df = lambda k: float(math.prod(range(1, 2 * k, 2)))  # noqa: E731
    r, s = 2.0 * ur, ur * ur + ui * ui
    b2 = CF(df(KFAD_ASYM_K - 1))
    b1 = r * b2 + df(KFAD_ASYM_K - 2)
    for k in range(KFAD_ASYM_K - 3, 0, -1):
        b1, b2 = r * b1 + (-s * b2 + df(k)), b1
    tr, ti = ur * b1 + (-s * b2 + 1.0), ui * b1
    pr, pim = a * tr - b * ti, a * ti + b * tr
    _ = (-0.56 * pim, 0.56 * pr)
    _ = (-1.77 * _[1], 1.77 * _[0])
    return Counter.n - c0


FAD_ASYM = faddeeva_asym_count()


def asym_ok(x, y):
    """the kernel's branch (torj_warm.hpp faddeeva_asym_ok)"""
    return abs(float(x)) >= KFAD_ASYM or float(y) >= KFAD_ASYM


def zetac(x, y, tr=None):
    """value from scipy (Z = i sqrt(pi) w), cost of the kernel's branch"""
    from scipy.special import wofz

    asym = asym_ok(x, y)
    Counter.n += FAD_ASYM if asym else FAD
    if tr is not None:
        tr.nfad += 1
        tr.nasym += int(asym)
    z = 1j * math.sqrt(math.pi) * wofz(complex(float(x), float(y)))
    return CC(z.real, z.imag)


class Trips:
    def __init__(self):
        self.ltrips = self.nfad = self.nasym = self.passes = self.lrm = 0
        self.converged = True


def larmornumber(yg, npl, mu, tr):
    dnl = 1.0 - npl * npl
    imax = 1
    nharm = int(math.floor((1.0 / yg).v))
    if (nharm * yg).v < 1.0:
        nharm += 1
    while True:
        tr.ltrips += 1
        ygn = nharm * yg
        rdu2 = ygn * ygn - dnl
        gg = (ygn - sqrt(npl * npl * rdu2)) / dnl
        if (mu * (gg - 1.0)).v > 15.0:
            break
        nharm += 1
        imax += 1
        if imax > 100:
            nharm = int(math.floor(yg.v))
            break
    return nharm


def fsup_side(sg, isa, inv, tr, state):
    """one is = sg*isa of fsup_s: returns the stored cf2 of l = isa .. isa+2"""
    yg, amu, psi, big = inv["yg"], inv["amu"], inv["psi"], inv["big"]
    is_ = sg * isa
    alpha = inv["anpl2hm1"] + is_ * yg
    phi2 = amu * alpha
    phim = sqrt(CF(abs(phi2.v)))
    if alpha.v >= 0:
        xp, yp, xm, ym, x0, y0 = psi - phim, 0.0, -psi - phim, 0.0, -phim, 0.0
    else:
        xp, yp, xm, ym, x0, y0 = psi, phim, -psi, phim, 0.0, phim
    mirror = alpha.v < 0
    czp = zetac(xp, yp, tr)
    if mirror:
        czm = CC(-czp.re, czp.im)
    else:
        czm = zetac(xm, ym, tr)
    cz0 = None
    if not big:
        cz0 = zetac(x0, y0, tr)
    cf12 = CC(0.0)
    if alpha.v != 0.0:
        i2phim = 0.5 * (1.0 / phim)
        cf12 = -((czp + czm) * i2phim) if alpha.v > 0 else -((czp + czm) * i2phim).itimes()
    if big:
        cf32 = -((czp - czm) * inv["i2psi"])
    else:
        cphi = CC(0.0, -phim) if alpha.v < 0 else CC(phim)
        cf32 = 2.0 * (1.0 - cphi * cz0)
    st = {"cf0": cf12, "cf1": cf32}

    def step(l):
        if big:
            cf2 = (1.0 + phi2 * st["cf0"] - (l - 0.5) * st["cf1"]) * inv["ipsi2"]
        else:
            cf2 = (1.0 + phi2 * st["cf1"]) * (1.0 / CF(l + 0.5))
        st["cf0"], st["cf1"] = st["cf1"], cf2
        state["steps"] += 1
        return cf2

    out = {}
    if is_ == 0:
        out[0] = cf32
    for l in range(1, isa):
        step(l)
    for ir in range(3):
        if isa + ir < 1:
            continue
        out[ir] = step(isa + ir)
    return out


def alpha_wr(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode):
    """the kernel's alpha_warm_v<1> on counting floats -> (alpha, n2, Trips)"""
    tr = Trips()
    X, Y, N_par, inv_dDdN = CF(X), CF(Y), CF(N_par), CF(inv_dDdN)
    Te = exp(CF(math.log(Te)))  # the kernel holds ln Te (plasma_point)
    n3 = [CF(N_abs), CF(0.0), CF(0.0)]  # |N| from the refractive-index vector
    Na = sqrt(n3[0] * n3[0] + n3[1] * n3[1] + n3[2] * n3[2])
    mu = (KME * KC * KC) / (Te * KE)
    d = Na * Na - N_par * N_par
    npr = sqrt(CF(max(d.v, 0.0)))
    nharm = larmornumber(Y, N_par, mu, tr)
    lrm = min(nharm, I_MAX)
    tr.lrm = lrm
    # dieltens_wr: per-call invariants
    anpl, amu, yg, xg = N_par, mu, Y, X
    anpl2 = anpl * anpl
    psi = sqrt(0.5 * amu) * anpl
    big = abs(psi.v) > 0.7
    inv = dict(yg=yg, amu=amu, psi=psi, big=big, anpl2hm1=anpl2 / 2.0 - 1.0)
    if big:
        inv["ipsi2"] = 1.0 / (psi * psi)
        inv["i2psi"] = 0.5 / psi
    amu_anpl, amu_anpl2 = amu * anpl, amu * anpl2
    iyg = 1.0 / yg
    iyg2 = iyg * iyg
    ca = [[CC(0.0) for _ in range(6)] for _ in range(lrm)]
    state = {"steps": 0}
    p0 = None
    for isa in range(lrm + 1):
        p = [CC(0.0)] * 3
        m = [CC(0.0)] * 3
        for sg in ((1,) if isa == 0 else (-1, 1)):
            out = fsup_side(sg, isa, inv, tr, state)
            for ir, cf2 in out.items():
                if isa == 0 and ir == 0:  # s = 0: cefp(0, 0) = cefm(0, 0) = cf32
                    p[0] = m[0] = cf2
                    continue
                p[ir] = p[ir] + cf2
                m[ir] = (m[ir] + cf2) if sg * isa > 0 else (m[ir] - cf2)
        if isa == 0:
            p0 = list(p)
        cq0p, cq0m = amu * p[0], amu * m[0]
        cq1p = amu_anpl * (p[0] - p[1])
        cq1m = amu_anpl * (m[0] - m[1])
        cq2p = p[1] + amu_anpl2 * (p[2] + p[0] - 2.0 * p[1])
        for l in range(max(isa, 1), lrm + 1):
            lm, k = l - 1, l - isa
            asl = (-1.0) ** k / (math.factorial(isa + l) * math.factorial(l - isa))  # table
            bsl = asl * (isa * isa + (2 * k * lm * (l + isa)) / (2 * l - 1))          # table
            ca[lm][0] = ca[lm][0] + (isa * isa * asl) * cq0p
            ca[lm][1] = ca[lm][1] + (isa * l * asl) * cq0m
            ca[lm][2] = ca[lm][2] + bsl * cq0p
            ca[lm][3] = ca[lm][3] + ((isa * asl) * iyg) * cq1m
            ca[lm][4] = ca[lm][4] + ((l * asl) * iyg) * cq1p
            ca[lm][5] = ca[lm][5] + (asl * iyg2) * cq2p
    base = iyg2 / amu  # (1/yg^2/amu)^lm by repeated multiplication
    pw = CF(1.0)
    eps = []
    for l in range(1, lrm + 1):
        if l > 1:
            pw = pw * base
        fcl = (0.5 ** l * math.factorial(2 * l) / math.factorial(l)) * pw  # table x power
        xf = xg * fcl
        e = [-(xf * ca[l - 1][0]), (xf * ca[l - 1][1]).itimes(), -(xf * ca[l - 1][2]),
             -(xf * ca[l - 1][3]), -((xf * ca[l - 1][4]).itimes()), -(xf * ca[l - 1][5])]
        eps.append(e)
    cq2p0 = p0[1] + amu_anpl2 * (p0[2] + p0[0] - 2.0 * p0[1])
    e330 = 1.0 - (xg * amu) * cq2p0
    eps[0][0] = eps[0][0] + 1.0
    eps[0][2] = eps[0][2] + 1.0
    # warmdisp_n2
    sox = mode if Y.v <= 1.0 else -mode
    anpr2a = CC(npr * npr)
    anpr2 = anpr2a
    errnpr = 1.0
    na = cnorm(anpr2a)
    tr.converged = False
    for i in range(1, 101):
        tr.passes = i
        if i > 2 and errnpr < 1e-4:  # before the sum: alpha needs no polarisation
            tr.converged = True
            break
        s = [CC(0.0)] * 6
        pwc = CC(1.0)
        for l in range(lrm):
            for q in range(6):
                s[q] = s[q] + eps[l][q] * pwc
            pwc = pwc * anpr2a
        e11, e12, e22, a13, a23, a33 = s
        a31, a32 = a13, -a23
        em, ep = e11 - anpl2, e22 - anpl2
        oa = 1.0 - a33
        a13p, a31p = a13 + anpl, a31 + anpl
        cc4 = em * oa + a13p * a31p
        cc2 = (-(e12 * e12 * oa) - a32 * e12 * a13p + a23 * e12 * a31p
               - (a23 * a32 + e330 + ep * oa) * em - a13p * a31p * ep)
        cc0 = e330 * (em * ep + e12 * e12)
        rr = cc2 * cc2 - 4.0 * cc0 * cc4
        if Y.v > 1.0:
            sg = float(sox) if rr.im.v > 0.0 else float(-sox)
        else:
            sg = float(-sox)
            if rr.re.v <= 0.0 and rr.im.v >= 0.0:
                sg = -sg
        anpr2, na, errnpr = root_update(cc2, sg, rr, cc4, na)
        anpr2a = anpr2
    if anpr2.re.v < 0.0 and anpr2.im.v < 0.0:
        anpr2 = CC(0.0)
    alpha = 2.0 * anpr2.im * CF(omega) / KC * inv_dDdN
    tr.steps = state["steps"]
    return alpha.v, anpr2.value(), tr


def component_counts():
    """per-trip op counts of the model in torj_hip/flops.py, each measured by
    running that piece of alpha_wr's arithmetic on counting floats"""
    c = {"FLOPS_WARM_FADDEEVA": FAD, "FLOPS_WARM_FADDEEVA_ASYM": FAD_ASYM}
    # larmornumber test: ygn, rdu2, gg, mu (gg - 1)
    yg, npl, mu, dnl = CF(0.6), CF(0.1), CF(300.0), CF(0.99)

    def trip():
        ygn = 2 * yg
        rdu2 = ygn * ygn - dnl
        gg = (ygn - sqrt(npl * npl * rdu2)) / dnl
        _ = mu * (gg - 1.0)
    c["FLOPS_WARM_LARMOR_TEST"] = _n(trip)
    # fsup side at its cheapest branch (alpha < 0, large psi), without the
    # Faddeeva evaluations and the recursion steps
    psi, phi2c, amu = CF(1.0), CF(-3.0), CF(300.0)
    czp, czm = CC(0.1, 0.2), CC(0.3, 0.1)

    def side():
        alpha = CF(-0.5) + (-1) * yg
        phi2 = amu * alpha
        phim = sqrt(CF(abs(phi2.v)))
        i2phim = 0.5 * (1.0 / phim)
        _ = -((czp + czm) * i2phim).itimes()
        _ = -((czp - czm) * CF(0.5))
    c["FLOPS_WARM_SIDE"] = _n(side)
    cf0, cf1 = CC(0.1, 0.2), CC(0.3, 0.4)
    c["FLOPS_WARM_STEP"] = _n(lambda: (1.0 + phi2c * cf1) * (1.0 / CF(2.5)))  # small-psi form
    p = [CC(0.1, 0.1)] * 3
    c["FLOPS_WARM_STORE"] = _n(lambda: (p[0] + cf0, p[1] - cf0))  # p[ir], m[ir] accumulation
    amu_anpl, amu_anpl2 = CF(1.0), CF(2.0)

    def isa_terms():
        _ = amu * p[0], amu * p[0]
        _ = amu_anpl * (p[0] - p[1]), amu_anpl * (p[0] - p[1])
        _ = p[1] + amu_anpl2 * (p[2] + p[0] - 2.0 * p[1])
    c["FLOPS_WARM_ISA"] = _n(isa_terms)
    cq, iyg, iyg2 = CC(0.1, 0.2), CF(1.5), CF(2.25)

    def pair():
        ca = [CC(0.0)] * 6
        ca[0] = ca[0] + 0.5 * cq
        ca[1] = ca[1] + 0.5 * cq
        ca[2] = ca[2] + 0.5 * cq
        ca[3] = ca[3] + (0.5 * iyg) * cq
        ca[4] = ca[4] + (0.5 * iyg) * cq
        ca[5] = ca[5] + (0.5 * iyg2) * cq
    c["FLOPS_WARM_PAIR"] = _n(pair)
    xg = CF(0.5)

    def order():
        pw = CF(1.0) * CF(2.0)
        xf = xg * (3.0 * pw)
        _ = [xf * cq for _ in range(6)]
    c["FLOPS_WARM_ORDER"] = _n(order)
    eps = [CC(0.1, 0.2)] * 6

    def sum_term():
        s = [CC(0.0)] * 6
        for q in range(6):
            s[q] = s[q] + eps[q] * cq
        _ = cq * cq
    c["FLOPS_WARM_SUM_TERM"] = _n(sum_term)
    c["FLOPS_WARM_UPDATE"] = _update_count()
    c["FLOPS_WARM_CALL"] = _call_count()
    return c


def _update_count():
    """one warmdisp update (cc4, cc2, cc0, discriminant, root, convergence test)"""
    e = [CC(0.1 * (q + 1), 0.05 * q) for q in range(6)]
    e330, anpl, anpl2 = CC(0.9, 0.01), CF(0.2), CF(0.04)
    na = CF(0.25)

    def upd():
        e11, e12, e22, a13, a23, a33 = e
        a31, a32 = a13, -a23
        em, ep = e11 - anpl2, e22 - anpl2
        oa = 1.0 - a33
        a13p, a31p = a13 + anpl, a31 + anpl
        cc4 = em * oa + a13p * a31p
        cc2 = (-(e12 * e12 * oa) - a32 * e12 * a13p + a23 * e12 * a31p
               - (a23 * a32 + e330 + ep * oa) * em - a13p * a31p * ep)
        cc0 = e330 * (em * ep + e12 * e12)
        rr = cc2 * cc2 - 4.0 * cc0 * cc4
        _ = root_update(cc2, 1.0, rr, cc4, na)
    return _n(upd)


def _call_count():
    """per call: Te, |N|, mu, N_perp, larmornumber setup, the tensor's per-call
    invariants (cheapest branch: large psi), e330, the l = 1 identity, the
    starting N_perp^2, alpha itself"""
    lnTe, N, Npar, X, Y = CF(8.0), [CF(0.3), CF(0.2), CF(0.1)], CF(0.2), CF(0.5), CF(0.6)
    p0 = [CC(0.1, 0.1)] * 3
    e0 = [CC(0.1, 0.1)] * 6

    def call():
        Te = exp(lnTe)
        Na = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2])
        mu = (KME * KC * KC) / (Te * KE)
        npr = sqrt(Na * Na - Npar * Npar)
        dnl = 1.0 - Npar * Npar
        _ = 1.0 / Y, 2 * Y  # floor(1/yg), nharm yg < 1
        anpl2 = Npar * Npar
        psi = sqrt(0.5 * mu) * Npar
        _ = anpl2 / 2.0 - 1.0, 1.0 / (psi * psi), 0.5 / psi
        amu_anpl2 = mu * Npar, mu * anpl2
        iyg = 1.0 / Y
        iyg2 = iyg * iyg
        _ = iyg2 / mu
        cq2p0 = p0[1] + amu_anpl2[1] * (p0[2] + p0[0] - 2.0 * p0[1])
        _ = 1.0 - (X * mu) * cq2p0
        _ = e0[0] + 1.0, e0[2] + 1.0
        a = CC(npr * npr)
        _ = cnorm(a)  # |anpr2a|^2 of the first pass
        _ = 2.0 * CF(0.1) * CF(1e11) / KC * CF(0.5)
    return _n(call)


def model_flops(tr_list, c):
    """flops.py's per-trip model from the trip counts of calls"""
    tot = 0
    for tr in tr_list:
        L = tr.lrm
        steps = L * L + 5 * L + 2
        stored = 2 + 6 * L
        upd = tr.passes - 1
        tot += (c["FLOPS_WARM_CALL"] + 1 * c["FLOPS_WARM_LARMOR_TEST"]
                + (tr.nfad - tr.nasym) * c["FLOPS_WARM_FADDEEVA"]
                + tr.nasym * c["FLOPS_WARM_FADDEEVA_ASYM"] + (2 * L + 1) * c["FLOPS_WARM_SIDE"]
                + steps * c["FLOPS_WARM_STEP"] + stored * c["FLOPS_WARM_STORE"]
                + (L + 1) * c["FLOPS_WARM_ISA"] + (L * L + 3 * L) // 2 * c["FLOPS_WARM_PAIR"]
                + L * c["FLOPS_WARM_ORDER"] + upd * L * c["FLOPS_WARM_SUM_TERM"]
                + upd * c["FLOPS_WARM_UPDATE"])
    return tot


if __name__ == "__main__":
    for k, v in component_counts().items():
        print(f"{k} = {v}")
