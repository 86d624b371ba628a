"""Warm-plasma absorption (src/general_absorption.jl) restated in numpy, repaired.

TEST INFRASTRUCTURE ONLY: the checker of the GPU's warm absorption
(torj_trace_cfg.absorption = 2, 3) -- never imported by the product.

The reference file is GRAY's warm dispersion module (Farina), transliterated to
Julia but never included (src/TorJ.jl:19-29) and not runnable as shipped
(SURVEY.md section 0.4).  This restatement follows its algorithm and repairs:

  R1  ssbi (:291-320): its @assert compares the series with an undefined
      `sphericalbesselj` (and the wrong function): dropped.  The series is
      I_{m+1/2}(z) / (z/2)^{m+1/2} = sum_k (z^2/4)^k / (k! Gamma(m+k+3/2)),
      summed with the reference's own stopping rule (relative term < 1e-10)
      and its Numerical-Recipes gammln, so the truncation matches.
  R2  warmdisp (:1158-1267): `anpr2` is only bound inside the loop (:1223) but
      read after it (:1229): initialised to the starting guess before the
      loop, i.e. the Fortran semantics (last computed value).
  R3  the t-grid _ttv/_extdtv (:8-13) is never initialised (set_extv! is never
      called): built here.
  R4  alpha (:1328-1337) has no caller: theta is the angle between N and B and
      v_g_perp = 1 / |dD/dN| -- the ray Hamiltonian's normalisation, so that
      alpha = 2 Im(N_perp^2) (omega/c) / |dD/dN| is the spatial damping rate of
      the power along the arc length of our rays (Im D = -Im N_perp^2).
  R5  the root selector sox: the reference passes `imod` straight through, but
      warmdisp's root choice flips with its own Y > 1 branch (:1203-1214), while
      TorJ's mode sign (src/solve.jl:110, src/dispersion.jl:28-32) labels one
      branch of the cold relation throughout: sox = mode for Y < 1 and -mode for
      Y > 1 is the choice whose cold limit (mu -> inf) is the ray's own cold
      root, checked in tests/test_oracle_pins.py on both sides of Y = 1.

Third-party arithmetic replaced by pinned libraries: expei = scipy.special.expi
(x) e^-x (reference: Cody's CALCEI), zetac = i sqrt(pi) scipy.special.wofz
(reference: ACM TOMS 680).  Parity of the repaired module with any executed
reference is unpinned (there is none).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import expi, wofz

ME, C, E = 9.1093837015e-31, 2.99792458e8, 1.602176634e-19
SQRT_PI = 1.7724538509055160272981674833411
NTV, TMAX = 501, 5.0
DT = 2.0 * TMAX / (NTV - 1)
I_MAX = 5  # src/constants.jl:4

_TTV = -TMAX + DT * np.arange(NTV)          # R3 (src/general_absorption.jl:8-13)
_EXTDTV = np.exp(-_TTV ** 2) * DT


def expei(x):
    """exp(-x) Ei(x) (src/general_absorption.jl:29-232); -xinf = -1.79e308 at 0
    (a finite value, so that zm * expei(zm) = 0 there as in the reference)."""
    x = np.asarray(x, dtype=float)
    with np.errstate(over="ignore", invalid="ignore"):
        out = np.where(x == 0.0, -1.79e308, expi(x) * np.exp(-x))
        # far tails: e^-x Ei(x) ~ 1/x (1 + 1/x + 2/x^2 ...) where exp over/underflows
        big = np.abs(x) > 700.0
        if np.any(big):
            xb = x[big]
            s = np.zeros_like(xb)
            term = np.ones_like(xb)
            for k in range(30):
                s += term
                term = term * (k + 1) / xb
            out = out.copy()
            out[big] = s / xb
    return out


def fact(k):
    """(src/general_absorption.jl:240-257)"""
    return 0.0 if k < 0 else float(math.factorial(k))


def gammln(x):
    """Numerical Recipes lnGamma (src/general_absorption.jl:265-283), kept for
    the series' truncation parity."""
    cof = (76.18009172947146, -86.50532032941677, 24.01409824083091, -1.231739572450155,
           0.1208650973866179e-2, -0.5395239384953e-5)
    y = x
    tmp = x + 5.5
    tmp = (x + 0.5) * math.log(tmp) - tmp
    ser = 1.000000000190015
    for c in cof:
        y += 1.0
        ser += c / y
    return tmp + math.log(2.5066282746310005 * ser / x)


def ssbi(zz, n, l):
    """sum_k (zz^2/4)^k / (k! Gamma(m+k+3/2)) for m = n .. l+2 (R1)."""
    z2q = 0.25 * zz * zz
    out = []
    for m in range(n, l + 3):
        c0 = 1.0 / math.exp(gammln(m + 1.5))
        s = c0
        for k in range(1, 51):
            c1 = c0 * z2q / ((m + k) + 0.5) / k
            s += c1
            if c1 / s < 1e-10:
                break
            c0 = c1
        out.append(s)
    return out


def zetac(x, y):
    """Plasma dispersion function Z(x + iy) = i sqrt(pi) w(x + iy) (:345-465)."""
    return 1j * SQRT_PI * wofz(complex(x, y))


def fsup(yg, anpl, amu, lrm):
    """Shkarofsky-function coefficients cefp/cefm (:473-561), (lrm+1) x 3."""
    cefp = np.zeros((lrm + 1, 3), complex)
    cefm = np.zeros((lrm + 1, 3), complex)
    anpl2hm1 = anpl * anpl / 2.0 - 1.0
    psi = math.sqrt(0.5 * amu) * anpl
    apsi = abs(psi)
    for is_ in range(-lrm, lrm + 1):
        alpha = anpl2hm1 + is_ * yg
        phi2 = amu * alpha
        phim = math.sqrt(abs(phi2))
        if alpha >= 0:
            xp, yp, xm, ym, x0, y0 = psi - phim, 0.0, -psi - phim, 0.0, -phim, 0.0
        else:
            xp, yp, xm, ym, x0, y0 = psi, phim, -psi, phim, 0.0, phim
        czp, czm = zetac(xp, yp), zetac(xm, ym)
        if alpha > 0:
            cf12 = -(czp + czm) / (2.0 * phim)
        elif alpha < 0:
            cf12 = -1j * (czp + czm) / (2.0 * phim)
        else:
            cf12 = 0j
        if apsi > 0.7:
            cf32 = -(czp - czm) / (2.0 * psi)
        else:
            cphi = -1j * phim if alpha < 0 else phim
            cf32 = 2.0 * (1.0 - cphi * zetac(x0, y0))
        cf0, cf1 = cf12, cf32
        if is_ == 0:
            cefp[0, 0] = cf32
            cefm[0, 0] = cf32
        isa = abs(is_)
        for l in range(1, isa + 3):
            if apsi > 0.7:
                cf2 = (1.0 + phi2 * cf0 - (l - 0.5) * cf1) / psi ** 2
            else:
                cf2 = (1.0 + phi2 * cf1) / (l + 0.5)
            ir = l - isa
            if ir >= 0:
                cefp[isa, ir] += cf2
                cefm[isa, ir] += cf2 if is_ > 0 else -cf2
            cf0, cf1 = cf1, cf2
    return cefp, cefm


def _finish_tensor(xg, epsl_acc, e330):
    epsl = epsl_acc
    epsl[0, 0, 0] += 1.0
    epsl[1, 1, 0] += 1.0
    epsl[1, 0, :] = -epsl[0, 1, :]
    epsl[2, 0, :] = epsl[0, 2, :]
    epsl[2, 1, :] = -epsl[1, 2, :]
    return e330, epsl


def dieltens_maxw_wr(xg, yg, anpl, amu, lrm):
    """Weakly relativistic tensor, Krivenski & Orefice (:573-638)."""
    anpl2 = anpl * anpl
    cefp, cefm = fsup(yg, anpl, amu, lrm)
    epsl = np.zeros((3, 3, lrm), complex)
    for l in range(1, lrm + 1):
        lm = l - 1
        fcl = 0.5 ** l * ((1.0 / yg) ** 2 / amu) ** lm * fact(2 * l) / fact(l)
        ca = np.zeros(6, complex)  # 11 12 22 13 23 33
        for is_ in range(0, l + 1):
            k = l - is_
            asl = (-1.0) ** k / (fact(is_ + l) * fact(l - is_))
            bsl = asl * (is_ * is_ + (2 * k * lm * (l + is_)) / (2 * l - 1))
            cq0p = amu * cefp[is_, 0]
            cq0m = amu * cefm[is_, 0]
            cq1p = amu * anpl * (cefp[is_, 0] - cefp[is_, 1])
            cq1m = amu * anpl * (cefm[is_, 0] - cefm[is_, 1])
            cq2p = cefp[is_, 1] + amu * anpl2 * (cefp[is_, 2] + cefp[is_, 0] - 2.0 * cefp[is_, 1])
            ca += np.array([is_ ** 2 * asl * cq0p, is_ * l * asl * cq0m, bsl * cq0p,
                            is_ * asl * cq1m / yg, l * asl * cq1p / yg, asl * cq2p / yg ** 2])
        epsl[0, 0, l - 1] = -xg * ca[0] * fcl
        epsl[0, 1, l - 1] = 1j * xg * ca[1] * fcl
        epsl[1, 1, l - 1] = -xg * ca[2] * fcl
        epsl[0, 2, l - 1] = -xg * ca[3] * fcl
        epsl[1, 2, l - 1] = -1j * xg * ca[4] * fcl
        epsl[2, 2, l - 1] = -xg * ca[5] * fcl
    cq2p = cefp[0, 1] + amu * anpl2 * (cefp[0, 2] + cefp[0, 0] - 2.0 * cefp[0, 1])
    return _finish_tensor(xg, epsl, 1.0 - xg * amu * cq2p)


def hermitian(yg, anpl, amu, lrm):
    """Hermitian part, numerical t-integration of the iwarm > 2 branch
    (:646-734): rr[n + lrm, k, m] for n in [-llm, llm], k = 0..2, m = 0..llm."""
    rr = np.zeros((2 * lrm + 1, 3, lrm + 1))
    cmxw = 1.0 + 15.0 / (8.0 * amu) + 105.0 / (128.0 * amu ** 2)
    cr = -amu * amu / (SQRT_PI * cmxw)
    llm = min(3, lrm)
    bth2 = 2.0 / amu
    bth = math.sqrt(bth2)
    amu2 = amu * amu
    amu4, amu6 = amu2 * amu2, amu2 * amu2 * amu2
    t = _TTV
    rxt = np.sqrt(1.0 + t * t / (2.0 * amu))
    x = t * rxt
    upl2 = bth2 * x * x
    upl = bth * x
    gx = 1.0 + t * t / amu
    exdx = cr * _EXTDTV * gx / rxt
    for n in range(-llm, llm + 1):
        gr = anpl * upl + n * yg
        zm = -amu * (gx - gr)
        s = amu * (gx + gr)
        fe0m = expei(zm)
        for m in range(abs(n), llm + 1):
            if m == 0:
                rr[lrm, 2, 0] += np.sum(-exdx * fe0m * upl2)
                continue
            zm2 = zm * zm
            if m == 1:
                ffe = (1.0 + s * (1.0 - zm * fe0m)) / amu2
            elif m == 2:
                ffe = (6.0 - 2.0 * zm + 4.0 * s + s * s * (1.0 + zm - zm2 * fe0m)) / amu4
            else:
                ffe = (18.0 * s * (s + 4.0 - zm) + 6.0 * (20.0 - 8.0 * zm + zm2)
                       + s ** 3 * (2.0 + zm + zm2 - zm2 * zm * fe0m)) / amu6
            rr[n + lrm, 0, m] += np.sum(exdx * ffe)
            rr[n + lrm, 1, m] += np.sum(exdx * ffe * upl)
            rr[n + lrm, 2, m] += np.sum(exdx * ffe * upl2)
    return rr


def antihermitian(yg, anpl, amu, lrm):
    """Anti-hermitian part (:951-1043): ri[n-1, k, m-1], m >= n."""
    ri = np.zeros((lrm, 3, lrm))
    dnl = 1.0 - anpl * anpl
    cmu = anpl * amu
    cmxw = 1.0 + 15.0 / (8.0 * amu) + 105.0 / (128.0 * amu ** 2)
    ci = math.sqrt(2.0 * math.pi * amu) * amu ** 2 / cmxw
    for n in range(1, lrm + 1):
        ygn = n * yg
        rdu2 = ygn * ygn - dnl
        if not rdu2 > 0.0:
            continue
        rdu = math.sqrt(rdu2)
        du = rdu / dnl
        ub = anpl * ygn / dnl
        aa = amu * anpl * du
        if abs(aa) > 5.0:
            up, um = ub + du, ub - du
            gp, gm = anpl * up + ygn, anpl * um + ygn
            xp, xm = up + 1.0 / cmu, um + 1.0 / cmu
            eem, eep = math.exp(-amu * (gm - 1.0)), math.exp(-amu * (gp - 1.0))
            f0p, f1p, f2p = -1.0 / cmu, -xp / cmu, -(1.0 / cmu ** 2 + xp * xp) / cmu
            f0m, f1m, f2m = -1.0 / cmu, -xm / cmu, -(1.0 / cmu ** 2 + xm * xm) / cmu
            for m in range(1, lrm + 1):
                g0p = -2.0 * m * (f1p - ub * f0p) / cmu
                g0m = -2.0 * m * (f1m - ub * f0m) / cmu
                g1p = -((1.0 + 2 * m) * f2p - 2.0 * (m + 1) * ub * f1p + up * um * f0p) / cmu
                g1m = -((1.0 + 2 * m) * f2m - 2.0 * (m + 1) * ub * f1m + up * um * f0m) / cmu
                g2p = (2.0 * (1 + m) * g1p - 2.0 * m * (ub * f2p - up * um * f1p)) / cmu
                g2m = (2.0 * (1 + m) * g1m - 2.0 * m * (ub * f2m - up * um * f1m)) / cmu
                if m >= n:
                    h = 0.5 * ci * dnl ** m
                    ri[n - 1, 0, m - 1] = h * (g0p * eep - g0m * eem)
                    ri[n - 1, 1, m - 1] = h * (g1p * eep - g1m * eem)
                    ri[n - 1, 2, m - 1] = h * (g2p * eep - g2m * eem)
                f0p, f1p, f2p, f0m, f1m, f2m = g0p, g1p, g2p, g0m, g1m, g2m
        else:
            ee = math.exp(-amu * (ygn - 1.0 + anpl * ub))
            fsbi = ssbi(aa, n, lrm)
            for m in range(n, lrm + 1):
                cm = SQRT_PI * fact(m) * du ** (2 * m + 1)
                cim = 0.5 * ci * dnl ** m
                mm = m - n
                fi0 = cm * fsbi[mm]
                fi1 = -0.5 * aa * cm * fsbi[mm + 1]
                fi2 = 0.5 * cm * (fsbi[mm + 1] + 0.5 * aa * aa * fsbi[mm + 2])
                ri[n - 1, 0, m - 1] = cim * ee * fi0
                ri[n - 1, 1, m - 1] = cim * ee * (du * fi1 + ub * fi0)
                ri[n - 1, 2, m - 1] = cim * ee * (du * du * fi2 + 2.0 * du * ub * fi1 + ub * ub * fi0)
    return ri


def dieltens_maxw_fr(xg, yg, anpl, amu, lrm):
    """Fully relativistic tensor, iwarm = 3 (:1056-1134)."""
    rr = hermitian(yg, anpl, amu, lrm)
    ri = antihermitian(yg, anpl, amu, lrm)
    epsl = np.zeros((3, 3, lrm), complex)
    for l in range(1, lrm + 1):
        lm = l - 1
        fal = -0.25 ** l * fact(2 * l) / (fact(l) ** 2 * yg ** (2 * lm))
        ca = np.zeros(6, complex)
        for is_ in range(0, l + 1):
            k = l - is_
            asl = (-1.0) ** k / (fact(is_ + l) * fact(l - is_))
            bsl = asl * (is_ * is_ + (2 * k * lm * (l + is_)) / (2 * l - 1))
            if is_ > 0:
                a, b = rr[lrm + is_, :, l], rr[lrm - is_, :, l]
                cq0p = complex(a[0] + b[0], ri[is_ - 1, 0, l - 1])
                cq0m = complex(a[0] - b[0], ri[is_ - 1, 0, l - 1])
                cq1p = complex(a[1] + b[1], ri[is_ - 1, 1, l - 1])
                cq1m = complex(a[1] - b[1], ri[is_ - 1, 1, l - 1])
                cq2p = complex(a[2] + b[2], ri[is_ - 1, 2, l - 1])
            else:
                cq0p = cq0m = complex(rr[lrm, 0, l])
                cq1p = cq1m = complex(rr[lrm, 1, l])
                cq2p = complex(rr[lrm, 2, l])
            ca += np.array([is_ ** 2 * asl * cq0p, is_ * l * asl * cq0m, bsl * cq0p,
                            is_ * asl * cq1m / yg, l * asl * cq1p / yg, asl * cq2p / yg ** 2])
        epsl[0, 0, l - 1] = -xg * ca[0] * fal
        epsl[0, 1, l - 1] = 1j * xg * ca[1] * fal
        epsl[1, 1, l - 1] = -xg * ca[2] * fal
        epsl[0, 2, l - 1] = -xg * ca[3] * fal
        epsl[1, 2, l - 1] = -1j * xg * ca[4] * fal
        epsl[2, 2, l - 1] = -xg * ca[5] * fal
    return _finish_tensor(xg, epsl, 1.0 + xg * rr[lrm, 2, 0])


def warmdisp(xg, yg, anpl, amu, anprc, sox, iwarm, lrm, info=None):
    """Warm dispersion relation for N_perp (:1158-1267) -> (anpr, ierr).
    info (a dict, optional) receives the iteration count, whether the
    fixed-point iteration met its own 1e-4 criterion, and the selector margin:
    the smallest relative distance of the root selector's sign test (Im rr for
    Y > 1, Re / Im rr otherwise) from its threshold -- where it is ~1e-12 the
    reference's choice of root is decided by rounding (test bookkeeping)."""
    anpr2a = complex(anprc * anprc)
    anpr2 = anpr2a  # R2
    anpl2 = anpl * anpl
    if iwarm == 1:
        e330, epsl = dieltens_maxw_wr(xg, yg, anpl, amu, lrm)
    else:
        e330, epsl = dieltens_maxw_fr(xg, yg, anpl, amu, lrm)
    errnpr = 1.0
    converged = False
    margin = np.inf  # smallest relative distance of the root selector's test from its threshold
    for i in range(1, 101):
        sepsl = np.zeros((3, 3), complex)
        for il in range(lrm):
            sepsl += epsl[:, :, il] * anpr2a ** il
        anpra = np.sqrt(anpr2a)
        e11, e22, e12 = sepsl[0, 0], sepsl[1, 1], sepsl[0, 1]
        a33, a13, a23 = sepsl[2, 2], sepsl[0, 2], sepsl[1, 2]
        a31, a32 = a13, -a23
        if i > 2 and errnpr < 1.0e-4:
            converged = True
            break
        cc4 = (e11 - anpl2) * (1.0 - a33) + (a13 + anpl) * (a31 + anpl)
        cc2 = (-e12 * e12 * (1.0 - a33) - a32 * e12 * (a13 + anpl) + a23 * e12 * (a31 + anpl)
               - (a23 * a32 + e330 + (e22 - anpl2) * (1.0 - a33)) * (e11 - anpl2)
               - (a13 + anpl) * (a31 + anpl) * (e22 - anpl2))
        cc0 = e330 * ((e11 - anpl2) * (e22 - anpl2) + e12 * e12)
        rr = cc2 * cc2 - 4.0 * cc0 * cc4
        if yg > 1.0:
            s = float(sox)
            if rr.imag <= 0.0:
                s = -s
            m = abs(rr.imag)
        else:
            s = float(-sox)
            if rr.real <= 0.0 and rr.imag >= 0.0:
                s = -s
            m = rr.real if rr.real > 0.0 else min(-rr.real, abs(rr.imag))
        margin = min(margin, m / max(abs(rr), 1e-300))
        anpr2 = (-cc2 + s * np.sqrt(rr)) / (2.0 * cc4)
        errnpr = abs(1.0 - abs(anpr2) / abs(anpr2a))
        anpr2a = anpr2
    if info is not None:
        info.update(iterations=i, converged=converged, margin=margin)
    ierr = 0
    if anpr2.real < 0.0 and anpr2.imag < 0.0:
        anpr2, ierr = 0j, 99
    return np.sqrt(anpr2), ierr


def larmornumber(yg, npl, mu):
    """Highest harmonic with mu (gamma - 1) <= 15 on the resonance (:1285-1326)."""
    dnl = 1.0 - npl * npl
    imax = 1
    nharm = int(math.floor(1.0 / yg))
    if nharm * yg < 1.0:
        nharm += 1
    while True:
        ygn = nharm * yg
        rdu2 = ygn * ygn - dnl
        gg = (ygn - math.sqrt(npl * npl * rdu2)) / dnl
        if mu * (gg - 1.0) > 15.0:
            break
        nharm += 1
        imax += 1
        if imax > 100:
            nharm = int(math.floor(yg))
            break
    return nharm


def alpha_warm(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode, iwarm=3, info=None):
    """alpha (:1328-1337) with theta from (N_abs, N_par) and v_g_perp = 1/|dD/dN|
    (R4), sox = +-mode (R5).  Returns (alpha [1/m], N_perp_warm complex)."""
    mu = ME * C * C / (Te * E)
    npr = math.sqrt(max(N_abs * N_abs - N_par * N_par, 0.0))
    nharm = larmornumber(Y, N_par, mu)
    lrm = min(I_MAX, nharm)
    sox = mode if Y <= 1.0 else -mode
    anpr, ierr = warmdisp(X, Y, N_par, mu, npr, sox, iwarm, lrm, info)
    return 2.0 * (anpr * anpr).imag * omega / C * inv_dDdN, anpr
