"""The weakly relativistic warm alpha (src/general_absorption.jl, iwarm = 1) in
mpmath at 50 significant digits: the "true value" of the reference's algorithm
at a point, against which the double-precision restatements are judged.

TEST INFRASTRUCTURE ONLY (never imported by the product).  It follows
oracle/warm_ref.py line by line -- the same repairs R1-R5 -- with every
quantity an mpmath number:

  * zetac (:345-465, ACM TOMS 680 in the reference) is Z(z) = i sqrt(pi) w(z)
    with w(z) = exp(-z^2) erfc(-i z), evaluated by mpmath to the working
    precision (the reference's, the oracle's and the product's Faddeeva
    implementations are all approximations of this function);
  * fsup (:473-561), dieltens_maxw_wr (:573-638) and warmdisp (:1158-1267)
    carry 50 digits through the Shkarofsky recurrence
    cf2 = (1 + phi^2 cf0 - (l - 1/2) cf1) / psi^2 (:536-557), whose
    cancellation is what limits the double-precision restatements at cold
    plasma edges;
  * larmornumber (:1285-1326) decides integer Larmor orders and is taken in
    double precision as in warm_ref (its thresholds are not at issue).

The inputs are doubles and are converted exactly."""
from __future__ import annotations

import math

import mpmath as mp

import warm_ref as W

DPS = 50
ME, C, E = W.ME, W.C, W.E


def zetac(z):
    """Z(z) = i sqrt(pi) w(z), w(z) = exp(-z^2) erfc(-i z)."""
    return 1j * mp.sqrt(mp.pi) * mp.exp(-z * z) * mp.erfc(-1j * z)


def fsup(yg, anpl, amu, lrm):
    """Shkarofsky coefficients cefp / cefm (:473-561) as dicts (is, ir) -> mpc."""
    cefp, cefm = {}, {}
    anpl2hm1 = anpl * anpl / 2 - 1
    psi = mp.sqrt(amu / 2) * anpl
    apsi = abs(psi)
    for is_ in range(-lrm, lrm + 1):
        alpha = anpl2hm1 + is_ * yg
        phi2 = amu * alpha
        phim = mp.sqrt(abs(phi2))
        if alpha >= 0:
            zp, zm, z0 = mp.mpc(psi - phim, 0), mp.mpc(-psi - phim, 0), mp.mpc(-phim, 0)
        else:
            zp, zm, z0 = mp.mpc(psi, phim), mp.mpc(-psi, phim), mp.mpc(0, phim)
        czp, czm = zetac(zp), zetac(zm)
        if alpha > 0:
            cf12 = -(czp + czm) / (2 * phim)
        elif alpha < 0:
            cf12 = -1j * (czp + czm) / (2 * phim)
        else:
            cf12 = mp.mpc(0)
        if apsi > mp.mpf("0.7"):
            cf32 = -(czp - czm) / (2 * psi)
        else:
            cphi = -1j * phim if alpha < 0 else phim
            cf32 = 2 * (1 - cphi * zetac(z0))
        cf0, cf1 = cf12, cf32
        if is_ == 0:
            cefp[0, 0] = cefp.get((0, 0), 0) + cf32
            cefm[0, 0] = cefm.get((0, 0), 0) + cf32
        isa = abs(is_)
        for l in range(1, isa + 3):
            if apsi > mp.mpf("0.7"):
                cf2 = (1 + phi2 * cf0 - (l - mp.mpf("0.5")) * cf1) / psi ** 2
            else:
                cf2 = (1 + phi2 * cf1) / (l + mp.mpf("0.5"))
            ir = l - isa
            if ir >= 0:
                cefp[isa, ir] = cefp.get((isa, ir), 0) + cf2
                cefm[isa, ir] = cefm.get((isa, ir), 0) + (cf2 if is_ > 0 else -cf2)
            cf0, cf1 = cf1, cf2
    for k in range(lrm + 1):
        for r in range(3):
            cefp.setdefault((k, r), mp.mpc(0))
            cefm.setdefault((k, r), mp.mpc(0))
    return cefp, cefm


def dieltens_maxw_wr(xg, yg, anpl, amu, lrm):
    """(:573-638) -> (e330, epsl[(i, j, l)])"""
    anpl2 = anpl * anpl
    cefp, cefm = fsup(yg, anpl, amu, lrm)
    epsl = {}
    for l in range(1, lrm + 1):
        lm = l - 1
        fcl = mp.mpf(0.5) ** l * ((1 / yg) ** 2 / amu) ** lm * math.factorial(2 * l) / math.factorial(l)
        ca = [mp.mpc(0)] * 6
        for is_ in range(0, l + 1):
            k = l - is_
            asl = mp.mpf((-1) ** k) / (math.factorial(is_ + l) * math.factorial(l - is_))
            bsl = asl * (is_ * is_ + mp.mpf(2 * k * lm * (l + is_)) / (2 * l - 1))
            cq0p = amu * cefp[is_, 0]
            cq0m = amu * cefm[is_, 0]
            cq1p = amu * anpl * (cefp[is_, 0] - cefp[is_, 1])
            cq1m = amu * anpl * (cefm[is_, 0] - cefm[is_, 1])
            cq2p = cefp[is_, 1] + amu * anpl2 * (cefp[is_, 2] + cefp[is_, 0] - 2 * cefp[is_, 1])
            add = [is_ ** 2 * asl * cq0p, is_ * l * asl * cq0m, bsl * cq0p,
                   is_ * asl * cq1m / yg, l * asl * cq1p / yg, asl * cq2p / yg ** 2]
            ca = [a + b for a, b in zip(ca, add)]
        epsl[0, 0, l] = -xg * ca[0] * fcl
        epsl[0, 1, l] = 1j * xg * ca[1] * fcl
        epsl[1, 1, l] = -xg * ca[2] * fcl
        epsl[0, 2, l] = -xg * ca[3] * fcl
        epsl[1, 2, l] = -1j * xg * ca[4] * fcl
        epsl[2, 2, l] = -xg * ca[5] * fcl
    epsl[0, 0, 1] += 1
    epsl[1, 1, 1] += 1
    cq2p = cefp[0, 1] + amu * anpl2 * (cefp[0, 2] + cefp[0, 0] - 2 * cefp[0, 1])
    return 1 - xg * amu * cq2p, epsl


def warmdisp(xg, yg, anpl, amu, anprc, sox, lrm):
    """(:1158-1267), iwarm = 1, with R2 -> N_perp (complex)."""
    anpr2a = mp.mpc(anprc * anprc)
    anpr2 = anpr2a
    anpl2 = anpl * anpl
    e330, epsl = dieltens_maxw_wr(xg, yg, anpl, amu, lrm)
    errnpr = mp.mpf(1)
    for i in range(1, 101):
        s = {}
        for (a, b) in ((0, 0), (1, 1), (0, 1), (2, 2), (0, 2), (1, 2)):
            s[a, b] = sum(epsl[a, b, l] * anpr2a ** (l - 1) for l in range(1, lrm + 1))
        e11, e22, e12 = s[0, 0], s[1, 1], s[0, 1]
        a33, a13, a23 = s[2, 2], s[0, 2], s[1, 2]
        a31, a32 = a13, -a23
        if i > 2 and errnpr < mp.mpf("1e-4"):
            break
        cc4 = (e11 - anpl2) * (1 - a33) + (a13 + anpl) * (a31 + anpl)
        cc2 = (-e12 * e12 * (1 - a33) - a32 * e12 * (a13 + anpl) + a23 * e12 * (a31 + anpl)
               - (a23 * a32 + e330 + (e22 - anpl2) * (1 - a33)) * (e11 - anpl2)
               - (a13 + anpl) * (a31 + anpl) * (e22 - anpl2))
        cc0 = e330 * ((e11 - anpl2) * (e22 - anpl2) + e12 * e12)
        rr = cc2 * cc2 - 4 * cc0 * cc4
        if yg > 1:
            sg = sox if rr.imag > 0 else -sox
        else:
            sg = -sox
            if rr.real <= 0 and rr.imag >= 0:
                sg = -sg
        anpr2 = (-cc2 + sg * mp.sqrt(rr)) / (2 * cc4)
        errnpr = abs(1 - abs(anpr2) / abs(anpr2a))
        anpr2a = anpr2
    if anpr2.real < 0 and anpr2.imag < 0:
        anpr2 = mp.mpc(0)
    return mp.sqrt(anpr2)


def alpha_warm_wr(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode):
    """alpha (:1328-1337), iwarm = 1, at DPS digits; returns an mpf."""
    with mp.workdps(DPS):
        mu = mp.mpf(ME) * mp.mpf(C) ** 2 / (mp.mpf(Te) * mp.mpf(E))
        npr = mp.sqrt(max(mp.mpf(N_abs) ** 2 - mp.mpf(N_par) ** 2, 0))
        nharm = W.larmornumber(Y, N_par, float(mu))
        lrm = min(W.I_MAX, nharm)
        sox = mode if Y <= 1.0 else -mode
        anpr = warmdisp(mp.mpf(X), mp.mpf(Y), mp.mpf(N_par), mu, npr, sox, lrm)
        return 2 * (anpr * anpr).imag * mp.mpf(omega) / mp.mpf(C) * mp.mpf(inv_dDdN)
