"""Instrumented op count of the ray-step algorithm.

TEST INFRASTRUCTURE: a pure-Python restatement of the arithmetic that the GPU
kernel performs per RK4 step (torj.jl_amd/csrc/torj_math.hpp: shared-basis
bicubic field evaluation, analytic dispersion gradients, Albajar absorption
with power-series Bessel factors), run on a counting float.  It serves two
purposes:
  1. the algorithmic FLOP figures committed in torj_hip/flops.py (used by
     bench.py's roofline) are produced by `python oracle/flopcount.py`;
  2. its values are checked against the dual-number C oracle in the tests, an
     independent check of the hand-derived gradients.

Counting convention: add/sub/mul/neg-free compare = 1
(compares are free), fma = 2 (not used: a*b+c counts 2), div = 1, sqrt = 1;
transcendentals as their expanded op sequences: exp 26, sin 20, cos 20,
acos 30 (fdlibm-style polynomial + reduction counts).
"""
from __future__ import annotations

import math
import os

COST = {"exp": 26, "sin": 20, "cos": 20, "acos": 30, "sqrt": 1}


class Counter:
    n = 0


def _real(o):
    return isinstance(o, (CF, int, float))


class CF:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = float(v.v if isinstance(v, CF) else v)

    @staticmethod
    def _v(o):
        return o.v if isinstance(o, CF) else float(o)

    def _op(self, r):
        Counter.n += 1
        return CF(r)

    # other operand types (the complex counting type of flopcount_warm.py) get
    # their reflected operator: NotImplemented
    def __add__(self, o): return self._op(self.v + self._v(o)) if _real(o) else NotImplemented
    def __radd__(self, o): return self._op(self._v(o) + self.v)
    def __sub__(self, o): return self._op(self.v - self._v(o)) if _real(o) else NotImplemented
    def __rsub__(self, o): return self._op(self._v(o) - self.v)
    def __mul__(self, o): return self._op(self.v * self._v(o)) if _real(o) else NotImplemented
    def __rmul__(self, o): return self._op(self._v(o) * self.v)
    def __truediv__(self, o): return self._op(self.v / self._v(o)) if _real(o) else NotImplemented
    def __rtruediv__(self, o): return self._op(self._v(o) / self.v)
    def __neg__(self): return CF(-self.v)
    def __lt__(self, o): return self.v < self._v(o)
    def __le__(self, o): return self.v <= self._v(o)
    def __gt__(self, o): return self.v > self._v(o)
    def __ge__(self, o): return self.v >= self._v(o)
    def __float__(self): return self.v


def _f(name, fn):
    def g(x):
        Counter.n += COST[name]
        return CF(fn(CF._v(x)))
    return g


exp = _f("exp", math.exp)
sin = _f("sin", math.sin)
cos = _f("cos", math.cos)
acos = _f("acos", math.acos)
sqrt = _f("sqrt", math.sqrt)

C_LIGHT, E, ME, EPS0 = 2.99792458e8, 1.602176634e-19, 9.1093837015e-31, 8.8541878128e-12


def bweights(d):
    p = 1.0 - d
    d2, p2 = d * d, p * p
    w = [p2 * p * (1 / 6), 2 / 3 - d2 + 0.5 * d2 * d, 2 / 3 - p2 + 0.5 * p2 * p, d2 * d * (1 / 6)]
    dw = [-0.5 * p2, -2.0 * d + 1.5 * d2, 2.0 * p - 1.5 * p2, 0.5 * d2]
    return w, dw


def eval_fields(coef, g, R, Z, ngrad, nval):
    """coef[field][iR][iZ] (padded).  Returns values, dR, dZ (in-grid path)."""
    nR, nZ, R1, Z1, invhR, invhZ = g
    uR, uZ = (R - R1) * invhR, (Z - Z1) * invhZ
    iR, iZ = min(max(int(math.floor(uR.v)), 0), nR - 2), min(max(int(math.floor(uZ.v)), 0), nZ - 2)
    wR, dwR = bweights(uR - iR)
    wZ, dwZ = bweights(uZ - iZ)
    nt = ngrad + nval
    v = [CF(0)] * nt
    gr = [CF(0)] * nt
    gz = [CF(0)] * nt
    grz = [CF(0)] * nt
    for b in range(4):
        for f in range(nt):
            sv, sd = CF(0), CF(0)
            for a in range(4):
                c = coef[f][iR + a][iZ + b]
                sv = sv + wR[a] * c
                sd = sd + dwR[a] * c
            v[f] = v[f] + wZ[b] * sv
            gz[f] = gz[f] + wZ[b] * 0 + dwZ[b] * sv if False else gz[f] + dwZ[b] * sv
            gr[f] = gr[f] + wZ[b] * sd
            if f < ngrad:
                grz[f] = grz[f] + dwZ[b] * sd
    vals = [v[f] for f in range(nt)]
    dR = [gr[f] * invhR for f in range(ngrad)]
    dZ = [gz[f] * invhZ for f in range(ngrad)]
    return vals, dR, dZ


def plasma_point(coef, g, x, omega, with_te=True):
    """coef order: Br, Bphi, Bz, lnne, lnTe"""
    Cx = E * E / (EPS0 * ME * omega * omega)
    Cy = E / (ME * omega)
    R = sqrt(x[0] * x[0] + x[1] * x[1])
    invR = 1.0 / R
    c, s = x[0] * invR, x[1] * invR
    v, dR, dZ = eval_fields(coef, g, R, x[2], 4, 1 if with_te else 0)
    Br, Bp, Bz = v[0], v[1], v[2]
    Bx, By = Br * c - Bp * s, Br * s + Bp * c
    BxR, ByR = dR[0] * c - dR[1] * s, dR[0] * s + dR[1] * c
    dB = [[BxR * c + s * By * invR, ByR * c - s * Bx * invR, dR[2] * c],
          [BxR * s - c * By * invR, ByR * s + c * Bx * invR, dR[2] * s],
          [dZ[0] * c - dZ[1] * s, dZ[0] * s + dZ[1] * c, dZ[2]]]
    Babs = sqrt(Bx * Bx + By * By + Bz * Bz)
    invB = 1.0 / Babs
    b = [Bx * invB, By * invB, Bz * invB]
    ne = exp(v[3])
    X = ne * Cx
    Y = Babs * Cy
    dl = [dR[3] * c, dR[3] * s, dZ[3]]
    dX = [X * dl[q] for q in range(3)]
    dY = [Cy * (b[0] * dB[q][0] + b[1] * dB[q][1] + b[2] * dB[q][2]) for q in range(3)]
    return dict(X=X, Y=Y, b=b, Babs=Babs, dB=dB, dX=dX, dY=dY, lnTe=v[4] if with_te else None)


def ns_partials(X, Y, Np, mode):
    md = float(mode)
    Np2, Y2 = Np * Np, Y * Y
    invY2 = 1.0 / Y2
    om, omX = 1.0 - Np2, 1.0 - X
    Delta = om * om + 4.0 * Np2 * omX * invY2
    sq = sqrt(Delta)
    A = 1.0 + md * sq + Np2
    Q = 2.0 * (-1.0 + X + Y2)
    invQ = 1.0 / Q
    G = X * Y2 * invQ
    dDX = -4.0 * Np2 * invY2
    dDY = -8.0 * Np2 * omX * invY2 / Y
    dDN = -4.0 * Np * om + 8.0 * Np * omX * invY2
    h = md * 0.5 / sq
    dAX, dAY, dAN = h * dDX, h * dDY, h * dDN + 2.0 * Np
    invQ2 = invQ * invQ
    dGX = 2.0 * Y2 * (Y2 - 1.0) * invQ2
    dGY = 4.0 * X * Y * (X - 1.0) * invQ2
    return 1.0 - X + A * G, -1.0 + dAX * G + A * dGX, dAY * G + A * dGY, dAN * G


def dispersion_grad(p, N, mode):
    b = p["b"]
    Npar = N[0] * b[0] + N[1] * b[1] + N[2] * b[2]
    Ns2, nX, nY, nN = ns_partials(p["X"], p["Y"], Npar, mode)
    N2 = N[0] * N[0] + N[1] * N[1] + N[2] * N[2]
    dDdN = [2.0 * N[q] - nN * b[q] for q in range(3)]
    invB = 1.0 / p["Babs"]
    dDdx = []
    for q in range(3):
        dBq = p["dB"][q]
        NdB = N[0] * dBq[0] + N[1] * dBq[1] + N[2] * dBq[2]
        bdB = b[0] * dBq[0] + b[1] * dBq[1] + b[2] * dBq[2]
        dNp = (NdB - Npar * bdB) * invB
        dDdx.append(-(nX * p["dX"][q] + nY * p["dY"][q] + nN * dNp))
    nrm = sqrt(dDdN[0] * dDdN[0] + dDdN[1] * dDdN[1] + dDdN[2] * dDdN[2])
    inv = 1.0 / nrm
    du = [dDdN[q] * inv for q in range(3)] + [-dDdx[q] * inv for q in range(3)]
    return N2 - Ns2, du, Npar


def _series_coef(nu, k):
    return 1.0 / (math.factorial(k) * math.factorial(k + nu))


_HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "torj.jl_amd", "csrc", "torj_bessel_coefs.hpp")
_BT = None


def bessel_table():
    """(terms per level, coef[level][nu-2][k]) parsed from the product's generated
    header torj_bessel_coefs.hpp (data only; tools/gen_bessel_coefs.py made it)."""
    global _BT
    if _BT is None:
        import re
        txt = open(_HDR).read()
        terms = [int(v) for v in re.search(r"kBesselTerms\[kBesselLevels\] = \{([^}]*)\}", txt).group(1).split(",")]
        body = txt[txt.index("kBesselCoef"):]
        rows = [[float(v) for v in r.split(",") if v.strip()] for r in re.findall(r"\{([-0-9.e, +]+)\}", body)]
        coef = [rows[3 * lv:3 * lv + 3] for lv in range(len(terms))]
        _BT = (terms, coef)
    return _BT


def series_level(x_m):
    return 0 if x_m <= 1.0 else 1 if x_m <= 2.0 else 2 if x_m <= 3.0 else 3 if x_m <= 4.0 else 4


def series_terms(x_m):
    """polynomial length of torj_math.hpp albajar_harmonic for argument x_m"""
    lv = series_level(x_m)
    return bessel_table()[0][lv] if lv < 4 else 44


def series_coef(nu, k, x_m):
    lv = series_level(x_m)
    return bessel_table()[1][lv][nu - 2][k] if lv < 4 else _series_coef(nu, k)


def albajar_harmonic(gl, mu, r, Npar, inv_sqNp, Nperp, omega_bar, Axz, ea, e3, m, count=None):
    """Node-pair form of abs_Al_integral_nume_fast x sqrt((m/m0)^2-1) (torj_math.hpp
    albajar_harmonic + pair_term, TORJ_PAIR_V2): the pair (+t, -t) shares every
    t-even factor, bracket(+-t) = P +- t Q, and gamma(+-t) = G0 +- G1 t, the
    resonance condition's linear form (harm_geom, TORJ_NODE_GAMMA_LIN, round 6)."""
    md = float(m)
    inv_md = 1.0 / md  # compile-time constant
    r2m1 = r * r - 1.0
    sq_r = sqrt(r2m1)
    x_m = Nperp * omega_bar * sq_r
    q = x_m * inv_sqNp * inv_md
    K0 = Axz * Axz + ea * ea
    K1 = Axz * ea * x_m * inv_md
    K2 = 4.0 * ea * ea * (inv_md * inv_md)
    K3 = q * q * e3 * e3
    K4 = 2.0 * q * Axz * e3
    K5 = q * ea * e3 * x_m * inv_md
    upa1 = inv_sqNp * sq_r
    # node exponent mu (1 - gamma(+-t)) = Y0 -+ Y1 t (the device takes it in base 2)
    Y0 = mu - mu * (r * inv_sqNp)
    Y1 = mu * (Npar * upa1)
    hx = 0.5 * x_m
    K = series_terms(x_m.v)
    if count is not None:
        count["harm_setup"] = Counter.n - count["_t0"]
    total = CF(0)
    n = len(gl)
    for i in range(n // 2 + (n & 1)):
        t, w, st, t2 = gl[i]
        single = (n & 1) and i == n // 2
        h = hx * st
        h2 = h * h
        z = -h2
        n0 = Counter.n
        xv = x_m.v
        Sm, Sm1 = CF(series_coef(m, K - 1, xv)), CF(series_coef(m + 1, K - 1, xv))
        for k in range(K - 2, -1, -1):
            Sm = Sm * z + series_coef(m, k, xv)
            Sm1 = Sm1 * z + series_coef(m + 1, k, xv)
        n_series = Counter.n - n0
        Sl = md * Sm - h2 * Sm1
        p = h
        for _ in range(1, 2 * m - 1):
            p = p * h
        hSm = h * Sm
        A = hSm * Sm
        T1 = h2 * Sm1
        B = K2 * Sl * (h * T1)
        Cc = st * Sm * (Sl - T1)
        P = A * (K3 * t2 + K0) + (Cc * K1 - B)
        wp = w * p
        n_node = 0
        if single:
            n1 = Counter.n
            E = exp(Y0)
            n_node = Counter.n - n1
            total = total + wp * P * E
        else:
            Q = A * K4 + Cc * K5
            n1 = Counter.n
            Ep = exp(Y0 - Y1 * t)
            n_node = Counter.n - n1
            Em = exp(Y0 + Y1 * t)
            total = total + wp * (P * (Ep + Em) + (t * Q) * (Ep - Em))
        if count is not None and "node" not in count:
            count["node"] = n_node
        if count is not None and "pair_shared" not in count:
            count["pair_shared"] = (Counter.n - n0) - n_series - (2 - bool(single)) * count["node"]
            count["term"] = n_series / (K - 1)
    n1 = Counter.n
    Pm = md / (Nperp * omega_bar)
    res = -mu * Pm * Pm * total * sq_r
    if count is not None:
        count["harm_post"] = Counter.n - n1
    return res


def abs_albajar_fast(gl, omega, X, Y, Nabs, Npar, Te, mode, count=None):
    """torj_math.hpp abs_albajar_fast (src/absorption.jl:191-226 restated for the
    device: sqrt(1 - cos^2) for sin(acos(cos)), one reciprocal per denominator)."""
    if count is not None:
        count["_t0"] = Counter.n
    if Te < 20.0:
        return CF(0)
    kmu = ME * C_LIGHT * C_LIGHT / E  # compile-time constant
    inv_mu = Te * (1.0 / kmu)
    mu = kmu * (1.0 / Te)
    omega_bar = 1.0 / Y
    cos_t = Npar * (1.0 / Nabs)
    sin_t = sqrt(1.0 - cos_t * cos_t)
    Nperp = sqrt(Nabs * Nabs - Npar * Npar)
    if X >= 1.0:
        return CF(0)
    s2, c2, omX = sin_t * sin_t, cos_t * cos_t, 1.0 - X
    Y2, invY2 = Y * Y, omega_bar * omega_bar
    rho = sqrt(Y2 * (s2 * s2) + 4.0 * omX * omX * c2)
    f = (2.0 * omX) * (1.0 / (2.0 * omX - Y2 * s2 - float(mode) * Y * rho))
    Nt = 1.0 - X * f
    if Nt < 0.0:
        return CF(0)
    Nt = sqrt(Nt)
    if not (Nt > 0.0) or Nt > 1.0:
        return CF(0)
    inv_Nt = 1.0 / Nt
    g = 1.0 - (1.0 - Y2) * f
    if c2 < 1e-5 or 1.0 - s2 < 1e-5:
        if mode > 0:
            ea = sqrt(inv_Nt)
            e1 = -(omega_bar * g) * ea
            e3 = CF(0)
        else:
            e1, ea, e3 = CF(0), CF(0), sqrt(inv_Nt)
    else:
        Nt2 = Nt * Nt
        den = omX - Nt2 * s2
        inv_den = 1.0 / den
        gg = invY2 * (g * g)
        ta = 1.0 + (omX * Nt2 * c2) * (inv_den * inv_den) * gg
        tb = 1.0 + (omX * inv_den) * gg
        ea = sqrt(inv_Nt * (1.0 / sqrt(s2 * (ta * ta) + c2 * (tb * tb))))
        if mode <= 0:
            ea = -ea
        e1 = -(omega_bar * g) * ea
        e3 = -((Nt2 * sin_t * cos_t) * inv_den) * e1
    sqNp = sqrt(1.0 - Npar * Npar)
    m0 = sqNp * omega_bar
    inv_sqNp = 1.0 / sqNp
    N_eff = (Nperp * Npar) * (inv_sqNp * inv_sqNp)
    Axz = e1 + N_eff * e3
    inv_m0 = inv_sqNp * Y
    if count is not None:
        count["alpha_pre"] = Counter.n - count["_t0"]
    c_abs = CF(0)
    hc = count  # per-harmonic figures from the first harmonic only
    for m in (2, 3):
        if not (m < m0):
            if hc is not None:
                hc["_t0"] = Counter.n
            c_abs = c_abs + albajar_harmonic(gl, mu, m * inv_m0, Npar, inv_sqNp, Nperp,
                                             omega_bar, Axz, ea, e3, m, count=hc)
            hc = None
    n1 = Counter.n
    a = 1.0 / (inv_mu * (inv_mu * (105.0 / 128.0) + 15.0 / 8.0) + 1.0)
    sm = sqrt(mu * (1.0 / (2.0 * math.pi)))
    c_abs = c_abs * (a * (sm * sm * sm))
    c_abs = -(c_abs * (2.0 * math.pi * math.pi) * inv_m0)
    res = c_abs * X * omega * (omega_bar * (1.0 / C_LIGHT))
    if count is not None:
        count["alpha_post"] = Counter.n - n1
    return res


def gl_table(n):
    import numpy as np
    t, w = np.polynomial.legendre.leggauss(n)
    return [(float(a), float(b), math.sqrt(1.0 - a * a), float(a * a)) for a, b in zip(t, w)]


def measure(coef, g, x, N, omega, mode, n_gl=24):
    """Op counts of one RHS at state (x, N): returns dict of components."""
    x = [CF(v) for v in x]
    N = [CF(v) for v in N]
    gl = gl_table(n_gl)
    Counter.n = 0
    p = plasma_point(coef, g, x, omega)
    D, du, Npar = dispersion_grad(p, N, mode)
    Nabs = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2])
    Te = exp(p["lnTe"])
    cold = Counter.n
    cnt = {}
    al = abs_albajar_fast(gl, omega, p["X"], p["Y"], Nabs, Npar, Te, mode, count=cnt)
    return dict(cold=cold, D=float(D), du=[float(v) for v in du], alpha=float(al), **cnt)


def rk4_overhead():
    """RK4 combination + psi evaluation + chunk bookkeeping per step (ops outside the RHS)."""
    Counter.n = 0
    x = [CF(1.0)] * 7
    k = [CF(0.5)] * 7
    # per stage: acc += w*k (7 mul-add = 14), stage point x + h k (6 fma = 12)
    for _ in range(4):
        acc = [x[i] * 2.0 + k[i] for i in range(7)]
        xt = [k[i] * 0.5 + x[i] for i in range(6)]
    xn = [x[i] + 0.1 * acc[i] for i in range(7)]
    P = exp(-xn[6])
    dP = P - 1.0
    n_rk = Counter.n
    # psi value at the new point: R (3 ops + sqrt) + 2 axis setups (~2 x 22) + 16 x 2 + 4 x 2
    return n_rk, dP


if __name__ == "__main__":
    import json
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "torj.jl_amd"))
    import numpy as np

    import oracle as O
    from torj_hip import synthetic as S

    eq = S.circular_tokamak()
    OP = O.OraclePlasma(*S.plasma_args(eq))
    fc = OP.field_coefs()
    coef = [fc[k] for k in ("Br", "Bphi", "Bz", "lnne", "lnTe")]
    R, Z = eq["R_coords"], eq["Z_coords"]
    g = (len(R), len(Z), R[0], Z[0], (len(R) - 1) / (R[-1] - R[0]), (len(Z) - 1) / (Z[-1] - Z[0]))
    O.abs_al_init(24)
    om = 2 * np.pi * 92.5e9
    N0 = O.pol_tor_angles_2_vector(np.deg2rad(30), 0)
    st, xp, Np, s0 = OP.ray_entry([2.5, 0, 0.4], N0, om, 1)
    r = OP.trace(xp[None], Np[None], om, 1, 1e-4, 1500)
    x, N = r["state"][0, :3], r["state"][0, 3:6]
    m = measure(coef, g, x, N, om, 1)
    n_rk, _ = rk4_overhead()
    psi_eval = 4 + 1 + 2 * 22 + 16 * 2 + 4 * 2  # R, axis setups, row + column sums
    out = {
        "FLOPS_RHS_COLD": m["cold"],
        "FLOPS_ALPHA_PRE": m["alpha_pre"],
        "FLOPS_ALPHA_POST": m["alpha_post"],
        "FLOPS_HARM": m["harm_setup"] + m["harm_post"],
        "FLOPS_PAIR_SHARED": m["pair_shared"],
        "FLOPS_NODE": m["node"],
        "FLOPS_SERIES_TERM": m["term"],
        "FLOPS_STEP_OVERHEAD": n_rk + psi_eval,
        "check": {"alpha_counted": m["alpha"], "alpha_oracle": OP.alpha_approx(x, N, om, 1),
                  "du_counted": m["du"], "du_oracle": list(OP.grad_lambda(x, N, om, 1))},
    }
    print(json.dumps(out, indent=1))
