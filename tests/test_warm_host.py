"""The product's warm-absorption math (torj.jl_amd/csrc/torj_warm.hpp, compiled
for the host by tests/native/Makefile -- the same source the trace kernels run)
against scipy and the warm oracle, on CPU.  SURVEY.md section 8(c) KAT (8):
zetac vs wofz <= 1e-13, expei vs expi; alpha / N_perp^2 vs oracle/warm_ref.py
with the tolerances of tests/test_gpu_warm.py."""
import ctypes as C
import math
import os
import subprocess
import warnings

import numpy as np
import pytest
from scipy.special import expi, iv, wofz

HERE = os.path.dirname(os.path.abspath(__file__))
_dp = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def H():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
    L = C.CDLL(os.path.join(HERE, "native", "build", "libwarm_host.so"))
    L.wh_larmornumber.argtypes = [C.c_double, C.c_double, C.c_double]
    L.wh_ssbi.argtypes = [C.c_double, C.c_int, C.c_int, _dp]
    return L


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(_dp)


@pytest.mark.parametrize("box", [(-3, 3, -3, 3), (-30, 30, -1, 1), (-8, 8, 1e-6, 0.1),
                                 (-8, 8, -0.1, -1e-6), (-200, 200, 0, 50)])
def test_zetac_matches_wofz(H, box):
    """Im z >= 0 is what the tensors use (phim >= 0); for Im z << 0 the reflection
    2 exp(-z^2) - w(-z) carries a condition number ~ |z|^2 in both libraries."""
    rng = np.random.default_rng(1)
    n = 20000
    x, y = rng.uniform(box[0], box[1], n), rng.uniform(box[2], box[3], n)
    out = np.zeros(2 * n)
    H.wh_zetac(n, _d(x), _d(y), _d(out))
    z = out[0::2] + 1j * out[1::2]
    ref = 1j * math.sqrt(math.pi) * wofz(x + 1j * y)
    fin = np.isfinite(ref)
    assert (np.abs(z - ref)[fin] / np.abs(ref)[fin]).max() <= 1e-13


def test_zetac_asymptotic_branch_vs_mpmath(H):
    """|x| >= 16 or Im z >= 16: the asymptotic series (torj_warm.hpp
    faddeeva_asym, 10 terms) against mpmath's w(z) = exp(-z^2) erfc(-iz) at 30
    digits, across the upper half plane and |z| up to 1.6e4: 2e-15 of |Z|, and
    the real part (the absorption) to the same relative accuracy wherever it is
    above 1e-30 of |Z| (on the real axis it is exp(-x^2), to the rounding).  Both sides
    of the branch boundary agree to the Weideman branch's 1e-13."""
    import mpmath as mp

    rng = np.random.default_rng(5)
    n = 1500
    r = 16.0 * np.exp(rng.uniform(0.0, np.log(1e3), n))
    th = np.where(rng.random(n) < 0.25, 0.0, rng.uniform(0.0, np.pi, n))
    x, y = r * np.cos(th), r * np.sin(th)
    keep = (np.abs(x) >= 16.0) | (y >= 16.0)
    x, y = x[keep], y[keep]
    m = len(x)
    out = np.zeros(2 * m)
    H.wh_zetac(m, _d(x), _d(y), _d(out))
    z = out[0::2] + 1j * out[1::2]
    with mp.workdps(30):
        ref = np.array([complex(1j * mp.sqrt(mp.pi) * mp.exp(-mp.mpc(a, b) ** 2) * mp.erfc(-1j * mp.mpc(a, b)))
                        for a, b in zip(x, y)])
    assert (np.abs(z - ref) / np.abs(ref)).max() <= 2e-15
    im = np.abs(ref.imag) > 1e-30 * np.abs(ref)  # Im Z = sqrt(pi) Re w
    assert (np.abs(z.imag - ref.imag)[im] / np.abs(ref.imag)[im]).max() <= 2e-15
    ax = y == 0.0
    ex = math.sqrt(math.pi) * np.exp(-x[ax] ** 2)
    assert ax.sum() > 100 and np.all(np.abs(z.imag[ax] - ex) <= 1e-15 * ex)
    # the branch boundary |x| = 16 (y < 16): both sides continuous to 1e-13
    xb = np.array([np.nextafter(16.0, 0.0), 16.0, -np.nextafter(16.0, 0.0), -16.0])
    for yb in (0.0, 1e-3, 0.5, 5.0, 15.9):
        o = np.zeros(8)
        H.wh_zetac(4, _d(xb), _d(np.full(4, yb)), _d(o))
        zz = o[0::2] + 1j * o[1::2]
        assert abs(zz[0] - zz[1]) <= 1e-13 * abs(zz[1]) and abs(zz[2] - zz[3]) <= 1e-13 * abs(zz[3])


def test_expei_matches_expi(H):
    rng = np.random.default_rng(2)
    x = np.concatenate([10 ** rng.uniform(-8, 2.8, 20000), -(10 ** rng.uniform(-8, 2.8, 20000))])
    out = np.zeros(len(x))
    H.wh_expei(len(x), _d(x), _d(out))
    ref = np.exp(-x) * expi(x)
    assert (np.abs(out - ref) / np.abs(ref)).max() <= 1e-11
    z = np.zeros(1)
    H.wh_expei(1, _d(np.zeros(1)), _d(z))
    assert z[0] == -1.79e308  # -xinf, as the reference (general_absorption.jl:29-60)


@pytest.mark.parametrize("z", [1e-3, 0.3, 2.0, 6.0])
def test_ssbi_matches_bessel(H, z):
    out = np.zeros(6)
    H.wh_ssbi(z, 0, 3, out.ctypes.data_as(_dp))
    ref = [iv(m + 0.5, z) / (z / 2) ** (m + 0.5) for m in range(6)]
    assert max(abs(a / b - 1) for a, b in zip(out, ref)) < 1e-9


def test_larmornumber_matches_oracle(H):
    import warm_ref as W

    rng = np.random.default_rng(3)
    for _ in range(2000):
        y, npl, mu = rng.uniform(0.2, 1.5), rng.uniform(-0.6, 0.6), 10 ** rng.uniform(1, 4.7)
        assert H.wh_larmornumber(y, npl, mu) == W.larmornumber(y, npl, mu)


@pytest.mark.parametrize("mode", [1, -1])
@pytest.mark.parametrize("iwarm,te_lo,tol_n2,tol_a", [(3, 10.0, 1e-10, 1e-9), (1, 1e3, 1e-7, 1e-7)])
def test_alpha_warm_matches_oracle(H, O, mode, iwarm, te_lo, tol_n2, tol_a):
    import warm_ref as W

    rng = np.random.default_rng(10 + iwarm)
    n = 200
    om = np.full(n, 2 * np.pi * 140e9)
    X, Y = rng.uniform(0.05, 0.9, n), rng.uniform(0.3, 1.4, n)
    Npar = rng.uniform(-0.5, 0.5, n)
    Te = 10 ** rng.uniform(math.log10(te_lo), 4.3, n)
    inv = rng.uniform(0.2, 2.0, n)
    N2 = np.array([float(O.refractive_index_sq(a, b, c, mode)) for a, b, c in zip(X, Y, Npar)])
    Nabs = np.sqrt(np.maximum(N2, Npar ** 2 + 1e-3))
    a, n2 = np.zeros(n), np.zeros(2 * n)
    H.wh_alpha_warm(n, _d(om), _d(X), _d(Y), _d(Nabs), _d(Npar), _d(Te), _d(inv), mode, iwarm,
                    a.ctypes.data_as(_dp), n2.ctypes.data_as(_dp))
    g = n2[0::2] + 1j * n2[1::2]
    ar, nr, conv = np.zeros(n), np.zeros(n, complex), np.zeros(n, bool)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in range(n):
            info = {}
            ar[i], anpr = W.alpha_warm(om[i], X[i], Y[i], Nabs[i], Npar[i], Te[i], inv[i], mode,
                                       iwarm, info)
            nr[i], conv[i] = anpr * anpr, info["converged"]
    both0 = (nr == 0) & (g == 0)
    e_n = np.where(both0, 0.0, np.abs(g - nr) / np.maximum(np.abs(nr), 1e-300))
    floor = 1e-9 * 2 * np.abs(nr) * om / 2.99792458e8 * inv
    e_a = np.abs(a - ar) / (np.abs(ar) + floor + 1e-300)
    assert conv.sum() > 0.8 * n
    assert e_n[conv].max() <= tol_n2 and e_a[conv].max() <= tol_a


def test_albajar_host_build_matches_golden(H):
    """abs_Albajar_fast of the product (host build of torj_math.hpp, the same
    restated prologue the kernels run: rcp_nz quotients, sqrt(1 - cos^2) for
    sin(acos(cos))) against the oracle's golden sweep: identical NaN / zero
    pattern (the edge semantics of src/absorption.jl:191-226), 1e-10 relative
    elsewhere."""
    import json
    d = json.load(open(os.path.join(HERE, "golden", "albajar.json")))
    rows = np.array(d["rows"], dtype=float)
    H.wh_albajar.argtypes = [C.c_int] + [_dp] * 6 + [C.c_int, _dp, _dp, C.c_int, _dp]
    t, w = np.polynomial.legendre.leggauss(24)
    for mode in (-1, 1):
        r = rows[rows[:, 6] == mode]
        n = len(r)
        out = np.zeros(n)
        cols = [np.ascontiguousarray(r[:, k]) for k in range(6)]
        H.wh_albajar(n, *[_d(c) for c in cols], mode, _d(t), _d(w), 24, _d(out))
        want = r[:, 7]
        nan = np.isnan(want)
        assert np.array_equal(np.isnan(out), nan)
        zero = want == 0
        assert np.all(out[zero] == 0)
        big = ~nan & ~zero & (np.abs(want) > 1e-12)
        assert (np.abs(out[big] - want[big]) / np.abs(want[big])).max() < 1e-10
        small = ~nan & ~zero & ~big
        assert np.abs(out[small] - want[small]).max() < 1e-20


def _stage_points(n_rays=24, every=50):
    """(omega, X, Y, |N|, N_par, Te) at states along rays of the headline fan
    (92.5 GHz X-mode, oracle RK4): the inputs abs_Albajar_fast sees in a trace."""
    import oracle as O
    from torj_hip import synthetic as S
    import torj_hip as T

    O.abs_al_init(24)
    eq = S.circular_tokamak()
    OP = O.OraclePlasma(*S.plasma_args(eq))
    s = S.SETUP
    f = s["f_abs_test"]
    om = 2 * np.pi * f
    N0 = O.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = O.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=92,
                                            min_azimuthal_points=11)
    idx = np.linspace(0, len(w) - 1, n_rays).astype(int)
    P = T.Plasma(*S.plasma_args(eq))
    xp, Np, s0, st = T.ray_entry(P, pos[idx], dirs[idx], om, 1)
    rows = []
    for k in range(every, 2001, every):
        r = OP.trace(xp, Np, om, 1, 1e-4, k)
        for i in range(len(idx)):
            x, N = r["state"][i, :3], r["state"][i, 3:6]
            X, Y, Npar, _ = OP.eval_plasma(x, N, om)
            rows.append((om, X, Y, np.linalg.norm(N), Npar, OP.T_e(x)))
    return np.array(rows)


def test_albajar_negligible_harmonic_skip_is_bit_identical(H):
    """The skip of a harmonic integral whose rigorous bound is below 2^-58 of
    the harmonics already summed (torj_math.hpp albajar_harmonic) leaves
    abs_Albajar_fast bit-identical: host build with the skip on and off over
    stage points along rays of the headline fan (where the third harmonic is
    summed beside the second) and the oracle's golden sweep; the skip fires.
    The same switch settles a call before its polarisation vector when every
    harmonic present is an exact zero: alpha is then a zero of either sign (the
    full evaluation's -0 or the early +0; no later operation sees the sign), so
    zeros are compared as zeros and every other value bit for bit."""
    import json

    rows = _stage_points()
    d = json.load(open(os.path.join(HERE, "golden", "albajar.json")))
    g = np.array(d["rows"], dtype=float)
    H.wh_albajar.argtypes = [C.c_int] + [_dp] * 6 + [C.c_int, _dp, _dp, C.c_int, _dp]
    H.wh_albajar_work.argtypes = [C.c_int] + [_dp] * 6 + [C.c_int, C.POINTER(C.c_uint)]
    H.wh_set_negl_skip.argtypes = [C.c_int]
    t, w = np.polynomial.legendre.leggauss(24)
    skipped = early = 0
    for pts, mode in ((rows, 1), (g[g[:, 6] == 1][:, :6], 1), (g[g[:, 6] == -1][:, :6], -1)):
        n = len(pts)
        cols = [np.ascontiguousarray(pts[:, k]) for k in range(6)]
        out = {}
        for on in (1, 0):
            a = np.zeros(n)
            H.wh_albajar(n, *[_d(c) for c in cols], mode, _d(t), _d(w), 24, _d(a))  # sets up the table
            H.wh_set_negl_skip(on)
            H.wh_albajar(n, *[_d(c) for c in cols], mode, _d(t), _d(w), 24, _d(a))
            wk = np.zeros(3 * n, dtype=np.uint32)
            H.wh_albajar_work(n, *[_d(c) for c in cols], mode, wk.ctypes.data_as(C.POINTER(C.c_uint)))
            out[on] = (a, wk.reshape(-1, 3))
        assert np.array_equal((out[1][0] + 0.0).view(np.int64), (out[0][0] + 0.0).view(np.int64))
        assert out[0][1][:, 2].sum() == 0 and (out[0][1][:, 1] >> 8).sum() == 0
        # every skipped integral is one the no-skip run evaluated; a call settled
        # early is one whose harmonics the no-skip run found exactly zero or never
        # reached (the polarisation's own early returns: N_par^2 >= 1, X >= 1 ...)
        assert out[1][1][:, 0].sum() + out[1][1][:, 2].sum() == out[0][1][:, 0].sum()
        on_zero, on_early = out[1][1][:, 1] & 0xFF, out[1][1][:, 1] >> 8
        assert np.all(on_zero + np.minimum(on_early, out[0][1][:, 1]) == out[0][1][:, 1])
        assert np.all(out[0][1][on_early > 0, 0] == 0)
        assert np.all(out[1][0][on_early > 0] == 0.0)
        skipped += int(out[1][1][:, 2].sum())
        early += int((on_early > 0).sum())
    H.wh_set_negl_skip(1)
    assert skipped > 0.2 * len(rows)
    assert early > 0.1 * len(rows)


@pytest.mark.parametrize("scale", [1e-170, 1e-160, 1e-3, 1.0, 1e3, 1e160, 1e170, 1e300])
def test_csqrt_extreme_magnitudes(H, scale):
    """warmdisp's complex square root (csqrt_) over |z| from 1e-170 to 1e300:
    where |z|^2 underflows or overflows it falls back to hypot, so near mode
    coupling (rr -> 0) the root stays small and finite, and matches numpy's
    principal branch to ~2 ulp everywhere, including re == 0 with a tiny im."""
    rng = np.random.default_rng(11)
    n = 2000
    ang = rng.uniform(-np.pi, np.pi, n)
    re, im = scale * np.cos(ang), scale * np.sin(ang)
    re[:4], im[:4] = 0.0, [scale, -scale, 0.5 * scale, 3.0 * scale]  # the pure-imaginary edge
    im[4:8], re[4:8] = 0.0, [scale, -scale, 2.0 * scale, -0.25 * scale]
    ore, oim = np.zeros(n), np.zeros(n)
    H.wh_csqrt(n, _d(re), _d(im), _d(ore), _d(oim))
    got = ore + 1j * oim
    ref = np.sqrt(re + 1j * im)
    assert np.isfinite(got).all()
    assert (np.abs(got - ref) / np.abs(ref)).max() <= 4e-16, scale
