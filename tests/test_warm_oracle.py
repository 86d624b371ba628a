"""Pin the warm-absorption oracle (oracle/warm_ref.py, the repaired
src/general_absorption.jl) before trusting it as the checker of absorption
models 2 and 3.

The reference module never ran, so nothing executed
can be compared with; the pins are (a) the special functions against scipy,
(b) the cold-plasma limit (mu -> inf), where the warm root must become the
ray's own cold root from refractive_index_sq (src/dispersion.jl:29-32) with
an O(1/mu) thermal correction -- on both sides of Y = 1, which is what fixes
the root selector (repair R5), and (c) the integrated second- and
third-harmonic X-mode damping against abs_Albajar_fast (src/absorption.jl:
191-226), an independent relativistic model, with the Hamiltonian's own
1 / |dD/dN| as group-velocity factor (repair R4)."""
import math
import warnings

import numpy as np
import pytest
from scipy.special import iv

OMEGA = 2 * np.pi * 140e9


@pytest.fixture(scope="module")
def W():
    import warm_ref

    return warm_ref


def _cold(O, X, Y, Npar, mode):
    """cold N^2 and 1/|dD/dN| of D = |N|^2 - refractive_index_sq (dispersion.jl:34-39)
    for N = (N_perp, 0, N_par) along b."""
    n2 = float(O.refractive_index_sq(X, Y, Npar, mode))
    h = 1e-6
    dn = (float(O.refractive_index_sq(X, Y, Npar + h, mode))
          - float(O.refractive_index_sq(X, Y, Npar - h, mode))) / (2 * h)
    nperp = math.sqrt(max(n2 - Npar * Npar, 0.0))
    return n2, 1.0 / math.hypot(2 * nperp, 2 * Npar - dn)


@pytest.mark.parametrize("z", [1e-3, 0.3, 2.0, 6.0])
def test_ssbi_is_scaled_modified_bessel(W, z):
    """R1: ssbi(z, n, l)[m - n] = I_{m+1/2}(z) / (z/2)^{m+1/2}, m = n .. l+2."""
    got = W.ssbi(z, 0, 3)
    ref = [iv(m + 0.5, z) / (z / 2) ** (m + 0.5) for m in range(6)]
    assert max(abs(a / b - 1) for a, b in zip(got, ref)) < 1e-9


def test_expei_limits(W):
    """exp(-x) Ei(x): the reference returns -xinf at 0 (general_absorption.jl:29-60);
    large-|x| asymptote 1/x."""
    assert W.expei(0.0) == -1.79e308
    for x in (200.0, -200.0):
        assert abs(W.expei(x) * x - 1) < 2e-2


def test_larmornumber_kat(W):
    """Y = 1/2, N_par = 0, mu = 1000: harmonic 2 sits at gamma = 1 (mu (gamma-1) = 0),
    harmonic 3 at gamma = 1.5 (mu (gamma-1) = 500 > 15) -> 3; hotter plasmas
    keep more harmonics."""
    assert W.larmornumber(0.5, 0.0, 1000.0) == 3
    assert W.larmornumber(0.5, 0.0, 20.0) > 3


@pytest.mark.parametrize("iwarm", [1, 3])
@pytest.mark.parametrize("mode,Y", [(1, 0.6), (1, 1.3), (-1, 0.6), (-1, 1.3)])
def test_cold_limit_recovers_ray_root(O, W, iwarm, mode, Y):
    """mu -> inf: N_perp^2 -> refractive_index_sq - N_par^2 of the SAME mode,
    with an error linear in Te (first-order thermal correction).  Y > 1 is where
    warmdisp's own root choice flips (R5)."""
    X, Npar = 0.3, 0.2
    n2, inv = _cold(O, X, Y, Npar, mode)
    cold = n2 - Npar * Npar
    errs = []
    for Te in (1.0, 10.0):
        _, anpr = W.alpha_warm(OMEGA, X, Y, math.sqrt(n2), Npar, Te, inv, mode, iwarm)
        errs.append(abs((anpr * anpr).real / cold - 1))
    assert errs[0] < 1e-4
    assert 5 < errs[1] / errs[0] < 20
    # the other mode's root is far away: the selector picked the right one
    other = float(O.refractive_index_sq(X, Y, Npar, -mode)) - Npar * Npar
    assert abs(other / cold - 1) > 1e-2


@pytest.mark.parametrize("iwarm,tol", [(3, 0.04), (1, 0.06)])
@pytest.mark.parametrize("Yc,Te", [(0.5, 1e3), (0.5, 3e3), (1 / 3, 3e3)])
def test_x_harmonic_damping_matches_albajar(O, W, iwarm, tol, Yc, Te):
    """Integral of alpha over Y across the X2 / X3 resonance vs abs_Albajar_fast
    (which covers harmonics 2 and 3, absorption.jl:213): 0.05-3 % (fully
    relativistic) -- checks the tensor, the root and alpha's normalisation (R4)."""
    X, Npar, mode = 0.3, 0.15, 1
    Ys = np.linspace(Yc - 0.04, Yc + 0.04, 81)
    aw, aa = [], []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for Y in Ys:
            n2, inv = _cold(O, X, Y, Npar, mode)
            a, _ = W.alpha_warm(OMEGA, X, Y, math.sqrt(n2), Npar, Te, inv, mode, iwarm)
            aw.append(a)
            aa.append(float(O.abs_albajar_fast(OMEGA, X, Y, math.sqrt(n2), Npar, Te, mode)))
    aw, aa = np.array(aw), np.array(aa)
    assert aw.min() >= 0.0
    ratio = np.trapezoid(aw, Ys) / np.trapezoid(aa, Ys)
    assert abs(ratio - 1) < tol, ratio


def test_o1_damping_where_albajar_has_none(O, W):
    """O-mode fundamental: abs_Albajar_fast skips harmonic 1 (absorption.jl:213),
    the warm model damps it -- the reason models 2 / 3 exist."""
    X, Npar, mode, Te = 0.3, 0.15, -1, 3e3
    tot = 0.0
    for Y in np.linspace(0.97, 1.05, 33):
        n2, inv = _cold(O, X, Y, Npar, mode)
        a, _ = W.alpha_warm(OMEGA, X, Y, math.sqrt(n2), Npar, Te, inv, mode, 3)
        assert a >= 0.0
        tot += a
        assert float(O.abs_albajar_fast(OMEGA, X, Y, math.sqrt(n2), Npar, Te, mode)) < 1e-40
    assert tot > 10.0
