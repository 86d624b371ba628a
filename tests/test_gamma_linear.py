"""The node loop's gamma as the resonance condition's linear form (round 6,
torj.jl_amd/csrc/torj_math.hpp harm_geom / pair_term, TORJ_NODE_GAMMA_LIN).

The reference evaluates gamma = sqrt(1 + u_par^2 + u_perp^2) on the
parametrisation u_par = (r N_par + sqrt(r^2 - 1) t) / sqrt(1 - N_par^2),
u_perp^2 = (r^2 - 1)(1 - t^2) of the resonance ellipse, r = m / m_0
(src/absorption.jl:176-179).  The ellipse is the square of gamma = m Y + N_par u_par,
so gamma(t) = (r + N_par sqrt(r^2 - 1) t) / sqrt(1 - N_par^2).  These tests hold
the identity in 40-digit arithmetic, and both double-precision forms within a
few ulp of the exact gamma (CPU only; the GPU path is held to the oracle by
tests/test_gpu_parity.py)."""
import numpy as np
import pytest

mp = pytest.importorskip("mpmath")


def _inputs(n, seed):
    rng = np.random.default_rng(seed)
    Y = rng.uniform(0.3, 1.2, n)
    Npar = rng.uniform(-0.9, 0.9, n)
    m = rng.choice([2, 3], n)
    t = rng.uniform(-1.0, 1.0, n)
    m0 = np.sqrt(1.0 - Npar ** 2) / Y
    ok = m >= m0  # harmonic present (src/absorption.jl:213-216)
    return Y[ok], Npar[ok], m[ok], t[ok]


def test_linear_gamma_is_the_reference_gamma_exactly():
    mp.mp.dps = 40
    for Y, Npar, m, t in zip(*_inputs(300, 1)):
        Ym, Nm, T = mp.mpf(Y), mp.mpf(Npar), mp.mpf(t)
        sq = mp.sqrt(1 - Nm ** 2)
        r = m * Ym / sq
        upar = (r * Nm + mp.sqrt(r * r - 1) * T) / sq
        g_ref = mp.sqrt(1 + upar ** 2 + (r * r - 1) * (1 - T * T))
        g_lin = (r + Nm * mp.sqrt(r * r - 1) * T) / sq
        assert abs(g_ref - g_lin) <= mp.mpf(10) ** -35 * g_ref
        assert g_lin >= 1  # positive over the whole ellipse


def test_linear_gamma_in_double_within_a_few_ulp():
    mp.mp.dps = 40
    e_ref, e_lin = [], []
    for Y, Npar, m, t in zip(*_inputs(3000, 2)):
        # the product's double arithmetic (harm_geom): r = m Y / sqrt(1 - N_par^2)
        isq = 1.0 / np.sqrt(1.0 - Npar * Npar)
        r = m * (isq * Y)
        sq_r = np.sqrt(r * r - 1.0)
        upa0, upa1 = isq * r * Npar, isq * sq_r
        g_sqrt = np.sqrt((upa0 + upa1 * t) ** 2 + 1.0 + (r * r - 1.0) * (1.0 - t * t))
        g_lin = r * isq + (Npar * upa1) * t
        Ym, Nm, T = mp.mpf(Y), mp.mpf(Npar), mp.mpf(t)
        R = m * Ym / mp.sqrt(1 - Nm ** 2)
        ge = (R + Nm * mp.sqrt(R * R - 1) * T) / mp.sqrt(1 - Nm ** 2)
        e_ref.append(float(abs(g_sqrt - ge) / ge))
        e_lin.append(float(abs(g_lin - ge) / ge))
    ulp = np.finfo(float).eps
    assert max(e_lin) < 8 * ulp and max(e_ref) < 8 * ulp
    assert np.median(e_lin) < 1.5 * ulp
