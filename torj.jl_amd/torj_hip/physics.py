"""Dispersion relation (src/dispersion.jl) and EC absorption (src/absorption.jl) on the GPU."""
from __future__ import annotations

import numpy as np

from ._lib import check, dptr, f64, lib, soa


def abs_Al_init(N_absz: int):
    """abs_Al_init(N_absz) (src/absorption.jl:1-7): Gauss-Legendre order of the
    resonance-ellipse integral.  Process-global, like the reference's module globals."""
    check(lib().torj_abs_al_init(int(N_absz)))


def abs_Albajar_fast(omega, X, Y, N_abs, N_par, Te, mode: int):
    """abs_Albajar_fast(omega, X, Y, N_abs, N_par, Te, mode) (src/absorption.jl:191-226).
    Scalars or equal-length arrays (batched on the GPU)."""
    scalar = np.ndim(X) == 0
    arrs = np.broadcast_arrays(*[np.atleast_1d(f64(a)) for a in (omega, X, Y, N_abs, N_par, Te)])
    arrs = [np.ascontiguousarray(a) for a in arrs]
    n = len(arrs[0])
    out = np.zeros(n)
    check(lib().torj_abs_albajar_fast(n, *[dptr(a) for a in arrs], int(mode), dptr(out)))
    return float(out[0]) if scalar else out


def alpha_warm(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode: int, iwarm: int = 3):
    """Warm-plasma absorption coefficient alpha (src/general_absorption.jl:1328-1337, the
    repaired module -- DESIGN.md section C5): iwarm 1 weakly relativistic, 3 fully
    relativistic; inv_dDdN = 1 / |dD/dN| of the cold ray Hamiltonian.
    Returns (alpha [1/m], N_perp^2) with N_perp^2 the complex warm root."""
    scalar = np.ndim(X) == 0
    arrs = np.broadcast_arrays(*[np.atleast_1d(f64(a))
                                 for a in (omega, X, Y, N_abs, N_par, Te, inv_dDdN)])
    arrs = [np.ascontiguousarray(a) for a in arrs]
    n = len(arrs[0])
    out = np.zeros(n)
    npr = np.zeros(2 * n)
    check(lib().torj_alpha_warm(n, *[dptr(a) for a in arrs], int(mode), int(iwarm), dptr(out),
                                dptr(npr)))
    n2 = npr[0::2] + 1j * npr[1::2]
    return (float(out[0]), complex(n2[0])) if scalar else (out, n2)


def refractive_index_sq(X, Y, N_par, mode: int):
    """refractive_index_sq(X, Y, N_par, mode) (src/dispersion.jl:29-32)."""
    scalar = np.ndim(X) == 0
    arrs = [np.ascontiguousarray(a) for a in
            np.broadcast_arrays(*[np.atleast_1d(f64(a)) for a in (X, Y, N_par)])]
    n = len(arrs[0])
    out = np.zeros(n)
    check(lib().torj_refractive_index_sq(n, *[dptr(a) for a in arrs], int(mode), dptr(out)))
    return float(out[0]) if scalar else out


def _disp(plasma, x, N, omega, mode, want_alpha):
    xs, Ns = soa(x), soa(N)
    n = xs.shape[1]
    D = np.zeros(n)
    du = np.zeros((6, n))
    al = np.zeros(n) if want_alpha else None
    check(lib().torj_dispersion(plasma.handle, n, dptr(xs), dptr(Ns), float(omega), int(mode),
                                dptr(D), dptr(du), dptr(al)))
    return D, du, al


def dispersion_relation(x, N, plasma, omega: float, mode: int):
    """dispersion_relation(x, N, plasma, omega, mode) (src/dispersion.jl:34-39)."""
    D, _, _ = _disp(plasma, x, N, omega, mode, False)
    return float(D[0]) if np.ndim(x) == 1 else D


def gradΛ(plasma, x, N, omega: float, mode: int):
    """Normalised Hamiltonian RHS of gradΛ! (src/solve.jl:85-93): (dx/ds, dN/ds)."""
    _, du, _ = _disp(plasma, x, N, omega, mode, False)
    return du[:, 0].copy() if np.ndim(x) == 1 else du.T.copy()


grad_lambda = gradΛ


def α_approx(x, N, plasma, omega: float, mode: int):
    """α_approx(x, N, plasma, omega, mode) (src/absorption.jl:228-235)."""
    _, _, al = _disp(plasma, x, N, omega, mode, True)
    return float(al[0]) if np.ndim(x) == 1 else al


alpha_approx = α_approx
