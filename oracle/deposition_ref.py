"""power_deposition_profile (src/plasma.jl:91-151) restated on scipy's FITPACK.

TEST INFRASTRUCTURE ONLY (the checker of the GPU's reference-faithful
deposition, torj_trace_cfg.deposition = 1); never imported by the product.

The reference fits `Dierckx.Spline1D(s, y, k=3)` (s = 0: interpolating),
finds `Dierckx.roots` and `Dierckx.integrate` -- Dierckx.jl 0.5.4
(Project.toml:33) wraps Paul Dierckx's FITPACK `curfit` / `sproot` / `splint`.
scipy.interpolate's `splrep(k=3, s=0)` / `sproot` / `splint` call the same
FITPACK routines, so this restatement is pinned to the reference's own
third-party arithmetic, not to a re-derivation.  `roots(spl; maxn=8)` is the
Dierckx.jl default (mest = 8).
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import splint, splrep, sproot


def power_deposition_profile(s, psi_s, dP_ds, psi_dP_dV, volume, maxn=8):
    """Literal restatement of src/plasma.jl:91-151.

    s, psi_s, dP_ds: the ray's arc length, psi(R(s), z(s)) and dP/ds samples
    (make_ray's vectors, incl. the vacuum launch point and the entry point);
    psi_dP_dV: shell boundaries; volume: callable V(psi) (volume_psi_spline).
    Returns (dP_dV, P) exactly as the reference (dP_dV[-1] = 0)."""
    s = np.asarray(s, dtype=float)
    psi_s = np.asarray(psi_s, dtype=float)
    grid = np.asarray(psi_dP_dV, dtype=float)
    dP_spl = splrep(s, np.asarray(dP_ds, dtype=float), k=3, s=0)   # :101
    dP_dV = np.zeros(len(grid))
    P = 0.0
    j = len(grid) - 1                                                 # :105 (0-based)
    outer_roots = list(sproot(splrep(s, psi_s - grid[j], k=3, s=0), mest=maxn))   # :106-108
    outer_volume = volume(grid[j])
    j -= 1
    while j >= 0:                                                     # :111
        inner_volume = volume(grid[j])
        dV = outer_volume - inner_volume
        inner_roots = list(sproot(splrep(s, psi_s - grid[j], k=3, s=0), mest=maxn))
        intervals = sorted(outer_roots + inner_roots)                 # :119
        if len(intervals) < 2:                                        # :120-124
            break
        elif len(intervals) % 2 != 0:                                 # :125-127
            intervals = intervals[:-1]
        dP = 0.0
        for k in range(0, len(intervals) - 1, 2):                     # :129-136
            dP += abs(splint(intervals[k], intervals[k + 1], dP_spl))
        dP_dV[j] = dP / dV                                            # :141
        P += dP
        j -= 1
        outer_volume = inner_volume
        outer_roots = inner_roots
    return dP_dV, P


def ray_vectors(x_launch, s0, ds, steps, samples, psi_launch):
    """make_ray's (s, psi_s, dP_ds) vectors for one ray from an oracle/GPU trace:
    launch point (s = 0, dP/ds = 0), entry point (s0, dP/ds = 0), then every
    RK4 step (src/solve.jl:148-172)."""
    k = int(steps)
    if samples.shape[1] > 2:  # the trace's own arc lengths (adaptive steps)
        s = np.concatenate([[0.0], samples[:k + 1, 2]])
    else:
        s = np.concatenate([[0.0, s0], s0 + ds * np.arange(1, k + 1)])
    psi = np.concatenate([[psi_launch], samples[:k + 1, 0]])
    dpds = np.concatenate([[0.0, 0.0], samples[1:k + 1, 1]])
    return s, psi, dpds
