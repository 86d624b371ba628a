"""Beam launch (src/launch.jl) and steering-angle conversion (IMAS convention)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import TorjError, check, dptr, f64, lib


def pol_tor_angles_2_vector(steering_angle_pol: float, steering_angle_tor: float) -> np.ndarray:
    """IMAS.pol_tor_angles_2_vector as used by make_beam (src/solve.jl:211)."""
    N = np.zeros(3)
    lib().torj_pol_tor_angles_2_vector(float(steering_angle_pol), float(steering_angle_tor), dptr(N))
    return N


def launch_peripheral_rays(x0, N0, w: float, inverse_curvature_radius: float, f: float, *,
                           N_rings: int = 3, min_azimuthal_points: int = 5,
                           normalize_weight_sum: bool = True, **kwargs):
    """launch_peripheral_rays (src/launch.jl:24-132) -> (ray_positions (n,3),
    ray_directions (n,3), ray_weights (n,))."""
    x0, N0 = f64(x0), f64(N0)
    n = C.c_int()
    rc = lib().torj_launch_peripheral_rays(dptr(x0), dptr(N0), w, inverse_curvature_radius, f,
                                           N_rings, min_azimuthal_points,
                                           int(normalize_weight_sum), C.byref(n), None, None, None)
    if rc != 0:
        msg = lib().torj_last_error().decode()
        if msg.startswith("ArgumentError"):
            raise ValueError(msg)
        raise TorjError(msg)
    n = n.value
    pos, dirs, wts = np.zeros((3, n)), np.zeros((3, n)), np.zeros(n)
    check(lib().torj_launch_peripheral_rays(dptr(x0), dptr(N0), w, inverse_curvature_radius, f,
                                            N_rings, min_azimuthal_points,
                                            int(normalize_weight_sum), None, dptr(pos), dptr(dirs),
                                            dptr(wts)))
    return pos.T.copy(), dirs.T.copy(), wts
