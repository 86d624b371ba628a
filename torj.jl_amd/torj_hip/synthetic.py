"""Synthetic circular-tokamak equilibrium used by the GPU configs.

Produces exactly the inputs of TorJ's `Plasma(R_coords, Z_coords, psi_norm_data,
psi_prof, ne_prof, Te_prof, Br_data, Bz_data, Bϕ_data, eqt1d_psi_norm,
eqt1d_volume)` constructor (src/plasma.jl:30-32), so the spline path is exercised
exactly as with an IMAS equilibrium.  All arrays are (nR, nZ) like Julia
matrices.  Pure numpy (input generation, not physics of the path).
"""
from __future__ import annotations

import numpy as np

R0 = 1.7      # major radius [m]
A_MINOR = 0.6  # minor radius [m]
B0 = 2.05     # toroidal field on axis [T] (X2 resonance at 92.5 GHz: R ≈ 2.11 m)
PSI_A = 0.105  # poloidal flux at the edge [Wb/rad] (q_edge ≈ 3)


def circular_tokamak(nR: int = 56, nZ: int = 56, n_prof: int = 101, n_eq: int = 101,
                     ne0: float = 3e19, ne_edge: float = 1e17, Te0: float = 3000.0,
                     Te_edge: float = 30.0, ne_scale: float = 1.0,
                     R_range=(1.0, 2.6), Z_range=(-0.8, 0.8)):
    R = np.linspace(R_range[0], R_range[1], nR)
    Z = np.linspace(Z_range[0], Z_range[1], nZ)
    RR, ZZ = np.meshgrid(R, Z, indexing="ij")
    psi_norm = ((RR - R0) ** 2 + ZZ ** 2) / A_MINOR ** 2
    # Psi = PSI_A * psi_norm; B_R = -(1/R) dPsi/dZ, B_Z = (1/R) dPsi/dR
    Br = -(PSI_A / RR) * 2.0 * ZZ / A_MINOR ** 2
    Bz = (PSI_A / RR) * 2.0 * (RR - R0) / A_MINOR ** 2
    Bphi = B0 * R0 / RR
    psi_prof = np.linspace(0.0, 1.0, n_prof)
    ne_prof = ne_scale * (ne0 * (1.0 - psi_prof) + ne_edge)
    Te_prof = Te0 * (1.0 - psi_prof) ** 2 + Te_edge
    eq_psi = np.linspace(0.0, 1.0, n_eq)
    eq_vol = 2.0 * np.pi ** 2 * R0 * A_MINOR ** 2 * eq_psi
    return dict(R_coords=R, Z_coords=Z, psi_norm_data=psi_norm, psi_prof=psi_prof,
                ne_prof=ne_prof, Te_prof=Te_prof, Br_data=Br, Bz_data=Bz, Bphi_data=Bphi,
                eqt1d_psi_norm=eq_psi, eqt1d_volume=eq_vol)


def plasma_args(eq: dict):
    """Positional argument tuple in `Plasma(...)` order."""
    return (eq["R_coords"], eq["Z_coords"], eq["psi_norm_data"], eq["psi_prof"], eq["ne_prof"],
            eq["Te_prof"], eq["Br_data"], eq["Bz_data"], eq["Bphi_data"], eq["eqt1d_psi_norm"],
            eq["eqt1d_volume"])


# test/tests/setup.jl:64-80 launch geometry
SETUP = dict(f=85.5e9, f_abs_test=92.5e9, R0=2.5, phi0=0.0, z0=0.4, spot_size=0.0174,
             inverse_curvature_radius=1.0 / 3.99, steering_angle_pol=np.deg2rad(30.0),
             steering_angle_tor=0.0)
