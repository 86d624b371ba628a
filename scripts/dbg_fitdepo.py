"""Print the achieved GPU-vs-FITPACK deposition errors (diagnostic)."""
import sys, os, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'torj.jl_amd')); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import torj_hip as T, oracle as O, deposition_ref as D
from torj_hip import synthetic as S
eq = S.circular_tokamak(); P = T.Plasma(*S.plasma_args(eq)); OP = O.OraclePlasma(*S.plasma_args(eq))
T.abs_Al_init(24); O.abs_al_init(24)
s = S.SETUP; f = s["f_abs_test"]; om = 2 * np.pi * f
N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0, s["z0"]], N0, s["spot_size"], s["inverse_curvature_radius"], f, N_rings=3)
for mode in (1, -1):
    xp, Np, s0, st = T.ray_entry(P, pos, dirs, om, mode)
    grid = np.linspace(0, 1, 250)
    g = T.trace(P, xp, Np, om, mode, n_steps=3000, psi_grid=grid, weights=w, deposition="reference", x_launch=pos, s0=s0)
    o = OP.trace(xp, Np, om, mode, 1e-4, 3000, psi_grid=grid, weights=w, samples=True, s0=s0)
    dV = np.diff([OP.volume(p) for p in grid]); shell = np.zeros(len(grid) - 1); Pr = np.zeros(len(w))
    for i in range(len(w)):
        sv, psi, dpds = D.ray_vectors(pos[i], s0[i], 1e-4, o["steps"][i], o["samples"][i], OP.evaluate("psi", pos[i]))
        prof, Pr[i] = D.power_deposition_profile(sv, psi, dpds, grid, OP.volume)
        shell += w[i] * prof[:-1] * dV
    print("mode", mode, "shell err / max", np.abs(g.dP_shell[:-2] - shell).max() / np.abs(shell).max(),
          "P err", np.abs(g.P_dep - Pr).max() / Pr.max(), "P", Pr[:3], "binned-vs-ref total", g.dP_shell[-1])
