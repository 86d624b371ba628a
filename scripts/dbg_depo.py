import sys, os, numpy as np
sys.path.insert(0, 'torj.jl_amd'); sys.path.insert(0, 'oracle')
import torj_hip as T, oracle as O
from torj_hip import synthetic as S
eq = S.circular_tokamak(); P = T.Plasma(*S.plasma_args(eq)); OP = O.OraclePlasma(*S.plasma_args(eq))
T.abs_Al_init(24); O.abs_al_init(24)
s = S.SETUP
N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], 0.0)
pos, dirs, w = T.launch_peripheral_rays([2.5,0,0.4], N0, s["spot_size"], s["inverse_curvature_radius"], 92.5e9, N_rings=14, min_azimuthal_points=5)
om = 2*np.pi*92.5e9
xp, Np, s0, st = T.ray_entry(P, pos, dirs, om, 1)
idx = np.arange(0, len(w), 4); grid = np.linspace(0,1,1000)
o = OP.trace(xp[idx], Np[idx], om, 1, 1e-4, 2000, psi_grid=grid, weights=w[idx])
for ray_sel in (idx, idx[:1], idx[5:6]):
    g = T.trace(P, xp[ray_sel], Np[ray_sel], om, 1, ds=1e-4, n_steps=2000, psi_grid=grid, weights=w[ray_sel])
    oo = OP.trace(xp[ray_sel], Np[ray_sel], om, 1, 1e-4, 2000, psi_grid=grid, weights=w[ray_sel])
    d = np.abs(g.dP_shell[:-1] - oo["dP"]); j = d.argmax()
    print(os.environ.get("TORJ_SCHED"), len(ray_sel), "maxdiff", d.max(), "at", j, g.dP_shell[j], oo["dP"][j], "Pdep diff", np.abs(g.P_dep-oo["Pdep"]).max(), "sum", g.dP_shell[:-1].sum()-oo["dP"].sum())
