"""Diagnostic: split path (sched 3) vs fused one-lane kernel, per-output differences."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
torch.cuda.init()
import torj_hip as T
from torj_hip import synthetic as S
T.abs_Al_init(24)
hp = T.Plasma(*S.plasma_args(S.circular_tokamak()))
s = S.SETUP
N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"], s["inverse_curvature_radius"], s["f_abs_test"], N_rings=14, min_azimuthal_points=5)
om = 2 * np.pi * s["f_abs_test"]
xp, Np, s0, st = T.ray_entry(hp, pos, dirs, om, 1, gpu=True)
for dep in ("none", "reference"):
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=100)
    if dep != "none":
        kw.update(psi_grid=np.linspace(0, 1, 1000), deposition=dep, x_launch=pos, s0=s0)
    res = []
    for sched in (0, 3):
        hp.set_sched(sched, 0)
        res.append(T.trace(hp, xp, Np, om, 1, **kw))
    hp.set_sched(-1)
    a, b = res
    d = np.abs(a.state - b.state)
    print(dep, "state cols differing:", [(c, int((d[:, c] > 0).sum()), float((d[:, c] / np.maximum(np.abs(a.state[:, c]), 1e-300)).max())) for c in range(7)])
    print(dep, "steps eq", np.array_equal(a.steps, b.steps), "status eq", np.array_equal(a.status, b.status), "Pdep maxrel", float(np.max(np.abs(a.P_dep - b.P_dep) / np.maximum(np.abs(a.P_dep), 1e-300))))
    fin = np.isfinite(a.traj)
    print(dep, "traj finite eq", np.array_equal(fin, np.isfinite(b.traj)), "traj max abs diff per field", [float(np.nanmax(np.abs(a.traj[..., f] - b.traj[..., f]))) for f in range(5)])
