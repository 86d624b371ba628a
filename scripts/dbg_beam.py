import os, sys, numpy as np
sys.path[:0] = ["tests", "torj.jl_amd", "oracle"]
import torch; torch.cuda.init()
import torj_hip as T
from torj_hip import synthetic as S
eq = S.circular_tokamak(); P = T.Plasma(*S.plasma_args(eq), device=0); T.abs_Al_init(24)
s = S.SETUP
N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"], s["inverse_curvature_radius"], s["f_abs_test"], N_rings=14, min_azimuthal_points=5)
om = 2 * np.pi * s["f_abs_test"]
xp, Np, s0, st = T.ray_entry(P, pos, dirs, om, 1, gpu=True)
kw = dict(ds=1e-4, n_steps=2000, psi_grid=np.linspace(0, 1, 1000), weights=w, traj_stride=100, deposition="reference", x_launch=pos, s0=s0)
P.set_sched(0)
a = T.trace(P, xp, Np, om, 1, **kw)
print("n", len(w), "s0[-2:]", s0[-2:], "a traj s0", a.traj[-2:, 0, 4])
for sync in ("0", "1"):
    os.environ["TORJ_BEAM_SYNC"] = sync
    for ns in (1, 2, 3, 4):
        b = T.trace(P, xp, Np, om, 1, n_gpus=1, n_shards=ns, **kw)
        bad = np.nonzero(~np.isclose(a.traj[:, 0, 4], b.traj[:, 0, 4], rtol=0, atol=1e-12))[0]
        print(f"sync {sync} shards {ns}: state eq {np.array_equal(a.state, b.state)} Pdep eq {np.array_equal(a.P_dep, b.P_dep)} traj eq {np.array_equal(a.traj, b.traj, equal_nan=True)} bad s rays {len(bad)} first {bad[:5]} b s {b.traj[bad[:3], 0, 4]}", flush=True)
