#!/usr/bin/env python3
"""Lane utilisation of the Albajar alpha kernel (k_alpha_pts) on the C3 beam:
a profiling build (python scripts/mkvariant.py aprof -DTORJ_ALPHA_PROF) counts,
per harmonic, the waves that run the node loop and the lanes of those waves
that need it, the waves / live lanes of the kernel, and the waves that reach
each region of abs_albajar_fast_body (Te >= 20, the polarisation prologue,
each harmonic past its exact-zero test and its skip bound).
usage: TORJ_HIP_LIB=.../libtorj_hip_aprof.so python tools/alpha_prof.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
import torj_hip as T  # noqa: E402
from torj_hip import synthetic as S  # noqa: E402


def main():
    L = T.lib()
    rd = L.torj_alpha_prof_read
    rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    eq = S.circular_tokamak()
    P = T.Plasma(*S.plasma_args(eq), device=0)
    T.abs_Al_init(24)
    s = S.SETUP
    f = 92.5e9
    om = 2 * np.pi * f
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=92,
                                            min_azimuthal_points=11)
    xp, Np, s0, st = T.ray_entry(P, pos, dirs, om, 1, gpu=True)
    buf = (ctypes.c_ulonglong * 16)()
    T.trace(P, xp, Np, om, 1, ds=1e-4, n_steps=2000)
    rd(buf)
    T.trace(P, xp, Np, om, 1, ds=1e-4, n_steps=2000)
    rd(buf)
    v = [int(x) for x in buf]
    out = {"rays": len(w), "kernel_waves": v[4], "kernel_live_lanes": v[5],
           "live_lane_fraction": v[5] / max(64 * v[4], 1)}
    for m in (2, 3):
        wv, ln = v[2 * (m - 2)], v[2 * (m - 2) + 1]
        out[f"harmonic{m}"] = {"node_loop_waves": wv, "node_loop_lanes": ln,
                               "lane_utilisation": ln / max(64 * wv, 1),
                               "waves_per_kernel_wave": wv / max(v[4], 1)}
    # waves that reached each region of abs_albajar_fast_body (per kernel wave)
    names = ["te_ge_20", "polarisation_prologue", "prologue_ok", "h2_not_zero", "h2_bound",
             "h3_not_zero", "h3_bound", "zero_flag_waves"]
    out["region_waves"] = {nm: v[6 + k] for k, nm in enumerate(names)}
    out["region_waves_per_kernel_wave"] = {nm: v[6 + k] / max(v[4], 1) for k, nm in enumerate(names)}
    # live lanes of the evaluated (not fully flagged) waves that carry a zero flag
    out["flagged_lanes_in_evaluated_waves"] = v[14]
    out["flagged_lane_fraction_of_evaluated"] = v[14] / max(v[5], 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
