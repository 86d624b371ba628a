#!/usr/bin/env python3
"""Region profile of the warm alpha kernel (k_alpha_warm_pts<1>) on the C5
beam: a profiling build (python scripts/mkvariant.py wprof -DTORJ_WARM_PROF)
charges each wave's wall clock between marks to regions of the algorithm
(torj_warm.hpp TORJ_WPROF); this runs the C5 trace once through that library
and prints each region's share.
usage: TORJ_HIP_LIB=.../libtorj_hip_wprof.so python tools/warm_prof.py [n_steps]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
import torj_hip as T  # noqa: E402
from torj_hip import synthetic as S  # noqa: E402

REGIONS = ["inputs+larmornumber", "faddeeva", "l-recurrence", "ca accumulation",
           "l-factors+store", "warmdisp", "epilogue", "unused"]


def main():
    n_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    L = T.lib()
    rd = L.torj_warm_prof_read
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
    buf = (ctypes.c_ulonglong * 9)()
    T.trace(P, xp, Np, om, 1, ds=1e-4, n_steps=n_steps, absorption=2)  # warm-up
    rd(buf)
    L.torj_warm_fad_read((ctypes.c_ulonglong * 9)())
    T.trace(P, xp, Np, om, 1, ds=1e-4, n_steps=n_steps, absorption=2)
    rd(buf)
    v = np.array(buf[:], dtype=np.float64)
    fr = L.torj_warm_fad_read
    fr.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    fb = (ctypes.c_ulonglong * 9)()
    fr(fb)
    f = [int(x) for x in fb]
    tot = v[1:].sum()
    out = {"waves": int(v[0]), "rays": len(w), "n_steps": n_steps,
           "regions": {REGIONS[k]: {"ticks_per_wave": v[1 + k] / max(v[0], 1), "share": v[1 + k] / tot}
                       for k in range(8) if v[1 + k] > 0}}
    out["faddeeva_pairs"] = {"wave_calls": f[0], "wave_calls_with_weideman": f[1],
                             "lane_calls": f[2], "lane_calls_with_weideman": f[3],
                             "weideman_args_by_z2": dict(zip(["<36", "<64", "<100", "<144", "<256"], f[4:9]))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
