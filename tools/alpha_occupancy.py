#!/usr/bin/env python3
"""How much of k_alpha_pts' SIMD width does the Albajar alpha use on the C3 beam?

Analysis only (host build of the product's alpha, tests/native; the C oracle's
trace for the stage inputs).  For G consecutive 64-ray groups of the headline
fan (the lanes of one k_alpha_pts wave: rays 64 q .. 64 q + 63 at one step and
stage), every step's point inputs (step ends, a proxy for the four stages) are
evaluated with the product's abs_Albajar_fast work counters, and the wave cost
(max over its live lanes of the lane's harmonic work) is set against the lane
work itself (sum / 64): the fraction of issued lane slots that do useful work,
and how that splits by cause (lanes settled early / not reached, harmonic count
and Bessel-level divergence).

usage: python tools/alpha_occupancy.py [n_groups] [first_group | -] [steps]"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402

_dp = C.POINTER(C.c_double)


def _d(a):
    return a.ctypes.data_as(_dp)


def main():
    n_groups = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    g0 = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    n_steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    import torj_hip as T
    from torj_hip import synthetic as S

    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "build/libwarm_host.so"])
    H = C.CDLL(os.path.join(ROOT, "tests", "native", "build", "libwarm_host.so"))
    H.wh_albajar.argtypes = [C.c_int] + [_dp] * 6 + [C.c_int, _dp, _dp, C.c_int, _dp]
    H.wh_albajar_work.argtypes = [C.c_int] + [_dp] * 6 + [C.c_int, C.POINTER(C.c_uint)]

    eq = S.circular_tokamak()
    OP = O.OraclePlasma(*S.plasma_args(eq))
    P = T.Plasma(*S.plasma_args(eq))
    s = S.SETUP
    f = s["f_abs_test"]
    om = 2 * np.pi * f
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=92,
                                            min_azimuthal_points=11)
    n_all = len(w)
    groups = (np.linspace(0, n_all // 64 - 1, n_groups).astype(int) if g0 is None
              else np.arange(g0, g0 + n_groups))
    idx = (groups[:, None] * 64 + np.arange(64)[None, :]).ravel()
    xp, Np, s0, st = T.ray_entry(P, pos[idx], dirs[idx], om, 1)
    O.abs_al_init(24)
    full = OP.trace(xp, Np, om, 1, 1e-4, n_steps)
    steps = full["steps"]
    t, wg = np.polynomial.legendre.leggauss(24)
    x, N = xp.copy(), Np.copy()
    n = len(idx)
    tot = dict(lane_slots=0, live_lanes=0, useful=0.0, wave_cost=0.0, waves=0, waves_all_early=0)
    cost_of = np.zeros(n)
    for k in range(n_steps):
        live = k < steps
        rows = np.zeros((n, 6))
        for i in range(n):
            X, Y, Npar, _ = OP.eval_plasma(x[i], N[i], om)
            rows[i] = (om, X, Y, np.linalg.norm(N[i]), Npar, OP.T_e(x[i]))
        cols = [np.ascontiguousarray(rows[:, c]) for c in range(6)]
        a = np.zeros(n)
        H.wh_albajar(n, *[_d(c) for c in cols], 1, _d(t), _d(wg), 24, _d(a))
        wk = np.zeros(3 * n, dtype=np.uint32)
        H.wh_albajar_work(n, *[_d(c) for c in cols], 1, wk.ctypes.data_as(C.POINTER(C.c_uint)))
        wk = wk.reshape(-1, 3)
        # lane cost in harmonic-evaluation units: an evaluated harmonic 1, a
        # negligible / zero one (setup and bound) 0.1, a call with neither 0.1
        cost_of = wk[:, 0] + 0.1 * (wk[:, 2] + (wk[:, 1] & 0xFF)) + 0.1
        cost_of[~live] = 0.0
        for g in range(len(groups)):
            sl = slice(64 * g, 64 * g + 64)
            if not live[sl].any():
                continue
            c = cost_of[sl]
            tot["waves"] += 1
            tot["lane_slots"] += 64
            tot["live_lanes"] += int(live[sl].sum())
            tot["useful"] += float(c.sum())
            tot["wave_cost"] += float(c.max()) * 64
            if (wk[sl, 0][live[sl]] == 0).all():
                tot["waves_all_early"] += 1
        r = OP.trace(x, N, om, 1, 1e-4, 1, chunk_steps=1, psi_exit=1e9, P_min=0.0, absorption=False)
        x, N = r["state"][:, :3].copy(), r["state"][:, 3:6].copy()
    tot["lane_efficiency"] = tot["useful"] / max(tot["wave_cost"], 1e-300)
    tot["groups"] = [int(g) for g in groups]
    tot["steps"] = n_steps
    print(json.dumps(tot, indent=1))


if __name__ == "__main__":
    main()
