#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.json).

Inputs and expected outputs come from the CPU restatement of the reference
(oracle/torj_oracle.c) on the synthetic equilibrium, cross-checked here against
independent libraries where one exists (numpy Gauss quadratures, scipy Bessel
functions and natural cubic splines).  The reference's only data-free known
answer (test/tests/test_launch_weights.jl:42-50) is recorded as such.
Regenerate with:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))

import oracle as O  # noqa: E402
from torj_hip import synthetic as S  # noqa: E402


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
        f.write("\n")


def main():
    rng = np.random.default_rng(20251015)
    O.abs_al_init(24)
    eq = S.circular_tokamak()
    P = O.OraclePlasma(*S.plasma_args(eq))
    s = S.SETUP

    # --- quadrature + launch (the reference's own data-free known answer) ---
    x, w = O.gauss_legendre(24)
    xr, wr = np.polynomial.legendre.leggauss(24)
    assert np.abs(x - xr).max() < 1e-15 and np.abs(w - wr).max() < 1e-15
    pos, dirs, wts = O.launch_peripheral_rays([0, 0, 0], [0, 0, 1.0], s["spot_size"],
                                              s["inverse_curvature_radius"], s["f_abs_test"],
                                              N_rings=21, min_azimuthal_points=11,
                                              normalize_weight_sum=False)
    N0 = O.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    p46, d46, w46 = O.launch_peripheral_rays([s["R0"], 0, s["z0"]], N0, s["spot_size"],
                                             s["inverse_curvature_radius"], s["f_abs_test"])
    dump("launch.json", {
        "source": "oracle (src/launch.jl restatement); KAT from test/tests/test_launch_weights.jl:42-50",
        "gl24_nodes": x.tolist(), "gl24_weights": w.tolist(),
        "kat_21_11": {"n_rays": len(wts), "weight_sum": float(wts.sum()), "tolerance_rel": 0.01},
        "default_fan": {"x0": [s["R0"], 0, s["z0"]], "N0": N0.tolist(), "n_rays": len(w46),
                        "positions": p46.tolist(), "directions": d46.tolist(),
                        "weights": w46.tolist()},
    })

    # --- field evaluations (test_trajectory.jl analogue) ---
    R = rng.uniform(0.9, 2.7, 64)
    Z = rng.uniform(-0.9, 0.9, 64)
    ph = rng.uniform(-0.5, 0.5, 64)
    pts = np.stack([R * np.cos(ph), R * np.sin(ph), Z], 1)
    Ns = rng.normal(size=(64, 3)) * 0.5
    om = 2 * np.pi * s["f_abs_test"]
    rows = []
    for p, N in zip(pts, Ns):
        X, Y, Npar, b = P.eval_plasma(p, N, om)
        rows.append({"x": p.tolist(), "N": N.tolist(), "B": P.B_spline(p).tolist(), "ne": P.n_e(p),
                     "Te": P.T_e(p), "psi": P.evaluate("psi", p), "X": X, "Y": Y, "Npar": Npar,
                     "b": b.tolist()})
    dump("fields.json", {"source": "oracle, synthetic circular tokamak (torj_hip.synthetic defaults)",
                         "omega": om, "points": rows})

    # --- dispersion / gradΛ / α at in-plasma states ---
    st, xp, Np, s0 = P.ray_entry([s["R0"], 0, s["z0"]], N0, om, 1)
    states = []
    cur_x, cur_N = xp.copy(), Np.copy()
    for k in range(20):
        rr = P.trace(cur_x[None], cur_N[None], om, 1, 1e-4, 100, absorption=False)
        cur_x, cur_N = rr["state"][0, :3], rr["state"][0, 3:6]
        for mode in (1, -1):
            states.append({"x": cur_x.tolist(), "N": cur_N.tolist(), "mode": mode,
                           "D": P.dispersion_relation(cur_x, cur_N, om, mode),
                           "du": P.grad_lambda(cur_x, cur_N, om, mode).tolist(),
                           "alpha": P.alpha_approx(cur_x, cur_N, om, mode)})
    dump("dispersion.json", {"source": "oracle (dual-number ForwardDiff restatement)", "omega": om,
                             "states": states})

    # --- Albajar α on a parameter sweep incl. the reference's edge branches ---
    from scipy.special import jv  # noqa: F401 (independent Bessel check in the tests)
    tup = []
    for _ in range(300):
        X = rng.uniform(0.0, 1.2)
        Y = rng.uniform(0.3, 1.1)
        Nabs = rng.uniform(0.2, 1.1)
        th = rng.uniform(0.02, np.pi - 0.02)
        Te = float(np.exp(rng.uniform(np.log(5.0), np.log(20000.0))))
        mode = int(rng.choice([-1, 1]))
        tup.append([om, X, Y, Nabs, Nabs * np.cos(th), Te, mode])
    # quasi-perpendicular (cos^2 theta < 1e-5) and near-parallel branches
    for mode in (1, -1):
        for c in (0.0, 1e-3, -2e-3, 0.9999999):
            tup.append([om, 0.3, 0.55, 0.9, 0.9 * c, 2000.0, mode])
    for t in tup:
        t.append(O.abs_albajar_fast(*t))
    dump("albajar.json", {"source": "oracle (libm jn Bessel), GL-24",
                          "columns": ["omega", "X", "Y", "N_abs", "N_par", "Te", "mode", "alpha"],
                          "rows": tup})

    # --- rays: entry + 2000-step traces with deposition ---
    pos, dirs, wr_ = O.launch_peripheral_rays([s["R0"], 0, s["z0"]], N0, s["spot_size"],
                                              s["inverse_curvature_radius"], s["f_abs_test"],
                                              N_rings=4, min_azimuthal_points=4)
    idx = np.linspace(0, len(wr_) - 1, 16).astype(int)
    grid = np.linspace(0, 1, 1000)
    rays = {}
    for mode in (1, -1):
        ent = [P.ray_entry(pos[i], dirs[i], om, mode) for i in idx]
        xs = np.array([e[1] for e in ent])
        Nsn = np.array([e[2] for e in ent])
        t = P.trace(xs, Nsn, om, mode, 1e-4, 2000, psi_grid=grid, weights=wr_[idx], traj_stride=200)
        nz = np.flatnonzero(t["dP"])
        rays[str(mode)] = {
            "launch_pos": pos[idx].tolist(), "launch_dir": dirs[idx].tolist(),
            "weights": wr_[idx].tolist(),
            "entry_status": [int(e[0]) for e in ent], "x0": xs.tolist(), "N0": Nsn.tolist(),
            "s0": [e[3] for e in ent],
            "state": t["state"].tolist(), "status": t["status"].tolist(),
            "steps": t["steps"].tolist(), "Pdep": t["Pdep"].tolist(),
            "dP_index": nz.tolist(), "dP_value": t["dP"][nz].tolist(),
            "traj": t["traj"].tolist(),
        }
    dump("rays.json", {"source": "oracle fixed-step RK4, ds=1e-4, 2000 steps, GL-24, psi grid "
                                 "linspace(0,1,1000), chunk 20", "omega": om, "ds": 1e-4,
                       "n_steps": 2000, "rays": rays})


if __name__ == "__main__":
    main()
