#!/usr/bin/env python3
"""Optical depths of the C3 beam that the 1e-10 bar cannot resolve unfloored:
the GPU trace of the whole fan against the oracle on the bench's evenly spaced
sample (n_sample rays), the rays with tau_cpu >= 1e-12 whose relative tau
difference exceeds 1e-10, and for every sampled ray with tau_cpu >= 1e-12 the
oracle's a-priori sensitivity (or_albajar_sensitivity: tau's change when each
stage point's alpha inputs move by 2^-45 relative, from the trajectory alone).
A ray is flagged when that change exceeds half the bar, as the C5 line flags
(bench.py).  Also the fused one-lane kernel's tau for the out-of-bar rays.
usage: python tools/c3_tau_diag.py [n_sample]   (GPU box; JSON on stdout)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import torj_hip as T  # noqa: E402
from torj_hip import synthetic as S  # noqa: E402


def main():
    n_sample = int(sys.argv[1]) if len(sys.argv) > 1 else 4224
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
    g = T.trace(P, xp, Np, om, 1, ds=1e-4, n_steps=2000)
    idx = np.linspace(0, len(w) - 1, num=n_sample, dtype=int)
    OP = O.OraclePlasma(*S.plasma_args(eq))
    O.abs_al_init(24)
    th = O.default_threads()
    r = OP.trace(xp[idx], Np[idx], om, 1, 1e-4, 2000, absorption=1, n_threads=th)
    tg, tc = g.state[idx, 6], r["state"][:, 6]
    rel = np.abs(tg - tc) / np.maximum(np.abs(tc), 1e-300)
    res = np.abs(tc) >= 1e-12
    bad = res & (rel > 1e-10)
    t0 = time.perf_counter()
    sens = np.full(len(idx), np.nan)
    sens[res] = OP.albajar_sensitivity(xp[idx][res], Np[idx][res], om, 1, 1e-4, r["steps"][res],
                                       n_threads=th)
    t_sens = time.perf_counter() - t0
    flagged = res & ~(sens <= 0.5e-10 * np.abs(tc))
    # the fused one-lane kernel on the out-of-bar rays (same alpha code, compiled out of line)
    fused = None
    if bad.any():
        try:
            P.set_sched(0, 0)
            gf = T.trace(P, xp[idx[bad]], Np[idx[bad]], om, 1, ds=1e-4, n_steps=2000)
        finally:
            P.set_sched(-1)
        fused = gf.state[:, 6]
    out = {
        "rays_sampled": int(len(idx)), "rays_tau_resolvable": int(res.sum()),
        "rays_out_of_bar_resolvable": int(bad.sum()),
        "max_rel_tau_resolvable": float(rel[res].max()),
        "rays_flagged": int(flagged.sum()),
        "rays_out_of_bar_unflagged": int((bad & ~flagged).sum()),
        "max_rel_tau_resolvable_unflagged": float(rel[res & ~flagged].max()) if (res & ~flagged).any() else None,
        "sensitivity_seconds": t_sens,
        "sens_over_tau_quantiles": {q: float(np.quantile((sens / np.abs(tc))[res], q))
                                    for q in (0.5, 0.9, 0.99, 1.0)},
        "out_of_bar": [
            {"fan_index": int(idx[k]), "tau_cpu": float(tc[k]), "tau_gpu": float(tg[k]),
             "rel": float(rel[k]), "sens_over_tau": float(sens[k] / abs(tc[k])),
             "flagged": bool(flagged[k]),
             "tau_gpu_fused": None if fused is None else float(fused[j])}
            for j, k in enumerate(np.nonzero(bad)[0])][:64],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
