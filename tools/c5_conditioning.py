#!/usr/bin/env python3
"""Which warm-alpha restatement is right where C5's optical depths disagree?

For chosen rays of the C5 beam (BASELINE configs[4]: the 100 203-ray fan,
X-mode 92.5 GHz, weakly relativistic alpha, 2 000 RK4 steps) this traces each
ray with the C oracle while recording every RK4 stage point's alpha inputs,
then evaluates alpha there four ways:

  * "product": torj_warm.hpp (the GPU's code, host build tests/native: Weideman's
    rational Faddeeva approximation; the device differs only by fma
    contraction),
  * "oracle":  oracle/torj_warm_oracle.c (TOMS 680, as the reference's zetac),
  * "scipy":   oracle/warm_ref.py (scipy's wofz),
  * "mp50":    oracle/warm_mp.py (mpmath, 50 digits: the algorithm's true value),

and sums each into the ray's optical depth with the RK4 weights.  Beside it,
the ray's a-priori sensitivity (oracle or_warm_sensitivity: how far tau moves
when every stage point's inputs move by 64 ulps), the flag bench.py's C5 parity
uses, and at the product's worst stage point the outcome of a one-ulp change of
Y in the C oracle.  Output: JSON on stdout.  Test infrastructure / analysis only.

usage: python tools/c5_conditioning.py [fan_index ...]"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import oracle as O  # noqa: E402
import warm_mp  # noqa: E402
import warm_ref  # noqa: E402

DS, N_STEPS = 1e-4, 2000


def host_lib():
    import subprocess

    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "build/libwarm_host.so"])
    H = C.CDLL(os.path.join(ROOT, "tests", "native", "build", "libwarm_host.so"))
    dp = C.POINTER(C.c_double)
    H.wh_alpha_warm.argtypes = [C.c_int] + [dp] * 7 + [C.c_int, C.c_int, dp, dp]
    return H


def fan():
    import torj_hip as T
    from torj_hip import synthetic as S

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
    return OP, P, T, pos, dirs, om


def record_ray(OP, xp, Np, om):
    """Trace one ray (C oracle, C warm alpha) recording each stage point's inputs."""
    pts = []

    def fn(omega, X, Y, Nabs, Npar, Te, inv, mode, model):
        a = O.alpha_warm(omega, X, Y, Nabs, Npar, Te, inv, mode, 1)[0]
        pts.append((omega, X, Y, Nabs, Npar, Te, inv, a))
        return a

    hook = O._ALPHA_FN(fn)
    install = O._install_warm_hook
    O._install_warm_hook = lambda on: O.lib().or_set_alpha_hook(hook)  # the trace installs ours
    try:
        r = OP.trace(xp[None], Np[None], om, 1, DS, N_STEPS, absorption=2, n_threads=1)
    finally:
        O._install_warm_hook = install
        O.lib().or_set_alpha_hook(None)
    return r, np.array(pts)


def tau_of(alpha, steps):
    """optical depth from the stage alphas with the RK4 weights, step by step"""
    a = alpha[: 4 * steps].reshape(steps, 4)
    tau = 0.0
    for k in range(steps):
        tau = tau + DS / 6.0 * (a[k, 0] + 2.0 * a[k, 1] + 2.0 * a[k, 2] + a[k, 3])
    return tau


def analyse(idx, OP, P, T, pos, dirs, om, H):
    xp, Np, s0, st = T.ray_entry(P, pos[idx][None], dirs[idx][None], om, 1)
    r, pts = record_ray(OP, xp[0], Np[0], om)
    steps = int(r["steps"][0])
    n = len(pts)
    cols = [np.ascontiguousarray(pts[:, k]) for k in range(7)]
    dp = C.POINTER(C.c_double)
    prod = np.zeros(n)
    n2 = np.zeros(2 * n)
    H.wh_alpha_warm(n, *[c.ctypes.data_as(dp) for c in cols], 1, 1, prod.ctypes.data_as(dp),
                    n2.ctypes.data_as(dp))
    t0 = time.time()
    mp50 = np.array([float(warm_mp.alpha_warm_wr(*p[:7], 1)) for p in pts])
    t_mp = time.time() - t0
    sci = np.array([warm_ref.alpha_warm(*p[:7], 1, 1)[0] for p in pts])
    orc = pts[:, 7]
    taus = {k: tau_of(v, steps) for k, v in (("mp50", mp50), ("product", prod), ("oracle", orc),
                                             ("scipy", sci))}
    ref = taus["mp50"]
    sens = float(OP.warm_sensitivity(xp, Np, om, 1, DS, r["steps"])[0])
    err_pt = {k: np.abs(v - mp50) / np.maximum(np.abs(mp50), 1e-300) for k, v in
              (("product", prod), ("oracle", orc), ("scipy", sci))}
    worst = int(np.argmax(np.abs(prod - mp50) * np.tile([1, 2, 2, 1], steps)[:n]))
    q = pts[worst].copy()
    q[2] = np.nextafter(q[2], 0.0)  # Y one ulp down
    flip = O.alpha_warm(*q[:7], 1, 1)[0]
    return {
        "fan_index": int(idx), "steps": steps, "status": int(r["status"][0]),
        "tau": {k: v for k, v in taus.items()},
        "tau_rel_err_vs_mp50": {k: abs(v - ref) / abs(ref) for k, v in taus.items() if k != "mp50"},
        "tau_oracle_trace": float(r["state"][0, 6]),
        "tau_sensitivity_64ulp_rel": sens / max(abs(ref), 1e-6),
        "points": n, "mp50_seconds": t_mp,
        "max_point_rel_err": {k: float(v.max()) for k, v in err_pt.items()},
        "worst_point_product": {
            "stage_index": worst, "Te_eV": float(pts[worst, 5]), "Y": float(pts[worst, 2]),
            "X": float(pts[worst, 1]), "N_par": float(pts[worst, 4]),
            "mu": float(warm_ref.ME * warm_ref.C ** 2 / (pts[worst, 5] * warm_ref.E)),
            "alpha_mp50": float(mp50[worst]),
            "rel_err": {k: float(v[worst]) for k, v in err_pt.items()},
            "oracle_alpha_Y_one_ulp_down": float(flip)},
    }


def main():
    idxs = [int(a) for a in sys.argv[1:]] or [94302, 89686]
    OP, P, T, pos, dirs, om = fan()
    O.abs_al_init(24)
    H = host_lib()
    out = [analyse(i, OP, P, T, pos, dirs, om, H) for i in idxs]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
