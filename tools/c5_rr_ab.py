#!/usr/bin/env python3
"""R6 A/B: does warmdisp's discriminant in twice the working precision (Dot2,
torj_warm.hpp TORJ_WARM_RR_COMP) bring the product's weakly relativistic
alpha onto the 50-digit branch where C5's optical depths disagree?

For the given rays of the C5 fan (default: the evidence rays 94302 and
89686 of profiles/r03/c5_conditioning_evidence.json) this traces each ray
with the C oracle recording every RK4 stage point's alpha inputs
(tools/c5_conditioning.py), then evaluates alpha there with the product's
warm code on the host (tests/native: libwarm_host.so as shipped and
libwarm_host_rrc.so with the Dot2 discriminant), the C oracle and the 50-digit
mpmath restatement, and sums each into tau with the RK4 weights.  Besides
tau, per variant: the stage points whose alpha is off the 50-digit value by
more than 1e-3 relative (a different root of warmdisp), and at the worst of
them the root selector's margin -- |Re rr| or |Im rr| over |rr| in double
(warm_ref's `margin`).  Test infrastructure / analysis only; JSON on stdout.

With --flagged: the flagged rays the round-4 C5 bench line lists
(profiles/r04/bench_c5.json), product against product-with-Dot2 only (no
50-digit values): whether the compensated discriminant changes any ray's tau.

usage: python tools/c5_rr_ab.py [fan_index ...] | --flagged"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import c5_conditioning as CC  # noqa: E402

O, warm_mp, warm_ref = CC.O, CC.warm_mp, CC.warm_ref


def host(name):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "build/" + name])
    H = C.CDLL(os.path.join(ROOT, "tests", "native", "build", name))
    dp = C.POINTER(C.c_double)
    H.wh_alpha_warm.argtypes = [C.c_int] + [dp] * 7 + [C.c_int, C.c_int, dp, dp]
    return H


def host_alpha(H, pts):
    n = len(pts)
    cols = [np.ascontiguousarray(pts[:, k]) for k in range(7)]
    dp = C.POINTER(C.c_double)
    out, n2 = np.zeros(n), np.zeros(2 * n)
    H.wh_alpha_warm(n, *[c.ctypes.data_as(dp) for c in cols], 1, 1, out.ctypes.data_as(dp), n2.ctypes.data_as(dp))
    return out


def flagged():
    d = json.load(open(os.path.join(ROOT, "profiles", "r04", "bench_c5.json")))
    idxs = d["parity"]["conditioning"]["flagged_fan_indices"]
    OP, P, T, pos, dirs, om = CC.fan()
    Hs = {"product": host("libwarm_host.so"), "product_dot2_rr": host("libwarm_host_rrc.so")}
    rows = []
    for idx in idxs:
        xp, Np, s0, st = T.ray_entry(P, pos[idx][None], dirs[idx][None], om, 1)
        r, pts = CC.record_ray(OP, xp[0], Np[0], om)
        steps = int(r["steps"][0])
        a, b = (host_alpha(H, pts) for H in Hs.values())
        ta, tb = CC.tau_of(a, steps), CC.tau_of(b, steps)
        rows.append({"fan_index": int(idx), "tau_product": float(ta), "tau_product_dot2_rr": float(tb),
                     "rel_diff": float(abs(ta - tb) / max(abs(ta), 1e-300)),
                     "points_differing_1e-12": int((np.abs(a - b) > 1e-12 * np.maximum(np.abs(a), 1e-300)).sum()),
                     "tau_oracle": float(r["state"][0, 6])})
    print(json.dumps({"rays": len(rows), "max_rel_diff": max(r["rel_diff"] for r in rows),
                      "rays_differing_1e-10": int(sum(r["rel_diff"] > 1e-10 for r in rows)),
                      "per_ray": rows}, indent=1))


def main():
    if sys.argv[1:] == ["--flagged"]:
        return flagged()
    idxs = [int(a) for a in sys.argv[1:]] or [94302, 89686]
    OP, P, T, pos, dirs, om = CC.fan()
    Hs = {"product": host("libwarm_host.so"), "product_dot2_rr": host("libwarm_host_rrc.so")}
    out = []
    for idx in idxs:
        xp, Np, s0, st = T.ray_entry(P, pos[idx][None], dirs[idx][None], om, 1)
        r, pts = CC.record_ray(OP, xp[0], Np[0], om)
        steps = int(r["steps"][0])
        vals = {k: host_alpha(H, pts) for k, H in Hs.items()}
        vals["oracle"] = pts[:, 7]
        t0 = time.time()
        mp50 = np.array([float(warm_mp.alpha_warm_wr(*p[:7], 1)) for p in pts])
        t_mp = time.time() - t0
        rec = {"fan_index": idx, "steps": steps, "mp50_seconds": t_mp,
               "tau": {"mp50": CC.tau_of(mp50, steps)}, "tau_rel_err_vs_mp50": {},
               "points_off_branch": {}, "worst": {}}
        for k, v in vals.items():
            tau = CC.tau_of(v, steps)
            rec["tau"][k] = tau
            rec["tau_rel_err_vs_mp50"][k] = abs(tau - rec["tau"]["mp50"]) / abs(rec["tau"]["mp50"])
            err = np.abs(v - mp50) / np.maximum(np.abs(mp50), 1e-300)
            off = np.nonzero(err > 1e-3)[0]
            rec["points_off_branch"][k] = int(len(off))
            w = int(np.argmax(err))
            info = {}
            warm_ref.alpha_warm(*pts[w, :7], 1, 1, info=info)
            rec["worst"][k] = {"stage_index": w, "rel_err": float(err[w]), "Y": float(pts[w, 2]),
                               "Te_eV": float(pts[w, 5]), "N_par": float(pts[w, 4]),
                               "selector_margin_double": float(info.get("margin", np.nan))}
        out.append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
