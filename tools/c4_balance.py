#!/usr/bin/env python3
"""Per-shard cost of C4's strong split on one MI355X (analysis, GPU).

C4 (BASELINE configs[3]) cuts the 1 005 293-ray fan into 8 contiguous 64-ray-
aligned shards (torj_hip/parallel.py group_shard, what torj_trace_beam and
`bench.py --gpus 8 --shard` use).  Contiguous ranges follow the fan's rings,
whose absorption work differs (harmonic content, exact-zero and negligible
skips, rays that leave the plasma), so the shards need not cost the same.
This traces each shard alone on device 0 through torj_trace_beam_device (the
library path a GPU of the 8-GPU run takes: 2 000 RK4 steps, Albajar, the
reference deposition on 1 000 shells) and reports its wall time, ray-steps
and work counters: max / mean of the shard times is the load imbalance an
8-GPU strong-scaling run would see on top of its reduce.

usage: python tools/c4_balance.py [n_shards] [n_rings]   -> JSON on stdout"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import torj_hip as T
    from test_gpu_beam import _device_shards
    from torj_hip import synthetic as S
    from torj_hip._lib import TraceCfg
    from torj_hip.parallel import group_shard, trace_beam_device

    n_shards = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n_rings = int(sys.argv[2]) if len(sys.argv) > 2 else 291
    eq = S.circular_tokamak()
    P = T.Plasma(*S.plasma_args(eq))
    T.abs_Al_init(24)
    s = S.SETUP
    f = s["f_abs_test"]
    om = 2 * np.pi * f
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=n_rings,
                                            min_azimuthal_points=11)
    n = len(w)
    xp, Np, s0, st = T.ray_entry(P, pos, dirs, om, 1, gpu=True)
    grid = np.linspace(0.0, 1.0, 1000)
    cfg = TraceCfg(om, 1, 1e-4, 2000, 20, 1.0, 1e-6, 1, 100, 1)
    dev = torch.device("cuda", 0)
    out = []
    for k in range(n_shards):
        sl = group_shard(n, n_shards, k)
        sh = _device_shards(torch, T, P, cfg, len(grid), grid, xp, Np, w, pos, s0, [sl], dev)
        trace_beam_device(P, cfg, len(grid), sh)  # warm-up (replica, workspace)
        torch.cuda.synchronize(dev)
        times = []
        for _ in range(2):
            sh[0]["counters"].zero_()
            sh[0]["dP_shell"].zero_()
            t0 = time.perf_counter()
            trace_beam_device(P, cfg, len(grid), sh)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t0)
        c = sh[0]["counters"].cpu().numpy()
        status = np.bincount(sh[0]["status"].cpu().numpy(), minlength=6)
        out.append({"shard": k, "rays": sl.stop - sl.start, "first_ray": sl.start,
                    "seconds": min(times), "ray_steps": int(c[0]),
                    "alpha_active": int(c[2]), "harmonic_integrals": int(c[3]),
                    "exact_zero": int(c[5]), "negligible": int(c[6]), "settled_early": int(c[7]),
                    "status_counts": {T.STATUS_NAMES[i]: int(v) for i, v in enumerate(status) if v}})
        print(f"shard {k}: {out[-1]['seconds'] * 1e3:.1f} ms", file=sys.stderr, flush=True)
        del sh
        torch.cuda.empty_cache()
    t = np.array([o["seconds"] for o in out])
    print(json.dumps({"workload": f"C4 fan N_rings={n_rings} ({n} rays), {n_shards} contiguous shards, "
                                  "2000 RK4 steps, Albajar, reference deposition n_psi=1000, each "
                                  "shard alone on device 0 via torj_trace_beam_device",
                      "shards": out, "max_over_mean": float(t.max() / t.mean()),
                      "sum_seconds": float(t.sum())}, indent=1))


if __name__ == "__main__":
    main()
