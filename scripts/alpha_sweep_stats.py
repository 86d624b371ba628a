"""Prints the GPU-vs-oracle error of abs_Albajar_fast on the random physical
sweep of tests/test_gpu_parity.py (the node loop's exp2_node / sqrt_node)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "torj.jl_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
import torj_hip as T  # noqa: E402
from test_gpu_parity import albajar_random_sweep  # noqa: E402

O.abs_al_init(24)
T.abs_Al_init(24)
rel, ab, inp = albajar_random_sweep(T, O, n=100000, seed=11)
worst = np.argsort(rel)[::-1][:8]
print(json.dumps({"tuples": 100000, "compared_rel": int(len(rel)), "max_rel": float(rel.max()),
                  "p99_rel": float(np.quantile(rel, 0.99)), "median_rel": float(np.median(rel)),
                  "max_abs_small": float(ab.max()) if len(ab) else 0.0,
                  "above_1e-10": int((rel > 1e-10).sum()),
                  "worst": [dict(zip(["X", "Y", "N_abs", "N_par", "Te", "mode", "gpu", "oracle", "rel"],
                                     [float(v) for v in inp[i]] + [float(rel[i])])) for i in worst]}))
