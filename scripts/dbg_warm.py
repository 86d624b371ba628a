"""Debug aid: GPU torj_alpha_warm batched vs one point per call, on the GPU-test
sweeps -> gpurun_out/dbg_warm.npz"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import oracle as O
import torj_hip as T
from test_gpu_warm import _sweep

out = {}
for mode in (1, -1):
    for iw, te in ((3, 10.0), (1, 1e3)):
        args = _sweep(O, 256, 7 + iw, mode, te)
        a, n2 = T.alpha_warm(*args, mode=mode, iwarm=iw)
        out[f"a_{mode}_{iw}"], out[f"n2_{mode}_{iw}"] = a, n2
        one = np.array([T.alpha_warm(*[v[i] for v in args], mode=mode, iwarm=iw)[1] for i in range(256)])
        out[f"one_{mode}_{iw}"] = one
        print(mode, iw, "batched vs single max diff", np.abs(one - n2).max())
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", os.environ.get("DBG_OUT", "dbg_warm") + ".npz"), **out)
