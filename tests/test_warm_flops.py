"""The algorithmic FLOP model of the weakly relativistic warm alpha
(torj_hip/flops.py algorithmic_flops_warm, C5's roofline numerator).

  * flops.py's FLOPS_WARM_* constants are what `python oracle/flopcount_warm.py`
    measures (the instrumented restatement of the kernel's arithmetic);
  * that restatement computes the C oracle's N_perp^2 (1e-7 relative at
    Te >= 1 keV, the fsup conditioning bound of tests/test_warm_oracle_c.py), so
    its branches and trip counts are the real ones;
  * the model, fed with the restatement's trip counts, is a lower bound of its
    instrumented count within 3 %;
  * GPU: the kernel's 8 work counters of a one-step warm trace equal the trip
    counts the restatement finds at the same RK4 stage points (exact integers).
"""
import math
import warnings

import numpy as np
import pytest


@pytest.fixture(scope="module")
def FW():
    import flopcount_warm

    return flopcount_warm


def test_constants_match_instrumented_count(FW):
    from torj_hip import flops as F

    for k, v in FW.component_counts().items():
        assert getattr(F, k) == v, k


def _points(O, n, seed, mode, te_lo):
    from test_warm_oracle_c import _sweep

    return _sweep(O, n, seed, mode, te_lo)


def _counters(trs):
    """the kernel's counters [1..7] from restatement trips"""
    return [len(trs), sum(t.nasym for t in trs), sum(t.nfad for t in trs),
            sum(t.passes for t in trs), sum(t.passes * t.lrm for t in trs),
            sum(t.lrm for t in trs), sum(t.lrm * t.lrm for t in trs)]


@pytest.mark.parametrize("mode", [1, -1])
def test_restatement_values_and_model_bound(O, FW, mode):
    from flopcount import Counter
    from torj_hip import flops as F

    args = _points(O, 120, 8, mode, 1e3)
    trs, count, errs = [], 0, []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in range(len(args[0])):
            pt = [float(v[i]) for v in args]
            _, n2 = O.alpha_warm(*pt, mode, 1)
            c0 = Counter.n
            _, n2r, tr = FW.alpha_wr(*pt, mode)
            c = Counter.n - c0
            if not (tr.converged and np.isfinite(n2)):
                continue
            errs.append(abs(n2r - n2) / max(abs(n2), 1e-300))
            trs.append(tr)
            count += c
            m = FW.model_flops([tr], FW.component_counts())
            # per point: larmornumber's tests are priced at one per call (the
            # counter slot carries the asymptotic Faddeeva evaluations), so a
            # cheap point with many resonance tests sits a few % low
            assert 0.94 * c <= m <= c, (pt, m, c)
    assert len(trs) > 90
    assert max(errs) <= 1e-7, max(errs)
    # flops.py's aggregate form (minus the cold RHS it adds per call) = the sum
    cnt = [0] + _counters(trs)
    model = F.algorithmic_flops_warm(cnt) - len(trs) * F.FLOPS_RHS_COLD
    assert model == pytest.approx(FW.model_flops(trs, FW.component_counts()), rel=1e-12)
    assert 0.97 * count <= model <= count


@pytest.mark.gpu
def test_gpu_warm_counters_equal_restatement_trips(gpu, T, hplasma, oplasma, FW):
    """8 rays of the X2 fan, one RK4 step of 1 mm with absorption 2: the four
    stage points per ray recomputed with the oracle's sys! right-hand side; the
    restatement's trips there = the kernel's counters."""
    import ctypes

    import torch
    from test_gpu_warm import _x2_rays

    pos, xp, Np, s0, w, om = _x2_rays(T, hplasma, n_rings=2, min_az=3)
    xp, Np = xp[:8], Np[:8]
    n, ds = len(xp), 1e-3
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    x0, N0 = t(xp.T), t(Np.T)
    state = torch.empty((7, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    k = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    cfg = T._lib.TraceCfg(om, 1, ds, 1, 1, 1.0, 1e-6, 2, 0)
    stream = torch.cuda.current_stream(dev)
    T._lib.check(T.lib().torj_trace_device(hplasma.handle, cfg, n, x0.data_ptr(), N0.data_ptr(),
                                           None, 0, None, state.data_ptr(), st.data_ptr(),
                                           k.data_ptr(), None, None, None,
                                           ctypes.c_void_p(cnt.data_ptr()), stream.cuda_stream))
    T._lib.check(T.lib().torj_trace_check(hplasma.handle, stream.cuda_stream))
    g = cnt.cpu().numpy()
    trs = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in range(n):
            u0 = np.concatenate([xp[i], Np[i]])
            f = lambda u: oplasma.grad_lambda(u[:3], u[3:], om, 1)
            k1 = f(u0)
            k2 = f(u0 + 0.5 * ds * k1)
            k3 = f(u0 + 0.5 * ds * k2)
            stages = [u0, u0 + 0.5 * ds * k1, u0 + 0.5 * ds * k2, u0 + ds * k3]
            for u in stages:
                X, Y, Npar, _ = oplasma.eval_plasma(u[:3], u[3:], om)
                inv = 1.0 / oplasma.grad_norm(u[:3], u[3:], om, 1)
                trs.append(FW.alpha_wr(om, X, Y, float(np.linalg.norm(u[3:])), Npar,
                                       oplasma.T_e(u[:3]), inv, 1)[2])
    assert g[0] == n and g[1] == 4 * n
    assert list(g[1:]) == _counters(trs), (list(g), _counters(trs))
