"""The split RK4 path (torj_set_sched mode 3): cold RK4
trajectories, the alpha evaluations as a separate fully parallel kernel and the
optical depth by an in-order scan, pipelined in blocks of steps over two
streams.  Its outputs equal the fused one-lane kernel's to rounding (1e-12:
the same arithmetic in separately compiled kernels, whose fma contraction may
differ by an ulp) with identical statuses, step counts and NaN pattern; vs the
oracle the parity bar (1e-10, statuses and steps exact)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fan(T, hplasma, mode=1, n_rings=14, min_az=5, f=None):
    from torj_hip import synthetic as S

    s = S.SETUP
    f = f or s["f_abs_test"]
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=n_rings,
                                            min_azimuthal_points=min_az)
    om = 2 * np.pi * f
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, mode, gpu=True)
    assert (st == T.OK).all()
    return pos, xp, Np, s0, w, om


def _run(T, hplasma, sched, waves, *args, **kw):
    try:
        hplasma.set_sched(sched, waves)
        return T.trace(hplasma, *args, **kw)
    finally:
        hplasma.set_sched(-1)


@pytest.mark.parametrize("deposition,traj,block", [("reference", 100, 0), ("reference", 100, 60),
                                                    ("binned", 0, 140), ("none", 7, 33)])
def test_split_equals_fused(gpu, T, hplasma, deposition, traj, block):
    from test_gpu_c3 import _close

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=traj)
    if deposition != "none":
        kw.update(psi_grid=np.linspace(0, 1, 1000), deposition=deposition, x_launch=pos, s0=s0)
    a = _run(T, hplasma, 0, 0, xp, Np, om, 1, **kw)
    b = _run(T, hplasma, 3, block, xp, Np, om, 1, **kw)
    if traj == 0:
        a.traj = b.traj = np.zeros(0)
    if deposition == "none":
        a.dP_shell = b.dP_shell = np.ones(1)
    _close(a, b, 1e-12)


def test_split_termination_vs_oracle(gpu, T, hplasma, oplasma):
    """ABSORBED (P_min raised so rays stop mid-block at chunk boundaries),
    LEFT_PLASMA (rays launched outwards), O-mode; with the trajectory samples
    past a stop NaN as in the fused kernel."""
    from test_gpu_parity import _compare_trace

    pos, xp, Np, s0, w, om = _fan(T, hplasma, n_rings=4)
    x_out = np.array([[2.1, 0.0, 0.0], [1.9, 0.0, 0.3]])
    N_out = np.array([[1.0, 0.0, 0.0], [0.2, 0.0, 1.0]])
    for i in range(len(x_out)):
        N_out[i] /= np.linalg.norm(N_out[i])
        lo, hi = 0.01, 1.5
        for _ in range(100):
            m = 0.5 * (lo + hi)
            d = oplasma.dispersion_relation(x_out[i], N_out[i] * m, om, 1)
            lo, hi = (m, hi) if d < 0 else (lo, m)
        N_out[i] *= lo
    xp, Np = np.vstack([xp, x_out]), np.vstack([Np, N_out])
    grid = np.linspace(0, 1, 300)
    kw = dict(ds=1e-4, n_steps=6000, chunk_steps=60, psi_grid=grid, traj_stride=50, P_min=1e-2)
    g = _run(T, hplasma, 3, 90, xp, Np, om, 1, **kw)
    a = _run(T, hplasma, 0, 0, xp, Np, om, 1, **kw)
    o = oplasma.trace(xp, Np, om, 1, 1e-4, 6000, chunk_steps=60, psi_grid=grid, traj_stride=50,
                      P_min=1e-2)
    _compare_trace(g, o)
    assert T.ABSORBED in g.status.tolist() and T.LEFT_PLASMA in g.status.tolist()
    assert np.array_equal(np.isfinite(g.traj), np.isfinite(a.traj))
    fin = np.isfinite(a.traj)
    assert np.abs(g.traj[fin] - a.traj[fin]).max() <= 1e-10 * np.abs(a.traj[fin]).max()
    assert np.abs(g.dP_shell[:-1] - o["dP"]).max() <= 1e-10 * np.abs(o["dP"]).max()


@pytest.mark.parametrize("zflag", ["0", "1"])
def test_split_counters_match_fused(gpu, T, hplasma, zflag):
    """The work counters (the algorithmic FLOP count's basis) of the split path
    equal the fused kernel's on a beam without mid-block stops.  With the block
    zero flags (TORJ_ALPHA_ZFLAG, the default) a wave whose rays are all flagged
    evaluates nothing, so its points count no settled-early harmonics (counter
    7): that counter is then at most the fused kernel's and the others equal
    (the outputs' bits: test_zero_flags_bit_identical)."""
    import ctypes
    import torch

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    n = len(w)
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    x0, N0 = t(xp.T), t(Np.T)
    out = []
    old = os.environ.get("TORJ_ALPHA_ZFLAG")
    os.environ["TORJ_ALPHA_ZFLAG"] = zflag
    for sched in (0, 3):
        state = torch.empty((7, n), dtype=torch.float64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        k = torch.empty(n, dtype=torch.int32, device=dev)
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        cfg = T._lib.TraceCfg(om, 1, 1e-4, 1500, 15, 1.0, 1e-6, 1, 0)
        stream = torch.cuda.current_stream(dev)
        hplasma.set_sched(sched, 0)
        try:
            T._lib.check(T.lib().torj_trace_device(hplasma.handle, cfg, n, x0.data_ptr(),
                                                   N0.data_ptr(), None, 0, None, state.data_ptr(),
                                                   st.data_ptr(), k.data_ptr(), None, None, None,
                                                   ctypes.c_void_p(cnt.data_ptr()),
                                                   stream.cuda_stream))
            T._lib.check(T.lib().torj_trace_check(hplasma.handle, stream.cuda_stream))
        finally:
            hplasma.set_sched(-1)
        out.append((cnt.cpu().numpy(), state.cpu().numpy()))
    if old is None:
        os.environ.pop("TORJ_ALPHA_ZFLAG", None)
    else:
        os.environ["TORJ_ALPHA_ZFLAG"] = old
    (cf, sf), (cs, ss) = out
    if zflag == "0":
        assert np.array_equal(cf, cs), (cf, cs)
    else:
        assert np.array_equal(cf[:7], cs[:7]) and cs[7] <= cf[7], (cf, cs)
        print(f"settled-early harmonics counted: fused {cf[7]}, split with zero flags {cs[7]}")


@pytest.mark.parametrize("tiny", ["1e-20", "0"])
def test_zero_flags_bit_identical(gpu, T, hplasma, tiny):
    """The block zero flags (torj_hip.hip zero_box_flag: the trajectory kernel
    proves per ray and ring block that every stored stage point has alpha = +-0,
    and an alpha wave whose rays are all flagged writes 0 without evaluating)
    change no output bit: TORJ_ALPHA_ZFLAG=0 against the default on the split
    path, with the tiny-alpha skip (default) and without it (the exact leg), on
    a fan whose rays start outside the resonance (flagged blocks) and cross it
    (unflagged ones), with mid-trace stops; statuses, steps, state, trajectory
    samples, P_dep and dP_shell all equal."""
    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=3000, chunk_steps=30, weights=w, traj_stride=30, P_min=5e-2,
              psi_grid=np.linspace(0, 1, 500), deposition="reference", x_launch=pos, s0=s0)
    out, cnts = {}, {}
    old = {k: os.environ.get(k) for k in ("TORJ_ALPHA_ZFLAG", "TORJ_TINY_ALPHA")}
    os.environ["TORJ_TINY_ALPHA"] = tiny
    T.abs_Al_init(24)
    try:
        for z in ("0", "1"):
            os.environ["TORJ_ALPHA_ZFLAG"] = z
            out[z] = _run(T, hplasma, 3, 60, xp, Np, om, 1, **kw)
            cnts[z] = _trace_counted(T, hplasma, 3, xp, Np, om)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        T.abs_Al_init(24)
    a, b = out["0"], out["1"]
    assert a.status.tolist().count(T.ABSORBED) >= 10, "need mid-trace stops"
    for f in ("state", "status", "steps", "P_dep", "dP_shell"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.array_equal(a.traj, b.traj, equal_nan=True)
    c0, c1 = cnts["0"], cnts["1"]
    assert np.array_equal(c0[:7], c1[:7]) and c1[7] <= c0[7], (c0, c1)
    print(f"tiny_alpha {tiny}: counters without flags {c0}, with {c1}")
    if tiny != "1e-20":
        return
    # the flags fire: under the test hook TORJ_TEST_ZFLAG_NAN=s a fully flagged
    # wave of a block starting at step s or later writes NaN, so its live rays
    # stop NAN at the first step of that block (a multiple of the 60-step block);
    # every other ray is untouched
    for s_from in (0, 60):
        h = _env_run(T, hplasma, {"TORJ_TEST_ZFLAG_NAN": str(s_from)}, xp, Np, om, 1, **kw)
        nan = h.status == T.NAN
        print(f"from step {s_from}: flagged waves stop {nan.sum()} of {len(nan)} rays, at steps "
              f"{np.unique(h.steps[nan], return_counts=True)}")
        assert nan.sum() >= 64
        assert (h.steps[nan] % 60 == 0).all() and (h.steps[nan] >= s_from).all()
        assert (h.steps[nan] < a.steps[nan]).all()
        for f in ("state", "status", "steps"):
            assert np.array_equal(getattr(h, f)[~nan], getattr(b, f)[~nan]), f


def test_split_on_129_grid_vs_oracle(gpu, T, O):
    """The split path on the 129 x 129 equilibrium, whose coefficients (1.1 MB)
    do not fit LDS: the trajectory kernel reads them through L2."""
    from test_gpu_parity import _compare_trace
    from torj_hip import synthetic as S

    eq = S.circular_tokamak(nR=129, nZ=129)
    hp = T.Plasma(*S.plasma_args(eq))
    op = O.OraclePlasma(*S.plasma_args(eq))
    pos, xp, Np, s0, w, om = _fan(T, hp, n_rings=6)
    grid = np.linspace(0, 1, 500)
    g = _run(T, hp, 3, 0, xp, Np, om, 1, ds=1e-4, n_steps=2000, psi_grid=grid, weights=w)
    o = op.trace(xp, Np, om, 1, 1e-4, 2000, psi_grid=grid, weights=w)
    _compare_trace(g, o)
    assert np.abs(g.dP_shell[:-1] - o["dP"]).max() <= 1e-10 * np.abs(o["dP"]).max()


@pytest.mark.parametrize("model,n_rings", [(2, 14), (3, 5)])
def test_split_warm_equals_fused(gpu, T, hplasma, model, n_rings):
    """The warm models on the split path (k_alpha_warm_pts: the group-velocity
    factor as a sixth stored input): the library's default for small warm beams
    (fewer groups than 3 per CU) and sched mode 3, against the fused work-queue
    kernel: statuses and steps exact, x, N 1e-12, tau 1e-10 (model 3; measured
    4e-15) and 1e-9 (model 2: measured 7e-12 with the node stencil in both, 1.5e-10
    since the split trajectory kernel evaluates the fields in per-cell power
    form -- positions within ~4e-16, and iwarm 1's cold-edge root selection is
    that sensitive: DESIGN.md 3.6, the a-priori conditioning flag of
    tests/test_gpu_c5.py), reference deposition 1e-9; the iwarm-1 work counters
    (integer trip counts of the same alpha code) equal."""
    import ctypes

    import torch

    pos, xp, Np, s0, w, om = _fan(T, hplasma, n_rings=n_rings)
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=100, absorption=model,
              psi_grid=np.linspace(0, 1, 500), deposition="reference", x_launch=pos, s0=s0)
    a = _run(T, hplasma, 1, 0, xp, Np, om, 1, **kw)   # fused work queue
    b = T.trace(hplasma, xp, Np, om, 1, **kw)           # default: split (small warm beam)
    c = _run(T, hplasma, 3, 0, xp, Np, om, 1, **kw)   # forced split
    for r in (b, c):
        assert np.array_equal(a.status, r.status) and np.array_equal(a.steps, r.steps)
        for cols in (slice(0, 3), slice(3, 6)):
            e = np.abs(a.state[:, cols] - r.state[:, cols]).max(1) / np.linalg.norm(a.state[:, cols], axis=1)
            assert e.max() <= 1e-12, e.max()
        assert a.state[:, 6].min() > 1.0  # the X2 layer is crossed
        assert (np.abs(a.state[:, 6] - r.state[:, 6]) / a.state[:, 6]).max() <= (1e-9 if model == 2 else 1e-10)
        assert np.abs(a.P_dep - r.P_dep).max() <= 1e-9
        assert np.abs(a.dP_shell - r.dP_shell).max() <= 1e-9 * np.abs(a.dP_shell).max()
    if model != 2:
        return
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    x0, N0, n = t(xp.T), t(Np.T), len(w)
    out = []
    for sched in (1, 3):
        state = torch.empty((7, n), dtype=torch.float64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        k = torch.empty(n, dtype=torch.int32, device=dev)
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        cfg = T._lib.TraceCfg(om, 1, 1e-4, 2000, 20, 1.0, 1e-6, 2, 0)
        stream = torch.cuda.current_stream(dev)
        hplasma.set_sched(sched, 0)
        try:
            T._lib.check(T.lib().torj_trace_device(hplasma.handle, cfg, n, x0.data_ptr(),
                                                   N0.data_ptr(), None, 0, None, state.data_ptr(),
                                                   st.data_ptr(), k.data_ptr(), None, None, None,
                                                   ctypes.c_void_p(cnt.data_ptr()),
                                                   stream.cuda_stream))
            T._lib.check(T.lib().torj_trace_check(hplasma.handle, stream.cuda_stream))
        finally:
            hplasma.set_sched(-1)
        out.append(cnt.cpu().numpy())
    assert np.array_equal(out[0], out[1]), (out[0], out[1])


@pytest.mark.parametrize("model", [2, 3])
def test_split_warm_deferred_points(gpu, T, hplasma, model):
    """k_alpha_warm_pts defers its points with Larmor order lrm > 3 to
    k_alpha_warm_big (the lrm <= 5 tensor), so that its own registers are
    sized for lrm <= 3.  At 140 GHz (third-harmonic layer) such points are
    common (iwarm 1: sum lrm^2 > 3 sum lrm in the work counters, which equal
    the fused kernel's).  With TORJ_WARM_DEFER_LRM=0 every point takes the
    deferred path (the list, its count, the lrm <= 5 tensor): the outputs are
    bit-identical to the default split (the tensor's size changes no
    arithmetic), and the fused work-queue kernel agrees on statuses and steps."""
    import ctypes

    import torch

    pos, xp, Np, s0, w, om = _fan(T, hplasma, n_rings=8, f=140e9)
    kw = dict(ds=1e-4, n_steps=1500, traj_stride=100, absorption=model, psi_grid=np.linspace(0, 1, 500),
              deposition="reference", x_launch=pos, s0=s0, weights=w)
    a = _env_run(T, hplasma, {}, xp, Np, om, 1, **kw)
    b = _env_run(T, hplasma, {"TORJ_WARM_DEFER_LRM": "0"}, xp, Np, om, 1, **kw)
    for f in ("state", "status", "steps", "P_dep", "dP_shell"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    c = _run(T, hplasma, 1, 0, xp, Np, om, 1, **kw)
    assert np.array_equal(a.status, c.status) and np.array_equal(a.steps, c.steps)
    if model != 2:
        return
    n = len(w)
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    x0, N0 = t(xp.T), t(Np.T)
    out = []
    for sched in (1, 3):
        state = torch.empty((7, n), dtype=torch.float64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        k = torch.empty(n, dtype=torch.int32, device=dev)
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        cfg = T._lib.TraceCfg(om, 1, 1e-4, 1500, 20, 1.0, 1e-6, model, 0)
        stream = torch.cuda.current_stream(dev)
        hplasma.set_sched(sched, 0)
        try:
            T._lib.check(T.lib().torj_trace_device(hplasma.handle, cfg, n, x0.data_ptr(),
                                                   N0.data_ptr(), None, 0, None, state.data_ptr(),
                                                   st.data_ptr(), k.data_ptr(), None, None, None,
                                                   ctypes.c_void_p(cnt.data_ptr()),
                                                   stream.cuda_stream))
            T._lib.check(T.lib().torj_trace_check(hplasma.handle, stream.cuda_stream))
        finally:
            hplasma.set_sched(-1)
        out.append(cnt.cpu().numpy())
    assert np.array_equal(out[0], out[1]), (out[0], out[1])
    assert out[0][7] > 3 * out[0][6], out[0]  # some points with lrm >= 4 (deferred)
    print(f"140 GHz model {model}: counters {out[0]}")


@pytest.mark.parametrize("deposition", ["reference", "binned"])
def test_split_serial_equals_overlapped(gpu, T, hplasma, deposition):
    """The trajectory and alpha kernels read the scan's stop word (sinfo) while
    the scan of an earlier block may still be writing it on another stream; the
    read only skips work nobody reads (torj_hip.hip traj_body).  Held here: with
    rays ABSORBED mid-block (P_min raised), TORJ_SPLIT_SERIAL=1 (every kernel on
    one stream, no overlap) and the default overlap give bit-identical state,
    steps, status, deposition and trajectory."""
    import os

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=3000, chunk_steps=30, weights=w, traj_stride=30, P_min=5e-2,
              psi_grid=np.linspace(0, 1, 500), deposition=deposition, x_launch=pos, s0=s0)
    out = {}
    old = os.environ.get("TORJ_SPLIT_SERIAL")
    try:
        for serial in ("1", "0"):
            os.environ["TORJ_SPLIT_SERIAL"] = serial
            out[serial] = _run(T, hplasma, 3, 90, xp, Np, om, 1, **kw)
    finally:
        if old is None:
            os.environ.pop("TORJ_SPLIT_SERIAL", None)
        else:
            os.environ["TORJ_SPLIT_SERIAL"] = old
    a, b = out["1"], out["0"]
    st = a.status.tolist()
    assert st.count(T.ABSORBED) >= 10 and a.steps.min() < 3000 - 90, "need mid-block stops"
    for f in ("state", "status", "steps", "P_dep"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.array_equal(a.traj, b.traj, equal_nan=True)
    if deposition == "reference":  # k_shell_sum: a fixed summation order
        assert np.array_equal(a.dP_shell, b.dP_shell)
    else:  # binned: fp64 atomics, order-dependent in the last bits
        assert np.abs(a.dP_shell - b.dP_shell).max() <= 1e-13 * np.abs(a.dP_shell).max()


def test_negligible_harmonic_skip_bit_identical(gpu, T, hplasma):
    """The skip of provably negligible harmonic integrals (torj_math.hpp
    albajar_harmonic: bound below 2^-58 of the harmonics already summed) leaves
    every output bit-identical: TORJ_NEGL_SKIP=0 (re-read by abs_Al_init, which
    re-uploads the GL table) against the default, on the split pipeline (the
    default for large beams) and the fused one-lane kernel; the skip fires
    (work counter [6]) and moves its integrals out of counter [3]."""
    import ctypes
    import os

    import torch

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    n = len(w)
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=100, psi_grid=np.linspace(0, 1, 1000),
              deposition="reference", x_launch=pos, s0=s0)
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    x0, N0 = t(xp.T), t(Np.T)

    def counters(sched):
        state = torch.empty((7, n), dtype=torch.float64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        k = torch.empty(n, dtype=torch.int32, device=dev)
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        cfg = T._lib.TraceCfg(om, 1, 1e-4, 2000, 20, 1.0, 1e-6, 1, 0)
        stream = torch.cuda.current_stream(dev)
        hplasma.set_sched(sched, 0)
        try:
            T._lib.check(T.lib().torj_trace_device(hplasma.handle, cfg, n, x0.data_ptr(), N0.data_ptr(),
                                                   None, 0, None, state.data_ptr(), st.data_ptr(),
                                                   k.data_ptr(), None, None, None,
                                                   ctypes.c_void_p(cnt.data_ptr()), stream.cuda_stream))
            T._lib.check(T.lib().torj_trace_check(hplasma.handle, stream.cuda_stream))
        finally:
            hplasma.set_sched(-1)
        return cnt.cpu().numpy()

    res, cnts = {}, {}
    old = os.environ.get("TORJ_NEGL_SKIP"), os.environ.get("TORJ_TINY_ALPHA")
    os.environ["TORJ_TINY_ALPHA"] = "0"  # the bounded tiny-alpha skip off: bit-identity holds
    try:
        for skip in ("0", "1"):
            os.environ["TORJ_NEGL_SKIP"] = skip
            T.abs_Al_init(24)
            for sched in (3, 0):
                res[skip, sched] = _run(T, hplasma, sched, 0, xp, Np, om, 1, **kw)
                cnts[skip, sched] = counters(sched)
    finally:
        for k, v in zip(("TORJ_NEGL_SKIP", "TORJ_TINY_ALPHA"), old):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        T.abs_Al_init(24)
    for sched in (3, 0):
        a, b = res["0", sched], res["1", sched]
        for f in ("state", "status", "steps", "P_dep", "dP_shell"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), (sched, f)
        assert np.array_equal(a.traj, b.traj, equal_nan=True)
        c0, c1 = cnts["0", sched], cnts["1", sched]
        assert c0[6] == 0 and c1[6] > 0.1 * c0[3], (c0, c1)
        assert c1[3] + c1[6] == c0[3] and np.array_equal(c0[[0, 1]], c1[[0, 1]])
        # calls settled before the polarisation vector (every harmonic present an
        # exact zero): their harmonics leave the zero count for counter [7]
        assert c0[7] == 0 and c1[7] > 0 and c1[2] < c0[2] and c1[5] < c0[5], (c0, c1)
        assert c1[5] + c1[7] >= c0[5], (c0, c1)
    assert np.array_equal(cnts["1", 3], cnts["1", 0])


def _trace_counted(T, hplasma, sched, xp, Np, om):
    """One traced launch's work counters (torj_trace_device with a counters array)."""
    import ctypes

    import torch

    n = len(xp)
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    x0, N0 = t(xp.T), t(Np.T)
    state = torch.empty((7, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    k = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    cfg = T._lib.TraceCfg(om, 1, 1e-4, 2000, 20, 1.0, 1e-6, 1, 0)
    stream = torch.cuda.current_stream(dev)
    hplasma.set_sched(sched, 0)
    try:
        T._lib.check(T.lib().torj_trace_device(hplasma.handle, cfg, n, x0.data_ptr(), N0.data_ptr(),
                                               None, 0, None, state.data_ptr(), st.data_ptr(),
                                               k.data_ptr(), None, None, None,
                                               ctypes.c_void_p(cnt.data_ptr()), stream.cuda_stream))
        T._lib.check(T.lib().torj_trace_check(hplasma.handle, stream.cuda_stream))
    finally:
        hplasma.set_sched(-1)
    return cnt.cpu().numpy()


@pytest.mark.parametrize("sched", [3, 0])
def test_tiny_alpha_skip_bounded(gpu, T, hplasma, sched):
    """The skip of harmonic integrals whose share of alpha is provably below
    tiny_alpha (torj_math.hpp albajar_harmonic / tiny_harmonic; default 1e-20
    m^-1, TORJ_TINY_ALPHA=0 evaluates every integral): on the split pipeline and
    the fused kernel, statuses, steps and trajectories are bit-identical, tau
    moves by at most 2 tiny_alpha per metre of ray (two harmonics) plus the
    rounding of the sums the skipped terms left, the deposited power likewise;
    the skip fires (counter [6] up, counter [3] down by as much)."""
    import os

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=100, psi_grid=np.linspace(0, 1, 1000),
              deposition="reference", x_launch=pos, s0=s0)
    res, cnts = {}, {}
    old = os.environ.get("TORJ_TINY_ALPHA")
    try:
        for tiny in ("0", "1e-20"):
            os.environ["TORJ_TINY_ALPHA"] = tiny
            T.abs_Al_init(24)
            res[tiny] = _run(T, hplasma, sched, 0, xp, Np, om, 1, **kw)
            cnts[tiny] = _trace_counted(T, hplasma, sched, xp, Np, om)
    finally:
        if old is None:
            os.environ.pop("TORJ_TINY_ALPHA", None)
        else:
            os.environ["TORJ_TINY_ALPHA"] = old
        T.abs_Al_init(24)
    a, b = res["0"], res["1e-20"]
    for f in ("status", "steps"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.array_equal(a.state[:, :6], b.state[:, :6])
    # trajectory samples (n, n_save, 5): x, y, z and s bit-identical, tau as tau
    rows = [0, 1, 2, 4]
    assert np.array_equal(a.traj[:, :, rows], b.traj[:, :, rows], equal_nan=True)
    assert np.array_equal(np.isfinite(a.traj[:, :, 3]), np.isfinite(b.traj[:, :, 3]))
    fin = np.isfinite(a.traj[:, :, 3])
    L = a.steps * 1e-4  # metres of ray traced
    assert (np.abs(a.traj[:, :, 3] - b.traj[:, :, 3])[fin] <= 2e-20 * 0.2 + 4e-16 * np.abs(a.traj[:, :, 3])[fin]).all()
    dtau = np.abs(a.state[:, 6] - b.state[:, 6])
    assert (dtau <= 2 * 1e-20 * L + 4e-16 * np.abs(a.state[:, 6])).all(), dtau.max()
    assert np.abs(a.P_dep - b.P_dep).max() <= 1e-12
    assert np.abs(a.dP_shell - b.dP_shell).max() <= 1e-12 * np.abs(a.dP_shell).max()
    c0, c1 = cnts["0"], cnts["1e-20"]
    assert np.array_equal(c0[[0, 1, 2, 5, 7]], c1[[0, 1, 2, 5, 7]]), (c0, c1)
    assert c1[6] > c0[6] and c1[3] + c1[6] == c0[3] + c0[6], (c0, c1)


def test_streamed_deposition_matches_one_pass(gpu, T, hplasma):
    """The reference profile's root walk streamed in windows behind each block's
    scan (k_depo_stream + k_depo_tail, torj_fitdepo.hpp) against the one-pass
    k_fit_depo after the trace (TORJ_DEPO_STREAM=0), and the windows on a stream
    of their own (=2) against the scan's stream (=1): the trace itself is
    bit-identical, the deposited power per ray and per shell equal to rounding
    (<= 1e-13), with rays ABSORBED mid-trace (the tail takes stopped rays) and
    blocks of 90 steps that do not align with the 64-segment windows."""
    import os

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=3000, chunk_steps=30, weights=w, traj_stride=30, P_min=5e-2,
              psi_grid=np.linspace(0, 1, 500), deposition="reference", x_launch=pos, s0=s0)
    out = {}
    old = os.environ.get("TORJ_DEPO_STREAM")
    try:
        for mode in ("0", "1", "2", "3", "4", "5"):
            os.environ["TORJ_DEPO_STREAM"] = mode
            out[mode] = _run(T, hplasma, 3, 90, xp, Np, om, 1, **kw)
    finally:
        if old is None:
            os.environ.pop("TORJ_DEPO_STREAM", None)
        else:
            os.environ["TORJ_DEPO_STREAM"] = old
    a, b = out["0"], out["1"]
    st = a.status.tolist()
    assert st.count(T.ABSORBED) >= 10 and a.steps.max() > 1000, "need long rays and mid-trace stops"
    for f in ("state", "status", "steps"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.abs(a.P_dep - b.P_dep).max() <= 1e-13 * np.abs(a.P_dep).max()
    assert np.abs(a.dP_shell - b.dP_shell).max() <= 1e-13 * np.abs(a.dP_shell).max()
    assert np.abs(a.dP_shell).max() > 0
    # the windows on a stream of their own (TORJ_DEPO_STREAM=2, overlapping the
    # next block's scan): the same windows, so the same bits as on the scan's stream
    # and the split form (=3: a window's elimination and walk as two launches;
    # =4: those two launches on a stream of their own; =5: on the trajectory
    # kernel's stream, two blocks behind their scans)
    for m in ("2", "3", "4", "5"):
        c = out[m]
        for f in ("state", "status", "steps", "P_dep", "dP_shell"):
            assert np.array_equal(getattr(b, f), getattr(c, f)), (m, f)


def _env_run(T, hplasma, env, *args, **kw):
    import os

    old = {k: os.environ.get(k) for k in env}
    try:
        for k, v in env.items():
            os.environ[k] = v
        return _run(T, hplasma, 3, 60, *args, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_node_stencil_modes_keep_round3_bars(gpu, T, hplasma, mode):
    """The widened bars of the split path (tau floor 1e-13 against the fused
    kernel, warm model 2 tau 1e-9) belong to the cell power form only
    (TORJ_TRAJ_LDS=3, the default): with a node-stencil trajectory kernel
    (0: L2, 1: whole-grid LDS, 2: node tile) -- the fused kernels' arithmetic --
    the split path holds the round-3 bars: x, N 1e-12, tau 1e-12 relative with
    a 1e-14 floor, and warm model 2 tau 1e-10 relative."""
    from test_gpu_c3 import _close

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=100, psi_grid=np.linspace(0, 1, 1000),
              deposition="reference", x_launch=pos, s0=s0)
    a = _run(T, hplasma, 0, 0, xp, Np, om, 1, **kw)
    b = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": mode}, xp, Np, om, 1, **kw)
    _close(a, b, 1e-12, tau_floor=1e-14)
    kw.update(absorption=2, psi_grid=np.linspace(0, 1, 500))
    a = _run(T, hplasma, 1, 0, xp, Np, om, 1, **kw)
    b = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": mode}, xp, Np, om, 1, **kw)
    assert np.array_equal(a.status, b.status) and np.array_equal(a.steps, b.steps)
    assert a.state[:, 6].min() > 1.0  # the X2 layer is crossed
    e = (np.abs(a.state[:, 6] - b.state[:, 6]) / a.state[:, 6]).max()
    assert e <= 1e-10, e
    print(f"TORJ_TRAJ_LDS={mode}: warm model 2 split vs fused tau {e:.1e}")


@pytest.mark.parametrize("mode", ["0", "1", "2", "3"])
def test_nan_alpha_replay_bit_identical(gpu, T, hplasma, mode):
    """A ray whose alpha goes non-finite at step s stops NAN with the state
    x_s, which k_split_final rebuilds from the chunk-boundary copy by replaying
    the steps since (cold_replay).  The replay uses the arithmetic of the
    trajectory kernel that ran (cell power form for TORJ_TRAJ_LDS=3, the node
    tile's global fallback for 2, the node stencil for 0 and 1), so x_s is bit
    for bit the trajectory's own (mode 1 reads the same values from LDS in a
    separately compiled kernel: 1e-14): the test hook
    TORJ_TEST_NAN_ALPHA_STEP=s makes the scan read alpha as NaN at step s for
    every third ray, and those rays must equal a clean trace of s steps."""
    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    s_nan = 537  # mid-chunk (chunk 20): a replay of 17 steps
    kw = dict(ds=1e-4, weights=w, traj_stride=0, chunk_steps=20)
    clean_full = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": mode}, xp, Np, om, 1, n_steps=1500, **kw)
    hooked = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": mode, "TORJ_TEST_NAN_ALPHA_STEP": str(s_nan)},
                      xp, Np, om, 1, n_steps=1500, **kw)
    clean_s = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": mode}, xp, Np, om, 1, n_steps=s_nan, **kw)
    idx = np.arange(len(w))
    hit = (idx % 3 == 0) & (clean_s.status == T.OK) & (clean_s.steps == s_nan)
    assert hit.sum() > 50
    assert (hooked.status[hit] == T.NAN).all() and (hooked.steps[hit] == s_nan).all()
    if mode == "1":
        e = np.abs(hooked.state[hit, :6] - clean_s.state[hit, :6]).max() / np.abs(clean_s.state[hit, :6]).max()
        assert e <= 1e-14, e
    else:
        assert np.array_equal(hooked.state[hit, :6], clean_s.state[hit, :6])
    rest = ~hit & ((idx % 3 != 0) | (clean_s.status != T.OK))
    for f in ("status", "steps"):
        assert np.array_equal(getattr(hooked, f)[rest], getattr(clean_full, f)[rest]), f
    assert np.array_equal(hooked.state[rest], clean_full.state[rest])


@pytest.mark.parametrize("tile,caps", [("2", ("30", "0")), ("3", ("2", "0"))])
def test_traj_tile_bit_identical_to_global_fallback(gpu, T, hplasma, tile, caps):
    """k_traj_tile (TORJ_TRAJ_LDS=2) stages per wave only the coefficient tile
    its rays can reach in the block and reads a stencil outside it from global
    memory (torj_hip.hip traj_body); k_traj_cell (=3) does the same with the
    cells' power-form records (torj_math.hpp cell_sums).  Either kernel with the
    tile's margin at 0 (rays leave their tile mid-block: the per-evaluation
    fallback), with a small cap (some waves untiled) and with no tile at all
    gives bit-identical outputs; against the whole-grid LDS kernel and the L2
    kernel (separately compiled; for =3 also a different rounding of the same
    interpolant) to 1e-12, statuses and steps exact."""
    from test_gpu_c3 import _close

    pos, xp, Np, s0, w, om = _fan(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, weights=w, traj_stride=100, psi_grid=np.linspace(0, 1, 1000),
              deposition="reference", x_launch=pos, s0=s0)
    ref = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": tile}, xp, Np, om, 1, **kw)
    for env in ({"TORJ_TILE_MARGIN": "0"}, {"TORJ_TILE_CAP": caps[0]}, {"TORJ_TILE_CAP": caps[1]}):
        r = _env_run(T, hplasma, dict(env, TORJ_TRAJ_LDS=tile), xp, Np, om, 1, **kw)
        for f in ("state", "status", "steps", "P_dep", "dP_shell"):
            assert np.array_equal(getattr(ref, f), getattr(r, f)), (env, f)
        assert np.array_equal(ref.traj, r.traj, equal_nan=True), env
    for mode in ("1", "0"):
        r = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": mode}, xp, Np, om, 1, **kw)
        _close(ref, r, 1e-12)
        e = (np.abs(ref.state[:, :3] - r.state[:, :3]).max(1) / np.linalg.norm(r.state[:, :3], axis=1)).max()
        print(f"TORJ_TRAJ_LDS={mode} vs {tile}: bit-identical state {np.array_equal(ref.state, r.state)}, "
              f"max rel x {e:.1e}")


@pytest.mark.parametrize("tile", ["2", "3"])
def test_traj_tile_vs_oracle_with_stops(gpu, T, hplasma, oplasma, tile):
    """The tiled trajectory kernels against the oracle with ABSORBED and
    LEFT_PLASMA stops mid-block (as test_split_termination_vs_oracle)."""
    from test_gpu_parity import _compare_trace

    pos, xp, Np, s0, w, om = _fan(T, hplasma, n_rings=4)
    grid = np.linspace(0, 1, 300)
    kw = dict(ds=1e-4, n_steps=4000, chunk_steps=40, psi_grid=grid, traj_stride=50, P_min=1e-2)
    g = _env_run(T, hplasma, {"TORJ_TRAJ_LDS": tile, "TORJ_TILE_MARGIN": "0.5"}, xp, Np, om, 1, **kw)
    o = oplasma.trace(xp, Np, om, 1, 1e-4, 4000, chunk_steps=40, psi_grid=grid, traj_stride=50,
                      P_min=1e-2)
    _compare_trace(g, o)
    assert np.abs(g.dP_shell[:-1] - o["dP"]).max() <= 1e-10 * np.abs(o["dP"]).max()
