"""make_beam's multi-GPU path in the library (torj_trace_beam, SURVEY.md §8(b)
/ (e); reference fan-out src/solve.jl:219-224 and reduce :233-240) on one
MI355X: the beam cut into shards traced in turn on the device, the dP_shell
partials summed (RCCL all-reduce when forced), against the unsplit
torj_trace_ex launch.  Per-ray outputs bit-identical (shard boundaries fall on
64-ray groups, so every wave holds the same rays); dP_shell equal to the order
of its fp64 sums (1e-13 of the profile maximum)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _beam(T, hplasma, n_rings=14, min_az=5):
    from torj_hip import synthetic as S

    s = S.SETUP
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], s["f_abs_test"],
                                            N_rings=n_rings, min_azimuthal_points=min_az)
    om = 2 * np.pi * s["f_abs_test"]
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, 1, gpu=True)
    assert (st == T.OK).all()
    return pos, xp, Np, s0, w, om


def _same(a, b):
    for f in ("state", "status", "steps", "P_dep"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.array_equal(a.traj, b.traj, equal_nan=True)
    assert np.abs(a.dP_shell - b.dP_shell).max() <= 1e-13 * np.abs(a.dP_shell).max()


@pytest.mark.parametrize("deposition", ["reference", "binned"])
@pytest.mark.parametrize("rccl", [False, True])
def test_trace_beam_shards_equal_unsplit(gpu, T, hplasma, deposition, rccl):
    pos, xp, Np, s0, w, om = _beam(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, psi_grid=np.linspace(0, 1, 1000), weights=w, traj_stride=100,
              deposition=deposition, x_launch=pos, s0=s0)
    old = os.environ.get("TORJ_BEAM_RCCL")
    try:
        hplasma.set_sched(0)  # one lane per ray in both (the 16-lane split is per-wave rounding)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        os.environ["TORJ_BEAM_RCCL"] = "1" if rccl else "0"
        b = T.trace(hplasma, xp, Np, om, 1, n_gpus=1, n_shards=4, **kw)
    finally:
        hplasma.set_sched(-1)
        if old is None:
            os.environ.pop("TORJ_BEAM_RCCL", None)
        else:
            os.environ["TORJ_BEAM_RCCL"] = old
    _same(a, b)
    assert b.dP_shell[-1] > 0


def test_trace_beam_default_scheduling_and_ragged(gpu, T, hplasma, oplasma):
    """Default scheduling per shard (16-lane kernel for these small shards),
    more shards than 64-ray groups (empty shards), a ragged last group; vs the
    oracle at the parity bar."""
    from test_gpu_parity import _compare_trace

    pos, xp, Np, s0, w, om = _beam(T, hplasma, n_rings=4, min_az=5)
    n = len(w)
    assert n % 64 != 0
    grid = np.linspace(0, 1, 400)
    g = T.trace(hplasma, xp, Np, om, 1, ds=1e-4, n_steps=1500, psi_grid=grid, weights=w,
                n_gpus=1, n_shards=(n + 63) // 64 + 3)
    o = oplasma.trace(xp, Np, om, 1, 1e-4, 1500, psi_grid=grid, weights=w)
    _compare_trace(g, o)
    assert np.abs(g.dP_shell[:-1] - o["dP"]).max() <= 1e-10 * np.abs(o["dP"]).max()
    e = T.trace(hplasma, np.zeros((0, 3)), np.zeros((0, 3)), om, 1, n_steps=10, psi_grid=grid,
                n_gpus=1)
    assert e.state.shape == (0, 7) and not e.dP_shell.any()


def test_trace_beam_errors(gpu, T, hplasma):
    pos, xp, Np, s0, w, om = _beam(T, hplasma, n_rings=2, min_az=3)
    with pytest.raises(T.TorjError, match="HIP devices are visible"):
        T.trace(hplasma, xp, Np, om, 1, n_steps=10, n_gpus=gpu + 1)
    bad = np.linspace(0, 1, 50)
    bad[10] = bad[9]
    with pytest.raises(T.TorjError, match="strictly increasing"):
        T.trace(hplasma, xp, Np, om, 1, n_steps=10, psi_grid=bad, n_gpus=1)


def test_make_beam_traj_stride_keeps_final_state(gpu, T, eq):
    """make_beam with traj_stride not dividing the step count: ray_powers[i][-1]
    is the ray's final P (the reference's absorbed-power check reads it)."""
    from torj_hip import synthetic as S

    P = T.Plasma(*S.plasma_args(S.circular_tokamak(ne_scale=0.3)))
    s = S.SETUP
    grid = np.linspace(0, 1, 200)
    args = (P, s["R0"], s["phi0"], s["z0"], s["steering_angle_tor"], s["steering_angle_pol"],
            s["spot_size"], s["inverse_curvature_radius"], s["f_abs_test"], 1, 0.3, grid)
    a1, t1, p1, d1, pa1, w1 = T.make_beam(*args, traj_stride=1)
    a7, t7, p7, d7, pa7, w7 = T.make_beam(*args, traj_stride=7, n_gpus=1)
    assert pa1 == pa7 and np.array_equal(d1, d7)
    for i in range(len(w1)):
        assert p7[i][-1] == p1[i][-1] and np.array_equal(t7[i][-1], t1[i][-1])
        # the appended final arc length is the kernel's single-rounding fma
        assert a7[i][-1] == a1[i][-1]
        assert np.array_equal(p7[i][2:-1], p1[i][2:][6::7][:len(p7[i]) - 3])


class _env:
    """Set environment variables for a block (the library reads these per call)."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("deposition", ["reference", "binned"])
def test_trace_beam_threaded_replicas_on_one_device(gpu, T, hplasma, deposition):
    """The multi-replica branch of torj_trace_beam -- one std::thread, stream and
    workspace per replica, the branch make_beam(...; n_gpus = 8) takes -- run on
    one MI355X with the test-only placement TORJ_BEAM_SAME_DEVICE=1 (both
    replicas on device 0, partials summed on the host).  Per-ray outputs
    bit-identical to the unsplit launch, dP_shell to its summation order."""
    pos, xp, Np, s0, w, om = _beam(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, psi_grid=np.linspace(0, 1, 1000), weights=w, traj_stride=100,
              deposition=deposition, x_launch=pos, s0=s0)
    try:
        hplasma.set_sched(0)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        with _env(TORJ_BEAM_SAME_DEVICE="1"):
            b = T.trace(hplasma, xp, Np, om, 1, n_gpus=2, n_shards=5, **kw)
            c = T.trace(hplasma, xp, Np, om, 1, n_gpus=3, **kw)
    finally:
        hplasma.set_sched(-1)
    _same(a, b)
    _same(a, c)
    assert b.dP_shell[-1] > 0


def _device_shards(torch, T, plasma, cfg, n_psi, grid, xp, Np, w, pos, s0, cuts, dev):
    """Device-resident shards for torj_trace_beam_device (all on `dev`)."""
    n_save = cfg.n_steps // cfg.traj_stride if cfg.traj_stride > 0 else 0

    def d(a, dtype=torch.float64):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype)

    shards = []
    for sl in cuts:
        m = sl.stop - sl.start
        shards.append(dict(
            n=m, x0=d(xp[sl].T), N0=d(Np[sl].T), weights=d(w[sl]), psi_grid=d(grid),
            x_launch=d(pos[sl].T), s0=d(s0[sl]),
            state=torch.empty((7, m), dtype=torch.float64, device=dev),
            status=torch.empty(m, dtype=torch.int32, device=dev),
            steps=torch.empty(m, dtype=torch.int32, device=dev),
            dP_shell=torch.zeros(n_psi + 1, dtype=torch.float64, device=dev),
            P_dep=torch.empty(m, dtype=torch.float64, device=dev),
            traj=torch.empty((max(n_save, 1), 5, m), dtype=torch.float64, device=dev) if n_save else None,
            counters=torch.zeros(8, dtype=torch.int64, device=dev)))
    return shards


def test_trace_beam_device_shards_threaded(gpu, T, hplasma):
    """torj_trace_beam_device (device-resident shards, the bench's multi-GPU
    library path) with three replicas on device 0 (TORJ_BEAM_SAME_DEVICE=1):
    each shard's outputs bit-identical to the unsplit torj_trace_ex launch of
    the same rays, every shard's dP_shell = the beam's sum after the reduce,
    and the work counters add up to the unsplit launch's."""
    import torch

    from torj_hip._lib import TraceCfg
    from torj_hip.parallel import group_shard, trace_beam_device

    pos, xp, Np, s0, w, om = _beam(T, hplasma)
    n = len(w)
    grid = np.linspace(0, 1, 1000)
    kw = dict(ds=1e-4, n_steps=2000, psi_grid=grid, weights=w, traj_stride=100,
              deposition="reference", x_launch=pos, s0=s0)
    cfg = TraceCfg(om, 1, 1e-4, 2000, 20, 1.0, 1e-6, 1, 100, 1)
    dev = torch.device("cuda", 0)
    try:
        hplasma.set_sched(0)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        cuts = [group_shard(n, 3, k) for k in range(3)]
        sh = _device_shards(torch, T, hplasma, cfg, len(grid), grid, xp, Np, w, pos, s0, cuts, dev)
        L = T.lib()
        T._lib.check(L.torj_timing(hplasma.handle, 1))
        with _env(TORJ_BEAM_SAME_DEVICE="1"):
            trace_beam_device(hplasma, cfg, len(grid), sh)
        # torj_beam_timing_read: one recorded call per replica, a trace phase
        # each, and no reduce time (the same-device placement sums on the host)
        import ctypes as C
        calls, t_tr, t_po, t_red = (C.c_int * 3)(), (C.c_double * 3)(), (C.c_double * 3)(), C.c_double(-1)
        T._lib.check(L.torj_beam_timing_read(hplasma.handle, 3, calls, t_tr, t_po, C.byref(t_red)))
        T._lib.check(L.torj_timing(hplasma.handle, 0))
        assert list(calls) == [1, 1, 1] and all(t > 0 for t in t_tr) and all(t > 0 for t in t_po)
        assert t_red.value >= 0.0
        assert L.torj_beam_timing_read(hplasma.handle, 9, calls, t_tr, t_po, None) != 0  # 3 replicas
        # torj_beam_comm_info: three replicas on device 0, no communicator (host sum)
        from torj_hip.parallel import beam_comm_info
        ci = beam_comm_info(hplasma, 3)
        assert ci == {"device": [0, 0, 0], "rccl_nranks": [0, 0, 0], "rccl_rank": [-1, -1, -1]}, ci
        assert L.torj_beam_comm_info(hplasma.handle, 9, (C.c_int * 9)(), (C.c_int * 9)(),
                                     (C.c_int * 9)()) != 0
        c1 = torch.zeros(8, dtype=torch.int64, device=dev)
        one = _device_shards(torch, T, hplasma, cfg, len(grid), grid, xp, Np, w, pos, s0, [slice(0, n)], dev)
        one[0]["counters"] = c1
        trace_beam_device(hplasma, cfg, len(grid), one)
    finally:
        hplasma.set_sched(-1)
    for sl, s in zip(cuts, sh):
        assert np.array_equal(s["state"].cpu().numpy().T, a.state[sl])
        assert np.array_equal(s["status"].cpu().numpy(), a.status[sl])
        assert np.array_equal(s["steps"].cpu().numpy(), a.steps[sl])
        assert np.array_equal(s["P_dep"].cpu().numpy(), a.P_dep[sl])
        assert np.array_equal(s["traj"].cpu().numpy().transpose(2, 0, 1), a.traj[sl], equal_nan=True)
        d = s["dP_shell"].cpu().numpy()
        assert np.abs(d - a.dP_shell).max() <= 1e-13 * np.abs(a.dP_shell).max()
    tot = sum(s["counters"].cpu().numpy() for s in sh)
    assert np.array_equal(tot, c1.cpu().numpy()) and tot[0] == int(a.steps.sum())
    assert np.array_equal(one[0]["dP_shell"].cpu().numpy(), a.dP_shell)


def test_trace_beam_one_replica_rccl_comm_info(gpu, T, hplasma):
    """One replica with the RCCL reduce forced (TORJ_BEAM_RCCL=1): a real
    one-rank communicator on device 0, which torj_beam_comm_info reports (rank
    count 1, rank 0); dP_shell is unchanged by the one-rank all-reduce."""
    from torj_hip.parallel import beam_comm_info

    pos, xp, Np, s0, w, om = _beam(T, hplasma)
    kw = dict(ds=1e-4, n_steps=200, psi_grid=np.linspace(0, 1, 100), weights=w, x_launch=pos, s0=s0)
    a = T.trace(hplasma, xp, Np, om, 1, n_gpus=1, **kw)
    with _env(TORJ_BEAM_RCCL="1"):
        b = T.trace(hplasma, xp, Np, om, 1, n_gpus=1, **kw)
    assert beam_comm_info(hplasma, 1) == {"device": [0], "rccl_nranks": [1], "rccl_rank": [0]}
    assert np.array_equal(a.dP_shell, b.dP_shell)


def test_trace_beam_two_devices(gpu, T, hplasma):
    """n_gpus = 2 on two real devices (skipped only on a one-GPU box; with two
    or more devices visible it runs and must pass): RCCL all-reduce over xGMI,
    per-ray bit-identical to the unsplit launch, and the communicator spans two
    ranks on two distinct devices (torj_beam_comm_info)."""
    from torj_hip.parallel import beam_comm_info

    if gpu < 2:
        pytest.skip(f"needs two HIP devices, {gpu} visible")
    pos, xp, Np, s0, w, om = _beam(T, hplasma)
    kw = dict(ds=1e-4, n_steps=2000, psi_grid=np.linspace(0, 1, 1000), weights=w, traj_stride=100,
              deposition="reference", x_launch=pos, s0=s0)
    try:
        hplasma.set_sched(0)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        b = T.trace(hplasma, xp, Np, om, 1, n_gpus=2, **kw)
        ci = beam_comm_info(hplasma, 2)
    finally:
        hplasma.set_sched(-1)
    _same(a, b)
    assert ci["rccl_nranks"] == [2, 2] and sorted(ci["rccl_rank"]) == [0, 1], ci
    assert len(set(ci["device"])) == 2, ci


def test_c4_million_ray_beam_sharded_rccl_batched(gpu, T, hplasma, oplasma):
    """C4 (BASELINE configs[3]) on one MI355X: the 1 005 293-ray fan
    (N_rings = 291, min_az = 11), 2 000 RK4 steps, Albajar, the reference
    deposition on 1 000 shells, through make_beam's library path
    torj_trace_beam with 8 shards, the RCCL reduce forced (TORJ_BEAM_RCCL=1) and
    the per-launch workspace capped at 4 GiB (TORJ_WS_GB) so every shard runs in
    ray batches.  Every 250th ray vs the CPU oracle at the parity bar (status
    and steps exact, x, N, tau 1e-10); per-ray outputs bit-identical to one
    unsplit torj_trace_ex launch of the beam (one launch under the default
    workspace budget, half the free device memory; both on the split pipeline,
    forced by set_sched(3), so every wave holds the same rays), dP_shell to its
    summation order."""
    from test_gpu_parity import _compare_trace
    from torj_hip import synthetic as S

    s = S.SETUP
    f = s["f_abs_test"]
    om = 2 * np.pi * f
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=291,
                                            min_azimuthal_points=11)
    assert len(w) == 1005293
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, 1, gpu=True)
    assert (st == T.OK).all()
    grid = np.linspace(0.0, 1.0, 1000)
    kw = dict(ds=1e-4, n_steps=2000, psi_grid=grid, weights=w, traj_stride=500,
              deposition="reference", x_launch=pos, s0=s0)
    try:
        hplasma.set_sched(3)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        with _env(TORJ_BEAM_RCCL="1", TORJ_WS_GB="4"):
            b = T.trace(hplasma, xp, Np, om, 1, n_gpus=1, n_shards=8, **kw)
    finally:
        hplasma.set_sched(-1)
    _same(a, b)
    idx = np.arange(0, len(w), 250)
    o = oplasma.trace(xp[idx], Np[idx], om, 1, 1e-4, 2000, psi_grid=grid, weights=w[idx])
    sub = type(b)(b.state[idx], b.status[idx], b.steps[idx], None, None, None)
    _compare_trace(sub, o)
    assert abs(b.dP_shell[-1] - np.dot(w, b.P_dep)) <= 1e-12 * b.dP_shell[-1]
    # make_beam's deposited power (normalised weights): most of the beam power is
    # absorbed in the X2 layer, though the 291-ring fan's outer rings miss it
    assert 0.5 < b.dP_shell[-1] <= 1.0 + 1e-12


@pytest.mark.parametrize("sched", [3, 1])
def test_trace_device_null_stream_equals_explicit_stream(gpu, T, hplasma, sched):
    """torj_trace_device_ex on the legacy NULL stream -- served on the handle's
    own non-blocking stream with fork / join events against it -- equals the
    same call on an explicit stream bit for bit (the split pipeline, sched 3,
    and the work queue, sched 1), and the outputs are complete when the NULL
    stream is synchronised."""
    import torch

    from torj_hip._lib import TraceCfg

    pos, xp, Np, s0, w, om = _beam(T, hplasma)
    n = len(w)
    grid = np.linspace(0, 1, 200)
    cfg = TraceCfg(om, 1, 1e-4, 600, 20, 1.0, 1e-6, 1, 100, 1)
    dev = torch.device("cuda", 0)
    outs = []
    try:
        hplasma.set_sched(sched)
        for explicit in (False, True):
            sh = _device_shards(torch, T, hplasma, cfg, len(grid), grid, xp, Np, w, pos, s0,
                                [slice(0, n)], dev)[0]
            torch.cuda.synchronize()
            st = torch.cuda.Stream(device=dev) if explicit else None
            T._lib.check(T.lib().torj_trace_device_ex(
                hplasma.handle, cfg, n, sh["x0"].data_ptr(), sh["N0"].data_ptr(), sh["weights"].data_ptr(),
                len(grid), sh["psi_grid"].data_ptr(), sh["x_launch"].data_ptr(), sh["s0"].data_ptr(),
                sh["state"].data_ptr(), sh["status"].data_ptr(), sh["steps"].data_ptr(),
                sh["dP_shell"].data_ptr(), sh["P_dep"].data_ptr(), sh["traj"].data_ptr(), None,
                st.cuda_stream if explicit else None))
            T._lib.check(T.lib().torj_trace_check(hplasma.handle, st.cuda_stream if explicit else None))
            outs.append({k: sh[k].cpu().numpy() for k in ("state", "status", "steps", "dP_shell", "P_dep", "traj")})
    finally:
        hplasma.set_sched(-1)
    a, b = outs
    assert (a["steps"] > 0).all()
    for k in ("state", "status", "steps", "dP_shell", "P_dep"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["traj"], b["traj"], equal_nan=True)
