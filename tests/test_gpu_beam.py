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
        assert abs(a7[i][-1] - a1[i][-1]) <= 1e-12
        assert np.array_equal(p7[i][2:-1], p1[i][2:][6::7][:len(p7[i]) - 3])
