"""The product's reference-faithful deposition (torj_fitdepo.hpp fit_depo_ray,
the body of k_fit_depo), host build (tests/native), against
power_deposition_profile restated on scipy's FITPACK (oracle/deposition_ref.py),
on the CPU oracle's make_ray vectors: the same check as
tests/test_gpu_deposition.py without a GPU, plus the open-shell cache's spill
path (a one-entry cache spills on every second open shell) giving results
bit-identical to the default cache."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
_dp, _ip = C.POINTER(C.c_double), C.POINTER(C.c_int)


@pytest.fixture(scope="module")
def H():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
    L = C.CDLL(os.path.join(HERE, "native", "build", "libwarm_host.so"))
    L.fd_profile.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, _dp, _dp, _ip, _dp, _dp, _dp,
                             C.c_int, _dp, _ip, _dp]
    L.fd_profile_stream.argtypes = L.fd_profile.argtypes
    return L


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(_dp)


def _run(H, n_steps, grid, s0, steps, psiL, smp, nc, ds=1e-4, stream=0):
    """nc: the open-shell cache; stream != 0: the streamed walk (fd_profile_stream,
    the scan's steps growing by |stream| per emulated block; < 0 the split form,
    elimination and walk of one window per block)"""
    n = len(s0)
    psi = np.ascontiguousarray(smp[:, :, 0].T)   # (n_steps + 1) x n
    dpds = np.ascontiguousarray(smp[:, :, 1].T)
    dPs = np.zeros((len(grid) - 1, n))
    kstar = np.zeros(n, dtype=np.int32)
    P = np.zeros(n)
    st = np.ascontiguousarray(steps, dtype=np.int32)
    f = H.fd_profile_stream if stream else H.fd_profile
    f(n, n_steps, len(grid), ds, _d(grid), _d(s0), st.ctypes.data_as(_ip), _d(psiL),
      _d(psi), _d(dpds), stream if stream else nc, _d(dPs), kstar.ctypes.data_as(_ip), _d(P))
    return dPs, kstar, P


@pytest.mark.parametrize("mode,grid_kind", [(1, "uniform"), (-1, "uniform"), (1, "graded")])
def test_host_deposition_matches_fitpack(H, T, hplasma, oplasma, mode, grid_kind):
    import deposition_ref as D
    from torj_hip import synthetic as S

    s = S.SETUP
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], s["f_abs_test"],
                                            N_rings=2, min_azimuthal_points=5)
    om = 2 * np.pi * s["f_abs_test"]
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, mode)
    assert (st == 0).all()
    # graded: boundaries packed towards the axis (the in-kernel lookup guesses as
    # if uniform and walks to the right boundary)
    grid = np.linspace(0, 1, 250) if grid_kind == "uniform" else np.linspace(0, 1, 250) ** 2
    n_steps = 3000
    o = oplasma.trace(xp, Np, om, mode, 1e-4, n_steps, psi_grid=grid, weights=w, samples=True, s0=s0)
    psiL = np.array([oplasma.evaluate("psi", p) for p in pos])
    dPs, kstar, P = _run(H, n_steps, grid, s0, o["steps"], psiL, o["samples"], 2)
    dV = np.diff([oplasma.volume(p) for p in grid])
    shell_ref, P_ref = np.zeros(len(grid) - 1), np.zeros(len(pos))
    shell = np.zeros(len(grid) - 1)
    for i in range(len(pos)):
        sv, psi, dpds = D.ray_vectors(pos[i], s0[i], 1e-4, o["steps"][i], o["samples"][i], psiL[i])
        prof, P_ref[i] = D.power_deposition_profile(sv, psi, dpds, grid, oplasma.volume)
        shell_ref += w[i] * prof[:-1] * dV
        keep = np.arange(len(grid) - 1) > kstar[i]  # k_shell_sum: shells above the break
        shell += w[i] * np.where(keep, dPs[:, i], 0.0)
    scale = np.abs(shell_ref).max()
    assert scale > 0
    assert np.abs(shell - shell_ref).max() <= 1e-11 * scale
    assert np.abs(P - P_ref).max() <= 1e-11 * max(P_ref.max(), 1e-300)
    # spill path: a one-entry open-shell cache keeps the second open shell in memory
    for nc in (1, 4):
        d2, k2, P2 = _run(H, n_steps, grid, s0, o["steps"], psiL, o["samples"], nc)
        assert np.array_equal(k2, kstar) and np.array_equal(P2, P) and np.array_equal(d2, dPs)
    # the streamed walk (windows behind the scan, then the tail): independent of
    # the block schedule bit for bit, and the one-pass walk's result to rounding
    d60, k60, P60 = _run(H, n_steps, grid, s0, o["steps"], psiL, o["samples"], 2, stream=60)
    d37, k37, P37 = _run(H, n_steps, grid, s0, o["steps"], psiL, o["samples"], 2, stream=37)
    assert np.array_equal(k60, k37) and np.array_equal(P60, P37) and np.array_equal(d60, d37)
    # the split form (TORJ_DEPO_STREAM=3: elimination and walk of one window as
    # two launches per block): the same windows, the same bits
    ds_, ks_, Ps_ = _run(H, n_steps, grid, s0, o["steps"], psiL, o["samples"], 2, stream=-60)
    assert np.array_equal(k60, ks_) and np.array_equal(P60, Ps_) and np.array_equal(d60, ds_)
    assert np.array_equal(k60, kstar)
    assert np.abs(P60 - P).max() <= 1e-13 * P.max()
    assert np.abs(d60 - dPs).max() <= 1e-13 * np.abs(dPs).max()


@pytest.mark.parametrize("periods", [3, 7])
def test_host_deposition_root_cap_maxn_8(H, oplasma, periods):
    """Dierckx.roots' maxn = 8 (src/plasma.jl:108,118; FITPACK sproot with
    mest = 8): a ray whose psi(s) oscillates across the same surfaces keeps only
    the first 8 roots of each boundary in s order.  Synthetic make_ray vectors
    (psi(s) = 0.5 + 0.03 sin, periods full oscillations over the path) through
    the product's fit (host build) against scipy's FITPACK restatement with
    mest = 8 -- and, for 7 periods (14 roots per boundary), not equal to the
    uncapped profile, so the cap is what is being checked."""
    import warnings

    import deposition_ref as D

    n_steps, ds, s0 = 3000, 1e-4, 0.05
    grid = np.linspace(0, 1, 250)
    s = s0 + ds * np.arange(n_steps + 1)
    u = (s - s0) / (n_steps * ds)
    # in from the edge (launch point outside, psi = 1 at entry) to psi = 0.5 over
    # the first 30 % of the path, then oscillating about it
    v = np.clip((u - 0.3) / 0.7, 0.0, 1.0)
    psi = np.where(u < 0.3, 1.0 - (0.5 / 0.3) * u, 0.5) + 0.03 * np.sin(2 * np.pi * periods * v) \
        + 0.002 * u
    dpds = np.exp(-((u - 0.45) / 0.3) ** 2) * (1.0 + 0.2 * np.cos(5 * u))
    dpds[0] = 0.0  # make_ray's dP/ds is 0 at the entry point
    psiL = 1.2
    smp = np.stack([psi, dpds, s], axis=1)[None]  # (1, n_steps + 1, 3)
    dPs, kstar, P = _run(H, n_steps, grid, np.array([s0]), np.array([n_steps]), np.array([psiL]),
                         smp, 2, ds)
    sv = np.concatenate([[0.0], s])
    psi_v = np.concatenate([[psiL], psi])
    dp_v = np.concatenate([[0.0], dpds])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # scipy: "The number of zeros exceeds mest"
        prof8, P8 = D.power_deposition_profile(sv, psi_v, dp_v, grid, oplasma.volume, maxn=8)
        prof_all, P_all = D.power_deposition_profile(sv, psi_v, dp_v, grid, oplasma.volume, maxn=1000)
    dV = np.diff([oplasma.volume(p) for p in grid])
    keep = np.arange(len(grid) - 1) > kstar[0]
    shell = np.where(keep, dPs[:, 0], 0.0)
    ref = prof8[:-1] * dV
    assert np.abs(shell - ref).max() <= 1e-11 * np.abs(ref).max()
    assert abs(P[0] - P8) <= 1e-11 * P8
    if periods == 7:
        assert abs(P_all - P8) > 1e-3 * P8  # the cap changes the reference's answer
    # open-shell spill path under the capped walk
    d1, k1, P1 = _run(H, n_steps, grid, np.array([s0]), np.array([n_steps]), np.array([psiL]), smp, 1, ds)
    assert np.array_equal(d1, dPs) and np.array_equal(k1, kstar) and np.array_equal(P1, P)
    # the streamed walk detects the runs and redoes the ray whole with the cap
    d2, k2, P2 = _run(H, n_steps, grid, np.array([s0]), np.array([n_steps]), np.array([psiL]), smp, 2, ds,
                      stream=60)
    if periods == 7:
        assert np.array_equal(d2, dPs) and np.array_equal(k2, kstar) and np.array_equal(P2, P)
    else:
        assert np.array_equal(k2, kstar) and abs(P2[0] - P[0]) <= 1e-13 * P[0]
        assert np.abs(d2 - dPs).max() <= 1e-13 * np.abs(dPs).max()
