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
    return L


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(_dp)


def _run(H, n_steps, grid, s0, steps, psiL, smp, nc, ds=1e-4):
    n = len(s0)
    psi = np.ascontiguousarray(smp[:, :, 0].T)   # (n_steps + 1) x n
    dpds = np.ascontiguousarray(smp[:, :, 1].T)
    dPs = np.zeros((len(grid) - 1, n))
    kstar = np.zeros(n, dtype=np.int32)
    P = np.zeros(n)
    st = np.ascontiguousarray(steps, dtype=np.int32)
    H.fd_profile(n, n_steps, len(grid), ds, _d(grid), _d(s0), st.ctypes.data_as(_ip), _d(psiL),
                 _d(psi), _d(dpds), nc, _d(dPs), kstar.ctypes.data_as(_ip), _d(P))
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
