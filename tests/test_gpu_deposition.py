"""GPU parity of the reference-faithful deposition (torj_trace_cfg.deposition = 1)
against power_deposition_profile restated on scipy's FITPACK
(oracle/deposition_ref.py -- the same curfit/sproot/splint Dierckx.jl wraps),
fed with the CPU oracle's make_ray vectors for the same rays.

Tolerance: shell powers and per-ray deposited power <= 1e-11 relative (measured
on MI355X: 1.4e-13 / 6e-14).  The GPU solves the not-a-knot interpolant in
second-derivative form (Thomas), FITPACK in B-spline form (Givens QR): both
interpolate the same points up to rounding, amplified by the spacing ratio
s0 / ds ~ 1e3 of the vacuum segment."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref_profile(D, oplasma, pos, s0, ds, o, grid, w):
    dV = np.diff([oplasma.volume(p) for p in grid])
    shell = np.zeros(len(grid) - 1)
    P = np.zeros(len(pos))
    for i in range(len(pos)):
        sv, psi, dpds = D.ray_vectors(pos[i], s0[i], ds, o["steps"][i], o["samples"][i],
                                      oplasma.evaluate("psi", pos[i]))
        prof, P[i] = D.power_deposition_profile(sv, psi, dpds, grid, oplasma.volume)
        shell += w[i] * prof[:-1] * dV
    return shell, P


def _fan(T, hplasma, mode, n_rings=3, min_az=5):
    from torj_hip import synthetic as S

    s = S.SETUP
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], s["f_abs_test"],
                                            N_rings=n_rings, min_azimuthal_points=min_az)
    om = 2 * np.pi * s["f_abs_test"]
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, mode)
    assert (st == 0).all()
    return pos, xp, Np, s0, w, om


@pytest.mark.parametrize("mode", [1, -1])
def test_reference_deposition_matches_fitpack(gpu, T, hplasma, oplasma, mode):
    import deposition_ref as D

    pos, xp, Np, s0, w, om = _fan(T, hplasma, mode)
    grid = np.linspace(0, 1, 250)
    kw = dict(ds=1e-4, n_steps=3000, psi_grid=grid, weights=w)
    g = T.trace(hplasma, xp, Np, om, mode, deposition="reference", x_launch=pos, s0=s0, **kw)
    o = oplasma.trace(xp, Np, om, mode, 1e-4, 3000, psi_grid=grid, weights=w, samples=True, s0=s0)
    assert np.array_equal(g.steps, o["steps"])
    shell, P = _ref_profile(D, oplasma, pos, s0, 1e-4, o, grid, w)
    scale = np.abs(shell).max()
    assert scale > 0
    assert np.abs(g.dP_shell[:-2] - shell).max() <= 1e-11 * scale
    assert g.dP_shell[-2] == 0.0
    assert np.abs(g.P_dep - P).max() <= 1e-11 * max(P.max(), 1e-300)
    assert abs(g.dP_shell[-1] - np.dot(w, P)) <= 1e-11 * max(np.dot(w, P), 1e-300)


def test_reference_deposition_nonuniform_grid_and_exits(gpu, T, hplasma, oplasma):
    """Binary-searched boundaries, rays that leave the plasma (LEFT_PLASMA: odd
    root counts, the reference drops the last root) and the break rule."""
    import deposition_ref as D

    pos, xp, Np, s0, w, om = _fan(T, hplasma, 1, n_rings=2, min_az=3)
    # plus rays launched from inside outwards (their 'launch point' is the start)
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
    x_l = x_out - 0.05 * N_out / np.linalg.norm(N_out, axis=1)[:, None]
    s_l = np.full(len(x_out), 0.05)
    pos, xp, Np = np.vstack([pos, x_l]), np.vstack([xp, x_out]), np.vstack([Np, N_out])
    s0, w = np.concatenate([s0, s_l]), np.concatenate([w, [0.1, 0.1]])
    grid = np.sort(np.concatenate([[0.0, 1.0], np.random.default_rng(3).uniform(0, 1, 120)]))
    g = T.trace(hplasma, xp, Np, om, 1, n_steps=6000, chunk_steps=60, psi_grid=grid, weights=w,
                deposition="reference", x_launch=pos, s0=s0)
    o = oplasma.trace(xp, Np, om, 1, 1e-4, 6000, chunk_steps=60, psi_grid=grid, weights=w,
                      samples=True, s0=s0)
    assert np.array_equal(g.status, o["status"]) and np.array_equal(g.steps, o["steps"])
    assert T.LEFT_PLASMA in g.status.tolist()
    shell, P = _ref_profile(D, oplasma, pos, s0, 1e-4, o, grid, w)
    scale = np.abs(shell).max()
    # rays turning inside the plasma graze some boundary: a near-double root is
    # located to ~sqrt(eps) by any method (FITPACK's and ours differ there)
    assert np.abs(g.dP_shell[:-2] - shell).max() <= 1e-8 * scale
    assert np.abs(g.P_dep - P).max() <= 1e-8 * max(P.max(), 1e-300)


def test_make_ray_reference_deposition(gpu, T, hplasma, oplasma):
    """make_ray's default deposition is the reference profile: compare the
    returned (dP_dV, deposited_power) with the FITPACK restatement."""
    import deposition_ref as D
    from torj_hip import synthetic as S

    s = S.SETUP
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    x0 = np.array([s["R0"], 0.0, s["z0"]])
    grid = np.linspace(0, 1, 400)
    sv, u, P_beam, dP_dV, pdep = T.make_ray(hplasma, x0, N0, s["f"], 1, 0.4, grid)
    om = 2 * np.pi * s["f"]
    st, xp, Np, s0 = oplasma.ray_entry(x0, N0, om, 1)
    o = oplasma.trace(xp[None], Np[None], om, 1, 1e-4, 4000, samples=True, s0=[s0])
    svr, psi, dpds = D.ray_vectors(x0, s0, 1e-4, o["steps"][0], o["samples"][0],
                                   oplasma.evaluate("psi", x0))
    prof, P = D.power_deposition_profile(svr, psi, dpds, grid, oplasma.volume)
    assert np.abs(sv - svr).max() < 1e-12
    assert np.abs(dP_dV - prof).max() <= 1e-11 * np.abs(prof).max()
    assert abs(pdep - P) <= 1e-11 * P


@pytest.mark.parametrize("n_psi", [250, 4500])
def test_reference_deposition_independent_of_scheduling(gpu, T, hplasma, n_psi):
    """Reference deposition after the work-queue kernel (groups handed between
    3 waves, samples written by different waves) is bit-identical to the one
    after the one-lane kernel, with the boundaries staged in LDS (250) and read
    from global memory (4 500)."""
    pos, xp, Np, s0, w, om = _fan(T, hplasma, 1, n_rings=8, min_az=7)
    grid = np.linspace(0, 1, n_psi)
    kw = dict(ds=1e-4, n_steps=3000, chunk_steps=150, psi_grid=grid, weights=w,
              deposition="reference", x_launch=pos, s0=s0, traj_stride=100)
    try:
        hplasma.set_sched(0)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        hplasma.set_sched(1, 3)  # 3 waves for the groups: hand-overs between waves
        b = T.trace(hplasma, xp, Np, om, 1, **kw)
    finally:
        hplasma.set_sched(-1)
    for f in ("state", "status", "steps", "P_dep", "dP_shell"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.abs(a.dP_shell).max() > 0


def test_reference_deposition_grid_beyond_lds(gpu, T, hplasma, oplasma):
    """4 500 boundaries: more than k_fit_depo stages in LDS (kFitGridLds = 4096),
    so the walk reads them from global memory; same FITPACK parity."""
    import deposition_ref as D

    pos, xp, Np, s0, w, om = _fan(T, hplasma, 1, n_rings=2, min_az=3)
    pos, xp, Np, s0, w = pos[:3], xp[:3], Np[:3], s0[:3], w[:3]
    grid = np.linspace(0, 1, 4500)
    kw = dict(ds=1e-4, n_steps=3000, psi_grid=grid, weights=w)
    g = T.trace(hplasma, xp, Np, om, 1, deposition="reference", x_launch=pos, s0=s0, **kw)
    o = oplasma.trace(xp, Np, om, 1, 1e-4, 3000, psi_grid=grid, weights=w, samples=True, s0=s0)
    assert np.array_equal(g.steps, o["steps"])
    shell, P = _ref_profile(D, oplasma, pos, s0, 1e-4, o, grid, w)
    scale = np.abs(shell).max()
    assert scale > 0
    # a fine grid makes near-grazing boundaries likelier (see the test above)
    assert np.abs(g.dP_shell[:-2] - shell).max() <= 1e-9 * scale
    assert np.abs(g.P_dep - P).max() <= 1e-9 * max(P.max(), 1e-300)


def test_reference_deposition_in_ray_batches(gpu, T, hplasma):
    """A beam whose reference-deposition workspace exceeds the budget
    (TORJ_WS_GB) is traced in contiguous batches of whole 64-ray groups: every
    per-ray output equals the single launch bit for bit, dP_shell to its
    summation order."""
    import os

    pos, xp, Np, s0, w, om = _fan(T, hplasma, 1, n_rings=14, min_az=5)
    grid = np.linspace(0, 1, 1000)
    kw = dict(ds=1e-4, n_steps=3000, psi_grid=grid, weights=w, deposition="reference", x_launch=pos,
              s0=s0, traj_stride=100)
    old = os.environ.get("TORJ_WS_GB")
    try:
        hplasma.set_sched(0)
        a = T.trace(hplasma, xp, Np, om, 1, **kw)
        os.environ["TORJ_WS_GB"] = "0.05"  # ~160 KB per ray: batches of 256 rays
        b = T.trace(hplasma, xp, Np, om, 1, **kw)
    finally:
        hplasma.set_sched(-1)
        if old is None:
            os.environ.pop("TORJ_WS_GB", None)
        else:
            os.environ["TORJ_WS_GB"] = old
    for f in ("state", "status", "steps", "P_dep"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert np.array_equal(a.traj, b.traj, equal_nan=True)
    assert np.abs(a.dP_shell - b.dP_shell).max() <= 1e-13 * np.abs(a.dP_shell).max()


def _oscillating_ray(periods, n=3001, s0=0.05, ds=1e-4, R0=1.7, a=0.6):
    """make_ray-style vectors of a synthetic path in the midplane whose psi goes
    from outside the plasma in to 0.5 and then oscillates about it (the
    circular equilibrium's psi_norm ~ ((R - R0)^2 + Z^2) / a^2)."""
    s = np.concatenate([[0.0], s0 + ds * np.arange(n)])
    u = (s[1:] - s0) / (ds * (n - 1))
    v = np.clip((u - 0.3) / 0.7, 0.0, 1.0)
    target = np.where(u < 0.3, 1.0 - (0.5 / 0.3) * u, 0.5) + 0.03 * np.sin(2 * np.pi * periods * v)
    target = np.concatenate([[1.2], target])
    R = R0 + a * np.sqrt(target)
    x = np.stack([R, np.zeros_like(R), np.zeros_like(R)], axis=1)
    uu = np.concatenate([[0.0], u])
    dpds = np.exp(-((uu - 0.45) / 0.3) ** 2) * (1.0 + 0.2 * np.cos(5 * uu))
    dpds[:2] = 0.0
    return s, x, dpds


@pytest.mark.parametrize("periods", [3, 7])
def test_power_deposition_profile_entry_root_cap(gpu, T, hplasma, oplasma, periods):
    """torj_power_deposition_profile (src/plasma.jl:91-151 as an entry point) on
    a synthetic ray whose psi(s) oscillates across the same surfaces: with 7
    oscillations each boundary near psi = 0.5 has 15 roots and Dierckx.roots'
    maxn = 8 keeps the first 8 in s order.  dP_dV and P vs scipy's FITPACK
    restatement with mest = 8, 1e-10 of the profile maximum; the uncapped
    profile differs (so the cap is what is checked)."""
    import warnings

    import deposition_ref as D

    s, x, dpds = _oscillating_ray(periods)
    grid = np.linspace(0, 1, 250)
    dP_dV, P = T.power_deposition_profile(hplasma, s, x, dpds, grid)
    psi = np.array([oplasma.evaluate("psi", p) for p in x])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # scipy: "The number of zeros exceeds mest"
        ref, P_ref = D.power_deposition_profile(s, psi, dpds, grid, oplasma.volume, maxn=8)
        _, P_all = D.power_deposition_profile(s, psi, dpds, grid, oplasma.volume, maxn=1000)
    assert np.abs(dP_dV - ref).max() <= 1e-10 * np.abs(ref).max()
    assert abs(P - P_ref) <= 1e-10 * P_ref and dP_dV[-1] == 0.0
    if periods == 7:
        assert abs(P_all - P_ref) > 1e-3 * P_ref


def test_power_deposition_profile_entry_on_rays(gpu, T, hplasma, oplasma, fan_states):
    """The entry point on make_ray's own vectors of traced rays (several rays in
    one call) vs the FITPACK restatement, and the reference's input errors."""
    import deposition_ref as D
    from torj_hip import synthetic as S

    s_ = S.SETUP
    N0 = T.pol_tor_angles_2_vector(s_["steering_angle_pol"], s_["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s_["R0"], 0.0, s_["z0"]], N0, s_["spot_size"],
                                            s_["inverse_curvature_radius"], s_["f_abs_test"],
                                            N_rings=3, min_azimuthal_points=5)
    om = 2 * np.pi * s_["f_abs_test"]
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, 1)
    idx = np.arange(0, len(w), 5)
    grid = np.linspace(0, 1, 400)
    o = oplasma.trace(xp[idx], Np[idx], om, 1, 1e-4, 2000, samples=True, s0=s0[idx], traj_stride=1)
    ss, xs, ds_, refs = [], [], [], []
    for k, i in enumerate(idx):
        m = int(o["steps"][k])
        sv, psi, dpds = D.ray_vectors(pos[i], s0[i], 1e-4, m, o["samples"][k],
                                      oplasma.evaluate("psi", pos[i]))
        xv = np.vstack([pos[i][None], xp[i][None], o["traj"][k, :m, :3]])
        psi_x = np.array([oplasma.evaluate("psi", p) for p in xv])
        ss.append(sv), xs.append(xv), ds_.append(dpds)
        refs.append(D.power_deposition_profile(sv, psi_x, dpds, grid, oplasma.volume))
    dP_dV, P = T.power_deposition_profile(hplasma, ss, xs, ds_, grid)
    for k in range(len(idx)):
        ref, P_ref = refs[k]
        assert np.abs(dP_dV[k] - ref).max() <= 1e-10 * max(np.abs(ref).max(), 1e-300)
        assert abs(P[k] - P_ref) <= 1e-10 * max(P_ref, 1e-300)
    with pytest.raises(T.TorjError, match="need >= 4"):
        T.power_deposition_profile(hplasma, ss[0][:3], xs[0][:3], ds_[0][:3], grid)
    bad = ss[0].copy()
    bad[5] = bad[4]
    with pytest.raises(T.TorjError, match="strictly increasing"):
        T.power_deposition_profile(hplasma, bad, xs[0], ds_[0], grid)
