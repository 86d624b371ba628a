"""GPU parity at the headline workload itself (BASELINE configs[2], SURVEY.md
§8(d) C3): the full 100 203-ray 92/11 fan, X-mode 92.5 GHz, 2 000 RK4 steps of
1e-4 m, Albajar alpha, the reference deposition on a 1 000-point psi grid --
traced with the library's DEFAULT scheduling -- the split RK4 path (DESIGN.md
3.7: cold trajectories, parallel alpha, in-order optical-depth scan, pipelined
over two streams), the regime bench.py times -- and with the work-queue kernel
k_trace_sched at its production wave count (~1 566 groups over ~1 468
persistent waves).

Checks (tolerances as tests/test_gpu_parity.py):
  * every 25th ray (4 009 rays) against the CPU oracle: status and step counts
    exact, x, N, tau <= 1e-10 relative;
  * per-ray deposited power of 24 evenly spaced rays against the FITPACK
    restatement of power_deposition_profile (oracle/deposition_ref.py) <= 1e-11;
  * the whole beam on the one-lane-per-ray kernel (set_sched(0)) vs the work
    queue (bit-identical per ray, dP_shell to the order of its fp64 sums) and
    vs the default split path (1e-12);
  * sum_j w P_dep = dP_shell[n_psi] (make_beam's deposited power).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_RINGS, MIN_AZ, N_STEPS, DS = 92, 11, 2000, 1e-4


@pytest.fixture(scope="module")
def c3(gpu, T, hplasma):
    from torj_hip import synthetic as S

    s = S.SETUP
    f = s["f_abs_test"]
    om = 2 * np.pi * f
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=N_RINGS,
                                            min_azimuthal_points=MIN_AZ)
    assert len(w) == 100203
    xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, 1, gpu=True)
    assert (st == T.OK).all()
    grid = np.linspace(0.0, 1.0, 1000)
    kw = dict(ds=DS, n_steps=N_STEPS, psi_grid=grid, weights=w, traj_stride=100,
              deposition="reference", x_launch=pos, s0=s0)
    hplasma.set_sched(-1)  # the default: work queue with the production wave count
    g = T.trace(hplasma, xp, Np, om, 1, **kw)
    return dict(pos=pos, xp=xp, Np=Np, s0=s0, w=w, om=om, grid=grid, kw=kw, g=g)


def test_c3_fan_sampled_parity(c3, oplasma):
    """Every 25th ray of the headline beam vs the oracle (1e-10, exact statuses)."""
    from test_gpu_parity import _compare_trace

    g, idx = c3["g"], np.arange(0, len(c3["w"]), 25)
    o = oplasma.trace(c3["xp"][idx], c3["Np"][idx], c3["om"], 1, DS, N_STEPS,
                      psi_grid=c3["grid"], weights=c3["w"][idx])
    sub = type(g)(g.state[idx], g.status[idx], g.steps[idx], None, None, None)
    _compare_trace(sub, o)
    # most of the beam is absorbed within the 0.2 m path (X2 layer)
    assert np.median(g.P_end) < 0.1
    assert abs(g.dP_shell[-1] - np.dot(c3["w"], g.P_dep)) <= 1e-12 * g.dP_shell[-1]


def test_c3_fan_reference_deposition_vs_fitpack(c3, oplasma):
    """P_dep of 24 rays of the work-queue run vs FITPACK's power_deposition_profile."""
    import deposition_ref as D

    g = c3["g"]
    idx = np.linspace(0, len(c3["w"]) - 1, 24).astype(int)
    o = oplasma.trace(c3["xp"][idx], c3["Np"][idx], c3["om"], 1, DS, N_STEPS, samples=True,
                      s0=c3["s0"][idx])
    assert np.array_equal(o["steps"], g.steps[idx])
    for k, i in enumerate(idx):
        sv, psi, dpds = D.ray_vectors(c3["pos"][i], c3["s0"][i], DS, o["steps"][k],
                                      o["samples"][k], oplasma.evaluate("psi", c3["pos"][i]))
        _, P = D.power_deposition_profile(sv, psi, dpds, c3["grid"], oplasma.volume)
        # + the tiny-alpha skip's bound: alpha moves by < 1e-20 m^-1 per
        # harmonic, so the ray's deposited power by < 2e-20 per metre traced
        assert abs(g.P_dep[i] - P) <= 1e-11 * P + 2e-20 * DS * o["steps"][k], (i, g.P_dep[i], P)


@pytest.fixture(scope="module")
def c3_exact(c3, T, hplasma):
    """The headline beam again with TORJ_TINY_ALPHA=0 (read at abs_Al_init): every
    harmonic integral with m >= m_0 evaluated, the reference's work."""
    import os

    old = os.environ.get("TORJ_TINY_ALPHA")
    os.environ["TORJ_TINY_ALPHA"] = "0"
    try:
        T.abs_Al_init(24)
        hplasma.set_sched(-1)
        return T.trace(hplasma, c3["xp"], c3["Np"], c3["om"], 1, **c3["kw"])
    finally:
        if old is None:
            del os.environ["TORJ_TINY_ALPHA"]
        else:
            os.environ["TORJ_TINY_ALPHA"] = old
        T.abs_Al_init(24)


def test_c3_fan_exact_leg_vs_fitpack(c3, c3_exact, oplasma):
    """The exact leg keeps the pre-round-5 bars: P_dep of the same 24 rays within
    1e-11 of FITPACK's power_deposition_profile, purely relative (no tiny-alpha
    term); statuses, steps and x, N bit-identical to the default leg (the skip
    touches alpha only); tau of the default leg within its bound of the exact one."""
    import deposition_ref as D

    g, ge = c3["g"], c3_exact
    for f in ("status", "steps"):
        assert np.array_equal(getattr(g, f), getattr(ge, f)), f
    assert np.array_equal(g.state[:, :6], ge.state[:, :6])
    # the default leg's tau moves by < 2 tiny_alpha per metre of ray (1e-20 m^-1)
    assert np.abs(g.state[:, 6] - ge.state[:, 6]).max() <= 2e-20 * DS * N_STEPS * 1.01
    idx = np.linspace(0, len(c3["w"]) - 1, 24).astype(int)
    o = oplasma.trace(c3["xp"][idx], c3["Np"][idx], c3["om"], 1, DS, N_STEPS, samples=True,
                      s0=c3["s0"][idx])
    assert np.array_equal(o["steps"], ge.steps[idx])
    for k, i in enumerate(idx):
        sv, psi, dpds = D.ray_vectors(c3["pos"][i], c3["s0"][i], DS, o["steps"][k],
                                      o["samples"][k], oplasma.evaluate("psi", c3["pos"][i]))
        _, P = D.power_deposition_profile(sv, psi, dpds, c3["grid"], oplasma.volume)
        assert abs(ge.P_dep[i] - P) <= 1e-11 * P, (i, ge.P_dep[i], P)


def test_c3_fan_exact_leg_tau_unfloored(c3, c3_exact, oplasma):
    """Every 25th ray: the exact leg's tau against the oracle with no floor at all
    (relative to tau_cpu wherever tau_cpu > 0); the default leg's unfloored tau on
    the rays with tau_cpu >= 1e-10 (where its rigorous bound, 2e-20 per metre /
    1e-10 = 4e-11 over the 0.2 m path, is inside the 1e-10 bar)."""
    idx = np.arange(0, len(c3["w"]), 25)
    o = oplasma.trace(c3["xp"][idx], c3["Np"][idx], c3["om"], 1, DS, N_STEPS,
                      psi_grid=c3["grid"], weights=c3["w"][idx])
    tc = o["state"][:, 6]
    pos = tc > 0
    e_exact = np.abs(c3_exact.state[idx, 6] - tc)[pos] / tc[pos]
    assert e_exact.max() <= 1e-10, e_exact.max()
    res = tc >= 1e-10
    e_def = np.abs(c3["g"].state[idx, 6] - tc)[res] / tc[res]
    assert e_def.max() <= 1e-10, e_def.max()


def _close(a, b, tol, tau_floor=1e-13):
    """Per-ray outputs equal to rounding: the split path's kernels are compiled
    separately from the fused one, so fma contraction may differ (~1e-15 on x, N;
    tau to tol relative, 1e-14 absolute)."""
    for f in ("status", "steps"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    sa, sb = a.state, b.state
    for cols in (slice(0, 3), slice(3, 6)):
        e = np.abs(sa[:, cols] - sb[:, cols]).max(1) / np.linalg.norm(sa[:, cols], axis=1)
        assert e.max() <= tol, e.max()
    # tau: relative, with an absolute floor of 1e-13 -- rays far from any
    # resonance carry tau ~ 1e-150 built from the tails of exp(-mu (gamma - 1)),
    # whose relative sensitivity to an ulp of position is ~ mu (gamma - 1)
    # (P = 1 - tau is exact there to 1e-16 either way); the split path's
    # trajectory kernel evaluates the fields in per-cell power form (the same
    # interpolant, other roundings: x, N within ~4e-16), which moves tau of a
    # weakly absorbed ray by up to ~3e-14 against the fused kernels' stencil
    # (the node-stencil trajectory modes keep the round-3 floor of 1e-14:
    # tests/test_gpu_split.py test_node_stencil_modes_keep_round3_bars)
    assert (np.abs(sa[:, 6] - sb[:, 6]) - tol * np.abs(sa[:, 6])).max() <= tau_floor
    # the reference deposition locates each shell-boundary root of the psi(s)
    # spline; where a ray grazes a boundary (near-double root) an ulp of
    # trajectory moves the root by ~sqrt(eps), or makes a tangency a root pair
    # or none: P_dep to 1e-9 of the ray's unit power
    assert np.abs(a.P_dep - b.P_dep).max() <= 1e-9
    fin = np.isfinite(a.traj)
    assert np.array_equal(fin, np.isfinite(b.traj))
    assert np.abs(a.dP_shell - b.dP_shell).max() <= tol * np.abs(a.dP_shell).max()


def test_c3_fan_schedules_agree(c3, T, hplasma):
    """The production schedules on the whole beam: the work-queue kernel
    (production wave count) equals the one-lane-per-ray kernel bit for bit; the
    default split path equals it to rounding (1e-12)."""
    try:
        hplasma.set_sched(0)
        a = T.trace(hplasma, c3["xp"], c3["Np"], c3["om"], 1, **c3["kw"])
        hplasma.set_sched(1)
        q = T.trace(hplasma, c3["xp"], c3["Np"], c3["om"], 1, **c3["kw"])
    finally:
        hplasma.set_sched(-1)
    for f in ("state", "status", "steps", "P_dep"):
        assert np.array_equal(getattr(a, f), getattr(q, f)), f
    assert np.array_equal(a.traj, q.traj, equal_nan=True)
    assert np.abs(a.dP_shell - q.dP_shell).max() <= 1e-13 * np.abs(a.dP_shell).max()
    _close(a, c3["g"], 1e-12)
