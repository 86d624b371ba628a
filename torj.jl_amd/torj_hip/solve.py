"""make_ray / make_beam (src/solve.jl) on top of the HIP ray-stepping kernel.

Integration semantics (DESIGN.md "Integrator"): fixed-step RK4 with
ds = 1e-4 m (the reference's dtmax, src/solve.jl:157), optical depth tau with
P = exp(-tau), termination checks (psi > 1, P < 1e-6) at the boundaries of the
reference's 100 chunks (src/solve.jl:145,174,176), and psi-shell deposition
binned in-kernel.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._lib import TraceCfg, TorjError, check, dptr, f64, iptr, lib, soa
from .launch import launch_peripheral_rays, pol_tor_angles_2_vector

OK, LEFT_PLASMA, ABSORBED, NAN, REFLECTED, ENTRY_FAIL, MAX_STEPS = range(7)
STATUS_NAMES = ("OK", "LEFT_PLASMA", "ABSORBED", "NAN", "REFLECTED", "ENTRY_FAIL", "MAX_STEPS")


class RayEntryError(AssertionError):
    """The reference's @assert failures in first_point/make_ray (src/solve.jl:32,138,141)
    and its unhandled reflection return (src/solve.jl:57-59)."""


def ray_entry(plasma, x0, N0, omega: float, mode: int, *, gpu: bool = False):
    """first_point + vacuum_plasma_refraction for a batch (src/solve.jl:7-74).
    Returns (x_plasma (n,3), N_plasma (n,3), s0 (n,), status (n,)).  gpu=True
    runs the one-lane-per-ray HIP kernel (torj_ray_entry_gpu); the default is
    the host C++ path (OpenMP), usable without a GPU."""
    xs, Ns = soa(x0), soa(N0)
    n = xs.shape[1]
    xp, Np = np.zeros((3, n)), np.zeros((3, n))
    s0 = np.zeros(n)
    st = np.zeros(n, dtype=np.int32)
    fn = lib().torj_ray_entry_gpu if gpu else lib().torj_ray_entry
    check(fn(plasma.handle, n, dptr(xs), dptr(Ns), float(omega), int(mode), dptr(xp), dptr(Np),
             dptr(s0), iptr(st)))
    return xp.T.copy(), Np.T.copy(), s0, st


@dataclass
class TraceResult:
    state: np.ndarray     # (n, 7): x, y, z, Nx, Ny, Nz, tau
    status: np.ndarray    # (n,)
    steps: np.ndarray     # (n,)
    dP_shell: np.ndarray  # (n_psi + 1,): sum_rays w * dP per shell, [n_psi] = sum w * P_dep
    P_dep: np.ndarray     # (n,)
    traj: np.ndarray | None  # (n, n_save, 5): x, y, z, tau, s

    @property
    def P_end(self):
        return np.exp(-self.state[:, 6])


DEPOSITION = {"binned": 0, "reference": 1}
INTEGRATOR = {"rk4": 0, "adaptive": 1}
ABSORPTION = {"none": 0, "albajar": 1, "warm_wr": 2, "warm_fr": 3}


def _absorption_code(absorption) -> int:
    """bool (True = Albajar, the reference's abs_Albajar_fast), a name from
    ABSORPTION, or the ABI integer 0..3."""
    if isinstance(absorption, str):
        return ABSORPTION[absorption]
    if isinstance(absorption, (bool, np.bool_)):
        return int(bool(absorption))
    a = int(absorption)
    if a not in (0, 1, 2, 3):
        raise ValueError(f"absorption must be 0..3, got {a}")
    return a


def trace(plasma, x0, N0, omega: float, mode: int, *, ds: float = 1e-4, n_steps: int,
          chunk_steps: int | None = None, psi_exit: float = 1.0, P_min: float = 1e-6,
          absorption=True, psi_grid=None, weights=None, traj_stride: int = 0,
          deposition: str = "binned", x_launch=None, s0=None, integrator: str = "rk4",
          abstol: float = 1e-6, reltol: float = 1e-6, s_max: float | None = None,
          n_chunks: int = 100, n_gpus: int | None = None, n_shards: int = 0) -> TraceResult:
    """Integrate rays from in-plasma start states (x0, N0: (n, 3)) on the GPU.

    deposition="binned": psi-shell binning of every step (P_dep = 1 - P_end per
    ray); "reference": power_deposition_profile's FITPACK semantics
    (src/plasma.jl:91-151) from make_ray's saved points, which needs the
    vacuum launch points x_launch (n, 3) and path lengths s0 (n,).

    integrator="rk4": n_steps fixed steps of ds; "adaptive": the reference's
    solve() -- Tsit5 with DiffEq's step control (abstol, reltol, dtmax = ds) over
    n_chunks tspans covering s_max from s0; n_steps is then the accepted-step
    capacity per ray (status MAX_STEPS when exceeded).

    n_gpus: None traces on the plasma's device (torj_trace_ex); an integer runs
    make_beam's multi-GPU path (torj_trace_beam): n_shards contiguous shards
    (0: one per GPU) over n_gpus devices, dP_shell summed by an RCCL all-reduce."""
    xs, Ns = soa(x0), soa(N0)
    n = xs.shape[1]
    if chunk_steps is None:
        chunk_steps = max(1, n_steps // 100)
    dmode = DEPOSITION[deposition]
    imode = INTEGRATOR[integrator]
    cfg = TraceCfg(float(omega), int(mode), float(ds), int(n_steps), int(chunk_steps),
                   float(psi_exit), float(P_min), _absorption_code(absorption), int(traj_stride), dmode,
                   imode, float(abstol), float(reltol),
                   float(s_max if s_max is not None else n_steps * ds), int(n_chunks))
    xl = soa(x_launch) if x_launch is not None else None
    sv = f64(s0) if s0 is not None else None
    g = f64(psi_grid) if psi_grid is not None else np.zeros(0)
    n_psi = len(g)
    w = f64(weights) if weights is not None else None
    state = np.zeros((7, n))
    status = np.zeros(n, dtype=np.int32)
    steps = np.zeros(n, dtype=np.int32)
    dP = np.zeros(n_psi + 1)
    Pdep = np.zeros(n)
    n_save = n_steps // traj_stride if traj_stride > 0 else 0
    traj = np.zeros((n_save, 5, n)) if n_save > 0 else None
    args = (plasma.handle, cfg, n, dptr(xs), dptr(Ns), dptr(w), n_psi, dptr(g) if n_psi else None,
            dptr(xl), dptr(sv), dptr(state), iptr(status), iptr(steps), dptr(dP), dptr(Pdep),
            dptr(traj))
    if n_gpus is None:
        check(lib().torj_trace_ex(*args))
    else:
        check(lib().torj_trace_beam(*args, int(n_gpus), int(n_shards)))
    return TraceResult(state.T.copy(), status, steps, dP, Pdep,
                       traj.transpose(2, 0, 1).copy() if traj is not None else None)


def _steps_for(s_max: float, ds: float) -> int:
    return max(1, int(round(s_max / ds)))


def make_ray(plasma, x0, N_vacuum, f: float, mode: int, s_max: float, psi_dP_dV, *,
             ds: float = 1e-4, deposition: str = "reference", integrator: str = "rk4",
             max_steps: int | None = None, absorption="albajar"):
    """make_ray (src/solve.jl:135-181) -> (s, u, P_beam, dP_dV_ray, deposited_power).
    deposition="reference" (default) follows power_deposition_profile; "binned"
    uses the in-kernel shell binning.  integrator="adaptive" runs the reference's
    solve() semantics (Tsit5, dtmax = ds, 100 chunks); "rk4" fixed steps of ds.
    absorption: "albajar" (alpha_approx, the reference's), "warm_wr" / "warm_fr"
    (general_absorption.jl's alpha, iwarm 1 / 3) or "none"."""
    omega = 2.0 * np.pi * f
    x0 = f64(x0)
    xp, Np, s0, st = ray_entry(plasma, x0[None], f64(N_vacuum)[None], omega, mode)
    if st[0] != OK:
        raise RayEntryError(f"ray entry failed: {STATUS_NAMES[st[0]]}")
    n_steps = _steps_for(s_max, ds)
    if integrator == "adaptive":
        n_steps = max_steps or 2 * n_steps + 400
    g = f64(psi_dP_dV)
    r = trace(plasma, xp, Np, omega, mode, ds=ds, n_steps=n_steps, psi_grid=g, traj_stride=1,
              deposition=deposition, x_launch=x0[None], s0=s0, integrator=integrator, s_max=s_max,
              absorption=absorption)
    if r.status[0] == MAX_STEPS:
        raise RuntimeError("make_ray: accepted-step capacity exhausted (raise max_steps)")
    k = int(r.steps[0])
    s = np.concatenate([[0.0, s0[0]], r.traj[0, :k, 4]])
    u = np.vstack([x0[None], xp, r.traj[0, :k, :3]])
    P_beam = np.concatenate([[1.0, 1.0], np.exp(-r.traj[0, :k, 3])])
    dV = plasma.shell_volumes(g)
    dP_dV = np.zeros(len(g))
    dP_dV[:-1] = r.dP_shell[:len(g) - 1] / dV
    return s, u, P_beam, dP_dV, float(r.P_dep[0])


def fma(a: float, b: float, c: float) -> float:
    """a * b + c with ONE rounding (Python 3.10 has no math.fma): the exact
    rational value, rounded once by the correctly rounded Fraction -> float."""
    from fractions import Fraction

    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _final_arc_length(res, i, s0, ds):
    """Arc length of ray i's final RK4 state: fma(steps, ds, s0), the single-
    rounding product-sum the trajectory kernel stores (its s0 + steps * ds is
    contracted to one v_fma_f64)."""
    return fma(float(int(res.steps[i])), float(ds), float(s0))


def make_beam(plasma, r: float, phi: float, z: float, steering_angle_tor: float,
              steering_angle_pol: float, spot_size: float, inverse_curvature_radius: float,
              f: float, mode: int, s_max: float, psi_dP_dV, *, ds: float = 1e-4,
              traj_stride: int = 1, deposition: str = "reference", integrator: str = "rk4",
              max_steps: int | None = None, absorption="albajar", n_gpus: int = 1, **kwargs):
    """make_beam (src/solve.jl:209-242) -> (arc_lengths, trajectories, ray_powers, dP_dV,
    deposited_power, ray_weights).  kwargs go to launch_peripheral_rays.  The rays
    are traced by torj_trace_beam over n_gpus devices of this process (the
    reference's per-ray Dagger tasks, src/solve.jl:219-224) and their deposition
    summed across them (:233-240).  traj_stride > 1 keeps every traj_stride-th
    step of each ray plus its final state, so ray_powers[i][-1] is the ray's
    final P as in the reference."""
    if integrator == "adaptive" and traj_stride > 1:
        # checked before any tracing: the adaptive integrator's final state is
        # not a saved sample and its arc length is not recorded
        raise ValueError("make_beam: integrator='adaptive' needs traj_stride = 1")
    omega = 2.0 * np.pi * f
    N0 = pol_tor_angles_2_vector(steering_angle_pol, steering_angle_tor)
    x0 = np.array([r * np.cos(phi), r * np.sin(phi), z])
    pos, dirs, w = launch_peripheral_rays(x0, N0, spot_size, inverse_curvature_radius, f, **kwargs)
    xp, Np, s0, st = ray_entry(plasma, pos, dirs, omega, mode, gpu=True)
    bad = np.flatnonzero(st != OK)
    if len(bad):
        raise RayEntryError(f"{len(bad)} rays failed entry, first: ray {bad[0]} "
                            f"{STATUS_NAMES[st[bad[0]]]}")
    n_steps = _steps_for(s_max, ds)
    if integrator == "adaptive":
        n_steps = max_steps or 2 * n_steps + 400
    g = f64(psi_dP_dV)
    res = trace(plasma, xp, Np, omega, mode, ds=ds, n_steps=n_steps, psi_grid=g, weights=w,
                traj_stride=traj_stride, deposition=deposition, x_launch=pos, s0=s0,
                integrator=integrator, s_max=s_max, absorption=absorption, n_gpus=n_gpus)
    if (res.status == MAX_STEPS).any():
        raise RuntimeError("make_beam: accepted-step capacity exhausted (raise max_steps)")
    dV = plasma.shell_volumes(g)
    dP_dV = np.zeros(len(g))
    dP_dV[:-1] = res.dP_shell[:len(g) - 1] / dV
    deposited_power = float(res.dP_shell[len(g)])
    arc_lengths, trajectories, ray_powers = [], [], []
    for i in range(len(w)):
        k = int(res.steps[i]) // traj_stride
        s_i, x_i, tau_i = res.traj[i, :k, 4], res.traj[i, :k, :3], res.traj[i, :k, 3]
        if int(res.steps[i]) % traj_stride:  # the final state is not a saved sample
            s_end = _final_arc_length(res, i, s0[i], ds)
            s_i = np.concatenate([s_i, [s_end]])
            x_i = np.vstack([x_i, res.state[i, :3][None]])
            tau_i = np.concatenate([tau_i, [res.state[i, 6]]])
        arc_lengths.append(np.concatenate([[0.0, s0[i]], s_i]))
        trajectories.append(np.vstack([pos[i][None], xp[i][None], x_i]))
        ray_powers.append(np.concatenate([[1.0, 1.0], np.exp(-tau_i)]))
    return arc_lengths, trajectories, ray_powers, dP_dV, deposited_power, w
