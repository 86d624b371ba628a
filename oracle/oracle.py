"""ctypes front-end of the CPU parity oracle (oracle/torj_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- as the checker / the timed CPU peer, never as
part of the product path.  Parity status: see torj_oracle.h / DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libtorj_oracle.so")

OK, LEFT_PLASMA, ABSORBED, NAN, REFLECTED, ENTRY_FAIL, MAX_STEPS = range(7)


def default_threads() -> int:
    """OMP_NUM_THREADS if set (16 on the GPU box), else up to 8 host cores."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env if env > 0 else min(os.cpu_count() or 1, 8)


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        L.or_abs_albajar_fast.restype = C.c_double
        L.or_abs_albajar_fast.argtypes = [C.c_double] * 6 + [C.c_int]
        L.or_alpha_approx.restype = C.c_double
        L.or_grad_norm.restype = C.c_double
        L.or_refractive_index_sq.restype = C.c_double
        L.or_refractive_index_sq.argtypes = [C.c_double, C.c_double, C.c_double, C.c_int]
        L.or_dispersion_relation.restype = C.c_double
        L.or_evaluate.restype = C.c_double
        L.or_n_e.restype = C.c_double
        L.or_T_e.restype = C.c_double
        L.or_spl1d_eval.restype = C.c_double
        L.or_spl1d_deriv.restype = C.c_double
        L.or_spl2d_eval.restype = C.c_double
        L.or_spl2d_eval.argtypes = [C.c_void_p, C.c_double, C.c_double]
        L.or_alpha_warm.restype = C.c_double
        L.or_expei.restype = C.c_double
        _lib = L
    return _lib


_ALPHA_FN = C.CFUNCTYPE(C.c_double, *([C.c_double] * 7), C.c_int, C.c_int)
_warm_hook = None


def _install_warm_hook(on):
    """on: or_set_alpha_hook -> warm_ref.alpha_warm (absorption models 2 / 3 through
    the numpy restatement, serial); off: the C restatement or_alpha_warm."""
    global _warm_hook
    if not on:
        lib().or_set_alpha_hook(None)
        return
    if _warm_hook is None:
        import warm_ref

        def fn(omega, X, Y, Nabs, Npar, Te, inv, mode, model):
            return warm_ref.alpha_warm(omega, X, Y, Nabs, Npar, Te, inv, mode,
                                       1 if model == 2 else 3)[0]

        _warm_hook = _ALPHA_FN(fn)
    lib().or_set_alpha_hook(_warm_hook)


def alpha_warm(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode, iwarm=3):
    """or_alpha_warm (oracle/torj_warm_oracle.c): (alpha, N_perp_warm^2 complex)."""
    n2 = np.zeros(2)
    a = lib().or_alpha_warm(C.c_double(omega), C.c_double(X), C.c_double(Y), C.c_double(N_abs),
                            C.c_double(N_par), C.c_double(Te), C.c_double(inv_dDdN),
                            C.c_int(mode), C.c_int(iwarm), _p(n2))
    return a, complex(n2[0], n2[1])


def expei(x):
    return lib().or_expei(C.c_double(x))


def zetac(x, y):
    out = np.zeros(2)
    lib().or_zetac(C.c_double(x), C.c_double(y), _p(out))
    return complex(out[0], out[1])


def _p(a):
    return a.ctypes.data_as(_dp)


def _c(a, dtype=np.float64):
    return np.ascontiguousarray(a, dtype=dtype)


class Spl2D(C.Structure):
    _fields_ = [("nR", C.c_int), ("nZ", C.c_int), ("R1", C.c_double), ("Z1", C.c_double),
                ("hR", C.c_double), ("hZ", C.c_double), ("Rn", C.c_double),
                ("Zn", C.c_double), ("coef", _dp)]

    def coefs(self):
        n = (self.nR + 2) * (self.nZ + 2)
        return np.ctypeslib.as_array(self.coef, shape=(n,)).reshape(self.nZ + 2, self.nR + 2).T.copy()


class Spl1D(C.Structure):
    _fields_ = [("n", C.c_int), ("x1", C.c_double), ("h", C.c_double), ("xn", C.c_double),
                ("coef", _dp)]


class _Plasma(C.Structure):
    _fields_ = [("psi", Spl2D), ("lnne", Spl2D), ("lnTe", Spl2D), ("Br", Spl2D),
                ("Bz", Spl2D), ("Bphi", Spl2D), ("vol", Spl1D), ("psi_prof_max", C.c_double)]


class OraclePlasma:
    """Oracle restatement of `Plasma(...)` (src/plasma.jl:30-58)."""

    def __init__(self, R, Z, psi_norm, psi_prof, ne_prof, Te_prof, Br, Bz, Bphi,
                 eq_psi, eq_vol):
        L = lib()
        R, Z = _c(R), _c(Z)
        nR, nZ = len(R), len(Z)
        # (nR, nZ) matrices, column-major like Julia -> R fastest
        def m(a):
            a = np.asarray(a, dtype=np.float64)
            assert a.shape == (nR, nZ)
            return np.ascontiguousarray(a.T)
        self._keep = [m(psi_norm), _c(psi_prof), _c(ne_prof), _c(Te_prof), m(Br), m(Bz),
                      m(Bphi), _c(eq_psi), _c(eq_vol)]
        k = self._keep
        self.s = _Plasma()
        rc = L.or_plasma_create(C.byref(self.s), nR, nZ, _p(R), _p(Z), _p(k[0]), len(k[1]),
                                _p(k[1]), _p(k[2]), _p(k[3]), _p(k[4]), _p(k[5]), _p(k[6]),
                                len(k[7]), _p(k[7]), _p(k[8]))
        if rc != 0:
            raise ValueError("or_plasma_create failed")
        self.ref = C.byref(self.s)

    def __del__(self):
        try:
            lib().or_plasma_free(self.ref)
        except Exception:
            pass

    @property
    def psi_prof_max(self):
        return self.s.psi_prof_max

    def field_coefs(self):
        """dict of (nR+2, nZ+2) B-spline coefficient arrays."""
        return {k: getattr(self.s, k).coefs() for k in ("psi", "lnne", "lnTe", "Br", "Bz", "Bphi")}

    # ---- field evaluation ----
    def evaluate(self, field, x):
        x = _c(x)
        return lib().or_evaluate(C.byref(getattr(self.s, field)), _p(x))

    def spl2d(self, field, R, Z):
        return lib().or_spl2d_eval(C.addressof(getattr(self.s, field)), R, Z)

    def volume(self, psi):
        return lib().or_spl1d_eval(C.byref(self.s.vol), C.c_double(psi))

    def B_spline(self, x):
        x = _c(x)
        B = np.zeros(3)
        lib().or_B_spline(self.ref, _p(x), _p(B))
        return B

    def n_e(self, x):
        return lib().or_n_e(self.ref, _p(_c(x)))

    def T_e(self, x):
        return lib().or_T_e(self.ref, _p(_c(x)))

    def eval_plasma(self, x, N, omega):
        X, Y, Np = C.c_double(), C.c_double(), C.c_double()
        b = np.zeros(3)
        lib().or_eval_plasma(self.ref, _p(_c(x)), _p(_c(N)), C.c_double(omega), C.byref(X),
                             C.byref(Y), C.byref(Np), _p(b))
        return X.value, Y.value, Np.value, b

    def dispersion_relation(self, x, N, omega, mode):
        return lib().or_dispersion_relation(self.ref, _p(_c(x)), _p(_c(N)), C.c_double(omega),
                                            C.c_int(mode))

    def grad_lambda(self, x, N, omega, mode):
        du = np.zeros(6)
        lib().or_grad_lambda(self.ref, _p(_c(x)), _p(_c(N)), C.c_double(omega), C.c_int(mode),
                             _p(du))
        return du

    def grad_norm(self, x, N, omega, mode):
        """|dD/dN| (src/solve.jl:85-95 normalisation)"""
        return lib().or_grad_norm(self.ref, _p(_c(x)), _p(_c(N)), C.c_double(omega),
                                  C.c_int(mode))

    def alpha_model(self, x, N, omega, mode, model):
        """optical-depth rate of absorption model 0..3 at (x, N), as the trace uses it"""
        if model == 0:
            return 0.0
        if model == 1:
            return self.alpha_approx(x, N, omega, mode)
        X, Y, Npar, _ = self.eval_plasma(x, N, omega)
        return alpha_warm(omega, X, Y, float(np.linalg.norm(N)), Npar, self.T_e(x),
                          1.0 / self.grad_norm(x, N, omega, mode), mode,
                          1 if model == 2 else 3)[0]

    def warm_sensitivity(self, x0, N0, omega, mode, ds, steps, iwarm=1, eta=2.0 ** -45,
                         n_threads=None):
        """or_warm_sensitivity: per ray, sum over its RK4 stage points (first
        steps[r] steps) of ds w_stage max |d alpha| under relative input
        perturbations eta -- how far tau moves when the warm alpha's inputs move
        by a few tens of ulps (the C5 parity bar's a-priori conditioning flag)."""
        x0, N0 = _c(x0).reshape(-1, 3), _c(N0).reshape(-1, 3)
        n = x0.shape[0]
        st = np.ascontiguousarray(steps, dtype=np.int32)
        out = np.zeros(n)
        lib().or_warm_sensitivity(self.ref, C.c_double(omega), C.c_int(mode), C.c_int(iwarm),
                                  C.c_double(ds), n, _p(x0), _p(N0), st.ctypes.data_as(_ip),
                                  C.c_double(eta), _p(out), n_threads or default_threads())
        return out

    def albajar_sensitivity(self, x0, N0, omega, mode, ds, steps, eta=2.0 ** -45, n_threads=None):
        """or_albajar_sensitivity: warm_sensitivity's a-priori flag for the Albajar
        model -- per ray, the sum over its RK4 stage points of ds w_stage max |d alpha|
        under relative perturbations eta of Y, and of (X, N_par, Te) jointly."""
        x0, N0 = _c(x0).reshape(-1, 3), _c(N0).reshape(-1, 3)
        n = x0.shape[0]
        st = np.ascontiguousarray(steps, dtype=np.int32)
        out = np.zeros(n)
        lib().or_albajar_sensitivity(self.ref, C.c_double(omega), C.c_int(mode), C.c_double(ds), n,
                                     _p(x0), _p(N0), st.ctypes.data_as(_ip), C.c_double(eta),
                                     _p(out), n_threads or default_threads())
        return out

    def alpha_approx(self, x, N, omega, mode):
        return lib().or_alpha_approx(self.ref, _p(_c(x)), _p(_c(N)), C.c_double(omega),
                                     C.c_int(mode))

    def ray_entry(self, x0, N0, omega, mode):
        xp, Np = np.zeros(3), np.zeros(3)
        s0 = C.c_double()
        st = lib().or_ray_entry(self.ref, _p(_c(x0)), _p(_c(N0)), C.c_double(omega),
                                C.c_int(mode), _p(xp), _p(Np), C.byref(s0))
        return st, xp, Np, s0.value

    def trace(self, x0, N0, omega, mode, ds, n_steps, chunk_steps=None, psi_exit=1.0,
              P_min=1e-6, absorption=True, psi_grid=None, weights=None, traj_stride=0,
              n_threads=None, samples=False, integrator=0, abstol=1e-6, reltol=1e-6, s_max=None,
              n_chunks=100, s0=None, warm="c"):
        """Fixed-step RK4 trace of rays (x0, N0: (n, 3) entry states).  samples=True
        adds "samples": (n, n_steps+1, 3) = (psi_k, dP/ds_k, s_k) at the entry point and
        every step (make_ray's psi / dP_ds vectors, src/solve.jl:151,171).
        integrator=1: the reference's adaptive solve() (Tsit5, DiffEq step control,
        n_chunks tspans over s_max from s0); n_steps is then the step capacity."""
        x0, N0 = _c(x0).reshape(-1, 3), _c(N0).reshape(-1, 3)
        n = x0.shape[0]
        if chunk_steps is None:
            chunk_steps = max(1, n_steps // 100)
        grid = _c(psi_grid) if psi_grid is not None else np.zeros(0)
        n_psi = len(grid)
        s0a = _c(s0) if s0 is not None else None
        cfg = _TraceCfg(omega, mode, ds, n_steps, chunk_steps, psi_exit, P_min, int(absorption),
                        n_psi, _p(grid) if n_psi else None, traj_stride, int(integrator), abstol,
                        reltol, float(s_max if s_max is not None else n_steps * ds), n_chunks,
                        _p(s0a) if s0a is not None else None)
        state = np.zeros((n, 7))
        status = np.zeros(n, dtype=np.int32)
        steps = np.zeros(n, dtype=np.int32)
        dP = np.zeros(max(n_psi, 1))
        Pdep = np.zeros(n)
        n_save = n_steps // traj_stride if traj_stride > 0 else 0
        traj = np.full((n, max(n_save, 1), 5), np.nan)
        w = _c(weights) if weights is not None else None
        nt = n_threads or default_threads()
        if int(absorption) >= 2:
            # warm alpha: the C restatement, multi-threaded; warm="numpy" routes it
            # through warm_ref.py by a callback instead (serial)
            _install_warm_hook(warm == "numpy")
            if warm == "numpy":
                nt = 1
        smp = np.zeros((n, n_steps + 1, 3)) if samples else None
        lib().or_trace_samples(self.ref, C.byref(cfg), n, _p(x0), _p(N0),
                               _p(w) if w is not None else None, _p(state),
                               status.ctypes.data_as(_ip), steps.ctypes.data_as(_ip), _p(dP),
                               _p(Pdep), _p(traj), _p(smp) if samples else None, nt)
        out = dict(state=state, status=status, steps=steps, dP=dP[:n_psi], Pdep=Pdep,
                   traj=traj[:, :n_save])
        if samples:
            out["samples"] = smp
        return out


class _TraceCfg(C.Structure):
    _fields_ = [("omega", C.c_double), ("mode", C.c_int), ("ds", C.c_double),
                ("n_steps", C.c_int), ("chunk_steps", C.c_int), ("psi_exit", C.c_double),
                ("P_min", C.c_double), ("absorption", C.c_int), ("n_psi", C.c_int),
                ("psi_grid", _dp), ("traj_stride", C.c_int), ("integrator", C.c_int),
                ("abstol", C.c_double), ("reltol", C.c_double), ("s_max", C.c_double),
                ("n_chunks", C.c_int), ("s0", _dp)]


# ---- free functions ----
def gauss_legendre(n):
    x, w = np.zeros(n), np.zeros(n)
    lib().or_gauss_legendre(n, _p(x), _p(w))
    return x, w


def gauss_hermite(n):
    x, w = np.zeros(n), np.zeros(n)
    lib().or_gauss_hermite(n, _p(x), _p(w))
    return x, w


def bspl1d_prefilter(y):
    y = _c(y)
    c = np.zeros(len(y) + 2)
    lib().or_bspl1d_prefilter(len(y), _p(y), _p(c))
    return c


def bspl2d_prefilter(y):
    """y: (nR, nZ) -> coefs (nR+2, nZ+2)"""
    y = np.asarray(y, dtype=np.float64)
    nR, nZ = y.shape
    yf = np.ascontiguousarray(y.T)
    c = np.zeros((nZ + 2) * (nR + 2))
    lib().or_bspl2d_prefilter(nR, nZ, _p(yf), _p(c))
    return c.reshape(nZ + 2, nR + 2).T.copy()


def natcubic(x, y, xq):
    x, y, xq = _c(x), _c(y), _c(xq)
    yq = np.zeros(len(xq))
    lib().or_natcubic(len(x), _p(x), _p(y), len(xq), _p(xq), _p(yq))
    return yq


def abs_al_init(n):
    if lib().or_abs_al_init(n) != 0:
        raise ValueError("bad GL order")


def abs_albajar_fast(omega, X, Y, N_abs, N_par, Te, mode):
    return lib().or_abs_albajar_fast(omega, X, Y, N_abs, N_par, Te, mode)


def refractive_index_sq(X, Y, Npar, mode):
    return lib().or_refractive_index_sq(X, Y, Npar, mode)


def pol_tor_angles_2_vector(pol, tor):
    N = np.zeros(3)
    lib().or_pol_tor_angles_2_vector(C.c_double(pol), C.c_double(tor), _p(N))
    return N


def launch_peripheral_rays(x0, N0, w, inv_curv, f, N_rings=3, min_azimuthal_points=5,
                           normalize_weight_sum=True):
    L = lib()
    n = L.or_launch_count(N_rings, min_azimuthal_points)
    if n < 0:
        raise ValueError(f"N_rings = {N_rings} < 2 which is the minimum")
    pos, dirs, wts = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros(n)
    L.or_launch_peripheral_rays(_p(_c(x0)), _p(_c(N0)), C.c_double(w), C.c_double(inv_curv),
                                C.c_double(f), N_rings, min_azimuthal_points,
                                int(normalize_weight_sum), _p(pos), _p(dirs), _p(wts))
    return pos, dirs, wts
