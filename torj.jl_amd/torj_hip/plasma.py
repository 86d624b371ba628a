"""`Plasma` and its field evaluations (src/plasma.jl) on the GPU.

Point functions accept one point (shape (3,)) like the reference or a batch
(shape (n, 3)); batches run as one kernel launch.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, f64, lib, soa

FIELDS = ("psi", "lnne", "lnTe", "Br", "Bz", "Bphi")


class Plasma:
    """Plasma(R_coords, Z_coords, psi_norm_data, psi_prof, ne_prof, Te_prof, Br_data,
    Bz_data, Bϕ_data, eqt1d_psi_norm, eqt1d_volume)  (src/plasma.jl:30-58).

    2-D maps are (nR, nZ) arrays like the reference's Julia matrices.  The
    cubic B-spline coefficients (Interpolations.jl Cubic(Line(OnGrid()))) are
    built by libtorj_hip and live in HBM on `device`.
    """

    def __init__(self, R_coords, Z_coords, psi_norm_data, psi_prof, ne_prof, Te_prof, Br_data,
                 Bz_data, Bphi_data, eqt1d_psi_norm, eqt1d_volume, device: int = 0):
        R, Z = f64(R_coords), f64(Z_coords)
        nR, nZ = len(R), len(Z)

        def m(a):
            a = np.asarray(a, dtype=np.float64)
            if a.shape != (nR, nZ):
                raise ValueError(f"2-D map has shape {a.shape}, expected {(nR, nZ)}")
            return np.ascontiguousarray(a.T)  # column-major (R fastest)

        keep = [m(psi_norm_data), f64(psi_prof), f64(ne_prof), f64(Te_prof), m(Br_data),
                m(Bz_data), m(Bphi_data), f64(eqt1d_psi_norm), f64(eqt1d_volume)]
        h = C.c_void_p()
        check(lib().torj_plasma_create(nR, nZ, dptr(R), dptr(Z), dptr(keep[0]), len(keep[1]),
                                       dptr(keep[1]), dptr(keep[2]), dptr(keep[3]), dptr(keep[4]),
                                       dptr(keep[5]), dptr(keep[6]), len(keep[7]), dptr(keep[7]),
                                       dptr(keep[8]), device, C.byref(h)))
        self._h = h
        self.device = device
        self.R_coords, self.Z_coords = R, Z
        self.psi_prof_max = lib().torj_plasma_psi_prof_max(h)

    @classmethod
    def from_coefs(cls, R_range, Z_range, coefs: dict, vol_psi_range, vol_coefs, psi_prof_max,
                   device: int = 0):
        """Build from Interpolations.jl coefficient arrays ((nR+2, nZ+2) each)."""
        self = cls.__new__(cls)
        c = {k: np.ascontiguousarray(np.asarray(coefs[k], dtype=np.float64).T) for k in FIELDS}
        nR, nZ = c["psi"].shape[1] - 2, c["psi"].shape[0] - 2
        vc = f64(vol_coefs)
        h = C.c_void_p()
        check(lib().torj_plasma_create_from_coefs(
            nR, nZ, R_range[0], R_range[1], Z_range[0], Z_range[1], *[dptr(c[k]) for k in FIELDS],
            len(vc) - 2, vol_psi_range[0], vol_psi_range[1], dptr(vc), psi_prof_max, device,
            C.byref(h)))
        self._h = h
        self.device = device
        self.R_coords = np.linspace(R_range[0], R_range[1], nR)
        self.Z_coords = np.linspace(Z_range[0], Z_range[1], nZ)
        self.psi_prof_max = psi_prof_max
        return self

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().torj_plasma_destroy(h)
            except Exception:
                pass
            self._h = None

    def coefs(self, field: str) -> np.ndarray:
        """B-spline coefficients of `field` as an (nR+2, nZ+2) array."""
        nR, nZ = len(self.R_coords), len(self.Z_coords)
        out = np.zeros((nZ + 2) * (nR + 2))
        check(lib().torj_plasma_get_coefs(self._h, FIELDS.index(field), dptr(out)))
        return out.reshape(nZ + 2, nR + 2).T.copy()

    def volume(self, psi):
        """plasma.volume_psi_spline(psi)"""
        p = np.atleast_1d(f64(psi))
        out = np.zeros_like(p)
        check(lib().torj_plasma_volume(self._h, len(p), dptr(p), dptr(out)))
        return out if np.ndim(psi) else float(out[0])

    def set_sched(self, mode: int = -1, waves: int = 0):
        """torj_set_sched: -1 default, 0 one lane per ray, 1 ready-queue waves,
        2 sixteen lanes per ray (small beams; equal to rounding)."""
        check(lib().torj_set_sched(self._h, int(mode), int(waves)))

    def shell_volumes(self, psi_grid):
        g = f64(psi_grid)
        dV = np.zeros(max(len(g) - 1, 0))
        check(lib().torj_shell_volumes(self._h, len(g), dptr(g), dptr(dV)))
        return dV

    # ---- batched GPU evaluation ----
    def eval_points(self, x, N=None, omega: float = 1.0) -> np.ndarray:
        """torj_eval_plasma: (13, n) table (see include/torj_hip.h)."""
        xs = soa(x)
        n = xs.shape[1]
        Ns = soa(N) if N is not None else np.zeros_like(xs)
        out = np.zeros((13, n))
        check(lib().torj_eval_plasma(self._h, n, dptr(xs), dptr(Ns), omega, dptr(out)))
        return out


def _single(x):
    return np.asarray(x).ndim == 1


def evaluate(plasma: Plasma, field: str, x):
    """evaluate(spline, x) for the psi spline (src/plasma.jl:61-65)."""
    if field not in ("psi", "psi_norm_spline"):
        raise ValueError("only the psi_norm spline is exposed point-wise; use n_e/T_e/B_spline")
    out = plasma.eval_points(x)[5]
    return float(out[0]) if _single(x) else out


def B_spline(plasma: Plasma, x):
    """B_spline(plasma, x) -> (Bx, By, Bz) (src/plasma.jl:73-81)."""
    out = plasma.eval_points(x)[0:3].T
    return out[0] if _single(x) else out


def n_e(plasma: Plasma, x):
    out = plasma.eval_points(x)[3]
    return float(out[0]) if _single(x) else out


def T_e(plasma: Plasma, x):
    out = plasma.eval_points(x)[4]
    return float(out[0]) if _single(x) else out


def eval_plasma(plasma: Plasma, x, N, omega: float):
    """eval_plasma(plasma, x, N, omega) -> (X, Y, N_par, b) (src/dispersion.jl:7-15)."""
    o = plasma.eval_points(x, N, omega)
    if _single(x):
        return float(o[6, 0]), float(o[7, 0]), float(o[8, 0]), o[9:12, 0].copy()
    return o[6], o[7], o[8], o[9:12].T.copy()


def power_deposition_profile(plasma, s, x, dP_ds, psi_dP_dV):
    """power_deposition_profile(plasma, s, x, dP_ds, psi_dP_dV) (src/plasma.jl:91-151)
    -> (dP_dV, P), on the GPU (torj_power_deposition_profile).  One ray: s (n,),
    x (n, 3) or a list of 3-vectors, dP_ds (n,).  Several rays: lists of such
    arrays -> (dP_dV (n_rays, n_psi), P (n_rays,))."""
    batched = isinstance(s, (list, tuple)) and len(s) > 0 and np.ndim(s[0]) == 1
    ss = [f64(v) for v in s] if batched else [f64(s)]
    xs = [np.asarray(v, dtype=np.float64).reshape(-1, 3) for v in x] if batched else \
        [np.asarray(x, dtype=np.float64).reshape(-1, 3)]
    ds = [f64(v) for v in dP_ds] if batched else [f64(dP_ds)]
    npts = np.array([len(v) for v in ss], dtype=np.int32)
    for a, b, c in zip(ss, xs, ds):
        if not (len(a) == len(b) == len(c)):
            raise ValueError("s, x and dP_ds must have one entry per point")
    s_all = np.ascontiguousarray(np.concatenate(ss))
    x_all = soa(np.concatenate(xs))
    d_all = np.ascontiguousarray(np.concatenate(ds))
    g = f64(psi_dP_dV)
    out = np.zeros((len(ss), len(g)))
    P = np.zeros(len(ss))
    check(lib().torj_power_deposition_profile(plasma.handle, len(ss), npts.ctypes.data_as(C.POINTER(C.c_int)),
                                              dptr(s_all), dptr(x_all), dptr(d_all), len(g), dptr(g),
                                              dptr(out), dptr(P)))
    return (out, P) if batched else (out[0], float(P[0]))
