"""ctypes binding of libtorj_hip.so (include/torj_hip.h).

The library is the product: every compute call below runs HIP kernels on the
GPU.  There is no CPU fallback -- if the library is missing or no GPU is
usable, calls raise TorjError.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)  # torj.jl_amd/
LIB_PATH = os.environ.get("TORJ_HIP_LIB") or os.path.join(_ROOT, "build", "libtorj_hip.so")
CSRC = os.path.join(_ROOT, "csrc")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_u64p = C.POINTER(C.c_uint64)


class TorjError(RuntimeError):
    pass


class TraceCfg(C.Structure):
    """torj_trace_cfg"""
    _fields_ = [("omega", C.c_double), ("mode", C.c_int), ("ds", C.c_double),
                ("n_steps", C.c_int), ("chunk_steps", C.c_int), ("psi_exit", C.c_double),
                ("P_min", C.c_double), ("absorption", C.c_int), ("traj_stride", C.c_int),
                ("deposition", C.c_int), ("integrator", C.c_int), ("abstol", C.c_double),
                ("reltol", C.c_double), ("s_max", C.c_double), ("n_chunks", C.c_int)]

    def __init__(self, omega, mode, ds, n_steps, chunk_steps, psi_exit, P_min, absorption,
                 traj_stride, deposition=0, integrator=0, abstol=1e-6, reltol=1e-6, s_max=0.0,
                 n_chunks=100):
        super().__init__(omega, mode, ds, n_steps, chunk_steps, psi_exit, P_min, absorption,
                         traj_stride, deposition, integrator, abstol, reltol, s_max, n_chunks)


class BeamShard(C.Structure):
    """torj_beam_shard: one device's shard of torj_trace_beam_device (device pointers)"""
    _fields_ = [("n", C.c_int), ("x0", C.c_void_p), ("N0", C.c_void_p), ("weights", C.c_void_p),
                ("psi_grid", C.c_void_p), ("x_launch", C.c_void_p), ("s0", C.c_void_p),
                ("state", C.c_void_p), ("status", C.c_void_p), ("steps", C.c_void_p),
                ("dP_shell", C.c_void_p), ("P_dep", C.c_void_p), ("traj", C.c_void_p),
                ("counters", C.c_void_p)]


_SIGS = {
    "torj_abi_version": (C.c_int, []),
    "torj_build_id": (C.c_char_p, []),
    "torj_last_error": (C.c_char_p, []),
    "torj_device_count": (C.c_int, [_ip]),
    "torj_abs_al_init": (C.c_int, [C.c_int]),
    "torj_plasma_create": (C.c_int, [C.c_int, C.c_int, _dp, _dp, _dp, C.c_int, _dp, _dp, _dp, _dp,
                                     _dp, _dp, C.c_int, _dp, _dp, C.c_int, C.POINTER(C.c_void_p)]),
    "torj_plasma_create_from_coefs": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double,
                                                C.c_double, C.c_double, _dp, _dp, _dp, _dp, _dp,
                                                _dp, C.c_int, C.c_double, C.c_double, _dp,
                                                C.c_double, C.c_int, C.POINTER(C.c_void_p)]),
    "torj_plasma_destroy": (C.c_int, [C.c_void_p]),
    "torj_plasma_get_coefs": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "torj_plasma_psi_prof_max": (C.c_double, [C.c_void_p]),
    "torj_plasma_volume": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp]),
    "torj_eval_plasma": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, C.c_double, _dp]),
    "torj_dispersion": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, C.c_double, C.c_int, _dp, _dp,
                                  _dp]),
    "torj_abs_albajar_fast": (C.c_int, [C.c_int, _dp, _dp, _dp, _dp, _dp, _dp, C.c_int, _dp]),
    "torj_alpha_warm": (C.c_int, [C.c_int] + [_dp] * 7 + [C.c_int, C.c_int, _dp, _dp]),
    "torj_refractive_index_sq": (C.c_int, [C.c_int, _dp, _dp, _dp, C.c_int, _dp]),
    "torj_pol_tor_angles_2_vector": (None, [C.c_double, C.c_double, _dp]),
    "torj_launch_peripheral_rays": (C.c_int, [_dp, _dp, C.c_double, C.c_double, C.c_double,
                                              C.c_int, C.c_int, C.c_int, _ip, _dp, _dp, _dp]),
    "torj_ray_entry": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, C.c_double, C.c_int, _dp, _dp,
                                 _dp, _ip]),
    "torj_ray_entry_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_double,
                                        C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]),
    "torj_ray_entry_gpu": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, C.c_double, C.c_int, _dp,
                                     _dp, _dp, _ip]),
    "torj_trace": (C.c_int, [C.c_void_p, C.POINTER(TraceCfg), C.c_int, _dp, _dp, _dp, C.c_int,
                             _dp, _dp, _ip, _ip, _dp, _dp, _dp]),
    "torj_trace_ex": (C.c_int, [C.c_void_p, C.POINTER(TraceCfg), C.c_int, _dp, _dp, _dp, C.c_int,
                                _dp, _dp, _dp, _dp, _ip, _ip, _dp, _dp, _dp]),
    "torj_trace_beam": (C.c_int, [C.c_void_p, C.POINTER(TraceCfg), C.c_int, _dp, _dp, _dp, C.c_int,
                                  _dp, _dp, _dp, _dp, _ip, _ip, _dp, _dp, _dp, C.c_int, C.c_int]),
    "torj_trace_beam_device": (C.c_int, [C.c_void_p, C.POINTER(TraceCfg), C.c_int, C.c_int,
                                         C.POINTER(BeamShard)]),
    "torj_set_sched": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "torj_trace_check": (C.c_int, [C.c_void_p, C.c_void_p]),
    "torj_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "torj_timing_read": (C.c_int, [C.c_void_p, _ip, _dp, _dp]),
    "torj_beam_timing_read": (C.c_int, [C.c_void_p, C.c_int, _ip, _dp, _dp, _dp]),
    "torj_beam_comm_info": (C.c_int, [C.c_void_p, C.c_int, _ip, _ip, _ip]),
    "torj_trace_device": (C.c_int, [C.c_void_p, C.POINTER(TraceCfg), C.c_int, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p]),
    "torj_trace_device_ex": (C.c_int, [C.c_void_p, C.POINTER(TraceCfg), C.c_int] +
                             [C.c_void_p] * 3 + [C.c_int] + [C.c_void_p] * 11),
    "torj_shell_volumes": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp]),
    "torj_power_deposition_profile": (C.c_int, [C.c_void_p, C.c_int, _ip, _dp, _dp, _dp, C.c_int, _dp,
                                                _dp, _dp]),
}

EXPORTED = tuple(_SIGS)
ABI_VERSION = 8  # include/torj_hip.h TORJ_ABI_VERSION

_lib = None


def build(force: bool = False) -> str:
    """Compile libtorj_hip.so in-tree (hipcc, gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", CSRC])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TorjError(f"libtorj_hip.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        v = L.torj_abi_version()
        if v != ABI_VERSION:
            raise TorjError(f"{LIB_PATH} has ABI version {v}, this mirror expects {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int):
    if rc != 0:
        raise TorjError(lib().torj_last_error().decode())


def dptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


def iptr(a):
    return a.ctypes.data_as(_ip) if a is not None else None


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def soa(v, n=None):
    """(n,3) or (3,) array -> component-major (3, n) contiguous float64."""
    v = np.asarray(v, dtype=np.float64)
    if v.ndim == 1:
        v = v[None, :]
    return np.ascontiguousarray(v.T)
