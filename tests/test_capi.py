"""C-ABI boundary (include/torj_hip.h): the library loads, exports every declared
symbol, and its host-side parts (Plasma construction, launch fan, ray entry,
shell volumes) agree with the oracle.  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, rel_err


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "torj_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(torj_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(T):
    lib = ctypes.CDLL(T.LIB_PATH)
    syms = _declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python mirror binds exactly these
    assert set(T.EXPORTED) == set(syms)


def test_abi_version_and_errors(T):
    assert T.lib().torj_abi_version() == T._lib.ABI_VERSION == 8
    bid = T.lib().torj_build_id().decode()
    assert re.fullmatch(r"[0-9a-f]{16}", bid), bid
    with pytest.raises(ValueError, match="N_rings"):
        T.launch_peripheral_rays([0, 0, 0], [0, 0, 1.0], 0.0174, 1 / 3.99, 92.5e9, N_rings=1)
    with pytest.raises(T.TorjError, match="abs_Al_init"):
        T.abs_Al_init(0)


def test_tiny_alpha_threshold_checked(T):
    """TORJ_TINY_ALPHA (the bounded tiny-alpha skip) is read at
    abs_Al_init: 0 and values below 1e-12 m^-1 are accepted, others refused with
    the library's error (the skip's bound is only argued for thresholds far below
    the parity bar's absolute floor)."""
    old = os.environ.get("TORJ_TINY_ALPHA")
    try:
        for ok in ("0", "1e-20", "1e-15"):
            os.environ["TORJ_TINY_ALPHA"] = ok
            T.abs_Al_init(24)
        for bad in ("1e-3", "-1e-20", "nan"):
            os.environ["TORJ_TINY_ALPHA"] = bad
            with pytest.raises(T.TorjError, match="TORJ_TINY_ALPHA"):
                T.abs_Al_init(24)
    finally:
        if old is None:
            os.environ.pop("TORJ_TINY_ALPHA", None)
        else:
            os.environ["TORJ_TINY_ALPHA"] = old
        T.abs_Al_init(24)


def test_plasma_coefficients_match_oracle(hplasma, oplasma):
    oc = oplasma.field_coefs()
    for k in ("psi", "lnne", "lnTe", "Br", "Bz", "Bphi"):
        a, b = hplasma.coefs(k), oc[k]
        assert a.shape == b.shape
        assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max(), k
    assert hplasma.psi_prof_max == oplasma.psi_prof_max
    for p in (0.0, 0.3, 0.77, 1.0, 1.2):
        assert abs(hplasma.volume(p) - oplasma.volume(p)) < 1e-12


def test_plasma_from_coefs_roundtrip(T, hplasma, eq):
    c = {k: hplasma.coefs(k) for k in ("psi", "lnne", "lnTe", "Br", "Bz", "Bphi")}
    P2 = T.Plasma.from_coefs((eq["R_coords"][0], eq["R_coords"][-1]),
                             (eq["Z_coords"][0], eq["Z_coords"][-1]), c, (0.0, 1.0),
                             np.zeros(len(eq["eqt1d_psi_norm"]) + 2), hplasma.psi_prof_max)
    for k in c:
        assert np.array_equal(P2.coefs(k), c[k])


def test_plasma_from_interpolations_layout_coefs(T, hplasma, oplasma, eq):
    """The Julia shim's GPUPlasma(::TorJ.Plasma) path: a handle built from
    Interpolations.jl-layout coefficient arrays ((nR+2, nZ+2), column-major,
    parent(spl.itp.itp.coefs)) -- here the oracle's own prefilter output (dense
    LU, independent of the product's Thomas solve) and its volume spline -- gives
    the ray entry (host path: bisection on psi + refraction) of the handle built
    from the raw maps."""
    oc = oplasma.field_coefs()
    v = oplasma.s.vol
    vol = np.ctypeslib.as_array(v.coef, shape=(v.n + 2,)).copy()
    P2 = T.Plasma.from_coefs((eq["R_coords"][0], eq["R_coords"][-1]),
                             (eq["Z_coords"][0], eq["Z_coords"][-1]), oc, (v.x1, v.xn), vol,
                             oplasma.psi_prof_max)
    for p in (0.0, 0.3, 0.77, 1.0):
        assert abs(P2.volume(p) - hplasma.volume(p)) < 1e-12
    om = 2 * np.pi * 92.5e9
    N0 = T.pol_tor_angles_2_vector(np.deg2rad(30), 0.0)
    pos, dirs, w = T.launch_peripheral_rays([2.5, 0, 0.4], N0, 0.0174, 1 / 3.99, 92.5e9,
                                            N_rings=4, min_azimuthal_points=5)
    a = T.ray_entry(hplasma, pos, dirs, om, 1)
    b = T.ray_entry(P2, pos, dirs, om, 1)
    assert np.array_equal(a[3], b[3]) and (a[3] == 0).all()
    for u, q in zip(a[:3], b[:3]):
        assert np.abs(u - q).max() < 1e-11


def test_launch_fan_matches_oracle(T, O):
    for kw in ({}, {"N_rings": 14, "min_azimuthal_points": 5},
               {"N_rings": 21, "min_azimuthal_points": 11, "normalize_weight_sum": False},
               {"N_rings": 150, "min_azimuthal_points": 11}):
        for inv in (1 / 3.99, -1 / 2.0, float("inf")):
            N0 = T.pol_tor_angles_2_vector(np.deg2rad(30), np.deg2rad(5))
            a = T.launch_peripheral_rays([2.5, 0.1, 0.4], N0, 0.0174, inv, 92.5e9, **kw)
            b = O.launch_peripheral_rays([2.5, 0.1, 0.4], N0, 0.0174, inv, 92.5e9, **kw)
            for u, v in zip(a, b):
                assert u.shape == v.shape
                assert np.abs(u - v).max() < 1e-14
    assert np.allclose(T.pol_tor_angles_2_vector(0.3, 0.2), O.pol_tor_angles_2_vector(0.3, 0.2),
                       atol=0, rtol=0)


def test_ray_entry_matches_oracle(T, O, hplasma, oplasma):
    om = 2 * np.pi * 92.5e9
    N0 = T.pol_tor_angles_2_vector(np.deg2rad(30), 0.0)
    pos, dirs, w = T.launch_peripheral_rays([2.5, 0, 0.4], N0, 0.0174, 1 / 3.99, 92.5e9,
                                            N_rings=5, min_azimuthal_points=5)
    # include launch points off the (R, Z) grid: first_point's toroidal intersection
    extra_p = np.array([[2.9, 0.0, 0.2], [2.0, 0.0, 1.2]])
    extra_d = np.array([[-1.0, 0.0, -0.1], [0.05, 0.0, -1.0]])
    extra_d /= np.linalg.norm(extra_d, axis=1)[:, None]
    pos, dirs = np.vstack([pos, extra_p]), np.vstack([dirs, extra_d])
    for mode in (1, -1):
        xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, mode)
        for i in range(len(pos)):
            so, xo, No, s0o = oplasma.ray_entry(pos[i], dirs[i], om, mode)
            assert st[i] == so
            if so == 0:
                assert np.abs(xp[i] - xo).max() < 1e-12
                assert np.abs(Np[i] - No).max() < 1e-12
                assert abs(s0[i] - s0o) < 1e-12
                assert abs(oplasma.dispersion_relation(xp[i], Np[i], om, mode)) < 1e-12
                assert oplasma.evaluate("psi", xp[i]) <= oplasma.psi_prof_max + 1e-12


def test_entry_reflection_status(T, eq):
    """N_s^2(N_par=0) <= 0 at the edge (src/solve.jl:57-59) -> REFLECTED status:
    O-mode above the edge cutoff."""
    from torj_hip import synthetic as S

    dense = S.circular_tokamak(ne_edge=3e20)
    P = T.Plasma(*S.plasma_args(dense))
    N0 = T.pol_tor_angles_2_vector(np.deg2rad(30), 0.0)
    xp, Np, s0, st = T.ray_entry(P, [[2.5, 0, 0.4]], [N0], 2 * np.pi * 92.5e9, -1)
    assert st[0] == T.REFLECTED


def test_shell_volumes(hplasma, oplasma):
    g = np.linspace(0, 1, 1000)
    dV = hplasma.shell_volumes(g)
    want = np.diff([oplasma.volume(p) for p in g])
    assert rel_err(dV, want).max() < 1e-10


def test_gpu_entry_points_fail_loudly_without_gpu(T, hplasma):
    """No CPU fallback: without a HIP device every compute call raises."""
    n = ctypes.c_int(0)
    if T.lib().torj_device_count(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(T.TorjError):
        T.trace(hplasma, [[2.2, 0, 0.2]], [[-0.9, 0, -0.4]], 6e11, 1, n_steps=10, absorption=False)
    with pytest.raises(T.TorjError):
        T.B_spline(hplasma, [2.0, 0.0, 0.1])


def test_trace_rejects_non_increasing_psi_grid(T, hplasma):
    """psi_dP_dV must be strictly increasing (the shell lookups assume it): the
    host-pointer call checks its copy before any device work, so this runs on
    CPU; the device-pointer call reports it through torj_trace_check (GPU test)."""
    x = np.array([[2.3, 0.0, 0.1]])
    N = np.array([[-0.9, 0.0, -0.3]])
    grid = np.array([0.0, 0.5, 0.5, 1.0])
    with pytest.raises(RuntimeError, match="strictly increasing"):
        T.trace(hplasma, x, N, 2 * np.pi * 92.5e9, 1, n_steps=10, psi_grid=grid)
