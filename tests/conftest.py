"""Shared fixtures.  `-m "not gpu"` runs on CPU (oracle pins, host-side product
code, C-ABI load/exports, gloo distributed); `-m gpu` needs an MI355X and runs
the HIP kernels through the C ABI against the oracle and golden fixtures."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (HIP kernels)")
    # build artefacts (in-tree): the oracle (test infrastructure) and the product
    if not os.path.exists(os.path.join(ROOT, "oracle", "build", "libtorj_oracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(os.path.join(ROOT, "torj.jl_amd", "build", "libtorj_hip.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "torj.jl_amd", "csrc")])


@pytest.fixture(scope="session")
def O():
    import oracle

    oracle.abs_al_init(24)
    return oracle


@pytest.fixture(scope="session")
def T():
    import torj_hip

    return torj_hip


@pytest.fixture(scope="session")
def eq():
    from torj_hip import synthetic

    return synthetic.circular_tokamak()


@pytest.fixture(scope="session")
def oplasma(O, eq):
    from torj_hip import synthetic

    return O.OraclePlasma(*synthetic.plasma_args(eq))


@pytest.fixture(scope="session")
def hplasma(T, eq):
    """Product Plasma handle (host-side construction works without a GPU)."""
    from torj_hip import synthetic

    return T.Plasma(*synthetic.plasma_args(eq))


@pytest.fixture(scope="session")
def gpu(T):
    import ctypes

    # PyTorch-ROCm carries its own HIP runtime; when both share a process (the
    # device-pointer tests, bench.py), torch's must initialise the device first
    # -- after libtorj_hip's runtime has, torch reports no HIP GPU
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
    n = ctypes.c_int(0)
    rc = T.lib().torj_device_count(ctypes.byref(n))
    if rc != 0 or n.value < 1:
        pytest.fail("no HIP device: GPU tests need an MI355X")
    T.abs_Al_init(24)
    return n.value


@pytest.fixture(scope="session")
def fan_states(T, hplasma, eq):
    """In-plasma start states of the test_make_beam geometry at 92.5 GHz (X and O mode)."""
    from torj_hip import synthetic as S

    s = S.SETUP
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], s["f_abs_test"],
                                            N_rings=14, min_azimuthal_points=5)
    om = 2 * np.pi * s["f_abs_test"]
    out = {}
    for mode in (1, -1):
        xp, Np, s0, st = T.ray_entry(hplasma, pos, dirs, om, mode)
        assert (st == 0).all()
        out[mode] = (xp, Np, w, om)
    return out


def rel_err(a, b, floor=0.0):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return np.abs(a - b) / np.maximum(np.abs(b), floor)
