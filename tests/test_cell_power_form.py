"""The cell-tiled trajectory kernel's field evaluation (torj_math.hpp
cell_power_table / cell_sums, k_traj_cell): each grid cell's bicubic in power
form against the node stencil the other kernels use (eval_fields on the
B-spline coefficients, Interpolations.jl's Cubic(Line(OnGrid())) convention,
src/plasma.jl:30-58), host build (tests/native).  The same interpolant: values
and gradients agree to rounding inside the grid, and the Line() extrapolation
outside it (gradient at the clamped point, the mixed term) is the same."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
_dp = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def H():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native"), "build/libwarm_host.so"])
    L = C.CDLL(os.path.join(HERE, "native", "build", "libwarm_host.so"))
    L.fe_eval.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, _dp, C.c_int,
                          _dp, _dp, C.c_int, _dp]
    return L


def _eval(H, nR, nZ, box, coef, R, Z, cell):
    out = np.zeros((len(R), 14))
    d = lambda a: np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(_dp)  # noqa: E731
    H.fe_eval(nR, nZ, *box, d(coef), len(R), d(R), d(Z), cell, out.ctypes.data_as(_dp))
    return out


@pytest.mark.parametrize("nR,nZ", [(56, 56), (17, 29)])
def test_cell_power_form_matches_node_stencil(H, nR, nZ):
    rng = np.random.default_rng(7 + nR)
    box = (1.1, 3.3, -1.4, 1.2)
    # smooth fields (as the physics' B, ln ne, ...) plus ulp-scale noise, 8
    # doubles per node over the (nR + 2) x (nZ + 2) padded node grid
    u = np.linspace(0, 1, nR + 2)[None, :, None]
    v = np.linspace(0, 1, nZ + 2)[:, None, None]
    f = np.arange(8)[None, None, :]
    coef = (np.sin(2.1 * u + 0.7 * f) * np.cos(1.3 * v - 0.3 * f) * (1 + f) + 40.0 * (f == 3)
            + 1e-3 * rng.standard_normal((nZ + 2, nR + 2, 8)))
    coef = np.ascontiguousarray(coef.reshape(-1))
    n = 4000
    R = rng.uniform(box[0], box[1], n)
    Z = rng.uniform(box[2], box[3], n)
    # grid edges, nodes exactly, and points outside (Line() extrapolation)
    R[:8] = [box[0], box[1], box[0], box[1], box[0] - 0.07, box[1] + 0.2, 2.0, 2.0]
    Z[:8] = [box[2], box[3], box[3], box[2], 0.1, -0.3, box[2] - 0.05, box[3] + 0.11]
    R[8:40] = box[0] + (box[1] - box[0]) * rng.integers(0, nR, 32) / (nR - 1)
    ref = _eval(H, nR, nZ, box, coef, R, Z, 0)
    got = _eval(H, nR, nZ, box, coef, R, Z, 1)
    # values to a few ulps of the field; gradients to a few ulps of the field's
    # size over the cell width (both forms difference O(1) coefficients whose
    # rounding, ~1e-16 of |c|, is amplified by 1 / h; e.g. ln ne ~ 40)
    vals = np.abs(got[:, :6] - ref[:, :6]) / np.abs(ref[:, :6]).max(0)
    assert vals.max() <= 4e-15, vals.max(0)
    fsz = np.abs(ref[:, :4]).max(0).repeat(2)
    invh = np.tile([(nR - 1) / (box[1] - box[0]), (nZ - 1) / (box[3] - box[2])], 4)
    grads = np.abs(got[:, 6:] - ref[:, 6:]) / (fsz * invh)
    assert grads.max() <= 2e-15, grads.max(0)
    print(f"cell power form vs node stencil: values {vals.max():.1e}, gradients {grads.max():.1e} "
          f"(of |f| / h)")
