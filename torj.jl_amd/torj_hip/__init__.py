"""torj_hip -- MI355X-native drop-in for TorJ.jl's ray-tracing path.

Python mirror of the reference API (TorJ.jl src/*.jl) over the C ABI of
libtorj_hip.so (include/torj_hip.h); every compute call runs on the GPU.
"""
from ._lib import EXPORTED, LIB_PATH, TorjError, build, lib
from .launch import launch_peripheral_rays, pol_tor_angles_2_vector
from .physics import (abs_Al_init, abs_Albajar_fast, alpha_warm, alpha_approx, dispersion_relation,
                      grad_lambda, gradΛ, refractive_index_sq, α_approx)
from .plasma import B_spline, Plasma, T_e, eval_plasma, evaluate, n_e, power_deposition_profile
from .solve import (ABSORBED, ENTRY_FAIL, LEFT_PLASMA, MAX_STEPS, NAN, OK, REFLECTED, STATUS_NAMES,
                    RayEntryError, TraceResult, make_beam, make_ray, ray_entry, trace)

__all__ = [
    "Plasma", "evaluate", "B_spline", "n_e", "T_e", "eval_plasma", "refractive_index_sq",
    "dispersion_relation", "gradΛ", "grad_lambda", "abs_Al_init", "abs_Albajar_fast", "alpha_warm",
    "α_approx", "alpha_approx", "launch_peripheral_rays", "pol_tor_angles_2_vector",
    "make_ray", "make_beam", "ray_entry", "trace", "TraceResult", "RayEntryError", "TorjError",
    "build", "lib", "LIB_PATH", "EXPORTED", "STATUS_NAMES", "power_deposition_profile",
]
