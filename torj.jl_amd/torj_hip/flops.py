"""Algorithmic FLOP accounting of the ray-stepping kernel (roofline numerator).

Per-component op counts produced by the instrumented restatement
`python oracle/flopcount.py` (counting convention: add/sub/mul/div/sqrt = 1,
exp 26, sin/cos 20, acos 30 -- SURVEY.md §8(d)).  The kernel reports exact
work counters per launch (ray-steps, RHS evaluations, absorption calls that
reach the harmonic sum, harmonic integrals), so the per-launch figure is exact
for the branches actually taken.  Absorption calls that exit early (Te < 20 eV,
N outside (0,1], X >= 1) are counted as zero work (conservative).
"""
from __future__ import annotations

FLOPS_RHS_COLD = 815        # spline fields + B rotation + analytic dD/dx, dD/dN + Te
FLOPS_ALPHA_PRE = 135       # abs_Albajar_fast up to the harmonic sum (pol. vector etc.)
FLOPS_ALPHA_POST = 22       # Maxwellian normalisation + final scaling
FLOPS_HARM = 30 + 6         # per harmonic: coefficients + post-scaling
FLOPS_NODE = 123            # per Gauss-Legendre node (2 x 15-term Bessel series, pol, gamma, exp)
FLOPS_STEP_OVERHEAD = 234   # RK4 combination, exp(-tau), psi evaluation


def algorithmic_flops(counters, n_gl: int = 24) -> float:
    """counters = (ray_steps, rhs_evals, alpha_active, harmonic_integrals)."""
    steps, rhs, act, harm = (float(c) for c in counters[:4])
    return (steps * FLOPS_STEP_OVERHEAD + rhs * FLOPS_RHS_COLD
            + act * (FLOPS_ALPHA_PRE + FLOPS_ALPHA_POST)
            + harm * (FLOPS_HARM + n_gl * FLOPS_NODE))
