"""Algorithmic FLOP accounting of the ray-stepping kernel (roofline numerator).

Per-component op counts produced by the instrumented restatement
`python oracle/flopcount.py` (counting convention: add/sub/mul/div/sqrt = 1,
exp 26, sin/cos 20, acos 30 -- SURVEY.md §8(d)) of the node-pair algorithm the
kernel runs (the regrouped pair form and reciprocal-based prologue of
torj_math.hpp: work the kernel no longer does is no longer counted).  The kernel reports exact work counters per launch (ray-steps, RHS
evaluations, absorption calls that reach the harmonic sum, harmonic integrals,
Bessel-series terms), so the per-launch figure is exact for the branches
actually taken.  Absorption calls that exit early (Te < 20 eV, N outside (0,1],
X >= 1) are counted as zero work (conservative).
"""
from __future__ import annotations

FLOPS_RHS_COLD = 815        # spline fields + B rotation + analytic dD/dx, dD/dN + Te
FLOPS_ALPHA_PRE = 83        # abs_Albajar_fast up to the harmonic sum (pol. vector etc.)
FLOPS_ALPHA_POST = 17       # Maxwellian normalisation + final scaling
FLOPS_HARM = 46             # per harmonic: K0..K5, C0..C2, u_par coefficients, post-scaling
FLOPS_PAIR_SHARED = 35      # per +-t node pair: Bessel argument, recurrence, P, Q, combination
FLOPS_NODE = 30             # per node: gamma^2, sqrt, exponent, exp
FLOPS_SERIES_TERM = 4       # per Horner term (two series, one fma each)
FLOPS_STEP_OVERHEAD = 234   # RK4 combination, exp(-tau), psi evaluation
FLOPS_ZERO_TEST = 12        # per harmonic found exactly zero: the gamma_min bound (its setup
                            # is FLOPS_HARM; the node loop it skips is not counted)


def algorithmic_flops(counters, n_gl: int = 24) -> float:
    """counters = (ray_steps, rhs_evals, alpha_active, harmonic_integrals, series_terms
    [, harmonic_integrals_exact_zero])."""
    steps, rhs, act, harm, terms = (float(c) for c in counters[:5])
    zero = float(counters[5]) if len(counters) > 5 else 0.0
    pairs = (n_gl + 1) // 2
    return (steps * FLOPS_STEP_OVERHEAD + rhs * FLOPS_RHS_COLD
            + act * (FLOPS_ALPHA_PRE + FLOPS_ALPHA_POST)
            + harm * (FLOPS_HARM + pairs * FLOPS_PAIR_SHARED + n_gl * FLOPS_NODE)
            + zero * (FLOPS_HARM + FLOPS_ZERO_TEST)
            + FLOPS_SERIES_TERM * (terms - harm * pairs))
