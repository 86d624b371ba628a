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
FLOPS_HARM = 40             # per harmonic: K0..K5, the node exponents' Y0 / Y1, post-scaling
FLOPS_PAIR_SHARED = 32      # per +-t node pair: Bessel argument, recurrence, P, Q, combination
FLOPS_NODE = 28             # per node: exponent Y0 -+ Y1 t (gamma linear in t, round 6), exp
FLOPS_SERIES_TERM = 4       # per Horner term (two series, one fma each)
FLOPS_STEP_OVERHEAD = 234   # RK4 combination, exp(-tau), psi evaluation
FLOPS_ZERO_TEST = 1         # per harmonic found exactly zero: the largest node exponent
                            # Y0 + |Y1| (its setup is FLOPS_HARM; the node loop it skips is not
                            # counted; round 5: 12 for the gamma_min bound of the quadratic form)
FLOPS_NEGL_TEST = 35        # per harmonic skipped as below an ulp of the sum (torj_math.hpp
                            # albajar_harmonic): the bound's Bessel/polarisation factors (33),
                            # E_max as 2^(ceil(ymax) + 1) (2; round 5: exp(mu (1 - gamma_min)),
                            # 26 + 3) -- on top of FLOPS_HARM and the
                            # gamma_min test; the node loop it skips is not counted.  Tests that
                            # do not skip cost the same and are not counted (conservative).
FLOPS_EARLY_HARM = 12       # per harmonic of a call settled before the polarisation vector
                            # (torj_math.hpp harm_geom: r, sqrt(r^2 - 1), u_par1, Y0, Y1 (11) and
                            # the zero test's Y0 + |Y1| (1); round 5: 27 with the quadratic
                            # form's C0..C2 and gamma_min); the call's own prologue
                            # (mu, omega_bar, N_perp, m_0: 12) is not counted (conservative).


def algorithmic_flops(counters, n_gl: int = 24) -> float:
    """counters = (ray_steps, rhs_evals, alpha_active, harmonic_integrals, series_terms
    [, harmonic_integrals_exact_zero [, harmonic_integrals_negligible
    [, harmonic_integrals_settled_early]]])."""
    steps, rhs, act, harm, terms = (float(c) for c in counters[:5])
    zero = float(counters[5]) if len(counters) > 5 else 0.0
    negl = float(counters[6]) if len(counters) > 6 else 0.0
    early = float(counters[7]) if len(counters) > 7 else 0.0
    pairs = (n_gl + 1) // 2
    return (steps * FLOPS_STEP_OVERHEAD + rhs * FLOPS_RHS_COLD + early * FLOPS_EARLY_HARM
            + act * (FLOPS_ALPHA_PRE + FLOPS_ALPHA_POST)
            + harm * (FLOPS_HARM + pairs * FLOPS_PAIR_SHARED + n_gl * FLOPS_NODE)
            + zero * (FLOPS_HARM + FLOPS_ZERO_TEST)
            + negl * (FLOPS_HARM + FLOPS_ZERO_TEST + FLOPS_NEGL_TEST)
            + FLOPS_SERIES_TERM * (terms - harm * pairs))


def algorithmic_flops_reference(counters, n_gl: int = 24) -> float:
    """The same launch priced as the reference's algorithm (the CPU restatement,
    SURVEY.md §8(d)): every harmonic integral with m >= m_0 evaluated with its
    full node loop -- the exactly-zero and the negligible integrals the kernel
    skips (bit-identically) at the cost of an evaluated one, with the shortest
    Bessel polynomial (7 terms; a lower bound), and the calls settled before
    the polarisation vector priced by their harmonics alone.  A figure beside
    algorithmic_flops, never instead of it: the roofline fraction is priced on
    the work the kernel does."""
    zero = float(counters[5]) if len(counters) > 5 else 0.0
    negl = float(counters[6]) if len(counters) > 6 else 0.0
    early = float(counters[7]) if len(counters) > 7 else 0.0
    pairs = (n_gl + 1) // 2
    skipped = zero + negl + early
    return (algorithmic_flops(counters, n_gl)
            - zero * (FLOPS_HARM + FLOPS_ZERO_TEST) - negl * (FLOPS_HARM + FLOPS_ZERO_TEST + FLOPS_NEGL_TEST)
            - early * FLOPS_EARLY_HARM
            + skipped * (FLOPS_HARM + pairs * FLOPS_PAIR_SHARED + n_gl * FLOPS_NODE
                         + FLOPS_SERIES_TERM * pairs * (7 - 1)))


# Weakly relativistic warm alpha (absorption 2, torj_warm.hpp alpha_warm_v<1>),
# per trip, from the instrumented restatement `python oracle/flopcount_warm.py`
# (same convention; factorial tables and loop invariants not counted; branch-
# dependent parts at their cheapest branch, so the model is a lower bound: 97.5-
# 99.8 % of the instrumented count, tests/test_warm_flops.py).
FLOPS_WARM_CALL = 80          # Te, |N|, mu, N_perp, per-call invariants, e330, alpha
FLOPS_WARM_LARMOR_TEST = 10   # per larmornumber resonance test
FLOPS_WARM_FADDEEVA = 176     # per Z(z) by Weideman's N = 36 sum (|z| < 16) by the real-coefficient recurrence (round 6; 278 by complex Horner)
FLOPS_WARM_FADDEEVA_ASYM = 60   # per Z(z) by the asymptotic series (|x| or Im z >= 16), 10 terms by the real-coefficient recurrence (round 6; 84 by complex Horner)
FLOPS_WARM_SIDE = 14          # per fsup side s = +-|s|: alpha_s, phi, cf12, cf32
FLOPS_WARM_STEP = 6           # per Shkarofsky recursion step
FLOPS_WARM_STORE = 4          # per stored recursion step: cefp, cefm accumulation
FLOPS_WARM_ISA = 22           # per |s|: cq0p .. cq2p
FLOPS_WARM_PAIR = 27          # per (|s|, l) term of the tensor sums
FLOPS_WARM_ORDER = 15         # per Larmor order l: f_l and the six components
FLOPS_WARM_SUM_TERM = 54      # per warmdisp update and order: sum eps_l N_perp^(2l)
FLOPS_WARM_UPDATE = 167       # per warmdisp update: cc4, cc2, cc0, root, convergence


def algorithmic_flops_warm(counters) -> float:
    """counters = the 8 work counters of an absorption-2 launch (include/torj_hip.h
    torj_trace_device): ray-steps, RHS evaluations (= warm alpha calls), Faddeeva
    evaluations by the asymptotic series, Faddeeva evaluations (all), warmdisp
    passes, passes x lrm, sum lrm, sum lrm^2.  larmornumber's resonance tests are
    priced at one per call (their least; a lower bound)."""
    steps, calls, asym, fad, passes, pass_l, sl, sl2 = (float(c) for c in counters[:8])
    tests = calls
    sides = 2.0 * sl + calls                  # is = -|s| .. |s|
    rsteps = sl2 + 5.0 * sl + 2.0 * calls     # recursion steps: lrm^2 + 5 lrm + 2 per call
    stored = 6.0 * sl + 2.0 * calls
    pairs = 0.5 * (sl2 + 3.0 * sl)            # (|s|, l), max(|s|, 1) <= l <= lrm
    updates = passes - calls                  # every pass but the breaking one
    sums = pass_l - sl                        # the breaking pass sums no tensor (torj_warm.hpp warmdisp_n2)
    return (steps * FLOPS_STEP_OVERHEAD + calls * (FLOPS_RHS_COLD + FLOPS_WARM_CALL)
            + tests * FLOPS_WARM_LARMOR_TEST + (fad - asym) * FLOPS_WARM_FADDEEVA
            + asym * FLOPS_WARM_FADDEEVA_ASYM
            + sides * FLOPS_WARM_SIDE + rsteps * FLOPS_WARM_STEP + stored * FLOPS_WARM_STORE
            + (sl + calls) * FLOPS_WARM_ISA + pairs * FLOPS_WARM_PAIR + sl * FLOPS_WARM_ORDER
            + sums * FLOPS_WARM_SUM_TERM + updates * FLOPS_WARM_UPDATE)
