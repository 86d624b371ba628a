// torj_math.hpp -- ray-physics math shared by the HIP kernels (device) and the
// host-side setup code (ray entry, Plasma construction) of libtorj_hip.
//
// MI355X design notes:
//  * All six 2-D B-spline fields live on ONE (R,Z) grid (src/plasma.jl:30-58), so
//    the 16 basis weights (+ R/Z derivative weights) are computed once per point
//    and applied to every field.  Coefficients are stored node-interleaved
//    (8 doubles = 64 B per node: Br, Bphi, Bz, ln ne, ln Te, psi, pad, pad) so a
//    4x4 stencil is 4 runs of 256 contiguous bytes.
//  * ForwardDiff's two gradients of the dispersion relation (src/solve.jl:89-90)
//    are replaced by ONE analytic evaluation of D, dD/dx and dD/dN (the spline
//    work is shared instead of being redone per dual pass).
//  * The Albajar Bessel factors J_{m-1}, J_m, J_{m+1} come from two Horner power
//    series (J_m, J_{m+1}) and the stable downward recurrence for J_{m-1}.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "torj_bessel_coefs.hpp"

#define TORJ_HD __host__ __device__ __forceinline__

namespace torj {

// src/constants.jl:13-26
constexpr double kC = 2.99792458e8;
constexpr double kE = 1.602176634e-19;
constexpr double kMe = 9.1093837015e-31;
constexpr double kEps0 = 8.8541878128e-12;
constexpr double kPi = 3.14159265358979323846;

constexpr int kNF = 8;  // doubles per coefficient node
enum Field { F_BR = 0, F_BPHI = 1, F_BZ = 2, F_LNNE = 3, F_LNTE = 4, F_PSI = 5 };

// ray status codes (include/torj_hip.h)
enum Status { ST_OK = 0, ST_LEFT_PLASMA = 1, ST_ABSORBED = 2, ST_NAN = 3, ST_REFLECTED = 4,
              ST_ENTRY_FAIL = 5, ST_MAX_STEPS = 6 };

struct Grid {
    int nR, nZ;          // data points (coefficients are (nR+2) x (nZ+2))
    double R1, Z1, Rn, Zn;
    double hR, hZ, invhR, invhZ;
};

// value_weights / gradient_weights of Interpolations.jl's Cubic B-spline
TORJ_HD void bweights(double d, double w[4], double dw[4]) {
    const double p = 1.0 - d;
    const double d2 = d * d, p2 = p * p;
    w[0] = p2 * p * (1.0 / 6.0);
    w[1] = 2.0 / 3.0 - d2 + 0.5 * d2 * d;
    w[2] = 2.0 / 3.0 - p2 + 0.5 * p2 * p;
    w[3] = d2 * d * (1.0 / 6.0);
    dw[0] = -0.5 * p2;
    dw[1] = -2.0 * d + 1.5 * d2;
    dw[2] = 2.0 * p - 1.5 * p2;
    dw[3] = 0.5 * d2;
}

TORJ_HD double clampd(double x, double lo, double hi) { return x > hi ? hi : (x < lo ? lo : x); }

// Julia's round(Int64, x) (RoundNearest: halfway cases to the even integer,
// e.g. the azimuthal point counts of src/launch.jl:81); C's lround would take
// them away from zero.  rint rounds in the default (to-nearest-even) mode and
// is exact for every representable halfway case.
TORJ_HD long round_ties_even(double x) { return (long)rint(x); }

// 1/x for the denominators of the ray RHS and the absorption prologue: on the
// device v_rcp_f64 + two Newton steps (<= 1 ulp) instead of the IEEE division
// sequence (div_scale x2, rcp, five fma, div_fmas, div_fixup per quotient).
// Special operands give NaN (0 and inf included), on the host too (same Newton
// steps after an exact 1/x), so host and device agree on which results are
// finite; the callers only pass denominators that are finite and non-zero on
// every physical input (a zero means a resonance/cutoff the reference also
// turns into a non-finite result).
TORJ_HD double rcp_nz(double x) {
#ifdef __HIP_DEVICE_COMPILE__
    double r = __builtin_amdgcn_rcp(x);
#else
    double r = 1.0 / x;
#endif
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// sqrt of a finite positive normal argument (lengths, |B|, |dD/dN|): on the
// device v_rsq_f64 + one Goldschmidt step + one Newton correction (~1 ulp; the
// library sequence adds a second correction for correct rounding plus denormal
// scaling and class checks).
TORJ_HD double sqrt_pos(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    return fma(fma(-g, g, x), h, g);
#else
    return sqrt(x);
#endif
}

// 1/sqrt(x) of a finite positive normal argument: v_rsq_f64 + two Newton steps
// (~1 ulp; 9 VALU against sqrt_pos + rcp_nz's 13 where only the reciprocal is
// needed, 10 with x * rsqrt_pos(x) where both are)
// (the host build runs the same Newton steps after an exact 1/sqrt, so host
// and device agree on the special operands: NaN at 0, inf, negative, NaN)
TORJ_HD double rsqrt_pos(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rsq(x);
#else
    double y = 1.0 / sqrt(x);
#endif
    double e = fma(-x * y, y, 1.0);
    y = fma(0.5 * y, e, y);
    e = fma(-x * y, y, 1.0);
    return fma(0.5 * y, e, y);
}

// sqrt for the absorption prologue and the harmonic setup: sqrt_pos plus the
// library's results at +-0 and +inf (a v_cmp_class and a select instead of the
// library's scaling, two Newton corrections and class fix-up: 11 VALU against
// 18).  Negative arguments and NaN give NaN like the library; the arguments
// are never denormal (lengths and squares of O(1) physical quantities or 0).
TORJ_HD double sqrt_nn(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double s = sqrt_pos(x);
    return __builtin_amdgcn_class(x, 0x260) ? x : s;  // -0, +0, +inf
#else
    return sqrt(x);
#endif
}

// gamma of the Albajar node loop: v_rsq_f64 + the Goldschmidt step of sqrt_pos
// without its Newton correction (a few ulp).  gamma enters only as
// exp(mu (1 - gamma)) with mu (gamma - 1) < 760 on every node that is not an
// exact zero, so a relative error e moves a node term by ~mu gamma e; the
// Albajar golden sweep and the headline-fan parity hold at 1e-10 (C3 trace
// phase -2.5 % on top of the degree-9 node exp).
TORJ_HD double sqrt_node(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    const double g = x * y, h = 0.5 * y;
    return fma(g, fma(-h, g, 0.5), g);
#else
    return sqrt(x);
#endif
}

// exp on the device: range reduction + degree-11 near-minimax polynomial +
// ldexp (~1 ulp).  No special-case paths: ldexp overflows to inf above ~709
// and underflows to 0 below ~-745, NaN stays NaN.  Used for n_e, T_e from
// their log splines (the node loop takes exp2_node below).
// A constant for a VALU operand, materialised in an SGPR pair at its use
// (exp_fast<true>): left to itself the compiler puts a straight-line Horner
// chain's coefficients in VGPRs, two v_mov_b32 per coefficient ahead of a
// v_fmac -- 20 VALU of exp_fast's 37 -- where two s_mov_b32 and a v_fma_f64
// with an SGPR operand do.  The empty asm is volatile so that it is neither
// hoisted nor merged: the pair lives for one instruction.  For kernels with
// SGPRs to spare only (k_alpha_pts: 103 of 106, no spills); the trajectory
// kernel, at 106 with spills, keeps its constants hoisted in VGPRs.
#ifndef TORJ_EXP_SCONST
#define TORJ_EXP_SCONST 1
#endif
template <bool S>
TORJ_HD double poly_c(double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (S && TORJ_EXP_SCONST) asm volatile("" : "+s"(c));
#endif
    return c;
}

template <bool SC = false>
TORJ_HD double exp_fast(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double k = __builtin_rint(x * 1.4426950408889634074);
    double r = fma(-k, 6.93147180559945286227e-01, x);
    r = fma(-k, 2.31904681384629955842e-17, r);
    // degree 11 near-minimax on |r| <= ln2/2 (tools/gen_exp_poly.py: 0.58 ulp,
    // against 1.5 ulp for the degree 12 Taylor polynomial)
    double p = poly_c<SC>(2.5100375832561234e-08);
    p = fma(p, r, poly_c<SC>(2.7620075879983367e-07));
    p = fma(p, r, poly_c<SC>(2.7557268480310024e-06));
    p = fma(p, r, poly_c<SC>(2.4801521322368692e-05));
    p = fma(p, r, poly_c<SC>(0.00019841269863040545));
    p = fma(p, r, poly_c<SC>(0.0013888888917196719));
    p = fma(p, r, poly_c<SC>(0.008333333333330065));
    p = fma(p, r, poly_c<SC>(0.041666666666624164));
    p = fma(p, r, poly_c<SC>(0.16666666666666669));
    p = fma(p, r, poly_c<SC>(0.5000000000000001));
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    // v_cvt_i32_f64 saturates out-of-range k (the C conversion would be UB),
    // and ldexp of a huge negative exponent underflows to 0
    int ki;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(ki) : "v"(k));
    return __builtin_amdgcn_ldexp(p, ki);
#else
    return exp(x);
#endif
}

// exp of the Albajar node loop, exp(mu (1 - gamma)), in base 2: exp2_node(y) =
// 2^y with y = mu log2(e) (1 - gamma) formed by the caller (mu log2(e) is a
// per-harmonic constant, so y costs the one fma the natural exponent did).
// k = round(y) by the 1.5 * 2^52 shifter (k in the low word of kd: no v_rndne,
// no v_cvt), r = y - k exact (Sterbenz, |r| <= 1/2), and a degree-9
// near-minimax polynomial for 2^r: exp's on |x| <= ln2/2 (round 4: degree 8,
// tools/gen_exp_poly.py 8: 4.3e-12 relative; degree 9 before, 7.4e-14) with its
// coefficients scaled by ln2^i.  Each node term carries it once; over 100 000
// random tuples alpha's median error against the libm oracle is 3e-13 (2e-14
// at degree 9), p99 2.9e-12 (1.8e-12), all under the 1e-10 parity bar but the
// conditioning-limited few.  12 VALU against exp_fast's 17: 3
// for the reduction instead of 5, degree 8 instead of 11.  Exact for |y| < 2^51;
// node arguments have mu = m_e c^2 / Te < 25 550 (Te >= 20 eV,
// src/absorption.jl:194).  Every node of a lane the exact-zero bound skips has
// y < -1096 and gives exactly +0, so the skip stays bit-identical.
TORJ_HD double exp2_node(double y) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double kd = y + 0x1.8p52;
    const double r = y - (kd - 0x1.8p52);
    double p = 1.3246387161221642e-06;
    p = fma(p, r, 1.5297323760701075e-05);
    p = fma(p, r, 0.00015403491754738786);
    p = fma(p, r, 0.0013333502386162772);
    p = fma(p, r, 0.009618129119704426);
    p = fma(p, r, 0.055504108839096185);
    p = fma(p, r, 0.24022650695910072);
    p = fma(p, r, 0.6931471805599453);
    p = fma(p, r, 1.0);
    const int ki = (int)(unsigned)__builtin_bit_cast(unsigned long long, kd);  // k, low word
    return __builtin_amdgcn_ldexp(p, ki);
#else
    return exp2(y);
#endif
}

// x 2^k (v_ldexp_f64 on the device)
TORJ_HD double ldexp_i(double x, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ldexp(x, k);
#else
    return ldexp(x, k);
#endif
}
#ifndef TORJ_EMAX_BOUND  // albajar_harmonic's skip tests: E_max by a power-of-two bound (1, round 6:
// C3 trace phase 40.28 / 40.29 -> 39.77 / 39.86 ms alternating) or by exp (0)
#define TORJ_EMAX_BOUND 1
#endif

// Stencil position on one axis: clamped coordinate, cell index, weights.
struct Axis {
    int i;
    double delta;  // x - clamp(x): Line() extrapolation distance
    double w[4], dw[4];
};

TORJ_HD void axis_setup(double x, double x1, double xn, double invh, int n, Axis &a) {
    const double xc = clampd(x, x1, xn);
    a.delta = x - xc;
    const double u = (xc - x1) * invh;
    int i = (int)floor(u);
    i = i < 0 ? 0 : (i > n - 2 ? n - 2 : i);
    bweights(u - (double)i, a.w, a.dw);
    a.i = i;
}

// Field values with physical R and Z derivatives, Line() extrapolation applied
// with exactly the derivative ForwardDiff sees through Interpolations'
// extrapolate(): inside an axis the gradient of the other axis' extension term
// contributes (mixed derivative), outside it the slope is constant.
template <int NGRAD, int NVAL>
struct FieldPack {
    static constexpr int NG1 = NGRAD > 0 ? NGRAD : 1;
    double v[NGRAD + NVAL];
    double dR[NG1], dZ[NG1];
};

// Evaluate fields [0, NGRAD) with gradients and [NGRAD, NGRAD+NVAL) value-only.
// `fidx` maps pack slot -> coefficient field index.  EXT = false assumes the
// point is inside the grid on both axes (Line() extrapolation distances 0) and
// skips the sums only the extrapolation needs (value-only fields' slopes, the
// mixed derivative); the results are then identical to EXT = true.
// The 4 x 4 stencil's tensor-product sums from the node at `c0` (the stencil's
// first node), `rs` doubles between rows of nodes, NS doubles per node,
// accumulated row by row (few live registers):
//   v = sum wZ wR c, gr = sum wZ dwR c, gz = sum dwZ wR c, grz = sum dwZ dwR c
// The same arithmetic whatever memory c0 points into (global / L2 or an LDS
// tile), so the results do not depend on where the coefficients were read.
// 16-byte view of a coefficient pointer, in its address space: the 6-field
// layouts of the LDS-staged coefficients (48 B per node) are read a field pair
// at a time (ds_read_b128, 256 B/clk/CU, where two 8-byte reads merge into a
// ds_read2_b64 at 128 B/clk/CU)
struct alignas(16) Dbl2 {
    double x, y;
};
template <class P>
struct Pair16Ptr {
    using type = const Dbl2 *;
};
#ifdef __HIP_DEVICE_COMPILE__
template <>
struct Pair16Ptr<const __attribute__((address_space(3))) double *> {
    using type = const __attribute__((address_space(3))) Dbl2 *;
};
template <>
struct Pair16Ptr<const __attribute__((address_space(1))) double *> {
    using type = const __attribute__((address_space(1))) Dbl2 *;
};
#endif

template <int NGRAD, int NVAL, bool EXT, int NS, class P = const double *>
TORJ_HD void stencil_sums(P c0, int rs, const Axis &aR, const Axis &aZ,
                          const int (&fidx)[NGRAD + NVAL], double (&v)[NGRAD + NVAL],
                          double (&gr)[NGRAD + NVAL], double (&gz)[NGRAD + NVAL],
                          double (&grz)[NGRAD + NVAL]) {
    constexpr int NT = NGRAD + NVAL;
#pragma unroll
    for (int f = 0; f < NT; f++) v[f] = gr[f] = gz[f] = grz[f] = 0.0;
    // one field's sums, from its 4 coefficients of row b (the order of every
    // fma is the same whichever way the coefficients were read)
    auto field = [&](int f, int b, const double (&c)[4]) {
        const bool slopes = EXT || f < NGRAD;
        double sv = 0.0, sd = 0.0;
#pragma unroll
        for (int a = 0; a < 4; a++) {
            sv = fma(aR.w[a], c[a], sv);
            if (slopes) sd = fma(aR.dw[a], c[a], sd);
        }
        v[f] = fma(aZ.w[b], sv, v[f]);
        if (slopes) {
            gz[f] = fma(aZ.dw[b], sv, gz[f]);
            gr[f] = fma(aZ.w[b], sd, gr[f]);
        }
        if (EXT && f < NGRAD) grz[f] = fma(aZ.dw[b], sd, grz[f]);
    };
    if constexpr (NS == 6) {
        // the 6-field layouts: per row, one field pair of the 4 nodes at a time
        // (4 x ds_read_b128 for two fields, short live ranges)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const P row = c0 + (size_t)b * rs;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                bool need = false;
#pragma unroll
                for (int f = 0; f < NT; f++) need = need || (fidx[f] >> 1) == k;
                if (!need) continue;
                double lo[4], hi[4];
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    const Dbl2 d = reinterpret_cast<typename Pair16Ptr<P>::type>(row + a * NS)[k];
                    lo[a] = d.x, hi[a] = d.y;
                }
#pragma unroll
                for (int f = 0; f < NT; f++)
                    if (fidx[f] == 2 * k)
                        field(f, b, lo);
                    else if (fidx[f] == 2 * k + 1)
                        field(f, b, hi);
            }
        }
        return;
    }
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const P row = c0 + (size_t)b * rs;
#pragma unroll
        for (int f = 0; f < NT; f++) {
            const bool slopes = EXT || f < NGRAD;
            double sv = 0.0, sd = 0.0;
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const double c = row[a * NS + fidx[f]];
                sv = fma(aR.w[a], c, sv);
                if (slopes) sd = fma(aR.dw[a], c, sd);
            }
            v[f] = fma(aZ.w[b], sv, v[f]);
            if (slopes) {
                gz[f] = fma(aZ.dw[b], sv, gz[f]);
                gr[f] = fma(aZ.w[b], sd, gr[f]);
            }
            if (EXT && f < NGRAD) grz[f] = fma(aZ.dw[b], sd, grz[f]);
        }
    }
}

// A wave's tile of the coefficient grid staged in LDS (the split pipeline's
// trajectory kernel): nodes [iR0, iR0 + tw) x [iZ0, iZ0 + th)
// at kTileNS doubles per node, R fastest; `g` is the whole grid (kNF per node)
// for a stencil that leaves the tile.  tw = 0: no tile, every read from g.
constexpr int kTileNS = 6;
struct TileCoef {
    const double *g;    // global coefficients, kNF doubles per node
    const double *lds;  // the tile
    int iR0, iZ0, tw, th;
};

template <int NGRAD, int NVAL, bool EXT>
TORJ_HD void fields_finish(const Grid &g, const Axis &aR, const Axis &aZ, const double *v,
                           const double *gr, const double *gz, const double *grz,
                           FieldPack<NGRAD, NVAL> &out);

// eval_fields reading the stencil from the wave's LDS tile when every lane's
// stencil lies inside it (one wave-uniform branch), from global memory
// otherwise; bit-identical to eval_fields on the whole grid either way.
template <int NGRAD, int NVAL, bool EXT = true, int NS = kNF>
TORJ_HD void eval_fields(const TileCoef &t, const Grid &g, double R, double Z,
                         const int (&fidx)[NGRAD + NVAL], FieldPack<NGRAD, NVAL> &out) {
    constexpr int NT = NGRAD + NVAL;
    Axis aR, aZ;
    axis_setup(R, g.R1, g.Rn, g.invhR, g.nR, aR);
    axis_setup(Z, g.Z1, g.Zn, g.invhZ, g.nZ, aZ);
    const int dR = aR.i - t.iR0, dZ = aZ.i - t.iZ0;
    bool in = dR >= 0 && dR <= t.tw - 4 && dZ >= 0 && dZ <= t.th - 4;
#ifdef __HIP_DEVICE_COMPILE__
    in = __all(in);
#endif
    double v[NT], gr[NT], gz[NT], grz[NT];
#ifdef __HIP_DEVICE_COMPILE__
    // explicit address spaces: ds_read from the tile, global_load otherwise (as
    // generic pointers the two paths merge into one flat load of either)
    using LdsP = const __attribute__((address_space(3))) double *;
    using GlbP = const __attribute__((address_space(1))) double *;
#else
    using LdsP = const double *;
    using GlbP = const double *;
#endif
    if (in)
        stencil_sums<NGRAD, NVAL, EXT, kTileNS, LdsP>((LdsP)t.lds + ((size_t)dZ * t.tw + dR) * kTileNS,
                                                      t.tw * kTileNS, aR, aZ, fidx, v, gr, gz, grz);
    else
        stencil_sums<NGRAD, NVAL, EXT, kNF, GlbP>((GlbP)t.g + ((size_t)aZ.i * (g.nR + 2) + aR.i) * kNF,
                                                  (g.nR + 2) * kNF, aR, aZ, fidx, v, gr, gz, grz);
    fields_finish<NGRAD, NVAL, EXT>(g, aR, aZ, v, gr, gz, grz, out);
}

template <int NGRAD, int NVAL, bool EXT = true, int NS = kNF>
TORJ_HD void eval_fields(const double *__restrict__ coef, const Grid &g, double R, double Z,
                         const int (&fidx)[NGRAD + NVAL], FieldPack<NGRAD, NVAL> &out) {
    constexpr int NT = NGRAD + NVAL;
    Axis aR, aZ;
    axis_setup(R, g.R1, g.Rn, g.invhR, g.nR, aR);
    axis_setup(Z, g.Z1, g.Zn, g.invhZ, g.nZ, aZ);
    const int mR = g.nR + 2;
    double v[NT], gr[NT], gz[NT], grz[NT];
    stencil_sums<NGRAD, NVAL, EXT, NS>(coef + ((size_t)aZ.i * mR + aR.i) * NS, mR * NS, aR, aZ, fidx,
                                       v, gr, gz, grz);
    fields_finish<NGRAD, NVAL, EXT>(g, aR, aZ, v, gr, gz, grz, out);
}

// physical gradients and Line() extrapolation from the stencil sums (the
// Line() distances dRx = R - clamp(R), dZx = Z - clamp(Z); gr, gz, grz: d/du,
// d/dv, d2/du dv in the grid's index coordinates)
template <int NGRAD, int NVAL, bool EXT, bool PHYS = false>
TORJ_HD void fields_finish_d(const Grid &g, double dRx, double dZx, const double *v,
                             const double *gr, const double *gz, const double *grz,
                             FieldPack<NGRAD, NVAL> &out);
template <int NGRAD, int NVAL, bool EXT>
TORJ_HD void fields_finish(const Grid &g, const Axis &aR, const Axis &aZ, const double *v,
                           const double *gr, const double *gz, const double *grz,
                           FieldPack<NGRAD, NVAL> &out) {
    fields_finish_d<NGRAD, NVAL, EXT>(g, aR.delta, aZ.delta, v, gr, gz, grz, out);
}
// PHYS: gr, gz, grz are already per metre (the cell records' scaled form)
template <int NGRAD, int NVAL, bool EXT, bool PHYS>
TORJ_HD void fields_finish_d(const Grid &g, double dRx, double dZx, const double *v,
                             const double *gr, const double *gz, const double *grz,
                             FieldPack<NGRAD, NVAL> &out) {
    constexpr int NT = NGRAD + NVAL;
    const bool outR = dRx != 0.0, outZ = dZx != 0.0;
#pragma unroll
    for (int f = 0; f < NT; f++) {
        const double gR = PHYS ? gr[f] : gr[f] * g.invhR, gZ = PHYS ? gz[f] : gz[f] * g.invhZ;
        if constexpr (EXT) {
            out.v[f] = v[f] + dRx * gR + dZx * gZ;
        } else {
            out.v[f] = v[f];
        }
        if (f < NGRAD) {
            const int q = f < NGRAD ? f : 0;
            if constexpr (EXT) {
                const double gRZ = PHYS ? grz[f] : grz[f] * (g.invhR * g.invhZ);
                out.dR[q] = outR ? gR : gR + dZx * gRZ;
                out.dZ[q] = outZ ? gZ : gZ + dRx * gRZ;
            } else {
                out.dR[q] = gR;
                out.dZ[q] = gZ;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The bicubic of one grid cell in power form (the split pipeline's cell-tiled
// trajectory kernel).  In cell (iR, iZ) with local coordinates
// tR, tZ in [0, 1] (axis_setup's cell and fraction), the B-spline sum
// sum_{b,a} wZ_b(tZ) wR_a(tR) c_{b,a} over the cell's 4 x 4 nodes is the
// polynomial sum_{j,i} A_ji tZ^j tR^i, A = B C B^T with B the uniform cubic
// B-spline's power-basis matrix (bweights), stored per metre: A_ji / (hR^i hZ^j)
// in the offsets sR = tR hR, sZ = tZ hZ from the cell's corner, so the
// derivatives come out per metre (no 1/h scaling per field):
//   a0 = (c0 + 4 c1 + c2) / 6, a1 = (c2 - c0) / 2, a2 = (c0 - 2 c1 + c2) / 2,
//   a3 = (-c0 + 3 c1 - 3 c2 + c3) / 6.
// Built once per plasma on the host (long double, one rounding per A_ji:
// cell_power_table), kCellRec doubles per cell: field slot f (kNF order 0..5)
// at f * 16, A_ji at j * 4 + i.  A field with its gradient is then 4 rows of a
// Horner value + derivative in tR (5 fma) and three Horner sums in tZ (8 fma):
// 28 fma against the stencil's 44, no basis weights; a value-only field 15
// against 20.  The same interpolant; the rounding differs from the stencil's
// by ulps (x, N ~1e-15 after 2 000 steps, tests/test_gpu_split.py).
constexpr int kCellNS = 6;
constexpr int kCellRec = kCellNS * 16;
struct CellAxis {
    int i;
    double t, delta;  // t: the offset from the cell's corner in metres
};
// axis_setup's cell, fraction (times h) and Line() distance
TORJ_HD void cell_axis(double x, double x1, double xn, double h, double invh, int n, CellAxis &a) {
    const double xc = clampd(x, x1, xn);
    a.delta = x - xc;
    const double u = (xc - x1) * invh;
    int i = (int)floor(u);
    i = i < 0 ? 0 : (i > n - 2 ? n - 2 : i);
    a.t = (u - (double)i) * h;
    a.i = i;
}
// A wave's tile of cell records staged in LDS: cells [cR0, cR0 + cw) x
// [cZ0, cZ0 + ch), R fastest; g: the whole table ((nR - 1) x (nZ - 1) cells).
// cw = 0: no tile.
struct TileCell {
    const double *g;
    const double *lds;
    int cR0, cZ0, cw, ch;
};
// one field's bicubic from its power-form record (16 coefficients in 8 pairs)
TORJ_HD void cell_field(const Dbl2 (&A)[8], double tR, double tZ, bool SLOPES, bool CROSS, double &v,
                        double &gr, double &gz, double &grz) {
    double p[4], d[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const Dbl2 lo = A[2 * j], hi = A[2 * j + 1];  // (a0, a1), (a2, a3) of row tZ^j
        // value and d/dtR by one Horner pass: p = ((a3 t + a2) t + a1) t + a0
        const double p1 = fma(hi.y, tR, hi.x);
        const double p2 = fma(p1, tR, lo.y);
        p[j] = fma(p2, tR, lo.x);
        if (SLOPES) d[j] = fma(fma(hi.y, tR, p1), tR, p2);
    }
    // over tZ: V = sum_j p_j tZ^j with dV/dtZ; d/dtR the same sum of d_j
    const double q1 = fma(p[3], tZ, p[2]);
    const double q2 = fma(q1, tZ, p[1]);
    v = fma(q2, tZ, p[0]);
    if (SLOPES) {
        gz = fma(fma(p[3], tZ, q1), tZ, q2);
        const double r1 = fma(d[3], tZ, d[2]);
        const double r2 = fma(r1, tZ, d[1]);
        gr = fma(r2, tZ, d[0]);
        if (CROSS) grz = fma(fma(d[3], tZ, r1), tZ, r2);
    }
}
// The fields' sums, each field's record read whole before its sums (208
// VGPRs; the former row-by-row form read two 16-byte pairs, waited and ran five
// fma).  A software-pipelined form that reads field f + 1's record while field
// f is summed ran the kernel alone 6 % faster (17.3 -> 16.3 ms per launch) but
// needs 234 VGPRs, and then two trajectory waves and an alpha wave no longer
// share a SIMD: the trace phase was the same.
template <int NGRAD, int NVAL, bool EXT, class P>
TORJ_HD void cell_sums(P c, const CellAxis &aR, const CellAxis &aZ, const int (&fidx)[NGRAD + NVAL],
                       double (&v)[NGRAD + NVAL], double (&gr)[NGRAD + NVAL], double (&gz)[NGRAD + NVAL],
                       double (&grz)[NGRAD + NVAL]) {
    constexpr int NT = NGRAD + NVAL;
    const double tR = aR.t, tZ = aZ.t;
    using Q = typename Pair16Ptr<P>::type;
#pragma unroll
    for (int f = 0; f < NT; f++) {
        Dbl2 A[8];
#pragma unroll
        for (int k = 0; k < 8; k++) A[k] = reinterpret_cast<Q>(c + fidx[f] * 16)[k];
        cell_field(A, tR, tZ, EXT || f < NGRAD, EXT && f < NGRAD, v[f], gr[f], gz[f], grz[f]);
    }
}
template <int NGRAD, int NVAL, bool EXT = true, int NS = kNF>
TORJ_HD void eval_fields(const TileCell &t, const Grid &g, double R, double Z,
                         const int (&fidx)[NGRAD + NVAL], FieldPack<NGRAD, NVAL> &out) {
    constexpr int NT = NGRAD + NVAL;
    CellAxis aR, aZ;
    cell_axis(R, g.R1, g.Rn, g.hR, g.invhR, g.nR, aR);
    cell_axis(Z, g.Z1, g.Zn, g.hZ, g.invhZ, g.nZ, aZ);
    const int dR = aR.i - t.cR0, dZ = aZ.i - t.cZ0;
    bool in = dR >= 0 && dR < t.cw && dZ >= 0 && dZ < t.ch;
#ifdef __HIP_DEVICE_COMPILE__
    in = __all(in);
    using LdsP = const __attribute__((address_space(3))) double *;
    using GlbP = const __attribute__((address_space(1))) double *;
#else
    using LdsP = const double *;
    using GlbP = const double *;
#endif
    double v[NT], gr[NT], gz[NT], grz[NT];
#pragma unroll
    for (int f = 0; f < NT; f++) gr[f] = gz[f] = grz[f] = 0.0;
    if (in)
        cell_sums<NGRAD, NVAL, EXT, LdsP>((LdsP)t.lds + (size_t)(dZ * t.cw + dR) * kCellRec, aR, aZ, fidx, v,
                                          gr, gz, grz);
    else
        cell_sums<NGRAD, NVAL, EXT, GlbP>((GlbP)t.g + ((size_t)aZ.i * (g.nR - 1) + aR.i) * kCellRec, aR, aZ,
                                          fidx, v, gr, gz, grz);
    fields_finish_d<NGRAD, NVAL, EXT, true>(g, aR.delta, aZ.delta, v, gr, gz, grz, out);
}
// the cell records of a plasma's node coefficients (kNF doubles per node,
// (nR + 2) x (nZ + 2) nodes) -> (nR - 1) x (nZ - 1) x kCellRec doubles
inline void cell_power_table(const double *coef, int nR, int nZ, double hR, double hZ, double *out) {
    const long double s6 = 1.0L / 6.0L;
    const long double B[4][4] = {{s6, 4 * s6, s6, 0.0L},
                                 {-0.5L, 0.0L, 0.5L, 0.0L},
                                 {0.5L, -1.0L, 0.5L, 0.0L},
                                 {-s6, 0.5L, -0.5L, s6}};
    const int mR = nR + 2;
    for (int iZ = 0; iZ < nZ - 1; iZ++)
        for (int iR = 0; iR < nR - 1; iR++)
            for (int f = 0; f < kCellNS; f++) {
                long double C[4][4];
                for (int b = 0; b < 4; b++)
                    for (int a = 0; a < 4; a++) C[b][a] = coef[((size_t)(iZ + b) * mR + iR + a) * kNF + f];
                double *o = out + ((size_t)iZ * (nR - 1) + iR) * kCellRec + f * 16;
                for (int j = 0; j < 4; j++)
                    for (int i = 0; i < 4; i++) {
                        long double acc = 0.0L;
                        for (int b = 0; b < 4; b++)
                            for (int a = 0; a < 4; a++) acc += B[j][b] * B[i][a] * C[b][a];
                        for (int k = 0; k < i; k++) acc /= (long double)hR;
                        for (int k = 0; k < j; k++) acc /= (long double)hZ;
                        o[j * 4 + i] = (double)acc;
                    }
            }
}

// Both coordinates inside the grid (no Line() extrapolation), for the whole
// wave on the device: selects the EXT = false evaluation without divergence.
TORJ_HD bool inside_grid(const Grid &g, double R, double Z) {
    const bool in = R >= g.R1 && R <= g.Rn && Z >= g.Z1 && Z <= g.Zn;
#ifdef __HIP_DEVICE_COMPILE__
    return __all(in);
#else
    return in;
#endif
}

// single value (e.g. psi for termination / deposition)
template <int NS = kNF, class CS = const double *>
TORJ_HD double eval_one(CS coef, const Grid &g, double R, double Z, int field) {
    FieldPack<0, 1> p;
    const int idx[1] = {field};
    if (inside_grid(g, R, Z))
        eval_fields<0, 1, false, NS>(coef, g, R, Z, idx, p);
    else
        eval_fields<0, 1, true, NS>(coef, g, R, Z, idx, p);
    return p.v[0];
}

// value + gradient of one field (psi gradient for the flux-surface normal,
// src/solve.jl:63)
TORJ_HD void eval_grad_one(const double *__restrict__ coef, const Grid &g, double R, double Z,
                           int field, double &v, double &dR, double &dZ) {
    FieldPack<1, 0> p;
    const int idx[1] = {field};
    // the reference calls gradient() on the extrapolated object at the point:
    // Interpolations evaluates the gradient at the clamped position.
    eval_fields<1, 0>(coef, g, clampd(R, g.R1, g.Rn), clampd(Z, g.Z1, g.Zn), idx, p);
    v = eval_one(coef, g, R, Z, field);
    dR = p.dR[0];
    dZ = p.dZ[0];
}

// ---------------------------------------------------------------------------
// dispersion: src/dispersion.jl:21-32 and its analytic partials
// ---------------------------------------------------------------------------
TORJ_HD double refractive_index_sq(double X, double Y, double Npar, int mode) {
    const double Np2 = Npar * Npar, Y2 = Y * Y;
    const double om = 1.0 - Np2;
    const double Delta = om * om + 4.0 * Np2 * (1.0 - X) / Y2;
    return 1.0 - X + (1.0 + (double)mode * sqrt(Delta) + Np2) / (2.0 * (-1.0 + X + Y2)) * X * Y2;
}

struct NsPartials {
    double Ns2, dX, dY, dNp;
};

// invY: 1 / Y when the caller has it (dispersion_grad: 1 / |B| times 1 / Cy),
// else 0 (one reciprocal here)
TORJ_HD NsPartials refractive_index_sq_partials(double X, double Y, double Npar, int mode, double invY = 0.0) {
    const double md = (double)mode;
    if (invY == 0.0) invY = rcp_nz(Y);
    const double Np2 = Npar * Npar, Y2 = Y * Y, invY2 = invY * invY;
    const double om = 1.0 - Np2, omX = 1.0 - X;
    const double Delta = om * om + 4.0 * Np2 * omX * invY2;
    // sqrt(Delta) and 1 / sqrt(Delta) from one rsqrt (Delta > 0 for X < 1);
    // at +-0 and +inf sqrt keeps its value and 1 / sqrt is NaN, as rcp_nz of it
    const double rsq = rsqrt_pos(Delta);
    double sq = Delta * rsq;
#ifdef __HIP_DEVICE_COMPILE__
    if (__builtin_amdgcn_class(Delta, 0x260)) sq = Delta;
#else
    if (Delta == 0.0 || Delta == HUGE_VAL) sq = Delta;  // the same fix-up (+-0, +inf) on the host
#endif
    const double A = 1.0 + md * sq + Np2;
    const double Q = 2.0 * (-1.0 + X + Y2);
    const double invQ = rcp_nz(Q);
    const double G = X * Y2 * invQ;
    const double dDel_dX = -4.0 * Np2 * invY2;
    const double dDel_dY = -8.0 * Np2 * omX * invY2 * invY;
    const double dDel_dNp = -4.0 * Npar * om + 8.0 * Npar * omX * invY2;
    const double h = md * 0.5 * rsq;
    const double dA_dX = h * dDel_dX, dA_dY = h * dDel_dY, dA_dNp = h * dDel_dNp + 2.0 * Npar;
    const double invQ2 = invQ * invQ;
    const double dG_dX = 2.0 * Y2 * (Y2 - 1.0) * invQ2;
    const double dG_dY = 4.0 * X * Y * (X - 1.0) * invQ2;
    NsPartials r;
    r.Ns2 = 1.0 - X + A * G;
    r.dX = -1.0 + dA_dX * G + A * dG_dX;
    r.dY = dA_dY * G + A * dG_dY;
    r.dNp = dA_dNp * G;
    return r;
}

// Plasma parameters at a point (eval_plasma, src/dispersion.jl:7-15;
// B_spline/n_e/T_e, src/plasma.jl:73-89), with the spatial derivatives the ray
// RHS needs kept in cylindrical form: the fields depend on (R, Z) only, so
// d/dx = c d/dR, d/dy = s d/dR, d/dz = d/dZ, and the rotation of B's
// components adds one tangential term (dispersion_grad).
struct PlasmaPoint {
    double X, Y, b[3], Babs, invB, B[3], ne;
    double lnTe, psi;
    double c, s, invR;         // x = R (c, s), 1 / R
    double Bc[3];              // (B_R, B_phi, B_Z)
    double dBR[3], dBZ[3];     // d/dR, d/dZ of (B_R, B_phi, B_Z)
    double dBabsR, dBabsZ;     // d|B|/dR, d|B|/dZ
    double dlnR, dlnZ;         // d ln ne / dR, d ln ne / dZ
    double Cy;                 // Y = |B| Cy
    double invCy;              // 1 / Cy
};

struct Consts {
    double Cx;  // X = ne * Cx
    double Cy;  // Y = |B| * Cy
    double invCy;
};

TORJ_HD Consts make_consts(double omega) {
    Consts c;
    c.Cx = kE * kE / (kEps0 * kMe * omega * omega);
    c.Cy = kE / (kMe * omega);
    c.invCy = (kMe * omega) / kE;
    return c;
}

// R = hypot(x, y) and 1 / R of a point (plasma_point's; the split trajectory
// kernel's step-end psi takes the same R, so psi from a stage-0 stencil and
// from eval_one at that point are the same bits)
TORJ_HD double cyl_radius(const double x[3], double &invR) {
    const double R2 = x[0] * x[0] + x[1] * x[1];
    invR = rsqrt_pos(R2);
    return R2 * invR;
}

// fields needed by the ray RHS: 4 with gradients (Br, Bphi, Bz, ln ne) + ln Te.
// WITH_PSI (the split trajectory kernel): psi as a sixth, value-only field of the
// same stencil -- the value eval_one(coef, g, R, Z, F_PSI) gives at the same
// point (the same R, the same per-field fma sequence) for 20 fma: the weights,
// the cell and the (ln Te, psi) pair loads are shared
template <bool WITH_TE, int NS = kNF, class CS = const double *, bool WITH_PSI = false>
TORJ_HD void plasma_point(CS coef, const Grid &g, const Consts &k,
                          const double x[3], PlasmaPoint &p) {
    static_assert(WITH_TE || !WITH_PSI, "psi rides with ln Te");
    double invR;
    const double R = cyl_radius(x, invR);
    const double c = x[0] * invR, s = x[1] * invR;
    constexpr int NV = WITH_TE ? (WITH_PSI ? 2 : 1) : 0;
    FieldPack<4, NV> f;
    const bool in = inside_grid(g, R, x[2]);
    if constexpr (WITH_PSI) {
        const int idx[6] = {F_BR, F_BPHI, F_BZ, F_LNNE, F_LNTE, F_PSI};
        if (in)
            eval_fields<4, 2, false, NS>(coef, g, R, x[2], idx, f);
        else
            eval_fields<4, 2, true, NS>(coef, g, R, x[2], idx, f);
        p.lnTe = f.v[4];
        p.psi = f.v[5];
    } else if constexpr (WITH_TE) {
        const int idx[5] = {F_BR, F_BPHI, F_BZ, F_LNNE, F_LNTE};
        if (in)
            eval_fields<4, 1, false, NS>(coef, g, R, x[2], idx, f);
        else
            eval_fields<4, 1, true, NS>(coef, g, R, x[2], idx, f);
        p.lnTe = f.v[4];
    } else {
        const int idx[4] = {F_BR, F_BPHI, F_BZ, F_LNNE};
        if (in)
            eval_fields<4, 0, false, NS>(coef, g, R, x[2], idx, f);
        else
            eval_fields<4, 0, true, NS>(coef, g, R, x[2], idx, f);
        p.lnTe = 0.0;
    }
    const double Br = f.v[0], Bp = f.v[1], Bz = f.v[2];
    const double Bx = Br * c - Bp * s, By = Br * s + Bp * c;
    p.c = c;
    p.s = s;
    p.invR = invR;
    p.Bc[0] = Br;
    p.Bc[1] = Bp;
    p.Bc[2] = Bz;
#pragma unroll
    for (int q = 0; q < 3; q++) {
        p.dBR[q] = f.dR[q];
        p.dBZ[q] = f.dZ[q];
    }
    p.B[0] = Bx;
    p.B[1] = By;
    p.B[2] = Bz;
    const double B2 = Bx * Bx + By * By + Bz * Bz;
    const double invB = rsqrt_pos(B2), Babs = B2 * invB;
    p.Babs = Babs;
    p.invB = invB;
    p.b[0] = Bx * invB;
    p.b[1] = By * invB;
    p.b[2] = Bz * invB;
    const double ne = exp_fast(f.v[3]);
    p.ne = ne;
    p.X = ne * k.Cx;
    p.Y = Babs * k.Cy;
    p.Cy = k.Cy;
    p.invCy = k.invCy;
    p.dlnR = f.dR[3];
    p.dlnZ = f.dZ[3];
    // d|B| = (B_cyl . dB_cyl) / |B|: |B| is axisymmetric (no tangential term)
    p.dBabsR = (Br * f.dR[0] + Bp * f.dR[1] + Bz * f.dR[2]) * invB;
    p.dBabsZ = (Br * f.dZ[0] + Bp * f.dZ[1] + Bz * f.dZ[2]) * invB;
}

// D(x,N) and its gradients (replaces ForwardDiff in gradΛ!, src/solve.jl:85-93).
// du = (dD/dN, -dD/dx) / |dD/dN|.
//
// dD/dx = -(dN_s^2/dX dX/dx + dN_s^2/dY dY/dx + dN_s^2/dN_par dN_par/dx) in
// cylindrical form.  X and Y depend on (R, Z) only; N_par = N . B / |B| with N
// held fixed, N . B = N_R B_R + N_phi B_phi + N_Z B_Z where N_R = N_x c + N_y s,
// N_phi = N_y c - N_x s turn with the point: d(N . B)/dx = c G_R + s W,
// d(N . B)/dy = s G_R - c W, d(N . B)/dz = G_Z, with G_R, G_Z the contractions
// of (N_R, N_phi, N_Z) with d/dR, d/dZ of (B_R, B_phi, B_Z) and
// W = (N_R B_phi - N_phi B_R) / R.  So every x-gradient is (c A_R + s A_W,
// s A_R - c A_W, A_Z): ~30 VALU per RHS fewer than the rotated 3 x 3 Jacobian.
TORJ_HD double dispersion_grad(const PlasmaPoint &p, const double N[3], int mode, double du[6],
                               double *Npar_out, double *inv_out = nullptr) {
    const double Npar = N[0] * p.b[0] + N[1] * p.b[1] + N[2] * p.b[2];
    const NsPartials ns = refractive_index_sq_partials(p.X, p.Y, Npar, mode, p.invB * p.invCy);
    const double N2 = N[0] * N[0] + N[1] * N[1] + N[2] * N[2];
    double dDdN[3];
#pragma unroll
    for (int q = 0; q < 3; q++) dDdN[q] = 2.0 * N[q] - ns.dNp * p.b[q];
    const double invB = p.invB;
    const double NR = N[0] * p.c + N[1] * p.s, NP = N[1] * p.c - N[0] * p.s;
    const double GR = NR * p.dBR[0] + NP * p.dBR[1] + N[2] * p.dBR[2];
    const double GZ = NR * p.dBZ[0] + NP * p.dBZ[1] + N[2] * p.dBZ[2];
    const double W = (NR * p.Bc[1] - NP * p.Bc[0]) * (p.invR * invB);
    // dN_par = (d(N . B) - N_par d|B|) / |B| (radial, vertical; tangential W)
    const double UR = (GR - Npar * p.dBabsR) * invB, UZ = (GZ - Npar * p.dBabsZ) * invB;
    const double gX = ns.dX * p.X, gY = ns.dY * p.Cy;
    const double DR = gX * p.dlnR + gY * p.dBabsR + ns.dNp * UR;
    const double DZ = gX * p.dlnZ + gY * p.dBabsZ + ns.dNp * UZ;
    const double DW = ns.dNp * W;
    const double dDdx[3] = {-(p.c * DR + p.s * DW), -(p.s * DR - p.c * DW), -DZ};
    const double inv = rsqrt_pos(dDdN[0] * dDdN[0] + dDdN[1] * dDdN[1] + dDdN[2] * dDdN[2]);
    if (inv_out) *inv_out = inv;
#pragma unroll
    for (int q = 0; q < 3; q++) {
        du[q] = dDdN[q] * inv;
        du[3 + q] = -dDdx[q] * inv;
    }
    if (Npar_out) *Npar_out = Npar;
    return N2 - ns.Ns2;
}


// ---------------------------------------------------------------------------
// Albajar absorption, src/absorption.jl:10-64, 132-226
// ---------------------------------------------------------------------------
constexpr int kMaxGL = 64;
constexpr int kSeriesFast = 16;   // Horner terms, truncation < 2^-58 rel. for arg <= 4
constexpr int kSeriesSlow = 44;   // arg <= 12
constexpr double kArgFast = 4.0;
constexpr double kArgSlow = 12.0;

constexpr double inv_fact(int k) {
    double f = 1.0;
    for (int i = 2; i <= k; i++) f *= (double)i;
    return 1.0 / f;
}
// c_nu[k] = 1/(k! (k+nu)!) : S_nu(z) = sum_k c_nu[k] z^k, J_nu(x) = (x/2)^nu S_nu(-x^2/4)
constexpr double series_coef(int nu, int k) { return inv_fact(k) * inv_fact(k + nu); }

// the default of GLTable::tiny_alpha (m^-1; torj_abs_al_init, TORJ_TINY_ALPHA)
constexpr double kTinyAlpha = 1e-20;
struct GLTable {
    int n;
    int negl_skip;  // 1: skip harmonic integrals provably below an ulp of the sum (default)
    double tiny_alpha;  // > 0: skip a harmonic whose rigorous bound on |alpha| is below it (m^-1)
    double t[kMaxGL], w[kMaxGL], st[kMaxGL], t2[kMaxGL];  // nodes, weights, sqrt(1-t^2), t^2
    // the node loop's per-node constants (pair_term), per harmonic m, one
    // 32-byte record per node (one scalar load of 8 dwords per pair): t, t^2,
    // s2 = 1 - t^2 and the weight with the Bessel argument's node factor folded
    // in, w s2^m
    struct Node {
        double t, t2, s2, wm;
    } nd[2][kMaxGL];
};
// the node records of node i from its t and w (host, at abs_Al_init), in long
// double so that each folded weight is rounded once
inline void gl_node_consts(GLTable &g, int i) {
    const long double t = g.t[i], s2 = 1.0L - t * t, w = g.w[i];
    for (int m = 2; m <= 3; m++) {
        GLTable::Node &q = g.nd[m - 2][i];
        q.t = g.t[i];
        q.t2 = g.t[i] * g.t[i];
        q.s2 = (double)s2;
        q.wm = (double)(m == 2 ? w * s2 * s2 : w * s2 * s2 * s2);
    }
}

#ifndef TORJ_ALBAJAR_NOINLINE
#define TORJ_ALBAJAR_NOINLINE 1
#endif

// Horner evaluation of S_nu and S_{nu+1} at z with K terms; coefficients are
// compile-time immediates (one v_fma_f64 each, constant operand in SGPRs).
template <int K, int NU>
TORJ_HD void series_pair(double z, double &Sa, double &Sb) {
    double a = series_coef(NU, K - 1), b = series_coef(NU + 1, K - 1);
#pragma unroll
    for (int k = K - 2; k >= 0; k--) {
        a = fma(a, z, series_coef(NU, k));
        b = fma(b, z, series_coef(NU + 1, k));
    }
    Sa = a;
    Sb = b;
}

// Slow path (arg > 4, unphysical for |N| <= 1): rolled loop over a
// constant-memory coefficient table so it costs no registers in the hot path.
constexpr int kSeriesMax = kSeriesSlow;
struct SeriesTable {
    double c[3][kSeriesMax];
};
constexpr SeriesTable make_series_table() {
    SeriesTable t{};
    for (int nu = 2; nu <= 4; nu++)
        for (int k = 0; k < kSeriesMax; k++) t.c[nu - 2][k] = series_coef(nu, k);
    return t;
}
#ifdef __HIP_DEVICE_COMPILE__
__constant__ constexpr SeriesTable kSeriesTab = make_series_table();
#else
constexpr SeriesTable kSeriesTab = make_series_table();
#endif

template <int NU>
TORJ_HD void series_pair_loop(double z, double &Sa, double &Sb) {
    const double *ca = kSeriesTab.c[NU - 2], *cb = kSeriesTab.c[NU - 1];
    double a = ca[kSeriesSlow - 1], b = cb[kSeriesSlow - 1];
#pragma unroll 1
    for (int k = kSeriesSlow - 2; k >= 0; k--) {
        a = fma(a, z, ca[k]);
        b = fma(b, z, cb[k]);
    }
    Sa = a;
    Sb = b;
}

#ifdef TORJ_ALPHA_PROF
// profiling build only (tools/alpha_prof.py): [2 (m - 2)] waves and [2 (m - 2) + 1]
// lanes that ran harmonic m's node loop, [4] waves and [5] live lanes of k_alpha_pts;
// [6 ..] waves that reached a region of abs_albajar_fast_body (kAprof*)
enum { kAprofTe = 6, kAprofPro, kAprofOk, kAprofH2, kAprofB2, kAprofH3, kAprofB3, kAprofZ, kAprofN = 14 };
#ifdef TORJ_TRAJ_TU
static
#endif
__device__ unsigned long long g_aprof[16];
#if defined(__HIP_DEVICE_COMPILE__)
#define TORJ_APROF_WAVE(K)                                                          \
    do {                                                                            \
        const unsigned long long am_ = __ballot(1);                                 \
        if ((int)__lane_id() == __builtin_ffsll((long long)am_) - 1) atomicAdd(&g_aprof[K], 1ull); \
    } while (0)
#endif
#endif
#ifndef TORJ_APROF_WAVE
#define TORJ_APROF_WAVE(K) \
    do {                   \
    } while (0)
#endif

// Per-harmonic constants of the node sum (abs_Al_pol_fact / abs_Al_integral_nume_fast)
struct HarmConst {
    double x_m, K0, K1, K2, K3, K4, K5, upa0, upa1, r2m1, mu;
    double mu2;  // mu log2(e): the node exponent in base 2 (exp2_node)
    // node-pair form: gamma_pm^2 = C0 + C1 t^2 pm C2 t, h = hx sqrt(1-t^2)
    double C0, C1, C2, hx;
    double Y0, Y1;  // node exponents mu log2(e) (1 - gamma(+-t)) = Y0 -+ Y1 t (TORJ_NODE_GAMMA_LIN)
    double hx2, K1h, K5h;  // hx^2, K1 / hx = 2 Axz ea / m, K5 / hx = 2 q ea e3 / m (pair_term)
};

// A symmetric pair of Gauss-Legendre nodes (+t, -t): w * pol_fact * exp(mu (1 -
// gamma)) summed over both, without the node-independent factor (-mu) (m / (N_perp
// omega_bar))^2.  GL nodes are symmetric with equal weights, and the Bessel
// argument x_m sqrt(1-t^2) is even in t, so the Bessel factors (2 Horner series
// S_m, S_{m+1} of K terms + the downward recurrence S_{m-1} = m S_m + z S_{m+1})
// are computed once per pair.  With `single`, only the +t node is taken (the
// middle node of an odd-order rule, t = 0).
#ifndef TORJ_PAIR_UNROLL
#define TORJ_PAIR_UNROLL 1
#endif
#ifndef TORJ_NODE_GAMMA_LIN  // the node loop's gamma as the resonance condition's linear form
// G0 +- G1 t (1, round 6) or as the reference's sqrt(1 + u_par^2 + u_perp^2) (0; harm_geom)
#define TORJ_NODE_GAMMA_LIN 1
#endif

// Series coefficients of one harmonic for the node loop (compile-time
// constants: the Horner FMAs take them as SGPR operands).
// LV 0..3: the near-minimax polynomials of torj_bessel_coefs.hpp on x_m <= 1, 2,
// 3, 4 (7 / 9 / 10 / 11 terms, as accurate as the 9 / 12 / 14 / 16-term Taylor
// series they replaced); LV 4: the 44-term Taylor loop (x_m <= 12).
constexpr int series_terms(int lv) { return lv >= 4 ? 0 : kBesselTerms[lv]; }
constexpr double level_coef(int lv, int nu, int k) { return kBesselCoef[lv][nu - 2][k]; }

template <int M, int LV>
struct SeriesCoefs {
    static constexpr int K = series_terms(LV);
    double a[K > 0 ? K : 1], b[K > 0 ? K : 1];
    TORJ_HD void load() {
        if constexpr (K > 0) {
#pragma unroll
            for (int k = 0; k < K; k++) {
                a[k] = level_coef(LV, M, k);
                b[k] = level_coef(LV, M + 1, k);
            }
        }
    }
    TORJ_HD void eval(double z, double &Sa, double &Sb) const {
        if constexpr (K > 0) {
            double x = a[K - 1], y = b[K - 1];
#pragma unroll
            for (int k = K - 2; k >= 0; k--) {
                x = fma(x, z, a[k]);
                y = fma(y, z, b[k]);
            }
            Sa = x;
            Sb = y;
        } else {
            series_pair_loop<M>(z, Sa, Sb);
        }
    }
};


// The two nodes of a pair share every t-even factor.  With
//   bracket(+-t) = P +- t Q,  P = A (K0 + K3 t^2) - B + Cc K1,  Q = A K4 + Cc K5
//   gamma(+-t)^2 = (u_par0 +- u_par1 t)^2 + 1 + (r^2-1)(1-t^2) = C0 + C1 t^2 +- C2 t
// the pair contributes w h^(2m-1) [P (E+ + E-) + t Q (E+ - E-)], E = exp(mu (1 - gamma))
// -- the same sum as abs_Al_pol_fact x abs_Al_integral_nume_fast's node terms
// (src/absorption.jl:132-189), regrouped.  With h = hx st (st = sqrt(1 - t^2)),
// A = h S_m^2, B = K2 h^2 S_{m-1} h S_{m+1}, Cc = st S_m D = (h / hx) S_m D,
// D = S_{m-1} - h^2 S_{m+1}, every term of P and Q carries one factor h, so
//   w h^(2m-1) [..] = hx^(2m) (w s2^m) [P' (E+ + E-) + t Q' (E+ - E-)],
//   P' = S_m^2 (K0 + K3 t^2) - K2 S_{m-1} u + (K1 / hx) S_m D,  u = h^2 S_{m+1},
//   Q' = K4 S_m^2 + (K5 / hx) S_m D,
// with s2 = 1 - t^2 and w s2^m per node (GLTable), K1 / hx and K5 / hx per
// harmonic (no quotient: K1 and K5 carry a factor x_m = 2 hx), and hx^(2m)
// applied once to the sum (albajar_harmonic): 25 VALU per pair besides the
// series, square roots and exponentials, against 34 for the direct form.
template <int M, int LV>
TORJ_HD double pair_term(const HarmConst &c, const SeriesCoefs<M, LV> &sc, double t, double s2,
                         double W, double t2, bool single) {
    constexpr double md = (double)M;
    const double h2 = c.hx2 * s2;  // (x_m sqrt(1 - t^2) / 2)^2, the series' -z
    double Sm, Sm1;
    sc.eval(-h2, Sm, Sm1);
    const double u = h2 * Sm1;
    const double Sl = fma(md, Sm, -u);  // S_{m-1} by the downward recurrence
    const double D = Sl - u;
    const double Sm2 = Sm * Sm, SmD = Sm * D;
    const double P = fma(Sm2, fma(c.K3, t2, c.K0), fma(c.K1h, SmD, -(c.K2 * (Sl * u))));
#if TORJ_NODE_GAMMA_LIN
    // gamma(+-t) = G0 +- G1 t on the resonance ellipse (harm_geom): the node
    // exponents are two fma, no square root
    if (single) return W * (P * exp2_node(c.Y0));
    const double Q = fma(c.K4, Sm2, c.K5h * SmD);
    const double Ep = exp2_node(fma(-c.Y1, t, c.Y0));
    const double Em = exp2_node(fma(c.Y1, t, c.Y0));
#else
    const double a = fma(c.C1, t2, c.C0);
    if (single) return W * (P * exp2_node(fma(-c.mu2, sqrt_node(a), c.mu2)));
    const double Q = fma(c.K4, Sm2, c.K5h * SmD);
    const double b = c.C2 * t;
    const double Ep = exp2_node(fma(-c.mu2, sqrt_node(a + b), c.mu2));
    const double Em = exp2_node(fma(-c.mu2, sqrt_node(a - b), c.mu2));
#endif
    return W * fma(P, Ep + Em, (t * Q) * (Ep - Em));
}

template <int M, int LV, int LPR = 1, int U = TORJ_PAIR_UNROLL>
TORJ_HD double node_sum(const GLTable &gl, const HarmConst &c, int sub = 0) {
    SeriesCoefs<M, LV> sc;
    sc.load();
    const int n = gl.n, half = n >> 1;
    const GLTable::Node *nd = gl.nd[M - 2];
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr (LPR > 1) {
        // LPR lanes per ray (small beams, latency-bound): lane `sub` of the ray's
        // group takes pairs sub, sub + LPR, ...; the group then adds the pair
        // terms in the one-lane order 0, 1, 2, ... (each from its lane): every
        // lane of the group holds the same sum, as LPR = 1 would compute it for
        // the same polynomial length (chosen per wave, so it can differ)
        constexpr int Q = (kMaxGL / 2 + LPR - 1) / LPR;
        double rr[Q];
#pragma unroll
        for (int q = 0; q < Q; q++) {
            rr[q] = 0.0;
            const int i = q * LPR + sub;
            if (q * LPR < half && i < half)
                rr[q] = pair_term<M, LV>(c, sc, nd[i].t, nd[i].s2, nd[i].wm, nd[i].t2, false);
        }
        const int base = (int)(threadIdx.x & 63u) & ~(LPR - 1);
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < Q; q++) {
            if (q * LPR >= half) break;
#pragma unroll
            for (int u = 0; u < LPR; u++) {
                const double v = __shfl(rr[q], base + u, 64);
                if (q * LPR + u < half) s += v;
            }
        }
        if (n & 1) s += pair_term<M, LV>(c, sc, nd[half].t, nd[half].s2, nd[half].wm, nd[half].t2, true);
        return s;
    }
#endif
    double acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = 0.0;
    // U independent node pairs per iteration (ILP for the dependent fp64
    // chains); each pair's four constants are one 32-byte record (one scalar
    // load, uniform across the wave; a look-ahead load of the next record,
    // consumed at the end of the iteration, is scheduled late by the compiler
    // anyway, and the other waves of the SIMD cover the latency)
    int i = 0;
#pragma unroll 1
    for (; i + U <= half; i += U) {
        double r[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const GLTable::Node q = nd[i + u];
            r[u] = pair_term<M, LV>(c, sc, q.t, q.s2, q.wm, q.t2, false);
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] += r[u];
    }
    // the remainder pairs (none when U = 1: the compiler still materialised the
    // pair's constants for this loop's preheader, ~67 SALU per node loop)
    if constexpr (U > 1) {
#pragma unroll 1
        for (; i < half; i++) acc[0] += pair_term<M, LV>(c, sc, nd[i].t, nd[i].s2, nd[i].wm, nd[i].t2, false);
    }
    if (n & 1) acc[0] += pair_term<M, LV>(c, sc, nd[half].t, nd[half].s2, nd[half].wm, nd[half].t2, true);
    double s = acc[0];
#pragma unroll
    for (int u = 1; u < U; u++) s += acc[u];
    return s;
}

// The geometry of harmonic m's resonance ellipse that needs no polarisation:
// gamma(t)^2 = C0 + C1 t^2 +- C2 t over the node pairs, gamma_min^2 = qmin, and
// whether the whole node sum underflows to an exact zero (albajar_harmonic).
// Depends on (mu, r = m / m_0, N_par) only, so abs_albajar_fast_body computes it
// before the polarisation vector and can settle alpha = 0 there.
struct HarmGeom {
    double r, r2m1, sq_r, upa0, upa1, C0, C1, C2, qmin;
    double Y0, Y1, ymax;  // TORJ_NODE_GAMMA_LIN: node exponents Y0 -+ Y1 t, their bound
    bool zero;
};

TORJ_HD HarmGeom harm_geom(double mu, double inv_mu, double r, double Npar, double inv_sqNp) {
    HarmGeom g;
    g.r = r;
    g.r2m1 = r * r - 1.0;
    g.sq_r = sqrt_nn(g.r2m1);
    g.upa0 = inv_sqNp * r * Npar;
    g.upa1 = inv_sqNp * g.sq_r;
#if TORJ_NODE_GAMMA_LIN
    // The ellipse is the square of the resonance condition gamma = m Y + N_par u_par
    // (src/absorption.jl:176-179 parametrise it by u_par = upa0 + upa1 t and
    // u_perp^2 = (r^2 - 1)(1 - t^2)), and with m Y = r sqrt(1 - N_par^2) that is
    //   gamma(t) = G0 + G1 t,  G0 = r / sqrt(1 - N_par^2),  G1 = N_par upa1,
    // positive over the whole ellipse (|N_par| < 1 and sqrt(r^2 - 1) < r): the
    // value of the reference's sqrt(1 + u_par^2 + u_perp^2) without the square
    // root, both forms within a few ulp of the exact gamma.  In base 2 the node
    // exponent mu log2(e) (1 - gamma(+-t)) is Y0 -+ Y1 t; its largest value over
    // |t| <= 1 is ymax = Y0 + |Y1| (gamma_min = G0 - |G1|: gamma is monotone in t).
    const double mu2 = mu * 1.4426950408889634074;
    g.Y0 = fma(-mu2, r * inv_sqNp, mu2);
    g.Y1 = mu2 * (Npar * g.upa1);
    g.ymax = g.Y0 + fabs(g.Y1);
    // Exact zero: every node's 2^y underflows to +0 (exp2_node returns exactly 0
    // below y = -1076) when ymax < -1096 -- round 3's mu (gamma_min - 1) > 760 in
    // base 2, whose margin covers the roundings of ymax and of each node's y (a
    // few 1e-13).  Then the node sum is +-0 and the loop is skipped with the same
    // value; NaN operands never skip.
    g.zero = g.ymax < -1096.0;
    g.C0 = g.C1 = g.C2 = g.qmin = 0.0;  // (the square-root form's, unused)
    (void)inv_mu;
#else
    g.Y0 = g.Y1 = g.ymax = 0.0;
    g.C0 = fma(g.upa0, g.upa0, r * r);
    g.C1 = g.r2m1 * (Npar * Npar) * (inv_sqNp * inv_sqNp);  // u_par1^2 - (r^2 - 1)
    g.C2 = 2.0 * g.upa0 * g.upa1;
    // Exact zero: every node's exp(mu (1 - gamma)) underflows to +0 (exp_fast
    // returns exactly 0 below -746) when mu (gamma_min - 1) exceeds 760, gamma_min
    // the least gamma(t) = sqrt(C0 + C1 t^2 + C2 t) over t in [-1, 1] (a bound
    // for every node of both signs, the vertex of the parabola or an end); the
    // margin of 14 covers the rounding of gamma^2 and mu (1 - gamma).  Then every
    // pair term is w p (P (0 + 0) + t Q (0 - 0)) = +-0 and the node sum is +-0:
    // the loop is skipped with the same value (the sign of a zero aside, which
    // no later operation sees) -- far from the resonance that is most of the
    // third harmonic's evaluations on a beam.  NaN operands never skip.
    const double qe = fma(g.C1, 1.0, g.C0) - fabs(g.C2);  // min of the ends t = -1, 1
    const double tv = -g.C2 * 0.5 * rcp_nz(g.C1);          // vertex (C1 > 0)
    const double qv = fma(-0.25 * g.C2, g.C2 * rcp_nz(g.C1), g.C0);
    g.qmin = (g.C1 > 0.0 && fabs(tv) <= 1.0) ? qv : qe;
    // mu (sqrt(qmin) - 1) > 760 as qmin > (1 + 760 / mu)^2 (no square root;
    // the threshold's few roundings are ~1e-15 of it, inside the margin of 14)
    const double th = fma(760.0, inv_mu, 1.0);
    g.zero = g.qmin > 1.0 && g.qmin > th * th;
#endif
    return g;
}


// Work counters of one lane (include/torj_hip.h torj_trace: counters[2..7]).
// Albajar (ABS 1) / warm weakly relativistic (ABS 2, torj_warm.hpp) meaning:
struct AlbajarWork {
    uint32_t n_active;  // calls that reached the harmonic loop / larmornumber tests
    uint32_t n_harm;    // harmonic integrals evaluated (node loop run) / Faddeeva evaluations
    uint32_t n_terms;   // Bessel-series terms (sum over node pairs of K) / warmdisp passes
    uint32_t n_zero;    // harmonic integrals found exactly zero / passes x Larmor order
    uint32_t n_l;       // - / sum of Larmor orders lrm
    uint32_t n_l2;      // - / sum of lrm^2
    uint32_t n_negl;    // harmonic integrals skipped as below an ulp of the sum / -
    uint32_t n_early;   // exact-zero harmonics of calls settled before the polarisation vector / -
};

// Resonance-ellipse integral for harmonic m (abs_Al_integral_nume_fast +
// abs_Al_pol_fact) times sqrt((m/m_0)^2 - 1), WITHOUT the Maxwellian
// normalisation a*(mu/2pi)^1.5 (common to both harmonics).
template <int M, int LPR = 1, int U = TORJ_PAIR_UNROLL>
TORJ_HD double albajar_harmonic(const GLTable &gl, double mu, const HarmGeom &hg,
                                double inv_sqNp, double N_perp, double omega_bar,
                                double Axz, double ea, double e3, AlbajarWork *work, int sub = 0,
                                double dom = 0.0, double hmax = 0.0) {
    constexpr double md = (double)M, inv_md = 1.0 / md;
    HarmConst c;
    c.r2m1 = hg.r2m1;
    const double sq_r = hg.sq_r;
    c.x_m = N_perp * omega_bar * sq_r;
    const double q = c.x_m * inv_sqNp * inv_md;  // x_m / (m sqrt(1 - N_par^2))
    c.K0 = Axz * Axz + ea * ea;
    c.K1 = Axz * ea * c.x_m * inv_md;
    c.K2 = 4.0 * ea * ea * (inv_md * inv_md);
    c.K3 = q * q * e3 * e3;
    c.K4 = 2.0 * q * Axz * e3;
    c.K5 = q * ea * e3 * c.x_m * inv_md;
    c.K1h = 2.0 * Axz * ea * inv_md;     // K1 / hx
    c.K5h = 2.0 * q * ea * e3 * inv_md;  // K5 / hx
    c.upa0 = hg.upa0;
    c.upa1 = hg.upa1;
    c.mu = mu;
    c.mu2 = mu * 1.4426950408889634074;
    c.C0 = hg.C0;
    c.C1 = hg.C1;
    c.C2 = hg.C2;
    c.Y0 = hg.Y0;
    c.Y1 = hg.Y1;
    c.hx = 0.5 * c.x_m;
    c.hx2 = c.hx * c.hx;
    const double qmin = hg.qmin;
    const bool zero = hg.zero;  // the exact-zero bound (harm_geom)
    // Bessel polynomial from the largest argument x_m (SeriesCoefs: x_m <= 1,
    // 2, 3, 4, each within a few ulp of mpmath's J_nu, checked in tests; the
    // 44-term Taylor loop beyond); physical rays have x_m < m.  The level is made
    // wave-uniform (max over the active lanes) so the node loop does not diverge.
    int level = c.x_m <= 1.0 ? 0 : (c.x_m <= 2.0 ? 1 : (c.x_m <= 3.0 ? 2 : (c.x_m <= kArgFast ? 3 : 4)));
    if (zero) level = 0;  // a skipping lane does not raise the wave's polynomial length
#ifdef __HIP_DEVICE_COMPILE__
    level = __ballot(level == 4) ? 4 : (__ballot(level == 3) ? 3 : (__ballot(level == 2) ? 2 : (__ballot(level == 1) ? 1 : 0)));
#endif
    const double den = N_perp * omega_bar;
    const double Pm = den == 0.0 ? INFINITY : md * rcp_nz(den);
    if (zero) {
        if (work) work->n_zero++;
        return -mu * Pm * Pm * 0.0 * sq_r;
    }
    TORJ_APROF_WAVE(M == 2 ? kAprofH2 : kAprofH3);
    // Negligible next to the harmonics already summed (dom = their sum so far,
    // abs_albajar_fast_body adds this one to it next): when a rigorous bound B
    // on |this integral| is below 2^-58 |dom|, dom + h rounds to dom exactly
    // (|h| < ulp(dom) / 4 with a 16x margin for B's own rounding and the node
    // loop's ~1e-13), so the node loop is skipped and alpha is bit-identical.
    // Far below the resonance of a higher harmonic its Maxwellian factor
    // exp(mu (1 - gamma)) is e^-40 .. e^-760 of the lower one's: most third-
    // harmonic integrals beside a second one.  B: |J_nu(x)| <= (x/2)^nu / nu!
    // bounds |S_m|, |S_{m+1}|, |S_{m-1}| by 1/nu!; with h <= hx, |t| <= 1,
    // every node's E <= E_max = exp(mu (1 - gamma_min)) and sum_i w_i = 2,
    // |node sum| <= 4 E_max hx^(2m-1) (Pmax + Qmax).  The level ballot above
    // already counted this lane, so the other lanes' polynomials do not change.
    //
    // Below any absorption a result can show (hmax > 0, GLTable::tiny_alpha):
    // the same bound B E_max on |this integral|, times the normalisation
    // albajar_finish applies, is an upper bound on the harmonic's share of
    // alpha; when it is below tiny_alpha (m^-1) the node loop is skipped.  Not
    // bit-identical: alpha moves by less than tiny_alpha per skipped harmonic,
    // tau by less than 2 tiny_alpha per metre of ray.
    const bool rel = gl.negl_skip && dom != 0.0 && fabs(dom) < INFINITY && fabs(dom) > 1e-290;
    if (rel || hmax > 0.0) {
        TORJ_APROF_WAVE(M == 2 ? kAprofB2 : kAprofB3);
        constexpr double iS = inv_fact(M), iS1 = inv_fact(M + 1), iSl = inv_fact(M - 1);
        const double hx = c.hx, hx2 = hx * hx;
        const double A = hx * (iS * iS), T1 = hx2 * iS1;
        const double Bv = fabs(c.K2) * iSl * hx * T1, Cc = iS * (iSl + T1);
        const double Pmax = A * (fabs(c.K0) + fabs(c.K3)) + Cc * fabs(c.K1) + Bv;
        const double Qmax = A * fabs(c.K4) + Cc * fabs(c.K5);
        double p = hx;  // hx^(2m-1)
#pragma unroll
        for (int k = 1; k < 2 * M - 1; k++) p *= hx;
        const double B0 = 4.0 * mu * (Pm * Pm) * sq_r * p * (Pmax + Qmax);
        const double R = B0 * rcp_nz(fabs(dom));
#if TORJ_NODE_GAMMA_LIN
        // E_max <= 2^(ceil(ymax) + 1): every node's y is at most ymax up to its
        // roundings (a few 1e-13), the extra factor 2 covers them and exp2_node's
        // 4e-12; a NaN ymax gives an infinite bound, which never skips
        const double yb = ceil(hg.ymax) + 1.0;
        const double Emax = ldexp_i(1.0, (int)fmax(fmin(yb, 2000.0), -2000.0));
        (void)qmin;
#elif TORJ_EMAX_BOUND
        // an upper bound on E_max = exp(mu (1 - gamma_min)) without the exponential:
        // 2^(ceil(y) + 1) with y = mu log2(e) (1 - gamma_min) from the node loop's
        // square root (a few ulp; the extra factor 2 covers y's rounding, |y| <
        // 2^16), so the bound stays rigorous with at most 4x of slack; a NaN y
        // gives an infinite bound (fmin / fmax return the non-NaN operand), which
        // never skips
        const double yb = ceil(c.mu2 * (1.0 - sqrt_node(qmin))) + 1.0;
        const double Emax = ldexp_i(1.0, (int)fmax(fmin(yb, 2000.0), -2000.0));
#else
        const double Emax = exp_fast<true>(mu * (1.0 - sqrt_nn(qmin)));
#endif
        // R, B0 < 1e300: an E_max that underflowed to 0 cannot hide a huge bound
        if ((rel && R < 1e300 && R * Emax < 0x1p-58) || (B0 < 1e300 && B0 * Emax < hmax)) {
            if (work) work->n_negl++;
            return 0.0;
        }
    }
#if defined(TORJ_ALPHA_PROF) && defined(__HIP_DEVICE_COMPILE__)
    {  // profiling build only: node loops run per wave and per lane (lane utilisation)
        const unsigned long long am = __ballot(1);
        if ((int)__lane_id() == __builtin_ffsll((long long)am) - 1) {
            atomicAdd(&g_aprof[2 * (M - 2)], 1ull);
            atomicAdd(&g_aprof[2 * (M - 2) + 1], (unsigned long long)__popcll(am));
        }
    }
#endif
    if (work) {
        constexpr int kTerms[5] = {series_terms(0), series_terms(1), series_terms(2), series_terms(3),
                                   kSeriesSlow};
        work->n_terms += (uint32_t)(kTerms[level] * ((gl.n + 1) >> 1));
    }
    double sum;
    switch (level) {
        case 0: sum = node_sum<M, 0, LPR, U>(gl, c, sub); break;
        case 1: sum = node_sum<M, 1, LPR, U>(gl, c, sub); break;
        case 2: sum = node_sum<M, 2, LPR, U>(gl, c, sub); break;
        case 3: sum = node_sum<M, 3, LPR, U>(gl, c, sub); break;
        default: sum = node_sum<M, 4, LPR, U>(gl, c, sub); break;
    }
    // hx^(2m), the node loop's common factor (pair_term)
    double hx2m = c.hx2;
#pragma unroll
    for (int k = 1; k < M; k++) hx2m *= c.hx2;
    sum *= hx2m;
    // (m / (N_perp omega_bar))^2 with Pm from a reciprocal (<= 1 ulp); N_perp = 0
    // (parallel propagation) stays an infinity as in the reference's quotient
    return -mu * Pm * Pm * sum * sq_r;
}

// abs_Albajar_fast (src/absorption.jl:191-226).  With TORJ_ALBAJAR_NOINLINE the
// device code keeps it out of line: the RK4 state is then saved once per call
// instead of competing for registers inside the node loop.
//
// Restated for the device (same quantities, fewer instructions):
//  * sin(acos(cos_t)) is sqrt(1 - cos_t^2) (an fma and a sqrt instead of the
//    acos and sin library sequences; NaN for |cos_t| > 1 as in the reference,
//    Appendix A.4);
//  * quotients by Te, Y, N_abs, Nt, den, sqrt(1 - N_par^2) and the Maxwellian
//    normalisation use rcp_nz (one reciprocal each, reused), 1/mu = Te e/(m c^2);
//  * 1 / m_0 = Y / sqrt(1 - N_par^2), 1/(Y c) folded into one product.
#if defined(__HIP_DEVICE_COMPILE__) && TORJ_ALBAJAR_NOINLINE
#define TORJ_ALB_ATTR __host__ __device__ __attribute__((noinline))
#else
#define TORJ_ALB_ATTR TORJ_HD
#endif
// The prologue of abs_Albajar_fast: everything the harmonic integrals and the
// final normalisation need.  ok = false: alpha is 0 (the reference's early
// returns, src/absorption.jl:191-212).
struct AlbPro {
    bool ok;
    double inv_mu, mu, omega_bar, N_perp, inv_sqNp, Axz, ea, e3, m_0, inv_m0;
};

// The polarisation-free part of the prologue (Te >= 20): what the harmonics'
// resonance geometry (harm_geom) needs, computed before the polarisation vector.
struct AlbPre {
    double inv_mu, mu, omega_bar, N_perp, sqNp, m_0, inv_sqNp, inv_m0;
};
TORJ_HD AlbPre albajar_pre(double Y, double N_abs, double N_par, double Te) {
    AlbPre p;
    constexpr double kMuTe = kMe * kC * kC / kE;  // mu Te
    p.inv_mu = Te * (1.0 / kMuTe);
    p.mu = kMuTe * rcp_nz(Te);
    p.omega_bar = rcp_nz(Y);
    p.N_perp = sqrt_nn(N_abs * N_abs - N_par * N_par);
    const double omNp2 = 1.0 - N_par * N_par;
    p.sqNp = sqrt_nn(omNp2);
    p.m_0 = p.sqNp * p.omega_bar;
    p.inv_sqNp = rsqrt_pos(omNp2);  // NaN where rcp_nz(sqNp) is (1 - N_par^2 <= 0, NaN)
    p.inv_m0 = p.inv_sqNp * Y;
    return p;
}

TORJ_HD AlbPro albajar_prologue(const AlbPre &pre, double X, double Y, double N_abs, double N_par,
                                int mode) {
    AlbPro q;
    q.ok = false;
    q.inv_mu = pre.inv_mu;
    q.mu = pre.mu;
    const double omega_bar = pre.omega_bar;
    q.omega_bar = omega_bar;
    const double cos_t = N_par * rcp_nz(N_abs);
    const double sin_t = sqrt_nn(fma(-cos_t, cos_t, 1.0));
    const double N_perp = pre.N_perp;
    q.N_perp = N_perp;
    // abs_Al_N_with_pol_vec (src/absorption.jl:10-64), real form:
    // e = (e1, i*ea, e3) with e1, ea, e3 real.
    if (X >= 1.0) return q;
    const double s2 = sin_t * sin_t, c2 = cos_t * cos_t, omX = 1.0 - X;
    const double Y2 = Y * Y, invY2 = omega_bar * omega_bar;
    double rho = Y2 * (s2 * s2) + 4.0 * omX * omX * c2;
    if (rho < 0.0) return q;
    rho = sqrt_nn(rho);
    const double f = (2.0 * omX) * rcp_nz(2.0 * omX - Y2 * s2 - (double)mode * Y * rho);
    double Nt = 1.0 - X * f;
    if (Nt < 0.0) return q;
    Nt = sqrt_nn(Nt);
    if (!(Nt > 0.0) || Nt > 1.0) return q;  // isnan || <= 0 || > 1
    const double inv_Nt = rcp_nz(Nt);
    const double g = 1.0 - (1.0 - Y2) * f;
    double e1 = 0.0, ea = 0.0, e3 = 0.0;
    if (c2 < 1e-5 || 1.0 - s2 < 1e-5) {
        if (mode > 0) {
            ea = sqrt_pos(inv_Nt);
            e1 = -(omega_bar * g) * ea;
        } else {
            e3 = sqrt_pos(inv_Nt);
        }
    } else {
        const double Nt2 = Nt * Nt;
        const double den = omX - Nt2 * s2;
        const double inv_den = rcp_nz(den);
        const double gg = invY2 * (g * g);
        const double ta = 1.0 + (omX * Nt2 * c2) * (inv_den * inv_den) * gg;
        const double tb = 1.0 + (omX * inv_den) * gg;
        const double a_sq = s2 * (ta * ta), b_sq = c2 * (tb * tb);
        ea = sqrt_pos(inv_Nt * rsqrt_pos(a_sq + b_sq));
        if (mode <= 0) ea = -ea;
        e1 = -(omega_bar * g) * ea;
        e3 = -((Nt2 * sin_t * cos_t) * inv_den) * e1;
    }
    q.m_0 = pre.m_0;
    q.inv_sqNp = pre.inv_sqNp;
    const double N_eff = (N_perp * N_par) * (q.inv_sqNp * q.inv_sqNp);
    q.Axz = e1 + N_eff * e3;
    q.ea = ea;
    q.e3 = e3;
    q.inv_m0 = pre.inv_m0;
    q.ok = true;
    return q;
}

// harmonic m of the sum (src/absorption.jl:213-223), if m >= m_0 (NaN m_0: no
// harmonic, as the reference's `m < m_0` test makes it)
template <int M, int LPR = 1, int U = TORJ_PAIR_UNROLL>
TORJ_HD double albajar_pro_harmonic(const GLTable &gl, const AlbPro &q, const HarmGeom &hg,
                                    AlbajarWork *work, int sub = 0, double dom = 0.0,
                                    double hmax = 0.0) {
    const uint32_t z0 = work ? work->n_zero + work->n_negl : 0u;
    const double h = albajar_harmonic<M, LPR, U>(gl, q.mu, hg, q.inv_sqNp, q.N_perp, q.omega_bar,
                                                 q.Axz, q.ea, q.e3, work, sub, dom, hmax);
    if (work && work->n_zero + work->n_negl == z0) work->n_harm++;
    return h;
}

// the Maxwellian normalisation and units (src/absorption.jl:224-226)
TORJ_HD double albajar_finish(const AlbPro &q, double c_abs, double X, double omega) {
    // 1 / (1 + 105/(128 mu^2) + 15/(8 mu)), (mu / 2 pi)^1.5
    const double a = rcp_nz(fma(q.inv_mu, fma(q.inv_mu, 105.0 / 128.0, 15.0 / 8.0), 1.0));
    const double sm = sqrt_pos(q.mu * (1.0 / (2.0 * kPi)));
    c_abs *= a * (sm * sm * sm);
    c_abs = -(c_abs * (2.0 * kPi * kPi) * q.inv_m0);
    return c_abs * X * omega * (q.omega_bar * (1.0 / kC));
}

// The largest harmonic integral (albajar_harmonic's units) whose share of alpha
// is provably below gl.tiny_alpha: tiny_alpha over an upper bound on the
// normalisation albajar_finish multiplies the sum by (its a <= 1 for mu > 0,
// (mu / 2 pi)^1.5 from a reciprocal square root, and a factor 1/2 for the
// roundings of this bound); 0 (no skip) when off or not finite.
TORJ_HD double tiny_harmonic(double tiny_alpha, const AlbPro &q, double X, double omega) {
    if (!(tiny_alpha > 0.0)) return 0.0;
    const double m = q.mu * (1.0 / (2.0 * kPi));
    const double F = fabs((2.0 * kPi * kPi) * q.inv_m0 * X * omega * (q.omega_bar * (1.0 / kC)) * m);
    const double h = 0.5 * tiny_alpha * rcp_nz(F) * rsqrt_pos(m);
    return h < INFINITY ? h : 0.0;
}

template <int LPR = 1, int U = TORJ_PAIR_UNROLL>
TORJ_HD double abs_albajar_fast_body(const GLTable &gl, double omega, double X, double Y,
                                     double N_abs, double N_par, double Te, int mode,
                                     AlbajarWork *work, int sub = 0, double tiny = 0.0) {
    if (Te < 20.0) return 0.0;
    TORJ_APROF_WAVE(kAprofTe);
    const AlbPre pre = albajar_pre(Y, N_abs, N_par, Te);
    const bool h2 = !(2.0 < pre.m_0), h3 = !(3.0 < pre.m_0);  // harmonic m present iff m >= m_0
    HarmGeom g2{}, g3{};
    if (h2) g2 = harm_geom(pre.mu, pre.inv_mu, 2.0 * pre.inv_m0, N_par, pre.inv_sqNp);
    if (h3) g3 = harm_geom(pre.mu, pre.inv_mu, 3.0 * pre.inv_m0, N_par, pre.inv_sqNp);
    // Settled before the polarisation vector: when every harmonic present is an
    // exact zero (harm_geom), alpha is a zero whatever the polarisation -- the
    // harmonics would return -mu Pm^2 0 sq_r, finite and zero because N_perp and
    // omega_bar are finite and positive and sq_r is finite, and the prologue's own
    // early returns are zeros too -- so the polarisation vector, the harmonics'
    // K coefficients and the normalisation are skipped (44 % of the stage points
    // of the headline beam: edge plasma and far from every resonance).  Off with
    // the negligible-harmonic skip (GLTable::negl_skip, TORJ_NEGL_SKIP=0).
    if (gl.negl_skip && pre.N_perp > 0.0 && pre.N_perp < INFINITY && pre.omega_bar > 0.0 &&
        pre.omega_bar < INFINITY && pre.mu < INFINITY &&
        (!h2 || (g2.zero && g2.sq_r < INFINITY)) && (!h3 || (g3.zero && g3.sq_r < INFINITY))) {
        if (work) work->n_early += (uint32_t)h2 + (uint32_t)h3;
        return 0.0;
    }
    TORJ_APROF_WAVE(kAprofPro);
    const AlbPro q = albajar_prologue(pre, X, Y, N_abs, N_par, mode);
    if (!q.ok) return 0.0;
    TORJ_APROF_WAVE(kAprofOk);
    if (work) work->n_active++;
    const double hmax = tiny_harmonic(tiny, q, X, omega);
    double c_abs = 0.0;
    if (h2) c_abs += albajar_pro_harmonic<2, LPR, U>(gl, q, g2, work, sub, 0.0, hmax);
    if (h3) c_abs += albajar_pro_harmonic<3, LPR, U>(gl, q, g3, work, sub, c_abs, hmax);
    return albajar_finish(q, c_abs, X, omega);
}
// the fused trace kernels' call (out of line there, see TORJ_ALB_ATTR); kernels
// with nothing else to hold (the split path's alpha kernel) inline the body
template <int LPR = 1>
TORJ_ALB_ATTR double abs_albajar_fast(const GLTable &gl, double omega, double X, double Y, double N_abs,
                                double N_par, double Te, int mode, AlbajarWork *work, int sub = 0,
                                double tiny = 0.0) {
    return abs_albajar_fast_body<LPR>(gl, omega, X, Y, N_abs, N_par, Te, mode, work, sub, tiny);
}

// one RHS evaluation of sys! (src/solve.jl:112-114 -> gradΛ!, :85-95)
template <bool ABS>
TORJ_HD void ray_rhs(const double *__restrict__ coef, const Grid &g, const Consts &k,
                     const GLTable &gl, double omega, int mode, const double x[3], const double N[3],
                     double du[6], double &alpha, AlbajarWork *work) {
    PlasmaPoint p;
    plasma_point<ABS>(coef, g, k, x, p);
    double Npar;
    dispersion_grad(p, N, mode, du, &Npar);
    if constexpr (ABS) {
        const double Nabs = sqrt_pos(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
        alpha = abs_albajar_fast(gl, omega, p.X, p.Y, Nabs, Npar, exp_fast(p.lnTe), mode, work, 0, gl.tiny_alpha);
    } else {
        alpha = 0.0;
    }
}

}  // namespace torj
