// torj_fitdepo.hpp -- power_deposition_profile (src/plasma.jl:91-151) with the
// reference's FITPACK semantics, one lane per ray, after the trace kernel has
// stored make_ray's per-step vectors psi(s_k) and dP/ds_k.
//
// The reference fits Dierckx.Spline1D(s, y, k=3) (FITPACK curfit, s = 0: the
// interpolating cubic with knots at the data points except the 2nd and the
// 2nd-to-last, i.e. the not-a-knot cubic spline) to psi_s - psi_j for every
// shell boundary j, takes its Dierckx.roots, sorts the roots of two
// neighbouring boundaries and integrates the dP/ds spline over consecutive
// pairs; shells are walked from the outside in and the walk stops at the
// first shell whose two boundaries have < 2 roots together.
//
// Here: one not-a-knot solve per ray for psi(s) and dP/ds(s) together (second-
// derivative form, Thomas; the roots of spline(psi_s - c) are the roots of
// spline(psi_s) = c since the fit is linear in the data), then ONE stream over
// the ray's segments: every boundary root is counted (cnt) and toggles the two
// shells it bounds; a toggle that closes a pair adds |F(r) - F(r_open)| to the
// shell's dP, with F the antiderivative of the dP/ds spline (compensated
// running sum).  The break shell k* (from the counts) is applied afterwards,
// by the atomic-free reductions k_shell_sum / k_ray_sum.  Root sets and
// pairings equal the reference's (sorted union, pairs (1,2), (3,4), ..., an
// odd last root dropped); parity is checked against scipy's FITPACK
// (oracle/deposition_ref.py).
//
// The sweeps are sequential per ray and latency-bound, so every sweep loads
// its next kChunk points at once (one memory latency per chunk, not per point)
// and the boundary search is an incremental cursor with the two bracketing
// boundaries in registers.
#pragma once
#include "torj_math.hpp"

namespace torj {

struct FitArgs {
    const double *coef;
    Grid g;
    int n, n_psi;  // rays, shell boundaries
    double ds;
    const double *grid;      // n_psi boundaries (ascending)
    int uniform;             // grid[k] == g0 + k dg to rounding: direct index guess
    double g0, ginv;
    const double *w;         // ray weights (n) or null
    const double *x_launch;  // 3 x n vacuum launch points (s = 0)
    const double *s0;        // n, vacuum path length to the entry point
    const int *steps;        // n
    const double *smp_psi, *smp_dpds, *smp_s;  // (n_steps + 1) x n (smp_s: arc length s_k)
    double *cp, *Mpsi, *MP;            // (n_steps + 2) x n Thomas / second derivatives
    unsigned char *cnt;                // n_psi x n root counts per boundary
    double *Fopen;                     // (n_psi - 1) x n: F at a shell's open root, NaN = closed
    double *dPs;                       // (n_psi - 1) x n: per-ray shell powers (before the break)
    int *kstar;                        // n: break shell
    double *dP;                        // n_psi + 1 (weighted sums; written by k_shell_sum)
    double *Pray;                      // n: per-ray deposited power (reference's P)
};

constexpr int kChunk = 8;  // points per prefetch batch of the sequential sweeps

struct RayData {
    const FitArgs *a;
    int i, m;  // lane's ray, number of points (steps + 2)
    double s0, psiL;
    __device__ double S(int j) const { return j == 0 ? 0.0 : a->smp_s[(size_t)(j - 1) * a->n + i]; }
    __device__ double h(int j) const { return j == 0 ? s0 : S(j + 1) - S(j); }
    __device__ double Ypsi(int j) const { return j == 0 ? psiL : a->smp_psi[(size_t)(j - 1) * a->n + i]; }
    __device__ double YP(int j) const { return j <= 1 ? 0.0 : a->smp_dpds[(size_t)(j - 1) * a->n + i]; }
    __device__ double &CP(int j) const { return a->cp[(size_t)j * a->n + i]; }
    __device__ double &MPSI(int j) const { return a->Mpsi[(size_t)j * a->n + i]; }
    __device__ double &MPP(int j) const { return a->MP[(size_t)j * a->n + i]; }
};

// not-a-knot cubic interpolation of psi and dP/ds (m >= 4 points): second
// derivatives M_j.  Rows r = 1..m-2 of the usual tridiagonal system, with
// M_0 = (1 + h0/h1) M_1 - (h0/h1) M_2 (third-derivative continuity at s_1)
// folded into row 1 and the mirror relation into row m-2.
__device__ void nak_solve(const RayData &R) {
    const int m = R.m;
    double cprev = 0.0, dpsi = 0.0, dPp = 0.0;
    double yl = R.Ypsi(0), yc = R.Ypsi(1), Pl = R.YP(0), Pc = R.YP(1);
    double hl = R.h(0);
    const double h0 = R.h(0), h1 = R.h(1), hm2 = R.h(m - 2), hm3 = R.h(m - 3);
    for (int r0 = 1; r0 <= m - 2; r0 += kChunk) {
        double yv[kChunk], Pv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int j = min(r0 + 1 + u, m - 1);
            yv[u] = R.Ypsi(j);
            Pv[u] = R.YP(j);
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int r = r0 + u;
            if (r > m - 2) break;
            const double hr = R.h(r);
            const double yn = yv[u], Pn = Pv[u];
            const double rp = 6.0 * ((yn - yc) / hr - (yc - yl) / hl);
            const double rP = 6.0 * ((Pn - Pc) / hr - (Pc - Pl) / hl);
            double sub = hl, dia = 2.0 * (hl + hr), sup = hr;
            if (r == 1) {
                dia = 3.0 * h0 + 2.0 * h1 + h0 * h0 / h1;
                sup = h1 - h0 * h0 / h1;
                sub = 0.0;
            }
            if (r == m - 2) {
                sub = hm3 - hm2 * hm2 / hm3;
                dia = (r == 1) ? dia : 2.0 * hm3 + 3.0 * hm2 + hm2 * hm2 / hm3;
                sup = 0.0;
            }
            const double den = dia - sub * cprev;
            cprev = sup / den;
            dpsi = (rp - sub * dpsi) / den;
            dPp = (rP - sub * dPp) / den;
            R.CP(r) = cprev;
            R.MPSI(r) = dpsi;
            R.MPP(r) = dPp;
            yl = yc, yc = yn, Pl = Pc, Pc = Pn, hl = hr;
        }
    }
    double Mp = R.MPSI(m - 2), MPn = R.MPP(m - 2);
    for (int r0 = m - 3; r0 >= 1; r0 -= kChunk) {
        double cv[kChunk], dv[kChunk], ev[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int r = max(r0 - u, 1);
            cv[u] = R.CP(r);
            dv[u] = R.MPSI(r);
            ev[u] = R.MPP(r);
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int r = r0 - u;
            if (r < 1) break;
            Mp = dv[u] - cv[u] * Mp;
            MPn = ev[u] - cv[u] * MPn;
            R.MPSI(r) = Mp;
            R.MPP(r) = MPn;
        }
    }
    const double q0 = h0 / h1, q1 = hm2 / hm3;
    R.MPSI(0) = (1.0 + q0) * R.MPSI(1) - q0 * R.MPSI(2);
    R.MPP(0) = (1.0 + q0) * R.MPP(1) - q0 * R.MPP(2);
    R.MPSI(m - 1) = (1.0 + q1) * R.MPSI(m - 2) - q1 * R.MPSI(m - 3);
    R.MPP(m - 1) = (1.0 + q1) * R.MPP(m - 2) - q1 * R.MPP(m - 3);
}

struct Cubic {  // y0 + t (b + t (c + t d)), t in [0, h]
    double y0, b, c, d, h;
    __device__ double f(double t) const { return fma(t, fma(t, fma(t, d, c), b), y0); }
    __device__ double df(double t) const { return fma(t, fma(t, 3.0 * d, 2.0 * c), b); }
    __device__ double G(double t) const {  // integral 0..t
        return t * fma(t, fma(t, fma(t, 0.25 * d, c * (1.0 / 3.0)), 0.5 * b), y0);
    }
};

__device__ Cubic make_cubic(double y0, double y1, double M0, double M1, double h) {
    Cubic q;
    q.y0 = y0;
    q.h = h;
    q.b = (y1 - y0) / h - h * (2.0 * M0 + M1) * (1.0 / 6.0);
    q.c = 0.5 * M0;
    q.d = (M1 - M0) / (6.0 * h);
    return q;
}

// smallest boundary index k with grid[k] > x (strict) / >= x
__device__ int level_above(const FitArgs &a, double x, bool strict) {
    int k;
    if (a.uniform) {
        const double u = (x - a.g0) * a.ginv;
        k = u < 0 ? 0 : (u > a.n_psi ? a.n_psi : (int)ceil(u));
        while (k > 0 && (strict ? a.grid[k - 1] > x : a.grid[k - 1] >= x)) k--;
        while (k < a.n_psi && (strict ? a.grid[k] <= x : a.grid[k] < x)) k++;
    } else {
        int lo = 0, hi = a.n_psi;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (strict ? a.grid[mid] > x : a.grid[mid] >= x)
                hi = mid;
            else
                lo = mid + 1;
        }
        k = lo;
    }
    return k;
}

// Incremental boundary cursor: c = #boundaries <= v for the current value v,
// with the two bracketing boundaries grid[c-1] <= v < grid[c] in registers, so
// a segment that crosses no boundary costs no memory access.
struct Cursor {
    const FitArgs *a;
    int c;
    double lo, hi;  // grid[c-1] (or -inf), grid[c] (or +inf)
    __device__ void load() {
        lo = c > 0 ? a->grid[c - 1] : -INFINITY;
        hi = c < a->n_psi ? a->grid[c] : INFINITY;
    }
    __device__ void seek(double v) {  // c = #boundaries <= v
        if (v >= lo && v < hi) return;
        while (c < a->n_psi && a->grid[c] <= v) c++;
        while (c > 0 && a->grid[c - 1] > v) c--;
        load();
    }
};

// root of the monotone cubic piece q(t) = L on [ta, tb], L strictly between
// the end values: Newton with a bisection safeguard, to the last bit
__device__ double cubic_root(const Cubic &q, double L, double ta, double tb, bool up) {
    double lo = ta, hi = tb, t = 0.5 * (ta + tb);
    for (int it = 0; it < 100; it++) {
        const double v = q.f(t) - L;
        if (v == 0.0) break;
        if ((v > 0.0) == up)
            hi = t;  // past the root
        else
            lo = t;
        double tn = t - v / q.df(t);
        if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
        if (tn == t || !(tn > lo && tn < hi)) break;
        t = tn;
    }
    return t;
}

struct Walker {
    const FitArgs *a;
    int i;
    double Fhi, Flo;  // compensated running integral of dP/ds at the segment start
    Cursor cur;
    // a root of boundary L_k at running integral Fr: count it and toggle the
    // shells it bounds (k-1 above it, k below it)
    __device__ void root(int k, double Fr) {
        unsigned char &c = a->cnt[(size_t)k * a->n + i];
        if (c < 255) c++;
#pragma unroll
        for (int dq = -1; dq <= 0; dq++) {
            const int q = k + dq;
            if (q < 0 || q > a->n_psi - 2) continue;
            double &fo = a->Fopen[(size_t)q * a->n + i];
            if (isnan(fo)) {
                fo = Fr;
            } else {
                a->dPs[(size_t)q * a->n + i] += fabs(Fr - fo);  // |integrate(dP_ds, r1, r2)|
                fo = NAN;
            }
        }
    }
};

// stream segment j of the psi spline: every boundary crossing in s order.
// End values are the data (y0, y1), so a boundary equal to a data value is
// found exactly once: roots lie in (s_j, s_{j+1}] (segment 0 also takes s = 0).
__device__ void walk_segment(Walker &W, const Cubic &qs, double y1, const Cubic &qP, bool first) {
    const FitArgs &a = *W.a;
    // fast path: no boundary between the end values and a monotone segment
    const double A = 3.0 * qs.d, B = 2.0 * qs.c, C = qs.b;
    const double disc = B * B - 4.0 * A * C;
    double cut[4];
    int nc = 0;
    cut[nc++] = 0.0;
    if (A != 0.0 ? disc > 0.0 : B != 0.0) {  // psi'(t) may vanish inside: split there
        double r1 = NAN, r2 = NAN;
        if (A != 0.0) {
            const double sq = sqrt(disc);
            const double qq = -0.5 * (B + (B >= 0.0 ? sq : -sq));
            r1 = qq / A;
            if (qq != 0.0) r2 = C / qq;
        } else {
            r1 = -C / B;
        }
        if (r2 < r1) {
            const double t = r1;
            r1 = r2;
            r2 = t;
        }
        if (r1 > 0.0 && r1 < qs.h) cut[nc++] = r1;
        if (r2 > 0.0 && r2 < qs.h && r2 != r1) cut[nc++] = r2;
    }
    cut[nc++] = qs.h;
    double fa = qs.y0;
    for (int p = 0; p + 1 < nc; p++) {
        const double ta = cut[p], tb = cut[p + 1];
        const double fb = (p + 2 == nc) ? y1 : qs.f(tb);
        if (fb > fa) {  // increasing: boundaries fa < L <= fb (fa <= L at s = 0), ascending
            int k = (first && p == 0) ? level_above(a, fa, false) : W.cur.c;
            W.cur.seek(fb);
            for (; k < W.cur.c; k++) {
                const double L = a.grid[k];
                const double t = (L == fb) ? tb : (L == fa ? ta : cubic_root(qs, L, ta, tb, true));
                W.root(k, W.Fhi + (W.Flo + qP.G(t)));
            }
        } else if (fb < fa) {  // decreasing: boundaries fb <= L < fa (<= fa at s = 0), descending
            const int top = (first && p == 0) ? level_above(a, fa, true) : W.cur.c - (fa == W.cur.lo);
            W.cur.seek(fb);
            const int bot = W.cur.c - (fb == W.cur.lo);  // #boundaries < fb
            for (int k = top - 1; k >= bot; k--) {
                const double L = a.grid[k];
                const double t = (L == fb) ? tb : (L == fa ? ta : cubic_root(qs, L, ta, tb, false));
                W.root(k, W.Fhi + (W.Flo + qP.G(t)));
            }
        } else {
            W.cur.seek(fb);
        }
        fa = fb;
    }
    // F(s_{j+1}) = F(s_j) + integral over the segment (TwoSum compensation)
    const double g = qP.G(qs.h);
    const double sum = W.Fhi + g;
    const double bp = sum - W.Fhi;
    W.Flo += (W.Fhi - (sum - bp)) + (g - bp);
    W.Fhi = sum;
}

__device__ void walk_ray(Walker &W, const RayData &R) {
    double yl = R.Ypsi(0), Pl = R.YP(0), Ml = R.MPSI(0), MPl = R.MPP(0);
    W.cur.c = level_above(*W.a, yl, true);  // #boundaries <= psi(s = 0)
    W.cur.load();
    for (int j0 = 0; j0 + 1 < R.m; j0 += kChunk) {
        double yv[kChunk], Pv[kChunk], Mv[kChunk], MPv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int j = min(j0 + 1 + u, R.m - 1);
            yv[u] = R.Ypsi(j);
            Pv[u] = R.YP(j);
            Mv[u] = R.MPSI(j);
            MPv[u] = R.MPP(j);
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int j = j0 + u;
            if (j + 1 >= R.m) break;
            const double h = R.h(j);
            const Cubic qs = make_cubic(yl, yv[u], Ml, Mv[u], h), qP = make_cubic(Pl, Pv[u], MPl, MPv[u], h);
            walk_segment(W, qs, yv[u], qP, j == 0);
            yl = yv[u], Pl = Pv[u], Ml = Mv[u], MPl = MPv[u];
        }
    }
}

}  // namespace torj
