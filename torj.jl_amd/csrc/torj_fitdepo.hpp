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

// Per-step arrays of a ray (the trace kernel's samples, the elimination's
// coefficients) in blocks of 64 rays: element (row j, ray i) at
// ((i / 64) rows + j) 64 + i % 64.  A wave streams its block's rows as one
// contiguous region instead of rows n x 8 B apart (a new page every few rows at
// 1e5 rays: address-translation misses dominated the walk).  rows = n_steps + 2;
// allocations hold ceil(n / 64) blocks.
constexpr int kSmpBlk = 64;
TORJ_HD size_t smp_at(size_t j, int i, size_t rows) {
    return ((size_t)((unsigned)i / kSmpBlk) * rows + j) * kSmpBlk + (unsigned)i % kSmpBlk;
}
TORJ_HD size_t smp_elems(size_t n, size_t rows) { return (n + kSmpBlk - 1) / kSmpBlk * kSmpBlk * rows; }

struct FitArgs {
    const double *coef;
    Grid g;
    int n, n_psi;  // rays, shell boundaries
    double ds;
    const double *grid;      // n_psi boundaries (ascending)
    const double *w;         // ray weights (n) or null
    const double *x_launch;  // 3 x n vacuum launch points (s = 0)
    const double *s0;        // n, vacuum path length to the entry point
    const int *steps;        // n
    const double *smp_psi, *smp_dpds, *smp_s;  // smp_at layout (smp_s: arc length s_k)
    size_t rows;                       // smp_at rows per ray: n_steps + 2
    int s_uniform;                     // fixed-step RK4: s_k = s0 + k ds (smp_s unused)
    double *E, *Gpsi, *GP;             // smp_at layout: backward-elimination coefficients
    int *cnt;                          // (n_psi + 1) x n root-count differences per boundary
    double *Fopen;                     // (n_psi - 1) x n: F at a spilled open shell's root, NaN = closed
    double *dPs;                       // (n_psi - 1) x n: per-ray shell powers (before the break)
    int *kstar;                        // n: break shell
    double *dP;                        // n_psi + 1 (weighted sums; written by k_shell_sum)
    double *Pray;                      // n: per-ray deposited power (reference's P)
    // torj_power_deposition_profile (caller-given vectors): points per ray; every
    // point j of ray i (s, psi, dP/ds) is then row j of smp_s / smp_psi /
    // smp_dpds, launch and entry points included.  Null for a trace's samples.
    const int *npts;
};

TORJ_HD int imin(int x, int y) { return x < y ? x : y; }
TORJ_HD int imax(int x, int y) { return x > y ? x : y; }

constexpr int kChunk = 8;      // points per prefetch batch of the sequential sweeps
constexpr int kWalkChunk = 4;  // the walk's batch (five streams, the heavy segment code)
// the streamed walk kernel's batch (k_depo_walk, TORJ_DEPO_STREAM=3): one
// segment at a time fits 168 VGPRs without spilling (three waves per SIMD
// beside the alpha waves); the batch of 4 needs 244
constexpr int kWalkChunkStream = 1;

struct RayData {
    const FitArgs *a;
    int i, m;  // lane's ray, number of points (steps + 2)
    double s0, psiL;
    // arc length of point j: 0 (launch), s0 (entry), s0 + (j-1) ds for RK4 (the
    // fma the trajectory output uses), else the integrator's stored s
    TORJ_HD double S(int j) const {
        if (a->npts) return a->smp_s[smp_at(j, i, a->rows)];
        if (j == 0) return 0.0;
        return a->s_uniform ? fma((double)(j - 1), a->ds, s0) : a->smp_s[smp_at(j - 1, i, a->rows)];
    }
    TORJ_HD double h(int j) const { return (j == 0 && !a->npts) ? s0 : S(j + 1) - S(j); }
    TORJ_HD double Ypsi(int j) const {
        if (a->npts) return a->smp_psi[smp_at(j, i, a->rows)];
        return j == 0 ? psiL : a->smp_psi[smp_at(j - 1, i, a->rows)];
    }
    TORJ_HD double YP(int j) const {
        if (a->npts) return a->smp_dpds[smp_at(j, i, a->rows)];
        return j <= 1 ? 0.0 : a->smp_dpds[smp_at(j - 1, i, a->rows)];
    }
    TORJ_HD double &EE(int j) const { return a->E[smp_at(j, i, a->rows)]; }
    TORJ_HD double &GPSI(int j) const { return a->Gpsi[smp_at(j, i, a->rows)]; }
    TORJ_HD double &GPP(int j) const { return a->GP[smp_at(j, i, a->rows)]; }
};

// not-a-knot cubic interpolation of psi and dP/ds (m >= 4 points): second
// derivatives M_j.  Rows r = 1..m-2 of the usual tridiagonal system, with
// M_0 = (1 + h0/h1) M_1 - (h0/h1) M_2 (third-derivative continuity at s_1)
// folded into row 1 and the mirror relation into row m-2.  Eliminated from the
// bottom up (this sweep stores e_r, g_r with M_r = g_r - e_r M_{r-1}), so the
// substitution runs upwards in s and fuses with the root walk (walk_ray): one
// stored sweep instead of two.
TORJ_HD void nak_eliminate_rows(const RayData &R, int r_lo, int r_hi);
TORJ_HD void nak_eliminate(const RayData &R) { nak_eliminate_rows(R, 1, R.m - 2); }

// Rows r_hi down to r_lo of the same elimination.  r_hi = m - 2 is the whole
// system's bottom (the not-a-knot end row); a smaller r_hi starts a window of
// the streamed deposition (k_depo_stream) as if M_{r_hi + 1} were 0: that
// start's influence on e_r, g_r decays by ~(2 - sqrt 3) = 0.27 per row upwards
// (5e-19 after the kDepoW rows a window carries past the segments it walks).
TORJ_HD void nak_eliminate_rows(const RayData &R, int r_lo, int r_hi) {
    const int m = R.m;
    const double h0 = R.h(0), h1 = R.h(1);
    double yn = R.Ypsi(r_hi + 1), yc = R.Ypsi(r_hi), Pn = R.YP(r_hi + 1), Pc = R.YP(r_hi);
    double hr = R.h(r_hi), ihr = rcp_nz(hr);
    double e = 0.0, gp = 0.0, gP = 0.0;
    for (int r0 = r_hi; r0 >= r_lo; r0 -= kChunk) {
        double yv[kChunk], Pv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int j = imax(r0 - 1 - u, 0);
            yv[u] = R.Ypsi(j);
            Pv[u] = R.YP(j);
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int r = r0 - u;
            if (r < r_lo) break;
            const double hl = R.h(r - 1), ihl = rcp_nz(hl);
            const double yl = yv[u], Pl = Pv[u];
            const double rp = 6.0 * ((yn - yc) * ihr - (yc - yl) * ihl);
            const double rP = 6.0 * ((Pn - Pc) * ihr - (Pc - Pl) * ihl);
            double sub = hl, dia = 2.0 * (hl + hr), sup = hr;
            if (r == 1) {
                dia = 3.0 * h0 + 2.0 * h1 + h0 * h0 / h1;
                sup = h1 - h0 * h0 / h1;
                sub = 0.0;
            }
            if (r == m - 2) {
                const double hm2 = hr, hm3 = hl;  // h(m - 2), h(m - 3)
                sub = hm3 - hm2 * hm2 / hm3;
                dia = 2.0 * hm3 + 3.0 * hm2 + hm2 * hm2 / hm3;
                sup = 0.0;
            }
            const double iden = rcp_nz(dia - sup * e);  // e = e_{r+1} (0 below row m-2)
            gp = (rp - sup * gp) * iden;
            gP = (rP - sup * gP) * iden;
            e = sub * iden;
            R.EE(r) = e;
            R.GPSI(r) = gp;
            R.GPP(r) = gP;
            yn = yc, yc = yl, Pn = Pc, Pc = Pl, hr = hl, ihr = ihl;
        }
    }
}

struct Cubic {  // y0 + t (b + t (c + t d)), t in [0, h]
    double y0, b, c, d, h;
    TORJ_HD double f(double t) const { return fma(t, fma(t, fma(t, d, c), b), y0); }
    TORJ_HD double df(double t) const { return fma(t, fma(t, 3.0 * d, 2.0 * c), b); }
    TORJ_HD double G(double t) const {  // integral 0..t
        return t * fma(t, fma(t, fma(t, 0.25 * d, c * (1.0 / 3.0)), 0.5 * b), y0);
    }
};

TORJ_HD Cubic make_cubic(double y0, double y1, double M0, double M1, double h, double ih) {
    Cubic q;
    q.y0 = y0;
    q.h = h;
    q.b = (y1 - y0) * ih - h * (2.0 * M0 + M1) * (1.0 / 6.0);
    q.c = 0.5 * M0;
    q.d = (M1 - M0) * ih * (1.0 / 6.0);
    return q;
}

// smallest boundary index k with grid[k] > x (strict) / >= x: a guess as if
// the grid were uniform (np.linspace), corrected by a local walk -- exact for
// any strictly increasing grid
TORJ_HD int level_above(const FitArgs &a, double x, bool strict) {
    const double g0 = a.grid[0], gn = a.grid[a.n_psi - 1];
    const double u = (x - g0) * ((double)(a.n_psi - 1) / (gn - g0));
    int k = u < 0 ? 0 : (u > a.n_psi ? a.n_psi : (int)ceil(u));
    while (k > 0 && (strict ? a.grid[k - 1] > x : a.grid[k - 1] >= x)) k--;
    while (k < a.n_psi && (strict ? a.grid[k] <= x : a.grid[k] < x)) k++;
    return k;
}

// Incremental boundary cursor: c = #boundaries <= v for the current value v,
// with the two bracketing boundaries grid[c-1] <= v < grid[c] in registers, so
// a segment that crosses no boundary costs no memory access.
struct Cursor {
    const FitArgs *a;
    int c;
    double lo, hi;  // grid[c-1] (or -inf), grid[c] (or +inf)
    TORJ_HD void load() {
        lo = c > 0 ? a->grid[c - 1] : -INFINITY;
        hi = c < a->n_psi ? a->grid[c] : INFINITY;
    }
    TORJ_HD void seek(double v) {  // c = #boundaries <= v
        if (v >= lo && v < hi) return;
        while (c < a->n_psi && a->grid[c] <= v) c++;
        while (c > 0 && a->grid[c - 1] > v) c--;
        load();
    }
};

#if defined(TORJ_ROOT_STATS) && !defined(__HIP_DEVICE_COMPILE__)
// host statistics build only (tests/native): cubic_root calls and Newton steps
inline unsigned long long g_root_calls = 0, g_root_iters = 0, g_root_hist[8] = {};
#endif
// root of the monotone cubic piece q(t) = L on [ta, tb], L strictly between
// the end values: Newton with a bisection safeguard, to the last bit
TORJ_HD double cubic_root(const Cubic &q, double L, double ta, double tb, double fa, double fb,
                          bool up) {
    double lo = ta, hi = tb, t = fma(L - fa, (tb - ta) * rcp_nz(fb - fa), ta);  // secant start
    if (!(t > lo && t < hi)) t = 0.5 * (ta + tb);
#if defined(TORJ_ROOT_STATS) && !defined(__HIP_DEVICE_COMPILE__)
    struct Tally {
        int it = 0;
        ~Tally() { g_root_calls++, g_root_iters += it, g_root_hist[it < 7 ? it : 7]++; }
    } tally;
#endif
    for (int it = 0; it < 100; it++) {
#if defined(TORJ_ROOT_STATS) && !defined(__HIP_DEVICE_COMPILE__)
        tally.it = it + 1;
#endif
        const double v = q.f(t) - L;
        if (v == 0.0) break;
        if ((v > 0.0) == up)
            hi = t;  // past the root
        else
            lo = t;
        double tn = t - v * rcp_nz(q.df(t));
        if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
        if (tn == t || !(tn > lo && tn < hi)) break;
        t = tn;
    }
    return t;
}

// Per-root state without per-root memory traffic (a wave's lanes sit at
// different boundaries, so every per-root access is 64 scattered lines):
//  * open shells (one root seen, waiting for its partner) live in a small
//    register cache; a third open shell spills the oldest entry to Fopen;
//  * root counts are kept as runs: consecutive roots at k, k+d, k+2d, ... (a
//    monotone crossing of the boundary levels) form one run, flushed as a
//    difference pair cdiff[lo] += 1, cdiff[hi + 1] -= 1, so cnt[k] is a prefix
//    sum (one flush per turning point of psi(s), not one update per root);
//  * a closed pair adds its |integral| to the shell with a no-return atomic on
//    the lane's own element.
constexpr int kOpenCache = 2;

// Dierckx.roots(spline; maxn = 8) (the reference's call, src/plasma.jl:108,118,
// default maxn of Dierckx.jl 0.5.4): FITPACK sproot with mest = 8 keeps the
// first 8 zeros of each boundary's spline in s order (scipy's sproot, the
// oracle's restatement, does the same and warns).  A boundary can have more
// than 8 roots only if psi(s) has more than 8 monotone runs (one root per
// boundary per run), so the walk counts its runs and re-walks the rare ray
// with more in the capped mode below (exact per-boundary counts in memory).
constexpr int kMaxRoots = 8;

template <int NC = kOpenCache, bool CAP = false>
struct Walker {
    const FitArgs *a;
    int i;
    double Fhi, Flo;  // compensated running integral of dP/ds at the segment start
    Cursor cur;
    int oq[NC];     // open shell ids (-1: free slot)
    double oF[NC];  // F at their opening root
    bool spilled;           // some open shell lives in Fopen
    int run_k0, run_k1, run_d;  // current run of roots (run_d = 0: none)
    int runs, last_d;       // monotone runs of psi(s) so far, direction of the last one
    TORJ_HD void init() {
#pragma unroll
        for (int u = 0; u < NC; u++) oq[u] = -1, oF[u] = 0.0;
        spilled = false;
        run_d = 0, run_k0 = run_k1 = 0;
        runs = 0, last_d = 0;
    }
    TORJ_HD void piece(int d) {  // a monotone piece of direction d (+1 / -1) of psi(s)
        if (d != last_d) runs++, last_d = d;
    }
    TORJ_HD void cadd(int k, int v) {
        __hip_atomic_fetch_add(a->cnt + (size_t)k * a->n + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    TORJ_HD void flush_run() {
        if (run_d == 0) return;
        const int lo = run_k0 < run_k1 ? run_k0 : run_k1, hi = run_k0 < run_k1 ? run_k1 : run_k0;
        cadd(lo, 1);
        cadd(hi + 1, -1);
        run_d = 0;
    }
    TORJ_HD void close(int q, double d) {  // |integrate(dP_ds, r1, r2)|
        double *p = a->dPs + (size_t)q * a->n + i;
        __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    TORJ_HD void toggle(int q, double Fr) {
        bool hit = false;
        double fo = 0.0;
#pragma unroll
        for (int u = 0; u < NC; u++)
            if (!hit && oq[u] == q) hit = true, fo = oF[u], oq[u] = -1;
        if (!hit && spilled) {  // maybe open in memory
            double &m = a->Fopen[(size_t)q * a->n + i];
            fo = m;
            if (!isnan(fo)) hit = true, m = NAN;
        }
        if (hit) {
            close(q, fabs(Fr - fo));
            return;
        }
        bool placed = false;
#pragma unroll
        for (int u = 0; u < NC; u++)
            if (!placed && oq[u] < 0) placed = true, oq[u] = q, oF[u] = Fr;
        if (!placed) {  // spill slot 0 (rare: > 2 shells open at once)
            a->Fopen[(size_t)oq[0] * a->n + i] = oF[0];
            spilled = true;
            oq[0] = q, oF[0] = Fr;
        }
    }
    // a root of boundary L_k at running integral Fr, found while the boundary
    // levels are crossed in direction d (+1 upwards, -1 downwards): count it and
    // toggle the shells it bounds (k-1 above it, k below it)
    TORJ_HD void root(int k, double Fr, int d) {
        if constexpr (CAP) {  // direct count of boundary k's roots so far: the 9th is dropped
            int &c = a->cnt[(size_t)k * a->n + i];
            if (c >= kMaxRoots) return;
            c++;
        } else if (d == run_d && k == run_k1 + d) {
            run_k1 = k;
        } else {
            flush_run();
            run_d = d, run_k0 = run_k1 = k;
        }
        if (k - 1 >= 0 && k - 1 <= a->n_psi - 2) toggle(k - 1, Fr);
        if (k <= a->n_psi - 2) toggle(k, Fr);
    }
};

// stream segment j of the psi spline: every boundary crossing in s order.
// End values are the data (y0, y1), so a boundary equal to a data value is
// found exactly once: roots lie in (s_j, s_{j+1}] (segment 0 also takes s = 0).
// The segment splits at the zeros of psi' into at most three monotone pieces
// [0, c1], [c1, c2], [c2, h] (absent cuts sit at h and give empty pieces); one
// rolled piece loop and one root loop keep the code (and registers) small.
template <class W_>
TORJ_HD void walk_segment(W_ &W, const Cubic &qs, double y1, const Cubic &qP, bool first) {
    const FitArgs &a = *W.a;
    const double A = 3.0 * qs.d, B = 2.0 * qs.c, C = qs.b;
    const double disc = B * B - 4.0 * A * C;
    double c1 = qs.h, c2 = qs.h;
    // psi'(0) = C and psi'(h) of one strict sign with the parabola's vertex
    // -B / 2A outside (0, h): no zero inside, no split (the sqrt is skipped)
    const double dh = fma(fma(A, qs.h, B), qs.h, C);
    const double tv = -B * A;  // vertex position times 2 A^2
    const bool keep = (C > 0.0 && dh > 0.0) || (C < 0.0 && dh < 0.0);
    const bool vout = A == 0.0 || tv <= 0.0 || tv >= 2.0 * A * A * qs.h;
    if (!(keep && vout) && (A != 0.0 ? disc > 0.0 : B != 0.0)) {  // psi'(t) may vanish inside: split there
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
        const bool in1 = r1 > 0.0 && r1 < qs.h, in2 = r2 > 0.0 && r2 < qs.h && r2 != r1;
        if (in1) c1 = r1;
        if (in2) {
            if (in1)
                c2 = r2;
            else
                c1 = r2;
        }
    }
    double fa = qs.y0, ta = 0.0;
#pragma unroll 1
    for (int p = 0; p < 3; p++) {
        const double tb = p == 0 ? c1 : (p == 1 ? c2 : qs.h);
        if (!(tb > ta) && p > 0) continue;  // empty piece (absent cut)
        const double fb = (tb == qs.h) ? y1 : qs.f(tb);
        const bool first0 = first && p == 0;
        int k, kend, d;
        if (fb > fa) {  // increasing: boundaries fa < L <= fb (fa <= L at s = 0), ascending
            d = 1;
            W.piece(1);
            k = first0 ? level_above(a, fa, false) : W.cur.c;
            W.cur.seek(fb);
            kend = W.cur.c;
        } else if (fb < fa) {  // decreasing: boundaries fb <= L < fa (<= fa at s = 0), descending
            d = -1;
            W.piece(-1);
            k = (first0 ? level_above(a, fa, true) : W.cur.c - (fa == W.cur.lo)) - 1;
            W.cur.seek(fb);
            kend = W.cur.c - (fb == W.cur.lo) - 1;  // #boundaries < fb, minus one
        } else {
            W.cur.seek(fb);
            d = 0, k = kend = 0;
        }
        for (; d > 0 ? k < kend : k > kend; k += d) {
            const double L = a.grid[k];
            const double t = (L == fb) ? tb : (L == fa ? ta : cubic_root(qs, L, ta, tb, fa, fb, d > 0));
            W.root(k, W.Fhi + (W.Flo + qP.G(t)), d);
        }
        fa = fb, ta = tb;
        if (tb == qs.h) break;
    }
    // F(s_{j+1}) = F(s_j) + integral over the segment (TwoSum compensation)
    const double g = qP.G(qs.h);
    const double sum = W.Fhi + g;
    const double bp = sum - W.Fhi;
    W.Flo += (W.Fhi - (sum - bp)) + (g - bp);
    W.Fhi = sum;
}

// The walk's position: segment j is next, with (M_j, M_{j+1}, M_{j+2}) of the psi
// and dP/ds splines and the data at point j (psi, dP/ds).
struct WalkCarry {
    double Ml, Mr, Mn, MPl, MPr, MPn, yl, Pl;
    int j;
};

// the walk's start (segment 0): rows 1 and 2 of the elimination are final
template <class W_>
TORJ_HD void walk_start(W_ &W, const RayData &R, WalkCarry &C) {
    const double q0 = R.h(0) / R.h(1);
    const double M1 = R.GPSI(1), M1P = R.GPP(1);
    const double M2 = R.GPSI(2) - R.EE(2) * M1, M2P = R.GPP(2) - R.EE(2) * M1P;
    C.Ml = (1.0 + q0) * M1 - q0 * M2, C.MPl = (1.0 + q0) * M1P - q0 * M2P;
    C.Mr = M1, C.MPr = M1P, C.Mn = M2, C.MPn = M2P;
    C.yl = R.Ypsi(0), C.Pl = R.YP(0);
    C.j = 0;
    W.cur.c = level_above(*W.a, C.yl, true);  // #boundaries <= psi(s = 0)
    W.cur.load();
}

// the root walk over segments [C.j, j_end), with the spline's second
// derivatives from the upward substitution M_r = g_r - e_r M_{r-1}
// (nak_eliminate) as it goes; rows C.j + 3 .. j_end + 2 (at most m - 2) of the
// elimination are final
template <int WC = kWalkChunk, class W_>
TORJ_HD void walk_segments(W_ &W, const RayData &R, WalkCarry &C, int j_end) {
    const int m = R.m;
    double Ml = C.Ml, Mr = C.Mr, Mn = C.Mn, MPl = C.MPl, MPr = C.MPr, MPn = C.MPn;
    double yl = C.yl, Pl = C.Pl;
    for (int j0 = C.j; j0 < j_end; j0 += WC) {
        double yv[WC], Pv[WC], ev[WC], gv[WC], gPv[WC];
#pragma unroll
        for (int u = 0; u < WC; u++) {
            const int j = imin(j0 + 1 + u, m - 1);
            yv[u] = R.Ypsi(j);
            Pv[u] = R.YP(j);
            const int r = imin(j0 + 3 + u, m - 2);  // row of M_{j+3}, prepared after segment j+1
            ev[u] = R.EE(r);
            gv[u] = R.GPSI(r);
            gPv[u] = R.GPP(r);
        }
#pragma unroll
        for (int u = 0; u < WC; u++) {
            const int j = j0 + u;
            if (j >= j_end) break;
            const double h = R.h(j), ih = rcp_nz(h);
            const Cubic qs = make_cubic(yl, yv[u], Ml, Mr, h, ih), qP = make_cubic(Pl, Pv[u], MPl, MPr, h, ih);
            walk_segment(W, qs, yv[u], qP, j == 0);
            yl = yv[u], Pl = Pv[u];
            // advance: (M_j, M_{j+1}, M_{j+2}) -> (M_{j+1}, M_{j+2}, M_{j+3})
            Ml = Mr, MPl = MPr, Mr = Mn, MPr = MPn;
            if (j + 3 <= m - 2) {
                Mn = gv[u] - ev[u] * Mr;
                MPn = gPv[u] - ev[u] * MPr;
            } else if (j + 3 == m - 1) {  // not-a-knot end: M_{m-1} from M_{m-2}, M_{m-3}
                const double q1 = R.h(m - 2) / R.h(m - 3);
                Mn = (1.0 + q1) * Mr - q1 * Ml;
                MPn = (1.0 + q1) * MPr - q1 * MPl;
            }
        }
    }
    C.Ml = Ml, C.Mr = Mr, C.Mn = Mn, C.MPl = MPl, C.MPr = MPr, C.MPn = MPn;
    C.yl = yl, C.Pl = Pl;
    C.j = j_end;
}

template <class W_>
TORJ_HD void walk_ray(W_ &W, const RayData &R) {
    WalkCarry C;
    walk_start(W, R, C);
    walk_segments(W, R, C, R.m - 1);
}

// The walk's end: flush the last root run, redo a ray whose psi(s) has more
// than kMaxRoots monotone runs with the root cap, then the reference's
// outside-in break shell k* and the ray's deposited power P.
template <int NC>
TORJ_HD void fit_depo_finish(const FitArgs &a, int i, const RayData &R, Walker<NC> &W) {
    W.flush_run();
    // the walk's root counts and shell sums are no-return atomics: wait for them
    // before this lane reads its own counts back
#ifdef __HIP_DEVICE_COMPILE__
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    const size_t n = a.n;
    const int L = a.n_psi;
    const bool capped = W.runs > kMaxRoots;
    if (capped) {  // some boundary may have > maxn roots: redo the ray with the cap
        for (int k = 0; k <= L; k++) a.cnt[(size_t)k * n + i] = 0;
        for (int q = 0; q + 1 < L; q++) {
            a.dPs[(size_t)q * n + i] = 0.0;
            a.Fopen[(size_t)q * n + i] = NAN;
        }
#ifdef __HIP_DEVICE_COMPILE__
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        // the whole-ray elimination again (a streamed walk's windows left other
        // rows behind; for fit_depo_ray the same values)
        nak_eliminate(R);
        Walker<NC, true> Wc{&a, i, 0.0, 0.0, Cursor{&a, 0, 0.0, 0.0}};
        Wc.init();
        walk_ray(Wc, R);
#ifdef __HIP_DEVICE_COMPILE__
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    }
    // the reference's outside-in walk stops at the first shell whose two
    // boundaries have < 2 roots together (src/plasma.jl:120-124)
    // root counts: cnt[k] = sum_{j <= k} cdiff[j] = -sum_{j > k} cdiff[j] (the
    // differences sum to zero), accumulated from the top; the capped walk
    // stores the counts themselves
    int kstar = -1;
    int suf = a.cnt[(size_t)L * n + i];  // sum_{j > L-1} cdiff[j]
    int c_up = capped ? a.cnt[(size_t)(L - 1) * n + i] : -suf;  // cnt[L-1]
    for (int k0 = L - 2; k0 >= 0 && kstar < 0; k0 -= kChunk) {
        int dv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) dv[u] = a.cnt[(size_t)imax(k0 - u + (capped ? 0 : 1), 0) * n + i];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {  // shell k = k0 - u: boundaries k and k + 1
            const int k = k0 - u;
            if (k >= 0 && kstar < 0) {
                suf += dv[u];  // now sum_{j > k}
                const int c_k = capped ? dv[u] : -suf;
                if (c_up + c_k < 2) kstar = k;
                c_up = c_k;
            }
        }
    }
    a.kstar[i] = kstar;
    double P = 0.0;
    for (int q0 = a.n_psi - 2; q0 > kstar; q0 -= kChunk) {
        double v[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) v[u] = a.dPs[(size_t)imax(q0 - u, 0) * n + i];
#pragma unroll
        for (int u = 0; u < kChunk; u++)
            if (q0 - u > kstar) P += v[u];
    }
    a.Pray[i] = P;
}

// One ray of power_deposition_profile (k_fit_depo; the CPU suite runs the host
// build through tests/native): spline fits, the root walk, the outside-in break
// shell k* and the ray's deposited power P.  psiL = psi at the launch point.
template <int NC>
TORJ_HD void fit_depo_ray(const FitArgs &a, int i, double psiL) {
    // a trace: launch point, entry point, one per step; or the caller's points
    const int m = a.npts ? a.npts[i] : a.steps[i] + 2;
    if (m < 4 || (!a.npts && !(a.s0[i] > 0.0))) {  // FITPACK needs > k = 3 strictly increasing points
        a.kstar[i] = a.n_psi;  // no shell counts
        a.Pray[i] = 0.0;
        return;
    }
    RayData R{&a, i, m, a.npts ? 0.0 : a.s0[i], psiL};
    nak_eliminate(R);
    Walker<NC> W{&a, i, 0.0, 0.0, Cursor{&a, 0, 0.0, 0.0}};
    W.init();
    walk_ray(W, R);
    fit_depo_finish(a, i, R, W);
}

// ---------------------------------------------------------------------------
// Streamed deposition (the split pipeline): the walk advances in windows of
// kDepoQ segments while the trace is still running, one k_depo_stream launch
// after each block's optical-depth scan, and k_depo_tail finishes every ray
// after the trace.  A window [j, j + kDepoQ) eliminates rows j + 3 ..
// j + kDepoQ + 2 + kDepoW from a start kDepoW rows below the last row it uses
// (nak_eliminate_rows), so it needs the ray's points up to j + kDepoQ + 3 +
// kDepoW and never the not-a-knot end.  Window boundaries are multiples of
// kDepoQ whatever the launch schedule (block size, ray batch) and each window
// recomputes its own rows, so the results do not depend on when the windows
// ran.  The rest of the ray after the last window that fits below its end
// point m - 2 is the exact elimination of the unstreamed kernel; a ray with no
// window (m < kDepoQ + kDepoW + 5) is exactly fit_depo_ray.  Against the one
// global elimination the second derivatives move by rounding only (the window
// start's influence is ~5e-19 where it is used).
#ifndef TORJ_DEPO_Q  // segments per streamed window
#define TORJ_DEPO_Q 64
#endif
constexpr int kDepoQ = TORJ_DEPO_Q, kDepoW = 32;
// one ray's walk between launches, SoA [field][n]
enum { kDsFhi, kDsFlo, kDsOF0, kDsOF1, kDsMl, kDsMr, kDsMn, kDsMPl, kDsMPr, kDsMPn, kDsYl, kDsPl, kDsNd };
enum { kDsJ, kDsC, kDsOQ0, kDsOQ1, kDsSpill, kDsRk0, kDsRk1, kDsRd, kDsRuns, kDsLast, kDsNi };
struct DepoStream {
    double *d;  // kDsNd x n
    int *v;     // kDsNi x n; v[kDsJ] = -1: not started
};
static_assert(kOpenCache == 2, "DepoStream holds two open-shell slots");

// the walk's state of ray i from / to the stream arrays; false: not started
TORJ_HD bool depo_load(const DepoStream &ds, size_t n, int i, Walker<kOpenCache> &W, WalkCarry &C) {
    const int j = ds.v[kDsJ * n + i];
    if (j < 0) return false;
    const double *d = ds.d + i;
    const int *v = ds.v + i;
    W.Fhi = d[kDsFhi * n], W.Flo = d[kDsFlo * n];
    W.oF[0] = d[kDsOF0 * n], W.oF[1] = d[kDsOF1 * n];
    C.Ml = d[kDsMl * n], C.Mr = d[kDsMr * n], C.Mn = d[kDsMn * n];
    C.MPl = d[kDsMPl * n], C.MPr = d[kDsMPr * n], C.MPn = d[kDsMPn * n];
    C.yl = d[kDsYl * n], C.Pl = d[kDsPl * n];
    C.j = j;
    W.cur.c = v[kDsC * n];
    W.cur.load();
    W.oq[0] = v[kDsOQ0 * n], W.oq[1] = v[kDsOQ1 * n];
    W.spilled = v[kDsSpill * n] != 0;
    W.run_k0 = v[kDsRk0 * n], W.run_k1 = v[kDsRk1 * n], W.run_d = v[kDsRd * n];
    W.runs = v[kDsRuns * n], W.last_d = v[kDsLast * n];
    return true;
}
TORJ_HD void depo_save(const DepoStream &ds, size_t n, int i, const Walker<kOpenCache> &W, const WalkCarry &C) {
    double *d = ds.d + i;
    int *v = ds.v + i;
    d[kDsFhi * n] = W.Fhi, d[kDsFlo * n] = W.Flo;
    d[kDsOF0 * n] = W.oF[0], d[kDsOF1 * n] = W.oF[1];
    d[kDsMl * n] = C.Ml, d[kDsMr * n] = C.Mr, d[kDsMn * n] = C.Mn;
    d[kDsMPl * n] = C.MPl, d[kDsMPr * n] = C.MPr, d[kDsMPn * n] = C.MPn;
    d[kDsYl * n] = C.yl, d[kDsPl * n] = C.Pl;
    v[kDsC * n] = W.cur.c;
    v[kDsOQ0 * n] = W.oq[0], v[kDsOQ1 * n] = W.oq[1];
    v[kDsSpill * n] = W.spilled ? 1 : 0;
    v[kDsRk0 * n] = W.run_k0, v[kDsRk1 * n] = W.run_k1, v[kDsRd * n] = W.run_d;
    v[kDsRuns * n] = W.runs, v[kDsLast * n] = W.last_d;
    v[kDsJ * n] = C.j;
}

// every whole window whose rows lie at or above row `last` (points up to
// `last` available, last <= m - 2); returns whether the walk has started
TORJ_HD bool depo_windows(const RayData &R, Walker<kOpenCache> &W, WalkCarry &C, bool started, int last) {
    for (;;) {
        const int ja = started ? C.j : 0, jb = ja + kDepoQ, r0 = jb + 2 + kDepoW;
        if (r0 + 1 > last) break;
        nak_eliminate_rows(R, started ? ja + 3 : 1, r0);
        if (!started) {
            walk_start(W, R, C);
            started = true;
        }
        walk_segments(W, R, C, jb);
    }
    return started;
}

// k_depo_stream: ray i's windows over its first S steps (the scan has passed
// them and the ray is still running, so its end point lies beyond them)
TORJ_HD void fit_depo_stream(const FitArgs &a, const DepoStream &ds, int i, double psiL, int S) {
    if (!(a.s0[i] > 0.0)) return;
    const int j = ds.v[kDsJ * (size_t)a.n + i];
    if ((j < 0 ? 0 : j) + kDepoQ + 3 + kDepoW > S) return;  // no new window yet
    RayData R{&a, i, S + 2, a.s0[i], psiL};
    Walker<kOpenCache> W{&a, i, 0.0, 0.0, Cursor{&a, 0, 0.0, 0.0}};
    W.init();
    WalkCarry C{};
    const bool started = depo_load(ds, a.n, i, W, C);
    if (depo_windows(R, W, C, started, S)) depo_save(ds, a.n, i, W, C);
}

// The split form of one streamed window (TORJ_DEPO_STREAM=3): the elimination
// and the walk of ray i's next window in two launches, so the elimination's
// latency-bound rows run in a small-register kernel beside the alpha waves
// and only the walk needs the large one.  At most one window per launch pair
// (the windows are schedule-independent; k_depo_tail takes what is left).
// The next window of ray i, if the scan's S steps cover it:
TORJ_HD bool depo_next_window(const DepoStream &ds, size_t n, int i, int S, int &ja, bool &started) {
    const int j = ds.v[kDsJ * n + i];
    started = j >= 0;
    ja = started ? j : 0;
    return ja + kDepoQ + 3 + kDepoW <= S;  // depo_windows' test with last = S
}
// k_depo_elim: the next window's rows of the elimination
TORJ_HD void fit_depo_stream_elim(const FitArgs &a, const DepoStream &ds, int i, double psiL, int S) {
    if (!(a.s0[i] > 0.0)) return;
    int ja;
    bool started;
    if (!depo_next_window(ds, a.n, i, S, ja, started)) return;
    RayData R{&a, i, S + 2, a.s0[i], psiL};
    nak_eliminate_rows(R, started ? ja + 3 : 1, ja + kDepoQ + 2 + kDepoW);
}
// k_depo_walk: that window's walk, after k_depo_elim on the same S
TORJ_HD void fit_depo_stream_walk(const FitArgs &a, const DepoStream &ds, int i, double psiL, int S) {
    if (!(a.s0[i] > 0.0)) return;
    int ja;
    bool started;
    if (!depo_next_window(ds, a.n, i, S, ja, started)) return;
    RayData R{&a, i, S + 2, a.s0[i], psiL};
    Walker<kOpenCache> W{&a, i, 0.0, 0.0, Cursor{&a, 0, 0.0, 0.0}};
    W.init();
    WalkCarry C{};
    if (started)
        depo_load(ds, a.n, i, W, C);
    else
        walk_start(W, R, C);
    // (a form reading the next segment's five values while this one is
    // walked spilled at three waves per SIMD and was no faster at three or two,
    // DESIGN.md 3.4, round 5)
    walk_segments<kWalkChunkStream>(W, R, C, ja + kDepoQ);
    depo_save(ds, a.n, i, W, C);
}

// k_depo_tail: the windows still left, the exact rest of the ray, the finish
TORJ_HD void fit_depo_tail(const FitArgs &a, const DepoStream &ds, int i, double psiL) {
    const int m = a.steps[i] + 2;
    if (m < 4 || !(a.s0[i] > 0.0)) {  // as fit_depo_ray (no window ever ran for such a ray)
        a.kstar[i] = a.n_psi;
        a.Pray[i] = 0.0;
        return;
    }
    RayData R{&a, i, m, a.s0[i], psiL};
    Walker<kOpenCache> W{&a, i, 0.0, 0.0, Cursor{&a, 0, 0.0, 0.0}};
    W.init();
    WalkCarry C{};
    bool started = depo_load(ds, a.n, i, W, C);
    started = depo_windows(R, W, C, started, m - 2);
    nak_eliminate_rows(R, started ? C.j + 3 : 1, m - 2);
    if (!started) walk_start(W, R, C);
    walk_segments(W, R, C, m - 1);
    fit_depo_finish(a, i, R, W);
}

}  // namespace torj
