// torj_entry.hpp -- ray entry: first_point + vacuum_plasma_refraction
// (src/solve.jl:7-74, checks of make_ray :138-141), one implementation for the
// host ABI (torj_ray_entry, OpenMP) and the GPU kernel (k_ray_entry, one lane
// per ray).
#pragma once
#include "torj_math.hpp"

namespace torj {

// IMAS.toroidal_intersection for the grid rectangle (src/solve.jl:22-24):
// smallest t > 0 at which p0 + t v meets the surface of revolution of the
// closed polygon (R_k, Z_k).  Parity unpinned (IMAS not available).
TORJ_HD double toroidal_intersection(const double *Rp, const double *Zp, int np, const double p0[3],
                                     const double v[3]) {
    double best = INFINITY;
    for (int s = 0; s + 1 < np; s++) {
        const double Ra = Rp[s], Za = Zp[s], Rb = Rp[s + 1], Zb = Zp[s + 1];
        if (Zb == Za) {  // annulus in a z-plane
            if (v[2] == 0.0) continue;
            const double t = (Za - p0[2]) / v[2];
            if (!(t > 0)) continue;
            const double x = p0[0] + t * v[0], y = p0[1] + t * v[1];
            const double R = sqrt(x * x + y * y);
            if (R >= fmin(Ra, Rb) && R <= fmax(Ra, Rb)) best = fmin(best, t);
            continue;
        }
        // cone through the segment: R(t) = al + be t with R(t)^2 = x(t)^2 + y(t)^2
        const double k = (Rb - Ra) / (Zb - Za);
        const double al = Ra + (p0[2] - Za) * k, be = v[2] * k;
        const double A = v[0] * v[0] + v[1] * v[1] - be * be;
        const double B = 2.0 * (p0[0] * v[0] + p0[1] * v[1] - al * be);
        const double C = p0[0] * p0[0] + p0[1] * p0[1] - al * al;
        double ts[2];
        int nt = 0;
        if (fabs(A) < 1e-300) {
            if (B != 0) ts[nt++] = -C / B;
        } else {
            const double disc = B * B - 4 * A * C;
            if (disc >= 0) {
                const double sq = sqrt(disc);
                ts[nt++] = (-B - sq) / (2 * A);
                ts[nt++] = (-B + sq) / (2 * A);
            }
        }
        for (int q = 0; q < nt; q++) {
            const double t = ts[q];
            if (!(t > 0)) continue;
            const double sp = (p0[2] + t * v[2] - Za) / (Zb - Za);
            if (sp < 0 || sp > 1 || al + be * t < 0) continue;
            best = fmin(best, t);
        }
    }
    return best;
}

TORJ_HD double psi_at(const double *coef, const Grid &g, const double x[3]) {
    return eval_one(coef, g, sqrt(x[0] * x[0] + x[1] * x[1]), x[2], F_PSI);
}

// first_point (src/solve.jl:7-38): the launch point moved onto the grid
// boundary (if off-grid), then along N0 to psi = psi_prof_max.
TORJ_HD int first_point(const double *coef, const Grid &g, double psi_max, const double x0[3],
                        const double N0[3], double out[3]) {
    double pp[3] = {x0[0], x0[1], x0[2]};
    const double R0 = sqrt(x0[0] * x0[0] + x0[1] * x0[1]);
    const bool on_grid = g.R1 <= R0 && R0 <= g.Rn && g.Z1 <= x0[2] && x0[2] <= g.Zn;  // :7-11
    if (!on_grid) {
        const double Rp[5] = {g.R1, g.Rn, g.Rn, g.R1, g.R1};
        const double Zp[5] = {g.Z1, g.Z1, g.Zn, g.Zn, g.Z1};
        const double t = toroidal_intersection(Rp, Zp, 5, x0, N0);
        if (!isfinite(t)) return ST_ENTRY_FAIL;
        for (int k = 0; k < 3; k++) pp[k] = x0[k] + N0[k] * t;
    }
    auto G = [&](double t) {
        const double q[3] = {pp[0] + t * N0[0], pp[1] + t * N0[1], pp[2] + t * N0[2]};
        return psi_at(coef, g, q) - psi_max;
    };
    // find_zero(g, (0, 0.5), Bisection()) (:29), bisected to machine precision
    double a = 0.0, b = 0.5, ga = G(a), gb = G(b);
    if (ga != 0.0 && gb != 0.0) {
        if ((ga > 0) == (gb > 0)) return ST_ENTRY_FAIL;
        for (int it = 0; it < 200; it++) {
            const double m = 0.5 * (a + b);
            if (m <= a || m >= b) break;
            const double gm = G(m);
            if (gm == 0.0) {
                a = b = m;
                ga = gb = 0.0;
                break;
            }
            if ((gm > 0) == (ga > 0)) {
                a = m;
                ga = gm;
            } else {
                b = m;
                gb = gm;
            }
        }
    }
    const double t = (fabs(ga) <= fabs(gb)) ? a : b;
    for (int k = 0; k < 3; k++) pp[k] += t * N0[k];
    const double psi_ref = psi_at(coef, g, pp);
    if (!(fabs(psi_ref - psi_max) < 1e-6)) return ST_ENTRY_FAIL;  // :32
    if (psi_ref > psi_max)                                        // :33-36
        for (int k = 0; k < 3; k++) pp[k] += 2.0 * (psi_ref - psi_max) * N0[k];
    for (int k = 0; k < 3; k++) out[k] = pp[k];
    return ST_OK;
}

TORJ_HD void plasma_xyb(const double *coef, const Grid &g, double omega, const double x[3],
                        double &X, double &Y, double b[3]) {
    PlasmaPoint pt;
    plasma_point<false>(coef, g, make_consts(omega), x, pt);
    X = pt.X;
    Y = pt.Y;
    for (int k = 0; k < 3; k++) b[k] = pt.b[k];
}

// vacuum_plasma_refraction (src/solve.jl:40-74).  The 3 refraction equations
// (:40-49) have the root N = n0 + (cos_i - sqrt(q^2 - sin_i^2)) n with
// q^2 = N_s^2(N.b): solved as a scalar Newton iteration in q.
TORJ_HD int refraction(const double *coef, const Grid &g, const double pp[3], const double N0[3],
                       double omega, int mode, double N[3]) {
    double X, Y, b[3];
    plasma_xyb(coef, g, omega, pp, X, Y, b);
    const double Nest = refractive_index_sq(X, Y, 0.0, mode);
    if (Nest <= 0) return ST_REFLECTED;  // :57-59
    double q = sqrt(Nest);
    const double R = sqrt(pp[0] * pp[0] + pp[1] * pp[1]);
    double v, dR, dZ;
    eval_grad_one(coef, g, R, pp[2], F_PSI, v, dR, dZ);
    double n[3] = {dR * pp[0] / R, dR * pp[1] / R, dZ};
    const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int k = 0; k < 3; k++) n[k] /= nn;
    const double n0n = sqrt(N0[0] * N0[0] + N0[1] * N0[1] + N0[2] * N0[2]);
    const double n0[3] = {N0[0] / n0n, N0[1] / n0n, N0[2] / n0n};
    const double ci = -(n[0] * n0[0] + n[1] * n0[1] + n[2] * n0[2]);
    const double si2 = 1.0 - ci * ci;
    const double nb = n[0] * b[0] + n[1] * b[1] + n[2] * b[2];
    const double n0b = n0[0] * b[0] + n0[1] * b[1] + n0[2] * b[2];
    auto resid = [&](double qq, bool &ok) {
        const double rt = qq * qq - si2;
        ok = rt >= 0;
        if (!ok) return 0.0;
        const double np = n0b + (ci - sqrt(rt)) * nb;
        return qq * qq - refractive_index_sq(X, Y, np, mode);
    };
    for (int it = 0; it < 100; it++) {
        bool ok;
        const double r = resid(q, ok);
        if (!ok) return ST_REFLECTED;
        const double h = 1e-7 * q;
        bool o1, o2;
        const double dr = (resid(q + h, o1) - resid(q - h, o2)) / (2 * h);
        if (!o1 || !o2 || !(dr != 0)) return ST_ENTRY_FAIL;
        const double dq = r / dr;
        q -= dq;
        if (fabs(dq) <= 1e-16 * q) break;
    }
    const double s = sqrt(q * q - si2);
    for (int k = 0; k < 3; k++) N[k] = n0[k] + (ci - s) * n[k];
    return ST_OK;
}

// One ray: start state in the plasma, vacuum path length s0 and status, with
// make_ray's assertions (src/solve.jl:138, :141) as statuses.
TORJ_HD int ray_entry_one(const double *coef, const Grid &g, double psi_max, const double a[3],
                          const double d[3], double omega, int mode, double xo[3], double No[3],
                          double &s0) {
    for (int k = 0; k < 3; k++) xo[k] = No[k] = NAN;
    int st = first_point(coef, g, psi_max, a, d, xo);
    if (st == ST_OK && !(psi_at(coef, g, xo) <= psi_max)) st = ST_ENTRY_FAIL;  // :138
    if (st == ST_OK) st = refraction(coef, g, xo, d, omega, mode, No);
    if (st == ST_OK) {  // :141 |D| < 1e-12
        double X, Y, b[3];
        plasma_xyb(coef, g, omega, xo, X, Y, b);
        const double Npar = No[0] * b[0] + No[1] * b[1] + No[2] * b[2];
        const double D = No[0] * No[0] + No[1] * No[1] + No[2] * No[2] -
                         refractive_index_sq(X, Y, Npar, mode);
        if (!(fabs(D) < 1e-12)) st = ST_ENTRY_FAIL;
    }
    s0 = sqrt((xo[0] - a[0]) * (xo[0] - a[0]) + (xo[1] - a[1]) * (xo[1] - a[1]) +
              (xo[2] - a[2]) * (xo[2] - a[2]));
    return st;
}

}  // namespace torj
