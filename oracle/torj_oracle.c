/*
 * torj_oracle.c -- CPU restatement of TorJ.jl's ray-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline peer).  Nothing in the
 * product (libtorj_hip.so / torj_hip) links or calls this file.
 *
 * Parity: unpinned against an executed reference (no Julia in the container,
 * reference golden data is an unfetchable network artifact).  Pinned against
 * the reference's data-free launch-weight test and against independent
 * implementations (scipy/numpy) -- see DESIGN.md "Oracle".
 *
 * Deliberately written as a literal restatement: ForwardDiff gradients are
 * reproduced with forward-mode dual numbers (3 partials, like ForwardDiff's
 * chunk-3 gradient), the Albajar polarisation vector uses C99 complex numbers
 * like the reference's ComplexF64, and Bessel functions come from libm jn()
 * (an algorithm independent of the GPU's power series).
 */
#include "torj_oracle.h"

#include <complex.h>
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI 3.14159265358979323846

/* ------------------------------------------------------------------------- */
/* forward-mode dual numbers (ForwardDiff.Dual with 3 partials)               */
/* ------------------------------------------------------------------------- */
typedef struct {
    double v, d[3];
} dual;

static inline dual dc(double v) {
    dual r = {v, {0, 0, 0}};
    return r;
}
static inline dual dvar(double v, int k) {
    dual r = dc(v);
    r.d[k] = 1.0;
    return r;
}
static inline dual dadd(dual a, dual b) {
    dual r = {a.v + b.v, {a.d[0] + b.d[0], a.d[1] + b.d[1], a.d[2] + b.d[2]}};
    return r;
}
static inline dual dsub(dual a, dual b) {
    dual r = {a.v - b.v, {a.d[0] - b.d[0], a.d[1] - b.d[1], a.d[2] - b.d[2]}};
    return r;
}
static inline dual dmul(dual a, dual b) {
    dual r;
    r.v = a.v * b.v;
    for (int k = 0; k < 3; k++) r.d[k] = a.d[k] * b.v + a.v * b.d[k];
    return r;
}
static inline dual ddiv(dual a, dual b) {
    dual r;
    r.v = a.v / b.v;
    for (int k = 0; k < 3; k++) r.d[k] = (a.d[k] * b.v - a.v * b.d[k]) / (b.v * b.v);
    return r;
}
static inline dual dscale(dual a, double s) {
    dual r = {a.v * s, {a.d[0] * s, a.d[1] * s, a.d[2] * s}};
    return r;
}
static inline dual daddc(dual a, double s) {
    a.v += s;
    return a;
}
static inline dual dcsub(double s, dual a) { /* s - a */
    dual r = {s - a.v, {-a.d[0], -a.d[1], -a.d[2]}};
    return r;
}
static inline dual dsq(dual a) { return dmul(a, a); }
static inline dual dsqrt(dual a) {
    dual r;
    r.v = sqrt(a.v);
    for (int k = 0; k < 3; k++) r.d[k] = a.d[k] / (2.0 * r.v);
    return r;
}
static inline dual dexp(dual a) {
    dual r;
    r.v = exp(a.v);
    for (int k = 0; k < 3; k++) r.d[k] = a.d[k] * r.v;
    return r;
}
static inline dual dcos(dual a) {
    dual r;
    r.v = cos(a.v);
    double s = -sin(a.v);
    for (int k = 0; k < 3; k++) r.d[k] = a.d[k] * s;
    return r;
}
static inline dual dsin(dual a) {
    dual r;
    r.v = sin(a.v);
    double c = cos(a.v);
    for (int k = 0; k < 3; k++) r.d[k] = a.d[k] * c;
    return r;
}
static inline dual dhypot(dual a, dual b) {
    dual r;
    r.v = hypot(a.v, b.v);
    for (int k = 0; k < 3; k++) r.d[k] = (a.v * a.d[k] + b.v * b.d[k]) / r.v;
    return r;
}
static inline dual datan2(dual y, dual x) {
    dual r;
    r.v = atan2(y.v, x.v);
    double den = x.v * x.v + y.v * y.v;
    for (int k = 0; k < 3; k++) r.d[k] = (x.v * y.d[k] - y.v * x.d[k]) / den;
    return r;
}

/* ------------------------------------------------------------------------- */
/* quadrature                                                                 */
/* ------------------------------------------------------------------------- */
/* FastGaussQuadrature.gausslegendre(n): ascending nodes on [-1,1]
 * (called from src/absorption.jl:4).  Newton on the 3-term recurrence. */
void or_gauss_legendre(int n, double *x, double *w) {
    int m = (n + 1) / 2;
    for (int i = 0; i < m; i++) {
        double z = cos(PI * (i + 0.75) / (n + 0.5)), z1, pp = 0;
        for (int it = 0; it < 100; it++) {
            double p1 = 1.0, p2 = 0.0;
            for (int j = 1; j <= n; j++) {
                double p3 = p2;
                p2 = p1;
                p1 = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
            }
            pp = n * (z * p1 - p2) / (z * z - 1.0);
            z1 = z;
            z = z1 - p1 / pp;
            if (fabs(z - z1) < 1e-16) break;
        }
        x[i] = -z;
        x[n - 1 - i] = z;
        w[i] = w[n - 1 - i] = 2.0 / ((1.0 - z * z) * pp * pp);
    }
}

/* Orthonormal Hermite recurrence p_0 = pi^(-1/4), p_{j+1} = z sqrt(2/(j+1)) p_j -
 * sqrt(j/(j+1)) p_{j-1}, rescaled by 2^-500 whenever it grows past 2^500 (the
 * exponent is returned in *e2): overflow-free for any n. */
static void herm_rec(int n, double z, double *pn, double *pn1, int *e2) {
    double p1 = 0.7511255444649425, p2 = 0.0;
    int e = 0;
    for (int j = 0; j < n; j++) {
        double p3 = p2;
        p2 = p1;
        p1 = z * sqrt(2.0 / (j + 1)) * p2 - sqrt((double)j / (j + 1)) * p3;
        if (fabs(p1) > 0x1p500) {
            p1 = ldexp(p1, -500);
            p2 = ldexp(p2, -500);
            e += 500;
        }
    }
    *pn = p1;
    *pn1 = p2;
    *e2 = e;
}

/* FastGaussQuadrature.gausshermite(n): ascending nodes, weight exp(-x^2)
 * (called from src/launch.jl:72).  Positive zeros bracketed by sign changes on
 * a grid finer than the smallest zero spacing (~pi/sqrt(2n+1), near the
 * origin), bisected, then Newton-polished; w = 2 / (2n p_{n-1}^2). */
void or_gauss_hermite(int n, double *x, double *w) {
    int half = n / 2, k = 0;
    double *pos = (double *)malloc(sizeof(double) * (half + 1));
    double *pw = (double *)malloc(sizeof(double) * (half + 1));
    const double zmax = sqrt(2.0 * n + 1.0) + 1.0;
    const double dz = 0.2 * PI / sqrt(2.0 * n + 1.0);
    double a = (n & 1) ? 0.5 * dz : 0.0, fa, fa1;
    int ea;
    herm_rec(n, a, &fa, &fa1, &ea);
    while (k < half && a < zmax) {
        double b = a + dz, fb, fb1;
        int eb;
        herm_rec(n, b, &fb, &fb1, &eb);
        if ((fa > 0) != (fb > 0) && fb != 0.0) {
            double lo = a, hi = b, flo = fa;
            for (int it = 0; it < 60; it++) {
                double m = 0.5 * (lo + hi), fm, fm1;
                int em;
                herm_rec(n, m, &fm, &fm1, &em);
                if ((fm > 0) == (flo > 0)) {
                    lo = m;
                    flo = fm;
                } else {
                    hi = m;
                }
            }
            double z = 0.5 * (lo + hi), pn, pn1;
            int e;
            for (int it = 0; it < 3; it++) {
                herm_rec(n, z, &pn, &pn1, &e);
                z -= pn / (sqrt(2.0 * n) * pn1);
            }
            herm_rec(n, z, &pn, &pn1, &e);
            pos[k] = z;
            pw[k] = ldexp(1.0 / (n * pn1 * pn1), -2 * e);
            k++;
        }
        a = b;
        fa = fb;
    }
    int m = 0;
    for (int i = k - 1; i >= 0; i--, m++) {
        x[m] = -pos[i];
        w[m] = pw[i];
    }
    if (n & 1) {
        double pn, pn1;
        int e;
        herm_rec(n, 0.0, &pn, &pn1, &e);
        x[m] = 0.0;
        w[m] = ldexp(1.0 / (n * pn1 * pn1), -2 * e);
        m++;
    }
    for (int i = 0; i < k; i++, m++) {
        x[m] = pos[i];
        w[m] = pw[i];
    }
    free(pos);
    free(pw);
}

/* ------------------------------------------------------------------------- */
/* cubic B-splines, Interpolations.jl BSpline(Cubic(Line(OnGrid())))         */
/* ------------------------------------------------------------------------- */
/* Dense LU (partial pivoting) of the (n+2)x(n+2) prefilter system:
 *   row 0     : c0 - 2 c1 + c2 = 0                   (Line(OnGrid): f''=0)
 *   row i     : c_{i-1}/6 + 2 c_i/3 + c_{i+1}/6 = y_i (i = 1..n)
 *   row n+1   : c_{n-1} - 2 c_n + c_{n+1} = 0
 * i.e. Interpolations' prefiltering_system for Cubic{Line{OnGrid}}. */
typedef struct {
    int m;
    double *a; /* m*m row-major LU */
    int *piv;
} lu_t;

static void lu_build(lu_t *L, int n) {
    int m = n + 2;
    L->m = m;
    L->a = (double *)calloc((size_t)m * m, sizeof(double));
    L->piv = (int *)malloc(sizeof(int) * m);
    double *A = L->a;
    A[0 * m + 0] = 1.0;
    A[0 * m + 1] = -2.0;
    A[0 * m + 2] = 1.0;
    for (int i = 1; i <= n; i++) {
        A[i * m + i - 1] = 1.0 / 6.0;
        A[i * m + i] = 2.0 / 3.0;
        A[i * m + i + 1] = 1.0 / 6.0;
    }
    A[(m - 1) * m + m - 3] = 1.0;
    A[(m - 1) * m + m - 2] = -2.0;
    A[(m - 1) * m + m - 1] = 1.0;
    for (int k = 0; k < m; k++) {
        int p = k;
        for (int i = k + 1; i < m; i++)
            if (fabs(A[i * m + k]) > fabs(A[p * m + k])) p = i;
        L->piv[k] = p;
        if (p != k)
            for (int j = 0; j < m; j++) {
                double t = A[k * m + j];
                A[k * m + j] = A[p * m + j];
                A[p * m + j] = t;
            }
        for (int i = k + 1; i < m; i++) {
            double f = A[i * m + k] / A[k * m + k];
            A[i * m + k] = f;
            for (int j = k + 1; j < m; j++) A[i * m + j] -= f * A[k * m + j];
        }
    }
}

static void lu_solve(const lu_t *L, double *b) {
    int m = L->m;
    const double *A = L->a;
    for (int k = 0; k < m; k++) { /* row interchanges first (LAPACK getrs order) */
        int p = L->piv[k];
        if (p != k) {
            double t = b[k];
            b[k] = b[p];
            b[p] = t;
        }
    }
    for (int k = 0; k < m; k++)
        for (int i = k + 1; i < m; i++) b[i] -= A[i * m + k] * b[k];
    for (int i = m - 1; i >= 0; i--) {
        double s = b[i];
        for (int j = i + 1; j < m; j++) s -= A[i * m + j] * b[j];
        b[i] = s / A[i * m + i];
    }
}

static void lu_free(lu_t *L) {
    free(L->a);
    free(L->piv);
}

void or_bspl1d_prefilter(int n, const double *y, double *c) {
    lu_t L;
    lu_build(&L, n);
    c[0] = 0.0;
    for (int i = 0; i < n; i++) c[i + 1] = y[i];
    c[n + 1] = 0.0;
    lu_solve(&L, c);
    lu_free(&L);
}

/* tensor-product prefilter: dim 1 (R) then dim 2 (Z); y is nR x nZ, R fastest */
void or_bspl2d_prefilter(int nR, int nZ, const double *y, double *c) {
    int mR = nR + 2, mZ = nZ + 2;
    lu_t LR, LZ;
    lu_build(&LR, nR);
    lu_build(&LZ, nZ);
    double *col = (double *)malloc(sizeof(double) * (mR > mZ ? mR : mZ));
    memset(c, 0, sizeof(double) * (size_t)mR * mZ);
    for (int j = 0; j < nZ; j++) {
        col[0] = 0.0;
        for (int i = 0; i < nR; i++) col[i + 1] = y[(size_t)j * nR + i];
        col[nR + 1] = 0.0;
        lu_solve(&LR, col);
        for (int i = 0; i < mR; i++) c[(size_t)(j + 1) * mR + i] = col[i];
    }
    for (int i = 0; i < mR; i++) {
        for (int j = 0; j < mZ; j++) col[j] = c[(size_t)j * mR + i];
        lu_solve(&LZ, col);
        for (int j = 0; j < mZ; j++) c[(size_t)j * mR + i] = col[j];
    }
    free(col);
    lu_free(&LR);
    lu_free(&LZ);
}

/* value_weights / gradient_weights of Interpolations' Cubic degree */
static inline void bw(double d, double w[4], double dw[4]) {
    double p = 1.0 - d;
    w[0] = p * p * p / 6.0;
    w[1] = 2.0 / 3.0 - d * d + 0.5 * d * d * d;
    w[2] = 2.0 / 3.0 - p * p + 0.5 * p * p * p;
    w[3] = d * d * d / 6.0;
    dw[0] = -0.5 * p * p;
    dw[1] = -2.0 * d + 1.5 * d * d;
    dw[2] = 2.0 * p - 1.5 * p * p;
    dw[3] = 0.5 * d * d;
}

static inline int cell(double u, int n) {
    int i = (int)floor(u);
    if (i < 0) i = 0;
    if (i > n - 2) i = n - 2;
    return i;
}

static inline double clampd(double x, double lo, double hi) {
    return x > hi ? hi : (x < lo ? lo : x);
}

double or_spl1d_eval(const or_spl1d *s, double x) {
    double xc = clampd(x, s->x1, s->xn);
    double u = (xc - s->x1) / s->h;
    int i = cell(u, s->n);
    double w[4], dw[4];
    bw(u - i, w, dw);
    double v = 0, g = 0;
    for (int a = 0; a < 4; a++) {
        v += w[a] * s->coef[i + a];
        g += dw[a] * s->coef[i + a];
    }
    g /= s->h;
    return v + (x - xc) * g;
}

double or_spl1d_deriv(const or_spl1d *s, double x) {
    double xc = clampd(x, s->x1, s->xn);
    double u = (xc - s->x1) / s->h;
    int i = cell(u, s->n);
    double w[4], dw[4];
    bw(u - i, w, dw);
    double g = 0;
    for (int a = 0; a < 4; a++) g += dw[a] * s->coef[i + a];
    return g / s->h;
}

static void spl2d_vgrad(const or_spl2d *s, double Rc, double Zc, double *v, double *gR,
                        double *gZ) {
    int mR = s->nR + 2;
    double uR = (Rc - s->R1) / s->hR, uZ = (Zc - s->Z1) / s->hZ;
    int iR = cell(uR, s->nR), iZ = cell(uZ, s->nZ);
    double wR[4], dwR[4], wZ[4], dwZ[4];
    bw(uR - iR, wR, dwR);
    bw(uZ - iZ, wZ, dwZ);
    double sv = 0, sR = 0, sZ = 0;
    for (int b = 0; b < 4; b++) {
        const double *row = s->coef + (size_t)(iZ + b) * mR + iR;
        double rv = 0, rd = 0;
        for (int a = 0; a < 4; a++) {
            rv += wR[a] * row[a];
            rd += dwR[a] * row[a];
        }
        sv += wZ[b] * rv;
        sR += wZ[b] * rd;
        sZ += dwZ[b] * rv;
    }
    *v = sv;
    *gR = sR / s->hR;
    *gZ = sZ / s->hZ;
}

double or_spl2d_eval(const or_spl2d *s, double R, double Z) {
    double Rc = clampd(R, s->R1, s->Rn), Zc = clampd(Z, s->Z1, s->Zn);
    double v, gR, gZ;
    spl2d_vgrad(s, Rc, Zc, &v, &gR, &gZ);
    return v + (R - Rc) * gR + (Z - Zc) * gZ;
}

/* Interpolations.gradient(itp, R, Z) (used at src/solve.jl:63); the reference
 * calls it on the extrapolated object: outside the box the gradient of the
 * Line extension is evaluated at the clamped point. */
void or_spl2d_grad(const or_spl2d *s, double R, double Z, double *dR, double *dZ) {
    double Rc = clampd(R, s->R1, s->Rn), Zc = clampd(Z, s->Z1, s->Zn);
    double v;
    spl2d_vgrad(s, Rc, Zc, &v, dR, dZ);
}

/* Extrapolation(Line) evaluated with dual coordinates: exactly what ForwardDiff
 * sees when it differentiates spl(hypot(x,y), z) (src/plasma.jl:61-65). */
static dual spl2d_eval_dual(const or_spl2d *s, dual R, dual Z) {
    dual Rc = (R.v > s->Rn) ? dc(s->Rn) : (R.v < s->R1 ? dc(s->R1) : R);
    dual Zc = (Z.v > s->Zn) ? dc(s->Zn) : (Z.v < s->Z1 ? dc(s->Z1) : Z);
    int mR = s->nR + 2;
    dual uR = ddiv(daddc(Rc, -s->R1), dc(s->hR));
    dual uZ = ddiv(daddc(Zc, -s->Z1), dc(s->hZ));
    int iR = cell(uR.v, s->nR), iZ = cell(uZ.v, s->nZ);
    dual dR = daddc(uR, -(double)iR), dZ = daddc(uZ, -(double)iZ);
    /* weights as duals */
    dual wR[4], dwR[4], wZ[4], dwZ[4];
    dual pR = dcsub(1.0, dR), pZ = dcsub(1.0, dZ);
#define BW_DUAL(d, p, w, dw)                                                          \
    do {                                                                              \
        w[0] = dscale(dmul(dmul(p, p), p), 1.0 / 6.0);                                \
        w[1] = dadd(dcsub(2.0 / 3.0, dmul(d, d)), dscale(dmul(dmul(d, d), d), 0.5));  \
        w[2] = dadd(dcsub(2.0 / 3.0, dmul(p, p)), dscale(dmul(dmul(p, p), p), 0.5));  \
        w[3] = dscale(dmul(dmul(d, d), d), 1.0 / 6.0);                                \
        dw[0] = dscale(dmul(p, p), -0.5);                                             \
        dw[1] = dadd(dscale(d, -2.0), dscale(dmul(d, d), 1.5));                       \
        dw[2] = dsub(dscale(p, 2.0), dscale(dmul(p, p), 1.5));                        \
        dw[3] = dscale(dmul(d, d), 0.5);                                              \
    } while (0)
    BW_DUAL(dR, pR, wR, dwR);
    BW_DUAL(dZ, pZ, wZ, dwZ);
#undef BW_DUAL
    dual sv = dc(0), sR = dc(0), sZ = dc(0);
    for (int b = 0; b < 4; b++) {
        const double *row = s->coef + (size_t)(iZ + b) * mR + iR;
        dual rv = dc(0), rd = dc(0);
        for (int a = 0; a < 4; a++) {
            rv = dadd(rv, dscale(wR[a], row[a]));
            rd = dadd(rd, dscale(dwR[a], row[a]));
        }
        sv = dadd(sv, dmul(wZ[b], rv));
        sR = dadd(sR, dmul(wZ[b], rd));
        sZ = dadd(sZ, dmul(dwZ[b], rv));
    }
    dual gR = ddiv(sR, dc(s->hR)), gZ = ddiv(sZ, dc(s->hZ));
    return dadd(sv, dadd(dmul(dsub(R, Rc), gR), dmul(dsub(Z, Zc), gZ)));
}

/* ------------------------------------------------------------------------- */
/* natural cubic spline (IMAS.interp1d(x, y, :cubic); parity unpinned)       */
/* ------------------------------------------------------------------------- */
void or_natcubic(int n, const double *x, const double *y, int nq, const double *xq,
                 double *yq) {
    double *z = (double *)calloc(n, sizeof(double));
    if (n >= 3) {
        int m = n - 2;
        double *dg = (double *)malloc(sizeof(double) * m);
        double *rh = (double *)malloc(sizeof(double) * m);
        double *up = (double *)malloc(sizeof(double) * m);
        for (int i = 1; i <= m; i++) {
            double h0 = x[i] - x[i - 1], h1 = x[i + 1] - x[i];
            dg[i - 1] = 2.0 * (h0 + h1);
            up[i - 1] = h1;
            rh[i - 1] = 6.0 * ((y[i + 1] - y[i]) / h1 - (y[i] - y[i - 1]) / h0);
        }
        /* Thomas; sub-diagonal of row i is h_{i} = x[i]-x[i-1] */
        for (int i = 1; i < m; i++) {
            double lo = x[i + 1] - x[i];
            double f = lo / dg[i - 1];
            dg[i] -= f * up[i - 1];
            rh[i] -= f * rh[i - 1];
        }
        z[m] = rh[m - 1] / dg[m - 1];
        for (int i = m - 1; i >= 1; i--) z[i] = (rh[i - 1] - up[i - 1] * z[i + 1]) / dg[i - 1];
        free(dg);
        free(rh);
        free(up);
    }
    for (int q = 0; q < nq; q++) {
        double t = xq[q];
        int i = 0;
        while (i < n - 2 && t > x[i + 1]) i++;
        if (t == x[i]) {
            yq[q] = y[i];
            continue;
        }
        if (t == x[i + 1]) {
            yq[q] = y[i + 1];
            continue;
        }
        double h = x[i + 1] - x[i], a = x[i + 1] - t, b = t - x[i];
        yq[q] = z[i] * a * a * a / (6.0 * h) + z[i + 1] * b * b * b / (6.0 * h) +
                (y[i + 1] / h - z[i + 1] * h / 6.0) * b + (y[i] / h - z[i] * h / 6.0) * a;
    }
    free(z);
}

/* ------------------------------------------------------------------------- */
/* Plasma constructor, src/plasma.jl:16-58                                    */
/* ------------------------------------------------------------------------- */
static void spl2d_init(or_spl2d *s, int nR, int nZ, const double *R, const double *Z,
                       const double *data) {
    s->nR = nR;
    s->nZ = nZ;
    s->R1 = R[0];
    s->Rn = R[nR - 1];
    s->Z1 = Z[0];
    s->Zn = Z[nZ - 1];
    s->hR = (s->Rn - s->R1) / (nR - 1);
    s->hZ = (s->Zn - s->Z1) / (nZ - 1);
    s->coef = (double *)malloc(sizeof(double) * (size_t)(nR + 2) * (nZ + 2));
    or_bspl2d_prefilter(nR, nZ, data, s->coef);
}

static void spl1d_init(or_spl1d *s, int n, double x1, double xn, const double *y) {
    s->n = n;
    s->x1 = x1;
    s->xn = xn;
    s->h = (xn - x1) / (n - 1);
    s->coef = (double *)malloc(sizeof(double) * (n + 2));
    or_bspl1d_prefilter(n, y, s->coef);
}

/* make_2d_prof_spline, src/plasma.jl:16-22 */
static void make_2d_prof_spline(or_spl2d *s, int nR, int nZ, const double *R,
                                const double *Z, int np, const double *psi,
                                const double *prof, const double *psi_norm) {
    double *pr = (double *)malloc(sizeof(double) * np);
    double *p2 = (double *)malloc(sizeof(double) * np);
    for (int i = 0; i < np; i++) pr[i] = psi[0] + (psi[np - 1] - psi[0]) * i / (np - 1.0);
    pr[np - 1] = psi[np - 1];
    or_natcubic(np, psi, prof, np, pr, p2);
    for (int i = 0; i < np; i++) p2[i] = log(p2[i]);
    or_spl1d s1;
    spl1d_init(&s1, np, psi[0], psi[np - 1], p2);
    double *d2 = (double *)malloc(sizeof(double) * (size_t)nR * nZ);
    for (size_t k = 0; k < (size_t)nR * nZ; k++) d2[k] = or_spl1d_eval(&s1, psi_norm[k]);
    spl2d_init(s, nR, nZ, R, Z, d2);
    free(d2);
    free(s1.coef);
    free(pr);
    free(p2);
}

int or_plasma_create(or_plasma *p, int nR, int nZ, const double *R, const double *Z,
                     const double *psi_norm, int n_prof, const double *psi_prof,
                     const double *ne_prof, const double *Te_prof, const double *Br,
                     const double *Bz, const double *Bphi, int n_eq, const double *eq_psi,
                     const double *eq_vol) {
    if (nR < 2 || nZ < 2 || n_prof < 2 || n_eq < 2) return -1;
    spl2d_init(&p->psi, nR, nZ, R, Z, psi_norm);
    make_2d_prof_spline(&p->lnne, nR, nZ, R, Z, n_prof, psi_prof, ne_prof, psi_norm);
    make_2d_prof_spline(&p->lnTe, nR, nZ, R, Z, n_prof, psi_prof, Te_prof, psi_norm);
    spl2d_init(&p->Br, nR, nZ, R, Z, Br);
    spl2d_init(&p->Bz, nR, nZ, R, Z, Bz);
    spl2d_init(&p->Bphi, nR, nZ, R, Z, Bphi);
    double *pr = (double *)malloc(sizeof(double) * n_eq);
    double *v2 = (double *)malloc(sizeof(double) * n_eq);
    for (int i = 0; i < n_eq; i++)
        pr[i] = eq_psi[0] + (eq_psi[n_eq - 1] - eq_psi[0]) * i / (n_eq - 1.0);
    pr[n_eq - 1] = eq_psi[n_eq - 1];
    or_natcubic(n_eq, eq_psi, eq_vol, n_eq, pr, v2);
    spl1d_init(&p->vol, n_eq, eq_psi[0], eq_psi[n_eq - 1], v2);
    free(pr);
    free(v2);
    double mx = psi_prof[0];
    for (int i = 1; i < n_prof; i++)
        if (psi_prof[i] > mx) mx = psi_prof[i];
    p->psi_prof_max = mx;
    return 0;
}

void or_plasma_free(or_plasma *p) {
    free(p->psi.coef);
    free(p->lnne.coef);
    free(p->lnTe.coef);
    free(p->Br.coef);
    free(p->Bz.coef);
    free(p->Bphi.coef);
    free(p->vol.coef);
    memset(p, 0, sizeof(*p));
}

/* ------------------------------------------------------------------------- */
/* field evaluation (dual), src/plasma.jl:61-89, src/dispersion.jl:7-15       */
/* ------------------------------------------------------------------------- */
static inline dual evaluate_d(const or_spl2d *s, const dual x[3]) {
    return spl2d_eval_dual(s, dhypot(x[0], x[1]), x[2]);
}

static void B_spline_d(const or_plasma *p, const dual x[3], dual B[3]) {
    dual Br = evaluate_d(&p->Br, x);
    dual Bp = evaluate_d(&p->Bphi, x);
    dual Bz = evaluate_d(&p->Bz, x);
    dual phi = datan2(x[1], x[0]);
    dual c = dcos(phi), s = dsin(phi);
    B[0] = dsub(dmul(Br, c), dmul(Bp, s));
    B[1] = dadd(dmul(Br, s), dmul(Bp, c));
    B[2] = Bz;
}

static inline dual norm3_d(const dual v[3]) {
    return dsqrt(dadd(dadd(dmul(v[0], v[0]), dmul(v[1], v[1])), dmul(v[2], v[2])));
}

static void eval_plasma_d(const or_plasma *p, const dual x[3], const dual N[3], double omega,
                          dual *X, dual *Y, dual *Npar, dual b[3]) {
    dual B[3];
    B_spline_d(p, x, B);
    dual Babs = norm3_d(B);
    for (int k = 0; k < 3; k++) b[k] = ddiv(B[k], Babs);
    *Npar = dadd(dadd(dmul(N[0], b[0]), dmul(N[1], b[1])), dmul(N[2], b[2]));
    dual ne = dexp(evaluate_d(&p->lnne, x));
    *X = ddiv(dscale(ne, OR_E * OR_E), dc(OR_EPS0 * OR_ME * omega * omega));
    *Y = ddiv(dscale(Babs, OR_E), dc(OR_ME * omega));
}

static dual refractive_index_sq_d(dual X, dual Y, dual Npar, int mode) {
    dual Np2 = dmul(Npar, Npar);
    dual Y2 = dmul(Y, Y);
    dual one_m = dcsub(1.0, Np2);
    dual Delta = dadd(dmul(one_m, one_m),
                      ddiv(dmul(dscale(Np2, 4.0), dcsub(1.0, X)), Y2)); /* dispersion.jl:21-23 */
    dual sq = dsqrt(Delta);
    dual num = dadd(daddc(dscale(sq, (double)mode), 1.0), Np2);
    dual den = dscale(daddc(dadd(X, Y2), -1.0), 2.0);
    return dadd(dcsub(1.0, X), dmul(dmul(ddiv(num, den), X), Y2)); /* dispersion.jl:29-32 */
}

static dual dispersion_d(const or_plasma *p, const dual x[3], const dual N[3], double omega,
                         int mode) {
    dual Nabs = norm3_d(N);
    dual X, Y, Npar, b[3];
    eval_plasma_d(p, x, N, omega, &X, &Y, &Npar, b);
    return dsub(dmul(Nabs, Nabs), refractive_index_sq_d(X, Y, Npar, mode));
}

double or_evaluate(const or_spl2d *s, const double x[3]) {
    return or_spl2d_eval(s, hypot(x[0], x[1]), x[2]);
}

void or_B_spline(const or_plasma *p, const double x[3], double B[3]) {
    dual xd[3] = {dc(x[0]), dc(x[1]), dc(x[2])}, Bd[3];
    B_spline_d(p, xd, Bd);
    for (int k = 0; k < 3; k++) B[k] = Bd[k].v;
}

double or_n_e(const or_plasma *p, const double x[3]) { return exp(or_evaluate(&p->lnne, x)); }
double or_T_e(const or_plasma *p, const double x[3]) { return exp(or_evaluate(&p->lnTe, x)); }

void or_eval_plasma(const or_plasma *p, const double x[3], const double N[3], double omega,
                    double *X, double *Y, double *Npar, double b[3]) {
    dual xd[3] = {dc(x[0]), dc(x[1]), dc(x[2])}, Nd[3] = {dc(N[0]), dc(N[1]), dc(N[2])};
    dual Xd, Yd, Nd_par, bd[3];
    eval_plasma_d(p, xd, Nd, omega, &Xd, &Yd, &Nd_par, bd);
    *X = Xd.v;
    *Y = Yd.v;
    *Npar = Nd_par.v;
    for (int k = 0; k < 3; k++) b[k] = bd[k].v;
}

double or_refractive_index_sq(double X, double Y, double Npar, int mode) {
    return refractive_index_sq_d(dc(X), dc(Y), dc(Npar), mode).v;
}

double or_dispersion_relation(const or_plasma *p, const double x[3], const double N[3],
                              double omega, int mode) {
    dual xd[3] = {dc(x[0]), dc(x[1]), dc(x[2])}, Nd[3] = {dc(N[0]), dc(N[1]), dc(N[2])};
    return dispersion_d(p, xd, Nd, omega, mode).v;
}

/* gradΛ! (src/solve.jl:85-93): two ForwardDiff gradients, normalisation by
 * |∂Λ/∂N|, sign flip of the spatial part. du = (dx/ds, dN/ds). */
void or_grad_lambda(const or_plasma *p, const double x[3], const double N[3], double omega,
                    int mode, double du[6]) {
    dual xd[3] = {dvar(x[0], 0), dvar(x[1], 1), dvar(x[2], 2)};
    dual Nc[3] = {dc(N[0]), dc(N[1]), dc(N[2])};
    dual Dx = dispersion_d(p, xd, Nc, omega, mode);
    dual xc[3] = {dc(x[0]), dc(x[1]), dc(x[2])};
    dual Nd[3] = {dvar(N[0], 0), dvar(N[1], 1), dvar(N[2], 2)};
    dual DN = dispersion_d(p, xc, Nd, omega, mode);
    for (int k = 0; k < 3; k++) {
        du[3 + k] = Dx.d[k];
        du[k] = DN.d[k];
    }
    double nrm = sqrt(du[0] * du[0] + du[1] * du[1] + du[2] * du[2]);
    for (int k = 0; k < 6; k++) du[k] /= nrm;
    for (int k = 3; k < 6; k++) du[k] = -du[k];
}

/* ------------------------------------------------------------------------- */
/* Albajar absorption, src/absorption.jl                                     */
/* ------------------------------------------------------------------------- */
static int g_n_gl = 0;
static double g_gl_x[256], g_gl_w[256];

/* abs_Al_init, src/absorption.jl:1-7 */
int or_abs_al_init(int n) {
    if (n < 1 || n > 256) return -1;
    or_gauss_legendre(n, g_gl_x, g_gl_w);
    g_n_gl = n;
    return 0;
}

/* abs_Al_N_with_pol_vec, src/absorption.jl:10-64 */
static double abs_al_n_with_pol_vec(double X, double Y, double cos_t, double sin_t, int mode,
                                    double complex e[3]) {
    e[0] = e[1] = e[2] = 0.0;
    if (X >= 1.0) return 0.0;
    double s2 = sin_t * sin_t, c2 = cos_t * cos_t;
    double rho = Y * Y * (s2 * s2) + 4.0 * (1.0 - X) * (1.0 - X) * c2;
    if (rho < 0.0) return 0.0;
    rho = sqrt(rho);
    double f = (2.0 * (1.0 - X)) / (2.0 * (1.0 - X) - Y * Y * s2 - (double)mode * Y * rho);
    double N = 1.0 - X * f;
    if (N < 0.0) return 0.0;
    N = sqrt(N);
    if (c2 < 1e-5 || 1.0 - s2 < 1e-5) {
        if (mode > 0) {
            e[1] = I * sqrt(1.0 / N);
            e[0] = (I * (1.0 / Y * (1.0 - (1.0 - Y * Y) * f))) * e[1];
        } else {
            e[2] = sqrt(1.0 / N);
        }
    } else {
        double den = 1.0 - X - N * N * s2;
        double g = 1.0 - (1.0 - Y * Y) * f;
        double ta = 1.0 + (((1.0 - X) * N * N * c2) / (den * den)) * 1.0 / (Y * Y) * (g * g);
        double a_sq = s2 * ta * ta;
        double tb = 1.0 + ((1.0 - X) / den) * 1.0 / (Y * Y) * (g * g);
        double b_sq = c2 * tb * tb;
        if (mode > 0)
            e[1] = I * sqrt(1.0 / (N * sqrt(a_sq + b_sq)));
        else
            e[1] = -I * sqrt(1.0 / (N * sqrt(a_sq + b_sq)));
        e[0] = (I * (1.0 / Y * g)) * e[1];
        e[2] = -((N * N * sin_t * cos_t) / den) * e[0];
    }
    return N;
}

/* abs_Al_pol_fact, src/absorption.jl:132-168 (pol_fact for a single node t) */
static double abs_al_pol_fact(double t, double omega_bar, double m_0, double N_par,
                              double N_perp, const double complex e[3], int m) {
    double md = (double)m;
    double x_m = N_perp * omega_bar * sqrt((md / m_0) * (md / m_0) - 1.0);
    double N_eff = (N_perp * N_par) / (1.0 - N_par * N_par);
    double complex Axz = e[0] + N_eff * e[2];
    double aAxz = cabs(Axz);
    double Axz_sq = aAxz * aAxz;
    double Re_Axz_ey = creal(I * Axz * conj(e[1]));
    double Re_Axz_ez = creal(Axz * conj(e[2]));
    double Re_ey_ez = creal(I * conj(e[1]) * e[2]);
    double aey = cabs(e[1]), aez = cabs(e[2]);
    double ey_sq = aey * aey, ez_sq = aez * aez;
    double arg = x_m * sqrt(1.0 - t * t);
    double Jl = jn(m - 1, arg), Jn = jn(m, arg), Ju = jn(m + 1, arg);
    double Jn2 = Jn * Jn;
    double deriv = arg / x_m * Jn * (Jl - Ju);
    double sq = sqrt(1.0 - N_par * N_par);
    double pol = (Axz_sq + ey_sq) * Jn2;
    pol += Re_Axz_ey * x_m / md * deriv;
    pol -= (arg / md) * (arg / md) * ey_sq * Jl * Ju;
    double q = x_m / (md * sq);
    pol += q * q * ez_sq * (t * t) * Jn2;
    pol += q * 2.0 * Re_Axz_ez * t * Jn2;
    pol += q * Re_ey_ez * t * x_m / md * deriv;
    double r = md / (N_perp * omega_bar);
    pol *= r * r;
    return pol;
}

/* abs_Al_integral_nume_fast, src/absorption.jl:170-189 */
static double abs_al_integral_nume_fast(double mu, double omega_bar, double m_0, double N_par,
                                        double N_perp, const double complex e[3], int m) {
    double md = (double)m;
    double sum = 0.0;
    double r = md / m_0;
    for (int i = 0; i < g_n_gl; i++) {
        double t = g_gl_x[i];
        double u_par = 1.0 / sqrt(1.0 - N_par * N_par) * (r * N_par + sqrt(r * r - 1.0) * t);
        double u_perp_sq = (r * r - 1.0) * (1.0 - t * t);
        double gamma = sqrt(1.0 + u_par * u_par + u_perp_sq);
        double pol = abs_al_pol_fact(t, omega_bar, m_0, N_par, N_perp, e, m);
        sum += g_gl_w[i] * pol * (-mu) * exp(mu * (1.0 - gamma));
    }
    double a = 1.0 / (1.0 + 105.0 / (128.0 * mu * mu) + 15.0 / (8.0 * mu));
    double s = sqrt(mu / (2.0 * PI));
    return sum * a * (s * s * s);
}

/* abs_Albajar_fast, src/absorption.jl:191-226.  Returns NaN if abs_Al_init was
 * never called (the reference throws ErrorException, :173-175). */
double or_abs_albajar_fast(double omega, double X, double Y, double N_abs, double N_par,
                           double Te, int mode) {
    if (Te < 20.0) return 0.0;
    double mu = OR_ME * OR_C * OR_C / (OR_E * Te);
    double omega_bar = 1.0 / Y;
    double c_abs = 0.0;
    double cos_t = N_par / N_abs;
    double sin_t = sin(acos(cos_t));
    double N_perp = sqrt(N_abs * N_abs - N_par * N_par);
    double complex e[3];
    double N_test = abs_al_n_with_pol_vec(X, Y, cos_t, sin_t, mode, e);
    if (isnan(N_test) || N_test <= 0.0 || N_test > 1.0) return 0.0;
    if (g_n_gl == 0) return NAN;
    double m_0 = sqrt(1.0 - N_par * N_par) * omega_bar;
    for (int m = 2; m <= 3; m++) {
        if ((double)m < m_0) continue;
        double c_abs_m = abs_al_integral_nume_fast(mu, omega_bar, m_0, N_par, N_perp, e, m);
        double r = (double)m / m_0;
        c_abs += sqrt(r * r - 1.0) * c_abs_m;
    }
    c_abs = -(c_abs * 2.0 * PI * PI / m_0);
    c_abs = c_abs * X * omega / (Y * OR_C);
    return c_abs;
}

/* α_approx, src/absorption.jl:228-235 */
/* |dD/dN| of D = |N|^2 - refractive_index_sq (src/dispersion.jl:34-39): the
 * normalisation of gradLambda (src/solve.jl:85-95); 1/|dD/dN| is the group-
 * velocity factor of the warm alpha (general_absorption.jl:1336, repair R4) */
double or_grad_norm(const or_plasma *p, const double x[3], const double N[3], double omega,
                    int mode) {
    dual xc[3] = {dc(x[0]), dc(x[1]), dc(x[2])};
    dual Nd[3] = {dvar(N[0], 0), dvar(N[1], 1), dvar(N[2], 2)};
    dual DN = dispersion_d(p, xc, Nd, omega, mode);
    return sqrt(DN.d[0] * DN.d[0] + DN.d[1] * DN.d[1] + DN.d[2] * DN.d[2]);
}

double or_alpha_approx(const or_plasma *p, const double x[3], const double N[3],
                       double omega, int mode) {
    double Nabs = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
    double X, Y, Npar, b[3];
    or_eval_plasma(p, x, N, omega, &X, &Y, &Npar, b);
    double Te = or_T_e(p, x);
    return or_abs_albajar_fast(omega, X, Y, Nabs, Npar, Te, mode);
}

/* ------------------------------------------------------------------------- */
/* launch fan, src/launch.jl:24-132                                          */
/* ------------------------------------------------------------------------- */
/* Julia's round(Int64, x), src/launch.jl:81: RoundNearest, halfway cases to
 * the even integer (lround would round them away from zero) */
long or_round_int(double x) { return (long)nearbyint(x); }

static void launch_rings(int N_rings, int min_az, double w, double *r_pts, double *r_w,
                         int *N_theta) {
    int n = 2 * N_rings + 2;
    double *x = (double *)malloc(sizeof(double) * n), *wt = (double *)malloc(sizeof(double) * n);
    or_gauss_hermite(n, x, wt);
    for (int i = 0; i < N_rings; i++) { /* v[N_rings+2:end], first N_rings used */
        r_pts[i] = x[N_rings + 1 + i] * (w / sqrt(2.0));
        r_w[i] = wt[N_rings + 1 + i] * (w / sqrt(2.0));
    }
    for (int i = 0; i < N_rings; i++) {
        long k = or_round_int(min_az * r_pts[i] / r_pts[0]);
        N_theta[i] = k < 1 ? 1 : (int)k;
    }
    free(x);
    free(wt);
}

int or_launch_count(int N_rings, int min_az) {
    if (N_rings < 2) return -1;
    double *r = (double *)malloc(sizeof(double) * N_rings);
    double *rw = (double *)malloc(sizeof(double) * N_rings);
    int *nt = (int *)malloc(sizeof(int) * N_rings);
    launch_rings(N_rings, min_az, 1.0, r, rw, nt);
    int tot = 0;
    for (int i = 0; i < N_rings; i++) tot += nt[i];
    free(r);
    free(rw);
    free(nt);
    return tot;
}

int or_launch_peripheral_rays(const double x0[3], const double N0[3], double w,
                              double inv_curv, double f, int N_rings, int min_az,
                              int normalize, double *pos, double *dir, double *weights) {
    if (N_rings < 2) return -1; /* ArgumentError, src/launch.jl:27-29 */
    double nn = sqrt(N0[0] * N0[0] + N0[1] * N0[1] + N0[2] * N0[2]);
    double n0[3] = {N0[0] / nn, N0[1] / nn, N0[2] / nn};
    int fin = isfinite(inv_curv);
    double w0 = w, xw[3] = {0, 0, 0};
    if (fin) {
        double Rc = 1.0 / inv_curv, lam = OR_C / f;
        w0 = (lam * fabs(Rc) * w) / sqrt(lam * lam * Rc * Rc + PI * PI * w * w * w * w);
        double zw = PI * PI * Rc * w * w * w * w / (lam * lam * Rc * Rc + PI * PI * w * w * w * w);
        for (int k = 0; k < 3; k++) xw[k] = x0[k] - n0[k] * zw;
    }
    double ec[3] = {1.0, 0.0, -n0[0] / n0[2]};
    double eu[3] = {-n0[0] * n0[1] / n0[2], n0[2] - n0[0], -n0[1]};
    double nc = sqrt(ec[0] * ec[0] + ec[1] * ec[1] + ec[2] * ec[2]);
    double nu = sqrt(eu[0] * eu[0] + eu[1] * eu[1] + eu[2] * eu[2]);
    for (int k = 0; k < 3; k++) {
        ec[k] /= nc;
        eu[k] /= nu;
    }
    double *r = (double *)malloc(sizeof(double) * N_rings);
    double *rw = (double *)malloc(sizeof(double) * N_rings);
    int *nt = (int *)malloc(sizeof(int) * N_rings);
    launch_rings(N_rings, min_az, w, r, rw, nt);
    int kk = 0;
    for (int i = 0; i < N_rings; i++) {
        for (int j = 0; j < nt[i]; j++) {
            double th = 2.0 * PI * (double)j / (double)nt[i];
            double thw = 2.0 * PI / (double)nt[i];
            double chi = r[i] * cos(th), ups = r[i] * sin(th);
            double *P = pos + 3 * (kk + j), *D = dir + 3 * (kk + j);
            for (int k = 0; k < 3; k++) P[k] = chi * ec[k] + ups * eu[k] + x0[k];
            if (fin) {
                double sg = inv_curv > 0 ? 1.0 : (inv_curv < 0 ? -1.0 : 0.0);
                for (int k = 0; k < 3; k++) D[k] = w0 / w * (chi * ec[k] + ups * eu[k]) * sg + xw[k];
                if (inv_curv < 0.0) {
                    for (int k = 0; k < 3; k++) D[k] -= P[k];
                } else {
                    for (int k = 0; k < 3; k++) D[k] = -D[k] + P[k];
                }
                double dn = sqrt(D[0] * D[0] + D[1] * D[1] + D[2] * D[2]);
                for (int k = 0; k < 3; k++) D[k] /= dn;
            } else {
                for (int k = 0; k < 3; k++) D[k] = n0[k];
            }
            weights[kk + j] = r[i] * rw[i] * thw;
        }
        kk += nt[i];
    }
    if (normalize) {
        double s = 0;
        for (int i = 0; i < kk; i++) s += weights[i];
        for (int i = 0; i < kk; i++) weights[i] /= s;
    } else {
        for (int i = 0; i < kk; i++) weights[i] *= 2.0 / (w * w * PI);
    }
    free(r);
    free(rw);
    free(nt);
    return kk;
}

/* IMAS.pol_tor_angles_2_vector (called at src/solve.jl:211); IMAS ec_launchers
 * convention angle_pol = atan2(-k_Z,-k_R), angle_tor = asin(k_phi/k).
 * Parity unpinned (IMAS is not available here). */
void or_pol_tor_angles_2_vector(double pol, double tor, double N[3]) {
    N[0] = -cos(pol) * cos(tor);
    N[1] = sin(tor);
    N[2] = -sin(pol) * cos(tor);
}

/* ------------------------------------------------------------------------- */
/* ray entry, src/solve.jl:7-74                                              */
/* ------------------------------------------------------------------------- */
/* IMAS.toroidal_intersection for the grid rectangle (src/solve.jl:22-24);
 * smallest t > 0 where p0 + t v meets the surface of revolution of the
 * polygon.  Parity unpinned (IMAS not available). */
static double toroidal_intersection(const double *Rp, const double *Zp, int np,
                                    const double p0[3], const double v[3]) {
    double best = INFINITY;
    for (int s = 0; s + 1 < np; s++) {
        double Ra = Rp[s], Za = Zp[s], Rb = Rp[s + 1], Zb = Zp[s + 1];
        if (Zb == Za) {
            if (v[2] == 0.0) continue;
            double t = (Za - p0[2]) / v[2];
            if (t <= 0) continue;
            double R = hypot(p0[0] + t * v[0], p0[1] + t * v[1]);
            if (R >= fmin(Ra, Rb) && R <= fmax(Ra, Rb) && t < best) best = t;
        } else {
            double k = (Rb - Ra) / (Zb - Za);
            double al = Ra + (p0[2] - Za) * k, be = v[2] * k;
            double A = v[0] * v[0] + v[1] * v[1] - be * be;
            double B = 2.0 * (p0[0] * v[0] + p0[1] * v[1] - al * be);
            double C = p0[0] * p0[0] + p0[1] * p0[1] - al * al;
            double ts[2];
            int nt = 0;
            if (fabs(A) < 1e-300) {
                if (B != 0) ts[nt++] = -C / B;
            } else {
                double disc = B * B - 4 * A * C;
                if (disc >= 0) {
                    double sq = sqrt(disc);
                    ts[nt++] = (-B - sq) / (2 * A);
                    ts[nt++] = (-B + sq) / (2 * A);
                }
            }
            for (int q = 0; q < nt; q++) {
                double t = ts[q];
                if (t <= 0) continue;
                double z = p0[2] + t * v[2];
                double sp = (z - Za) / (Zb - Za);
                if (sp < 0 || sp > 1) continue;
                if (al + be * t < 0) continue;
                if (t < best) best = t;
            }
        }
    }
    return best;
}

static int on_grid(const or_plasma *p, const double x[3]) {
    double R = hypot(x[0], x[1]);
    return p->psi.R1 <= R && R <= p->psi.Rn && p->psi.Z1 <= x[2] && x[2] <= p->psi.Zn;
}

/* first_point, src/solve.jl:18-38.  Bisection is run to machine precision
 * (Roots.Bisection with xtol=1e-6 stops earlier; parity unpinned). */
static int first_point(const or_plasma *p, const double x0[3], const double N0[3],
                       double out[3]) {
    double pp[3] = {x0[0], x0[1], x0[2]};
    if (!on_grid(p, x0)) {
        double Rp[5] = {p->psi.R1, p->psi.Rn, p->psi.Rn, p->psi.R1, p->psi.R1};
        double Zp[5] = {p->psi.Z1, p->psi.Z1, p->psi.Zn, p->psi.Zn, p->psi.Z1};
        double t = toroidal_intersection(Rp, Zp, 5, x0, N0);
        if (!isfinite(t)) return OR_ENTRY_FAIL;
        for (int k = 0; k < 3; k++) pp[k] = x0[k] + N0[k] * t;
    }
    double a = 0.0, b = 0.5;
#define G(t) (or_evaluate(&p->psi, (double[3]){pp[0] + (t)*N0[0], pp[1] + (t)*N0[1], pp[2] + (t)*N0[2]}) - p->psi_prof_max)
    double ga = G(a), gb = G(b);
    if (ga == 0.0)
        b = a;
    else if (gb == 0.0)
        a = b;
    else {
        if ((ga > 0) == (gb > 0)) return OR_ENTRY_FAIL;
        for (int it = 0; it < 200; it++) {
            double m = 0.5 * (a + b);
            if (m <= a || m >= b) break;
            double gm = G(m);
            if (gm == 0.0) {
                a = b = m;
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
    double t = (fabs(ga) <= fabs(gb)) ? a : b;
#undef G
    for (int k = 0; k < 3; k++) pp[k] += t * N0[k];
    double psi_ref = or_evaluate(&p->psi, pp);
    if (!(fabs(psi_ref - p->psi_prof_max) < 1e-6)) return OR_ENTRY_FAIL; /* :32 */
    if (psi_ref > p->psi_prof_max)
        for (int k = 0; k < 3; k++) pp[k] += 2.0 * (psi_ref - p->psi_prof_max) * N0[k];
    for (int k = 0; k < 3; k++) out[k] = pp[k];
    return OR_OK;
}

/* vacuum_plasma_refraction, src/solve.jl:40-74.  The 3 refraction equations
 * (:40-49) are solved through their scalar reduction N = n0 + (cos_i -
 * sqrt(q^2 - sin_i^2)) n with q^2 = N_s^2(N.b) (same root; NLsolve itself is
 * not restated). */
static int vacuum_plasma_refraction(const or_plasma *p, const double pp[3], const double N0[3],
                                    double omega, int mode, double N[3]) {
    double X, Y, Npar, b[3];
    or_eval_plasma(p, pp, N0, omega, &X, &Y, &Npar, b);
    double Nest = or_refractive_index_sq(X, Y, 0.0, mode);
    if (Nest <= 0) return OR_REFLECTED;
    double q = sqrt(Nest);
    double R = hypot(pp[0], pp[1]), dR, dZ;
    or_spl2d_grad(&p->psi, R, pp[2], &dR, &dZ);
    double n[3] = {dR * pp[0] / R, dR * pp[1] / R, dZ};
    double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int k = 0; k < 3; k++) n[k] /= nn;
    double n0n = sqrt(N0[0] * N0[0] + N0[1] * N0[1] + N0[2] * N0[2]);
    double n0[3] = {N0[0] / n0n, N0[1] / n0n, N0[2] / n0n};
    double ci = -(n[0] * n0[0] + n[1] * n0[1] + n[2] * n0[2]);
    double si2 = 1.0 - ci * ci;
    double nb = n[0] * b[0] + n[1] * b[1] + n[2] * b[2];
    double n0b = n0[0] * b[0] + n0[1] * b[1] + n0[2] * b[2];
    for (int it = 0; it < 100; it++) {
        double rt = q * q - si2;
        if (rt < 0) return OR_REFLECTED;
        double s = sqrt(rt);
        double Np = n0b + (ci - s) * nb;
        double r = q * q - or_refractive_index_sq(X, Y, Np, mode);
        double h = 1e-7 * q;
        double s2 = sqrt((q + h) * (q + h) - si2), s1 = sqrt((q - h) * (q - h) - si2);
        double rp = (q + h) * (q + h) - or_refractive_index_sq(X, Y, n0b + (ci - s2) * nb, mode);
        double rm = (q - h) * (q - h) - or_refractive_index_sq(X, Y, n0b + (ci - s1) * nb, mode);
        double dr = (rp - rm) / (2 * h);
        double dq = r / dr;
        q -= dq;
        if (fabs(dq) <= 1e-16 * q) break;
    }
    double s = sqrt(q * q - si2);
    for (int k = 0; k < 3; k++) N[k] = n0[k] + (ci - s) * n[k];
    return OR_OK;
}

int or_ray_entry(const or_plasma *p, const double x0[3], const double N0[3], double omega,
                 int mode, double xp[3], double Np[3], double *s0) {
    int st = first_point(p, x0, N0, xp);
    if (st != OR_OK) return st;
    if (!(or_evaluate(&p->psi, xp) <= p->psi_prof_max)) return OR_ENTRY_FAIL; /* :138 */
    st = vacuum_plasma_refraction(p, xp, N0, omega, mode, Np);
    if (st != OR_OK) return st;
    double D = or_dispersion_relation(p, xp, Np, omega, mode);
    if (!(fabs(D) < 1e-12)) return OR_ENTRY_FAIL; /* :141 */
    *s0 = sqrt((xp[0] - x0[0]) * (xp[0] - x0[0]) + (xp[1] - x0[1]) * (xp[1] - x0[1]) +
               (xp[2] - x0[2]) * (xp[2] - x0[2]));
    return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* trace: fixed-step RK4 of sys! (src/solve.jl:112-114) + deposition          */
/* ------------------------------------------------------------------------- */
/* warm absorption (models 2 and 3): or_alpha_warm (torj_warm_oracle.c), or,
 * when the harness installs one, a hook (oracle/warm_ref.py's numpy restatement
 * of src/general_absorption.jl, serial) */
static or_alpha_fn g_alpha_hook = NULL;

void or_set_alpha_hook(or_alpha_fn fn) { g_alpha_hook = fn; }

/* optical-depth rate of model 0 (none), 1 (alpha_approx: abs_Albajar_fast) or
 * 2 / 3 (warm alpha, iwarm 1 / 3, with v_g_perp = 1/|dD/dN|) */
static double alpha_model(const or_plasma *p, const double u[6], double omega, int mode,
                          int model) {
    if (model == 0) return 0.0;
    if (model == 1) return or_alpha_approx(p, u, u + 3, omega, mode);
    double X, Y, Npar, b[3];
    or_eval_plasma(p, u, u + 3, omega, &X, &Y, &Npar, b);
    const double Nabs = sqrt(u[3] * u[3] + u[4] * u[4] + u[5] * u[5]);
    const double inv = 1.0 / or_grad_norm(p, u, u + 3, omega, mode);
    if (g_alpha_hook)
        return g_alpha_hook(omega, X, Y, Nabs, Npar, or_T_e(p, u), inv, mode, model);
    return or_alpha_warm(omega, X, Y, Nabs, Npar, or_T_e(p, u), inv, mode, model == 2 ? 1 : 3,
                         NULL);
}

static void rhs(const or_plasma *p, const double u[6], double omega, int mode, int absorb,
                double du[6], double *alpha) {
    or_grad_lambda(p, u, u + 3, omega, mode, du);
    *alpha = alpha_model(p, u, omega, mode, absorb);
}

/* A-priori sensitivity of a warm-model trace's optical depth (test
 * infrastructure for the C5 parity bar).  For each ray, over its
 * first steps[r] fixed RK4 steps (the trajectory is alpha-independent), every
 * stage point's warm alpha is re-evaluated at inputs perturbed by a relative eta
 * -- Y up and down (the harmonic resonance makes alpha steepest in Y), and
 * (X, N_par, Te) jointly both ways -- and the largest change, with the RK4
 * weight ds/6 (1, 2, 2, 1), is summed: out_sens[r] = sum |d tau|.  A ray whose
 * tau moves by more than the parity bar under perturbations of a few tens of
 * ulps has a tau that no double-precision restatement determines to that bar:
 * the fsup recurrence's cancellation (:536-557) at cold plasma edges, or a
 * stage point sitting on a discontinuity of warmdisp's root selection (the
 * selector test rr.re <= 0 of :1203-1214 decided at the 1e-11 level), where
 * one ulp of Y picks the other root.  The flag depends on the shared trajectory
 * only, not on the result of the implementation under test. */
static void warm_inputs(const or_plasma *p, const double u[6], double omega, int mode, double *X,
                        double *Y, double *Nabs, double *Npar, double *Te, double *inv) {
    double b[3];
    or_eval_plasma(p, u, u + 3, omega, X, Y, Npar, b);
    *Nabs = sqrt(u[3] * u[3] + u[4] * u[4] + u[5] * u[5]);
    *inv = 1.0 / or_grad_norm(p, u, u + 3, omega, mode);
    *Te = or_T_e(p, u);
}

static double warm_stage_sens(const or_plasma *p, const double u[6], double omega, int mode,
                              int iwarm, double eta) {
    double X, Y, Nabs, Npar, Te, inv;
    warm_inputs(p, u, omega, mode, &X, &Y, &Nabs, &Npar, &Te, &inv);
    const double a0 = or_alpha_warm(omega, X, Y, Nabs, Npar, Te, inv, mode, iwarm, NULL);
    static const double f[4][4] = {{0, 1, 0, 0}, {0, -1, 0, 0}, {1, 0, 1, -1}, {-1, 0, -1, 1}};
    double d = 0.0;
    for (int k = 0; k < 4; k++) {
        const double a = or_alpha_warm(omega, X * (1.0 + eta * f[k][0]), Y * (1.0 + eta * f[k][1]), Nabs,
                                       Npar * (1.0 + eta * f[k][2]), Te * (1.0 + eta * f[k][3]), inv,
                                       mode, iwarm, NULL);
        const double e = fabs(a - a0);
        if (!(e <= d)) d = e;  /* NaN propagates as "unbounded" */
    }
    return d;
}

void or_warm_sensitivity(const or_plasma *p, double omega, int mode, int iwarm, double ds,
                         int n_rays, const double *x0, const double *N0, const int *steps,
                         double eta, double *out_sens, int n_threads) {
    int nth = n_threads > 0 ? n_threads : 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
#endif
    for (int r = 0; r < n_rays; r++) {
        double u[6], sens = 0.0;
        for (int k = 0; k < 3; k++) {
            u[k] = x0[3 * r + k];
            u[3 + k] = N0[3 * r + k];
        }
        for (int s = 0; s < steps[r]; s++) {
            double k1[6], k2[6], k3[6], k4[6], ut[6], dummy;
            rhs(p, u, omega, mode, 0, k1, &dummy);
            sens += ds / 6.0 * warm_stage_sens(p, u, omega, mode, iwarm, eta);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + 0.5 * ds * k1[k];
            rhs(p, ut, omega, mode, 0, k2, &dummy);
            sens += ds / 3.0 * warm_stage_sens(p, ut, omega, mode, iwarm, eta);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + 0.5 * ds * k2[k];
            rhs(p, ut, omega, mode, 0, k3, &dummy);
            sens += ds / 3.0 * warm_stage_sens(p, ut, omega, mode, iwarm, eta);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + ds * k3[k];
            rhs(p, ut, omega, mode, 0, k4, &dummy);
            sens += ds / 6.0 * warm_stage_sens(p, ut, omega, mode, iwarm, eta);
            for (int k = 0; k < 6; k++) u[k] = u[k] + ds / 6.0 * (k1[k] + 2.0 * k2[k] + 2.0 * k3[k] + k4[k]);
        }
        out_sens[r] = sens;
    }
}

/* The same a-priori sensitivity for the Albajar model (absorption 1, the C3
 * parity statistic over resolvable optical depths): each stage point's
 * abs_Albajar_fast re-evaluated with Y moved up and down by eta, and with
 * (X, N_par, Te) jointly both ways.  Near a harmonic's threshold (r = m / m_0
 * just above 1) alpha carries sqrt(r^2 - 1), whose relative change under a
 * relative change eta of Y is eta r^2 / (r^2 - 1): a ray whose tiny optical
 * depth comes from such points has a tau that inputs differing by a few ulps
 * (the GPU's trajectory against this one's, 1e-15) move beyond 1e-10. */
static double albajar_stage_sens(const or_plasma *p, const double u[6], double omega, int mode,
                                 double eta) {
    double X, Y, Npar, b[3];
    or_eval_plasma(p, u, u + 3, omega, &X, &Y, &Npar, b);
    const double Nabs = sqrt(u[3] * u[3] + u[4] * u[4] + u[5] * u[5]);
    const double Te = or_T_e(p, u);
    const double a0 = or_abs_albajar_fast(omega, X, Y, Nabs, Npar, Te, mode);
    static const double f[4][4] = {{0, 1, 0, 0}, {0, -1, 0, 0}, {1, 0, 1, -1}, {-1, 0, -1, 1}};
    double d = 0.0;
    for (int k = 0; k < 4; k++) {
        const double a = or_abs_albajar_fast(omega, X * (1.0 + eta * f[k][0]), Y * (1.0 + eta * f[k][1]),
                                             Nabs, Npar * (1.0 + eta * f[k][2]),
                                             Te * (1.0 + eta * f[k][3]), mode);
        const double e = fabs(a - a0);
        if (!(e <= d)) d = e;
    }
    return d;
}

void or_albajar_sensitivity(const or_plasma *p, double omega, int mode, double ds, int n_rays,
                            const double *x0, const double *N0, const int *steps, double eta,
                            double *out_sens, int n_threads) {
    int nth = n_threads > 0 ? n_threads : 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
#endif
    for (int r = 0; r < n_rays; r++) {
        double u[6], sens = 0.0;
        for (int k = 0; k < 3; k++) {
            u[k] = x0[3 * r + k];
            u[3 + k] = N0[3 * r + k];
        }
        for (int s = 0; s < steps[r]; s++) {
            double k1[6], k2[6], k3[6], k4[6], ut[6], dummy;
            rhs(p, u, omega, mode, 0, k1, &dummy);
            sens += ds / 6.0 * albajar_stage_sens(p, u, omega, mode, eta);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + 0.5 * ds * k1[k];
            rhs(p, ut, omega, mode, 0, k2, &dummy);
            sens += ds / 3.0 * albajar_stage_sens(p, ut, omega, mode, eta);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + 0.5 * ds * k2[k];
            rhs(p, ut, omega, mode, 0, k3, &dummy);
            sens += ds / 3.0 * albajar_stage_sens(p, ut, omega, mode, eta);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + ds * k3[k];
            rhs(p, ut, omega, mode, 0, k4, &dummy);
            sens += ds / 6.0 * albajar_stage_sens(p, ut, omega, mode, eta);
            for (int k = 0; k < 6; k++) u[k] = u[k] + ds / 6.0 * (k1[k] + 2.0 * k2[k] + 2.0 * k3[k] + k4[k]);
        }
        out_sens[r] = sens;
    }
}

/* shell index j with grid[j] <= v < grid[j+1]; clamps to [0, n-2] */
static int shell_of(const double *g, int n, double v) {
    int lo = 0, hi = n - 1;
    while (hi - lo > 1) {
        int mid = (lo + hi) / 2;
        if (g[mid] <= v)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

/* Deposit dP for a step whose psi moves linearly from pa to pb: each shell
 * [g_j, g_{j+1}] receives the fraction of the step spent inside it.  Power
 * deposited outside [g_0, g_{n-1}] is not counted (as in the reference, whose
 * shells only span the psi_dP_dV grid; src/plasma.jl:104-144). */
static double deposit(const double *g, int n, double pa, double pb, double dP, double w,
                      double *acc) {
    if (!(dP != 0.0) || n < 2) return 0.0;
    double lo = pa < pb ? pa : pb, hi = pa < pb ? pb : pa;
    double g0 = g[0], gl = g[n - 1], inside = 0.0;
    if (hi == lo) {
        if (lo < g0 || lo > gl) return 0.0;
        int j = shell_of(g, n, lo);
        acc[j] += w * dP;
        return dP;
    }
    if (hi <= g0 || lo >= gl) return 0.0;
    int j = shell_of(g, n, lo < g0 ? g0 : lo);
    double span = hi - lo;
    for (; j < n - 1 && g[j] < hi; j++) {
        double a = lo > g[j] ? lo : g[j];
        double b = hi < g[j + 1] ? hi : g[j + 1];
        if (b <= a) continue;
        double part = dP * ((b - a) / span);
        acc[j] += w * part;
        inside += part;
    }
    return inside;
}

/* ------------------------------------------------------------------------- */
/* The reference's integrator: solve(ODEProblem(sys!, u0, tspan; dtmax, abstol, */
/* reltol), callback) with no algorithm argument (src/solve.jl:154-162; the     */
/* intended OwrenZen3() lands in the parameter slot).   */
/* DifferentialEquations then picks its default method, which for a non-stiff  */
/* problem at reltol = 1e-6 is Tsit5 (OrdinaryDiffEq Tsit5 tableau, PI step     */
/* controller beta1 = 7/50, beta2 = 2/25, gamma = 9/10, qmin = 1/5, qmax = 10,   */
/* qold0 = qoldmin = 1e-4, RMS error norm of utilde / (abstol + max(|uprev|,    */
/* |u|) reltol), Hairer's initial step ode_determine_initdt, tstop snapping     */
/* within 100 eps).  Parity unpinned: no Julia to run the reference here; this  */
/* restates OrdinaryDiffEq's published algorithm.  u = (x, N, P), dP/ds = -P a. */
/* ------------------------------------------------------------------------- */
static const double TS_A[7][6] = {
    {0, 0, 0, 0, 0, 0},
    {0.161, 0, 0, 0, 0, 0},
    {-0.008480655492356989, 0.335480655492357, 0, 0, 0, 0},
    {2.897153057105493, -6.359448489975075, 4.3622954328695815, 0, 0, 0},
    {5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525, 0, 0},
    {5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401,
     -0.028269050394068383, 0},
    {0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081,
     2.324710524099774}};
static const double TS_BT[7] = {-0.00178001105222577714, -0.0008164344596567469,
                                0.007880878010261995,    -0.1447110071732629,
                                0.5823571654525552,      -0.45808210592918697,
                                0.015151515151515152};

static void rhs7(const or_plasma *p, const double u[7], double omega, int mode, int absorb,
                 double du[7]) {
    double a;
    rhs(p, u, omega, mode, absorb, du, &a);
    du[6] = -u[6] * a; /* sys!: du[7] = -P alpha (src/solve.jl:113) */
}

static double rms7(const double v[7]) {
    double s = 0.0;
    for (int k = 0; k < 7; k++) s += v[k] * v[k];
    return sqrt(s / 7.0);
}

/* ode_determine_initdt (OrdinaryDiffEq initdt.jl), order 5 */
static double ts_initdt(const or_plasma *p, const or_trace_cfg *c, const double u0[7],
                        const double f0[7], double dtmax) {
    double sk[7], t0[7], t1[7], u1[7], f1[7];
    for (int k = 0; k < 7; k++) {
        sk[k] = c->abstol + fabs(u0[k]) * c->reltol;
        t0[k] = u0[k] / sk[k];
        t1[k] = f0[k] / sk[k];
    }
    const double d0 = rms7(t0), d1 = rms7(t1);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : (d0 / d1) / 100.0;
    dt0 = fmin(dt0, dtmax);
    for (int k = 0; k < 7; k++) u1[k] = u0[k] + dt0 * f0[k];
    rhs7(p, u1, c->omega, c->mode, c->absorption, f1);
    int same = 1;
    for (int k = 0; k < 7; k++) same &= (f0[k] == f1[k]);
    if (same) return 100.0 * dt0;
    for (int k = 0; k < 7; k++) t0[k] = (f1[k] - f0[k]) / sk[k];
    const double d2 = rms7(t0) / dt0;
    const double m = fmax(d1, d2);
    const double dt1 = (m <= 1e-15) ? fmax(1e-6, dt0 * 1e-3) : pow(10.0, -(2.0 + log10(m)) / 5.0);
    return fmin(fmin(100.0 * dt0, dt1), dtmax);
}

/* one ray of the adaptive integration (u = x, N, P in/out); returns status */
static int ts_ray(const or_plasma *p, const or_trace_cfg *c, int r, double u[7], double s_start,
                  double w, double *acc, double *Pdep, int *steps_out, double *traj, int n_save,
                  double *smp) {
    const double dtmax = c->ds, s_step = c->s_max / (double)c->n_chunks;
    const int cap = c->n_steps;
    int steps = 0, status = OR_OK;
    double psi_a = or_evaluate(&p->psi, u);
    double k[7][7], ut[7];
    for (int ch = 1; ch <= c->n_chunks && status == OR_OK; ch++) {
        double t = (double)(ch - 1) * s_step + s_start; /* Float64(i-1)*s_step + s0 */
        const double tf = (double)ch * s_step + s_start;
        rhs7(p, u, c->omega, c->mode, c->absorption, k[0]); /* fsalfirst */
        double dt = ts_initdt(p, c, u, k[0], dtmax);
        double qold = 1e-4, q11 = 0.0;
        while (t < tf) {
            if (steps >= cap) { /* no room for another accepted step */
                status = OR_MAX_STEPS;
                break;
            }
            dt = fmin(fabs(dt), tf - t); /* modify_dt_for_tstops! */
            for (int s = 1; s < 7; s++) {
                for (int q = 0; q < 7; q++) {
                    double a = 0.0;
                    for (int j = 0; j < s; j++) a += TS_A[s][j] * k[j][q];
                    ut[q] = u[q] + dt * a;
                }
                rhs7(p, ut, c->omega, c->mode, c->absorption, k[s]);
            }
            /* ut = u_{n+1} (row 7 = b), k[6] = f(u_{n+1}) (FSAL) */
            double e[7];
            int bad = 0;
            for (int q = 0; q < 7; q++) {
                double a = 0.0;
                for (int j = 0; j < 7; j++) a += TS_BT[j] * k[j][q];
                e[q] = dt * a / (c->abstol + fmax(fabs(u[q]), fabs(ut[q])) * c->reltol);
                if (!isfinite(ut[q])) bad = 1;
            }
            if (bad) {
                status = OR_NAN;
                break;
            }
            const double EEst = rms7(e);
            double qq;
            if (EEst == 0.0) {
                qq = 1.0 / 10.0;
            } else {
                q11 = pow(EEst, 0.14);
                qq = q11 / pow(qold, 0.08);
                qq = fmax(1.0 / 10.0, fmin(5.0, qq / 0.9));
            }
            if (EEst <= 1.0) { /* accept (qsteady_min = qsteady_max = 1) */
                qold = fmax(EEst, 1e-4);
                const double dtnew = dt / qq;
                double tn = t + dt;
                if (fabs(tn - tf) < 100.0 * DBL_EPSILON * fmax(fabs(t), fabs(tf))) tn = tf;
                const double Pa = u[6];
                memcpy(u, ut, sizeof(double) * 7);
                memcpy(k[0], k[6], sizeof(double) * 7);
                /* ContinuousCallback(u[7] < 0, affect!) (src/solve.jl:78-83,159-160):
                 * P projected to 0 at the end of the accepted step that crossed
                 * (DiffEq root-finds the crossing inside the step: unpinned) */
                if (u[6] < 0.0) {
                    u[6] = 0.0;
                    k[0][6] = -0.0;
                }
                t = tn;
                steps++;
                const double psi_b = or_evaluate(&p->psi, u);
                if (smp) {
                    smp[3 * steps] = psi_b;
                    smp[3 * steps + 1] = -k[0][6]; /* P alpha at the saved point (FSAL) */
                    smp[3 * steps + 2] = t;
                }
                if (acc && Pdep) *Pdep += deposit(c->psi_grid, c->n_psi, psi_a, psi_b, Pa - u[6], w, acc);
                psi_a = psi_b;
                if (n_save > 0 && (steps % c->traj_stride) == 0) {
                    double *T = traj + ((size_t)r * n_save + steps / c->traj_stride - 1) * 5;
                    T[0] = u[0], T[1] = u[1], T[2] = u[2], T[3] = -log(u[6]), T[4] = t;
                }
                dt = fmin(dtmax, dtnew); /* calc_dt_propose! */
            } else { /* reject: step_reject_controller!(PIController) */
                dt /= fmin(5.0, q11 / 0.9);
            }
        }
        if (status != OR_OK) break;
        if (or_evaluate(&p->psi, u) > c->psi_exit) status = OR_LEFT_PLASMA; /* :174 */
        else if (u[6] < c->P_min) status = OR_ABSORBED;                      /* :176 */
    }
    *steps_out = steps;
    return status;
}

int or_trace(const or_plasma *p, const or_trace_cfg *cfg, int n_rays, const double *x0,
             const double *N0, const double *weights, double *out_state, int *out_status,
             int *out_steps, double *out_dP, double *out_Pdep, double *out_traj,
             int n_threads) {
    return or_trace_samples(p, cfg, n_rays, x0, N0, weights, out_state, out_status, out_steps,
                            out_dP, out_Pdep, out_traj, NULL, n_threads);
}

int or_trace_samples(const or_plasma *p, const or_trace_cfg *cfg, int n_rays, const double *x0,
                     const double *N0, const double *weights, double *out_state, int *out_status,
                     int *out_steps, double *out_dP, double *out_Pdep, double *out_traj,
                     double *out_samples, int n_threads) {
    const double ds = cfg->ds;
    const int n_psi = cfg->n_psi;
    int n_save = cfg->traj_stride > 0 ? cfg->n_steps / cfg->traj_stride : 0;
    if (out_dP && n_psi > 0) memset(out_dP, 0, sizeof(double) * n_psi);
    int nth = n_threads > 0 ? n_threads : 1;
    double *acc_all = NULL;
    if (n_psi > 0) acc_all = (double *)calloc((size_t)nth * n_psi, sizeof(double));
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
#endif
    for (int r = 0; r < n_rays; r++) {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        double *acc = acc_all ? acc_all + (size_t)tid * n_psi : NULL;
        double w = weights ? weights[r] : 1.0;
        double u[6], tau = 0.0;
        for (int k = 0; k < 3; k++) {
            u[k] = x0[3 * r + k];
            u[3 + k] = N0[3 * r + k];
        }
        int status = OR_OK, steps = 0;
        double psi_a = (n_psi > 0) ? or_evaluate(&p->psi, u) : 0.0;
        double Pdep = 0.0;
        double *smp = out_samples ? out_samples + (size_t)r * (cfg->n_steps + 1) * 3 : NULL;
        const double s_start = cfg->s0 ? cfg->s0[r] : 0.0;
        if (smp) {
            for (int k = 0; k < 3 * (cfg->n_steps + 1); k++) smp[k] = NAN;
            smp[0] = or_evaluate(&p->psi, u);
            smp[1] = 0.0;
            smp[2] = s_start;
        }
        if (cfg->integrator == 1) {
            double u7[7] = {u[0], u[1], u[2], u[3], u[4], u[5], 1.0};
            status = ts_ray(p, cfg, r, u7, s_start, w, acc, n_psi > 0 ? &Pdep : NULL, &steps,
                            out_traj, n_save, smp);
            for (int k = 0; k < 6; k++) out_state[7 * r + k] = u7[k];
            out_state[7 * r + 6] = -log(u7[6]);
            out_status[r] = status;
            out_steps[r] = steps;
            if (out_Pdep) out_Pdep[r] = Pdep;
            continue;
        }
        for (int s = 0; s < cfg->n_steps; s++) {
            double k1[6], k2[6], k3[6], k4[6], a1, a2, a3, a4, ut[6];
            rhs(p, u, cfg->omega, cfg->mode, cfg->absorption, k1, &a1);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + 0.5 * ds * k1[k];
            rhs(p, ut, cfg->omega, cfg->mode, cfg->absorption, k2, &a2);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + 0.5 * ds * k2[k];
            rhs(p, ut, cfg->omega, cfg->mode, cfg->absorption, k3, &a3);
            for (int k = 0; k < 6; k++) ut[k] = u[k] + ds * k3[k];
            rhs(p, ut, cfg->omega, cfg->mode, cfg->absorption, k4, &a4);
            double un[6];
            int bad = 0;
            for (int k = 0; k < 6; k++) {
                un[k] = u[k] + ds / 6.0 * (k1[k] + 2.0 * k2[k] + 2.0 * k3[k] + k4[k]);
                if (!isfinite(un[k])) bad = 1;
            }
            double taun = tau + ds / 6.0 * (a1 + 2.0 * a2 + 2.0 * a3 + a4);
            if (!isfinite(taun)) bad = 1;
            if (bad) {
                status = OR_NAN;
                break;
            }
            double dP = exp(-tau) - exp(-taun);
            memcpy(u, un, sizeof(u));
            tau = taun;
            steps = s + 1;
            double psi_b = or_evaluate(&p->psi, u);
            if (smp) { /* dP_ds = P alpha_approx at the saved point (src/solve.jl:171) */
                smp[3 * steps] = psi_b;
                smp[3 * steps + 1] =
                    cfg->absorption ? exp(-tau) * alpha_model(p, u, cfg->omega, cfg->mode, cfg->absorption)
                                    : 0.0;
                smp[3 * steps + 2] = s_start + steps * ds;
            }
            if (n_psi > 0) {
                Pdep += deposit(cfg->psi_grid, n_psi, psi_a, psi_b, dP, w, acc);
                psi_a = psi_b;
            }
            if (n_save > 0 && (steps % cfg->traj_stride) == 0) {
                int si = steps / cfg->traj_stride - 1;
                double *T = out_traj + ((size_t)r * n_save + si) * 5;
                T[0] = u[0];
                T[1] = u[1];
                T[2] = u[2];
                T[3] = tau;
                T[4] = s_start + steps * ds;
            }
            if (cfg->chunk_steps > 0 && (steps % cfg->chunk_steps) == 0) {
                if (psi_b > cfg->psi_exit) { /* src/solve.jl:174 */
                    status = OR_LEFT_PLASMA;
                    break;
                }
                if (exp(-tau) < cfg->P_min) { /* src/solve.jl:176 */
                    status = OR_ABSORBED;
                    break;
                }
            }
        }
        for (int k = 0; k < 6; k++) out_state[7 * r + k] = u[k];
        out_state[7 * r + 6] = tau;
        out_status[r] = status;
        out_steps[r] = steps;
        if (out_Pdep) out_Pdep[r] = Pdep;
    }
    if (acc_all) {
        for (int t = 0; t < nth; t++)
            for (int j = 0; j < n_psi; j++) out_dP[j] += acc_all[(size_t)t * n_psi + j];
        free(acc_all);
    }
    return 0;
}
