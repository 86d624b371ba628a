/*
 * torj_warm_oracle.c -- warm-plasma absorption (absorption models 2 / 3) of the
 * CPU oracle: a C restatement of oracle/warm_ref.py, which restates (and
 * repairs, R1-R5 there) GRAY's warm dispersion module as transliterated in
 * src/general_absorption.jl.
 *
 * TEST INFRASTRUCTURE ONLY (see torj_oracle.h): the checker of the GPU's warm
 * alpha inside the oracle's multi-threaded trace, and the all-core CPU peer of
 * bench.py's warm workloads (C5).  Never linked by the product.
 *
 * Pinned by tests/test_warm_oracle_c.py against warm_ref.py (numpy + scipy's
 * expi / wofz) point by point and through whole traces.  Parity with an executed
 * reference is unpinned (the reference module is not runnable).
 *
 * Third-party arithmetic, restated here rather than taken from scipy:
 *   zetac  -- ACM TOMS 680 (Poppe & Wijers), the algorithm the reference itself
 *             transliterates (src/general_absorption.jl:345-465);
 *   expei  -- e^-x Ei(x): the reference uses Cody's CALCEI rational fits
 *             (:29-232); here the power series (|x| <= 1, x <= 40), the E1
 *             continued fraction (x < -1) and the asymptotic series (x > 40),
 *             the same function to ~1e-15 relative (tests pin it to scipy).
 */
#include "torj_oracle.h"

#include <complex.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SQRT_PI 1.7724538509055160272981674833411
#define EULER 0.57721566490153286060651209008240
#define NTV 501
#define TMAX 5.0
#define I_MAX 5 /* src/constants.jl:4 */

typedef double complex cplx;
#ifndef CMPLX /* C11; gnu99 has the builtin */
#define CMPLX(r, i) __builtin_complex((double)(r), (double)(i))
#endif

/* ---- the t-grid of the hermitian integration (repair R3; :8-13) ---- */
static double g_ttv[NTV], g_extdtv[NTV];

__attribute__((constructor)) static void init_tgrid(void) {
    const double dt = 2.0 * TMAX / (NTV - 1);
    for (int k = 0; k < NTV; ++k) {
        g_ttv[k] = -TMAX + dt * k;
        g_extdtv[k] = exp(-g_ttv[k] * g_ttv[k]) * dt;
    }
}

/* ---- e^-x Ei(x) (src/general_absorption.jl:29-232); -1.79e308 at 0 ---- */
double or_expei(double x) {
    if (x == 0.0) return -1.79e308;
    const double ax = fabs(x);
    if (ax > 700.0 || x > 40.0) {
        /* asymptotic: (1/x) sum_k k! / x^k; beyond 700 the 30-term sum of
         * warm_ref.expei, below it (x in (40, 700]) summed to its smallest term */
        double s = 0.0, term = 1.0;
        if (ax > 700.0) {
            for (int k = 0; k < 30; ++k) {
                s += term;
                term *= (k + 1) / x;
            }
        } else {
            for (int k = 0; k < 200; ++k) {
                s += term;
                const double nt = term * (k + 1) / x;
                if (fabs(nt) >= fabs(term) || fabs(nt) < 1e-17 * fabs(s)) break;
                term = nt;
            }
        }
        return s / x;
    }
    if (x < -1.0) {
        /* E1(y) = e^-y / (y + 1 - 1^2 / (y + 3 - 2^2 / (y + 5 - ...))) by modified
         * Lentz; e^-x Ei(x) = -e^y E1(y) is the bare fraction */
        const double y = -x, tiny = 1e-300;
        double b = y + 1.0, c = 1.0 / tiny, d = 1.0 / b, h = d;
        for (int i = 1; i < 1000; ++i) {
            const double an = -(double)i * i;
            b += 2.0;
            d = 1.0 / (an * d + b);
            c = b + an / c;
            const double del = c * d;
            h *= del;
            if (fabs(del - 1.0) < 1e-16) break;
        }
        return -h;
    }
    /* Ei(x) = gamma + ln|x| + sum_k x^k / (k k!), x in [-1, 40] */
    double s = 0.0, term = 1.0;
    for (int k = 1; k < 300; ++k) {
        term *= x / k;
        const double t = term / k;
        s += t;
        if (fabs(t) < 1e-17 * fabs(s)) break;
    }
    return (EULER + log(ax) + s) * exp(-x);
}

static double fact(int k) {  /* :240-257 */
    if (k < 0) return 0.0;
    double f = 1.0;
    for (int i = 2; i <= k; ++i) f *= i;
    return f;
}

/* Numerical Recipes lnGamma (:265-283), kept for ssbi's truncation parity */
static double gammln(double x) {
    static const double cof[6] = {76.18009172947146, -86.50532032941677, 24.01409824083091,
                                  -1.231739572450155, 0.1208650973866179e-2,
                                  -0.5395239384953e-5};
    double y = x, tmp = x + 5.5;
    tmp = (x + 0.5) * log(tmp) - tmp;
    double ser = 1.000000000190015;
    for (int j = 0; j < 6; ++j) {
        y += 1.0;
        ser += cof[j] / y;
    }
    return tmp + log(2.5066282746310005 * ser / x);
}

/* sum_k (zz^2/4)^k / (k! Gamma(m+k+3/2)), m = n .. l+2 (:291-320, repair R1) */
static void ssbi(double zz, int n, int l, double *out) {
    const double z2q = 0.25 * zz * zz;
    for (int m = n; m <= l + 2; ++m) {
        double c0 = 1.0 / exp(gammln(m + 1.5)), s = c0;
        for (int k = 1; k <= 50; ++k) {
            const double c1 = c0 * z2q / ((m + k) + 0.5) / k;
            s += c1;
            if (c1 / s < 1e-10) break;
            c0 = c1;
        }
        out[m - n] = s;
    }
}

/* Z(x + iy) = i sqrt(pi) w(x + iy) by TOMS 680 (:345-465) */
static cplx zetac(double xi, double yi) {
    const double factor = 1.12837916709551257388, rpi = 2.0 / factor;
    const double xabs = fabs(xi), yabs = fabs(yi);
    const double x = xabs / 6.3, y = yabs / 4.4;
    double qrho = x * x + y * y;
    double xquad = xabs * xabs - yabs * yabs;
    const double yquad = 2.0 * xabs * yabs;
    double u, v, u2 = 0.0, v2 = 0.0;
    if (qrho < 0.085264) {
        /* power series, Abramowitz & Stegun 7.1.5 */
        qrho = (1.0 - 0.85 * y) * sqrt(qrho);
        const int n = (int)nearbyint(6.0 + 72.0 * qrho);
        int j = 2 * n + 1;
        double xsum = 1.0 / j, ysum = 0.0;
        for (int i = n; i >= 1; --i) {
            j -= 2;
            const double xaux = (xsum * xquad - ysum * yquad) / i;
            ysum = (xsum * yquad + ysum * xquad) / i;
            xsum = xaux + 1.0 / j;
        }
        const double u1 = -factor * (xsum * yabs + ysum * xabs) + 1.0;
        const double v1 = factor * (xsum * xabs - ysum * yabs);
        const double daux = exp(-xquad);
        u2 = daux * cos(yquad);
        v2 = -daux * sin(yquad);
        u = u1 * u2 - v1 * v2;
        v = u1 * v2 + v1 * u2;
    } else {
        /* Laplace continued fraction or truncated Taylor expansion */
        double h = 0.0, h2 = 0.0, qlambda = 0.0;
        int kapn = 0, nu;
        if (qrho > 1.0) {
            qrho = sqrt(qrho);
            nu = 3 + (int)trunc(1442.0 / (26.0 * qrho + 77.0));
        } else {
            qrho = (1.0 - y) * sqrt(1.0 - qrho);
            h = 1.88 * qrho;
            h2 = 2.0 * h;
            kapn = (int)nearbyint(7.0 + 34.0 * qrho);
            nu = (int)nearbyint(16.0 + 26.0 * qrho);
        }
        if (h > 0.0) qlambda = pow(h2, kapn);
        double rx = 0.0, ry = 0.0, sx = 0.0, sy = 0.0;
        for (int n = nu; n >= 0; --n) {
            const int np1 = n + 1;
            double tx = yabs + h + np1 * rx;
            const double ty = xabs - np1 * ry;
            const double c = 0.5 / (tx * tx + ty * ty);
            rx = c * tx;
            ry = c * ty;
            if (h > 0.0 && n <= kapn) {
                tx = qlambda + sx;
                sx = rx * tx - ry * sy;
                sy = ry * tx + rx * sy;
                qlambda /= h2;
            }
        }
        if (h == 0.0) {
            u = factor * rx;
            v = factor * ry;
        } else {
            u = factor * sx;
            v = factor * sy;
        }
        if (yabs == 0.0) u = exp(-xabs * xabs);
    }
    if (yi < 0.0) {  /* the other quadrants (unused by fsup, whose y >= 0) */
        if (qrho < 0.085264) {
            u2 *= 2.0;
            v2 *= 2.0;
        } else {
            xquad = -xquad;
            const double w1 = 2.0 * exp(xquad);
            u2 = w1 * cos(yquad);
            v2 = -w1 * sin(yquad);
        }
        u = u2 - u;
        v = v2 - v;
        if (xi > 0.0) v = -v;
    } else if (xi < 0.0) {
        v = -v;
    }
    return CMPLX(-v * rpi, u * rpi);
}

void or_zetac(double x, double y, double out[2]) {
    const cplx z = zetac(x, y);
    out[0] = creal(z);
    out[1] = cimag(z);
}

/* Shkarofsky-function coefficients cefp / cefm[(lrm+1)][3] (:473-561) */
static void fsup(double yg, double anpl, double amu, int lrm, cplx cefp[][3],
                 cplx cefm[][3]) {
    memset(cefp, 0, sizeof(cplx) * 3 * (lrm + 1));
    memset(cefm, 0, sizeof(cplx) * 3 * (lrm + 1));
    const double anpl2hm1 = anpl * anpl / 2.0 - 1.0;
    const double psi = sqrt(0.5 * amu) * anpl, apsi = fabs(psi);
    for (int is = -lrm; is <= lrm; ++is) {
        const double alpha = anpl2hm1 + is * yg, phi2 = amu * alpha;
        const double phim = sqrt(fabs(phi2));
        double xp, yp, xm, ym, x0, y0;
        if (alpha >= 0) {
            xp = psi - phim; yp = 0.0; xm = -psi - phim; ym = 0.0; x0 = -phim; y0 = 0.0;
        } else {
            xp = psi; yp = phim; xm = -psi; ym = phim; x0 = 0.0; y0 = phim;
        }
        const cplx czp = zetac(xp, yp), czm = zetac(xm, ym);
        cplx cf12;
        if (alpha > 0)
            cf12 = -(czp + czm) / (2.0 * phim);
        else if (alpha < 0)
            cf12 = -I * (czp + czm) / (2.0 * phim);
        else
            cf12 = 0.0;
        cplx cf32;
        if (apsi > 0.7) {
            cf32 = -(czp - czm) / (2.0 * psi);
        } else {
            const cplx cphi = alpha < 0 ? -I * phim : (cplx)phim;
            cf32 = 2.0 * (1.0 - cphi * zetac(x0, y0));
        }
        cplx cf0 = cf12, cf1 = cf32;
        if (is == 0) {
            cefp[0][0] = cf32;
            cefm[0][0] = cf32;
        }
        const int isa = abs(is);
        for (int l = 1; l <= isa + 2; ++l) {
            cplx cf2;
            if (apsi > 0.7)
                cf2 = (1.0 + phi2 * cf0 - (l - 0.5) * cf1) / (psi * psi);
            else
                cf2 = (1.0 + phi2 * cf1) / (l + 0.5);
            const int ir = l - isa;
            if (ir >= 0) {
                cefp[isa][ir] += cf2;
                cefm[isa][ir] += is > 0 ? cf2 : -cf2;
            }
            cf0 = cf1;
            cf1 = cf2;
        }
    }
}

/* the 6 independent tensor components per order l (11 12 22 13 23 33), from
 * the harmonic sums ca, with warm_ref._finish_tensor's +1 on 11 / 22 at l = 1 */
static void tensor_order(double xg, double f, const cplx ca[6], int l, cplx eps[6]) {
    eps[0] = -xg * ca[0] * f;
    eps[1] = I * xg * ca[1] * f;
    eps[2] = -xg * ca[2] * f;
    eps[3] = -xg * ca[3] * f;
    eps[4] = -I * xg * ca[4] * f;
    eps[5] = -xg * ca[5] * f;
    if (l == 1) {
        eps[0] += 1.0;
        eps[2] += 1.0;
    }
}

static void harmonic_terms(int l, int is, double yg, cplx cq0p, cplx cq0m, cplx cq1p,
                           cplx cq1m, cplx cq2p, cplx ca[6]) {
    const int lm = l - 1, k = l - is;
    const double asl = ((k & 1) ? -1.0 : 1.0) / (fact(is + l) * fact(l - is));
    const double bsl = asl * (is * is + (double)(2 * k * lm * (l + is)) / (2 * l - 1));
    ca[0] += (double)(is * is) * asl * cq0p;
    ca[1] += (double)(is * l) * asl * cq0m;
    ca[2] += bsl * cq0p;
    ca[3] += is * asl * cq1m / yg;
    ca[4] += l * asl * cq1p / yg;
    ca[5] += asl * cq2p / (yg * yg);
}

/* weakly relativistic tensor, Krivenski & Orefice (:573-638) */
static cplx dieltens_wr(double xg, double yg, double anpl, double amu, int lrm,
                        cplx epsl[][6]) {
    const double anpl2 = anpl * anpl;
    cplx cefp[I_MAX + 1][3], cefm[I_MAX + 1][3];
    fsup(yg, anpl, amu, lrm, cefp, cefm);
    for (int l = 1; l <= lrm; ++l) {
        const int lm = l - 1;
        const double fcl = pow(0.5, l) * pow((1.0 / yg) * (1.0 / yg) / amu, lm) *
                           fact(2 * l) / fact(l);
        cplx ca[6] = {0};
        for (int is = 0; is <= l; ++is) {
            const cplx cq0p = amu * cefp[is][0], cq0m = amu * cefm[is][0];
            const cplx cq1p = amu * anpl * (cefp[is][0] - cefp[is][1]);
            const cplx cq1m = amu * anpl * (cefm[is][0] - cefm[is][1]);
            const cplx cq2p = cefp[is][1] +
                              amu * anpl2 * (cefp[is][2] + cefp[is][0] - 2.0 * cefp[is][1]);
            harmonic_terms(l, is, yg, cq0p, cq0m, cq1p, cq1m, cq2p, ca);
        }
        tensor_order(xg, fcl, ca, l, epsl[l - 1]);
    }
    const cplx cq2p = cefp[0][1] + amu * anpl2 * (cefp[0][2] + cefp[0][0] - 2.0 * cefp[0][1]);
    return 1.0 - xg * amu * cq2p;
}

/* hermitian part, t-integration of the iwarm > 2 branch (:646-734):
 * rr[n + lrm][k][m], n in [-llm, llm], k = 0..2, m = 0..llm */
static void hermitian(double yg, double anpl, double amu, int lrm,
                      double rr[2 * I_MAX + 1][3][I_MAX + 1]) {
    memset(rr, 0, sizeof(double) * (2 * I_MAX + 1) * 3 * (I_MAX + 1));
    const double cmxw = 1.0 + 15.0 / (8.0 * amu) + 105.0 / (128.0 * amu * amu);
    const double cr = -amu * amu / (SQRT_PI * cmxw);
    const int llm = lrm < 3 ? lrm : 3;
    const double bth2 = 2.0 / amu, bth = sqrt(bth2);
    const double amu2 = amu * amu, amu4 = amu2 * amu2, amu6 = amu2 * amu2 * amu2;
    for (int k = 0; k < NTV; ++k) {
        const double t = g_ttv[k];
        const double rxt = sqrt(1.0 + t * t / (2.0 * amu));
        const double x = t * rxt, upl2 = bth2 * x * x, upl = bth * x;
        const double gx = 1.0 + t * t / amu;
        const double exdx = cr * g_extdtv[k] * gx / rxt;
        for (int n = -llm; n <= llm; ++n) {
            const double gr = anpl * upl + n * yg;
            const double zm = -amu * (gx - gr), s = amu * (gx + gr);
            const double fe0m = or_expei(zm);
            for (int m = abs(n); m <= llm; ++m) {
                if (m == 0) {
                    rr[lrm][2][0] += -exdx * fe0m * upl2;
                    continue;
                }
                const double zm2 = zm * zm;
                double ffe;
                if (m == 1)
                    ffe = (1.0 + s * (1.0 - zm * fe0m)) / amu2;
                else if (m == 2)
                    ffe = (6.0 - 2.0 * zm + 4.0 * s + s * s * (1.0 + zm - zm2 * fe0m)) / amu4;
                else
                    ffe = (18.0 * s * (s + 4.0 - zm) + 6.0 * (20.0 - 8.0 * zm + zm2) +
                           s * s * s * (2.0 + zm + zm2 - zm2 * zm * fe0m)) / amu6;
                rr[n + lrm][0][m] += exdx * ffe;
                rr[n + lrm][1][m] += exdx * ffe * upl;
                rr[n + lrm][2][m] += exdx * ffe * upl2;
            }
        }
    }
}

/* anti-hermitian part (:951-1043): ri[n-1][k][m-1], m >= n */
static void antihermitian(double yg, double anpl, double amu, int lrm,
                          double ri[I_MAX][3][I_MAX]) {
    memset(ri, 0, sizeof(double) * I_MAX * 3 * I_MAX);
    const double dnl = 1.0 - anpl * anpl, cmu = anpl * amu;
    const double cmxw = 1.0 + 15.0 / (8.0 * amu) + 105.0 / (128.0 * amu * amu);
    const double ci = sqrt(2.0 * M_PI * amu) * amu * amu / cmxw;
    for (int n = 1; n <= lrm; ++n) {
        const double ygn = n * yg, rdu2 = ygn * ygn - dnl;
        if (!(rdu2 > 0.0)) continue;
        const double rdu = sqrt(rdu2), du = rdu / dnl, ub = anpl * ygn / dnl;
        const double aa = amu * anpl * du;
        if (fabs(aa) > 5.0) {
            const double up = ub + du, um = ub - du;
            const double gp = anpl * up + ygn, gm = anpl * um + ygn;
            const double xp = up + 1.0 / cmu, xm = um + 1.0 / cmu;
            const double eem = exp(-amu * (gm - 1.0)), eep = exp(-amu * (gp - 1.0));
            double f0p = -1.0 / cmu, f1p = -xp / cmu, f2p = -(1.0 / (cmu * cmu) + xp * xp) / cmu;
            double f0m = -1.0 / cmu, f1m = -xm / cmu, f2m = -(1.0 / (cmu * cmu) + xm * xm) / cmu;
            for (int m = 1; m <= lrm; ++m) {
                const double g0p = -2.0 * m * (f1p - ub * f0p) / cmu;
                const double g0m = -2.0 * m * (f1m - ub * f0m) / cmu;
                const double g1p =
                    -((1.0 + 2 * m) * f2p - 2.0 * (m + 1) * ub * f1p + up * um * f0p) / cmu;
                const double g1m =
                    -((1.0 + 2 * m) * f2m - 2.0 * (m + 1) * ub * f1m + up * um * f0m) / cmu;
                const double g2p = (2.0 * (1 + m) * g1p - 2.0 * m * (ub * f2p - up * um * f1p)) / cmu;
                const double g2m = (2.0 * (1 + m) * g1m - 2.0 * m * (ub * f2m - up * um * f1m)) / cmu;
                if (m >= n) {
                    const double h = 0.5 * ci * pow(dnl, m);
                    ri[n - 1][0][m - 1] = h * (g0p * eep - g0m * eem);
                    ri[n - 1][1][m - 1] = h * (g1p * eep - g1m * eem);
                    ri[n - 1][2][m - 1] = h * (g2p * eep - g2m * eem);
                }
                f0p = g0p; f1p = g1p; f2p = g2p;
                f0m = g0m; f1m = g1m; f2m = g2m;
            }
        } else {
            const double ee = exp(-amu * (ygn - 1.0 + anpl * ub));
            double fsbi[I_MAX + 3];
            ssbi(aa, n, lrm, fsbi);
            for (int m = n; m <= lrm; ++m) {
                const double cm = SQRT_PI * fact(m) * pow(du, 2 * m + 1);
                const double cim = 0.5 * ci * pow(dnl, m);
                const int mm = m - n;
                const double fi0 = cm * fsbi[mm];
                const double fi1 = -0.5 * aa * cm * fsbi[mm + 1];
                const double fi2 = 0.5 * cm * (fsbi[mm + 1] + 0.5 * aa * aa * fsbi[mm + 2]);
                ri[n - 1][0][m - 1] = cim * ee * fi0;
                ri[n - 1][1][m - 1] = cim * ee * (du * fi1 + ub * fi0);
                ri[n - 1][2][m - 1] = cim * ee * (du * du * fi2 + 2.0 * du * ub * fi1 + ub * ub * fi0);
            }
        }
    }
}

/* fully relativistic tensor, iwarm = 3 (:1056-1134) */
static cplx dieltens_fr(double xg, double yg, double anpl, double amu, int lrm,
                        cplx epsl[][6]) {
    double rr[2 * I_MAX + 1][3][I_MAX + 1], ri[I_MAX][3][I_MAX];
    hermitian(yg, anpl, amu, lrm, rr);
    antihermitian(yg, anpl, amu, lrm, ri);
    for (int l = 1; l <= lrm; ++l) {
        const int lm = l - 1;
        const double fl = fact(l);
        const double fal = -pow(0.25, l) * fact(2 * l) / (fl * fl * pow(yg, 2 * lm));
        cplx ca[6] = {0};
        for (int is = 0; is <= l; ++is) {
            cplx cq0p, cq0m, cq1p, cq1m, cq2p;
            if (is > 0) {
                const double *a = rr[lrm + is][0], *b = rr[lrm - is][0];
                const int st = I_MAX + 1; /* stride between k rows */
                const double i0 = ri[is - 1][0][l - 1], i1 = ri[is - 1][1][l - 1],
                             i2 = ri[is - 1][2][l - 1];
                cq0p = CMPLX(a[l] + b[l], i0);
                cq0m = CMPLX(a[l] - b[l], i0);
                cq1p = CMPLX(a[st + l] + b[st + l], i1);
                cq1m = CMPLX(a[st + l] - b[st + l], i1);
                cq2p = CMPLX(a[2 * st + l] + b[2 * st + l], i2);
            } else {
                cq0p = cq0m = rr[lrm][0][l];
                cq1p = cq1m = rr[lrm][1][l];
                cq2p = rr[lrm][2][l];
            }
            harmonic_terms(l, is, yg, cq0p, cq0m, cq1p, cq1m, cq2p, ca);
        }
        tensor_order(xg, fal, ca, l, epsl[l - 1]);
    }
    return 1.0 + xg * rr[lrm][2][0];
}

/* warm dispersion relation for N_perp (:1158-1267, repair R2) -> anpr^2 */
static cplx warmdisp(double xg, double yg, double anpl, double amu, double anprc, int sox,
                     int iwarm, int lrm, int *ierr) {
    cplx anpr2a = anprc * anprc, anpr2 = anpr2a;
    const double anpl2 = anpl * anpl;
    cplx epsl[I_MAX][6];
    const cplx e330 = iwarm == 1 ? dieltens_wr(xg, yg, anpl, amu, lrm, epsl)
                                 : dieltens_fr(xg, yg, anpl, amu, lrm, epsl);
    double errnpr = 1.0;
    for (int i = 1; i <= 100; ++i) {
        cplx sep[6] = {0}, pw = 1.0;
        for (int il = 0; il < lrm; ++il) {
            for (int c = 0; c < 6; ++c) sep[c] += epsl[il][c] * pw;
            pw *= anpr2a;
        }
        const cplx e11 = sep[0], e12 = sep[1], e22 = sep[2];
        const cplx a13 = sep[3], a23 = sep[4], a33 = sep[5];
        const cplx a31 = a13, a32 = -a23;
        if (i > 2 && errnpr < 1.0e-4) break;
        const cplx cc4 = (e11 - anpl2) * (1.0 - a33) + (a13 + anpl) * (a31 + anpl);
        const cplx cc2 = -e12 * e12 * (1.0 - a33) - a32 * e12 * (a13 + anpl) +
                         a23 * e12 * (a31 + anpl) -
                         (a23 * a32 + e330 + (e22 - anpl2) * (1.0 - a33)) * (e11 - anpl2) -
                         (a13 + anpl) * (a31 + anpl) * (e22 - anpl2);
        const cplx cc0 = e330 * ((e11 - anpl2) * (e22 - anpl2) + e12 * e12);
        const cplx rr = cc2 * cc2 - 4.0 * cc0 * cc4;
        double s;
        if (yg > 1.0) {
            s = sox;
            if (cimag(rr) <= 0.0) s = -s;
        } else {
            s = -sox;
            if (creal(rr) <= 0.0 && cimag(rr) >= 0.0) s = -s;
        }
        anpr2 = (-cc2 + s * csqrt(rr)) / (2.0 * cc4);
        errnpr = fabs(1.0 - cabs(anpr2) / cabs(anpr2a));
        anpr2a = anpr2;
    }
    *ierr = 0;
    if (creal(anpr2) < 0.0 && cimag(anpr2) < 0.0) {
        anpr2 = 0.0;
        *ierr = 99;
    }
    return anpr2;
}

/* highest harmonic with mu (gamma - 1) <= 15 on the resonance (:1285-1326) */
static int larmornumber(double yg, double npl, double mu) {
    const double dnl = 1.0 - npl * npl;
    int imax = 1, nharm = (int)floor(1.0 / yg);
    if (nharm * yg < 1.0) nharm += 1;
    for (;;) {
        const double ygn = nharm * yg, rdu2 = ygn * ygn - dnl;
        const double gg = (ygn - sqrt(npl * npl * rdu2)) / dnl;
        if (mu * (gg - 1.0) > 15.0) break;
        nharm += 1;
        imax += 1;
        if (imax > 100) {
            nharm = (int)floor(yg);
            break;
        }
    }
    return nharm;
}

/* alpha (:1328-1337) with theta from (N_abs, N_par), v_g_perp = 1 / |dD/dN| (R4)
 * and sox = +-mode (R5).  N_perp_warm^2 into n2[2] when n2 != NULL. */
double or_alpha_warm(double omega, double X, double Y, double N_abs, double N_par, double Te,
                     double inv_dDdN, int mode, int iwarm, double *n2) {
    const double mu = OR_ME * OR_C * OR_C / (Te * OR_E);
    const double npr = sqrt(fmax(N_abs * N_abs - N_par * N_par, 0.0));
    const int nharm = larmornumber(Y, N_par, mu);
    const int lrm = nharm < I_MAX ? nharm : I_MAX;
    const int sox = Y <= 1.0 ? mode : -mode;
    int ierr;
    const cplx anpr = csqrt(warmdisp(X, Y, N_par, mu, npr, sox, iwarm, lrm, &ierr));
    const cplx a2 = anpr * anpr;
    if (n2) {
        n2[0] = creal(a2);
        n2[1] = cimag(a2);
    }
    return 2.0 * cimag(a2) * omega / OR_C * inv_dDdN;
}
