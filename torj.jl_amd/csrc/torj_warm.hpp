// torj_warm.hpp -- warm-plasma EC absorption (src/general_absorption.jl,
// GRAY's warm dispersion module), restated for the device and repaired as
// described in oracle/warm_ref.py (R1-R5):
//   warmdisp (:1158-1267) solves the warm dispersion relation for N_perp with
//   the weakly relativistic tensor (iwarm 1: fsup + the plasma dispersion
//   function, :473-638) or the fully relativistic one (iwarm 3, what the
//   reference's alpha hard-codes: hermitian part by the 501-node t-quadrature
//   with exp(-x) Ei(x), anti-hermitian part analytic, :646-1134); larmornumber
//   (:1285-1326) sets the Larmor-radius order; alpha (:1328-1337) =
//   2 Im(N_perp^2) (omega / c) v_g_perp with v_g_perp = 1 / |dD/dN|.
// One lane evaluates one point; small tensors live in the lane's private
// memory.  This is the heavy-VALU configuration C5 (~1e5 flop per alpha).
#pragma once
#include "torj_faddeeva_coefs.hpp"
#include "torj_math.hpp"

namespace torj {

// Region timers of the warm alpha kernel -- a profiling build only
// (-DTORJ_WARM_PROF; scripts/mkvariant.py, tools/warm_prof.py), compiled out
// otherwise.  TORJ_WPROF(k) charges the wave's wall clock since its previous
// mark to region k; the first active lane keeps the stamps in LDS (one wave
// per workgroup), k_alpha_warm_pts flushes them once per wave.
#ifdef TORJ_WARM_PROF
constexpr int kWProfN = 8;
#ifdef TORJ_TRAJ_TU
static
#endif
__device__ unsigned long long g_wprof[kWProfN + 1];
#ifdef TORJ_TRAJ_TU
static
#endif
__device__ unsigned long long g_wfad[9];  // faddeeva_upper2's branch statistics (see there)
#endif
#if defined(TORJ_WARM_PROF) && defined(__HIP_DEVICE_COMPILE__)
__shared__ unsigned long long s_wprof[kWProfN + 1];
__device__ __forceinline__ bool wprof_leader() {
    return (int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1;
}
__device__ __forceinline__ void wprof_mark(int k) {
    const unsigned long long t = clock64();
    if (wprof_leader()) {
        s_wprof[1 + k] += t - s_wprof[0];
        s_wprof[0] = t;
    }
}
__device__ __forceinline__ void wprof_init() {
    if (wprof_leader()) {
        for (int k = 1; k <= kWProfN; k++) s_wprof[k] = 0;
        s_wprof[0] = clock64();
    }
}
__device__ __forceinline__ void wprof_flush() {
    if (wprof_leader()) {
        for (int k = 1; k <= kWProfN; k++) atomicAdd(&g_wprof[k], s_wprof[k]);
        atomicAdd(&g_wprof[0], 1ull);
    }
}
#define TORJ_WPROF(k) wprof_mark(k)
#else
#define TORJ_WPROF(k) ((void)0)
#endif

struct cplx {
    double re, im;
};
TORJ_HD cplx C(double r, double i = 0.0) { return cplx{r, i}; }
TORJ_HD cplx operator+(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
TORJ_HD cplx operator-(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
TORJ_HD cplx operator-(cplx a) { return {-a.re, -a.im}; }
TORJ_HD cplx operator*(cplx a, cplx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
TORJ_HD cplx operator*(double s, cplx a) { return {s * a.re, s * a.im}; }
TORJ_HD cplx operator*(cplx a, double s) { return {s * a.re, s * a.im}; }
TORJ_HD cplx operator/(cplx a, double s) {
    const double r = 1.0 / s;
    return {a.re * r, a.im * r};
}
TORJ_HD cplx operator/(cplx a, cplx b) {  // Smith's algorithm
    if (fabs(b.re) >= fabs(b.im)) {
        const double r = b.im / b.re, id = 1.0 / (b.re + b.im * r);
        return {(a.re + a.im * r) * id, (a.im - a.re * r) * id};
    }
    const double r = b.re / b.im, id = 1.0 / (b.re * r + b.im);
    return {(a.re * r + a.im) * id, (a.im * r - a.re) * id};
}
TORJ_HD cplx operator+(double s, cplx a) { return {s + a.re, a.im}; }
TORJ_HD cplx operator-(double s, cplx a) { return {s - a.re, -a.im}; }
TORJ_HD cplx operator+(cplx a, double s) { return {a.re + s, a.im}; }
TORJ_HD cplx operator-(cplx a, double s) { return {a.re - s, a.im}; }
TORJ_HD cplx I_times(cplx a) { return {-a.im, a.re}; }
TORJ_HD double cabs_(cplx a) { return hypot(a.re, a.im); }
TORJ_HD double cnorm_(cplx a) { return fma(a.re, a.re, a.im * a.im); }  // |a|^2
// principal branch, as Julia's sqrt(::ComplexF64): for the moderate operands of
// warmdisp (|z|^2 a normal double) |z| from the sum of squares without hypot's
// scaling, one reciprocal instead of two divisions (~1 ulp); where |z|^2
// underflows to 0 / a subnormal or overflows (|z| beyond ~1e-154 .. 1e154, e.g.
// the discriminant near mode coupling) |z| by hypot, as before -- one compare,
// almost never taken
TORJ_HD cplx csqrt_(cplx z) {
    if (z.re == 0.0 && z.im == 0.0) return {0.0, z.im};
    const double n2 = cnorm_(z);
    const double r = (n2 >= 0x1p-1022 && n2 < INFINITY) ? sqrt_nn(n2) : hypot(z.re, z.im);
    const double t = sqrt_nn(0.5 * (r + fabs(z.re))), h = 0.5 * rcp_nz(t);
    if (z.re >= 0.0) return {t, z.im * h};
    return {fabs(z.im) * h, copysign(t, z.im)};
}

constexpr double kSqrtPi = 1.7724538509055160272981674833411;
constexpr double kEulerGamma = 0.57721566490153286060651209008240243;
constexpr int kWarmMaxL = 5;  // i_max (src/constants.jl:4)
constexpr int kNtv = 501;     // t-quadrature (src/constants.jl:1-3)
constexpr double kTmax = 5.0, kDtv = 2.0 * kTmax / (kNtv - 1);

// exp(x) in constant evaluation (x <= 0): x = k ln2 + r, |r| <= ln2/2, a
// 24-term Taylor sum for e^r and an exact power-of-two scaling (~1 ulp)
constexpr double cexp(double x) {
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
    const double kf = x / (ln2hi + ln2lo);
    const long k = (long)(kf < 0 ? kf - 0.5 : kf + 0.5);
    const double r = (x - k * ln2hi) - k * ln2lo;
    double term = 1.0, sum = 1.0;
    for (int i = 1; i < 24; i++) {
        term *= r / i;
        sum += term;
    }
    for (long j = 0; j < (k < 0 ? -k : k); j++) sum = k < 0 ? sum * 0.5 : sum * 2.0;
    return sum;
}
// the quadrature weights exp(-t_i^2) dt of the fully relativistic hermitian
// part (:646-950): t-only, so a compile-time table (scalar loads: i is uniform)
struct FrWeights {
    double w[kNtv];
};
constexpr FrWeights make_fr_weights() {
    FrWeights f{};
    for (int i = 0; i < kNtv; i++) {
        const double t = -kTmax + i * kDtv;
        f.w[i] = cexp(-t * t) * kDtv;
    }
    return f;
}
#ifdef __HIP_DEVICE_COMPILE__
__constant__ constexpr FrWeights kFrW = make_fr_weights();
#else
constexpr FrWeights kFrW = make_fr_weights();
#endif

// exp(-x) Ei(x) (expei, :29-232): W. J. Cody's CALCEI (int = 3), the
// algorithm the reference transliterates -- fixed-cost rational
// approximations per interval (Cody & Thacher, Math. Comp. 22 (1968) and 23
// (1969); SPECFUN), with their published coefficients:
//   x < 0:       y = -x: y <= 1  (ln y - P6(y)/Q6(y)) e^y,
//                        y <= 4  -P8(1/y)/Q8(1/y),
//                        y > 4   w (w P9(w)/Q9(w) - 1), w = 1/y;
//   0 < x < 6:   Chebyshev-form ratio in t = 2x/3 - 2, with ln(x/x0) near the
//                zero x0 of Ei;
//   6 <= x < 24: J-fractions; x >= 24: J-fraction in 1/x.
// -1.79e308 at x = 0 (the reference's -xinf).
namespace cody {
constexpr double A[7] = {1.1669552669734461083368e2, 2.1500672908092918123209e3, 1.5924175980637303639884e4,
                         8.9904972007457256553251e4, 1.5026059476436982420737e5, -1.4815102102575750838086e5,
                         5.0196785185439843791020e0};
constexpr double B[6] = {4.0205465640027706061433e1, 7.5043163907103936624165e2, 8.1258035174768735759855e3,
                         5.2440529172056355429883e4, 1.8434070063353677359298e5, 2.5666493484897117319268e5};
constexpr double C[9] = {3.828573121022477169108e-1, 1.107326627786831743809e+1, 7.246689782858597021199e+1,
                         1.700632978311516129328e+2, 1.698106763764238382705e+2, 7.633628843705946890896e+1,
                         1.487967702840464066613e+1, 9.999989642347613068437e-1, 1.737331760720576030932e-8};
constexpr double D[9] = {8.258160008564488034698e-2, 4.344836335509282083360e+0, 4.662179610356861756812e+1,
                         1.775728186717289799677e+2, 2.953136335677908517423e+2, 2.342573504717625153053e+2,
                         9.021658450529372642314e+1, 1.587964570758947927903e+1, 1.0};
constexpr double E[10] = {1.3276881505637444622987e+2, 3.5846198743996904308695e+4, 1.7283375773777593926828e+5,
                          2.6181454937205639647381e+5, 1.7503273087497081314708e+5, 5.9346841538837119172356e+4,
                          1.0816852399095915622498e+4, 1.0611777263550331766871e+3, 5.2199632588522572481039e+1,
                          9.9999999999999999087819e-1};
constexpr double F[10] = {3.9147856245556345627078e+4, 2.5989762083608489777411e+5, 5.5903756210022864003380e+5,
                          5.4616842050691155735758e+5, 2.7858134710520842139357e+5, 7.9231787945279043698718e+4,
                          1.2842808586627297365998e+4, 1.1635769915320848035459e+3, 5.4199632588522559414924e+1,
                          1.0};
constexpr double PLG[4] = {-2.4562334077563243311e+01, 2.3642701335621505212e+02, -5.4989956895857911039e+02,
                           3.5687548468071500413e+02};
constexpr double QLG[4] = {-3.5553900764052419184e+01, 1.9400230218539473193e+02, -3.3442903192607538956e+02,
                           1.7843774234035750207e+02};
constexpr double P[10] = {-1.2963702602474830028590e+01, -1.2831220659262000678155e+03, -1.4287072500197005777376e+04,
                          -1.4299841572091610380064e+06, -3.1398660864247265862050e+05, -3.5377809694431133484800e+08,
                          3.1984354235237738511048e+08, -2.5301823984599019348858e+10, 1.2177698136199594677580e+10,
                          -2.0829040666802497120940e+11};
constexpr double Q[10] = {7.6886718750000000000000e+01, -5.5648470543369082846819e+03, 1.9418469440759880361415e+05,
                          -4.2648434812177161405483e+06, 6.4698830956576428587653e+07, -7.0108568774215954065376e+08,
                          5.4229617984472955011862e+09, -2.8986272696554495342658e+10, 9.8900934262481749439886e+10,
                          -8.9673749185755048616855e+10};
constexpr double R[10] = {-2.645677793077147237806e+00, -2.378372882815725244124e+00, -2.421106956980653511550e+01,
                          1.052976392459015155422e+01, 1.945603779539281810439e+01, -3.015761863840593359165e+01,
                          1.120011024227297451523e+01, -3.988850730390541057912e+00, 9.565134591978630774217e+00,
                          9.981193787537396413219e-1};
constexpr double S[9] = {1.598517957704779356479e-4, 4.644185932583286942650e+00, 3.697412299772985940785e+02,
                         -8.791401054875438925029e+00, 7.608194509086645763123e+02, 2.852397548119248700147e+01,
                         4.731097187816050252967e+02, -2.369210235636181001661e+02, 1.249884822712447891440e+00};
constexpr double P1[10] = {-1.647721172463463140042e+00, -1.860092121726437582253e+01, -1.000641913989284829961e+01,
                           -2.105740799548040450394e+01, -9.134835699998742552432e-1, -3.323612579343962284333e+01,
                           2.495487730402059440626e+01, 2.652575818452799819855e+01, -1.845086232391278674524e+00,
                           9.999933106160568739091e-1};
constexpr double Q1[9] = {9.792403599217290296840e+01, 6.403800405352415551324e+01, 5.994932325667407355255e+01,
                          2.538819315630708031713e+02, 4.429413178337928401161e+01, 1.192832423968601006985e+03,
                          1.991004470817742470726e+02, -1.093556195391091143924e+01, 1.001533852045342697818e+00};
constexpr double P2[10] = {1.75338801265465972390e+02, -2.23127670777632409550e+02, -1.81949664929868906455e+01,
                           -2.79798528624305389340e+01, -7.63147701620253630855e+00, -1.52856623636929636839e+01,
                           -7.06810977895029358836e+00, -5.00006640413131002475e+00, -3.00000000320981265753e+00,
                           1.00000000000000485503e+00};
constexpr double Q2[9] = {3.97845977167414720840e+04, 3.97277109100414518365e+00, 1.37790390235747998793e+02,
                          1.17179220502086455287e+02, 7.04831847180424675988e+01, -1.20187763547154743238e+01,
                          -7.99243595776339741065e+00, -2.99999894040324959612e+00, 1.99999999999048104167e+00};
constexpr double kX0 = 0.37250741078136663466;  // zero of Ei
constexpr double kX01 = 381.5, kX11 = 1024.0, kX02 = -5.1182968633365538008e-5;

// P(u) / Q(u) with leading coefficients first (Horner), N terms each
template <int NP, int NQ>
TORJ_HD double ratio(const double (&p)[NP], const double (&q)[NQ], double u) {
    double sp = p[0], sq = q[0];
#pragma unroll
    for (int i = 1; i < NP; i++) sp = fma(sp, u, p[i]);
#pragma unroll
    for (int i = 1; i < NQ; i++) sq = fma(sq, u, q[i]);
    return sp * rcp_nz(sq);  // Cody's denominators are positive on their intervals
}

// J-fraction s1/(r1 + x + s2/(r2 + x + ...)), evaluated from the innermost term
template <int N>
TORJ_HD double jfrac(const double (&r)[N + 1], const double (&s)[N], double x) {
    double f = 0.0;
#pragma unroll
    for (int i = 0; i < N; i++) f = s[i] * rcp_nz(r[i] + x + f);
    return f;
}
}  // namespace cody

TORJ_HD double expei(double x) {
    if (x == 0.0) return -1.79e308;
    if (x < 0.0) {
        const double y = -x;
        if (y <= 1.0) {  // the y <= 1 numerator is stored in the reference's order: its last term leads
            double sp = fma(cody::A[6], y, cody::A[0]), sq = y + cody::B[0];
#pragma unroll
            for (int i = 1; i < 6; i++) {
                sp = fma(sp, y, cody::A[i]);
                sq = fma(sq, y, cody::B[i]);
            }
            return (log(y) - sp / sq) * exp(y);
        }
        const double w = rcp_nz(y);
        if (y <= 4.0) return -cody::ratio(cody::C, cody::D, w);
        return w * (w * cody::ratio(cody::E, cody::F, w) - 1.0);
    }
    if (x < 6.0) {  // Chebyshev-form ratio in t (Clenshaw-like three-term recurrence)
        const double t = (x + x) / 3.0 - 2.0;
        double pm1 = 0.0, qm1 = 0.0, pc = cody::P[0], qc = cody::Q[0];
#pragma unroll
        for (int i = 1; i < 9; i++) {
            const double pn = t * pc - pm1 + cody::P[i], qn = t * qc - qm1 + cody::Q[i];
            pm1 = pc, qm1 = qc, pc = pn, qc = qn;
        }
        const double frac = (0.5 * t * pc - pm1 + cody::P[9]) / (0.5 * t * qc - qm1 + cody::Q[9]);
        const double xmx0 = (x - cody::kX01 / cody::kX11) - cody::kX02;
        if (fabs(xmx0) >= 0.037) return exp(-x) * (log(x / cody::kX0) + xmx0 * frac);
        const double yy = xmx0 / (x + cody::kX0), ysq = yy * yy;  // ln(x/x0) near x0
        double sp = cody::PLG[0], sq = ysq + cody::QLG[0];
#pragma unroll
        for (int i = 1; i < 4; i++) {
            sp = fma(sp, ysq, cody::PLG[i]);
            sq = fma(sq, ysq, cody::QLG[i]);
        }
        return exp(-x) * (sp / (sq * (x + cody::kX0)) + frac) * xmx0;
    }
    if (x < 12.0) return (cody::R[9] + cody::jfrac<9>(cody::R, cody::S, x)) / x;
    if (x <= 24.0) return (cody::P1[9] + cody::jfrac<9>(cody::P1, cody::Q1, x)) / x;
    const double y = rcp_nz(x);
    return y + y * y * (cody::P2[9] + cody::jfrac<9>(cody::P2, cody::Q2, x));
}

TORJ_HD double factd(int k) {
    double f = 1.0;
    for (int i = 2; i <= k; i++) f *= (double)i;
    return k < 0 ? 0.0 : f;
}

// Numerical Recipes lnGamma, the reference's gammln (:265-283)
TORJ_HD double gammln_nr(double x) {
    const double cof[6] = {76.18009172947146,     -86.50532032941677, 24.01409824083091,
                           -1.231739572450155,    0.1208650973866179e-2, -0.5395239384953e-5};
    double y = x, tmp = x + 5.5;
    tmp = (x + 0.5) * log(tmp) - tmp;
    double ser = 1.000000000190015;
    for (int j = 0; j < 6; j++) {
        y += 1.0;
        ser += cof[j] / y;
    }
    return tmp + log(2.5066282746310005 * ser / x);
}

// I_{m+1/2}(z)/(z/2)^{m+1/2} series for m = n .. l+2 (ssbi, :291-320, R1)
TORJ_HD void ssbi(double zz, int n, int l, double out[kWarmMaxL + 3]) {
    const double z2q = 0.25 * zz * zz;
    for (int m = n; m <= l + 2; m++) {
        double c0 = 1.0 / exp(gammln_nr(m + 1.5)), s = c0;
        for (int k = 1; k <= 50; k++) {
            const double c1 = c0 * z2q / ((m + k) + 0.5) / k;
            s += c1;
            if (c1 / s < 1e-10) break;
            c0 = c1;
        }
        out[m - n] = s;
    }
}

// 1/x for normal x > 0: v_rcp_f64 plus two Newton steps on the device
// (~5 instructions against ~10 for the IEEE division sequence)
TORJ_HD double rcp_pos(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
#else
    return 1.0 / x;
#endif
}

// Faddeeva w(z) for Z(z) = i sqrt(pi) w(z) (zetac, :345-465): Poppe & Wijers,
// ACM TOMS 680 (series near the origin, Laplace continued fraction / truncated
// Taylor expansion otherwise, reflection for Im z < 0)
TORJ_HD cplx faddeeva(double xi, double yi) {
    const double factor = 1.12837916709551257388;  // 2/sqrt(pi)
    const double xabs = fabs(xi), yabs = fabs(yi);
    const double x = xabs * (1.0 / 6.3), y = yabs * (1.0 / 4.4);
    double qrho = x * x + y * y;
    const double xquad = xabs * xabs - yabs * yabs, yquad = 2.0 * xabs * yabs;
    double u, v, u2 = 0.0, v2 = 0.0;
    const bool small = qrho < 0.085264;
    if (small) {
        qrho = (1.0 - 0.85 * y) * sqrt(qrho);
        const int n = (int)rint(6.0 + 72.0 * qrho);
        int j = 2 * n + 1;
        double xsum = 1.0 / j, ysum = 0.0;
        for (int i = n; i >= 1; i--) {
            j -= 2;
            const double ri = rcp_pos((double)i);
            const double xaux = (xsum * xquad - ysum * yquad) * ri;
            ysum = (xsum * yquad + ysum * xquad) * ri;
            xsum = xaux + rcp_pos((double)j);
        }
        const double u1 = -factor * (xsum * yabs + ysum * xabs) + 1.0;
        const double v1 = factor * (xsum * xabs - ysum * yabs);
        const double daux = exp(-xquad);
        u2 = daux * cos(yquad);
        v2 = -daux * sin(yquad);
        u = u1 * u2 - v1 * v2;
        v = u1 * v2 + v1 * u2;
    } else {
        double h = 0.0, h2 = 0.0;
        int kapn = 0, nu;
        if (qrho > 1.0) {
            qrho = sqrt(qrho);
            nu = 3 + (int)floor(1442.0 / (26.0 * qrho + 77.0));
        } else {
            qrho = (1.0 - y) * sqrt(1.0 - qrho);
            h = 1.88 * qrho;
            h2 = 2.0 * h;
            kapn = (int)rint(7.0 + 34.0 * qrho);
            nu = (int)rint(16.0 + 26.0 * qrho);
        }
        double qlambda = h > 0.0 ? pow(h2, (double)kapn) : 0.0;
        const double inv_h2 = h > 0.0 ? 1.0 / h2 : 0.0;
        double rx = 0.0, ry = 0.0, sx = 0.0, sy = 0.0;
        for (int n = nu; n >= 0; n--) {
            const double np1 = n + 1.0;
            double tx = yabs + h + np1 * rx, ty = xabs - np1 * ry;
            const double c = 0.5 * rcp_pos(tx * tx + ty * ty);
            rx = c * tx;
            ry = c * ty;
            if (h > 0.0 && n <= kapn) {
                tx = qlambda + sx;
                sx = rx * tx - ry * sy;
                sy = ry * tx + rx * sy;
                qlambda *= inv_h2;
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
    if (yi < 0.0) {
        if (small) {
            u2 *= 2.0;
            v2 *= 2.0;
        } else {
            const double w1 = 2.0 * exp(-xquad);
            u2 = w1 * cos(yquad);
            v2 = -w1 * sin(yquad);
        }
        u = u2 - u;
        v = v2 - v;
        if (xi > 0.0) v = -v;
    } else if (xi < 0.0) {
        v = -v;
    }
    return {u, v};
}
// w(z) for Im z >= 0 with |x| >= 16 or y >= 16 (so |z| >= 16): the asymptotic
// series w(z) ~ i / (sqrt(pi) z) sum_{k < 10} (2k-1)!! / (2 z^2)^k, nested as
// 1 + u (1 + 3 u (1 + 5 u (...))), u = 1 / (2 z^2); its 10th term is below 2e-17
// of the first there.  Against mpmath's w over |z| in [16, 1.6e4] across the
// upper half plane: 4.5e-16 relative, Re w included wherever it exceeds 1e-30
// |w| (Weideman: 2.5e-14; tests/test_warm_host.py).  On the real axis Re w =
// exp(-x^2) is set exactly, as in the Weideman branch; just above the axis the
// series omits the exponentially small Stokes term (<= exp(1 - x^2) |w| ~ 1e-111
// |w| for y < 1 at |x| >= 16), which Weideman's absolute error does not resolve
// either.  It serves ~90 % of the C5 beam's evaluations (median |z| ~ 40) at
// about half the Weideman cost: C5 trace phase 162.1 -> 143.8 ms.
constexpr double kFadAsym = 16.0;
constexpr int kFadAsymK = 10;
constexpr double dfact_odd(int k) {  // (2k - 1)!!, (-1)!! = 1: exact below 2^53
    double f = 1.0;
    for (int j = 1; j <= k; j++) f *= (double)(2 * j - 1);
    return f;
}
TORJ_HD bool faddeeva_asym_ok(double x, double y) { return fabs(x) >= kFadAsym || y >= kFadAsym; }
// T = sum_{k < K} (2k - 1)!! u^k by Horner with the double factorials as
// constants (4 VALU per term; the nested 1 + (2j - 1) u (...) form took 6)
// (TORJ_ASYM_KNUTH, round 6: the real coefficients by Knuth's recurrence as in
// weid_poly, two fma per term; against 30-digit sums over |z| in [16, 1e4] across
// the upper half plane the same error as complex Horner, 1.6e-16 at most)
#ifndef TORJ_ASYM_KNUTH
#define TORJ_ASYM_KNUTH 1
#endif
template <int K>
TORJ_HD void asym_horner(double ur, double ui, double &tr, double &ti) {
#if TORJ_ASYM_KNUTH
    static_assert(K >= 3, "the recurrence needs three terms");
    const double r = 2.0 * ur, s = fma(ur, ur, ui * ui);
    double b2 = dfact_odd(K - 1);
    double b1 = fma(r, b2, dfact_odd(K - 2));
#pragma unroll
    for (int k = K - 3; k >= 1; k--) {  // b_k = (2k - 1)!! + r b_(k+1) - s b_(k+2)
        const double b = fma(r, b1, fma(-s, b2, dfact_odd(k)));
        b2 = b1;
        b1 = b;
    }
    tr = fma(ur, b1, fma(-s, b2, 1.0));  // T = 1 - s b_2 + u b_1
    ti = ui * b1;
#else
    tr = dfact_odd(K - 1), ti = 0.0;
#pragma unroll
    for (int k = K - 2; k >= 0; k--) {  // T = T u + (2k - 1)!!
        const double t = fma(tr, ur, fma(-ti, ui, dfact_odd(k)));
        ti = fma(tr, ui, ti * ur);
        tr = t;
    }
#endif
}
// The series' length (TORJ_FAD_ASYM_ADAPT): the fewest terms K whose first
// omitted term (2K - 1)!! / (2 |z|^2)^K is at most 2^-56 of the leading 1, for
// the smallest |z|^2 the wave evaluates (wave-uniform on the device, so the
// Horner chain does not diverge): |z|^2 >= 0.5 ((2K - 1)!! 2^56)^(1/K), i.e.
// 10 terms from |z|^2 = 256 (the branch's edge), 9 from 256.9, 8 from 393.2,
// 7 from 692.2, 6 from 1506.9, 5 from 4630.2 (each threshold rounded up)
#ifndef TORJ_FAD_ASYM_ADAPT
#define TORJ_FAD_ASYM_ADAPT 0
#endif
TORJ_HD int asym_terms(double r2) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ballot(r2 < 256.9) ? 10 : __ballot(r2 < 393.2) ? 9 : __ballot(r2 < 692.2) ? 8
         : __ballot(r2 < 1506.9) ? 7 : __ballot(r2 < 4630.2) ? 6 : 5;
#else
    return r2 < 256.9 ? 10 : r2 < 393.2 ? 9 : r2 < 692.2 ? 8 : r2 < 1506.9 ? 7 : r2 < 4630.2 ? 6 : 5;
#endif
}
TORJ_HD cplx faddeeva_asym(double x, double y) {
    constexpr double kInvSqrtPi = 0.56418958354775628695;
    const double r2 = fma(x, x, y * y);
    const double ir2 = rcp_nz(r2);
    const double a = x * ir2, b = -y * ir2;  // 1 / z
    const double ur = 0.5 * fma(a, a, -b * b), ui = a * b;  // u = (1 / z)^2 / 2
    double tr, ti;
#if TORJ_FAD_ASYM_ADAPT
    switch (asym_terms(r2)) {
        case 5: asym_horner<5>(ur, ui, tr, ti); break;
        case 6: asym_horner<6>(ur, ui, tr, ti); break;
        case 7: asym_horner<7>(ur, ui, tr, ti); break;
        case 8: asym_horner<8>(ur, ui, tr, ti); break;
        case 9: asym_horner<9>(ur, ui, tr, ti); break;
        default: asym_horner<kFadAsymK>(ur, ui, tr, ti); break;
    }
#else
    asym_horner<kFadAsymK>(ur, ui, tr, ti);
#endif
    const double pr = fma(a, tr, -b * ti), pim = fma(a, ti, b * tr);  // T / z
    cplx w;
    w.re = -kInvSqrtPi * pim;  // i T / (sqrt(pi) z)
    w.im = kInvSqrtPi * pr;
    if (y == 0.0) w.re = exp(-x * x);
    return w;
}

// w(z) for Im z >= 0 by Weideman's rational approximation (N = 36,
// tools/gen_faddeeva_coefs.py; 2.5e-14 relative to scipy's wofz): a fixed-cost
// complex Horner sum with no branches, where TOMS 680 picks a series or a
// continued fraction of data-dependent length per argument -- divergent across
// a wave.  On the real axis Re w = exp(-x^2) exactly (as TOMS 680 sets it:
// the absorption is that term).
// (|z| < 16; faddeeva_asym above).
#ifndef TORJ_WEID_KNUTH  // Weideman's polynomial by the real-coefficient recurrence (1, round 6) or complex Horner (0)
#define TORJ_WEID_KNUTH 1
#endif
// Weideman's polynomial p(Z) = sum_k kWeidA[k] Z^(N-1-k) at complex Z: its
// coefficients are real, so (Knuth, TAOCP 4.6.4) with r = 2 Re Z and s = |Z|^2
// the recurrence b_k = a_k + r b_(k+1) - s b_(k+2) in real arithmetic gives
// p(Z) = a_0 - s b_2 + Z b_1: two fma per term against complex Horner's four
// VALU, and the term's critical path is one fma (the inner fma takes b_(k+2)).
// Over 20 000 arguments |z| < 16, Im z in [1e-6, 16), against scipy's wofz:
// the same error as complex Horner to the digit (median 4.3e-15, max 2.4e-14:
// Weideman's own truncation).
TORJ_HD void weid_poly(double Zr, double Zi, double &pr, double &pim) {
    const double r = 2.0 * Zr, s = fma(Zr, Zr, Zi * Zi);
    double b2 = kWeidA[0];
    double b1 = fma(r, b2, kWeidA[1]);
#pragma unroll
    for (int k = 2; k < kWeidN - 1; k++) {
        const double b = fma(r, b1, fma(-s, b2, kWeidA[k]));
        b2 = b1;
        b1 = b;
    }
    pr = fma(Zr, b1, fma(-s, b2, kWeidA[kWeidN - 1]));
    pim = Zi * b1;
}

TORJ_HD cplx faddeeva_upper(double x, double y) {
    constexpr double kInvSqrtPi = 0.56418958354775628695;
    if (faddeeva_asym_ok(x, y)) return faddeeva_asym(x, y);
    const double dr = kWeidL + y, di = -x;  // D = L - iz, Re D >= L > 0
    const double id = rcp_nz(fma(dr, dr, di * di));
    const double ir = dr * id, ii = -di * id;  // 1 / D
    const double nr = kWeidL - y, ni = x;      // L + iz
    const double Zr = fma(nr, ir, -ni * ii), Zi = fma(nr, ii, ni * ir);
#if TORJ_WEID_KNUTH
    double pr, pim;
    weid_poly(Zr, Zi, pr, pim);
#else
    double pr = kWeidA[0], pim = 0.0;
#pragma unroll
    for (int k = 1; k < kWeidN; k++) {
        const double t = fma(pr, Zr, fma(-pim, Zi, kWeidA[k]));
        pim = fma(pr, Zi, pim * Zr);
        pr = t;
    }
#endif
    const double i2r = fma(ir, ir, -ii * ii), i2i = 2.0 * ir * ii;  // 1 / D^2
    cplx w;
    w.re = fma(2.0, fma(pr, i2r, -pim * i2i), kInvSqrtPi * ir);
    w.im = fma(2.0, fma(pr, i2i, pim * i2r), kInvSqrtPi * ii);
    if (y == 0.0) w.re = exp(-x * x);
    return w;
}

// two arguments at once, their Horner chains interleaved (each the same
// operation sequence as faddeeva_upper, so the same bits): the warm kernels
// run one wave per SIMD, where a single dependent fp64 chain leaves every
// other issue slot empty
TORJ_HD void faddeeva_upper2(double x0, double y0, double x1, double y1, cplx &w0, cplx &w1) {
    constexpr double kInvSqrtPi = 0.56418958354775628695;
    const bool a0 = faddeeva_asym_ok(x0, y0), a1 = faddeeva_asym_ok(x1, y1);
#if defined(TORJ_WARM_PROF) && defined(__HIP_DEVICE_COMPILE__)
    {  // profiling build: pair calls per wave -- all lanes asymptotic / some lane Weideman,
       // and lanes with a Weideman argument; plus |z|^2 of those in bins [<36, <64, <100, <144, <256]
        const unsigned long long am = __ballot(1), wm = __ballot(!(a0 && a1));
        if ((int)__lane_id() == __builtin_ffsll((long long)am) - 1) {
            atomicAdd(&g_wfad[0], 1ull);
            atomicAdd(&g_wfad[1], wm ? 1ull : 0ull);
            atomicAdd(&g_wfad[2], (unsigned long long)__popcll(am));
            atomicAdd(&g_wfad[3], (unsigned long long)__popcll(wm));
        }
        const double zz[2] = {x0 * x0 + y0 * y0, x1 * x1 + y1 * y1};
        const bool aa[2] = {a0, a1};
        for (int q = 0; q < 2; q++)
            if (!aa[q]) {
                const int b = zz[q] < 36 ? 0 : zz[q] < 64 ? 1 : zz[q] < 100 ? 2 : zz[q] < 144 ? 3 : 4;
                atomicAdd(&g_wfad[4 + b], 1ull);
            }
    }
#endif
    if (a0 || a1) {  // the same branches as faddeeva_upper, so the same bits
        w0 = a0 ? faddeeva_asym(x0, y0) : faddeeva_upper(x0, y0);
        w1 = a1 ? faddeeva_asym(x1, y1) : faddeeva_upper(x1, y1);
        return;
    }
    const double xs[2] = {x0, x1}, ys[2] = {y0, y1};
    double ir[2], ii[2], Zr[2], Zi[2], pr[2], pim[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const double dr = kWeidL + ys[q], di = -xs[q];
        const double id = rcp_nz(fma(dr, dr, di * di));
        ir[q] = dr * id;
        ii[q] = -di * id;
        const double nr = kWeidL - ys[q], ni = xs[q];
        Zr[q] = fma(nr, ir[q], -ni * ii[q]);
        Zi[q] = fma(nr, ii[q], ni * ir[q]);
        pr[q] = kWeidA[0];
        pim[q] = 0.0;
    }
#if TORJ_WEID_KNUTH
    {  // weid_poly of both arguments, interleaved (the same operations, so the same bits)
        double r[2], s[2], b1[2], b2[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            r[q] = 2.0 * Zr[q];
            s[q] = fma(Zr[q], Zr[q], Zi[q] * Zi[q]);
            b2[q] = kWeidA[0];
            b1[q] = fma(r[q], b2[q], kWeidA[1]);
        }
#pragma unroll
        for (int k = 2; k < kWeidN - 1; k++) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const double b = fma(r[q], b1[q], fma(-s[q], b2[q], kWeidA[k]));
                b2[q] = b1[q];
                b1[q] = b;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
            pr[q] = fma(Zr[q], b1[q], fma(-s[q], b2[q], kWeidA[kWeidN - 1]));
            pim[q] = Zi[q] * b1[q];
        }
    }
#else
#pragma unroll
    for (int k = 1; k < kWeidN; k++) {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const double t = fma(pr[q], Zr[q], fma(-pim[q], Zi[q], kWeidA[k]));
            pim[q] = fma(pr[q], Zi[q], pim[q] * Zr[q]);
            pr[q] = t;
        }
    }
#endif
    cplx w[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const double i2r = fma(ir[q], ir[q], -ii[q] * ii[q]), i2i = 2.0 * ir[q] * ii[q];
        w[q].re = fma(2.0, fma(pr[q], i2r, -pim[q] * i2i), kInvSqrtPi * ir[q]);
        w[q].im = fma(2.0, fma(pr[q], i2i, pim[q] * i2r), kInvSqrtPi * ii[q]);
        if (ys[q] == 0.0) w[q].re = exp(-xs[q] * xs[q]);
    }
    w0 = w[0];
    w1 = w[1];
}

// Z(z) = i sqrt(pi) w(z) (zetac, :345-465); the warm tensor's arguments all
// have Im z >= 0 (zetac_upper); TOMS 680 serves Im z < 0
TORJ_HD cplx zetac_upper(double x, double y) {
    const cplx w = faddeeva_upper(x, y);
    return {-kSqrtPi * w.im, kSqrtPi * w.re};
}
TORJ_HD void zetac_upper2(double x0, double y0, double x1, double y1, cplx &z0, cplx &z1) {
    cplx w0, w1;
    faddeeva_upper2(x0, y0, x1, y1, w0, w1);
    z0 = {-kSqrtPi * w0.im, kSqrtPi * w0.re};
    z1 = {-kSqrtPi * w1.im, kSqrtPi * w1.re};
}
TORJ_HD cplx zetac(double x, double y) {
    if (y >= 0.0) return zetac_upper(x, y);
    const cplx w = faddeeva(x, y);
    return {-kSqrtPi * w.im, kSqrtPi * w.re};
}

template <int L>
struct Tensor {  // epsl(3,3,lrm) upper triangle (11 12 22 13 23 33) + e330, lrm <= L
    cplx e[L][6];
    cplx e330;
};

// the l-sum of the tensor (shared by both models): fl, ca -> epsl(:,:,l)
template <int L>
TORJ_HD void tensor_store(Tensor<L> &T, int l, double xg, double fl, const cplx ca[6]) {
    T.e[l - 1][0] = -xg * ca[0] * fl;
    T.e[l - 1][1] = I_times(xg * ca[1] * fl);
    T.e[l - 1][2] = -xg * ca[2] * fl;
    T.e[l - 1][3] = -xg * ca[3] * fl;
    T.e[l - 1][4] = -I_times(xg * ca[4] * fl);
    T.e[l - 1][5] = -xg * ca[5] * fl;
}

// Shkarofsky coefficients of one |s| (fsup, :473-561): p[ir] = cefp(isa, ir),
// m[ir] = cefm(isa, ir), ir = 0..2, summed over is = -isa then +isa in the
// reference's order.  Only the last three steps of the l-recurrence are
// stored, so p / m are indexed statically and stay in registers.  The two
// sides' Faddeeva evaluations run as interleaved pairs (zetac_upper2).
// fsup's per-call invariants (the same for every |s|)
struct WrInv {
    double anpl2hm1, psi, ipsi2, i2psi;
    bool big_psi;
};
TORJ_HD WrInv wr_inv(double anpl, double amu) {
    WrInv v;
    v.anpl2hm1 = anpl * anpl / 2.0 - 1.0;
    v.psi = sqrt_nn(0.5 * amu) * anpl;
    v.big_psi = fabs(v.psi) > 0.7;
    v.ipsi2 = v.big_psi ? 1.0 / (v.psi * v.psi) : 0.0;
    v.i2psi = v.big_psi ? 0.5 / v.psi : 0.0;
    return v;
}
TORJ_HD int fsup_s(double yg, double amu, const WrInv &iv, int isa, cplx p[3], cplx m[3]) {
    TORJ_WPROF(3);  // (the previous |s|'s accumulation into ca)
    const double anpl2hm1 = iv.anpl2hm1, psi = iv.psi;
    const bool big_psi = iv.big_psi;
    const double ipsi2 = iv.ipsi2, i2psi = iv.i2psi;
    for (int ir = 0; ir < 3; ir++) p[ir] = m[ir] = C(0.0);
    // side q = 0: is = -isa, q = 1: is = +isa (isa = 0: side 1 only; side 0
    // then repeats it as the partner of the pairs, and is not used)
    double alpha[2], phi2[2], phim[2], zx[2][3], zy[2][3];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int is = q == 0 ? -isa : isa;
        alpha[q] = anpl2hm1 + is * yg;
        phi2[q] = amu * alpha[q];
        phim[q] = sqrt_nn(fabs(phi2[q]));
        if (alpha[q] >= 0) {
            zx[q][0] = psi - phim[q], zy[q][0] = 0.0, zx[q][1] = -psi - phim[q], zy[q][1] = 0.0;
            zx[q][2] = -phim[q], zy[q][2] = 0.0;
        } else {
            zx[q][0] = psi, zy[q][0] = phim[q], zx[q][1] = -psi, zy[q][1] = phim[q];
            zx[q][2] = 0.0, zy[q][2] = phim[q];
        }
    }
    // Below the resonance (alpha < 0) z_m = -conj(z_p), and the algorithm's
    // w(-conj z) is conj(w(z)) bit for bit (it evaluates |x| and flips Im w),
    // so Z(z_m) = -conj(Z(z_p)) and one evaluation serves both.
    const bool mirror[2] = {alpha[0] < 0, alpha[1] < 0};
    cplx cz[2][3];
    if (isa == 0) {  // one side (s = 0; isa is the caller's loop counter: wave-uniform)
        cz[1][0] = zetac_upper(zx[1][0], zy[1][0]);
        if (!big_psi) cz[1][2] = zetac_upper(zx[1][2], zy[1][2]);
        cz[1][1] = mirror[1] ? C(-cz[1][0].re, cz[1][0].im) : zetac_upper(zx[1][1], zy[1][1]);
        cz[0][0] = cz[1][0], cz[0][1] = cz[1][1], cz[0][2] = cz[1][2];  // (side 0 unused)
    } else {
        zetac_upper2(zx[0][0], zy[0][0], zx[1][0], zy[1][0], cz[0][0], cz[1][0]);
        if (!big_psi) zetac_upper2(zx[0][2], zy[0][2], zx[1][2], zy[1][2], cz[0][2], cz[1][2]);
        if (!mirror[0] && !mirror[1]) {
            zetac_upper2(zx[0][1], zy[0][1], zx[1][1], zy[1][1], cz[0][1], cz[1][1]);
        } else {
#pragma unroll
            for (int q = 0; q < 2; q++)
                cz[q][1] = mirror[q] ? C(-cz[q][0].re, cz[q][0].im) : zetac_upper(zx[q][1], zy[q][1]);
        }
    }
    TORJ_WPROF(1);  // the Faddeeva evaluations
    // Faddeeva evaluations of the reference's algorithm and those of them the
    // asymptotic series serves (the work counters, torj_hip/flops.py), packed
    // as nfad | nasym << 16
    int nfad = 0;
#pragma unroll
    for (int q = 0; q < 2; q++) {
        if (q == 0 && isa == 0) continue;
        const int is = q == 0 ? -isa : isa;
        nfad += (big_psi ? 2 : 3) - (mirror[q] ? 1 : 0);
        nfad += (faddeeva_asym_ok(zx[q][0], zy[q][0]) + (!mirror[q] && faddeeva_asym_ok(zx[q][1], zy[q][1])) +
                 (!big_psi && faddeeva_asym_ok(zx[q][2], zy[q][2])))
                << 16;
        const cplx czp = cz[q][0], czm = cz[q][1], cz0 = cz[q][2];
        cplx cf12 = C(0.0);
        if (alpha[q] != 0.0) {
            const double i2phim = 0.5 * rcp_pos(phim[q]);
            cf12 = alpha[q] > 0 ? -((czp + czm) * i2phim) : -I_times((czp + czm) * i2phim);
        }
        cplx cf32;
        if (big_psi) {
            cf32 = -((czp - czm) * i2psi);
        } else {
            const cplx cphi = alpha[q] < 0 ? C(0.0, -phim[q]) : C(phim[q]);
            cf32 = 2.0 * (1.0 - cphi * cz0);
        }
        cplx cf0 = cf12, cf1 = cf32;
        const double ph2 = phi2[q];
        auto step = [&](int l) {
            const cplx cf2 = big_psi ? (1.0 + ph2 * cf0 - (l - 0.5) * cf1) * ipsi2
                                     : (1.0 + ph2 * cf1) * rcp_pos(l + 0.5);
            cf0 = cf1;
            cf1 = cf2;
            return cf2;
        };
        if (is == 0) p[0] = m[0] = cf32;
        for (int l = 1; l < isa; l++) step(l);  // l < isa: not stored
#pragma unroll
        for (int ir = 0; ir < 3; ir++) {
            if (isa + ir < 1) continue;  // s = 0: ir = 0 is cf32 itself
            const cplx cf2 = step(isa + ir);
            p[ir] = p[ir] + cf2;
            m[ir] = is > 0 ? m[ir] + cf2 : m[ir] - cf2;
        }
    }
    TORJ_WPROF(2);  // the l-recurrences
    return nfad;
}

// weakly relativistic tensor (fsup + dieltens_maxw_wr, :473-638).  The |s|
// loop runs outermost and adds its terms to every l >= |s|, in the
// reference's summation order; ca[l][.] is indexed statically (registers).
// The (|s|, l) coefficients of dieltens_maxw_wr's tensor sums (:598-627), a
// compile-time table [|s|][l - 1][.]: is^2 a_sl, is l a_sl, b_sl, is a_sl,
// l a_sl, a_sl with a_sl = (-1)^(l-|s|) / ((l+|s|)! (l-|s|)!) and
// b_sl = a_sl (is^2 + 2 (l-|s|)(l-1)(l+|s|) / (2l-1)) -- each the value the
// per-term expressions give (the same operations, rounded once at compile time)
constexpr double cfact(int k) {
    double f = 1.0;
    for (int i = 2; i <= k; i++) f *= (double)i;
    return f;
}
struct WrCoef {
    double c[kWarmMaxL + 1][kWarmMaxL][6];
    double fl[kWarmMaxL + 1];  // 0.5^l (2l)! / l! = (2l - 1)!!, exact
};
constexpr WrCoef make_wr_coef() {
    WrCoef w{};
    for (int isa = 0; isa <= kWarmMaxL; isa++)
        for (int l = 1; l <= kWarmMaxL; l++) {
            if (l < isa) continue;
            const int lm = l - 1, k = l - isa;
            const double is = isa;
            const double asl = ((k & 1) ? -1.0 : 1.0) / (cfact(isa + l) * cfact(l - isa));
            const double bsl = asl * (is * is + (double)(2 * k * lm * (l + isa)) / (2 * l - 1));
            double *c = w.c[isa][lm];
            c[0] = (is * is) * asl;
            c[1] = (is * l) * asl;
            c[2] = bsl;
            c[3] = is * asl;
            c[4] = (double)l * asl;
            c[5] = asl;
        }
    for (int l = 1; l <= kWarmMaxL; l++) {
        double f = 1.0;
        for (int j = 1; j <= l; j++) f *= (double)(2 * j - 1);
        w.fl[l] = f;
    }
    return w;
}
#ifdef __HIP_DEVICE_COMPILE__
__constant__ constexpr WrCoef kWrCoef = make_wr_coef();
#else
constexpr WrCoef kWrCoef = make_wr_coef();
#endif

template <int L>
TORJ_HD int dieltens_wr(double xg, double yg, double anpl, double amu, int lrm, Tensor<L> &T) {
    const double anpl2 = anpl * anpl;
    const double iyg = 1.0 / yg, iyg2 = 1.0 / (yg * yg);  // operator/ (cplx, double)'s reciprocals
    const WrInv iv = wr_inv(anpl, amu);
    cplx ca[L][6];
#pragma unroll
    for (int l = 0; l < L; l++)
        for (int q = 0; q < 6; q++) ca[l][q] = C(0.0);
    cplx p0[3];
    int nfad = 0;
    for (int isa = 0; isa <= lrm; isa++) {
        cplx p[3], m[3];
        nfad += fsup_s(yg, amu, iv, isa, p, m);
        if (isa == 0) p0[0] = p[0], p0[1] = p[1], p0[2] = p[2];
        const cplx cq0p = amu * p[0], cq0m = amu * m[0];
        const cplx cq1p = amu * anpl * (p[0] - p[1]);
        const cplx cq1m = amu * anpl * (m[0] - m[1]);
        const cplx cq2p = p[1] + amu * anpl2 * (p[2] + p[0] - 2.0 * p[1]);
#pragma unroll
        for (int l = 1; l <= L; l++) {
            if (l > lrm || l < isa) continue;
            const int lm = l - 1;
            const double *c = kWrCoef.c[isa][lm];
            ca[lm][0] = ca[lm][0] + c[0] * cq0p;
            ca[lm][1] = ca[lm][1] + c[1] * cq0m;
            ca[lm][2] = ca[lm][2] + c[2] * cq0p;
            ca[lm][3] = ca[lm][3] + (c[3] * cq1m) * iyg;
            ca[lm][4] = ca[lm][4] + (c[4] * cq1p) * iyg;
            ca[lm][5] = ca[lm][5] + (c[5] * cq2p) * iyg2;
        }
    }
    TORJ_WPROF(3);
    // f_l = 0.5^l (1 / yg^2 / amu)^(l-1) (2l)! / l!: the power by products
    const double u = iyg * iyg / amu;
    double upow = 1.0;
#pragma unroll
    for (int l = 1; l <= L; l++) {
        if (l > lrm) break;
        if (l > 1) upow *= u;
        tensor_store(T, l, xg, kWrCoef.fl[l] * upow, ca[l - 1]);
    }
    const cplx cq2p = p0[1] + amu * anpl2 * (p0[2] + p0[0] - 2.0 * p0[1]);
    T.e330 = 1.0 - xg * amu * cq2p;
    TORJ_WPROF(4);  // the l-factors and the tensor's store
    return nfad;
}

// fully relativistic tensor (hermitian iwarm > 2 + antihermitian +
// dieltens_maxw_fr, :646-1134)
template <int L>
TORJ_HD void dieltens_fr(double xg, double yg, double anpl, double amu, int lrm, Tensor<L> &T) {
    const int llm = lrm < 3 ? lrm : 3;
    // rr[n + 3][k][m], n in [-llm, llm], m in [|n|, llm]
    double rr[7][3][4];
    for (int a = 0; a < 7; a++)
        for (int b = 0; b < 3; b++)
            for (int c = 0; c < 4; c++) rr[a][b][c] = 0.0;
    const double cmxw = 1.0 + 15.0 / (8.0 * amu) + 105.0 / (128.0 * amu * amu);
    const double cr = -amu * amu / (kSqrtPi * cmxw);
    const double bth2 = 2.0 / amu, bth = sqrt(bth2);
    const double amu2 = amu * amu, amu4 = amu2 * amu2, amu6 = amu4 * amu2;
    const double iamu = 1.0 / amu, i2amu = 0.5 * iamu;
    // node-outer: the t-only quantities of node i once for every n (the
    // reference's n-outer loop recomputes them per n); acc[n + 3][m][k] sums
    // over i in the same order, statically indexed so it stays in registers
    double acc[7][4][3];
#pragma unroll
    for (int a = 0; a < 7; a++)
#pragma unroll
        for (int m = 0; m < 4; m++) acc[a][m][0] = acc[a][m][1] = acc[a][m][2] = 0.0;
    for (int i = 0; i < kNtv; i++) {
        const double t = -kTmax + i * kDtv, t2 = t * t;
        const double rxt = sqrt_pos(fma(t2, i2amu, 1.0)), x = t * rxt;
        const double upl2 = bth2 * x * x, upl = bth * x, gx = fma(t2, iamu, 1.0);
        const double exdx = cr * kFrW.w[i] * gx * rcp_nz(rxt);
#pragma unroll
        for (int n = -3; n <= 3; n++) {
            const int mlo = n < 0 ? -n : n;
            if (mlo > llm) continue;
            const double gr = anpl * upl + n * yg;
            const double zm = -amu * (gx - gr), s = amu * (gx + gr);
            const double fe0m = expei(zm), zm2 = zm * zm;
#pragma unroll
            for (int m = mlo; m <= 3; m++) {
                if (m > llm) break;
                if (m == 0) {
                    acc[n + 3][0][2] += -exdx * fe0m * upl2;
                    continue;
                }
                double ffe;
                if (m == 1)
                    ffe = (1.0 + s * (1.0 - zm * fe0m)) / amu2;
                else if (m == 2)
                    ffe = (6.0 - 2.0 * zm + 4.0 * s + s * s * (1.0 + zm - zm2 * fe0m)) / amu4;
                else
                    ffe = (18.0 * s * (s + 4.0 - zm) + 6.0 * (20.0 - 8.0 * zm + zm2) +
                           s * s * s * (2.0 + zm + zm2 - zm2 * zm * fe0m)) / amu6;
                acc[n + 3][m][0] += exdx * ffe;
                acc[n + 3][m][1] += exdx * ffe * upl;
                acc[n + 3][m][2] += exdx * ffe * upl2;
            }
        }
    }
#pragma unroll
    for (int n = -3; n <= 3; n++) {
        const int mlo = n < 0 ? -n : n;
#pragma unroll
        for (int m = mlo; m <= 3; m++)
            if (m <= llm)
#pragma unroll
                for (int k = 0; k < 3; k++) rr[n + 3][k][m] = acc[n + 3][m][k];
    }
    // anti-hermitian part ri[n-1][k][m-1], m >= n
    double ri[kWarmMaxL][3][kWarmMaxL];
    for (int a = 0; a < kWarmMaxL; a++)
        for (int b = 0; b < 3; b++)
            for (int c = 0; c < kWarmMaxL; c++) ri[a][b][c] = 0.0;
    const double dnl = 1.0 - anpl * anpl, cmu = anpl * amu;
    const double ci = sqrt(2.0 * kPi * amu) * amu * amu / cmxw;
    for (int n = 1; n <= lrm; n++) {
        const double ygn = n * yg, rdu2 = ygn * ygn - dnl;
        if (!(rdu2 > 0.0)) continue;
        const double du = sqrt(rdu2) / dnl, ub = anpl * ygn / dnl, aa = amu * anpl * du;
        if (fabs(aa) > 5.0) {
            const double up = ub + du, um = ub - du;
            const double gp = anpl * up + ygn, gm = anpl * um + ygn;
            const double xp = up + 1.0 / cmu, xm = um + 1.0 / cmu;
            const double eem = exp(-amu * (gm - 1.0)), eep = exp(-amu * (gp - 1.0));
            double f0p = -1.0 / cmu, f1p = -xp / cmu, f2p = -(1.0 / (cmu * cmu) + xp * xp) / cmu;
            double f0m = -1.0 / cmu, f1m = -xm / cmu, f2m = -(1.0 / (cmu * cmu) + xm * xm) / cmu;
            for (int m = 1; m <= lrm; m++) {
                const double g0p = -2.0 * m * (f1p - ub * f0p) / cmu;
                const double g0m = -2.0 * m * (f1m - ub * f0m) / cmu;
                const double g1p = -((1.0 + 2 * m) * f2p - 2.0 * (m + 1) * ub * f1p + up * um * f0p) / cmu;
                const double g1m = -((1.0 + 2 * m) * f2m - 2.0 * (m + 1) * ub * f1m + up * um * f0m) / cmu;
                const double g2p = (2.0 * (1 + m) * g1p - 2.0 * m * (ub * f2p - up * um * f1p)) / cmu;
                const double g2m = (2.0 * (1 + m) * g1m - 2.0 * m * (ub * f2m - up * um * f1m)) / cmu;
                if (m >= n) {
                    const double h = 0.5 * ci * pow(dnl, m);
                    ri[n - 1][0][m - 1] = h * (g0p * eep - g0m * eem);
                    ri[n - 1][1][m - 1] = h * (g1p * eep - g1m * eem);
                    ri[n - 1][2][m - 1] = h * (g2p * eep - g2m * eem);
                }
                f0p = g0p, f1p = g1p, f2p = g2p, f0m = g0m, f1m = g1m, f2m = g2m;
            }
        } else {
            const double ee = exp(-amu * (ygn - 1.0 + anpl * ub));
            double fsbi[kWarmMaxL + 3];
            ssbi(aa, n, lrm, fsbi);
            for (int m = n; m <= lrm; m++) {
                const double cm = kSqrtPi * factd(m) * pow(du, 2 * m + 1);
                const double cim = 0.5 * ci * pow(dnl, m);
                const int mm = m - n;
                const double fi0 = cm * fsbi[mm], fi1 = -0.5 * aa * cm * fsbi[mm + 1];
                const double fi2 = 0.5 * cm * (fsbi[mm + 1] + 0.5 * aa * aa * fsbi[mm + 2]);
                ri[n - 1][0][m - 1] = cim * ee * fi0;
                ri[n - 1][1][m - 1] = cim * ee * (du * fi1 + ub * fi0);
                ri[n - 1][2][m - 1] = cim * ee * (du * du * fi2 + 2.0 * du * ub * fi1 + ub * ub * fi0);
            }
        }
    }
    // rr is only populated for |n| <= llm <= 3 and m <= llm (the reference's
    // rr(n,k,m) with m > llm stays 0): read through a guard
    auto RR = [&](int n, int k, int m) -> double {
        return (n >= -3 && n <= 3 && m <= 3) ? rr[n + 3][k][m] : 0.0;
    };
#pragma unroll
    for (int l = 1; l <= L; l++) {  // static l, is: the tensor stays in registers
        if (l > lrm) break;
        const int lm = l - 1;
        const double fal = -pow(0.25, l) * factd(2 * l) / (factd(l) * factd(l) * pow(yg, 2 * lm));
        cplx ca[6] = {C(0), C(0), C(0), C(0), C(0), C(0)};
#pragma unroll
        for (int is = 0; is <= l; is++) {
            const int k = l - is;
            const double asl = ((k & 1) ? -1.0 : 1.0) / (factd(is + l) * factd(l - is));
            const double bsl = asl * (is * is + (double)(2 * k * lm * (l + is)) / (2 * l - 1));
            cplx cq0p, cq0m, cq1p, cq1m, cq2p;
            if (is > 0) {
                cq0p = C(RR(is, 0, l) + RR(-is, 0, l), ri[is - 1][0][l - 1]);
                cq0m = C(RR(is, 0, l) - RR(-is, 0, l), ri[is - 1][0][l - 1]);
                cq1p = C(RR(is, 1, l) + RR(-is, 1, l), ri[is - 1][1][l - 1]);
                cq1m = C(RR(is, 1, l) - RR(-is, 1, l), ri[is - 1][1][l - 1]);
                cq2p = C(RR(is, 2, l) + RR(-is, 2, l), ri[is - 1][2][l - 1]);
            } else {
                cq0p = cq0m = C(RR(0, 0, l));
                cq1p = cq1m = C(RR(0, 1, l));
                cq2p = C(RR(0, 2, l));
            }
            ca[0] = ca[0] + (double)(is * is) * asl * cq0p;
            ca[1] = ca[1] + (double)(is * l) * asl * cq0m;
            ca[2] = ca[2] + bsl * cq0p;
            ca[3] = ca[3] + (double)is * asl * cq1m / yg;
            ca[4] = ca[4] + (double)l * asl * cq1p / yg;
            ca[5] = ca[5] + asl * cq2p / (yg * yg);
        }
        tensor_store(T, l, xg, fal, ca);
    }
    T.e330 = C(1.0 + xg * rr[3][2][0]);
}

#ifndef TORJ_WARM_RR_COMP
#define TORJ_WARM_RR_COMP 0
#endif
// a0 b0 + a1 b1 + a2 b2 + a3 b3 as if in twice the working precision (Ogita,
// Rump & Oishi's Dot2: error-free products by fma, error-free sums)
TORJ_HD double dot2_4(const double (&a)[4], const double (&b)[4]) {
    double p = a[0] * b[0], s = fma(a[0], b[0], -p);
#pragma unroll
    for (int k = 1; k < 4; k++) {
        const double h = a[k] * b[k], r = fma(a[k], b[k], -h);
        const double t = p + h, z = t - p, q = (p - (t - z)) + (h - z);
        p = t;
        s += q + r;
    }
    return p + s;
}

// warmdisp (:1158-1267) -> N_perp^2 (complex); anpr2 initialised (R2)
template <int L>
TORJ_HD cplx warmdisp_n2(double xg, double yg, double anpl, double anprc, int sox, int lrm,
                          const Tensor<L> &T, int &passes) {
    cplx anpr2a = C(anprc * anprc), anpr2 = anpr2a;
    const double anpl2 = anpl * anpl;
    double errnpr = 1.0, na = cnorm_(anpr2a);  // |anpr2a|^2
    passes = 0;  // passes of the reference's loop, the breaking one included (the work counters)
    for (int i = 1; i <= 100; i++) {
        passes = i;
        // the reference sums the tensor before this test, for the polarisation
        // of its breaking pass (:1172-1196); alpha needs N_perp^2 only
        if (i > 2 && errnpr < 1.0e-4) break;
        cplx s[6] = {C(0), C(0), C(0), C(0), C(0), C(0)};
        cplx pw = C(1.0);
#pragma unroll
        for (int l = 0; l < L; l++) {  // static l: the tensor stays in registers
            if (l >= lrm) break;
            for (int q = 0; q < 6; q++) s[q] = s[q] + T.e[l][q] * pw;
            pw = pw * anpr2a;
        }
        // diagonal identity terms for l = 1 are already in T.e[0]
        const cplx e11 = s[0], e12 = s[1], e22 = s[2], a13 = s[3], a23 = s[4], a33 = s[5];
        const cplx a31 = a13, a32 = -a23;
        const cplx cc4 = (e11 - anpl2) * (1.0 - a33) + (a13 + anpl) * (a31 + anpl);
        const cplx cc2 = -e12 * e12 * (1.0 - a33) - a32 * e12 * (a13 + anpl) + a23 * e12 * (a31 + anpl) -
                         (a23 * a32 + T.e330 + (e22 - anpl2) * (1.0 - a33)) * (e11 - anpl2) -
                         (a13 + anpl) * (a31 + anpl) * (e22 - anpl2);
        const cplx cc0 = T.e330 * ((e11 - anpl2) * (e22 - anpl2) + e12 * e12);
#if TORJ_WARM_RR_COMP
        // R6 (an A/B, off by default): the discriminant in twice the working
        // precision (Dot2), so that its own cancellation cannot decide the root
        // selector below
        const double ar[4] = {cc2.re, cc2.im, cc0.re, cc0.im}, br[4] = {cc2.re, -cc2.im, -4.0 * cc4.re, 4.0 * cc4.im};
        const double ai[4] = {2.0 * cc2.re, cc0.re, cc0.im, 0.0}, bi[4] = {cc2.im, -4.0 * cc4.im, -4.0 * cc4.re, 0.0};
        const cplx rr = C(dot2_4(ar, br), dot2_4(ai, bi));
#else
        const cplx rr = cc2 * cc2 - 4.0 * cc0 * cc4;
#endif
        double sg;
        if (yg > 1.0) {
            sg = (double)sox;
            if (rr.im <= 0.0) sg = -sg;
        } else {
            sg = (double)(-sox);
            if (rr.re <= 0.0 && rr.im >= 0.0) sg = -sg;
        }
        // (-cc2 + sg sqrt(rr)) / (2 cc4) as a product with conj(cc4) / (2 |cc4|^2)
        const double ic = 0.5 * rcp_nz(cnorm_(cc4));
        anpr2 = (-cc2 + sg * csqrt_(rr)) * C(cc4.re * ic, -cc4.im * ic);
        // |1 - |anpr2| / |anpr2a||, the moduli from their squares
        const double n2 = cnorm_(anpr2);
        errnpr = fabs(1.0 - sqrt_nn(n2 * rcp_nz(na)));
        anpr2a = anpr2;
        na = n2;
    }
    if (anpr2.re < 0.0 && anpr2.im < 0.0) anpr2 = C(0.0);  // ierr = 99
    TORJ_WPROF(5);  // warmdisp
    return anpr2;
}

// larmornumber (:1285-1326); trips = resonance tests made (the work counters)
TORJ_HD int larmornumber(double yg, double npl, double mu, int &trips) {
    const double dnl = 1.0 - npl * npl;
    int imax = 1;
    int nharm = (int)floor(1.0 / yg);
    if (nharm * yg < 1.0) nharm++;
    trips = 0;
    for (;;) {
        trips++;
        const double ygn = nharm * yg, rdu2 = ygn * ygn - dnl;
        const double gg = (ygn - sqrt(npl * npl * rdu2)) / dnl;
        if (mu * (gg - 1.0) > 15.0) break;
        nharm++;
        imax++;
        if (imax > 100) {
            nharm = (int)floor(yg);
            break;
        }
    }
    return nharm;
}
TORJ_HD int larmornumber(double yg, double npl, double mu) {
    int trips;
    return larmornumber(yg, npl, mu, trips);
}

// alpha (:1328-1337): iwarm 1 (weakly relativistic) or 3 (fully relativistic,
// the reference's choice); inv_dDdN = 1 / |dD/dN| (R4); sox from mode (R5).
// Returns alpha [1/m] and N_perp^2 (warm) by value.
//
// No pointer into a caller's private (scratch) frame crosses a call here:
// with this ROCm 7.2 gfx950 toolchain, a non-inlined function that receives a
// flat pointer to its caller's stack frame, as alpha_warm_t's former
// `cplx *n2` out-argument and dieltens_fr(..., Tensor &T) behind a noinline
// call did, read its OWN local arrays back wrong (the fully relativistic
// tensor's anti-hermitian part came out 0 or ~1e-10 of its value) once the
// caller had a frame of its own -- the same callee was exact when the pointer
// went to global memory, or the caller had no frame (tests/native/
// warm_check.hip reproduces it: "tensor in the kernel frame" vs "tensor in
// global memory").  A printf changed the frame layout and hid
// it.  The warm kernels inline this code; the out-of-line build
// (TORJ_WARM_ATTR noinline) returns by value and is pinned by the same tests.
#ifndef TORJ_WARM_ATTR
#define TORJ_WARM_ATTR TORJ_HD
#endif
struct WarmAlpha {
    double alpha;
    cplx n2;
    // trip counts of the data-dependent loops (iwarm 1: Faddeeva evaluations;
    // both: warmdisp passes, Larmor order, larmornumber tests) -> torj_hip/flops.py
    int nfad, passes, lrm, ltrips;
    int nasym;  // of the nfad, those by the asymptotic series (faddeeva_asym)
};
template <int IWARM, int L>
TORJ_HD WarmAlpha alpha_core(double omega, double X, double Y, double N_par, double mu, double npr,
                             int lrm, double inv_dDdN, int mode) {
    Tensor<L> T;
    int nfad = 0, passes;
    if constexpr (IWARM == 1)
        nfad = dieltens_wr<L>(X, Y, N_par, mu, lrm, T);
    else
        dieltens_fr<L>(X, Y, N_par, mu, lrm, T);
    // identity on the l = 1 diagonal (:629-630 / :1125-1126)
    T.e[0][0] = T.e[0][0] + 1.0;
    T.e[0][2] = T.e[0][2] + 1.0;
    const int sox = Y <= 1.0 ? mode : -mode;
    const cplx a2 = warmdisp_n2<L>(X, Y, N_par, npr, sox, lrm, T, passes);
    return {2.0 * a2.im * omega / kC * inv_dDdN, a2, nfad & 0xffff, passes, lrm, 0, nfad >> 16};
}

// The tensor is sized for lrm <= 3 (the common case: one to three Larmor
// orders up to the third harmonic) or lrm <= 5; on the device the choice is
// made per wave (ballot), so the heavy code never diverges between the two.
// (The split pipeline's k_alpha_warm_pts instead defers its lrm > 3 points to
// k_alpha_warm_big, so that its own registers are sized for lrm <= 3.)
// The call's setup (alpha, :1328-1337, up to the tensor): mu, N_perp of the
// cold root and the Larmor order by larmornumber
struct WarmSetup {
    double mu, npr;
    int lrm, ltrips;
};
TORJ_HD WarmSetup warm_setup(double Y, double N_abs, double N_par, double Te) {
    WarmSetup w;
    w.mu = kMe * kC * kC / (Te * kE);
    w.npr = sqrt(fmax(N_abs * N_abs - N_par * N_par, 0.0));
    const int nharm = larmornumber(Y, N_par, w.mu, w.ltrips);
    w.lrm = nharm < kWarmMaxL ? nharm : kWarmMaxL;
    TORJ_WPROF(0);  // inputs, larmornumber
    return w;
}
// the rest of the call with the tensor sized for lrm <= L
template <int IWARM, int L>
TORJ_HD WarmAlpha alpha_warm_l(double omega, double X, double Y, double N_par, const WarmSetup &w,
                               double inv_dDdN, int mode) {
    WarmAlpha r = alpha_core<IWARM, L>(omega, X, Y, N_par, w.mu, w.npr, w.lrm, inv_dDdN, mode);
    r.ltrips = w.ltrips;
    return r;
}
template <int IWARM>
TORJ_WARM_ATTR WarmAlpha alpha_warm_v(double omega, double X, double Y, double N_abs, double N_par,
                                      double Te, double inv_dDdN, int mode) {
    const WarmSetup w = warm_setup(Y, N_abs, N_par, Te);
#if defined(__HIP_DEVICE_COMPILE__)
    const bool big = __ballot(w.lrm > 3) != 0;
#else
    const bool big = w.lrm > 3;
#endif
    return big ? alpha_warm_l<IWARM, kWarmMaxL>(omega, X, Y, N_par, w, inv_dDdN, mode)
               : alpha_warm_l<IWARM, 3>(omega, X, Y, N_par, w, inv_dDdN, mode);
}

template <int IWARM>
TORJ_HD double alpha_warm_t(double omega, double X, double Y, double N_abs, double N_par,
                            double Te, double inv_dDdN, int mode, cplx *n2) {
    const WarmAlpha r = alpha_warm_v<IWARM>(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode);
    if (n2) *n2 = r.n2;
    return r.alpha;
}

// runtime iwarm (1 or 3): the point entry torj_alpha_warm and the host tests
TORJ_HD double alpha_warm(double omega, double X, double Y, double N_abs, double N_par, double Te,
                          double inv_dDdN, int mode, int iwarm, cplx *n2) {
    return iwarm == 1 ? alpha_warm_t<1>(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode, n2)
                      : alpha_warm_t<3>(omega, X, Y, N_abs, N_par, Te, inv_dDdN, mode, n2);
}

// one RHS evaluation: ABS 0 cold, 1 Albajar (abs_Albajar_fast), 2 warm weakly
// relativistic (iwarm 1), 3 warm fully relativistic (iwarm 3); separate
// instances keep each model's registers and private frame out of the others
// TINY: the Albajar model's bounded tiny-alpha skip (GLTable::tiny_alpha) on
// (fixed-step RK4); the adaptive integrator evaluates every integral, so that
// its step control sees the exact alpha
template <int ABS, int LPR = 1, bool TINY = true>
TORJ_HD void ray_rhs_m(const double *__restrict__ coef, const Grid &g, const Consts &k,
                       const GLTable &gl, double omega, int mode, int model, const double x[3],
                       const double N[3], double du[6], double &alpha, AlbajarWork *work,
                       int sub = 0) {
    PlasmaPoint p;
    plasma_point<(ABS != 0)>(coef, g, k, x, p);
    double Npar, inv;
    dispersion_grad(p, N, mode, du, &Npar, &inv);
    if constexpr (ABS == 1) {
        const double Nabs = sqrt_pos(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
        alpha = abs_albajar_fast<LPR>(gl, omega, p.X, p.Y, Nabs, Npar, exp_fast(p.lnTe), mode, work, sub,
                                      TINY ? gl.tiny_alpha : 0.0);
    } else if constexpr (ABS >= 2) {
        const double Nabs = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
        const WarmAlpha r =
            alpha_warm_v<ABS == 2 ? 1 : 3>(omega, p.X, p.Y, Nabs, Npar, exp(p.lnTe), inv, mode);
        alpha = r.alpha;
        if (ABS == 2 && work) {  // the weakly relativistic op count's trips (flops.py)
            work->n_active += r.nasym;
            work->n_harm += r.nfad;
            work->n_terms += r.passes;
            work->n_zero += r.passes * r.lrm;
            work->n_l += r.lrm;
            work->n_l2 += r.lrm * r.lrm;
        }
    } else {
        alpha = 0.0;
    }
}

}  // namespace torj
