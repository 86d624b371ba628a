// Host build of the product's warm-absorption math (torj.jl_amd/csrc/
// torj_warm.hpp is __host__ __device__): lets the CPU suite check the special
// functions and alpha of the device code against scipy / oracle/warm_ref.py
// without a GPU.  Test harness only; the product calls these on the device.
#include "torj_warm.hpp"

#include <mutex>

extern "C" {
void wh_zetac(int n, const double *x, const double *y, double *out) {
    for (int i = 0; i < n; i++) {
        const torj::cplx z = torj::zetac(x[i], y[i]);
        out[2 * i] = z.re, out[2 * i + 1] = z.im;
    }
}

void wh_expei(int n, const double *x, double *out) {
    for (int i = 0; i < n; i++) out[i] = torj::expei(x[i]);
}

void wh_ssbi(double z, int n, int l, double *out) {
    double v[torj::kWarmMaxL + 3];
    torj::ssbi(z, n, l, v);
    for (int m = 0; m <= l + 2 - n; m++) out[m] = v[m];
}

int wh_larmornumber(double yg, double npl, double mu) { return torj::larmornumber(yg, npl, mu); }

void wh_alpha_warm(int n, const double *om, const double *X, const double *Y, const double *Nabs,
                   const double *Npar, const double *Te, const double *inv, int mode, int iwarm,
                   double *alpha, double *n2) {
    for (int i = 0; i < n; i++) {
        torj::cplx c;
        alpha[i] = torj::alpha_warm(om[i], X[i], Y[i], Nabs[i], Npar[i], Te[i], inv[i], mode, iwarm, &c);
        n2[2 * i] = c.re, n2[2 * i + 1] = c.im;
    }
}

// abs_Albajar_fast of the product (torj_math.hpp, host build: same arithmetic
// as the device except that the hardware reciprocal seed and the node-loop
// sqrt/exp are the exact host ones)
static torj::GLTable g_wh_gl;
static std::once_flag g_wh_gl_once;
void wh_albajar(int n, const double *om, const double *X, const double *Y, const double *Nabs,
                const double *Npar, const double *Te, int mode, const double *t, const double *w,
                int ngl, double *alpha) {
    std::call_once(g_wh_gl_once, [&] {
        g_wh_gl.n = ngl;
        for (int i = 0; i < torj::kMaxGL; i++) {  // ascending nodes, zero-padded (torj_abs_al_init)
            g_wh_gl.t[i] = i < ngl ? t[i] : 0.0;
            g_wh_gl.w[i] = i < ngl ? w[i] : 0.0;
            g_wh_gl.st[i] = i < ngl ? sqrt(1.0 - t[i] * t[i]) : 0.0;
            g_wh_gl.t2[i] = i < ngl ? t[i] * t[i] : 0.0;
        }
    });
    for (int i = 0; i < n; i++)
        alpha[i] = torj::abs_albajar_fast(g_wh_gl, om[i], X[i], Y[i], Nabs[i], Npar[i], Te[i], mode, nullptr);
}
}
