// Host build of the product's warm-absorption math (torj.jl_amd/csrc/
// torj_warm.hpp is __host__ __device__): lets the CPU suite check the special
// functions and alpha of the device code against scipy / oracle/warm_ref.py
// without a GPU.  Test harness only; the product calls these on the device.
#include "torj_warm.hpp"
#include "torj_fitdepo.hpp"

#include <cmath>
#include <cstdlib>
#include <mutex>
#include <vector>

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

// the product's complex square root (torj_warm.hpp csqrt_), n points
void wh_csqrt(int n, const double *re, const double *im, double *out_re, double *out_im) {
    for (int i = 0; i < n; i++) {
        const torj::cplx r = torj::csqrt_(torj::cplx{re[i], im[i]});
        out_re[i] = r.re;
        out_im[i] = r.im;
    }
}
int wh_larmornumber(double yg, double npl, double mu) { return torj::larmornumber(yg, npl, mu); }

// the product's Julia round(Int64, x) (launch ring point counts, src/launch.jl:81)
long wh_round_ties_even(double x) { return torj::round_ties_even(x); }

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
        const char *e = getenv("TORJ_NEGL_SKIP");  // as torj_abs_al_init
        g_wh_gl.negl_skip = e ? (atoi(e) != 0) : 1;
        for (int i = 0; i < torj::kMaxGL; i++) {  // ascending nodes, zero-padded (torj_abs_al_init)
            g_wh_gl.t[i] = i < ngl ? t[i] : 0.0;
            g_wh_gl.w[i] = i < ngl ? w[i] : 0.0;
            g_wh_gl.st[i] = i < ngl ? sqrt(1.0 - t[i] * t[i]) : 0.0;
            g_wh_gl.t2[i] = i < ngl ? t[i] * t[i] : 0.0;
            if (i < ngl) torj::gl_node_consts(g_wh_gl, i);
        }
    });
    for (int i = 0; i < n; i++)
        alpha[i] = torj::abs_albajar_fast(g_wh_gl, om[i], X[i], Y[i], Nabs[i], Npar[i], Te[i], mode, nullptr);
}

// the negligible-harmonic skip on (1) / off (0) for the following wh_albajar
// calls (after the first, which sets up the table), and the per-point work of
// the same evaluation: [0] harmonics evaluated, [1] exact zero, [2] skipped as
// negligible (AlbajarWork n_harm, n_zero, n_negl)
void wh_set_negl_skip(int on) { g_wh_gl.negl_skip = on; }
void wh_albajar_work(int n, const double *om, const double *X, const double *Y, const double *Nabs,
                     const double *Npar, const double *Te, int mode, unsigned *work3) {
    for (int i = 0; i < n; i++) {
        torj::AlbajarWork w{};
        (void)torj::abs_albajar_fast(g_wh_gl, om[i], X[i], Y[i], Nabs[i], Npar[i], Te[i], mode, &w);
        work3[3 * i] = w.n_harm, work3[3 * i + 1] = w.n_zero, work3[3 * i + 2] = w.n_negl;
        work3[3 * i + 1] |= w.n_early << 8;  // settled before the polarisation vector
    }
}

// power_deposition_profile of the product (torj_fitdepo.hpp fit_depo_ray, the
// body of k_fit_depo) on the host, one call per ray, with an open-shell cache
// of nc = 1, 2 or 4 entries (1 exercises the spill path).  Samples are the
// oracle's (psi_k, dP/ds_k) at the entry point and each RK4 step, (n_steps+1) x n;
// outputs: dPs (n_psi-1) x n shell powers before the break, kstar, P per ray.
void fd_profile(int n, int n_steps, int n_psi, double ds, const double *grid, const double *s0,
                const int *steps, const double *psiL, const double *smp_psi, const double *smp_dpds,
                int nc, double *dPs, int *kstar, double *Pray) {
    const size_t K = (size_t)n_steps + 2, N = (size_t)n, L = (size_t)n_psi, KN = torj::smp_elems(N, K);
    std::vector<double> E(KN), G1(KN), G2(KN), Fo(L * N, NAN), dp(L * N, 0.0);
    // the product's per-step layout (torj::smp_at: 64-ray blocks)
    std::vector<double> sp(KN), sd(KN);
    for (size_t j = 0; j <= (size_t)n_steps; j++)
        for (size_t i = 0; i < N; i++) {
            sp[torj::smp_at(j, (int)i, K)] = smp_psi[j * N + i];
            sd[torj::smp_at(j, (int)i, K)] = smp_dpds[j * N + i];
        }
    std::vector<int> cnt((L + 1) * N, 0);
    torj::FitArgs fa{};
    fa.n = n;
    fa.n_psi = n_psi;
    fa.ds = ds;
    fa.grid = grid;
    fa.s0 = s0;
    fa.steps = steps;
    fa.smp_psi = sp.data();
    fa.smp_dpds = sd.data();
    fa.smp_s = nullptr;
    fa.rows = K;
    fa.s_uniform = 1;
    fa.E = E.data(), fa.Gpsi = G1.data(), fa.GP = G2.data();
    fa.cnt = cnt.data();
    fa.Fopen = Fo.data();
    fa.dPs = dp.data();
    fa.kstar = kstar;
    fa.Pray = Pray;
    for (int i = 0; i < n; i++) {
        if (nc == 1)
            torj::fit_depo_ray<1>(fa, i, psiL[i]);
        else if (nc == 4)
            torj::fit_depo_ray<4>(fa, i, psiL[i]);
        else
            torj::fit_depo_ray<2>(fa, i, psiL[i]);
    }
    for (size_t k = 0; k + 1 < L; k++)
        for (size_t i = 0; i < N; i++) dPs[k * N + i] = dp[k * N + i];
}

// the streamed deposition of the split pipeline (k_depo_stream after each
// scan, k_depo_tail after the trace) on the host: the scan's steps S grow by
// `inc` per emulated block while the ray runs (S < steps[i]), then the tail
void fd_profile_stream(int n, int n_steps, int n_psi, double ds, const double *grid, const double *s0,
                       const int *steps, const double *psiL, const double *smp_psi,
                       const double *smp_dpds, int inc, double *dPs, int *kstar, double *Pray) {
    const size_t K = (size_t)n_steps + 2, N = (size_t)n, L = (size_t)n_psi, KN = torj::smp_elems(N, K);
    std::vector<double> E(KN), G1(KN), G2(KN), Fo(L * N, NAN), dp(L * N, 0.0);
    std::vector<double> sp(KN), sd(KN);
    for (size_t j = 0; j <= (size_t)n_steps; j++)
        for (size_t i = 0; i < N; i++) {
            sp[torj::smp_at(j, (int)i, K)] = smp_psi[j * N + i];
            sd[torj::smp_at(j, (int)i, K)] = smp_dpds[j * N + i];
        }
    std::vector<int> cnt((L + 1) * N, 0);
    std::vector<double> dsd(torj::kDsNd * N, 0.0);
    std::vector<int> dsv(torj::kDsNi * N, 0);
    for (size_t i = 0; i < N; i++) dsv[torj::kDsJ * N + i] = -1;
    torj::DepoStream dst{dsd.data(), dsv.data()};
    torj::FitArgs fa{};
    fa.n = n;
    fa.n_psi = n_psi;
    fa.ds = ds;
    fa.grid = grid;
    fa.s0 = s0;
    fa.steps = steps;
    fa.smp_psi = sp.data();
    fa.smp_dpds = sd.data();
    fa.smp_s = nullptr;
    fa.rows = K;
    fa.s_uniform = 1;
    fa.E = E.data(), fa.Gpsi = G1.data(), fa.GP = G2.data();
    fa.cnt = cnt.data();
    fa.Fopen = Fo.data();
    fa.dPs = dp.data();
    fa.kstar = kstar;
    fa.Pray = Pray;
    for (int i = 0; i < n; i++) {
        // as k_depo_stream: psi at the launch point only for the walk's start;
        // inc < 0: the split form (k_depo_elim then k_depo_walk, one window per block)
        const int step = inc < 0 ? -inc : inc;
        for (int S = step; S < steps[i]; S += step) {
            const double pl = dsv[torj::kDsJ * N + i] < 0 ? psiL[i] : 0.0;
            if (inc < 0) {
                torj::fit_depo_stream_elim(fa, dst, i, pl, S);
                torj::fit_depo_stream_walk(fa, dst, i, pl, S);
            } else {
                torj::fit_depo_stream(fa, dst, i, pl, S);
            }
        }
        torj::fit_depo_tail(fa, dst, i, psiL[i]);
    }
    for (size_t k = 0; k + 1 < L; k++)
        for (size_t i = 0; i < N; i++) dPs[k * N + i] = dp[k * N + i];
}

// the split trajectory kernel's field evaluations, host build: the node stencil
// (eval_fields on kNF doubles per node) and the per-cell power form
// (cell_power_table + eval_fields on a TileCell without a tile, i.e. the global
// fallback of k_traj_cell) at the same points; out: n x 14 per variant (six
// values, then dR, dZ of the four gradient fields Br, Bphi, Bz, ln ne)
void fe_eval(int nR, int nZ, double R1, double Rn, double Z1, double Zn, const double *coef, int n,
             const double *R, const double *Z, int cell, double *out) {
    torj::Grid g{};
    g.nR = nR, g.nZ = nZ, g.R1 = R1, g.Rn = Rn, g.Z1 = Z1, g.Zn = Zn;
    g.hR = (Rn - R1) / (nR - 1), g.hZ = (Zn - Z1) / (nZ - 1);
    g.invhR = 1.0 / g.hR, g.invhZ = 1.0 / g.hZ;
    std::vector<double> tab;
    if (cell) {
        tab.resize((size_t)(nR - 1) * (nZ - 1) * torj::kCellRec);
        torj::cell_power_table(coef, nR, nZ, g.hR, g.hZ, tab.data());
    }
    const torj::TileCell tc{tab.data(), nullptr, 0, 0, 0, 0};
    const int idx[6] = {torj::F_BR, torj::F_BPHI, torj::F_BZ, torj::F_LNNE, torj::F_LNTE, torj::F_PSI};
    for (int k = 0; k < n; k++) {
        torj::FieldPack<4, 2> f;
        if (cell)
            torj::eval_fields<4, 2, true>(tc, g, R[k], Z[k], idx, f);
        else
            torj::eval_fields<4, 2, true>(coef, g, R[k], Z[k], idx, f);
        double *o = out + (size_t)k * 14;
        for (int q = 0; q < 6; q++) o[q] = f.v[q];
        for (int q = 0; q < 4; q++) o[6 + 2 * q] = f.dR[q], o[7 + 2 * q] = f.dZ[q];
    }
}
#if defined(TORJ_ROOT_STATS) && !defined(__HIP_DEVICE_COMPILE__)
// statistics build only: cubic_root calls, Newton steps, histogram of steps per call
void fd_root_stats(unsigned long long *out) {
    out[0] = torj::g_root_calls, out[1] = torj::g_root_iters;
    for (int k = 0; k < 8; k++) out[2 + k] = torj::g_root_hist[k];
    torj::g_root_calls = torj::g_root_iters = 0;
    for (int k = 0; k < 8; k++) torj::g_root_hist[k] = 0;
}
#endif
}
