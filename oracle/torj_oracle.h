/*
 * torj_oracle.h -- CPU restatement of TorJ.jl's ray-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it,
 * and only as the checker or the timed CPU peer.  The product (libtorj_hip.so,
 * torj_hip) never links or calls it.
 *
 * Parity status (see DESIGN.md "Oracle"): the reference (Julia) cannot run in
 * this container and its golden data is a network artifact, so the oracle is
 * pinned only by the reference's data-free known-answer test
 * (test/tests/test_launch_weights.jl:42-50) and by identities/independent
 * libraries (scipy jv/leggauss/hermgauss/CubicSpline, complex-step checks).
 * Everything else is "parity unpinned" against an executed reference.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to the TorJ.jl repository root).
 */
#ifndef TORJ_ORACLE_H
#define TORJ_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Physical constants, src/constants.jl:13-26 */
#define OR_C      2.99792458e8
#define OR_E      1.602176634e-19
#define OR_ME     9.1093837015e-31
#define OR_EPS0   8.8541878128e-12

/* ray status codes (shared convention with include/torj_hip.h) */
#define OR_OK          0
#define OR_LEFT_PLASMA 1
#define OR_ABSORBED    2
#define OR_NAN         3
#define OR_REFLECTED   4
#define OR_ENTRY_FAIL  5
#define OR_MAX_STEPS   6

/* 2-D cubic B-spline with Line() extrapolation (Interpolations.jl
 * cubic_spline_interpolation((r_range,z_range), data; extrapolation_bc=Line()),
 * src/plasma.jl:36,39-41).  coef is (nR+2) x (nZ+2), R fastest. */
typedef struct {
    int nR, nZ;
    double R1, Z1, hR, hZ, Rn, Zn;
    double *coef;
} or_spl2d;

typedef struct {
    int n;
    double x1, h, xn;
    double *coef; /* n+2 */
} or_spl1d;

/* struct Plasma, src/plasma.jl:2-14 */
typedef struct {
    or_spl2d psi, lnne, lnTe, Br, Bz, Bphi;
    or_spl1d vol;
    double psi_prof_max;
} or_plasma;

/* ---- quadrature (FastGaussQuadrature restatement) ---- */
void or_gauss_legendre(int n, double *x, double *w);
void or_gauss_hermite(int n, double *x, double *w);

/* ---- splines ---- */
void or_bspl1d_prefilter(int n, const double *y, double *c);
void or_bspl2d_prefilter(int nR, int nZ, const double *y, double *c);
double or_spl1d_eval(const or_spl1d *s, double x);
double or_spl1d_deriv(const or_spl1d *s, double x);
double or_spl2d_eval(const or_spl2d *s, double R, double Z);
void or_spl2d_grad(const or_spl2d *s, double R, double Z, double *dR, double *dZ);
/* natural cubic spline through (x,y) evaluated at xq (IMAS.interp1d :cubic,
 * parity unpinned: the reference's third-party interpolant is restated as the
 * natural cubic spline) */
void or_natcubic(int n, const double *x, const double *y, int nq, const double *xq, double *yq);

/* ---- Plasma constructor, src/plasma.jl:30-58 ---- */
int or_plasma_create(or_plasma *p, int nR, int nZ, const double *R, const double *Z,
                     const double *psi_norm, int n_prof, const double *psi_prof,
                     const double *ne_prof, const double *Te_prof, const double *Br,
                     const double *Bz, const double *Bphi, int n_eq, const double *eq_psi,
                     const double *eq_vol);
void or_plasma_free(or_plasma *p);

/* ---- field evaluation, src/plasma.jl:61-89, src/dispersion.jl:7-15 ---- */
double or_evaluate(const or_spl2d *s, const double x[3]);
void or_B_spline(const or_plasma *p, const double x[3], double B[3]);
double or_n_e(const or_plasma *p, const double x[3]);
double or_T_e(const or_plasma *p, const double x[3]);
void or_eval_plasma(const or_plasma *p, const double x[3], const double N[3], double omega,
                    double *X, double *Y, double *Npar, double b[3]);

/* ---- dispersion, src/dispersion.jl:21-39 ---- */
double or_refractive_index_sq(double X, double Y, double Npar, int mode);
double or_dispersion_relation(const or_plasma *p, const double x[3], const double N[3],
                              double omega, int mode);
/* gradΛ!/sys! without the α part (src/solve.jl:85-93) via forward-mode duals */
void or_grad_lambda(const or_plasma *p, const double x[3], const double N[3], double omega,
                    int mode, double du[6]);

/* ---- absorption, src/absorption.jl ---- */
int or_abs_al_init(int n);
double or_abs_albajar_fast(double omega, double X, double Y, double N_abs, double N_par,
                           double Te, int mode);
double or_alpha_approx(const or_plasma *p, const double x[3], const double N[3],
                       double omega, int mode);
/* |dD/dN| (the gradLambda normalisation, src/solve.jl:85-95) */
double or_grad_norm(const or_plasma *p, const double x[3], const double N[3], double omega,
                    int mode);
/* warm alpha for absorption models 2 / 3 (iwarm 1 / 3), torj_warm_oracle.c:
 * the repaired src/general_absorption.jl:1328-1337 as oracle/warm_ref.py states
 * it; N_perp_warm^2 (re, im) into n2 when n2 != NULL */
double or_alpha_warm(double omega, double X, double Y, double N_abs, double N_par, double Te,
                     double inv_dDdN, int mode, int iwarm, double *n2);
double or_expei(double x);                      /* e^-x Ei(x), :29-232 */
void or_zetac(double x, double y, double out[2]); /* Z(x + iy), TOMS 680, :345-465 */
/* optional override of models 2 / 3 in the trace: (omega, X, Y, N_abs, N_par,
 * Te, 1/|dD/dN|, mode, model) -> alpha (the harness's numpy cross-check; NULL
 * restores or_alpha_warm) */
typedef double (*or_alpha_fn)(double, double, double, double, double, double, double, int, int);
void or_set_alpha_hook(or_alpha_fn fn);

/* ---- launch, src/launch.jl:24-132 and IMAS.pol_tor_angles_2_vector ---- */
long or_round_int(double x); /* Julia round(Int64, x): ties to even (src/launch.jl:81) */
int or_launch_count(int N_rings, int min_az);
int or_launch_peripheral_rays(const double x0[3], const double N0[3], double w,
                              double inv_curv, double f, int N_rings, int min_az,
                              int normalize, double *pos, double *dir, double *weights);
void or_pol_tor_angles_2_vector(double pol, double tor, double N[3]);

/* ---- ray entry, src/solve.jl:7-74 ---- */
int or_ray_entry(const or_plasma *p, const double x0[3], const double N0[3], double omega,
                 int mode, double xp[3], double Np[3], double *s0);

/* ---- fixed-step RK4 trace of sys! with optical depth + psi-shell deposition ----
 * Restates the make_ray loop (src/solve.jl:144-177) with the build's fixed-step
 * RK4 (ds), tau = -ln P (dtau/ds = alpha), termination checks at chunk
 * boundaries, and the shell-binned deposition defined in DESIGN.md. */
typedef struct {
    double omega;
    int mode;
    double ds;
    int n_steps;
    int chunk_steps;
    double psi_exit;
    double P_min;
    int absorption;          /* 0 none, 1 Albajar, 2 / 3 warm (or_alpha_warm) */
    int n_psi;               /* 0: no deposition */
    const double *psi_grid;  /* n_psi */
    int traj_stride;         /* 0: no trajectory */
    /* integrator 1: the reference's adaptive solve() -- see or_trace_samples */
    int integrator;
    double abstol, reltol, s_max;
    int n_chunks;
    const double *s0;        /* n_rays start arc lengths (tspans begin at s0), may be NULL */
} or_trace_cfg;

/* x0,N0: n_rays x 3 (ray-major); weights may be NULL (=1).
 * out_state n_rays x 7 (x, N, tau); out_dP n_psi (sum over rays of w*dP per
 * shell, NOT divided by dV); out_Pdep n_rays (unweighted deposited power);
 * out_traj n_rays x n_save x 5 (x,y,z,tau,s), n_save = n_steps/traj_stride
 * (integrator 1: n_steps = capacity of accepted steps, s the step's arc length). */
int or_trace(const or_plasma *p, const or_trace_cfg *cfg, int n_rays, const double *x0,
             const double *N0, const double *weights, double *out_state, int *out_status,
             int *out_steps, double *out_dP, double *out_Pdep, double *out_traj,
             int n_threads);

/* Same, plus the per-step samples make_ray stores for power_deposition_profile
 * (src/solve.jl:164-172): out_samples n_rays x (n_steps+1) x 3 =
 * (psi(x_k), dP/ds_k = P_k alpha_approx(x_k, N_k), s_k) for k = 0 (entry
 * point, dP/ds = 0 as the reference's initial vector, :151) .. steps; NaN beyond. */
/* a-priori sensitivity of warm traces' optical depths to relative input
 * perturbations eta at every RK4 stage point (see torj_oracle.c): out_sens[r] =
 * sum over ray r's stages (first steps[r] steps) of ds w_stage max |d alpha| */
void or_warm_sensitivity(const or_plasma *p, double omega, int mode, int iwarm, double ds,
                         int n_rays, const double *x0, const double *N0, const int *steps,
                         double eta, double *out_sens, int n_threads);
/* the same for the Albajar model (abs_Albajar_fast's inputs X, Y, N_par, Te) */
void or_albajar_sensitivity(const or_plasma *p, double omega, int mode, double ds, int n_rays,
                            const double *x0, const double *N0, const int *steps, double eta,
                            double *out_sens, int n_threads);
int or_trace_samples(const or_plasma *p, const or_trace_cfg *cfg, int n_rays, const double *x0,
                     const double *N0, const double *weights, double *out_state, int *out_status,
                     int *out_steps, double *out_dP, double *out_Pdep, double *out_traj,
                     double *out_samples, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
