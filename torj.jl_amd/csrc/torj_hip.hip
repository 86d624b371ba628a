// torj_hip.hip -- libtorj_hip.so: HIP (gfx950) kernels for TorJ.jl's ray-tracing
// hot path plus the C ABI declared in include/torj_hip.h.
//
// Layout of work:
//   k_trace<ABS,DEPO,TRAJ>  one lane per ray; the whole make_ray integration loop
//                           (src/solve.jl:154-177) runs in registers: fixed-step
//                           RK4 of gradΛ!/sys! (src/solve.jl:85-114), optical
//                           depth from abs_Albajar_fast (src/absorption.jl:191-226),
//                           chunk-granular termination, psi-shell deposition
//                           accumulated per lane and flushed with fp64 atomics.
//   k_eval_plasma / k_dispersion / k_albajar / k_refr
//                           batched point evaluations mirroring the reference's
//                           unit-tested functions (test_trajectory.jl, test_absorption.jl).
// Host side (this file): Plasma construction (Interpolations.jl-equivalent
// prefilter), the launch fan and the ray entry -- setup work the reference also
// does per beam/ray on the CPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/torj_hip.h"
#include "torj_math.hpp"
#include "torj_entry.hpp"
#include "torj_fitdepo.hpp"
#include "torj_warm.hpp"

using namespace torj;

// The split pipeline's trajectory kernel k_traj_cell is compiled in its own
// translation unit (torj_traj.hip, which includes this file up to the
// trajectory kernels with TORJ_TRAJ_TU defined) without machine-level loop-
// invariant code motion: hoisted out of the step loop, the kernel arguments'
// loads and constants held 208 VGPRs and spilled 15 SGPRs; left in place, 160
// VGPRs and no spill, so two trajectory waves and two 80-VGPR alpha waves share
// a SIMD.  The alpha kernel keeps the hoisting (without
// it +3.4 % VALU and +49 % SALU).  That TU's device globals are its own copies.
#ifndef TORJ_TRAJ_OWN_TU  // 1 (the Makefile): k_traj_cell comes from torj_traj.hip
#define TORJ_TRAJ_OWN_TU 0
#endif
#ifdef TORJ_TRAJ_TU
#define TORJ_TU_LOCAL static
#else
#define TORJ_TU_LOCAL
#endif

// ===========================================================================
// error handling
// ===========================================================================
static thread_local std::string g_err;

static int fail(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}

#define HIPCK(expr)                                                                       \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) return fail("%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// ===========================================================================
// Gauss-Legendre table in constant memory (abs_Al_init, src/absorption.jl:1-7)
// ===========================================================================
TORJ_TU_LOCAL __constant__ GLTable c_gl;

static std::mutex g_gl_mu;
static GLTable g_gl_host;
static int g_gl_version = 0;         // 0: abs_Al_init never called
static int g_gl_uploaded[64] = {0};  // per device

static void gauss_legendre(int n, double *x, double *w) {
    const int m = (n + 1) / 2;
    for (int i = 0; i < m; i++) {
        double z = std::cos(kPi * (i + 0.75) / (n + 0.5)), pp = 1.0;
        for (int it = 0; it < 100; it++) {
            double p0 = 1.0, p1 = z;  // P_0, P_1
            for (int j = 2; j <= n; j++) {
                const double p2 = ((2.0 * j - 1.0) * z * p1 - (j - 1.0) * p0) / j;
                p0 = p1;
                p1 = p2;
            }
            if (n == 1) p0 = 1.0, p1 = z;
            pp = n * (z * p1 - p0) / (z * z - 1.0);
            const double dz = p1 / pp;
            z -= dz;
            if (std::fabs(dz) < 1e-16) break;
        }
        x[i] = -z;
        x[n - 1 - i] = z;
        w[i] = w[n - 1 - i] = 2.0 / ((1.0 - z * z) * pp * pp);
    }
}

static int ensure_gl_on_device(int dev) {
    std::lock_guard<std::mutex> lk(g_gl_mu);
    if (g_gl_version == 0)
        return fail(
            "The weights and abscissae for the absorption were never initialized. Call "
            "`abs_Al_init` before using the absorption.");
    if (dev < 0 || dev >= 64) return fail("device index %d out of range", dev);
    if (g_gl_uploaded[dev] != g_gl_version) {
        HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(c_gl), &g_gl_host, sizeof(GLTable)));
        g_gl_uploaded[dev] = g_gl_version;
    }
    return 0;
}

// ===========================================================================
// kernels
// ===========================================================================
struct TraceArgs {
    const double *coef;
    const double *cellp;  // the coefficients' per-cell power form (torj_math.hpp cell_power_table)
    Grid g;
    Consts k;
    double omega;
    int mode;
    double ds;
    int n_steps;
    int chunk_steps;
    double psi_exit;
    double P_min;
    int n;
    const double *x0;  // 3 x n
    const double *N0;  // 3 x n
    const double *w;   // n or null
    double *state;     // 7 x n
    int *status;
    int *steps;
    int n_psi;
    const double *grid;
    double *dP;  // n_psi + 1
    double *Pdep;
    int traj_stride;
    int n_save;
    double *traj;  // n_save x 4 x n
    unsigned long long *counters;
    double *smp_psi;   // DEPO == 2: psi(x_k), torj::smp_at layout
    double *smp_dpds;  // DEPO == 2: P_k alpha(x_k), torj::smp_at layout
    double *smp_s;     // DEPO == 2: arc length s_k, torj::smp_at layout
    size_t smp_rows;   // rows per ray of the smp_at layout (n_steps + 2)
    int abs_model;     // 1 Albajar, 2 warm weakly relativistic, 3 warm fully relativistic
    const double *s0;  // n: arc length at the entry point (null: 0)
    // integrator 1 (the reference's adaptive solve)
    double abstol, reltol, s_step;
    int n_chunks;
    int *chunk;  // n: chunks done (work-queue visits carry it)
    // binned deposition in the work-queue kernel: per-wave LDS histogram of
    // n_hist shells at dynamic-LDS offset hist_off (doubles); 0 = global atomics
    int n_hist, hist_off;
};

// DEPO modes of the trace kernels
constexpr int kDepoNone = 0, kDepoBinned = 1, kDepoSamples = 2;

// psi shell j with grid[j] <= v < grid[j+1], clamped to [0, n-2]; identical
// result to a binary search on the grid array.
__device__ __forceinline__ int shell_of(const TraceArgs &a, double v) {
    // first guess as if the grid were uniform; accept it only if it brackets v,
    // else binary search: the result equals a binary search for any monotone grid
    const int nm2 = a.n_psi - 2;
    const double g0 = a.grid[0];
    int j = (int)floor((v - g0) * ((double)(a.n_psi - 1) / (a.grid[a.n_psi - 1] - g0)));
    j = j < 0 ? 0 : (j > nm2 ? nm2 : j);
    if (a.grid[j] <= v && (v < a.grid[j + 1] || j == nm2)) return j;
    int lo = 0, hi = a.n_psi - 1;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a.grid[mid] <= v)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

struct DepoAcc {
    int cur;
    double acc;
};

// a lane's finished run of deposits into one shell: the wave's LDS histogram
// (flushed to dP once per queue visit) or, without one, a global atomic
__device__ __forceinline__ void depo_flush(const TraceArgs &a, const DepoAcc &d) {
    if (d.cur < 0) return;
    if (a.n_hist > 0) {
        extern __shared__ double lds_dyn[];
        atomicAdd(lds_dyn + a.hist_off + d.cur, d.acc);
    } else {
        atomicAdd(a.dP + d.cur, d.acc);
    }
}

__device__ __forceinline__ void depo_add(const TraceArgs &a, DepoAcc &d, int j, double v) {
    if (j == d.cur) {
        d.acc += v;
    } else {
        depo_flush(a, d);
        d.cur = j;
        d.acc = v;
    }
}

// power dP deposited over a step whose psi runs linearly pa -> pb
__device__ __forceinline__ double deposit(const TraceArgs &a, DepoAcc &d, double pa, double pb,
                                          double dP, double w) {
    if (!(dP != 0.0)) return 0.0;
    const double lo = pa < pb ? pa : pb, hi = pa < pb ? pb : pa;
    const double g0 = a.grid[0], gl = a.grid[a.n_psi - 1];
    if (hi == lo) {
        if (lo < g0 || lo > gl) return 0.0;
        depo_add(a, d, shell_of(a, lo), w * dP);
        return dP;
    }
    if (hi <= g0 || lo >= gl) return 0.0;
    const double span = hi - lo;
    double inside = 0.0;
    for (int j = shell_of(a, lo < g0 ? g0 : lo); j < a.n_psi - 1 && a.grid[j] < hi; j++) {
        const double gj = a.grid[j], gj1 = a.grid[j + 1];
        const double x0 = lo > gj ? lo : gj, x1 = hi < gj1 ? hi : gj1;
        if (x1 <= x0) continue;
        const double part = dP * ((x1 - x0) / span);
        depo_add(a, d, j, w * part);
        inside += part;
    }
    return inside;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

#ifndef TORJ_BLOCK
#define TORJ_BLOCK 256
#endif
#ifndef TORJ_MIN_WAVES
#define TORJ_MIN_WAVES 2
#endif

// Per-lane ray state carried through a segment of steps.
struct RayState {
    double x[3], N[3], tau, Pdep;
    int status, steps;
};

// Integrate one ray from its current step to `s_end` (the make_ray loop,
// src/solve.jl:154-177): classic RK4 of sys!, optical depth, chunk-boundary
// termination, shell deposition, trajectory samples.  Shared by the one-shot
// and the work-queue kernels.
// LPR > 1: the ray's LPR lanes integrate it together (identical state in every
// lane; the absorption's node pairs are split between them) and lane sub = 0
// does the ray's stores.
template <int ABS, int DEPO, bool TRAJ, int LPR = 1>
__device__ __forceinline__ void ray_segment(const TraceArgs &a, int i, double w, RayState &r,
                                            int s_end, AlbajarWork &work, int sub = 0) {
    static_assert(LPR == 1 || (ABS == 1 && DEPO != kDepoBinned), "lanes per ray: Albajar, no binning");
    const bool wr = LPR == 1 || sub == 0;
    const GLTable &gl = c_gl;
    double *x = r.x, *N = r.N;
    double tau = r.tau;
    double P = exp(-tau);  // bitwise the value the previous step computed
    double psi_a = 0.0;
    DepoAcc dacc = {-1, 0.0};
    if constexpr (DEPO != kDepoNone) psi_a = eval_one(a.coef, a.g, sqrt(x[0] * x[0] + x[1] * x[1]), x[2], F_PSI);
    if constexpr (DEPO == kDepoSamples) {
        if (r.steps == 0 && wr) {  // entry point: make_ray's dP_ds starts with 0 (src/solve.jl:151)
            a.smp_psi[smp_at(0, i, a.smp_rows)] = psi_a;
            a.smp_dpds[smp_at(0, i, a.smp_rows)] = 0.0;  // arc lengths are implicit: s_k = s0 + k ds (FitArgs::S)
        }
    }
    const double ds = a.ds, hds = 0.5 * a.ds, ds6 = a.ds / 6.0;
    for (int s = r.steps; s < s_end; s++) {
        // classic RK4 with a single RHS call site (one copy of the spline +
        // Albajar code live -> lower VGPR pressure)
        double acc[6] = {0, 0, 0, 0, 0, 0}, acc_a = 0.0, xt[3], Nt[3], k[6], al, al0 = 0.0;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            xt[c] = x[c];
            Nt[c] = N[c];
        }
#pragma unroll 1
        for (int st = 0; st < 4; st++) {
            ray_rhs_m<ABS, LPR>(a.coef, a.g, a.k, gl, a.omega, a.mode, a.abs_model, xt, Nt, k, al,
                                wr ? &work : nullptr, sub);
            const double wgt = (st == 0 || st == 3) ? 1.0 : 2.0;
            const double h = (st < 2) ? hds : ds;
#pragma unroll
            for (int c = 0; c < 6; c++) acc[c] = fma(wgt, k[c], acc[c]);
            acc_a = fma(wgt, al, acc_a);
            if constexpr (DEPO == kDepoSamples) al0 = (st == 0) ? al : al0;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                xt[c] = fma(h, k[c], x[c]);
                Nt[c] = fma(h, k[3 + c], N[c]);
            }
        }
        double xn[3], Nn[3];
        bool bad = false;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            xn[c] = x[c] + ds6 * acc[c];
            Nn[c] = N[c] + ds6 * acc[3 + c];
            bad |= !isfinite(xn[c]) || !isfinite(Nn[c]);
        }
        const double taun = tau + ds6 * acc_a;
        bad |= !isfinite(taun);
        if (bad) {
            r.status = ST_NAN;
            break;
        }
        const double Pn = exp(-taun);
        const double dP = P - Pn;
        if constexpr (DEPO == kDepoSamples) {
            // dP/ds at the saved point x_s = P_s alpha_approx(x_s) (src/solve.jl:171):
            // the stage-0 RHS of this step evaluated exactly that alpha (al0)
            if (s > 0 && wr) a.smp_dpds[smp_at(s, i, a.smp_rows)] = P * al0;
        }
#pragma unroll
        for (int c = 0; c < 3; c++) {
            x[c] = xn[c];
            N[c] = Nn[c];
        }
        tau = taun;
        P = Pn;
        r.steps = s + 1;
        const bool check = a.chunk_steps > 0 && (r.steps % a.chunk_steps) == 0;
        double psi_b = 0.0;
        if (DEPO != kDepoNone || check)
            psi_b = eval_one(a.coef, a.g, sqrt(x[0] * x[0] + x[1] * x[1]), x[2], F_PSI);
        if constexpr (DEPO == kDepoSamples) {
            if (wr) a.smp_psi[smp_at(r.steps, i, a.smp_rows)] = psi_b;
        }
        if constexpr (DEPO == kDepoBinned) {
            r.Pdep += deposit(a, dacc, psi_a, psi_b, dP, w);
            psi_a = psi_b;
        }
        if constexpr (TRAJ) {
            if (wr && a.traj_stride > 0 && (r.steps % a.traj_stride) == 0) {
                const size_t si = (size_t)(r.steps / a.traj_stride - 1);
                double *T = a.traj + si * 5 * (size_t)a.n + i;
                T[0] = x[0];
                T[(size_t)a.n] = x[1];
                T[2 * (size_t)a.n] = x[2];
                T[3 * (size_t)a.n] = tau;
                T[4 * (size_t)a.n] = (a.s0 ? a.s0[i] : 0.0) + r.steps * a.ds;
            }
        }
        if (check) {
            if (psi_b > a.psi_exit) {  // src/solve.jl:174
                r.status = ST_LEFT_PLASMA;
                break;
            }
            if (P < a.P_min) {  // src/solve.jl:176
                r.status = ST_ABSORBED;
                break;
            }
        }
    }
    r.tau = tau;
    if constexpr (DEPO == kDepoBinned) {
        depo_flush(a, dacc);
    }
}

__device__ __forceinline__ void load_start(const TraceArgs &a, int i, RayState &r) {
#pragma unroll
    for (int c = 0; c < 3; c++) {
        r.x[c] = a.x0[c * a.n + i];
        r.N[c] = a.N0[c * a.n + i];
    }
    r.tau = 0.0;
    r.Pdep = 0.0;
    r.status = ST_OK;
    r.steps = 0;
}

__device__ __forceinline__ void store_state(const TraceArgs &a, int i, const RayState &r) {
#pragma unroll
    for (int c = 0; c < 3; c++) {
        a.state[c * a.n + i] = r.x[c];
        a.state[(3 + c) * a.n + i] = r.N[c];
    }
    a.state[6 * a.n + i] = r.tau;
    a.status[i] = r.status;
    a.steps[i] = r.steps;
    if (a.Pdep) a.Pdep[i] = r.Pdep;
}

__device__ __forceinline__ void flush_counters(const TraceArgs &a, unsigned long long steps,
                                               unsigned long long rhs, const AlbajarWork &work) {
    if (!a.counters) return;
    const unsigned long long s0 = wave_sum(steps);
    const unsigned long long s1 = wave_sum(rhs);
    const unsigned long long s2 = wave_sum((unsigned long long)work.n_active);
    const unsigned long long s3 = wave_sum((unsigned long long)work.n_harm);
    const unsigned long long s4 = wave_sum((unsigned long long)work.n_terms);
    const unsigned long long s5 = wave_sum((unsigned long long)work.n_zero);
    // [6]: Albajar's negligible-harmonic skips, or the warm model's sum of lrm
    // (each model leaves the other's field 0)
    const unsigned long long s6 = wave_sum((unsigned long long)(work.n_l + work.n_negl));
    const unsigned long long s7 = wave_sum((unsigned long long)(work.n_l2 + work.n_early));
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(a.counters + 0, s0);
        atomicAdd(a.counters + 1, s1);
        atomicAdd(a.counters + 2, s2);
        atomicAdd(a.counters + 3, s3);
        atomicAdd(a.counters + 4, s4);
        atomicAdd(a.counters + 5, s5);
        atomicAdd(a.counters + 6, s6);
        atomicAdd(a.counters + 7, s7);
    }
}

// One-shot kernel: LPR lanes per ray (1, or 16 for small beams whose rays
// would leave most SIMDs idle: the node pairs of the absorption integral are
// split between the ray's lanes), all steps in one pass.
template <int ABS, int DEPO, bool TRAJ, int LPR = 1>
__global__ void __launch_bounds__(TORJ_BLOCK, TORJ_MIN_WAVES) k_trace(TraceArgs a) {
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = gt / LPR, sub = gt % LPR;
    AlbajarWork work = {};
    unsigned long long steps = 0;
    if (i < a.n) {
        RayState r;
        load_start(a, i, r);
        const double w = (DEPO == kDepoBinned && a.w) ? a.w[i] : 1.0;
        ray_segment<ABS, DEPO, TRAJ, LPR>(a, i, w, r, a.n_steps, work, sub);
        if (sub == 0) {
            store_state(a, i, r);
            if constexpr (DEPO == kDepoBinned) atomicAdd(a.dP + a.n_psi, w * r.Pdep);  // sum_rays w P_dep
            steps = r.steps;
        }
    }
    flush_counters(a, steps, 4ull * steps, work);
}


// ---------------------------------------------------------------------------
// The reference's adaptive integration (integrator 1): one tspan chunk of
// solve(ODEProblem(sys!, u0, tspan; dtmax, abstol, reltol)) per visit
// (src/solve.jl:154-177), DifferentialEquations' default non-stiff method
// Tsit5 with OrdinaryDiffEq's PI controller and initial-step heuristic, on
// u = (x, N, P) with dP/ds = -P alpha.  The oracle restates the same
// algorithm (oracle/torj_oracle.c ts_ray); parity with DiffEq is unpinned.
// The seven stage vectors live in LDS (7 x 7 x 64 lanes x 8 B = 25 KB/wave).
// ---------------------------------------------------------------------------
TORJ_TU_LOCAL __constant__ double c_ts_a[7][6] = {
    {0, 0, 0, 0, 0, 0},
    {0.161, 0, 0, 0, 0, 0},
    {-0.008480655492356989, 0.335480655492357, 0, 0, 0, 0},
    {2.897153057105493, -6.359448489975075, 4.3622954328695815, 0, 0, 0},
    {5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525, 0, 0},
    {5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401,
     -0.028269050394068383, 0},
    {0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081,
     2.324710524099774}};
TORJ_TU_LOCAL __constant__ double c_ts_bt[7] = {-0.00178001105222577714, -0.0008164344596567469,
                                  0.007880878010261995,    -0.1447110071732629,
                                  0.5823571654525552,      -0.45808210592918697,
                                  0.015151515151515152};
constexpr int kTsLds = 7 * 7 * 64;  // doubles per wave

template <int ABS>
__device__ __forceinline__ void rhs7(const TraceArgs &a, const double u[7], double du[7],
                                     AlbajarWork &work, unsigned long long &nrhs) {
    double al;
    ray_rhs_m<ABS, 1, false>(a.coef, a.g, a.k, c_gl, a.omega, a.mode, a.abs_model, u, u + 3, du, al, &work);
    du[6] = -u[6] * al;  // sys!: du[7] = -P alpha (src/solve.jl:113)
    nrhs++;
}

__device__ __forceinline__ double rms7(const double v[7]) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 7; q++) s = fma(v[q], v[q], s);
    return sqrt(s * (1.0 / 7.0));
}

template <int ABS, int DEPO, bool TRAJ>
__device__ void ray_chunk_tsit5(const TraceArgs &a, int i, double w, RayState &r, int ch,
                                double *kl, AlbajarWork &work, unsigned long long &nrhs) {
    // kl: this wave's LDS stage store, [stage][component][lane].  One RHS call
    // site: the loop walks the phases fsalfirst (st = -2), the initial-step
    // probe (st = -1) and the Tsit5 stages 1..6; all lanes stay in lockstep.
    const int lane = threadIdx.x & 63;
    auto K = [&](int st, int q) -> double & { return kl[(st * 7 + q) * 64 + lane]; };
    const double s_start = a.s0 ? a.s0[i] : 0.0;
    double t = (double)(ch - 1) * a.s_step + s_start;  // Float64(i-1)*s_step + s0
    const double tf = (double)ch * a.s_step + s_start;
    double u[7] = {r.x[0], r.x[1], r.x[2], r.N[0], r.N[1], r.N[2], r.tau};  // tau slot holds P
    double ut[7], dt = 0.0, dt0 = 0.0, d1 = 0.0, qold = 1e-4, q11 = 0.0;
    double psi_a = 0.0;
    if constexpr (DEPO == kDepoBinned) psi_a = eval_one(a.coef, a.g, sqrt(u[0] * u[0] + u[1] * u[1]), u[2], F_PSI);
    DepoAcc dacc = {-1, 0.0};
    int st = -2;
#pragma unroll 1
    for (;;) {
        if (st == -2) {
#pragma unroll
            for (int q = 0; q < 7; q++) ut[q] = u[q];
        } else if (st == -1) {
#pragma unroll
            for (int q = 0; q < 7; q++) ut[q] = fma(dt0, K(0, q), u[q]);
        } else {
            if (st == 1 && r.steps >= a.n_steps) {  // no room for another accepted step
                r.status = ST_MAX_STEPS;
                break;
            }
#pragma unroll
            for (int q = 0; q < 7; q++) {
                double acc = 0.0;
#pragma unroll 1
                for (int j = 0; j < st; j++) acc = fma(c_ts_a[st][j], K(j, q), acc);
                ut[q] = fma(dt, acc, u[q]);
            }
        }
        double kq[7];
        rhs7<ABS>(a, ut, kq, work, nrhs);
        if (st == -2) {  // fsalfirst; ode_determine_initdt, first half
#pragma unroll
            for (int q = 0; q < 7; q++) K(0, q) = kq[q];
            double v0[7], v1[7];
#pragma unroll
            for (int q = 0; q < 7; q++) {
                const double sk = a.abstol + fabs(u[q]) * a.reltol;
                v0[q] = u[q] / sk;
                v1[q] = kq[q] / sk;
            }
            const double d0 = rms7(v0);
            d1 = rms7(v1);
            dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : (d0 / d1) / 100.0;
            dt0 = fmin(dt0, a.ds);
            st = -1;
            continue;
        }
        if (st == -1) {  // ode_determine_initdt, second half (order 5)
            bool same = true;
            double v[7];
#pragma unroll
            for (int q = 0; q < 7; q++) {
                same &= (K(0, q) == kq[q]);
                v[q] = (kq[q] - K(0, q)) / (a.abstol + fabs(u[q]) * a.reltol);
            }
            if (same) {
                dt = 100.0 * dt0;
            } else {
                const double d2 = rms7(v) / dt0, m = fmax(d1, d2);
                const double dt1 = (m <= 1e-15) ? fmax(1e-6, dt0 * 1e-3) : pow(10.0, -(2.0 + log10(m)) / 5.0);
                dt = fmin(fmin(100.0 * dt0, dt1), a.ds);
            }
            if (!(t < tf)) break;
            dt = fmin(fabs(dt), tf - t);  // modify_dt_for_tstops!
            st = 1;
            continue;
        }
#pragma unroll
        for (int q = 0; q < 7; q++) K(st, q) = kq[q];
        if (st < 6) {
            st++;
            continue;
        }
        // ut = u_{n+1}; stage 6 is f(u_{n+1}) (FSAL): error estimate and step control
        double e[7];
        bool bad = false;
#pragma unroll
        for (int q = 0; q < 7; q++) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < 7; j++) acc = fma(c_ts_bt[j], K(j, q), acc);
            e[q] = dt * acc / (a.abstol + fmax(fabs(u[q]), fabs(ut[q])) * a.reltol);
            bad |= !isfinite(ut[q]);
        }
        if (bad) {
            r.status = ST_NAN;
            break;
        }
        const double EEst = rms7(e);
        double qq;
        if (EEst == 0.0) {
            qq = 0.1;
        } else {
            q11 = pow(EEst, 0.14);
            qq = fmax(0.1, fmin(5.0, (q11 / pow(qold, 0.08)) / 0.9));
        }
        if (EEst <= 1.0) {  // accept (qsteady_min = qsteady_max = 1)
            qold = fmax(EEst, 1e-4);
            const double dtnew = dt / qq;
            double tn = t + dt;
            if (fabs(tn - tf) < 100.0 * 2.220446049250313e-16 * fmax(fabs(t), fabs(tf))) tn = tf;
            const double Pa = u[6];
#pragma unroll
            for (int q = 0; q < 7; q++) {
                u[q] = ut[q];
                K(0, q) = K(6, q);
            }
            // the reference's ContinuousCallback(u[7] < 0, affect!): P is
            // projected to 0 (src/solve.jl:78-83,159-160), applied at the end of
            // the accepted step that crossed (DiffEq would root-find the crossing
            // inside the step; that location is unpinned here), and the FSAL
            // derivative follows: dP/ds = -P alpha = -0
            if (u[6] < 0.0) {
                u[6] = 0.0;
                K(0, 6) = -0.0;
            }
            t = tn;
            r.steps++;
            if constexpr (DEPO != kDepoNone) {
                const double psi_b = eval_one(a.coef, a.g, sqrt(u[0] * u[0] + u[1] * u[1]), u[2], F_PSI);
                if constexpr (DEPO == kDepoSamples) {
                    const size_t o = smp_at(r.steps, i, a.smp_rows);
                    a.smp_psi[o] = psi_b;
                    a.smp_dpds[o] = -K(0, 6);  // P alpha at the saved point (FSAL)
                    a.smp_s[o] = t;
                }
                if constexpr (DEPO == kDepoBinned) {
                    r.Pdep += deposit(a, dacc, psi_a, psi_b, Pa - u[6], w);
                    psi_a = psi_b;
                }
            }
            if constexpr (TRAJ) {
                if (a.traj_stride > 0 && (r.steps % a.traj_stride) == 0 &&
                    r.steps / a.traj_stride <= a.n_save) {
                    double *T = a.traj + (size_t)(r.steps / a.traj_stride - 1) * 5 * a.n + i;
                    T[0] = u[0];
                    T[(size_t)a.n] = u[1];
                    T[2 * (size_t)a.n] = u[2];
                    T[3 * (size_t)a.n] = -log(u[6]);
                    T[4 * (size_t)a.n] = t;
                }
            }
            dt = fmin(a.ds, dtnew);  // calc_dt_propose! (dtmax)
            if (!(t < tf)) break;
        } else {  // reject: step_reject_controller!(PIController)
            dt /= fmin(5.0, q11 / 0.9);
        }
        dt = fmin(fabs(dt), tf - t);  // modify_dt_for_tstops!
        st = 1;
    }
    if constexpr (DEPO == kDepoBinned) {
        depo_flush(a, dacc);
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
        r.x[c] = u[c];
        r.N[c] = u[3 + c];
    }
    r.tau = u[6];
    if (r.status == ST_OK) {  // chunk-end checks (src/solve.jl:174, :176)
        if (eval_one(a.coef, a.g, sqrt(u[0] * u[0] + u[1] * u[1]), u[2], F_PSI) > a.psi_exit)
            r.status = ST_LEFT_PLASMA;
        else if (u[6] < a.P_min)
            r.status = ST_ABSORBED;
    }
}

// Work-queue kernel (ready-queue of ray groups).
// The beam is cut into G groups of 64 rays (one wave each); a group's
// integration is done in visits of `cs` steps (the reference's termination
// chunk).  Waves pop a ready group, integrate one chunk, store its state and
// push it back (or retire it when all its rays are done).  Groups therefore
// migrate between SIMDs: SIMDs holding one wave (which runs a wave ~1.7x
// faster than a SIMD holding two) absorb more visits, evening out the 1.53
// waves/SIMD of a 1e5-ray beam.
//
// Queue: pops take head tickets h; h < G are the initial visits of group h;
// h >= G consume push position p = h - G, published as one 8-byte granule
// {tag = p + 1, group} (agent-scope release fence after the state stores, then
// a relaxed agent store).  Pop: relaxed agent poll of the granule, then an
// agent acquire fence before the state loads (MI355X_MICROARCH.md visibility
// rules).  Every spin is bounded (err flag after 120 s without a push or a
// retirement anywhere) and every wave exits once all G groups have retired,
// so the grid always drains.
struct SchedCtl {
    unsigned head, tail, finished, err;
};

constexpr unsigned kGroupExit = 0xffffffffu;
constexpr unsigned long long kStallTicks = 120ull * 100000000ull;  // 120 s at 100 MHz

// returns the group index; bit 31 set = first visit (state from x0/N0)
__device__ __forceinline__ unsigned sched_pop(SchedCtl *ctl, unsigned long long *slots, unsigned S,
                                              unsigned G) {
    unsigned g = kGroupExit;
    if (threadIdx.x == 0) {
        const unsigned h = __hip_atomic_fetch_add(&ctl->head, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        if (h < G) {
            g = h | 0x80000000u;
        } else {
            const unsigned long long pos = h - G;
            unsigned long long *slot = slots + (pos % S);
            // stall watchdog: no push and no retirement anywhere in the grid for
            // kStallTicks of the 100 MHz realtime clock (a long chunk of heavy
            // physics is progress elsewhere, not a stall)
            unsigned long long t_prog = __builtin_amdgcn_s_memrealtime();
            unsigned prog = 0xffffffffu;
            for (unsigned spins = 0;; spins++) {
                unsigned long long v = __hip_atomic_load(slot, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                if ((v >> 32) == pos + 1) {
                    g = (unsigned)v;
                    break;
                }
                if (__hip_atomic_load(&ctl->finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= G) {
                    v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    g = ((v >> 32) == pos + 1) ? (unsigned)v : kGroupExit;
                    break;
                }
                if ((spins & 255u) == 0) {
                    const unsigned pr =
                        __hip_atomic_load(&ctl->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                        __hip_atomic_load(&ctl->finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                    if (pr != prog) {
                        prog = pr;
                        t_prog = now;
                    } else if (now - t_prog > kStallTicks) {  // never hang the device
                        __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(4);
            }
        }
    }
    g = __shfl(g, 0, 64);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return g;
}

__device__ __forceinline__ void sched_publish_begin() {
    // every lane's state stores are issued by this one wave: drain them, then
    // write back the XCD L2 (agent release) before the granule / counter
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// warm kernels: one wave per SIMD -- the 512-VGPR budget holds the warm
// tensor without spills (C5: 458 vs 505 ms at two waves per SIMD)
// rays per work-queue group (one wave's lanes; fewer leaves the upper lanes idle)
#ifndef TORJ_GROUP
#define TORJ_GROUP 64
#endif
#ifndef TORJ_WARM_MIN_WAVES
#define TORJ_WARM_MIN_WAVES 1
#endif
template <int ABS, int DEPO, bool TRAJ, int INTEG>
__global__ void __launch_bounds__(64, ABS >= 2 ? TORJ_WARM_MIN_WAVES : TORJ_MIN_WAVES) k_trace_sched(TraceArgs a, SchedCtl *ctl,
                                                                     unsigned long long *slots,
                                                                     unsigned S, int G, int cs) {
    extern __shared__ double lds_k[];  // integrator 1: Tsit5 stage vectors of this wave
    AlbajarWork work = {};
    unsigned long long steps = 0, nrhs = 0;
    double *hist = lds_k + a.hist_off;  // binned deposition: this wave's shell histogram
    if constexpr (DEPO == kDepoBinned) {
        for (int k = threadIdx.x; k < a.n_hist; k += 64) hist[k] = 0.0;
    }
    for (;;) {
        const unsigned t = sched_pop(ctl, slots, S, (unsigned)G);
        if (t == kGroupExit) break;
        const unsigned g = t & 0x7fffffffu;
        const int i = (int)g * TORJ_GROUP + threadIdx.x;
        bool alive = false;
        if (threadIdx.x < TORJ_GROUP && i < a.n) {
            RayState r;
            int ch = 0;
            if (t & 0x80000000u) {
                load_start(a, i, r);
                if constexpr (INTEG == 1) r.tau = 1.0;  // the tau slot carries P
            } else {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    r.x[c] = a.state[c * a.n + i];
                    r.N[c] = a.state[(3 + c) * a.n + i];
                }
                r.tau = a.state[6 * a.n + i];
                r.status = a.status[i];
                r.steps = a.steps[i];
                r.Pdep = a.Pdep ? a.Pdep[i] : 0.0;
                if constexpr (INTEG == 1) ch = a.chunk[i];
            }
            const double w = (DEPO == kDepoBinned && a.w) ? a.w[i] : 1.0;
            if constexpr (INTEG == 0) {
                if (r.status == ST_OK && r.steps < a.n_steps) {
                    const int s0 = r.steps;
                    const int s_end = min(a.n_steps, (s0 / cs + 1) * cs);
                    ray_segment<ABS, DEPO, TRAJ>(a, i, w, r, s_end, work);
                    steps += (unsigned long long)(r.steps - s0);
                    nrhs += 4ull * (unsigned long long)(r.steps - s0);
                    alive = r.status == ST_OK && r.steps < a.n_steps;
                    if constexpr (DEPO == kDepoBinned) {
                        if (!alive) atomicAdd(a.dP + a.n_psi, w * r.Pdep);  // sum_rays w P_dep
                    }
                }
                store_state(a, i, r);
            } else {
                const bool ran = r.status == ST_OK && ch < a.n_chunks;
                if (ran) {
                    const int s0 = r.steps;
                    if constexpr (DEPO == kDepoSamples) {
                        if (ch == 0) {  // entry point (src/solve.jl:151)
                            const size_t o = smp_at(0, i, a.smp_rows);
                            a.smp_psi[o] = eval_one(a.coef, a.g, sqrt(r.x[0] * r.x[0] + r.x[1] * r.x[1]), r.x[2], F_PSI);
                            a.smp_dpds[o] = 0.0;
                            a.smp_s[o] = a.s0 ? a.s0[i] : 0.0;
                        }
                    }
                    ch++;
                    ray_chunk_tsit5<ABS, DEPO, TRAJ>(a, i, w, r, ch, lds_k, work, nrhs);
                    steps += (unsigned long long)(r.steps - s0);
                    alive = r.status == ST_OK && ch < a.n_chunks;
                    if constexpr (DEPO == kDepoBinned) {
                        if (!alive) atomicAdd(a.dP + a.n_psi, w * r.Pdep);
                    }
                }
                a.chunk[i] = ch;
                // the tau slot carries P while the ray runs and tau = -ln P once it
                // has finished -- converted on the visit that finished it only (a
                // finished ray of a live group is reloaded and stored again)
                if (ran && !alive) r.tau = -log(r.tau);  // final state carries tau = -ln P
                store_state(a, i, r);
            }
        }
        const bool any_alive = __any(alive);
        if constexpr (DEPO == kDepoBinned) {  // the visit's shell sums: LDS -> dP
            if (a.n_hist > 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                for (int k = threadIdx.x; k < a.n_hist; k += 64) {
                    const double v = hist[k];
                    if (v != 0.0) {
                        atomicAdd(a.dP + k, v);
                        hist[k] = 0.0;
                    }
                }
            }
        }
        sched_publish_begin();
        if (threadIdx.x == 0) {
            if (any_alive) {
                const unsigned long long pos = __hip_atomic_fetch_add(&ctl->tail, 1u, __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(slots + (pos % S), ((pos + 1) << 32) | (unsigned long long)g,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_fetch_add(&ctl->finished, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    flush_counters(a, steps, nrhs, work);
}

// ---------------------------------------------------------------------------
// Split RK4 path: trajectory and optical depth as separate, overlapped kernels
// (fixed-step RK4, Albajar).
//
// In sys! (src/solve.jl:112-114) dx/ds and dN/ds are gradΛ!(x, N) alone: the
// absorption only drives u[7].  So the trajectory of every ray is fixed before
// any alpha is known, and the 4 x n_steps alpha evaluations of a ray are
// independent of each other -- the step's chain is the cheap cold RHS, the
// expensive part is embarrassingly parallel.  Per block of B steps:
//   k_traj      one lane per ray: the cold RK4 steps (the same arithmetic as
//               ray_segment), writing each stage's alpha inputs (X, Y, |N|,
//               N_par, Te), psi per step, chunk-boundary states, trajectory
//               samples; stops LEFT_PLASMA / NAN exactly as ray_segment;
//   k_alpha_pts one lane per (ray, step, stage): abs_albajar_fast at the
//               stored inputs -- a fully occupied grid, no step chain;
//   k_tau_scan  one lane per ray, in step order: tau += ds/6 (a0 + 2a1 + 2a2 +
//               a3) with ray_segment's fma order, P = exp(-tau), the ABSORBED
//               check at chunk boundaries (after T's psi check, as the
//               reference), make_ray's dP/ds samples, binned deposition, tau in
//               the trajectory samples;
// then k_split_final assembles the final state (a ray the scan stops earlier
// than the trajectory takes its chunk-boundary state, or replays the last
// steps when alpha itself went non-finite).  k_traj of block b+1 runs on the
// caller's stream while k_alpha_pts / k_tau_scan of block b run on a second
// stream: the trajectory waves (~1.5 per SIMD on a 1e5-ray beam) and the alpha
// waves share the SIMDs.  A wave of k_alpha_pts holds the 64 rays of a 64-ray
// group at one (step, stage): the same lanes as the fused kernel's wave there,
// so the per-wave Bessel-level ballot and every alpha are the same bits.
// ---------------------------------------------------------------------------
constexpr int kAinF = 5;  // X, Y, |N|^2, N_par, ln Te (warm: X, Y, |N|, N_par, Te, 1 / |dD/dN|: kAinFW)
constexpr int kAinFW = 6;

struct SplitArgs {
    double *ain;          // [j][stage][f][n]: this block's alpha inputs, nf fields
    double *alpha;        // [j][stage][n]
    unsigned *awork;      // [j][stage][n] (null unless counted): alpha work counts; Albajar: bit 0 active,
                          // bits 1-2 harmonics, 3-4 exact-zero harmonics, 5-15 Bessel terms,
                          // 16-17 negligible harmonics;
                          // warm: bits 0-6 larmornumber tests, 7-13 Faddeeva evaluations,
                          // 14-20 warmdisp passes, 21-23 Larmor order
    double *psib;         // binned deposition: psi at the end of step k0 + j, [j][n]
    double *cbx;          // [c][6][n]: x, N at chunk boundary c (steps = c * chunk_steps)
    double *tx;           // [6][n]: the trajectory kernel's carry
    int *tinfo;           // steps | status << 24: the trajectory kernel's stop (one store)
    double *stau, *spsi, *sPdep;  // the scan's carry
    int *sinfo;           // steps | status << 24: the scan's stop
    unsigned char *zflag;  // per ray, this block (ring slot): 1 = Albajar alpha provably +-0 at every
                           // stage point the trajectory kernel stored (zero_box_flag); null: off
    double zval;           // what a fully flagged alpha wave writes: 0, or NaN under the test hook
                           // TORJ_TEST_ZFLAG_NAN=1 (the flagged waves then stop their rays NAN)
    int k0, kb;           // block: steps [k0, k0 + kb)
    int nf;               // alpha input fields per point: kAinF (Albajar) or kAinFW (warm)
    int tile_cap;         // k_traj_tile: most nodes a wave stages (<= kTileNodes)
    double tile_margin;   // k_traj_tile: the box's margin in units of the block's path, (kb + 1) ds
    int traj_mode;        // the trajectory kernel (kTrajL2 .. kTrajCell): the NaN-alpha replay uses its arithmetic
    int nan_step;         // test hook (TORJ_TEST_NAN_ALPHA_STEP, default -1): the scan reads alpha as NaN
                          // at this step for every third ray, to exercise the NaN-alpha replay
    unsigned long long *defer;  // warm: the block's points with lrm > 3, (js << 32) | i, for k_alpha_warm_big
    unsigned *defer_cnt;        // warm: their count (this block's slot, zeroed per launch)
    int defer_lrm;              // warm: points with lrm above this are deferred (3; TORJ_WARM_DEFER_LRM
                                // lowers it: a test sends every point through the deferred path)
};

// steps | status << 24: split launches need n_steps < kSplitMaxSteps (the
// fused kernels have no such limit and take longer traces)
constexpr int kSplitMaxSteps = 1 << 24;
__device__ __forceinline__ int info_steps(int v) { return v & 0xffffff; }
__device__ __forceinline__ int info_status(int v) { return (unsigned)v >> 24; }
__device__ __forceinline__ int make_info(int steps, int st) { return steps | (st << 24); }

// The alpha-input box of one ray over a block (round 6): the range of ln Te,
// Y, N_par^2 and N_perp^2 over every stage point the trajectory kernel stored.
// zero_box_flag proves from it that abs_albajar_fast_body returns +-0 at every
// one of them -- all Te < 20 eV, or each harmonic m = 2, 3 absent (m Y <
// sqrt(1 - N_par^2)) or an exact zero (every node's exp(mu (1 - gamma))
// underflows: gamma_min > 1 + 760 / mu, with gamma_min >= m Y / (1 + |N_par|)
// on the resonance gamma - N_par u_par = m Y, |u_par| <= gamma) -- the early
// settle of abs_albajar_fast_body (and its exact-zero test), which returns +0
// there, decided for a whole block with relative margins of 1e-9 against
// their roundings.  k_alpha_pts then writes 0 for a wave whose 64 rays all
// carry the flag instead of evaluating it (42 % of its waves settle early on the
// headline beam).
struct ZBox {
    double lte = -INFINITY, ylo = INFINITY, yhi = -INFINITY, np2 = -INFINITY, perp = INFINITY;
    double chk = 0.0;  // stays 0 unless an input was NaN or infinite
};
// v_max_f64 / v_min_f64 as one instruction each: fmax / fmin would first
// quiet both operands (two more v_max_f64 per call, 24 VALU per stage point
// for the box instead of 12); NaN inputs are caught by chk, not by these
__device__ __forceinline__ double zb_max(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double zb_min(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ void zero_box_add(ZBox &b, double lnTe, double Y, double Npar, double N2) {
    const double np2 = Npar * Npar;
    b.lte = zb_max(b.lte, lnTe);
    b.ylo = zb_min(b.ylo, Y);
    b.yhi = zb_max(b.yhi, Y);
    b.np2 = zb_max(b.np2, np2);
    b.perp = zb_min(b.perp, fma(-1e-9, N2, N2 - np2));  // N_perp^2 with a relative margin
    b.chk = fma((lnTe + Y) + (Npar + N2), 0.0, b.chk);  // NaN once any input is NaN or infinite
}
__device__ __forceinline__ bool zero_box_flag(const ZBox &b) {
    if (!(b.chk == 0.0)) return false;
    if (b.lte < 2.9957322735539909 - 1e-9) return true;  // every Te < 20 eV (ln 20)
    if (!(b.ylo > 1e-200 && b.yhi < 1e200 && b.perp > 0.0 && b.np2 < 1.0 - 1e-9 && b.lte < 700.0))
        return false;
    constexpr double kMuTe = kMe * kC * kC / kE;  // mu Te (albajar_pre)
    const double delta = 760.0 * (1.0 + 1e-9) * exp(b.lte) * (1.0 / kMuTe);  // 760 / mu_min
    const double npm = sqrt(b.np2), sq = sqrt(1.0 - b.np2);
    bool ok = true;
#pragma unroll
    for (int m = 2; m <= 3; m++) {
        const bool absent = m * b.yhi * (1.0 + 1e-9) < sq * (1.0 - 1e-9);
        const bool zero = m * b.ylo > (1.0 + delta) * (1.0 + npm) * (1.0 + 1e-9);
        ok = ok && (absent || zero);
    }
    return ok;
}

#ifndef TORJ_AIN_TRAJ_MATH  // 1: the trajectory kernel stores |N| and Te for k_alpha_pts (not |N|^2, ln Te)
#define TORJ_AIN_TRAJ_MATH 0
#endif
// One cold RK4 step of ray_segment's arithmetic (plasma_point with ln Te, as
// the absorbing kernels evaluate it); STORE: this step's alpha inputs -> ain.
// PSI: stage 0's stencil also sums psi at x (the step's start), returned in
// *psi_x -- the psi the previous step's end needs (traj_run), bit for bit the
// eval_one at that point.
template <bool STORE, int NS = kNF, class CS = const double *, bool PSI = false>
__device__ __forceinline__ bool cold_step(const TraceArgs &a, CS coef,
                                          const SplitArgs &sp, int j, int i, const double x[3],
                                          const double N[3], double xn[3], double Nn[3],
                                          double *psi_x, ZBox &zb, bool zon) {
    const double hds = 0.5 * a.ds, ds6 = a.ds / 6.0;
    double acc[6] = {0, 0, 0, 0, 0, 0}, xt[3], Nt[3], k[6];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        xt[c] = x[c];
        Nt[c] = N[c];
    }
#pragma unroll 1
    for (int st = 0; st < 4; st++) {
        PlasmaPoint p;
        if constexpr (PSI) {
            // stage 0 with the sixth field (a branch around whole evaluations: a
            // per-field gate inside the stencil split its blocks and spilled)
            if (st == 0) {
                plasma_point<true, NS, CS, true>(coef, a.g, a.k, xt, p);
                *psi_x = p.psi;
            } else {
                plasma_point<true, NS>(coef, a.g, a.k, xt, p);
            }
        } else {
            plasma_point<true, NS>(coef, a.g, a.k, xt, p);
        }
        double Npar, inv;
        dispersion_grad(p, Nt, a.mode, k, &Npar, &inv);
        if constexpr (STORE) {
            double *o = sp.ain + ((size_t)(j * 4 + st) * sp.nf) * a.n + i;
            const double N2 = Nt[0] * Nt[0] + Nt[1] * Nt[1] + Nt[2] * Nt[2];
            if (zon) zero_box_add(zb, p.lnTe, p.Y, Npar, N2);
            o[0] = p.X;
            o[(size_t)a.n] = p.Y;
            o[3 * (size_t)a.n] = Npar;
            if (sp.nf > kAinF) {  // the warm inputs as ray_rhs_m<2 / 3> forms them
                o[2 * (size_t)a.n] = sqrt(N2);
                o[4 * (size_t)a.n] = exp(p.lnTe);
                o[kAinF * (size_t)a.n] = inv;
            } else if constexpr (TORJ_AIN_TRAJ_MATH) {
                // |N| and Te by the functions k_alpha_pts would apply (the same
                // bits), on the trajectory chain, which has slack once the alpha
                // chain is the pipeline's critical one
                o[2 * (size_t)a.n] = sqrt_pos(N2);
                o[4 * (size_t)a.n] = exp_fast<true>(p.lnTe);
            } else {
                // |N|^2 and ln Te: k_alpha_pts takes the square root and the
                // exponential (the same functions ray_rhs applies), off the
                // latency-bound trajectory chain and onto the parallel alpha lanes
                o[2 * (size_t)a.n] = N2;
                o[4 * (size_t)a.n] = p.lnTe;
            }
        }
        const double wgt = (st == 0 || st == 3) ? 1.0 : 2.0;
        const double h = (st < 2) ? hds : a.ds;
#pragma unroll
        for (int c = 0; c < 6; c++) acc[c] = fma(wgt, k[c], acc[c]);
#pragma unroll
        for (int c = 0; c < 3; c++) {
            xt[c] = fma(h, k[c], x[c]);
            Nt[c] = fma(h, k[3 + c], N[c]);
        }
    }
    bool bad = false;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        xn[c] = x[c] + ds6 * acc[c];
        Nn[c] = N[c] + ds6 * acc[3 + c];
        bad |= !isfinite(xn[c]) || !isfinite(Nn[c]);
    }
    return bad;
}

#ifndef TORJ_TRAJ_WAVES
#define TORJ_TRAJ_WAVES TORJ_MIN_WAVES
#endif
#ifndef TORJ_ALPHA_WAVES  // k_alpha_pts' waves per SIMD bound (6: <= 80 VGPRs; round 5 with the tiny-alpha
// skip, alternating: 40.01 / 40.01 ms against 40.23 / 40.12 at 4, 96 VGPRs; 8 spills: 48.6 ms)
#define TORJ_ALPHA_WAVES 6
#endif
#ifndef TORJ_ALPHA_UNROLL  // node pairs per iteration of the alpha kernel's node loop (ILP)
#define TORJ_ALPHA_UNROLL 1
#endif
// Where the trajectory kernel reads the field coefficients:
//   kTrajL2    the global array through L1 / L2 (any grid);
//   kTrajLds   the whole grid staged in LDS (6 fp64 per node, 161 KB for a 56 x 56
//              grid: one workgroup of up to 8 waves per CU);
//   kTrajTile  per wave and block, only the tile of nodes its rays can reach in
//              the block's kb steps (|dx/ds| = 1, so within (kb + 1) ds of where
//              they start), a few KB: the kernel is no longer capped at one
//              workgroup per CU, and its waves share every SIMD with the alpha
//              waves.  A stencil outside the tile reads the global array (the
//              same values: results bit-identical in every mode).
//   kTrajCell  per wave and block, the tile of CELLS its rays can reach, each
//              cell's bicubic in power form (torj_math.hpp cell_sums: 28 fma per
//              field with its gradient against the node stencil's 44, no basis
//              weights); the same fallback to the global cell table.
enum { kTrajL2 = 0, kTrajLds = 1, kTrajTile = 2, kTrajCell = 3 };
constexpr int kTrajLdsNS = 6;
static_assert(kTrajLdsNS == kTileNS, "LDS layouts");
#ifndef TORJ_TILE_NODES
#define TORJ_TILE_NODES 256  // 12 KB of LDS per wave
#endif
constexpr int kTileNodes = TORJ_TILE_NODES;
#ifndef TORJ_TILE_CELLS
#define TORJ_TILE_CELLS 20  // 15 KB of LDS per wave
#endif
constexpr int kTileCells = TORJ_TILE_CELLS;

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
// the cell index axis_setup gives a coordinate (monotone in x)
__device__ __forceinline__ int cell_index(double x, double x1, double xn, double invh, int n) {
    const int i = (int)floor((clampd(x, x1, xn) - x1) * invh);
    return i < 0 ? 0 : (i > n - 2 ? n - 2 : i);
}

#ifndef TORJ_TRAJ_PREWAIT
#define TORJ_TRAJ_PREWAIT 1
#endif
// the trajectory steps of one ray over the block, from its carry (x, N, steps)
template <int DEPO, bool TRAJ, int NS, class CS>
__device__ __forceinline__ void traj_run(const TraceArgs &a, const SplitArgs &sp, CS coef, int i,
                                         double x[3], double N[3], int steps, int st) {
    if (sp.k0 == 0) {
        if constexpr (DEPO != kDepoNone) {
            const double psi0 = eval_one<NS>(coef, a.g, sqrt(x[0] * x[0] + x[1] * x[1]), x[2], F_PSI);
            sp.spsi[i] = psi0;  // the scan's psi_a at step 0
            if constexpr (DEPO == kDepoSamples) {
                a.smp_psi[smp_at(0, i, a.smp_rows)] = psi0;
                a.smp_dpds[smp_at(0, i, a.smp_rows)] = 0.0;
            }
        }
    }
    const int s_end = min(a.n_steps, sp.k0 + sp.kb);
    // psi at the end of step s - 1 is psi at x_s, which step s's stage 0 sums
    // from its own stencil (cold_step<PSI>): the end-of-step work that needs it
    // (make_ray's psi sample, the binned deposition's psi, the psi_exit check)
    // runs one iteration late, before step s's outcome is looked at, so the
    // order of stops is ray_segment's (psi check, then the next step's NaN);
    // the block's last step takes the one eval_one left.  A ray stopped by the
    // check has stored step s's alpha inputs too -- beyond its steps, so
    // k_alpha_pts and the scan never read them.
    auto step_end = [&](int k, double psi_b) -> bool {  // after step k (steps = k + 1)
        const int sk = k + 1;
        if constexpr (DEPO == kDepoSamples) a.smp_psi[smp_at(sk, i, a.smp_rows)] = psi_b;
        if constexpr (DEPO == kDepoBinned) sp.psib[(size_t)(k - sp.k0) * a.n + i] = psi_b;
        return a.chunk_steps > 0 && (sk % a.chunk_steps) == 0 && psi_b > a.psi_exit;  // src/solve.jl:174
    };
    const int s_first = steps;
    bool pending = false;  // step steps - 1 still needs its psi
    // (a value and a flag, not a pointer: a local behind a conditional pointer
    // lived in scratch, 56 B per lane, and slowed the kernel by ~14 %)
    ZBox zb;
    const bool zon = sp.zflag != nullptr;
#if defined(__HIP_DEVICE_COMPILE__) && TORJ_TRAJ_PREWAIT
    // every load before the step loop complete here (s_waitcnt vmcnt(0)): the
    // compiler otherwise waits at the loop header for the carry's loads, every
    // step, and on gfx9 vmcnt counts stores too -- each step would then wait for
    // its own last stage's alpha-input stores to reach memory
    __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
    for (int s = s_first; s < s_end; s++) {
        double xn[3], Nn[3], psi_x;
        const bool bad = cold_step<true, NS, CS, true>(a, coef, sp, s - sp.k0, i, x, N, xn, Nn, &psi_x, zb, zon);
        if (pending) {
            pending = false;
            if (step_end(s - 1, psi_x)) {
                st = ST_LEFT_PLASMA;
                break;
            }
        }
        if (bad) {
            st = ST_NAN;
            break;
        }
#pragma unroll
        for (int c = 0; c < 3; c++) {
            x[c] = xn[c];
            N[c] = Nn[c];
        }
        steps = s + 1;
        const bool check = a.chunk_steps > 0 && (steps % a.chunk_steps) == 0;
        pending = DEPO != kDepoNone || check;
        if constexpr (TRAJ) {
            if (a.traj_stride > 0 && (steps % a.traj_stride) == 0) {
                double *T = a.traj + (size_t)(steps / a.traj_stride - 1) * 5 * a.n + i;
                T[0] = x[0];
                T[(size_t)a.n] = x[1];
                T[2 * (size_t)a.n] = x[2];
                T[4 * (size_t)a.n] = (a.s0 ? a.s0[i] : 0.0) + steps * a.ds;
            }
        }
        if (check) {
            double *cb = sp.cbx + (size_t)(steps / a.chunk_steps) * 6 * a.n + i;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                cb[c * (size_t)a.n] = x[c];
                cb[(3 + c) * (size_t)a.n] = N[c];
            }
        }
    }
    double invR;
    if (pending && step_end(steps - 1, eval_one<NS>(coef, a.g, cyl_radius(x, invR), x[2], F_PSI)))
        st = ST_LEFT_PLASMA;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        sp.tx[c * (size_t)a.n + i] = x[c];
        sp.tx[(3 + c) * (size_t)a.n + i] = N[c];
    }
    sp.tinfo[i] = make_info(steps, st);
    if (zon) sp.zflag[i] = zero_box_flag(zb) ? 1 : 0;
}


template <int DEPO, bool TRAJ, int MODE>
__device__ __forceinline__ void traj_body(const TraceArgs &a, const SplitArgs &sp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double x[3] = {0, 0, 0}, N[3] = {0, 0, 0};
    int steps = 0, st = ST_OK;
    bool live = i < a.n;
    if (live) {
        if (sp.k0 == 0) {
#pragma unroll
            for (int c = 0; c < 3; c++) {
                x[c] = a.x0[c * a.n + i];
                N[c] = a.N0[c * a.n + i];
                sp.cbx[c * (size_t)a.n + i] = x[c];
                sp.cbx[(3 + c) * (size_t)a.n + i] = N[c];
            }
        } else {
            const int v = sp.tinfo[i];
            steps = info_steps(v);
            st = info_status(v);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                x[c] = sp.tx[c * (size_t)a.n + i];
                N[c] = sp.tx[(3 + c) * (size_t)a.n + i];
            }
        }
        // a ray the scan has stopped (ABSORBED) needs no more trajectory.  sinfo is
        // written by k_tau_scan on another stream while this kernel may run, so the
        // read can be stale.  INVARIANT: this early-out only saves work, it never
        // decides an output -- a stale OK just traces steps nobody reads (the scan
        // stopped first; k_split_final rebuilds the state from the chunk-boundary
        // copy and the scan's carry).  Keep it that way: tests/test_gpu_split.py
        // test_split_serial_equals_overlapped holds both orders bit-identical.
        live = st == ST_OK && !(sp.k0 > 0 && info_status(sp.sinfo[i]) != ST_OK);
        // a ray without trajectory steps in this block needs no alpha in it
        if (!live && sp.zflag) sp.zflag[i] = 1;
    }
    if constexpr (MODE == kTrajTile) {
        // one wave per workgroup: the wave's live rays' (R, Z) box, widened by
        // the path the block can take, and its nodes staged in LDS
        __shared__ __attribute__((aligned(16))) double s_tile[kTileNodes * kTileNS];
        const double R = sqrt(x[0] * x[0] + x[1] * x[1]);
        const double inf = __builtin_inf();
        const double rmin = wave_min(live ? R : inf), rmax = wave_max(live ? R : -inf);
        const double zmin = wave_min(live ? x[2] : inf), zmax = wave_max(live ? x[2] : -inf);
        if (!(rmin <= rmax && zmin <= zmax)) return;  // no live ray in the wave (wave-uniform)
        const double m = (double)(sp.kb + 1) * a.ds * sp.tile_margin;
        const int iR0 = cell_index(rmin - m, a.g.R1, a.g.Rn, a.g.invhR, a.g.nR),
                  iR1 = cell_index(rmax + m, a.g.R1, a.g.Rn, a.g.invhR, a.g.nR),
                  iZ0 = cell_index(zmin - m, a.g.Z1, a.g.Zn, a.g.invhZ, a.g.nZ),
                  iZ1 = cell_index(zmax + m, a.g.Z1, a.g.Zn, a.g.invhZ, a.g.nZ);
        TileCoef tc{a.coef, s_tile, iR0, iZ0, iR1 - iR0 + 4, iZ1 - iZ0 + 4};
        if (tc.tw * tc.th > sp.tile_cap) {
            tc.tw = tc.th = 0;  // too wide for the tile: every stencil from global memory
        } else {
            const int mR = a.g.nR + 2, cnt = tc.tw * tc.th * kTileNS;
            for (int k = threadIdx.x; k < cnt; k += 64) {
                const int node = k / kTileNS, f = k - node * kTileNS;
                const int zr = node / tc.tw, rr = node - zr * tc.tw;
                s_tile[k] = a.coef[((size_t)(iZ0 + zr) * mR + iR0 + rr) * kNF + f];
            }
        }
        __syncthreads();
        if (!live) return;
        traj_run<DEPO, TRAJ, kTileNS>(a, sp, tc, i, x, N, steps, st);
    } else if constexpr (MODE == kTrajCell) {
        // the cells the wave's live rays can reach in the block (the node tile's
        // box, by cell), their power-form records staged in LDS
        __shared__ __attribute__((aligned(16))) double s_cell[kTileCells * kCellRec];
        const double R = sqrt(x[0] * x[0] + x[1] * x[1]);
        const double inf = __builtin_inf();
        const double rmin = wave_min(live ? R : inf), rmax = wave_max(live ? R : -inf);
        const double zmin = wave_min(live ? x[2] : inf), zmax = wave_max(live ? x[2] : -inf);
        if (!(rmin <= rmax && zmin <= zmax)) return;  // no live ray in the wave (wave-uniform)
        const double m = (double)(sp.kb + 1) * a.ds * sp.tile_margin;
        const int iR0 = cell_index(rmin - m, a.g.R1, a.g.Rn, a.g.invhR, a.g.nR),
                  iR1 = cell_index(rmax + m, a.g.R1, a.g.Rn, a.g.invhR, a.g.nR),
                  iZ0 = cell_index(zmin - m, a.g.Z1, a.g.Zn, a.g.invhZ, a.g.nZ),
                  iZ1 = cell_index(zmax + m, a.g.Z1, a.g.Zn, a.g.invhZ, a.g.nZ);
        // the box is wave-uniform: scalar registers for the copy's loop
        const int cR0 = __builtin_amdgcn_readfirstlane(iR0), cZ0 = __builtin_amdgcn_readfirstlane(iZ0);
        const int cw = __builtin_amdgcn_readfirstlane(iR1 - iR0 + 1), ch = __builtin_amdgcn_readfirstlane(iZ1 - iZ0 + 1);
        TileCell tc{a.cellp, s_cell, cR0, cZ0, cw, ch};
        if (cw * ch > sp.tile_cap) {
            tc.cw = tc.ch = 0;  // too wide for the tile: every cell from global memory
        } else {
            // one cell record (48 x 16 B) per pass, lanes 0..47 (measured: four
            // loads in flight per lane over the flattened tile is no faster)
            const int cR = a.g.nR - 1;
            const Dbl2 *src = reinterpret_cast<const Dbl2 *>(a.cellp);
            Dbl2 *dst = reinterpret_cast<Dbl2 *>(s_cell);
            for (int zr = 0; zr < ch; zr++)
                for (int rr = 0; rr < cw; rr++)
                    if (threadIdx.x < kCellRec / 2)
                        dst[(zr * cw + rr) * (kCellRec / 2) + threadIdx.x] =
                            src[((size_t)(cZ0 + zr) * cR + cR0 + rr) * (kCellRec / 2) + threadIdx.x];
        }
        __syncthreads();
        if (!live) return;
        traj_run<DEPO, TRAJ, kTileNS>(a, sp, tc, i, x, N, steps, st);
    } else if constexpr (MODE == kTrajLds) {
        extern __shared__ __attribute__((aligned(16))) double s_coef[];
        const int nodes = (a.g.nR + 2) * (a.g.nZ + 2);
        for (int k = threadIdx.x; k < nodes * kTrajLdsNS; k += blockDim.x)
            s_coef[k] = a.coef[(size_t)(k / kTrajLdsNS) * kNF + k % kTrajLdsNS];
        __syncthreads();
        if (!live) return;
        traj_run<DEPO, TRAJ, kTrajLdsNS>(a, sp, (const double *)s_coef, i, x, N, steps, st);
    } else {
        if (!live) return;
        traj_run<DEPO, TRAJ, kNF>(a, sp, (const double *)a.coef, i, x, N, steps, st);
    }
}

template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64, TORJ_TRAJ_WAVES) k_traj(TraceArgs a, SplitArgs sp) {
    traj_body<DEPO, TRAJ, kTrajL2>(a, sp);
}
#ifndef TORJ_TRAJ_LDS_WAVES
#define TORJ_TRAJ_LDS_WAVES 1
#endif
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(512, TORJ_TRAJ_LDS_WAVES) k_traj_lds(TraceArgs a, SplitArgs sp) {
    traj_body<DEPO, TRAJ, kTrajLds>(a, sp);
}
#ifndef TORJ_TRAJ_TILE_WAVES
#define TORJ_TRAJ_TILE_WAVES 2
#endif
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64, TORJ_TRAJ_TILE_WAVES) k_traj_tile(TraceArgs a, SplitArgs sp) {
    traj_body<DEPO, TRAJ, kTrajTile>(a, sp);
}
// measurement knob: a VGPR budget for the cell kernel between the 2- and 3-wave
// bounds (176: two trajectory waves and two 80-VGPR alpha waves share a SIMD)
#ifdef TORJ_TRAJ_CELL_VGPR
#define TORJ_TRAJ_CELL_ATTR __attribute__((amdgpu_num_vgpr(TORJ_TRAJ_CELL_VGPR)))
#else
#define TORJ_TRAJ_CELL_ATTR
#endif
#if defined(TORJ_TRAJ_TU) || !TORJ_TRAJ_OWN_TU
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64, TORJ_TRAJ_TILE_WAVES) TORJ_TRAJ_CELL_ATTR k_traj_cell(TraceArgs a, SplitArgs sp) {
    traj_body<DEPO, TRAJ, kTrajCell>(a, sp);
}
#else
// defined and instantiated in torj_traj.hip (its own compile flags, above)
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64, TORJ_TRAJ_TILE_WAVES) TORJ_TRAJ_CELL_ATTR k_traj_cell(TraceArgs a, SplitArgs sp);
#endif

#ifndef TORJ_TRAJ_TU  // the rest of the library (torj_traj.hip stops here)

// alpha at the stored stage points of one block: block = kAlphaBlock lanes
// (TORJ_ALPHA_BLOCK, default 128: two groups of 64 rays) at one (step j,
// stage); lanes of rays the trajectory did not
// reach this step with (or the scan has stopped) sit out, as in the fused wave
// (a measured alternative -- harmonic 2 in a second pass over a compacted list
// of the points needing it -- executed more instructions in total: the points
// needing harmonic 2 cluster in whole waves)
// COUNT: a counted launch (sp.awork set) -- the work words are written; an
// uncounted one carries no work struct at all (with its address taken
// conditionally it lived in scratch: 32 B of stores per lane and point, ~25 GB
// per headline launch)
#ifndef TORJ_ALPHA_BLOCK
#define TORJ_ALPHA_BLOCK 128  // lanes per alpha workgroup (groups of 64 rays at one (step, stage)): two
// waves, placed beside the trajectory waves SIMD pair by SIMD pair (256: 47.4-47.8 ms
// trace phase, 128: 45.6-45.7, 64: 46.7-48.6 alternating)
#endif
constexpr int kAlphaBlock = TORJ_ALPHA_BLOCK;
#ifndef TORJ_ALPHA_SETPRIO
#define TORJ_ALPHA_SETPRIO 0
#endif
template <bool COUNT>
__global__ void __launch_bounds__(kAlphaBlock, TORJ_ALPHA_WAVES) k_alpha_pts(TraceArgs a, SplitArgs sp, int nq) {
#if TORJ_ALPHA_SETPRIO
    __builtin_amdgcn_s_setprio(TORJ_ALPHA_SETPRIO);  // measurement knob: the alpha waves' issue priority
#endif
    const int q = blockIdx.x, js = blockIdx.y;  // js = j * 4 + stage (a 2-D grid: no division)
    const int i = q * kAlphaBlock + threadIdx.x;
    if (i >= a.n) return;
    const int j = js >> 2;
    // the stop words and the block's zero flag first
    const int ti = sp.tinfo[i], si = sp.sinfo[i];
    const int zf = sp.zflag ? sp.zflag[i] : 0;
    // the trajectory kernel's block zero flags: a wave whose rays all carry one
    // writes 0 (abs_albajar_fast_body's early settle returns +0 there) and ends
    // before its input loads are issued (round 6: waiting for the five inputs
    // too, as below, cost the flagged 39 % of the waves a memory latency and
    // ~12 GB of reads per launch; C3 trace -1.2 ms alternating,
    // profiles/r06/ab_log.txt r6zff)
    if (__all(zf != 0)) {
#if defined(TORJ_ALPHA_PROF) && defined(__HIP_DEVICE_COMPILE__)
        TORJ_APROF_WAVE(kAprofZ);
#endif
        sp.alpha[(size_t)js * a.n + i] = sp.zval;
        if constexpr (COUNT) sp.awork[(size_t)js * a.n + i] = 0u;
        return;
    }
    // the five inputs at once (one memory latency, not three in a row; their
    // addresses are valid for any i < n whether or not the point is live)
    const double *in = sp.ain + (size_t)js * sp.nf * a.n + i;
    const double X = in[0], Y = in[(size_t)a.n], N2 = in[2 * (size_t)a.n], Npar = in[3 * (size_t)a.n];
    const double lnTe = in[4 * (size_t)a.n];
    // (an empty asm that consumes them: the compiler would otherwise sink the
    // input loads below the stop test and the Te test, three latencies in a row)
    asm volatile("" ::"v"(ti), "v"(si), "v"(X), "v"(Y), "v"(N2), "v"(Npar), "v"(lnTe));
    // sinfo may be stale (k_tau_scan of an earlier block runs on another
    // stream): an optimisation only, as in traj_body -- a stale OK evaluates an
    // alpha the scan never reads
    if (sp.k0 + j >= info_steps(ti) || info_status(si) != ST_OK) return;
#if defined(TORJ_ALPHA_PROF) && defined(__HIP_DEVICE_COMPILE__)
    {
        // [14]: the live lanes of these (not fully flagged) waves that carry a
        // zero flag -- what compacting the unflagged points into full waves would save
        const unsigned long long am = __ballot(1), zm = __ballot(zf != 0);
        if ((int)__lane_id() == __builtin_ffsll((long long)am) - 1) {
            atomicAdd(&g_aprof[4], 1ull);
            atomicAdd(&g_aprof[5], (unsigned long long)__popcll(am));
            atomicAdd(&g_aprof[14], (unsigned long long)__popcll(zm));
        }
    }
#endif
    const double Nabs = TORJ_AIN_TRAJ_MATH ? N2 : sqrt_pos(N2), Te = TORJ_AIN_TRAJ_MATH ? lnTe : exp_fast<true>(lnTe);
    if constexpr (COUNT) {
        AlbajarWork work = {};
        sp.alpha[(size_t)js * a.n + i] = abs_albajar_fast_body<1, TORJ_ALPHA_UNROLL>(
            c_gl, a.omega, X, Y, Nabs, Npar, Te, a.mode, &work, 0, c_gl.tiny_alpha);
        sp.awork[(size_t)js * a.n + i] = (work.n_active & 1u) | ((work.n_harm & 3u) << 1) |
                                     ((work.n_zero & 3u) << 3) | (min(work.n_terms, 2047u) << 5) |
                                     ((work.n_negl & 3u) << 16) | ((work.n_early & 3u) << 18);
    } else {
        sp.alpha[(size_t)js * a.n + i] = abs_albajar_fast_body<1, TORJ_ALPHA_UNROLL>(
            c_gl, a.omega, X, Y, Nabs, Npar, Te, a.mode, nullptr, 0, c_gl.tiny_alpha);
    }
}

// k_alpha_pts with each workgroup taking P consecutive (step, stage) points of
// its rays (TORJ_ALPHA_PPW = P > 1, a measurement variant): the kernel's per-wave
// setup (arguments, the 2-D index, the rays' stop words) once per P points, and
// the next point's five inputs loaded while the current one is evaluated.  The
// lanes of a wave at one point are the same rays as k_alpha_pts' wave there, so
// the Bessel-level ballot and every alpha are the same bits.
#ifndef TORJ_ALPHA_PPW
#define TORJ_ALPHA_PPW 1
#endif
#ifndef TORJ_ALPHA_PREFETCH
#define TORJ_ALPHA_PREFETCH 1
#endif
template <bool COUNT, int P>
__global__ void __launch_bounds__(kAlphaBlock, TORJ_ALPHA_WAVES) k_alpha_pts_mp(TraceArgs a, SplitArgs sp, int nq) {
    const int i = blockIdx.x * kAlphaBlock + threadIdx.x;
    if (i >= a.n) return;
    const int js0 = blockIdx.y * P;
    const int np = min(P, 4 * sp.kb - js0);  // workgroup-uniform
    const int ti = sp.tinfo[i], si = sp.sinfo[i];
    // the ray's last stored point + 1 (0 when the scan has stopped it: sinfo may
    // be stale, an optimisation only, as in k_alpha_pts)
    const int js_end = info_status(si) != ST_OK ? 0 : 4 * (info_steps(ti) - sp.k0);
    const size_t n = (size_t)a.n, stride = (size_t)sp.nf * n;
    const double *in = sp.ain + (size_t)js0 * stride + i;
    double X = in[0], Y = in[n], N2 = in[2 * n], Npar = in[3 * n], lnTe = in[4 * n];
    for (int p = 0; p < np; p++) {
        const int js = js0 + p;
        // the quadrature table's address laundered per point: its loads (and the
        // address arithmetic) stay inside the loop instead of being hoisted into
        // registers live across the whole body (hundreds of SGPR spills otherwise)
        const GLTable *glp = &c_gl;
        asm volatile("" : "+s"(glp));
#if TORJ_ALPHA_PREFETCH
        double Xn = 0.0, Yn = 0.0, N2n = 0.0, Nparn = 0.0, lnTen = 0.0;
        if (p + 1 < np) {  // the next point's inputs in flight during this one
            const double *nx = in + (size_t)(p + 1) * stride;
            Xn = nx[0], Yn = nx[n], N2n = nx[2 * n], Nparn = nx[3 * n], lnTen = nx[4 * n];
        }
#endif
        if (js < js_end) {
            const double Nabs = TORJ_AIN_TRAJ_MATH ? N2 : sqrt_pos(N2),
                         Te = TORJ_AIN_TRAJ_MATH ? lnTe : exp_fast<true>(lnTe);
            if constexpr (COUNT) {
                AlbajarWork work = {};
                sp.alpha[(size_t)js * n + i] = abs_albajar_fast_body<1, TORJ_ALPHA_UNROLL>(
                    *glp, a.omega, X, Y, Nabs, Npar, Te, a.mode, &work, 0, glp->tiny_alpha);
                sp.awork[(size_t)js * n + i] = (work.n_active & 1u) | ((work.n_harm & 3u) << 1) |
                                               ((work.n_zero & 3u) << 3) | (min(work.n_terms, 2047u) << 5) |
                                               ((work.n_negl & 3u) << 16) | ((work.n_early & 3u) << 18);
            } else {
                sp.alpha[(size_t)js * n + i] = abs_albajar_fast_body<1, TORJ_ALPHA_UNROLL>(
                    *glp, a.omega, X, Y, Nabs, Npar, Te, a.mode, nullptr, 0, glp->tiny_alpha);
            }
        }
#if TORJ_ALPHA_PREFETCH
        X = Xn, Y = Yn, N2 = N2n, Npar = Nparn, lnTe = lnTen;
#else
        if (p + 1 < np) {
            const double *nx = in + (size_t)(p + 1) * stride;
            X = nx[0], Y = nx[n], N2 = nx[2 * n], Npar = nx[3 * n], lnTe = nx[4 * n];
        }
#endif
    }
}

// the warm alpha (absorption 2 / 3, iwarm 1 / 3) at the stored stage points:
// the same points and lanes as k_alpha_pts, with the group-velocity factor
// stored by the trajectory kernel as the sixth input.  Without a ray's state
// and step chain the heavy warm code has the registers to itself
// (waves per SIMD: iwarm 1 two -- 221 ms fused, 235 at one wave, 166 at two on
// the C5 beam; iwarm 3 one -- 20.4 s, 22.2 s at two).
#ifndef TORJ_WARM1_ALPHA_WAVES
#define TORJ_WARM1_ALPHA_WAVES 2
#endif
#ifndef TORJ_WARM3_ALPHA_WAVES
#define TORJ_WARM3_ALPHA_WAVES 1
#endif
#ifndef TORJ_ALPHA_WARM_BLOCK
#define TORJ_ALPHA_WARM_BLOCK 64  // lanes per warm-alpha workgroup (C5: 139.3 ms against 142.6-143.2
// at 128 and 149.0 at 256, alternating)
#endif
constexpr int kAlphaWarmBlock = TORJ_ALPHA_WARM_BLOCK;
// COUNT: a counted launch (sp.awork set) stores the work word; without it the
// trip counts are dead and the compiler drops their arithmetic
template <bool COUNT>
__device__ __forceinline__ void warm_store(const SplitArgs &sp, int js, int i, int n, const WarmAlpha &r) {
    sp.alpha[(size_t)js * n + i] = r.alpha;
    if constexpr (COUNT)
        sp.awork[(size_t)js * n + i] = (unsigned)min(r.nasym, 127) | ((unsigned)min(r.nfad, 127) << 7) |
                                   ((unsigned)min(r.passes, 127) << 14) | ((unsigned)r.lrm << 21);
}
template <int IWARM, bool COUNT>
__global__ void __launch_bounds__(kAlphaWarmBlock, IWARM == 1 ? TORJ_WARM1_ALPHA_WAVES : TORJ_WARM3_ALPHA_WAVES)
    k_alpha_warm_pts(TraceArgs a, SplitArgs sp, int nq) {
    const int q = blockIdx.x, js = blockIdx.y;  // js = j * 4 + stage
    const int i = q * kAlphaWarmBlock + threadIdx.x;
    if (i >= a.n) return;
    const int j = js >> 2;
    // every load of the point at once (as k_alpha_pts)
    const int ti = sp.tinfo[i], si = sp.sinfo[i];
    const double *in = sp.ain + (size_t)js * kAinFW * a.n + i;
    const double X = in[0], Y = in[(size_t)a.n], Nabs = in[2 * (size_t)a.n], Npar = in[3 * (size_t)a.n];
    const double Te = in[4 * (size_t)a.n], inv = in[5 * (size_t)a.n];
    asm volatile("" ::"v"(ti), "v"(si), "v"(X), "v"(Y), "v"(Nabs), "v"(Npar), "v"(Te), "v"(inv));
    if (sp.k0 + j >= info_steps(ti) || info_status(si) != ST_OK) return;
#if defined(TORJ_WARM_PROF) && defined(__HIP_DEVICE_COMPILE__)
    static_assert(kAlphaWarmBlock == 64, "region timers: one wave per workgroup");
    wprof_init();
#endif
    const WarmSetup w = warm_setup(Y, Nabs, Npar, Te);
    // a point with lrm > 3 (~0.1 % of the C5 beam's) goes to k_alpha_warm_big:
    // this kernel then holds the lrm <= 3 tensor only (its registers, and so
    // the waves per SIMD, are sized for that), and no wave runs the lrm <= 5
    // code for all its lanes because one of them needs it
    const bool big = w.lrm > sp.defer_lrm;
    const unsigned long long bmask = __ballot(big);
    if (bmask) {  // wave-aggregated append
        const int lane = (int)__lane_id(), lead = __builtin_ffsll((long long)bmask) - 1;
        unsigned base = 0;
        if (lane == lead) base = atomicAdd(sp.defer_cnt, (unsigned)__popcll(bmask));
        base = __shfl(base, lead);
        if (big)
            sp.defer[base + __popcll(bmask & ((1ull << lane) - 1))] =
                ((unsigned long long)js << 32) | (unsigned)i;
    }
    if (big) return;
    const WarmAlpha r = alpha_warm_l<IWARM, 3>(a.omega, X, Y, Npar, w, inv, a.mode);
    warm_store<COUNT>(sp, js, i, a.n, r);
#if defined(TORJ_WARM_PROF) && defined(__HIP_DEVICE_COMPILE__)
    TORJ_WPROF(6);  // the stores
    wprof_flush();
#endif
}

// the points k_alpha_warm_pts deferred (lrm > 3), with the lrm <= 5 tensor;
// after it on the same stream, a fixed grid striding over the block's list
#ifndef TORJ_WARM_BIG_GRID
#define TORJ_WARM_BIG_GRID 512  // workgroups of 64: two waves per CU
#endif
template <int IWARM, bool COUNT>
__global__ void __launch_bounds__(64) k_alpha_warm_big(TraceArgs a, SplitArgs sp) {
    const unsigned cnt = *sp.defer_cnt;
    for (unsigned k = blockIdx.x * 64 + threadIdx.x; k < cnt; k += gridDim.x * 64) {
        const unsigned long long e = sp.defer[k];
        const int js = (int)(e >> 32), i = (int)(unsigned)e;
        const double *in = sp.ain + (size_t)js * kAinFW * a.n + i;
        const double Npar = in[3 * (size_t)a.n];
        const WarmSetup w = warm_setup(in[(size_t)a.n], in[2 * (size_t)a.n], Npar, in[4 * (size_t)a.n]);
        const WarmAlpha r = alpha_warm_l<IWARM, kWarmMaxL>(a.omega, in[0], in[(size_t)a.n], Npar, w,
                                                            in[5 * (size_t)a.n], a.mode);
        warm_store<COUNT>(sp, js, i, a.n, r);
    }
}

// RK4 ray_segment from x, N over `k` steps (the NaN-alpha replay) in the
// arithmetic of the trajectory kernel that ran (sp.traj_mode): the same
// cold_step instance -- its stage-0 stencil with psi and its alpha-input
// stores, which change the compiler's fma contraction, here into row j = 0 of
// the ring slot sp.ain (no alpha kernel reads it any more: k_split_final runs
// after the last scan) -- read from the global table its tile falls back to
// (bit for bit the tile's values): the cell power form after k_traj_cell, the
// node tile's fallback after k_traj_tile, the node stencil otherwise (k_traj;
// k_traj_lds reads the same values from LDS, in a separately compiled kernel)
__device__ void cold_replay(const TraceArgs &a, const SplitArgs &sp, int i, double x[3], double N[3], int k) {
    const TileCell cg{a.cellp, nullptr, 0, 0, 0, 0};
    const TileCoef ng{a.coef, nullptr, 0, 0, 0, 0};
    ZBox zb;  // (unused: the replay stores no zero flags)
    for (int s = 0; s < k; s++) {
        double xn[3], Nn[3], psi;
        if (sp.traj_mode == kTrajCell)
            cold_step<true, kTileNS, TileCell, true>(a, cg, sp, 0, i, x, N, xn, Nn, &psi, zb, false);
        else if (sp.traj_mode == kTrajTile)
            cold_step<true, kTileNS, TileCoef, true>(a, ng, sp, 0, i, x, N, xn, Nn, &psi, zb, false);
        else
            cold_step<true, kNF, const double *, true>(a, a.coef, sp, 0, i, x, N, xn, Nn, &psi, zb, false);
#pragma unroll
        for (int c = 0; c < 3; c++) {
            x[c] = xn[c];
            N[c] = Nn[c];
        }
    }
}

// COUNT: a counted launch (work words and counters); the uncounted scan
// carries neither the accumulators nor their loads (fewer registers beside the
// alpha waves it shares the SIMDs with)
template <int DEPO, bool TRAJ, bool COUNT>
__device__ __forceinline__ void tau_scan_body(const TraceArgs &a, const SplitArgs &sp) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    // counters [2..7] (include/torj_hip.h): Albajar or warm iwarm 1 meanings
    unsigned long long nsteps = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
    const int am = a.abs_model;
    if (i < a.n) {
        int steps = 0, st = ST_OK;
        double tau = 0.0, psi_a = 0.0, Pdep = 0.0;
        if (sp.k0 > 0) {
            const int v = sp.sinfo[i];
            steps = info_steps(v);
            st = info_status(v);
            tau = sp.stau[i];
            Pdep = sp.sPdep[i];
        }
        if constexpr (DEPO == kDepoBinned) psi_a = sp.spsi[i];
        if (st == ST_OK) {
            const int tv = sp.tinfo[i];  // packed: steps and status written together
            const int tT = info_steps(tv), tS = info_status(tv);
            const double w = (DEPO == kDepoBinned && a.w) ? a.w[i] : 1.0;
            const double ds6 = a.ds / 6.0;
            double P = exp(-tau);  // bitwise the value the previous step computed
            DepoAcc dacc = {-1, 0.0};
            const int s_end = min(a.n_steps, sp.k0 + sp.kb);
            // the steps' alphas are loaded kScanBatch steps at a time (one memory
            // latency per batch instead of one per step: the scan is a serial
            // chain per lane); the loads stay inside the block's ring slot
            constexpr int kScanBatch = 4;
            bool done = false;
            for (int sb = steps; sb < s_end && !done; sb += kScanBatch) {
                double alb[kScanBatch][4];
#pragma unroll
                for (int v = 0; v < kScanBatch; v++) {
                    const size_t ov = (size_t)(min(sb + v, s_end - 1) - sp.k0) * 4 * a.n + i;
#pragma unroll
                    for (int q = 0; q < 4; q++) alb[v][q] = sp.alpha[ov + q * (size_t)a.n];
                }
#pragma unroll
                for (int v = 0; v < kScanBatch; v++) {
                    const int s = sb + v;
                    if (s >= s_end) break;
                    if (s >= tT) {  // the trajectory stopped before step s
                        if (tS == ST_NAN) st = ST_NAN;  // non-finite x / N at step s (ray_segment's `bad`)
                        done = true;
                        break;
                    }
                    const size_t o = (size_t)(s - sp.k0) * 4 * a.n + i;
                    const double al0 = (s == sp.nan_step && i % 3 == 0) ? (double)NAN : alb[v][0];
                    const double al1 = alb[v][1], al2 = alb[v][2], al3 = alb[v][3];
                    double acc_a = fma(1.0, al0, 0.0);
                    acc_a = fma(2.0, al1, acc_a);
                    acc_a = fma(2.0, al2, acc_a);
                    acc_a = fma(1.0, al3, acc_a);
                    const double taun = tau + ds6 * acc_a;
                    if (!isfinite(taun)) {  // alpha went non-finite: NAN at step s, state x_s
                        st = ST_NAN | 0x40;  // internal: the final state needs the replay
                        done = true;
                        break;
                    }
#pragma unroll
                    for (int q = 0; q < 4 && COUNT; q++) {
                        const unsigned wk = sp.awork[o + q * (size_t)a.n];
                        if (am == 1) {
                            c2 += wk & 1u;
                            c3 += (wk >> 1) & 3u;
                            c5 += (wk >> 3) & 3u;
                            c4 += (wk >> 5) & 2047u;
                            c6 += (wk >> 16) & 3u;
                            c7 += (wk >> 18) & 3u;
                        } else if (am == 2) {
                            const unsigned lrm = wk >> 21, passes = (wk >> 14) & 127u;
                            c2 += wk & 127u;
                            c3 += (wk >> 7) & 127u;
                            c4 += passes;
                            c5 += passes * lrm;
                            c6 += lrm;
                            c7 += lrm * lrm;
                        }
                    }
                    const double Pn = exp(-taun);
                    const double dP = P - Pn;
                    if constexpr (DEPO == kDepoSamples) {
                        if (s > 0) a.smp_dpds[smp_at(s, i, a.smp_rows)] = P * al0;
                    }
                    tau = taun;
                    P = Pn;
                    steps = s + 1;
                    nsteps++;
                    if constexpr (DEPO == kDepoBinned) {
                        const double psi_b = sp.psib[(size_t)(s - sp.k0) * a.n + i];
                        Pdep += deposit(a, dacc, psi_a, psi_b, dP, w);
                        psi_a = psi_b;
                    }
                    if constexpr (TRAJ) {
                        if (a.traj_stride > 0 && (steps % a.traj_stride) == 0)
                            a.traj[((size_t)(steps / a.traj_stride - 1) * 5 + 3) * a.n + i] = tau;
                    }
                    if (steps == tT && tS == ST_LEFT_PLASMA) {  // psi check first (src/solve.jl:174)
                        st = ST_LEFT_PLASMA;
                        done = true;
                        break;
                    }
                    if (a.chunk_steps > 0 && (steps % a.chunk_steps) == 0 && P < a.P_min) {  // :176
                        st = ST_ABSORBED;
                        done = true;
                        break;
                    }
                }
            }
            if constexpr (DEPO == kDepoBinned) depo_flush(a, dacc);
            sp.stau[i] = tau;
            sp.sPdep[i] = Pdep;
            if constexpr (DEPO == kDepoBinned) sp.spsi[i] = psi_a;
            sp.sinfo[i] = make_info(steps, st);
        }
    }
    if (COUNT) {
        const unsigned long long s0 = wave_sum(nsteps), s2 = wave_sum(c2), s3 = wave_sum(c3),
                                 s4 = wave_sum(c4), s5 = wave_sum(c5), s6 = wave_sum(c6),
                                 s7 = wave_sum(c7);
        if (threadIdx.x == 0) {
            atomicAdd(a.counters + 0, s0);
            atomicAdd(a.counters + 1, 4ull * s0);
            atomicAdd(a.counters + 2, s2);
            atomicAdd(a.counters + 3, s3);
            atomicAdd(a.counters + 4, s4);
            atomicAdd(a.counters + 5, s5);
            atomicAdd(a.counters + 6, s6);
            atomicAdd(a.counters + 7, s7);
        }
    }
}
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64) k_tau_scan(TraceArgs a, SplitArgs sp) {
    tau_scan_body<DEPO, TRAJ, false>(a, sp);
}
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64) k_tau_scan_counted(TraceArgs a, SplitArgs sp) {
    tau_scan_body<DEPO, TRAJ, true>(a, sp);
}

// final state, status and steps; trajectory samples past an earlier scan stop
template <int DEPO, bool TRAJ>
__global__ void __launch_bounds__(64) k_split_final(TraceArgs a, SplitArgs sp) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const int sv = sp.sinfo[i], tv = sp.tinfo[i];
    const int steps = info_steps(sv), tT = info_steps(tv);
    int st = info_status(sv);
    double x[3], N[3];
    if (steps == tT && !(st & 0x40)) {  // the scan ran to the trajectory's end: its carry
#pragma unroll
        for (int c = 0; c < 3; c++) {
            x[c] = sp.tx[c * (size_t)a.n + i];
            N[c] = sp.tx[(3 + c) * (size_t)a.n + i];
        }
    } else {  // stopped earlier: from the chunk-boundary state (+ replay to step `steps`)
        const int cs = a.chunk_steps > 0 ? a.chunk_steps : 1 << 30;
        const int c0 = a.chunk_steps > 0 ? steps / cs : 0;
        const double *cb = sp.cbx + (size_t)c0 * 6 * a.n + i;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            x[c] = cb[c * (size_t)a.n];
            N[c] = cb[(3 + c) * (size_t)a.n];
        }
        cold_replay(a, sp, i, x, N, steps - c0 * (a.chunk_steps > 0 ? cs : 0));
        if constexpr (TRAJ) {  // samples the trajectory wrote past the stop
            if (a.traj_stride > 0)
                for (int k = steps / a.traj_stride; k < min(tT, a.n_steps) / a.traj_stride; k++)
                    for (int r = 0; r < 5; r++) a.traj[((size_t)k * 5 + r) * a.n + i] = NAN;
        }
    }
    st &= 0x3f;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        a.state[c * a.n + i] = x[c];
        a.state[(3 + c) * a.n + i] = N[c];
    }
    a.state[6 * a.n + i] = sp.stau[i];
    a.status[i] = st;
    a.steps[i] = steps;
    const double Pdep = sp.sPdep[i];
    if (a.Pdep) a.Pdep[i] = Pdep;
    if constexpr (DEPO == kDepoBinned) {
        const double w = a.w ? a.w[i] : 1.0;
        atomicAdd(a.dP + a.n_psi, w * Pdep);  // sum_rays w P_dep
    }
}

// ---------------------------------------------------------------------------
// GPU ray entry (src/solve.jl:7-74): one lane per ray.  The bisection to the
// psi_prof_max surface runs ~55 spline evaluations per lane; lanes of a wave
// take nearly the same number, so 64-lane blocks keep divergence low.
// ---------------------------------------------------------------------------
struct EntryArgs {
    const double *coef;
    Grid g;
    double psi_max, omega;
    int mode, n;
    const double *x0, *N0;
    double *xp, *Np, *s0;
    int *status;
};

__global__ void __launch_bounds__(64) k_ray_entry(EntryArgs a) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const double x0[3] = {a.x0[i], a.x0[a.n + i], a.x0[2 * a.n + i]};
    const double N0[3] = {a.N0[i], a.N0[a.n + i], a.N0[2 * a.n + i]};
    double xo[3], No[3], s0;
    const int st = ray_entry_one(a.coef, a.g, a.psi_max, x0, N0, a.omega, a.mode, xo, No, s0);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        a.xp[k * a.n + i] = xo[k];
        a.Np[k * a.n + i] = No[k];
    }
    a.s0[i] = s0;
    a.status[i] = st;
}

// dP/ds at a ray's last saved point (every other point's alpha is the next
// step's stage-0 RHS inside the trace kernel): P alpha_approx(x, N) from the
// final state (src/solve.jl:171)
template <int ABS>
__global__ void __launch_bounds__(64) k_final_alpha(TraceArgs a) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const int k = a.steps[i];
    if (k <= 0) return;
    double x[3], N[3], du[6], al = 0.0;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        x[c] = a.state[c * a.n + i];
        N[c] = a.state[(3 + c) * a.n + i];
    }
    if constexpr (ABS != 0) ray_rhs_m<ABS>(a.coef, a.g, a.k, c_gl, a.omega, a.mode, a.abs_model, x, N, du, al, nullptr);
    a.smp_dpds[smp_at(k, i, a.smp_rows)] = exp(-a.state[6 * a.n + i]) * al;
}

// ---------------------------------------------------------------------------
// Reference-faithful deposition (torj_fitdepo.hpp): one lane per ray
// ---------------------------------------------------------------------------
// boundaries up to this many are staged in LDS by k_fit_depo (32 KB per wave)
constexpr int kFitGridLds = 4096;

__global__ void __launch_bounds__(64, 2) k_fit_depo(FitArgs a) {
    // the walk's boundary lookups (cursor moves, root levels) form serial
    // dependency chains: LDS latency instead of L2 latency on each
    extern __shared__ double s_grid[];
    if (a.n_psi <= kFitGridLds) {
        for (int k = threadIdx.x; k < a.n_psi; k += 64) s_grid[k] = a.grid[k];
        __syncthreads();
        a.grid = s_grid;
    }
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const double xl[3] = {a.x_launch[i], a.x_launch[a.n + i], a.x_launch[2 * a.n + i]};
    fit_depo_ray<kOpenCache>(a, i, psi_at(a.coef, a.g, xl));
}
// the streamed deposition (torj_fitdepo.hpp): windows of the walk behind the
// split pipeline's scan (S = the scan's steps of a still-running ray), then the
// rest of every ray after the trace
__device__ __forceinline__ bool fit_grid_lds(FitArgs &a) {
    extern __shared__ double s_grid[];
    if (a.n_psi > kFitGridLds) return false;
    for (int k = threadIdx.x; k < a.n_psi; k += 64) s_grid[k] = a.grid[k];
    __syncthreads();
    a.grid = s_grid;
    return true;
}
// The windows' gate: a ray still running (a stopped one is k_depo_tail's),
// S = its scanned steps capped at s_cap, a new window ready; psi at the launch
// point (point 0) only for the walk's start.  s_cap: the steps whose samples
// this launch may read (the end of the block whose scan it follows).  On its
// own stream (TORJ_DEPO_STREAM=2) the launch can overlap the next block's
// scan, so sinfo may already hold that scan's carry, whose samples need not
// be visible yet: S is capped at the block end (and a ray that scan stopped is
// left to k_depo_tail).  Windows are schedule-independent (torj_fitdepo.hpp),
// so the outputs do not depend on which carry the read saw.
__device__ __forceinline__ bool depo_stream_gate(const FitArgs &a, const DepoStream &ds, const int *sinfo,
                                                 int s_cap, int i, int &S, double &psiL) {
    const int v = __hip_atomic_load(sinfo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (info_status(v) != ST_OK) return false;
    S = min(info_steps(v), s_cap);
    const int j = ds.v[kDsJ * (size_t)a.n + i];
    if ((j < 0 ? 0 : j) + kDepoQ + 3 + kDepoW > S) return false;  // no new window yet
    psiL = 0.0;
    if (j < 0) {
        const double xl[3] = {a.x_launch[i], a.x_launch[a.n + i], a.x_launch[2 * a.n + i]};
        psiL = psi_at(a.coef, a.g, xl);
    }
    return true;
}
__global__ void __launch_bounds__(64, 2) k_depo_stream(FitArgs a, DepoStream ds, const int *sinfo, int s_cap) {
    fit_grid_lds(a);
    const int i = blockIdx.x * 64 + threadIdx.x;
    int S;
    double psiL;
    if (i >= a.n || !depo_stream_gate(a, ds, sinfo, s_cap, i, S, psiL)) return;
    fit_depo_stream(a, ds, i, psiL, S);
}
// TORJ_DEPO_STREAM=3: a window's elimination and walk as two launches
// (torj_fitdepo.hpp fit_depo_stream_elim / _walk), the same S and gating
#ifndef TORJ_DEPO_ELIM_WAVES
#define TORJ_DEPO_ELIM_WAVES 4
#endif
__global__ void __launch_bounds__(64, TORJ_DEPO_ELIM_WAVES) k_depo_elim(FitArgs a, DepoStream ds, const int *sinfo,
                                                                        int s_cap) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    int S;
    double psiL;
    if (i >= a.n || !depo_stream_gate(a, ds, sinfo, s_cap, i, S, psiL)) return;
    fit_depo_stream_elim(a, ds, i, psiL, S);
}
#ifndef TORJ_DEPO_WALK_WAVES
#define TORJ_DEPO_WALK_WAVES 3  // 168 VGPRs at kWalkChunkStream = 1, no spill
#endif
__global__ void __launch_bounds__(64, TORJ_DEPO_WALK_WAVES) k_depo_walk(FitArgs a, DepoStream ds, const int *sinfo,
                                                                        int s_cap) {
    fit_grid_lds(a);
    const int i = blockIdx.x * 64 + threadIdx.x;
    int S;
    double psiL;
    if (i >= a.n || !depo_stream_gate(a, ds, sinfo, s_cap, i, S, psiL)) return;
    fit_depo_stream_walk(a, ds, i, psiL, S);
}
__global__ void __launch_bounds__(64, 2) k_depo_tail(FitArgs a, DepoStream ds) {
    fit_grid_lds(a);
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const double xl[3] = {a.x_launch[i], a.x_launch[a.n + i], a.x_launch[2 * a.n + i]};
    fit_depo_tail(a, ds, i, psi_at(a.coef, a.g, xl));
}
// torj_power_deposition_profile: the caller's vectors of ray i (points off[i] ..
// off[i] + npts[i] - 1) into the fit's per-point rows, psi(s_j) from the psi
// spline at x_j (src/plasma.jl:95-98: psi_norm_spline(hypot(x, y), z))
__global__ void __launch_bounds__(64) k_profile_samples(FitArgs a, const long *off, const double *s,
                                                        const double *x, size_t n_all, const double *dpds) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    for (int j = 0; j < a.npts[i]; j++) {
        const size_t q = (size_t)off[i] + j;
        const double xq[3] = {x[q], x[n_all + q], x[2 * n_all + q]};
        const size_t o = smp_at(j, i, a.rows);
        // (FitArgs holds the sample rows read-only for the fit; this kernel fills them)
        const_cast<double *>(a.smp_psi)[o] = psi_at(a.coef, a.g, xq);
        const_cast<double *>(a.smp_dpds)[o] = dpds[q];
        const_cast<double *>(a.smp_s)[o] = s[q];
    }
}
__global__ void __launch_bounds__(64, 2) k_fit_profile(FitArgs a) {
    extern __shared__ double s_grid[];
    if (a.n_psi <= kFitGridLds) {
        for (int k = threadIdx.x; k < a.n_psi; k += 64) s_grid[k] = a.grid[k];
        __syncthreads();
        a.grid = s_grid;
    }
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    fit_depo_ray<kOpenCache>(a, i, 0.0);
}
// a work-queue launch's outcome into the handle's sticky flags (bit 1 stall
// watchdog, bit 2 not every group retired); read by torj_trace_check
__global__ void k_sched_fold(const SchedCtl *ctl, unsigned G, int *flags) {
    int f = 0;
    if (ctl->err) f |= 2;
    if (ctl->finished != G) f |= 4;
    if (f) atomicOr(flags, f);
}
// psi_dP_dV strictly increasing (the shell lookups assume it)
__global__ void __launch_bounds__(256) k_grid_check(const double *grid, int n, int *flags) {
    bool bad = false;
    for (int k = threadIdx.x + 1; k < n; k += 256) bad |= !(grid[k] > grid[k - 1]);
    if (bad) atomicOr(flags, 1);
}

__global__ void __launch_bounds__(256) k_shell_sum(FitArgs a) {
    const int k = blockIdx.x;
    double acc = 0.0;
    // each thread's rays i, i + 256, ... in order, their loads eight at a time
    // (one memory latency per eight rays instead of one per ray; the same sum)
    constexpr int kB = 8;
    const bool shell = k < a.n_psi - 1;
    const double *row = shell ? a.dPs + (size_t)k * a.n : a.Pray;
    for (int i0 = threadIdx.x; i0 < a.n; i0 += 256 * kB) {
        double v[kB], wv[kB];
        bool on[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int i = i0 + 256 * u;
            on[u] = i < a.n;
            v[u] = on[u] ? row[i] : 0.0;
            wv[u] = on[u] && a.w ? a.w[i] : 1.0;
            if (shell && on[u]) on[u] = k > a.kstar[i];
        }
#pragma unroll
        for (int u = 0; u < kB; u++)
            if (on[u]) acc += wv[u] * v[u];
    }
    __shared__ double red[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = (red[0] + red[1]) + (red[2] + red[3]);
        a.dP[k < a.n_psi - 1 ? k : a.n_psi] += t;
    }
}

struct EvalArgs {
    const double *coef;
    Grid g;
    Consts k;
    double omega;
    int mode;
    int n;
    const double *x, *N;
    double *out;
    double *D, *du, *alpha;
};

__global__ void __launch_bounds__(256, 1) k_eval_plasma(EvalArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    double x[3], N[3];
    for (int c = 0; c < 3; c++) {
        x[c] = a.x[c * a.n + i];
        N[c] = a.N[c * a.n + i];
    }
    PlasmaPoint p;
    plasma_point<true>(a.coef, a.g, a.k, x, p);
    const double R = sqrt(x[0] * x[0] + x[1] * x[1]);
    double *o = a.out;
    const size_t n = a.n;
    o[0 * n + i] = p.B[0];
    o[1 * n + i] = p.B[1];
    o[2 * n + i] = p.B[2];
    o[3 * n + i] = p.ne;
    o[4 * n + i] = exp(p.lnTe);
    o[5 * n + i] = eval_one(a.coef, a.g, R, x[2], F_PSI);
    o[6 * n + i] = p.X;
    o[7 * n + i] = p.Y;
    o[8 * n + i] = N[0] * p.b[0] + N[1] * p.b[1] + N[2] * p.b[2];
    o[9 * n + i] = p.b[0];
    o[10 * n + i] = p.b[1];
    o[11 * n + i] = p.b[2];
    o[12 * n + i] = p.Babs;
}

template <bool ABS>
__global__ void __launch_bounds__(256, 1) k_dispersion(EvalArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    double x[3], N[3], du[6], alpha;
    for (int c = 0; c < 3; c++) {
        x[c] = a.x[c * a.n + i];
        N[c] = a.N[c * a.n + i];
    }
    PlasmaPoint p;
    plasma_point<ABS>(a.coef, a.g, a.k, x, p);
    double Npar;
    const double D = dispersion_grad(p, N, a.mode, du, &Npar);
    if (a.D) a.D[i] = D;
    if (a.du)
        for (int c = 0; c < 6; c++) a.du[c * a.n + i] = du[c];
    if constexpr (ABS) {
        const double Nabs = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
        alpha = abs_albajar_fast(c_gl, a.omega, p.X, p.Y, Nabs, Npar, exp(p.lnTe), a.mode, nullptr);
        a.alpha[i] = alpha;
    }
}

struct AlbArgs {
    int n, mode;
    const double *omega, *X, *Y, *Nabs, *Npar, *Te;
    double *out;
    const double *inv;  // warm: 1 / |dD/dN|
    double *n2;         // warm: N_perp^2 (re, im interleaved), may be null
    int iwarm;
};

// warm absorption alpha (torj_warm.hpp) at arbitrary points: one lane each
__global__ void __launch_bounds__(64) k_alpha_warm(AlbArgs a) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    cplx n2;
    a.out[i] = alpha_warm(a.omega[i], a.X[i], a.Y[i], a.Nabs[i], a.Npar[i], a.Te[i], a.inv[i],
                          a.mode, a.iwarm, &n2);
    if (a.n2) {
        a.n2[2 * i] = n2.re;
        a.n2[2 * i + 1] = n2.im;
    }
}

__global__ void __launch_bounds__(256, 1) k_albajar(AlbArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    a.out[i] = abs_albajar_fast(c_gl, a.omega[i], a.X[i], a.Y[i], a.Nabs[i], a.Npar[i], a.Te[i],
                                a.mode, nullptr);
}

__global__ void k_refr(AlbArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    a.out[i] = refractive_index_sq(a.X[i], a.Y[i], a.Npar[i], a.mode);
}

// ===========================================================================
// Plasma construction (host), src/plasma.jl:16-58
// ===========================================================================
// Cubic{Line{OnGrid}} prefilter of Interpolations.jl.  The boundary rows
// c0 - 2c1 + c2 = 0 combined with the first interpolation row give c1 = y1
// (same at the far end), leaving a [1 4 1]/6 tridiagonal system for the
// interior coefficients (solved with the Thomas algorithm).
static void bspl1d_prefilter(int n, const double *y, size_t ystride, double *c, size_t cstride) {
    // c has n+2 entries
    auto C = [&](int k) -> double & { return c[(size_t)k * cstride]; };
    auto Y = [&](int k) { return y[(size_t)k * ystride]; };
    C(1) = Y(0);
    C(n) = Y(n - 1);
    const int m = n - 2;  // interior unknowns c_2..c_{n-1}
    if (m > 0) {
        std::vector<double> cp(m), dp(m);
        for (int k = 0; k < m; k++) {
            double r = 6.0 * Y(k + 1);
            if (k == 0) r -= C(1);
            if (k == m - 1) r -= C(n);
            const double den = 4.0 - (k > 0 ? cp[k - 1] : 0.0);
            cp[k] = 1.0 / den;
            dp[k] = (r - (k > 0 ? dp[k - 1] : 0.0)) / den;
        }
        C(m + 1) = dp[m - 1];
        for (int k = m - 2; k >= 0; k--) C(k + 2) = dp[k] - cp[k] * C(k + 3);
    }
    C(0) = 2.0 * C(1) - C(2);
    C(n + 1) = 2.0 * C(n) - C(n - 1);
}

// y: nR x nZ (R fastest) -> c: (nR+2) x (nZ+2) (R fastest)
static void bspl2d_prefilter(int nR, int nZ, const double *y, double *c) {
    const int mR = nR + 2, mZ = nZ + 2;
    std::fill(c, c + (size_t)mR * mZ, 0.0);
    for (int j = 0; j < nZ; j++)
        bspl1d_prefilter(nR, y + (size_t)j * nR, 1, c + (size_t)(j + 1) * mR, 1);
    std::vector<double> row(nZ);
    for (int i = 0; i < mR; i++) {
        for (int j = 0; j < nZ; j++) row[j] = c[(size_t)(j + 1) * mR + i];
        bspl1d_prefilter(nZ, row.data(), 1, c + i, (size_t)mR);
    }
}

static double bspl1d_eval(const std::vector<double> &c, int n, double x1, double xn, double x) {
    const double h = (xn - x1) / (n - 1);
    const double xc = clampd(x, x1, xn);
    const double u = (xc - x1) / h;
    int i = (int)std::floor(u);
    i = std::max(0, std::min(n - 2, i));
    double w[4], dw[4];
    bweights(u - i, w, dw);
    double v = 0, g = 0;
    for (int a = 0; a < 4; a++) {
        v += w[a] * c[i + a];
        g += dw[a] * c[i + a];
    }
    return v + (x - xc) * (g / h);
}

// natural cubic spline through (x, y) evaluated at xq (IMAS.interp1d :cubic;
// parity unpinned -- exact at the nodes, so any interpolant agrees when the
// profile grid is already uniform)
static void natcubic(int n, const double *x, const double *y, int nq, const double *xq,
                     double *yq) {
    std::vector<double> M(n, 0.0);
    if (n >= 3) {
        const int m = n - 2;
        std::vector<double> a(m), b(m), c(m), r(m);
        for (int i = 1; i <= m; i++) {
            const double h0 = x[i] - x[i - 1], h1 = x[i + 1] - x[i];
            a[i - 1] = h0;
            b[i - 1] = 2.0 * (h0 + h1);
            c[i - 1] = h1;
            r[i - 1] = 6.0 * ((y[i + 1] - y[i]) / h1 - (y[i] - y[i - 1]) / h0);
        }
        for (int i = 1; i < m; i++) {
            const double f = a[i] / b[i - 1];
            b[i] -= f * c[i - 1];
            r[i] -= f * r[i - 1];
        }
        M[m] = r[m - 1] / b[m - 1];
        for (int i = m - 1; i >= 1; i--) M[i] = (r[i - 1] - c[i - 1] * M[i + 1]) / b[i - 1];
    }
    for (int q = 0; q < nq; q++) {
        const double t = xq[q];
        const int i = std::max(0, std::min(n - 2, (int)(std::upper_bound(x, x + n, t) - x) - 1));
        if (t == x[i]) {
            yq[q] = y[i];
            continue;
        }
        if (t == x[i + 1]) {
            yq[q] = y[i + 1];
            continue;
        }
        const double h = x[i + 1] - x[i], A = x[i + 1] - t, B = t - x[i];
        yq[q] = M[i] * A * A * A / (6.0 * h) + M[i + 1] * B * B * B / (6.0 * h) +
                (y[i + 1] / h - M[i + 1] * h / 6.0) * B + (y[i] / h - M[i] * h / 6.0) * A;
    }
}

static std::vector<double> uniform_range(double a, double b, int n) {
    std::vector<double> r(n);
    for (int i = 0; i < n; i++) r[i] = a + (b - a) * i / (n - 1.0);
    r[n - 1] = b;
    return r;
}

struct torj_plasma_s {
    int device = 0;
    Grid g{};
    std::vector<double> coef;  // interleaved host copy
    double *d_coef = nullptr;
    double *d_cellp = nullptr;  // per-cell power form of coef (the cell-tiled trajectory kernel)
    int n_vol = 0;
    double v1 = 0, vn = 0;
    std::vector<double> vol_coef;
    double psi_prof_max = 0;
    hipStream_t stream = nullptr;
    void *d_sched = nullptr;  // work-queue control block + ready-queue ring (zeroed per launch)
    size_t sched_cap = 0;
    int sched_mode = -1, sched_waves = 0;  // torj_set_sched
    int lanes_per_ray = 0;                 // one-shot kernel: 0 auto, 1 or 16 forced (torj_set_sched)
    int *d_chunk = nullptr;                // integrator 1: chunks done per ray
    size_t chunk_cap = 0;
    void *d_fit = nullptr;                 // reference-faithful deposition workspace
    size_t fit_cap = 0;
    bool timing = false;                   // torj_timing: HIP events around each phase
    int timing_calls = 0;                  // trace calls recorded since torj_timing(p, 1)
    void *d_batch = nullptr;               // ray-batch staging of torj_trace_device_ex
    size_t batch_cap = 0;
    std::vector<hipEvent_t> ev_pool;       // 3 per recorded call (start, trace end, post end)
    size_t ev_used = 0;
    double *d_ws = nullptr;        // per-ray workspace (P_dep when the caller passes none)
    // sticky launch error flags, ORed by every launch since the last
    // torj_trace_check (which reads and clears them): bit 0 psi grid not
    // strictly increasing, bit 1 work-queue watchdog, bit 2 unretired groups
    int *d_flags = nullptr;
    size_t ws_cap = 0;
    int n_cu = 256;
    std::mutex mu;
    // torj_trace_beam: handles of the same plasma on further devices (replica k
    // on device (device + k) mod count; k = 0 is this handle) and the
    // single-process RCCL communicator over the first nccl_n of them
    std::vector<torj_plasma_s *> replicas;
    std::vector<ncclComm_t> comms;
    // torj_trace_beam's host staging on this replica (beam_worker): one or two
    // shard slots of device buffers and of host buffers (grow-only; pinned up
    // to a budget, pageable above it), the copy stream and the slots' events
    // (upload done, trace done, download done)
    struct BeamStage {
        void *d = nullptr, *h = nullptr;
        size_t d_cap = 0, h_cap = 0;
        bool h_pinned = false;
        hipStream_t sc = nullptr;
        hipEvent_t up[2] = {}, tr[2] = {}, dn[2] = {};
    } stage;
    // torj_timing of the all-reduce of make_beam's reduce (beam_reduce, host
    // clock around the grouped all-reduce and its stream waits)
    double reduce_ms = 0.0;
    int reduce_calls = 0;
    // split RK4 path: workspace, the second stream of the
    // alpha / scan kernels and the pipeline's events
    void *d_split = nullptr;
    size_t split_cap = 0;
    hipStream_t stream2 = nullptr, streamT = nullptr;  // alpha; trajectory (high priority)
    hipStream_t streamS = nullptr;                      // optical-depth scan
    hipStream_t streamD = nullptr;                      // streamed deposition windows (TORJ_DEPO_STREAM=2)
    static constexpr int kRing = 4;                     // alpha-input buffers in flight
    hipEvent_t ev_T[kRing] = {}, ev_A[kRing] = {}, ev_S[kRing] = {}, ev_J = nullptr, ev_F = nullptr;
    hipEvent_t ev_D = nullptr;
    hipEvent_t ev_Nin = nullptr, ev_Nout = nullptr;  // a NULL caller stream's fork / join
};

static const int kFieldSlot[6] = {F_PSI, F_LNNE, F_LNTE, F_BR, F_BZ, F_BPHI};

static int plasma_finish(torj_plasma_s *p, int nR, int nZ, double R1, double Rn, double Z1,
                         double Zn, const double *const fields[6], int device,
                         torj_plasma_t *out) {
    p->device = device;
    Grid &g = p->g;
    g.nR = nR;
    g.nZ = nZ;
    g.R1 = R1;
    g.Rn = Rn;
    g.Z1 = Z1;
    g.Zn = Zn;
    g.hR = (Rn - R1) / (nR - 1);
    g.hZ = (Zn - Z1) / (nZ - 1);
    g.invhR = 1.0 / g.hR;
    g.invhZ = 1.0 / g.hZ;
    const size_t nodes = (size_t)(nR + 2) * (nZ + 2);
    p->coef.assign(nodes * kNF, 0.0);
    for (int f = 0; f < 6; f++)
        for (size_t k = 0; k < nodes; k++) p->coef[k * kNF + kFieldSlot[f]] = fields[f][k];
    *out = p;
    return 0;
}

// Device-side state is created on first GPU use, so the host-side parts of
// the ABI (Plasma construction, ray entry, launch fan) work without a GPU.
static int ensure_device(torj_plasma_s *p) {
    std::lock_guard<std::mutex> lk(p->mu);
    int ndev = 0;
    HIPCK(hipGetDeviceCount(&ndev));
    if (p->device < 0 || p->device >= ndev)
        return fail("device %d not available (%d HIP devices)", p->device, ndev);
    HIPCK(hipSetDevice(p->device));
    if (p->d_coef) return 0;
    HIPCK(hipMalloc(&p->d_coef, p->coef.size() * sizeof(double)));
    HIPCK(hipMemcpy(p->d_coef, p->coef.data(), p->coef.size() * sizeof(double),
                    hipMemcpyHostToDevice));
    {
        std::vector<double> cp((size_t)(p->g.nR - 1) * (p->g.nZ - 1) * kCellRec);
        cell_power_table(p->coef.data(), p->g.nR, p->g.nZ, p->g.hR, p->g.hZ, cp.data());
        HIPCK(hipMalloc(&p->d_cellp, cp.size() * sizeof(double)));
        HIPCK(hipMemcpy(p->d_cellp, cp.data(), cp.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    HIPCK(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    HIPCK(hipDeviceGetAttribute(&p->n_cu, hipDeviceAttributeMultiprocessorCount, p->device));
    HIPCK(hipMalloc(&p->d_flags, sizeof(int)));
    HIPCK(hipMemset(p->d_flags, 0, sizeof(int)));
    return 0;
}

static int ensure_sched(torj_plasma_s *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->sched_cap >= bytes) return 0;
    if (p->d_sched) HIPCK(hipFree(p->d_sched));
    p->d_sched = nullptr;
    p->sched_cap = 0;
    HIPCK(hipMalloc(&p->d_sched, bytes));
    p->sched_cap = bytes;
    return 0;
}

static int ensure_chunks(torj_plasma_s *p, size_t n) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->chunk_cap >= n) return 0;
    if (p->d_chunk) HIPCK(hipFree(p->d_chunk));
    p->d_chunk = nullptr;
    p->chunk_cap = 0;
    HIPCK(hipMalloc(&p->d_chunk, n * sizeof(int)));
    p->chunk_cap = n;
    return 0;
}

static int ensure_fit(torj_plasma_s *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->fit_cap >= bytes) return 0;
    if (p->d_fit) HIPCK(hipFree(p->d_fit));
    p->d_fit = nullptr;
    p->fit_cap = 0;
    HIPCK(hipMalloc(&p->d_fit, bytes));
    p->fit_cap = bytes;
    return 0;
}

// a split-pipeline stream's priority: `dflt`, or the environment's value clamped
// to the device's range (measurement knobs: TORJ_TRAJ_PRIO, TORJ_ALPHA_PRIO,
// TORJ_SCAN_PRIO, TORJ_DEPO_PRIO; TORJ_PRIO_VERBOSE=1 prints the range)
static int stream_prio(const char *name, int dflt, int lo, int hi) {
    static const bool verbose = [&] {
        const char *v = getenv("TORJ_PRIO_VERBOSE");
        const bool on = v && atoi(v) != 0;
        if (on) fprintf(stderr, "torj: stream priority range least %d greatest %d\n", lo, hi);
        return on;
    }();
    const char *e = getenv(name);
    int v = dflt;
    if (e) v = std::min(std::max(atoi(e), std::min(lo, hi)), std::max(lo, hi));
    if (verbose) fprintf(stderr, "torj: %s -> %d\n", name, v);
    return v;
}

static int ensure_split(torj_plasma_s *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (!p->stream2) {
        // the trajectory chain is the critical path: its stream gets the highest
        // priority, so its waves are dispatched ahead of the alpha kernel's
        int lo = 0, hi = 0;
        HIPCK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        // TORJ_TRAJ_CUS=X: the trajectory stream on X of the device's CUs (evenly
        // spread over the mask's bits), the alpha and scan streams on the rest
        int dev = 0, ncu = 0;
        HIPCK(hipGetDevice(&dev));
        HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        const char *tc = getenv("TORJ_TRAJ_CUS"), *ac = getenv("TORJ_ALPHA_CUS");
        const int X = tc ? atoi(tc) : 0, Y = ac ? atoi(ac) : 0;
        if (Y > 0 && Y < ncu) {
            // TORJ_ALPHA_CUS=Y: only the alpha and scan streams masked (to Y CUs),
            // the trajectory stream on every CU -- the others never hold alpha waves
            std::vector<uint32_t> mA((ncu + 31) / 32, 0u);
            for (int c = 0; c < ncu; c++)
                if (((long)(c + 1) * Y) / ncu != ((long)c * Y) / ncu) mA[c / 32] |= 1u << (c % 32);
            HIPCK(hipStreamCreateWithPriority(&p->streamT, hipStreamNonBlocking, hi));
            HIPCK(hipExtStreamCreateWithCUMask(&p->stream2, (uint32_t)mA.size(), mA.data()));
            HIPCK(hipExtStreamCreateWithCUMask(&p->streamS, (uint32_t)mA.size(), mA.data()));
        } else if (X > 0 && X < ncu) {
            std::vector<uint32_t> mT((ncu + 31) / 32, 0u), mA((ncu + 31) / 32, 0u);
            for (int c = 0; c < ncu; c++) {
                const bool t = ((long)(c + 1) * X) / ncu != ((long)c * X) / ncu;
                (t ? mT : mA)[c / 32] |= 1u << (c % 32);
            }
            HIPCK(hipExtStreamCreateWithCUMask(&p->streamT, (uint32_t)mT.size(), mT.data()));
            HIPCK(hipExtStreamCreateWithCUMask(&p->stream2, (uint32_t)mA.size(), mA.data()));
            HIPCK(hipExtStreamCreateWithCUMask(&p->streamS, (uint32_t)mA.size(), mA.data()));
        } else {
            HIPCK(hipStreamCreateWithPriority(&p->streamT, hipStreamNonBlocking, stream_prio("TORJ_TRAJ_PRIO", hi, lo, hi)));
            HIPCK(hipStreamCreateWithPriority(&p->stream2, hipStreamNonBlocking, stream_prio("TORJ_ALPHA_PRIO", lo, lo, hi)));
            // TORJ_SCAN_CUS=Z (measurement knob): the scan's stream -- the optical-depth
            // scan and the streamed deposition's elimination and walk, latency-bound
            // waves of up to 168 VGPRs -- on Z evenly spread CUs only, so the others
            // keep their registers for the alpha waves
            const char *sc = getenv("TORJ_SCAN_CUS");
            const int Z = sc ? atoi(sc) : 0;
            if (Z > 0 && Z < ncu) {
                std::vector<uint32_t> mS((ncu + 31) / 32, 0u);
                for (int c = 0; c < ncu; c++)
                    if (((long)(c + 1) * Z) / ncu != ((long)c * Z) / ncu) mS[c / 32] |= 1u << (c % 32);
                HIPCK(hipExtStreamCreateWithCUMask(&p->streamS, (uint32_t)mS.size(), mS.data()));
            } else {
                HIPCK(hipStreamCreateWithPriority(&p->streamS, hipStreamNonBlocking, stream_prio("TORJ_SCAN_PRIO", lo, lo, hi)));
            }
        }
        for (int q = 0; q < torj_plasma_s::kRing; q++) {
            HIPCK(hipEventCreateWithFlags(&p->ev_T[q], hipEventDisableTiming));
            HIPCK(hipEventCreateWithFlags(&p->ev_A[q], hipEventDisableTiming));
            HIPCK(hipEventCreateWithFlags(&p->ev_S[q], hipEventDisableTiming));
        }
        HIPCK(hipEventCreateWithFlags(&p->ev_J, hipEventDisableTiming));
        HIPCK(hipEventCreateWithFlags(&p->ev_F, hipEventDisableTiming));
        HIPCK(hipEventCreateWithFlags(&p->ev_D, hipEventDisableTiming));
    }
    if (p->split_cap >= bytes) return 0;
    if (p->d_split) HIPCK(hipFree(p->d_split));
    p->d_split = nullptr;
    p->split_cap = 0;
    HIPCK(hipMalloc(&p->d_split, bytes));
    p->split_cap = bytes;
    return 0;
}

static int ensure_workspace(torj_plasma_s *p, size_t n) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->ws_cap >= n) return 0;
    if (p->d_ws) HIPCK(hipFree(p->d_ws));
    p->d_ws = nullptr;
    p->ws_cap = 0;
    HIPCK(hipMalloc(&p->d_ws, n * sizeof(double)));
    p->ws_cap = n;
    return 0;
}

// ===========================================================================
// launch fan (host), src/launch.jl:24-132
// ===========================================================================
// Orthonormal Hermite recurrence, rescaled by 2^-500 past 2^500 (overflow-free
// for any n); returns p_n, p_{n-1} and the binary exponent of the scale.
static void herm_rec(int n, double z, double &pn, double &pn1, int &e2) {
    double p1 = 0.7511255444649425, p2 = 0.0;  // pi^(-1/4)
    int e = 0;
    for (int j = 0; j < n; j++) {
        const double p3 = p2;
        p2 = p1;
        p1 = z * std::sqrt(2.0 / (j + 1)) * p2 - std::sqrt((double)j / (j + 1)) * p3;
        if (std::fabs(p1) > 0x1p500) {
            p1 = std::ldexp(p1, -500);
            p2 = std::ldexp(p2, -500);
            e += 500;
        }
    }
    pn = p1;
    pn1 = p2;
    e2 = e;
}

// FastGaussQuadrature.gausshermite(n) (src/launch.jl:72): ascending nodes,
// weight exp(-x^2).  Zeros are bracketed by sign changes on a grid finer than
// the smallest zero spacing (~pi/sqrt(2n+1), at the origin), bisected and
// Newton-polished -- robust for every n (asymptotic initial guesses are not).
static void gauss_hermite(int n, std::vector<double> &x, std::vector<double> &w) {
    std::vector<double> pos, pw;
    const int half = n / 2;
    const double zmax = std::sqrt(2.0 * n + 1.0) + 1.0;
    const double dz = 0.2 * kPi / std::sqrt(2.0 * n + 1.0);
    double a = (n & 1) ? 0.5 * dz : 0.0, fa, fa1;
    int ea;
    herm_rec(n, a, fa, fa1, ea);
    while ((int)pos.size() < half && a < zmax) {
        const double b = a + dz;
        double fb, fb1;
        int eb;
        herm_rec(n, b, fb, fb1, eb);
        if ((fa > 0) != (fb > 0) && fb != 0.0) {
            double lo = a, hi = b, flo = fa;
            for (int it = 0; it < 60; it++) {
                const double m = 0.5 * (lo + hi);
                double fm, fm1;
                int em;
                herm_rec(n, m, fm, fm1, em);
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
                herm_rec(n, z, pn, pn1, e);
                z -= pn / (std::sqrt(2.0 * n) * pn1);
            }
            herm_rec(n, z, pn, pn1, e);
            pos.push_back(z);
            pw.push_back(std::ldexp(1.0 / (n * pn1 * pn1), -2 * e));
        }
        a = b;
        fa = fb;
    }
    x.clear();
    w.clear();
    for (int i = (int)pos.size() - 1; i >= 0; i--) {
        x.push_back(-pos[i]);
        w.push_back(pw[i]);
    }
    if (n & 1) {
        double pn, pn1;
        int e;
        herm_rec(n, 0.0, pn, pn1, e);
        x.push_back(0.0);
        w.push_back(std::ldexp(1.0 / (n * pn1 * pn1), -2 * e));
    }
    for (size_t i = 0; i < pos.size(); i++) {
        x.push_back(pos[i]);
        w.push_back(pw[i]);
    }
}

struct Rings {
    std::vector<double> r, rw;
    std::vector<int> nth;
    int total = 0;
};

static Rings make_rings(int N_rings, int min_az, double w) {
    Rings R;
    std::vector<double> x, wt;
    gauss_hermite(2 * N_rings + 2, x, wt);  // :72
    for (int i = 0; i < N_rings; i++) {
        R.r.push_back(x[N_rings + 1 + i] * (w / std::sqrt(2.0)));
        R.rw.push_back(wt[N_rings + 1 + i] * (w / std::sqrt(2.0)));
    }
    for (int i = 0; i < N_rings; i++) {  // :80-83, Julia's round(Int64, x): ties to even
        const long k = round_ties_even(min_az * R.r[i] / R.r[0]);
        R.nth.push_back(k < 1 ? 1 : (int)k);
        R.total += R.nth.back();
    }
    return R;
}

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int torj_abi_version(void) { return TORJ_ABI_VERSION; }

#ifndef TORJ_BUILD_ID
#define TORJ_BUILD_ID "unstamped"
#endif
const char *torj_build_id(void) { return TORJ_BUILD_ID; }

#ifdef TORJ_ALPHA_PROF
// profiling build only (not in include/torj_hip.h): g_aprof, read and reset
int torj_alpha_prof_read(unsigned long long *out) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_aprof), sizeof(g_aprof)));
    static const unsigned long long zero[16] = {};
    HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(g_aprof), zero, sizeof(g_aprof)));
    return 0;
}
#endif
#ifdef TORJ_WARM_PROF
// profiling build only (not in include/torj_hip.h): the warm alpha's region
// timers -- out[0] waves, out[1 + k] clock ticks of region k -- read and reset
int torj_warm_prof_read(unsigned long long *out) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wprof), sizeof(g_wprof)));
    static const unsigned long long zero[kWProfN + 1] = {};
    HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(g_wprof), zero, sizeof(g_wprof)));
    return 0;
}
int torj_warm_fad_read(unsigned long long *out) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wfad), sizeof(g_wfad)));
    static const unsigned long long zero[9] = {};
    HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(g_wfad), zero, sizeof(g_wfad)));
    return 0;
}
#endif

const char *torj_last_error(void) { return g_err.c_str(); }

int torj_device_count(int *n) {
    HIPCK(hipGetDeviceCount(n));
    return 0;
}

int torj_abs_al_init(int n) {
    if (n < 1 || n > kMaxGL) return fail("abs_Al_init: order %d outside [1, %d]", n, kMaxGL);
    std::lock_guard<std::mutex> lk(g_gl_mu);
    GLTable t{};
    t.n = n;
    // the bit-identical skip of provably negligible harmonic integrals
    // (torj_math.hpp albajar_harmonic); env TORJ_NEGL_SKIP=0 turns it off (A/B
    // and the test that holds both bit-identical), read at each abs_Al_init
    const char *ne = getenv("TORJ_NEGL_SKIP");
    t.negl_skip = ne ? (atoi(ne) != 0) : 1;
    // the bounded skip of a harmonic whose share of alpha is provably below
    // tiny_alpha m^-1 (albajar_harmonic; ray tracing only -- the point entry
    // torj_abs_albajar_fast evaluates every harmonic): tau moves by less than
    // 2 tiny_alpha per metre of ray, 4e-21 on the headline rays, against the
    // parity bar's 1e-16 absolute floor (C3 trace phase 45.1 -> 40.7 ms, DESIGN.md
    // 3.7).  Env TORJ_TINY_ALPHA overrides (0 = off: every integral evaluated),
    // read at each abs_Al_init
    const char *ta = getenv("TORJ_TINY_ALPHA");
    t.tiny_alpha = ta ? atof(ta) : kTinyAlpha;
    if (!(t.tiny_alpha >= 0.0 && t.tiny_alpha < 1e-12)) return fail("TORJ_TINY_ALPHA=%s outside [0, 1e-12)", ta);
    gauss_legendre(n, t.t, t.w);
    for (int i = 0; i < n; i++) {
        t.st[i] = std::sqrt(1.0 - t.t[i] * t.t[i]);
        t.t2[i] = t.t[i] * t.t[i];
        gl_node_consts(t, i);
    }
    g_gl_host = t;
    g_gl_version++;
    return 0;
}

int torj_plasma_create(int nR, int nZ, const double *R, const double *Z, const double *psi_norm,
                       int n_prof, const double *psi_prof, const double *ne_prof,
                       const double *Te_prof, const double *Br, const double *Bz,
                       const double *Bphi, int n_eq, const double *eq_psi, const double *eq_vol,
                       int device, torj_plasma_t *out) {
    if (!out) return fail("out is NULL");
    if (nR < 2 || nZ < 2 || n_prof < 2 || n_eq < 2) return fail("Plasma: grids need >= 2 points");
    const size_t nd = (size_t)nR * nZ, nc = (size_t)(nR + 2) * (nZ + 2);
    std::vector<double> cpsi(nc), cne(nc), cte(nc), cbr(nc), cbz(nc), cbp(nc);
    bspl2d_prefilter(nR, nZ, psi_norm, cpsi.data());
    bspl2d_prefilter(nR, nZ, Br, cbr.data());
    bspl2d_prefilter(nR, nZ, Bz, cbz.data());
    bspl2d_prefilter(nR, nZ, Bphi, cbp.data());
    // make_2d_prof_spline (src/plasma.jl:16-22)
    auto prof2d = [&](const double *prof, std::vector<double> &c2) {
        std::vector<double> pr = uniform_range(psi_prof[0], psi_prof[n_prof - 1], n_prof);
        std::vector<double> p2(n_prof), c1(n_prof + 2), d2(nd);
        natcubic(n_prof, psi_prof, prof, n_prof, pr.data(), p2.data());
        for (double &v : p2) v = std::log(v);
        bspl1d_prefilter(n_prof, p2.data(), 1, c1.data(), 1);
        for (size_t k = 0; k < nd; k++)
            d2[k] = bspl1d_eval(c1, n_prof, psi_prof[0], psi_prof[n_prof - 1], psi_norm[k]);
        bspl2d_prefilter(nR, nZ, d2.data(), c2.data());
    };
    prof2d(ne_prof, cne);
    prof2d(Te_prof, cte);
    auto *p = new torj_plasma_s();
    // volume_psi_spline (src/plasma.jl:42-44)
    std::vector<double> pr = uniform_range(eq_psi[0], eq_psi[n_eq - 1], n_eq), v2(n_eq);
    natcubic(n_eq, eq_psi, eq_vol, n_eq, pr.data(), v2.data());
    p->n_vol = n_eq;
    p->v1 = eq_psi[0];
    p->vn = eq_psi[n_eq - 1];
    p->vol_coef.assign(n_eq + 2, 0.0);
    bspl1d_prefilter(n_eq, v2.data(), 1, p->vol_coef.data(), 1);
    p->psi_prof_max = *std::max_element(psi_prof, psi_prof + n_prof);
    const double *fields[6] = {cpsi.data(), cne.data(), cte.data(), cbr.data(), cbz.data(), cbp.data()};
    const int rc = plasma_finish(p, nR, nZ, R[0], R[nR - 1], Z[0], Z[nZ - 1], fields, device, out);
    if (rc) delete p;
    return rc;
}

int torj_plasma_create_from_coefs(int nR, int nZ, double R1, double Rn, double Z1, double Zn,
                                  const double *c_psi, const double *c_lnne, const double *c_lnTe,
                                  const double *c_Br, const double *c_Bz, const double *c_Bphi,
                                  int n_vol, double vol_psi1, double vol_psin,
                                  const double *vol_coefs, double psi_prof_max, int device,
                                  torj_plasma_t *out) {
    if (!out) return fail("out is NULL");
    if (nR < 2 || nZ < 2 || n_vol < 2) return fail("Plasma: grids need >= 2 points");
    auto *p = new torj_plasma_s();
    p->n_vol = n_vol;
    p->v1 = vol_psi1;
    p->vn = vol_psin;
    p->vol_coef.assign(vol_coefs, vol_coefs + n_vol + 2);
    p->psi_prof_max = psi_prof_max;
    const double *fields[6] = {c_psi, c_lnne, c_lnTe, c_Br, c_Bz, c_Bphi};
    const int rc = plasma_finish(p, nR, nZ, R1, Rn, Z1, Zn, fields, device, out);
    if (rc) delete p;
    return rc;
}

int torj_plasma_destroy(torj_plasma_t p) {
    if (!p) return 0;
    for (ncclComm_t c : p->comms) (void)ncclCommDestroy(c);
    for (size_t k = 1; k < p->replicas.size(); k++) torj_plasma_destroy(p->replicas[k]);
    if (p->d_coef) (void)hipSetDevice(p->device);
    if (p->stage.sc) (void)hipStreamSynchronize(p->stage.sc);
    if (p->stage.d) (void)hipFree(p->stage.d);
    if (p->stage.h) {
        if (p->stage.h_pinned)
            (void)hipHostFree(p->stage.h);
        else
            free(p->stage.h);
    }
    for (int r = 0; r < 2; r++) {
        if (p->stage.up[r]) (void)hipEventDestroy(p->stage.up[r]);
        if (p->stage.tr[r]) (void)hipEventDestroy(p->stage.tr[r]);
        if (p->stage.dn[r]) (void)hipEventDestroy(p->stage.dn[r]);
    }
    if (p->stage.sc) (void)hipStreamDestroy(p->stage.sc);
    if (p->d_coef) (void)hipFree(p->d_coef);
    if (p->d_cellp) (void)hipFree(p->d_cellp);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    if (p->ev_Nin) (void)hipEventDestroy(p->ev_Nin);
    if (p->ev_Nout) (void)hipEventDestroy(p->ev_Nout);
    if (p->d_sched) (void)hipFree(p->d_sched);
    if (p->d_fit) (void)hipFree(p->d_fit);
    if (p->d_flags) (void)hipFree(p->d_flags);
    if (p->d_chunk) (void)hipFree(p->d_chunk);
    for (hipEvent_t e : p->ev_pool) (void)hipEventDestroy(e);
    if (p->d_ws) (void)hipFree(p->d_ws);
    if (p->d_split) (void)hipFree(p->d_split);
    if (p->d_batch) (void)hipFree(p->d_batch);
    for (int q = 0; q < torj_plasma_s::kRing; q++) {
        if (p->ev_T[q]) (void)hipEventDestroy(p->ev_T[q]);
        if (p->ev_A[q]) (void)hipEventDestroy(p->ev_A[q]);
        if (p->ev_S[q]) (void)hipEventDestroy(p->ev_S[q]);
    }
    if (p->ev_J) (void)hipEventDestroy(p->ev_J);
    if (p->ev_F) (void)hipEventDestroy(p->ev_F);
    if (p->ev_D) (void)hipEventDestroy(p->ev_D);
    if (p->stream2) (void)hipStreamDestroy(p->stream2);
    if (p->streamT) (void)hipStreamDestroy(p->streamT);
    if (p->streamS) (void)hipStreamDestroy(p->streamS);
    if (p->streamD) (void)hipStreamDestroy(p->streamD);
    delete p;
    return 0;
}

int torj_plasma_get_coefs(torj_plasma_t p, int field, double *out) {
    if (!p || field < 0 || field > 5) return fail("bad plasma handle or field index");
    const size_t nodes = (size_t)(p->g.nR + 2) * (p->g.nZ + 2);
    for (size_t k = 0; k < nodes; k++) out[k] = p->coef[k * kNF + kFieldSlot[field]];
    return 0;
}

double torj_plasma_psi_prof_max(torj_plasma_t p) { return p ? p->psi_prof_max : NAN; }

int torj_plasma_volume(torj_plasma_t p, int n, const double *psi, double *vol) {
    if (!p) return fail("bad plasma handle");
    for (int i = 0; i < n; i++) vol[i] = bspl1d_eval(p->vol_coef, p->n_vol, p->v1, p->vn, psi[i]);
    return 0;
}

int torj_shell_volumes(torj_plasma_t p, int n_psi, const double *g, double *dV) {
    if (!p) return fail("bad plasma handle");
    for (int j = 0; j + 1 < n_psi; j++)
        dV[j] = bspl1d_eval(p->vol_coef, p->n_vol, p->v1, p->vn, g[j + 1]) -
                bspl1d_eval(p->vol_coef, p->n_vol, p->v1, p->vn, g[j]);
    return 0;
}

void torj_pol_tor_angles_2_vector(double pol, double tor, double N[3]) {
    // IMAS ec_launchers convention: angle_pol = atan2(-k_Z, -k_R), angle_tor = asin(k_phi / k)
    N[0] = -std::cos(pol) * std::cos(tor);
    N[1] = std::sin(tor);
    N[2] = -std::sin(pol) * std::cos(tor);
}

int torj_launch_peripheral_rays(const double x0[3], const double N0[3], double w,
                                double inv_curv, double f, int N_rings, int min_az, int normalize,
                                int *n_rays, double *pos, double *dir, double *weights) {
    if (N_rings < 2) return fail("ArgumentError: N_rings = %d < 2 which is the minimum", N_rings);
    const Rings RG = make_rings(N_rings, min_az, w);
    if (n_rays) *n_rays = RG.total;
    if (!pos) return 0;
    const int n = RG.total;
    const double nn = std::sqrt(N0[0] * N0[0] + N0[1] * N0[1] + N0[2] * N0[2]);
    const double n0[3] = {N0[0] / nn, N0[1] / nn, N0[2] / nn};
    const bool fin = std::isfinite(inv_curv);
    double w0 = w, xw[3] = {0, 0, 0};
    if (fin) {  // :34-47 Gaussian-beam waist
        const double Rc = 1.0 / inv_curv, lam = kC / f;
        const double w4 = w * w * w * w;
        w0 = (lam * std::fabs(Rc) * w) / std::sqrt(lam * lam * Rc * Rc + kPi * kPi * w4);
        const double zw = kPi * kPi * Rc * w4 / (lam * lam * Rc * Rc + kPi * kPi * w4);
        for (int k = 0; k < 3; k++) xw[k] = x0[k] - n0[k] * zw;
    }
    double ec[3] = {1.0, 0.0, -n0[0] / n0[2]};                     // :54-57
    double eu[3] = {-n0[0] * n0[1] / n0[2], n0[2] - n0[0], -n0[1]};  // :61-64
    const double nc = std::sqrt(ec[0] * ec[0] + ec[1] * ec[1] + ec[2] * ec[2]);
    const double nu = std::sqrt(eu[0] * eu[0] + eu[1] * eu[1] + eu[2] * eu[2]);
    for (int k = 0; k < 3; k++) {
        ec[k] /= nc;
        eu[k] /= nu;
    }
    const double sg = inv_curv > 0 ? 1.0 : (inv_curv < 0 ? -1.0 : 0.0);
    int kk = 0;
    for (int i = 0; i < N_rings; i++) {
        const int nt = RG.nth[i];
        for (int j = 0; j < nt; j++) {
            const double th = 2.0 * kPi * (double)j / (double)nt;
            const double chi = RG.r[i] * std::cos(th), ups = RG.r[i] * std::sin(th);
            const int q = kk + j;
            double P[3], D[3];
            for (int k = 0; k < 3; k++) P[k] = chi * ec[k] + ups * eu[k] + x0[k];
            if (fin) {
                for (int k = 0; k < 3; k++) D[k] = w0 / w * (chi * ec[k] + ups * eu[k]) * sg + xw[k];
                if (inv_curv < 0.0)
                    for (int k = 0; k < 3; k++) D[k] -= P[k];
                else
                    for (int k = 0; k < 3; k++) D[k] = -D[k] + P[k];
                const double dn = std::sqrt(D[0] * D[0] + D[1] * D[1] + D[2] * D[2]);
                for (double &c : D) c /= dn;
            } else {
                for (int k = 0; k < 3; k++) D[k] = n0[k];
            }
            for (int k = 0; k < 3; k++) {
                pos[(size_t)k * n + q] = P[k];
                dir[(size_t)k * n + q] = D[k];
            }
            weights[q] = RG.r[i] * RG.rw[i] * (2.0 * kPi / (double)nt);
        }
        kk += nt;
    }
    if (normalize) {  // :125-129
        double s = 0;
        for (int i = 0; i < n; i++) s += weights[i];
        for (int i = 0; i < n; i++) weights[i] /= s;
    } else {
        for (int i = 0; i < n; i++) weights[i] *= 2.0 / (w * w * kPi);
    }
    return 0;
}

int torj_ray_entry(torj_plasma_t p, int n, const double *x0, const double *N0, double omega,
                   int mode, double *xp, double *Np, double *s0, int *status) {
    if (!p) return fail("bad plasma handle");
    if (mode != 1 && mode != -1) return fail("mode must be +1 (X) or -1 (O)");
    const double *coef = p->coef.data();
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++) {
        const double a[3] = {x0[i], x0[(size_t)n + i], x0[2 * (size_t)n + i]};
        const double d[3] = {N0[i], N0[(size_t)n + i], N0[2 * (size_t)n + i]};
        double xo[3], No[3];
        status[i] = ray_entry_one(coef, p->g, p->psi_prof_max, a, d, omega, mode, xo, No, s0[i]);
        for (int k = 0; k < 3; k++) {
            xp[(size_t)k * n + i] = xo[k];
            Np[(size_t)k * n + i] = No[k];
        }
    }
    return 0;
}


}  // extern "C"

// ---- device helpers ----
template <typename T>
static int dupload(T **d, const T *h, size_t n, hipStream_t s) {
    *d = nullptr;
    if (!h || n == 0) return 0;
    HIPCK(hipMalloc(d, n * sizeof(T)));
    HIPCK(hipMemcpyAsync(*d, h, n * sizeof(T), hipMemcpyHostToDevice, s));
    return 0;
}
template <typename T>
static int dalloc(T **d, size_t n, bool want) {
    *d = nullptr;
    if (!want || n == 0) return 0;
    HIPCK(hipMalloc(d, n * sizeof(T)));
    return 0;
}
template <typename T>
static int ddownload(T *h, const T *d, size_t n, hipStream_t s) {
    if (!h || !d || n == 0) return 0;
    HIPCK(hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, s));
    return 0;
}

struct DevBufs {
    std::vector<void *> ptrs;
    ~DevBufs() {
        for (void *q : ptrs)
            if (q) (void)hipFree(q);
    }
    template <typename T>
    T *track(T *q) {
        ptrs.push_back((void *)q);
        return q;
    }
    // dupload / dalloc whose buffer is owned from the moment it exists (freed
    // on every early return, a failed copy after a good allocation included)
    template <typename T>
    int up(T **d, const T *h, size_t n, hipStream_t s) {
        const int r = dupload(d, h, n, s);
        track(*d);
        return r;
    }
    template <typename T>
    int alloc(T **d, size_t n, bool want) {
        const int r = dalloc(d, n, want);
        track(*d);
        return r;
    }
};

static inline int nblocks(int n, int b) { return (n + b - 1) / b; }

extern "C" {

int torj_eval_plasma(torj_plasma_t p, int n, const double *x, const double *N, double omega,
                     double *out) {
    if (!p) return fail("bad plasma handle");
    if (n <= 0) return 0;
    if (ensure_device(p)) return -1;
    DevBufs B;
    double *dx, *dN, *dout;
    if (B.up(&dx, x, 3 * (size_t)n, p->stream) || B.up(&dN, N, 3 * (size_t)n, p->stream) ||
        B.alloc(&dout, 13 * (size_t)n, true))
        return -1;
    EvalArgs a{};
    a.coef = p->d_coef;
    a.g = p->g;
    a.k = make_consts(omega);
    a.omega = omega;
    a.n = n;
    a.x = dx;
    a.N = dN;
    a.out = dout;
    hipLaunchKernelGGL(k_eval_plasma, dim3(nblocks(n, 256)), dim3(256), 0, p->stream, a);
    HIPCK(hipGetLastError());
    if (ddownload(out, dout, 13 * (size_t)n, p->stream)) return -1;
    HIPCK(hipStreamSynchronize(p->stream));
    return 0;
}

int torj_dispersion(torj_plasma_t p, int n, const double *x, const double *N, double omega,
                    int mode, double *D, double *du, double *alpha) {
    if (!p) return fail("bad plasma handle");
    if (n <= 0) return 0;
    if (ensure_device(p)) return -1;
    if (alpha && ensure_gl_on_device(p->device)) return -1;
    DevBufs B;
    double *dx, *dN, *dD, *ddu, *dal;
    if (B.up(&dx, x, 3 * (size_t)n, p->stream) || B.up(&dN, N, 3 * (size_t)n, p->stream) ||
        B.alloc(&dD, n, D != nullptr) || B.alloc(&ddu, 6 * (size_t)n, du != nullptr) ||
        B.alloc(&dal, n, alpha != nullptr))
        return -1;
    EvalArgs a{};
    a.coef = p->d_coef;
    a.g = p->g;
    a.k = make_consts(omega);
    a.omega = omega;
    a.mode = mode;
    a.n = n;
    a.x = dx;
    a.N = dN;
    a.D = dD;
    a.du = ddu;
    a.alpha = dal;
    if (alpha)
        hipLaunchKernelGGL(k_dispersion<true>, dim3(nblocks(n, 256)), dim3(256), 0, p->stream, a);
    else
        hipLaunchKernelGGL(k_dispersion<false>, dim3(nblocks(n, 256)), dim3(256), 0, p->stream, a);
    HIPCK(hipGetLastError());
    if (ddownload(D, dD, n, p->stream) || ddownload(du, ddu, 6 * (size_t)n, p->stream) ||
        ddownload(alpha, dal, n, p->stream))
        return -1;
    HIPCK(hipStreamSynchronize(p->stream));
    return 0;
}

static int batched_scalar(bool albajar, int n, const double *omega, const double *X,
                          const double *Y, const double *Nabs, const double *Npar,
                          const double *Te, int mode, double *out) {
    if (n <= 0) return 0;
    int dev = 0;
    HIPCK(hipGetDevice(&dev));
    if (albajar && ensure_gl_on_device(dev)) return -1;
    DevBufs B;
    AlbArgs a{};
    a.n = n;
    a.mode = mode;
    double *d[7];
    const double *h[6] = {omega, X, Y, Nabs, Npar, Te};
    for (int k = 0; k < 6; k++) {
        d[k] = nullptr;
        if (h[k] && B.up(&d[k], h[k], n, nullptr)) return -1;
    }
    if (B.alloc(&d[6], n, true)) return -1;
    a.omega = d[0], a.X = d[1], a.Y = d[2], a.Nabs = d[3], a.Npar = d[4], a.Te = d[5];
    a.out = d[6];
    if (albajar)
        hipLaunchKernelGGL(k_albajar, dim3(nblocks(n, 256)), dim3(256), 0, nullptr, a);
    else
        hipLaunchKernelGGL(k_refr, dim3(nblocks(n, 256)), dim3(256), 0, nullptr, a);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpy(out, d[6], n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int torj_abs_albajar_fast(int n, const double *omega, const double *X, const double *Y,
                          const double *Nabs, const double *Npar, const double *Te, int mode,
                          double *alpha) {
    return batched_scalar(true, n, omega, X, Y, Nabs, Npar, Te, mode, alpha);
}

int torj_alpha_warm(int n, const double *omega, const double *X, const double *Y,
                    const double *Nabs, const double *Npar, const double *Te,
                    const double *inv_dDdN, int mode, int iwarm, double *alpha, double *Nperp2) {
    if (n <= 0) return 0;
    if (iwarm != 1 && iwarm != 3) return fail("iwarm must be 1 or 3");
    if (mode != 1 && mode != -1) return fail("mode must be +1 (X) or -1 (O)");
    DevBufs B;
    AlbArgs a{};
    a.n = n;
    a.mode = mode;
    a.iwarm = iwarm;
    double *d[9];
    const double *h[7] = {omega, X, Y, Nabs, Npar, Te, inv_dDdN};
    for (int k = 0; k < 7; k++) {
        if (!h[k]) return fail("torj_alpha_warm: every input array is required");
        if (B.up(&d[k], h[k], n, nullptr)) return -1;
    }
    if (B.alloc(&d[7], n, true) || B.alloc(&d[8], 2 * (size_t)n, true)) return -1;
    a.omega = d[0], a.X = d[1], a.Y = d[2], a.Nabs = d[3], a.Npar = d[4], a.Te = d[5];
    a.inv = d[6], a.out = d[7], a.n2 = d[8];
    hipLaunchKernelGGL(k_alpha_warm, dim3(nblocks(n, 64)), dim3(64), 0, nullptr, a);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpy(alpha, d[7], n * sizeof(double), hipMemcpyDeviceToHost));
    if (Nperp2) HIPCK(hipMemcpy(Nperp2, d[8], 2 * n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int torj_refractive_index_sq(int n, const double *X, const double *Y, const double *Npar, int mode,
                             double *out) {
    return batched_scalar(false, n, nullptr, X, Y, nullptr, Npar, nullptr, mode, out);
}

int torj_ray_entry_device(torj_plasma_t p, int n, const double *x0, const double *N0, double omega,
                          int mode, double *xp, double *Np, double *s0, int *status, void *stream) {
    if (!p) return fail("bad plasma handle");
    if (mode != 1 && mode != -1) return fail("mode must be +1 (X) or -1 (O)");
    if (n <= 0) return 0;
    if (ensure_device(p)) return -1;
    EntryArgs a{p->d_coef, p->g, p->psi_prof_max, omega, mode, n, x0, N0, xp, Np, s0, status};
    hipLaunchKernelGGL(k_ray_entry, dim3(nblocks(n, 64)), dim3(64), 0, (hipStream_t)stream, a);
    HIPCK(hipGetLastError());
    return 0;
}

int torj_ray_entry_gpu(torj_plasma_t p, int n, const double *x0, const double *N0, double omega,
                       int mode, double *xp, double *Np, double *s0, int *status) {
    if (!p) return fail("bad plasma handle");
    if (n <= 0) return 0;
    if (ensure_device(p)) return -1;
    hipStream_t s = p->stream;
    DevBufs B;
    double *dx0, *dN0, *dxp, *dNp, *ds0;
    int *dst;
    if (B.up(&dx0, x0, 3 * (size_t)n, s) || B.up(&dN0, N0, 3 * (size_t)n, s)) return -1;
    if (B.alloc(&dxp, 3 * (size_t)n, true) || B.alloc(&dNp, 3 * (size_t)n, true) ||
        B.alloc(&ds0, n, true) || B.alloc(&dst, n, true))
        return -1;
    if (torj_ray_entry_device(p, n, dx0, dN0, omega, mode, dxp, dNp, ds0, dst, s)) return -1;
    if (ddownload(xp, dxp, 3 * (size_t)n, s) || ddownload(Np, dNp, 3 * (size_t)n, s) ||
        ddownload(s0, ds0, n, s) || ddownload(status, dst, n, s))
        return -1;
    HIPCK(hipStreamSynchronize(s));
    return 0;
}

}  // extern "C"

// the reference deposition walk's per-boundary root counts, open-shell spill
// (NaN: every shell closed) and per-ray shell powers, cleared before the walk
// (2 GB on the headline beam: ~0.5 ms)
static int fit_zero(const FitArgs &fa, hipStream_t st) {
    const size_t L = (size_t)fa.n_psi, N = (size_t)fa.n;
    HIPCK(hipMemsetAsync(fa.cnt, 0, (L + 1) * N * sizeof(int), st));
    HIPCK(hipMemsetAsync(fa.Fopen, 0xFF, L * N * sizeof(double), st));
    HIPCK(hipMemsetAsync(fa.dPs, 0, L * N * sizeof(double), st));
    return 0;
}

// The split RK4 path's launches: per block of kb steps, the
// trajectory kernel on the handle's high-priority stream, the alpha and scan
// kernels on its low-priority one, a ring of kRing alpha-input buffers so the
// trajectory runs up to kRing blocks ahead of the alpha; forked from and
// joined back into `s`.
static int split_trace(torj_plasma_s *p, TraceArgs a, int DM, bool tr, int cs, hipStream_t s,
                       const FitArgs *fa, DepoStream *dso) {
    const size_t n = (size_t)a.n;
    const int n_steps = a.n_steps;
    // steps per block: kRing alpha-input buffers within the budget (TORJ_SPLIT_MB
    // per buffer, default 1024: measured 66.5 / 67.8 / 69.4 ms at 1 / 2 / 4 GiB on
    // the headline beam), a multiple of the chunk length
    static const size_t budget_env = [] {
        const char *e = getenv("TORJ_SPLIT_MB");
        return (size_t)(e ? atol(e) : 1024) << 20;
    }();
    // ... and at most 1/16 of the device memory free now for each of the kRing
    // buffers (a quarter of it for the whole ring; 1 GiB on an idle MI355X)
    size_t free_b = 0, total_b = 0;
    HIPCK(hipMemGetInfo(&free_b, &total_b));
    const size_t budget = std::max<size_t>(std::min(budget_env, free_b / 16), 1);
    constexpr int R = torj_plasma_s::kRing;
    const int nf = a.abs_model >= 2 ? kAinFW : kAinF;
    const size_t per_step = 4 * (size_t)nf * sizeof(double) * n;
    long kb = (long)std::max<size_t>(1, budget / per_step);
    kb = std::min<long>(kb, 16383);  // the alpha kernels' grid.y = 4 kb stays <= 65535
    if (a.chunk_steps > 0 && kb >= a.chunk_steps) kb -= kb % a.chunk_steps;
    if (p->sched_mode == 3 && p->sched_waves > 0) kb = std::min(p->sched_waves, 16383);  // torj_set_sched(p, 3, steps per block)
    kb = std::min<long>(kb, n_steps);
    const int n_cb = (a.chunk_steps > 0 ? n_steps / a.chunk_steps : 0) + 1;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    // work words exist only for a counted launch (a.counters): uncounted
    // (production) launches neither write nor read them, nor reserve them
    const size_t b_ain = al(per_step * kb), b_alpha = al(4 * sizeof(double) * n * kb),
                 b_awork = a.counters ? al(4 * sizeof(unsigned) * n * kb) : 0,
                 b_psib = DM == kDepoBinned ? al(sizeof(double) * n * kb) : 0,
                 b_cbx = al(6 * sizeof(double) * n * n_cb), b_n8 = al(8 * n), b_n4 = al(4 * n);
    // the block zero flags (ZBox): Albajar with the early settle on (GLTable::negl_skip);
    // TORJ_ALPHA_ZFLAG=0 (read per call) turns them off
    const char *zf_e = getenv("TORJ_ALPHA_ZFLAG");
    const bool zflag_on = a.abs_model == 1 && g_gl_host.negl_skip && !(zf_e && atoi(zf_e) == 0);
    const size_t b_zf = zflag_on ? al(n) : 0;
    // the streamed deposition's per-ray walk state (fa: the reference profile;
    // TORJ_DEPO_STREAM=0 runs the whole walk after the trace instead)
    // TORJ_DEPO_STREAM=1: the windows on the scan's stream, after each scan;
    // =2: on a stream of their own, each after its block's scan, so the next
    // scan (and the ring slot it releases) does not wait behind them; =3: on
    // the scan's stream, each window's elimination and walk as two launches
    // (the default since round 4: DESIGN.md 3.4); =4: the two launches on a
    // stream of their own (as 2)
    const char *dstream_e = getenv("TORJ_DEPO_STREAM");  // read per call (tests compare both)
    const int dstream_env = dstream_e ? atoi(dstream_e) : 3;
    const bool dstream = fa && dso && dstream_env != 0;
    const size_t b_dsd = dstream ? al(kDsNd * sizeof(double) * n) : 0,
                 b_dsi = dstream ? al(kDsNi * sizeof(int) * n) : 0;
    // warm: the list of deferred (lrm > 3) points of a block (one list: the
    // alpha kernels of consecutive blocks are ordered on one stream) and one
    // counter per block
    // TORJ_SPLIT_FIRST: the first block's steps (a multiple of the chunk; 0 =
    // uniform blocks): a short first block lets the alpha kernel start sooner,
    // while the trajectory kernel alone cannot fill the chip
    const char *first_e = getenv("TORJ_SPLIT_FIRST");
    long first = first_e ? atol(first_e) : 0;
    if (a.chunk_steps > 0 && first > 0) first = std::max<long>(a.chunk_steps, first - first % a.chunk_steps);
    if (first >= kb || first >= n_steps) first = 0;
    const int n_blk = first ? 1 + (int)((n_steps - first + kb - 1) / kb) : (int)((n_steps + kb - 1) / kb);
    const size_t b_defer = a.abs_model >= 2 ? al(4 * sizeof(unsigned long long) * n * kb) : 0,
                 b_dcnt = a.abs_model >= 2 ? al(sizeof(unsigned) * n_blk) : 0;
    const size_t bytes = R * (b_ain + b_alpha + b_awork) + R * b_psib + b_cbx + 6 * b_n8 + 3 * b_n8 +
                         2 * b_n4 + b_dsd + b_dsi + b_defer + b_dcnt + R * b_zf;
    if (ensure_split(p, bytes)) return -1;
    char *q = (char *)p->d_split;
    auto take = [&](size_t b) {
        char *r = q;
        q += b;
        return r;
    };
    double *ain[R];
    for (int r = 0; r < R; r++) ain[r] = (double *)take(b_ain);
    SplitArgs sp{};
    double *alphas[R];
    unsigned *aworks[R];
    for (int r = 0; r < R; r++) {
        alphas[r] = (double *)take(b_alpha);
        aworks[r] = (unsigned *)take(b_awork);
    }
    sp.nf = nf;
    double *psib[R] = {};
    if (b_psib)
        for (int r = 0; r < R; r++) psib[r] = (double *)take(b_psib);
    unsigned char *zflags[R] = {};
    if (b_zf)
        for (int r = 0; r < R; r++) zflags[r] = (unsigned char *)take(b_zf);
    sp.cbx = (double *)take(b_cbx);
    sp.tx = (double *)take(6 * b_n8);
    sp.stau = (double *)take(b_n8);
    sp.spsi = (double *)take(b_n8);
    sp.sPdep = (double *)take(b_n8);
    sp.tinfo = (int *)take(b_n4);
    sp.sinfo = (int *)take(b_n4);
    unsigned long long *defer = b_defer ? (unsigned long long *)take(b_defer) : nullptr;
    unsigned *dcnt = b_dcnt ? (unsigned *)take(b_dcnt) : nullptr;
    sp.defer = defer;
    DepoStream ds{};
    if (dstream) {
        ds.d = (double *)take(b_dsd);
        ds.v = (int *)take(b_dsi);
        *dso = ds;
    } else if (dso) {
        *dso = DepoStream{};
    }

    // TORJ_SPLIT_SERIAL=1: every kernel on the caller's stream, no overlap (a
    // measurement aid; read per call so a test can compare both orders)
    const char *serial_e = getenv("TORJ_SPLIT_SERIAL");
    const bool serial = serial_e && atoi(serial_e) != 0;
    // the scan on a third stream (TORJ_SPLIT_SCAN=0: behind the alpha kernel on
    // the second), so the alpha kernel of block b + 1 need not wait for the
    // latency-bound one-lane-per-ray scan of block b
    static const bool scan_own = [] {
        const char *e = getenv("TORJ_SPLIT_SCAN");
        return !e || atoi(e) != 0;
    }();
    hipStream_t sT = serial ? s : p->streamT, s2 = serial ? s : p->stream2;
    hipStream_t s3 = serial ? s : (scan_own ? p->streamS : p->stream2);
    const bool depo_own = dstream && (dstream_env == 2 || dstream_env == 4) && !serial;
    // =5: the windows' two launches on the trajectory kernel's stream, each
    // window `lag` blocks behind its scan (TORJ_DEPO_LAG, default 2, < kRing):
    // the walk's waves then alternate with the trajectory's instead of
    // holding registers beside both it and the alpha kernel
    const bool depo_traj = dstream && dstream_env == 5 && !serial;
    const char *lag_e = getenv("TORJ_DEPO_LAG");
    const int depo_lag = std::min(torj_plasma_s::kRing - 1, std::max(1, lag_e ? atoi(lag_e) : 2));
    if (depo_own && !p->streamD) {  // created on first use only: one more queue otherwise
        int lo = 0, hi = 0;
        HIPCK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCK(hipStreamCreateWithPriority(&p->streamD, hipStreamNonBlocking, stream_prio("TORJ_DEPO_PRIO", lo, lo, hi)));
    }
    hipStream_t sD = depo_own ? p->streamD : s3;
    if (!serial) {  // fork from the caller's stream
        HIPCK(hipEventRecord(p->ev_F, s));
        HIPCK(hipStreamWaitEvent(sT, p->ev_F, 0));
        HIPCK(hipStreamWaitEvent(s2, p->ev_F, 0));
        if (s3 != s2) HIPCK(hipStreamWaitEvent(s3, p->ev_F, 0));
    }
    // the scan's carry starts at (steps 0, OK), tau = 0, P_dep = 0
    HIPCK(hipMemsetAsync(sp.stau, 0, 3 * b_n8, sT));
    HIPCK(hipMemsetAsync(sp.sinfo, 0, b_n4, sT));
    if (dstream) HIPCK(hipMemsetAsync(ds.v + kDsJ * n, 0xFF, n * sizeof(int), sT));  // j = -1: not started
    if (dcnt) HIPCK(hipMemsetAsync(dcnt, 0, n_blk * sizeof(unsigned), s2));  // the alpha kernels' stream
    // the walk's arrays on the scan's stream: the first window runs after the
    // first scan there (or, for TORJ_DEPO_STREAM=2, after an event recorded
    // there), so the clearing overlaps the first trajectory block instead of
    // delaying it (0.5 ms per headline launch)
    if (fa && fit_zero(*fa, s3)) return -1;
    const size_t fit_lds = fa && fa->n_psi <= kFitGridLds ? (size_t)fa->n_psi * sizeof(double) : 0;
    const int G = (int)((n + 63) / 64);
    // the trajectory kernel with the coefficients staged in LDS whenever the grid
    // fits 160 KiB at 6 fp64 per node (56 x 56: 161 KB), one workgroup of wpb
    // waves per CU (measured: trajectory kernel 28.2 -> 24.3 ms, pipeline 67.2 ->
    // 61.6 ms on the headline beam; TORJ_TRAJ_LDS=0 reads them through L2)
    // (read per call: the tests compare the modes; TORJ_TILE_CAP / TORJ_TILE_MARGIN
    // shrink the tile to exercise the global-memory fallback)
    // TORJ_TRAJ_LDS: 3 (default since round 4) the cell-tiled power-form kernel
    // k_traj_cell (trace phase 51.4-51.5 -> 48.9-49.3 ms on the headline beam,
    // alternating); 1 the whole-grid node table in LDS; 2 the node tile; 0 L2
    const char *lds_e = getenv("TORJ_TRAJ_LDS");
    const int lds_env = lds_e ? atoi(lds_e) : 3;
    const char *cap_e = getenv("TORJ_TILE_CAP"), *mar_e = getenv("TORJ_TILE_MARGIN");
    const int tile_max = lds_env == 3 ? kTileCells : kTileNodes;  // cells / nodes
    sp.tile_cap = std::min(tile_max, cap_e ? atoi(cap_e) : tile_max);
    sp.tile_margin = mar_e ? atof(mar_e) : 1.001;
    // test hook only (tests/test_gpu_split.py): the scan reads alpha as NaN at
    // this step for every third ray -- a stray setting corrupts results, so say so
    const char *nan_e = getenv("TORJ_TEST_NAN_ALPHA_STEP");
    sp.nan_step = nan_e ? atoi(nan_e) : -1;
    if (sp.nan_step >= 0) {
        static std::atomic<bool> warned{false};
        if (!warned.exchange(true))
            fprintf(stderr, "libtorj_hip: TORJ_TEST_NAN_ALPHA_STEP=%d is set -- a TEST HOOK: alpha is "
                            "read as NaN at that step for every third ray\n", sp.nan_step);
    }
    // test hook only (tests/test_gpu_split.py): TORJ_TEST_ZFLAG_NAN=s -- the fully
    // flagged alpha waves of the blocks that start at step s or later write NaN
    // instead of 0, so that the rays they hold stop NAN where the flags fired
    const char *zn_e = getenv("TORJ_TEST_ZFLAG_NAN");
    const int zflag_nan_from = zn_e ? std::max(0, atoi(zn_e)) : -1;
    sp.zval = 0.0;
    if (zflag_nan_from >= 0) {
        static std::atomic<bool> warned{false};
        if (!warned.exchange(true))
            fprintf(stderr, "libtorj_hip: TORJ_TEST_ZFLAG_NAN is set -- a TEST HOOK: fully flagged alpha "
                            "waves write NaN\n");
    }
    const char *dl_e = getenv("TORJ_WARM_DEFER_LRM");
    sp.defer_lrm = dl_e ? std::min(3, std::max(0, atoi(dl_e))) : 3;
    const size_t lds_bytes = (size_t)(a.g.nR + 2) * (a.g.nZ + 2) * kTrajLdsNS * sizeof(double);
    const bool lds_traj = lds_env == 1 && lds_bytes <= 160 * 1024;
    const bool tile_traj = lds_env == 2, cell_traj = lds_env == 3;
    sp.traj_mode = cell_traj ? kTrajCell : tile_traj ? kTrajTile : lds_traj ? kTrajLds : kTrajL2;
    const int wpb = std::min(8, std::max(1, (G + p->n_cu - 1) / p->n_cu));
    const int n_blocks = n_blk;
#define TORJ_SPLIT_DISPATCH(K, ...)                                                         \
    do {                                                                                    \
        if (DM == kDepoSamples) {                                                           \
            if (tr) hipLaunchKernelGGL((K<kDepoSamples, true>), __VA_ARGS__);               \
            else hipLaunchKernelGGL((K<kDepoSamples, false>), __VA_ARGS__);                 \
        } else if (DM == kDepoBinned) {                                                     \
            if (tr) hipLaunchKernelGGL((K<kDepoBinned, true>), __VA_ARGS__);                \
            else hipLaunchKernelGGL((K<kDepoBinned, false>), __VA_ARGS__);                  \
        } else {                                                                            \
            if (tr) hipLaunchKernelGGL((K<kDepoNone, true>), __VA_ARGS__);                  \
            else hipLaunchKernelGGL((K<kDepoNone, false>), __VA_ARGS__);                    \
        }                                                                                   \
    } while (0)
    for (int b = 0; b < n_blocks; b++) {
        sp.k0 = (int)(first ? (b == 0 ? 0 : first + (long)(b - 1) * kb) : b * kb);
        sp.kb = (int)std::min<long>(first && b == 0 ? first : kb, n_steps - sp.k0);
        const int r = b % R;
        sp.ain = ain[r];
        sp.psib = psib[r];
        sp.zflag = zflags[r];
        sp.zval = (zflag_nan_from >= 0 && sp.k0 >= zflag_nan_from) ? NAN : 0.0;
        sp.alpha = alphas[r];
        sp.awork = b_awork ? aworks[r] : nullptr;  // work words only for a counted launch
        // this ring slot's previous readers (alpha and scan of block b - R) are done
        if (b >= R) HIPCK(hipStreamWaitEvent(sT, p->ev_S[r], 0));
        if (depo_traj && b >= depo_lag) {  // block b - lag's window, behind its scan
            const int bw = b - depo_lag;
            HIPCK(hipStreamWaitEvent(sT, p->ev_S[bw % R], 0));
            const int cap = (int)(first ? (bw == 0 ? first : first + (long)bw * kb) : std::min<long>((long)(bw + 1) * kb, n_steps));
            hipLaunchKernelGGL(k_depo_elim, dim3(G), dim3(64), 0, sT, *fa, ds, sp.sinfo, cap);
            hipLaunchKernelGGL(k_depo_walk, dim3(G), dim3(64), fit_lds, sT, *fa, ds, sp.sinfo, cap);
        }
        if (cell_traj)
            TORJ_SPLIT_DISPATCH(k_traj_cell, dim3(G), dim3(64), 0, sT, a, sp);
        else if (tile_traj)
            TORJ_SPLIT_DISPATCH(k_traj_tile, dim3(G), dim3(64), 0, sT, a, sp);
        else if (lds_traj)
            TORJ_SPLIT_DISPATCH(k_traj_lds, dim3(nblocks(G, wpb)), dim3(64 * wpb), lds_bytes, sT, a, sp);
        else
            TORJ_SPLIT_DISPATCH(k_traj, dim3(G), dim3(64), 0, sT, a, sp);
        HIPCK(hipEventRecord(p->ev_T[r], sT));
        HIPCK(hipStreamWaitEvent(s2, p->ev_T[r], 0));
        const int nqA = (int)((n + kAlphaBlock - 1) / kAlphaBlock);
        const dim3 agridA((unsigned)nqA, (unsigned)(4 * sp.kb));  // ray groups fastest
        const int nqW = (int)((n + kAlphaWarmBlock - 1) / kAlphaWarmBlock);
        const dim3 agridW((unsigned)nqW, (unsigned)(4 * sp.kb));
        sp.defer_cnt = dcnt ? dcnt + b : nullptr;
#define TORJ_WARM_LAUNCH(IW, C)                                                                     \
    do {                                                                                            \
        hipLaunchKernelGGL((k_alpha_warm_pts<IW, C>), agridW, dim3(kAlphaWarmBlock), 0, s2, a, sp, nqW); \
        hipLaunchKernelGGL((k_alpha_warm_big<IW, C>), dim3(TORJ_WARM_BIG_GRID), dim3(64), 0, s2, a, sp); \
    } while (0)
        if (a.abs_model == 3) {
            if (sp.awork) TORJ_WARM_LAUNCH(3, true);
            else TORJ_WARM_LAUNCH(3, false);
        } else if (a.abs_model == 2) {
            if (sp.awork) TORJ_WARM_LAUNCH(1, true);
            else TORJ_WARM_LAUNCH(1, false);
        }
#undef TORJ_WARM_LAUNCH
#if TORJ_ALPHA_PPW > 1
        else {
            const dim3 agridP((unsigned)nqA, (unsigned)((4 * sp.kb + TORJ_ALPHA_PPW - 1) / TORJ_ALPHA_PPW));
            if (sp.awork)
                hipLaunchKernelGGL((k_alpha_pts_mp<true, TORJ_ALPHA_PPW>), agridP, dim3(kAlphaBlock), 0, s2, a, sp, nqA);
            else
                hipLaunchKernelGGL((k_alpha_pts_mp<false, TORJ_ALPHA_PPW>), agridP, dim3(kAlphaBlock), 0, s2, a, sp, nqA);
        }
#else
        else if (sp.awork)  // a counted launch
            hipLaunchKernelGGL(k_alpha_pts<true>, agridA, dim3(kAlphaBlock), 0, s2, a, sp, nqA);
        else
            hipLaunchKernelGGL(k_alpha_pts<false>, agridA, dim3(kAlphaBlock), 0, s2, a, sp, nqA);
#endif
        HIPCK(hipEventRecord(p->ev_A[r], s2));
        if (s3 != s2) HIPCK(hipStreamWaitEvent(s3, p->ev_A[r], 0));
        if (a.counters)
            TORJ_SPLIT_DISPATCH(k_tau_scan_counted, dim3(G), dim3(64), 0, s3, a, sp);
        else
            TORJ_SPLIT_DISPATCH(k_tau_scan, dim3(G), dim3(64), 0, s3, a, sp);
        HIPCK(hipEventRecord(p->ev_S[r], s3));
        // the deposition walk's windows behind this scan (same stream: after it,
        // and the next scan after them; the ring slot is already released)
        // (measured on the headline beam: after every block on the scan's stream
        // 3.62-3.63e9 ray-steps/s; every 2nd / 4th block 3.45-3.64 / 3.58-3.59e9;
        // behind the alpha or the trajectory kernel's stream 3.03 / 2.98e9)
        if (dstream && !depo_traj && b + 1 < n_blocks) {
            if (depo_own) HIPCK(hipStreamWaitEvent(sD, p->ev_S[r], 0));
            if (dstream_env == 3 || dstream_env == 4) {  // elimination and walk as two launches
                // each pair advances a ray by at most one window of kDepoQ
                // segments, so a block of more steps than that takes as many pairs
                // as it has windows (blocks of 120 steps: two), and the walk keeps
                // up with the scan instead of leaving windows for k_depo_tail
                for (int w = 0; w < (sp.kb + kDepoQ - 1) / kDepoQ; w++) {
                    hipLaunchKernelGGL(k_depo_elim, dim3(G), dim3(64), 0, sD, *fa, ds, sp.sinfo, sp.k0 + sp.kb);
                    hipLaunchKernelGGL(k_depo_walk, dim3(G), dim3(64), fit_lds, sD, *fa, ds, sp.sinfo,
                                       sp.k0 + sp.kb);
                }
            } else {
                hipLaunchKernelGGL(k_depo_stream, dim3(G), dim3(64), fit_lds, sD, *fa, ds, sp.sinfo,
                                   sp.k0 + sp.kb);
            }
        }
    }
    if (depo_traj) {  // the last blocks' windows (every block's but the last, as above)
        for (int bw = std::max(0, n_blocks - depo_lag); bw + 1 < n_blocks; bw++) {
            HIPCK(hipStreamWaitEvent(sT, p->ev_S[bw % R], 0));
            const int cap = (int)(first ? (bw == 0 ? first : first + (long)bw * kb) : std::min<long>((long)(bw + 1) * kb, n_steps));
            hipLaunchKernelGGL(k_depo_elim, dim3(G), dim3(64), 0, sT, *fa, ds, sp.sinfo, cap);
            hipLaunchKernelGGL(k_depo_walk, dim3(G), dim3(64), fit_lds, sT, *fa, ds, sp.sinfo, cap);
        }
    }
    TORJ_SPLIT_DISPATCH(k_split_final, dim3(G), dim3(64), 0, s3, a, sp);
#undef TORJ_SPLIT_DISPATCH
    if (!serial) {  // join: the final kernel followed every scan, each scan its alpha kernel
                    // and each alpha kernel its trajectory
        HIPCK(hipEventRecord(p->ev_J, s3));
        HIPCK(hipStreamWaitEvent(s, p->ev_J, 0));
        if (depo_own || depo_traj) {
            HIPCK(hipEventRecord(p->ev_D, depo_traj ? sT : sD));
            HIPCK(hipStreamWaitEvent(s, p->ev_D, 0));
        }
    }
    HIPCK(hipGetLastError());
    return 0;
}

extern "C" {

int torj_trace_device(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                      const double *N0, const double *weights, int n_psi, const double *grid,
                      double *state, int *status, int *steps, double *dP, double *Pdep,
                      double *traj, uint64_t *counters, void *stream) {
    return torj_trace_device_ex(p, cfg, n, x0, N0, weights, n_psi, grid, nullptr, nullptr, state,
                                status, steps, dP, Pdep, traj, counters, stream);
}

}  // extern "C"

static int trace_device_one(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                            const double *N0, const double *weights, int n_psi, const double *grid,
                            const double *x_launch, const double *s0, double *state, int *status,
                            int *steps, double *dP, double *Pdep, double *traj, uint64_t *counters,
                            void *stream);

// Device-memory budget of one launch's per-ray workspace (the reference
// deposition's per-step samples and elimination coefficients, root counts and
// shell arrays: ~116 KB per ray at 2 000 steps and 1 000 shells).  A beam whose
// workspace would exceed it is traced in contiguous batches of whole 64-ray
// groups, each batch's inputs gathered into and outputs scattered from
// compact device buffers.  TORJ_WS_GB (read per call, tests vary it) sets the
// budget; by default it is half of the device memory this handle could use
// (free + its own fit workspace, which a larger one replaces), at least 16 GiB:
// on a 288 GB MI355X the 1e6-ray C4 beam (~116 GB) then runs as one launch
// (606 against 675 ms in seven 16 GiB batches, each with its own pipeline fill
// and drain), with room left for the split ring and the caller's buffers.
// The device must be current (ensure_device).
static size_t ws_budget(const torj_plasma_s *p) {
    const char *e = getenv("TORJ_WS_GB");
    if (e) return (size_t)(atof(e) * (double)(1ull << 30));
    const size_t floor16 = 16ull << 30;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return floor16;
    return std::max(floor16, (free_b + p->fit_cap) / 2);
}

static int ensure_batch(torj_plasma_s *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->batch_cap >= bytes) return 0;
    if (p->d_batch) HIPCK(hipFree(p->d_batch));
    p->d_batch = nullptr;
    p->batch_cap = 0;
    HIPCK(hipMalloc(&p->d_batch, bytes));
    p->batch_cap = bytes;
    return 0;
}

extern "C" {

int torj_trace_device_ex(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                         const double *N0, const double *weights, int n_psi, const double *grid,
                         const double *x_launch, const double *s0, double *state, int *status,
                         int *steps, double *dP, double *Pdep, double *traj, uint64_t *counters,
                         void *stream) {
    if (!p || !cfg) return fail("bad plasma handle or cfg");
    if (n <= 0) return 0;
    if (!stream) {
        // the NULL (legacy default) stream as the caller's: the trace runs on the
        // handle's own non-blocking stream, after the NULL stream's earlier work
        // and before its later work (the same ordering); enqueued on the NULL
        // stream itself the trace phase ran ~0.4 ms slower per headline launch
        // (implicit synchronisation with the blocking streams)
        if (ensure_device(p)) return -1;
        if (!p->ev_Nin) {
            HIPCK(hipEventCreateWithFlags(&p->ev_Nin, hipEventDisableTiming));
            HIPCK(hipEventCreateWithFlags(&p->ev_Nout, hipEventDisableTiming));
        }
        HIPCK(hipEventRecord(p->ev_Nin, nullptr));
        HIPCK(hipStreamWaitEvent(p->stream, p->ev_Nin, 0));
        const int rc = torj_trace_device_ex(p, cfg, n, x0, N0, weights, n_psi, grid, x_launch, s0, state,
                                            status, steps, dP, Pdep, traj, counters, p->stream);
        HIPCK(hipEventRecord(p->ev_Nout, p->stream));
        HIPCK(hipStreamWaitEvent(nullptr, p->ev_Nout, 0));
        return rc;
    }
    if (p->timing) p->timing_calls++;
    const bool fit = n_psi >= 2 && grid && dP && cfg->deposition == 1;
    // TORJ_SPLIT_BATCH=R (read per call; fixed-step absorbing beams): trace in
    // contiguous batches of R rays (a multiple of 64), each its own pipeline
    const char *sb_e = getenv("TORJ_SPLIT_BATCH");
    const long sb_rays = (sb_e && cfg->integrator == 0 && cfg->absorption >= 1) ? atol(sb_e) / 64 * 64 : 0;
    if ((fit || sb_rays > 0) && cfg->n_steps > 0 && x0 && N0 && state && status && steps) {
        const size_t K = (size_t)cfg->n_steps + 2, L = (size_t)n_psi;
        const size_t per_ray = fit ? (cfg->integrator == 1 ? 6 : 5) * 8 * K + 4 * (L + 1) + 16 * L + 4 : 0;
        if (ensure_device(p)) return -1;
        const size_t budget = ws_budget(p);
        size_t nb_ws = fit && (size_t)n * per_ray > budget ? std::max<size_t>(64, budget / per_ray / 64 * 64) : (size_t)n;
        if (sb_rays > 0 && (size_t)sb_rays < nb_ws) nb_ws = (size_t)sb_rays;
        if (nb_ws < (size_t)n) {
            const int nb = (int)nb_ws;
            hipStream_t s = (hipStream_t)stream;
            const int n_save = cfg->traj_stride > 0 && traj ? cfg->n_steps / cfg->traj_stride : 0;
            const size_t D = sizeof(double), B = (size_t)nb;
            // staging: x0, N0, x_launch (3 rows), w, s0, P_dep (1), state (7), traj (5 n_save);
            // status, steps (int)
            const size_t rows = 3 + 3 + 3 + 1 + 1 + 1 + 7 + 5 * (size_t)n_save;
            if (ensure_batch(p, rows * B * D + 2 * B * sizeof(int))) return -1;
            double *q = (double *)p->d_batch;
            double *bx0 = q, *bN0 = bx0 + 3 * B, *bxl = bN0 + 3 * B, *bw = bxl + 3 * B, *bs0 = bw + B,
                   *bP = bs0 + B, *bst = bP + B, *btr = bst + 7 * B;
            int *bstat = (int *)(btr + 5 * (size_t)n_save * B), *bsteps = bstat + B;
            for (int lo = 0; lo < n; lo += nb) {
                const int c = std::min(nb, n - lo);
                auto gather = [&](double *d, const double *h, int r) -> int {
                    if (!h) return 0;
                    HIPCK(hipMemcpy2DAsync(d, c * D, h + lo, (size_t)n * D, c * D, r,
                                           hipMemcpyDeviceToDevice, s));
                    return 0;
                };
                auto scatter = [&](double *h, const double *d, int r) -> int {
                    if (!h) return 0;
                    HIPCK(hipMemcpy2DAsync(h + lo, (size_t)n * D, d, c * D, c * D, r,
                                           hipMemcpyDeviceToDevice, s));
                    return 0;
                };
                if (gather(bx0, x0, 3) || gather(bN0, N0, 3) || gather(bxl, x_launch, 3) ||
                    gather(bw, weights, 1) || gather(bs0, s0, 1))
                    return -1;
                if (trace_device_one(p, cfg, c, bx0, bN0, weights ? bw : nullptr, n_psi, grid,
                                     x_launch ? bxl : nullptr, s0 ? bs0 : nullptr, bst, bstat, bsteps,
                                     dP, bP, n_save ? btr : nullptr, counters, stream))
                    return -1;
                if (scatter(state, bst, 7) || scatter(Pdep, bP, 1) ||
                    scatter(n_save ? traj : nullptr, btr, 5 * n_save))
                    return -1;
                HIPCK(hipMemcpyAsync(status + lo, bstat, c * sizeof(int), hipMemcpyDeviceToDevice, s));
                HIPCK(hipMemcpyAsync(steps + lo, bsteps, c * sizeof(int), hipMemcpyDeviceToDevice, s));
            }
            return 0;
        }
    }
    return trace_device_one(p, cfg, n, x0, N0, weights, n_psi, grid, x_launch, s0, state, status,
                            steps, dP, Pdep, traj, counters, stream);
}

}  // extern "C"

// one launch of the hot path over n rays (the body of torj_trace_device_ex)
static int trace_device_one(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                            const double *N0, const double *weights, int n_psi, const double *grid,
                            const double *x_launch, const double *s0, double *state, int *status,
                            int *steps, double *dP, double *Pdep, double *traj, uint64_t *counters,
                            void *stream) {
    if (n <= 0) return 0;
    if (!x0 || !N0 || !state || !status || !steps) return fail("x0, N0, state, status, steps required");
    if (cfg->n_steps < 0) return fail("n_steps < 0");
    if (cfg->mode != 1 && cfg->mode != -1) return fail("mode must be +1 (X) or -1 (O)");
    if (!(cfg->ds > 0)) return fail("ds must be > 0");
    if (cfg->deposition != 0 && cfg->deposition != 1) return fail("deposition must be 0 or 1");
    if (cfg->integrator != 0 && cfg->integrator != 1) return fail("integrator must be 0 or 1");
    if (cfg->integrator == 1 && (!(cfg->s_max > 0) || cfg->n_chunks < 1 || !(cfg->abstol > 0) ||
                                 !(cfg->reltol > 0) || cfg->n_steps < 1))
        return fail("integrator 1 needs s_max > 0, n_chunks >= 1, abstol, reltol > 0, n_steps >= 1");
    const bool depo = n_psi >= 2 && grid && dP;
    const bool fit = depo && cfg->deposition == 1;
    if (fit && (!x_launch || !s0))
        return fail("deposition = 1 (reference profile) needs x_launch and s0 (torj_trace_ex)");
    const bool tr = cfg->traj_stride > 0 && traj;
    if (ensure_device(p)) return -1;
    if (cfg->absorption < 0 || cfg->absorption > 3) return fail("absorption must be 0..3");
    if (cfg->absorption == 1 && ensure_gl_on_device(p->device)) return -1;
    hipStream_t s = (hipStream_t)stream;
    TraceArgs a{};
    a.coef = p->d_coef;
    a.cellp = p->d_cellp;
    a.g = p->g;
    a.k = make_consts(cfg->omega);
    a.omega = cfg->omega;
    a.mode = cfg->mode;
    a.ds = cfg->ds;
    a.n_steps = cfg->n_steps;
    a.chunk_steps = cfg->chunk_steps;
    a.psi_exit = cfg->psi_exit;
    a.P_min = cfg->P_min;
    a.n = n;
    a.x0 = x0;
    a.N0 = N0;
    a.w = weights;
    a.state = state;
    a.status = status;
    a.steps = steps;
    a.counters = (unsigned long long *)counters;
    a.s0 = s0;
    a.abs_model = cfg->absorption;
    if (cfg->integrator == 1) {
        a.abstol = cfg->abstol;
        a.reltol = cfg->reltol;
        a.s_step = cfg->s_max / cfg->n_chunks;
        a.n_chunks = cfg->n_chunks;
        if (ensure_chunks(p, (size_t)n)) return -1;
        a.chunk = p->d_chunk;
    }
    if (depo) {
        a.n_psi = n_psi;
        a.grid = grid;  // uniform-grid fast path is set up in-kernel from grid[0], grid[n-1]
        a.dP = dP;
        if (!Pdep) {  // the work-queue kernel carries P_dep across chunks: workspace
            if (ensure_workspace(p, (size_t)n)) return -1;
            Pdep = p->d_ws;
        }
        a.Pdep = Pdep;
    }
    FitArgs fa{};
    if (fit) {
        // samples (psi, dP/ds) per step, Thomas/second-derivative arrays,
        // per-boundary root counts, per-shell open-root integrals
        const size_t K = (size_t)cfg->n_steps + 2, N = (size_t)n, L = (size_t)n_psi;
        const size_t KN = smp_elems(N, K);  // smp_at layout: 64-ray blocks of K rows
        // arc lengths are stored by the adaptive integrator only (RK4: s0 + k ds)
        const size_t n_smp = cfg->integrator == 1 ? 3 : 2;
        const size_t b_smp = n_smp * KN * sizeof(double), b_m = 3 * KN * sizeof(double);
        const size_t b_cnt = ((L + 1) * N * sizeof(int) + 255) & ~(size_t)255, b_fo = L * N * sizeof(double);
        const size_t b_ks = (N * sizeof(int) + 255) & ~(size_t)255;
        if (ensure_fit(p, b_smp + b_m + b_cnt + 2 * b_fo + b_ks)) return -1;
        char *base = (char *)p->d_fit;
        a.smp_psi = (double *)base;
        a.smp_dpds = a.smp_psi + KN;
        a.smp_s = cfg->integrator == 1 ? a.smp_dpds + KN : nullptr;
        a.smp_rows = K;
        fa.rows = K;
        fa.E = (double *)(base + b_smp);
        fa.Gpsi = fa.E + KN;
        fa.GP = fa.Gpsi + KN;
        fa.cnt = (int *)(base + b_smp + b_m);
        fa.Fopen = (double *)(base + b_smp + b_m + b_cnt);
        fa.dPs = fa.Fopen + L * N;
        fa.kstar = (int *)(base + b_smp + b_m + b_cnt + 2 * b_fo);
        // (the walk's per-boundary / per-shell arrays are cleared by fit_zero:
        // on the split path on its scan stream, beside the first trajectory
        // block, else on `s` before the trace)
        fa.coef = p->d_coef;
        fa.g = p->g;
        fa.n = n;
        fa.n_psi = n_psi;
        fa.ds = cfg->ds;
        fa.grid = grid;
        fa.w = weights;
        fa.x_launch = x_launch;
        fa.s0 = s0;
        fa.steps = steps;
        fa.smp_psi = a.smp_psi;
        fa.smp_dpds = a.smp_dpds;
        fa.smp_s = a.smp_s;
        fa.s_uniform = cfg->integrator == 0;  // RK4: s_k = s0 + k ds, not stored
        fa.dP = dP;
        fa.Pray = Pdep;
        // boundary lookups guess from grid[0], grid[n-1] in-kernel and correct
        // locally: no host read of the (device-resident) grid, no stream sync
    }
    if (depo)  // psi_dP_dV strictly increasing: checked on the device, reported by torj_trace_check
        hipLaunchKernelGGL(k_grid_check, dim3(1), dim3(256), 0, s, grid, n_psi, p->d_flags);
    const int DM = !depo ? kDepoNone : (fit ? kDepoSamples : kDepoBinned);
    DepoStream dstr{};  // the split pipeline's streamed deposition (split_trace)
    if (tr) {
        a.traj_stride = cfg->traj_stride;
        a.n_save = cfg->n_steps / cfg->traj_stride;
        a.traj = traj;
        if (a.n_save > 0)
            HIPCK(hipMemsetAsync(traj, 0xFF, (size_t)a.n_save * 5 * n * sizeof(double), s));  // NaN
    }
    static const int sched_env = [] {
        const char *e = getenv("TORJ_SCHED");
        return e ? atoi(e) : 1;
    }();
    const int G = (n + TORJ_GROUP - 1) / TORJ_GROUP;
    const int cs = cfg->chunk_steps > 0 ? cfg->chunk_steps : std::max(cfg->n_steps, 1);
    // default: the queue pays off once the beam exceeds one wave per SIMD
    // (measured: 42k rays 111 vs 106 ms one-shot; 100k rays 151 vs 174 ms)
    const bool adaptive = cfg->integrator == 1;
    const int use_sched = adaptive || cfg->absorption >= 2
                              ? 1  // the adaptive path runs one tspan chunk per visit; warm always queues
                                   : p->sched_mode >= 0 ? p->sched_mode
                                                        : (sched_env && G > p->n_cu * 4 ? 1 : 0);
// every <absorption, deposition mode, trajectory> instance of a trace kernel
// (warm models: the TRAJ instance only, with traj_stride = 0 when no
// trajectory is wanted -- fewer instances of the heavy warm code)
#define TORJ_DISPATCH_T(L, A, D)            \
    do {                                    \
        if (tr)                             \
            L(A, D, true);                  \
        else                                \
            L(A, D, ((A) >= 2 ? true : false)); \
    } while (0)
#define TORJ_DISPATCH_D(L, A)                                 \
    do {                                                      \
        if (DM == kDepoBinned)                                \
            TORJ_DISPATCH_T(L, A, kDepoBinned);               \
        else if (DM == kDepoSamples)                          \
            TORJ_DISPATCH_T(L, A, kDepoSamples);              \
        else                                                  \
            TORJ_DISPATCH_T(L, A, kDepoNone);                 \
    } while (0)
#define TORJ_DISPATCH_TRACE(L)              \
    do {                                    \
        if (cfg->absorption == 3)           \
            TORJ_DISPATCH_D(L, 3);          \
        else if (cfg->absorption == 2)      \
            TORJ_DISPATCH_D(L, 2);          \
        else if (cfg->absorption == 1)      \
            TORJ_DISPATCH_D(L, 1);          \
        else                                \
            TORJ_DISPATCH_D(L, 0);          \
    } while (0)
// the one-lane-per-ray kernel: cold and Albajar only (warm always queues)
#define TORJ_DISPATCH_TRACE01(L)            \
    do {                                    \
        if (cfg->absorption == 1)           \
            TORJ_DISPATCH_D(L, 1);          \
        else                                \
            TORJ_DISPATCH_D(L, 0);          \
    } while (0)
    static const int split_env = [] {
        const char *e = getenv("TORJ_SPLIT");
        return e ? atoi(e) : 1;
    }();
    static const int split_warm_env = [] {  // -1 auto, 0 off, 1 on
        const char *e = getenv("TORJ_SPLIT_WARM");
        return e ? atoi(e) : -1;
    }();
    // the split RK4 path (fixed steps; sched mode 3 forces it):
    //  * Albajar: by default for beams that would use the work queue;
    //  * warm weakly relativistic (2): by default -- its alpha kernel runs two
    //    waves per SIMD where the fused queue kernel holds one (C5: 165 vs 221 ms);
    //  * warm fully relativistic (3): by default for beams of fewer 64-ray groups
    //    than 3 per CU, where the one-wave-per-SIMD queue kernel leaves SIMDs idle
    //    and the split's alpha kernel spreads the points over all of them (129
    //    rays: 13.1 s -> 0.1 s); on the 1e5-ray fan the queue kernel is faster
    //    (19.7 vs 20.4 s)
    const bool albajar_split = cfg->absorption == 1 && split_env == 1 && sched_env && G > p->n_cu * 4;
    const bool warm_split = cfg->absorption >= 2 && split_env == 1 &&
                            (split_warm_env == 1 ||
                             (split_warm_env < 0 && (cfg->absorption == 2 || G < p->n_cu * 3)));
    // (the split kernels pack a ray's step count into 24 bits beside its status)
    const bool use_split = !adaptive && cfg->absorption >= 1 && cfg->n_steps > 0 &&
                           cfg->n_steps < kSplitMaxSteps &&
                           (p->sched_mode == 3 || (p->sched_mode < 0 && (albajar_split || warm_split)));
    // the fused / queue paths clear the deposition workspace before the trace
    // phase's first event (outside trace_ms, as before round 5); the split path
    // clears it on its scan stream, overlapped with the first trajectory block
    if (fit && !use_split && fit_zero(fa, s)) return -1;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    if (p->timing) {
        if (p->ev_used + 3 > p->ev_pool.size()) {
            for (int q = 0; q < 3; q++) {
                hipEvent_t e;
                HIPCK(hipEventCreate(&e));
                p->ev_pool.push_back(e);
            }
        }
        for (int q = 0; q < 3; q++) ev[q] = p->ev_pool[p->ev_used + q];
        p->ev_used += 3;
        HIPCK(hipEventRecord(ev[0], s));
    }
    if (use_split) {
        if (split_trace(p, a, DM, tr, cs, s, fit ? &fa : nullptr, &dstr)) return -1;
    } else if (use_sched && cfg->n_steps > 0) {
        // W persistent waves: at most 2 per SIMD (4 SIMDs per CU), and fewer
        // than G so the ready queue keeps a backlog (a wave never waits for a
        // group while another holds it); TORJ_SCHED_W overrides.
        static const int w_env = [] {
            const char *e = getenv("TORJ_SCHED_W");
            return e ? atoi(e) : 0;
        }();
        int W = p->sched_waves > 0 ? p->sched_waves
                : w_env > 0        ? w_env
                                   : std::min(p->n_cu * 4 * (cfg->absorption >= 2 ? TORJ_WARM_MIN_WAVES
                                                                                  : TORJ_MIN_WAVES),
                                              G - G / 16);
        W = std::max(1, std::min(W, G));
        const unsigned S = 4u * (unsigned)(G + W);  // ring slots (tag check makes reuse safe)
        const size_t bytes = 256 + (size_t)S * sizeof(unsigned long long);
        if (ensure_sched(p, bytes)) return -1;
        HIPCK(hipMemsetAsync(p->d_sched, 0, bytes, s));
        SchedCtl *ctl = (SchedCtl *)p->d_sched;
        unsigned long long *slots = (unsigned long long *)((char *)p->d_sched + 256);
        const dim3 grd(W), blk(64);
        // binned shells: a per-wave LDS histogram (RK4, up to 4096 shells; the
        // adaptive path's 25 KB of stage vectors leave no room without losing
        // occupancy, it keeps the global atomics)
        a.hist_off = adaptive ? kTsLds : 0;
        a.n_hist = (DM == kDepoBinned && !adaptive && n_psi <= 4096) ? n_psi : 0;
        const size_t lds = (size_t)(a.hist_off + a.n_hist) * sizeof(double);
#define LAUNCH(A, D, T)                                                                            \
    do {                                                                                           \
        if (adaptive)                                                                              \
            hipLaunchKernelGGL((k_trace_sched<A, D, T, 1>), grd, blk, lds, s, a, ctl, slots, S, G, cs); \
        else                                                                                       \
            hipLaunchKernelGGL((k_trace_sched<A, D, T, 0>), grd, blk, lds, s, a, ctl, slots, S, G, cs); \
    } while (0)
        TORJ_DISPATCH_TRACE(LAUNCH);
#undef LAUNCH
        // the queue's watchdog / retirement state into the sticky flags
        hipLaunchKernelGGL(k_sched_fold, dim3(1), dim3(1), 0, s, ctl, (unsigned)G, p->d_flags);
    } else {
        // small Albajar beams: 16 lanes per ray while n x 16 lanes fit two
        // waves per SIMD (the latency of a ray's step chain sets the time there)
        // (TORJ_LPR=1 in the environment turns the automatic choice off)
        static const int lpr_env = [] {
            const char *e = getenv("TORJ_LPR");
            return e ? atoi(e) : 0;
        }();
        const bool split = cfg->absorption == 1 && DM != kDepoBinned && p->lanes_per_ray != 1 &&
                           (p->lanes_per_ray == 16 ||
                            (lpr_env != 1 && (size_t)n * 16 <= (size_t)p->n_cu * 4 * 2 * 64));
        const dim3 blk(TORJ_BLOCK);
        if (split) {
            const dim3 grd(nblocks(n * 16, TORJ_BLOCK));
            if (DM == kDepoSamples) {
                if (tr)
                    hipLaunchKernelGGL((k_trace<1, kDepoSamples, true, 16>), grd, blk, 0, s, a);
                else
                    hipLaunchKernelGGL((k_trace<1, kDepoSamples, false, 16>), grd, blk, 0, s, a);
            } else {
                if (tr)
                    hipLaunchKernelGGL((k_trace<1, kDepoNone, true, 16>), grd, blk, 0, s, a);
                else
                    hipLaunchKernelGGL((k_trace<1, kDepoNone, false, 16>), grd, blk, 0, s, a);
            }
        } else {
            const dim3 grd(nblocks(n, TORJ_BLOCK));
#define LAUNCH(A, D, T) hipLaunchKernelGGL((k_trace<A, D, T>), grd, blk, 0, s, a)
            TORJ_DISPATCH_TRACE01(LAUNCH);
#undef LAUNCH
        }
    }
    HIPCK(hipGetLastError());
    if (ev[1]) HIPCK(hipEventRecord(ev[1], s));
    if (fit) {
        if (adaptive)
            ;  // the last accepted step's FSAL stage already gave P alpha there
        else if (cfg->absorption == 3)
            hipLaunchKernelGGL(k_final_alpha<3>, dim3(nblocks(n, 64)), dim3(64), 0, s, a);
        else if (cfg->absorption == 2)
            hipLaunchKernelGGL(k_final_alpha<2>, dim3(nblocks(n, 64)), dim3(64), 0, s, a);
        else if (cfg->absorption == 1)
            hipLaunchKernelGGL(k_final_alpha<1>, dim3(nblocks(n, 64)), dim3(64), 0, s, a);
        else
            hipLaunchKernelGGL(k_final_alpha<0>, dim3(nblocks(n, 64)), dim3(64), 0, s, a);
        const size_t lds = n_psi <= kFitGridLds ? (size_t)n_psi * sizeof(double) : 0;
        if (dstr.v)  // the streamed walk's windows ran behind the scans
            hipLaunchKernelGGL(k_depo_tail, dim3(nblocks(n, 64)), dim3(64), lds, s, fa, dstr);
        else
            hipLaunchKernelGGL(k_fit_depo, dim3(nblocks(n, 64)), dim3(64), lds, s, fa);
        hipLaunchKernelGGL(k_shell_sum, dim3(n_psi), dim3(256), 0, s, fa);
        HIPCK(hipGetLastError());
    }
    if (ev[2]) HIPCK(hipEventRecord(ev[2], s));
    return 0;
}

extern "C" {

int torj_power_deposition_profile(torj_plasma_t p, int n_rays, const int *n_points, const double *s,
                                  const double *x, const double *dP_ds, int n_psi,
                                  const double *grid, double *dP_dV, double *P) {
    if (!p) return fail("bad plasma handle");
    if (n_rays < 0 || n_psi < 2 || !grid) return fail("power_deposition_profile: n_rays >= 0, n_psi >= 2 needed");
    if (n_rays == 0) return 0;
    if (!n_points || !s || !x || !dP_ds || !dP_dV || !P) return fail("power_deposition_profile: null argument");
    for (int k = 1; k < n_psi; k++)
        if (!(grid[k] > grid[k - 1])) return fail("psi_dP_dV must be strictly increasing");
    std::vector<long> off(n_rays);
    long tot = 0;
    int rows = 0;
    for (int r = 0; r < n_rays; r++) {
        // Dierckx.Spline1D(s, y, k = 3) needs m > k points with strictly
        // increasing s (FITPACK curfit's input check)
        if (n_points[r] < 4) return fail("power_deposition_profile: ray %d has %d points (need >= 4)", r, n_points[r]);
        for (int j = 1; j < n_points[r]; j++)
            if (!(s[tot + j] > s[tot + j - 1]))
                return fail("power_deposition_profile: s must be strictly increasing (ray %d, point %d)", r, j);
        off[r] = tot;
        tot += n_points[r];
        rows = std::max(rows, n_points[r]);
    }
    if (ensure_device(p)) return -1;
    hipStream_t st = p->stream;
    const size_t N = (size_t)n_rays, L = (size_t)n_psi, K = (size_t)rows, KN = smp_elems(N, K);
    DevBufs B;
    double *d_s, *d_x, *d_dp, *d_grid, *d_smp, *d_Pr;
    int *d_np, *d_kstar, *d_cnt;
    long *d_off;
    if (B.up(&d_s, s, (size_t)tot, st) || B.up(&d_x, x, 3 * (size_t)tot, st) ||
        B.up(&d_dp, dP_ds, (size_t)tot, st) || B.up(&d_grid, grid, L, st) ||
        B.up(&d_np, n_points, N, st) || B.up(&d_off, off.data(), N, st) ||
        B.alloc(&d_smp, 6 * KN + 2 * L * N, true) || B.alloc(&d_cnt, (L + 1) * N, true) ||
        B.alloc(&d_kstar, N, true) || B.alloc(&d_Pr, N, true))
        return -1;
    FitArgs fa{};
    fa.coef = p->d_coef;
    fa.g = p->g;
    fa.n = n_rays;
    fa.n_psi = n_psi;
    fa.grid = d_grid;
    fa.rows = K;
    fa.npts = d_np;
    fa.steps = d_np;
    fa.smp_psi = d_smp;
    fa.smp_dpds = d_smp + KN;
    fa.smp_s = d_smp + 2 * KN;
    fa.E = d_smp + 3 * KN;
    fa.Gpsi = d_smp + 4 * KN;
    fa.GP = d_smp + 5 * KN;
    fa.Fopen = d_smp + 6 * KN;
    fa.dPs = fa.Fopen + L * N;
    fa.cnt = d_cnt;
    fa.kstar = d_kstar;
    fa.Pray = d_Pr;
    HIPCK(hipMemsetAsync(fa.cnt, 0, (L + 1) * N * sizeof(int), st));
    HIPCK(hipMemsetAsync(fa.Fopen, 0xFF, L * N * sizeof(double), st));  // NaN: every shell closed
    HIPCK(hipMemsetAsync(fa.dPs, 0, L * N * sizeof(double), st));
    hipLaunchKernelGGL(k_profile_samples, dim3(nblocks(n_rays, 64)), dim3(64), 0, st, fa, d_off, d_s, d_x,
                       (size_t)tot, d_dp);
    const size_t lds = n_psi <= kFitGridLds ? (size_t)n_psi * sizeof(double) : 0;
    hipLaunchKernelGGL(k_fit_profile, dim3(nblocks(n_rays, 64)), dim3(64), lds, st, fa);
    HIPCK(hipGetLastError());
    std::vector<double> dPs(L * N);
    std::vector<int> kstar(N);
    if (ddownload(dPs.data(), fa.dPs, (L - 1) * N, st) || ddownload(kstar.data(), d_kstar, N, st) ||
        ddownload(P, d_Pr, N, st))
        return -1;
    HIPCK(hipStreamSynchronize(st));
    // dP_dV[j] = dP_j / (V(psi_{j+1}) - V(psi_j)) above the break shell, 0 below it
    // and at the last boundary (src/plasma.jl:141)
    std::vector<double> dV(L - 1);
    if (torj_shell_volumes(p, n_psi, grid, dV.data())) return -1;
    for (size_t r = 0; r < N; r++) {
        double *row = dP_dV + r * L;
        for (size_t j = 0; j < L; j++)
            row[j] = (j + 1 < L && (int)j > kstar[r]) ? dPs[j * N + r] / dV[j] : 0.0;
    }
    return 0;
}

int torj_timing(torj_plasma_t p, int enable) {
    if (!p) return fail("bad plasma handle");
    std::lock_guard<std::mutex> lk(p->mu);
    // the handle and its torj_trace_beam replicas (new replicas inherit it)
    for (size_t k = 0; k < std::max<size_t>(1, p->replicas.size()); k++) {
        torj_plasma_s *q = k == 0 ? p : p->replicas[k];
        q->timing = enable != 0;
        q->ev_used = 0;
        q->timing_calls = 0;
    }
    p->reduce_ms = 0.0;
    p->reduce_calls = 0;
    return 0;
}

int torj_timing_read(torj_plasma_t p, int *calls, double *trace_ms, double *post_ms) {
    if (!p) return fail("bad plasma handle");
    double t = 0.0, q = 0.0;
    for (size_t k = 0; k + 3 <= p->ev_used; k += 3) {
        float a = 0.f, b = 0.f;
        HIPCK(hipEventSynchronize(p->ev_pool[k + 2]));
        HIPCK(hipEventElapsedTime(&a, p->ev_pool[k], p->ev_pool[k + 1]));
        HIPCK(hipEventElapsedTime(&b, p->ev_pool[k + 1], p->ev_pool[k + 2]));
        t += a;
        q += b;
    }
    if (calls) *calls = p->timing_calls;  // a batched call records one triple per batch
    if (trace_ms) *trace_ms = t;
    if (post_ms) *post_ms = q;
    p->ev_used = 0;
    p->timing_calls = 0;
    return 0;
}

int torj_beam_timing_read(torj_plasma_t p, int n_gpus, int *calls, double *trace_ms, double *post_ms,
                          double *reduce_ms) {
    if (!p) return fail("bad plasma handle");
    if (n_gpus < 1) return fail("n_gpus must be >= 1");
    int dev0 = 0;
    HIPCK(hipGetDevice(&dev0));
    // the replica list (torj_timing and beam_replicas take it too): held from the
    // range check on, so a concurrent fan-out cannot change it in between
    std::lock_guard<std::mutex> lk(p->mu);
    if (n_gpus > std::max<int>(1, (int)p->replicas.size()))
        return fail("n_gpus = %d, but the handle has %d replica(s)", n_gpus, std::max<int>(1, (int)p->replicas.size()));
    int rc = 0;
    for (int k = 0; k < n_gpus && rc == 0; k++) {
        torj_plasma_s *q = k == 0 ? p : p->replicas[k];
        if (hipSetDevice(q->device) != hipSuccess)
            rc = fail("hipSetDevice(%d) failed", q->device);
        else if (torj_timing_read(q, calls ? calls + k : nullptr, trace_ms ? trace_ms + k : nullptr,
                                  post_ms ? post_ms + k : nullptr))
            rc = -1;
    }
    (void)hipSetDevice(dev0);  // the caller's device on every path
    if (rc) return rc;
    if (reduce_ms) *reduce_ms = p->reduce_ms;
    p->reduce_ms = 0.0;
    p->reduce_calls = 0;
    return 0;
}

int torj_beam_comm_info(torj_plasma_t p, int n_gpus, int *device, int *nranks, int *rank) {
    if (!p) return fail("bad plasma handle");
    if (n_gpus < 1) return fail("n_gpus must be >= 1");
    if (!device || !nranks || !rank) return fail("device, nranks and rank must be arrays of n_gpus");
    std::lock_guard<std::mutex> lk(p->mu);
    if (n_gpus > std::max<int>(1, (int)p->replicas.size()))
        return fail("n_gpus = %d, but the handle has %d replica(s)", n_gpus, std::max<int>(1, (int)p->replicas.size()));
    // the communicator of the last RCCL reduce (beam_reduce_run keeps one per
    // replica of that fan-out; rebuilt when the replica count changes)
    const bool comm = (int)p->comms.size() == n_gpus;
    for (int k = 0; k < n_gpus; k++) {
        device[k] = (k == 0 ? p : p->replicas[k])->device;
        nranks[k] = 0;
        rank[k] = -1;
        if (comm && p->comms[k]) {
            if (ncclCommCount(p->comms[k], nranks + k) != ncclSuccess ||
                ncclCommUserRank(p->comms[k], rank + k) != ncclSuccess)
                return fail("ncclCommCount / ncclCommUserRank failed for replica %d", k);
        }
    }
    return 0;
}

int torj_set_sched(torj_plasma_t p, int mode, int waves) {
    if (!p) return fail("bad plasma handle");
    if (mode < -1 || mode > 3) return fail("sched mode must be -1, 0, 1, 2 or 3");
    if (waves < 0) return fail("waves must be >= 0");
    p->sched_mode = mode == 2 ? 0 : mode;
    p->lanes_per_ray = mode == 0 ? 1 : (mode == 2 ? 16 : 0);
    p->sched_waves = waves;
    return 0;
}

int torj_trace(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
               const double *N0, const double *weights, int n_psi, const double *grid,
               double *state, int *status, int *steps, double *dP, double *Pdep, double *traj) {
    return torj_trace_ex(p, cfg, n, x0, N0, weights, n_psi, grid, nullptr, nullptr, state, status,
                         steps, dP, Pdep, traj);
}

int torj_trace_ex(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                  const double *N0, const double *weights, int n_psi, const double *grid,
                  const double *x_launch, const double *s0, double *state, int *status,
                  int *steps, double *dP, double *Pdep, double *traj) {
    if (!p || !cfg) return fail("bad plasma handle or cfg");
    if (n <= 0) return 0;
    const bool depo = n_psi >= 2 && grid;
    if (depo)  // host copy at hand: checked before any device work
        for (int k = 1; k < n_psi; k++)
            if (!(grid[k] > grid[k - 1])) return fail("psi_dP_dV must be strictly increasing");
    if (ensure_device(p)) return -1;
    hipStream_t s = p->stream;
    const int n_save = cfg->traj_stride > 0 ? cfg->n_steps / cfg->traj_stride : 0;
    DevBufs B;
    double *dx0, *dN0, *dw = nullptr, *dgrid = nullptr, *dstate, *ddP = nullptr, *dPdep = nullptr,
                                *dtraj = nullptr;
    int *dstatus, *dsteps;
    if (B.up(&dx0, x0, 3 * (size_t)n, s) || B.up(&dN0, N0, 3 * (size_t)n, s)) return -1;
    if (weights) {
        if (B.up(&dw, weights, n, s)) return -1;
    }
    if (depo) {
        if (B.up(&dgrid, grid, n_psi, s) || B.alloc(&ddP, n_psi + 1, true) ||
            B.alloc(&dPdep, n, true))
            return -1;
        HIPCK(hipMemsetAsync(ddP, 0, (n_psi + 1) * sizeof(double), s));
    }
    if (B.alloc(&dstate, 7 * (size_t)n, true) || B.alloc(&dstatus, n, true) ||
        B.alloc(&dsteps, n, true))
        return -1;
    if (traj && n_save > 0) {
        if (B.alloc(&dtraj, (size_t)n_save * 5 * n, true)) return -1;
    }
    double *dxl = nullptr, *ds0 = nullptr;
    if (x_launch) {
        if (B.up(&dxl, x_launch, 3 * (size_t)n, s)) return -1;
    }
    if (s0) {
        if (B.up(&ds0, s0, n, s)) return -1;
    }
    if (torj_trace_device_ex(p, cfg, n, dx0, dN0, dw, depo ? n_psi : 0, dgrid, dxl, ds0, dstate,
                             dstatus, dsteps, ddP, dPdep, dtraj, nullptr, s))
        return -1;
    if (ddownload(state, dstate, 7 * (size_t)n, s) || ddownload(status, dstatus, n, s) ||
        ddownload(steps, dsteps, n, s))
        return -1;
    if (depo) {
        if (ddownload(dP, ddP, n_psi + 1, s) || ddownload(Pdep, dPdep, n, s)) return -1;
    } else {
        if (dP) std::fill(dP, dP + (n_psi > 0 ? n_psi + 1 : 1), 0.0);
        if (Pdep) std::fill(Pdep, Pdep + n, 0.0);
    }
    if (traj && n_save > 0 && ddownload(traj, dtraj, (size_t)n_save * 5 * n, s)) return -1;
    return torj_trace_check(p, s);
}

}  // extern "C"

// ---- make_beam across the GPUs of this process (src/solve.jl:209-240) -----
// Replica k of a plasma handle: the same coefficients on device (device + k)
// mod the device count, with its own stream, scratch and scheduling copy.
//
// Test-only placement: env TORJ_BEAM_SAME_DEVICE=1 (read per call) puts every
// replica on the handle's own device, so the multi-replica branch -- one host
// thread, stream and workspace per replica -- runs on a one-GPU machine.  RCCL
// rejects a communicator with a device twice, so those partials are summed on
// the host, in replica order, instead of by the all-reduce.
static bool beam_same_device() {
    const char *e = getenv("TORJ_BEAM_SAME_DEVICE");
    return e && atoi(e) != 0;
}

static int beam_replicas(torj_plasma_s *p, int n_gpus, bool same) {
    int ndev = 0;
    HIPCK(hipGetDeviceCount(&ndev));
    if (n_gpus < 1 || (!same && n_gpus > ndev))
        return fail("n_gpus = %d, but %d HIP devices are visible", n_gpus, ndev);
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->replicas.empty()) p->replicas.push_back(p);
    auto dev_of = [&](size_t k) { return same ? p->device : (p->device + (int)k) % ndev; };
    for (size_t k = 1; k < p->replicas.size(); k++)
        if (p->replicas[k]->device != dev_of(k)) {  // placement changed: rebuild them all
            for (ncclComm_t c : p->comms) (void)ncclCommDestroy(c);
            p->comms.clear();
            for (size_t j = 1; j < p->replicas.size(); j++) torj_plasma_destroy(p->replicas[j]);
            p->replicas.resize(1);
            break;
        }
    while ((int)p->replicas.size() < n_gpus) {
        auto *q = new torj_plasma_s();
        q->device = dev_of(p->replicas.size());
        q->g = p->g;
        q->coef = p->coef;
        q->n_vol = p->n_vol;
        q->v1 = p->v1;
        q->vn = p->vn;
        q->vol_coef = p->vol_coef;
        q->psi_prof_max = p->psi_prof_max;
        q->timing = p->timing;
        p->replicas.push_back(q);
    }
    for (int k = 1; k < n_gpus; k++) {  // scheduling knobs follow the base handle
        p->replicas[k]->sched_mode = p->sched_mode;
        p->replicas[k]->sched_waves = p->sched_waves;
        p->replicas[k]->lanes_per_ray = p->lanes_per_ray;
    }
    return 0;
}

// Run f(k) for k < n_gpus: inline for one replica, else one host thread per
// replica (each drives its own device and stream).  Returns the first failure,
// naming its device.
template <class F>
static int beam_fanout(torj_plasma_s *p, int n_gpus, const char *what, F &&f) {
    std::vector<std::string> errs(n_gpus);
    std::vector<int> rc(n_gpus, 0);
    auto run = [&](int k) {
        rc[k] = -1;
        if (hipSetDevice(p->replicas[k]->device) != hipSuccess) {
            errs[k] = "hipSetDevice failed";
            return;
        }
        rc[k] = f(k);
        if (rc[k]) errs[k] = g_err;
    };
    if (n_gpus == 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < n_gpus; k++) th.emplace_back(run, k);
        for (auto &t : th) t.join();
    }
    for (int k = 0; k < n_gpus; k++)
        if (rc[k]) return fail("%s, device %d: %s", what, p->replicas[k]->device, errs[k].c_str());
    return 0;
}

// make_beam's reduce (src/solve.jl:233-240): d_dP[k] (n_psi + 1 fp64 on replica
// k's device) <- sum over k, in place on every replica (all-reduce semantics).
// RCCL over xGMI from a single-process communicator (ncclCommInitAll, kept on
// the handle) enqueued on the replicas' streams; the test-only same-device
// placement sums on the host.  Synchronous: the replicas' streams are drained.
static int beam_reduce_run(torj_plasma_s *p, int n_gpus, const std::vector<double *> &d_dP,
                           int n_psi, bool same);
static int beam_reduce(torj_plasma_s *p, int n_gpus, const std::vector<double *> &d_dP, int n_psi,
                       bool same) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = beam_reduce_run(p, n_gpus, d_dP, n_psi, same);
    if (p->timing && !rc) {
        p->reduce_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        p->reduce_calls++;
    }
    return rc;
}
static int beam_reduce_run(torj_plasma_s *p, int n_gpus, const std::vector<double *> &d_dP,
                           int n_psi, bool same) {
    const size_t m = (size_t)n_psi + 1;
    if (same) {
        std::vector<double> acc(m, 0.0), part(m);
        for (int k = 0; k < n_gpus; k++) {
            torj_plasma_s *q = p->replicas[k];
            HIPCK(hipSetDevice(q->device));
            HIPCK(hipMemcpyAsync(part.data(), d_dP[k], m * sizeof(double), hipMemcpyDeviceToHost, q->stream));
            HIPCK(hipStreamSynchronize(q->stream));
            for (size_t j = 0; j < m; j++) acc[j] += part[j];
        }
        for (int k = 0; k < n_gpus; k++) {
            torj_plasma_s *q = p->replicas[k];
            HIPCK(hipSetDevice(q->device));
            HIPCK(hipMemcpyAsync(d_dP[k], acc.data(), m * sizeof(double), hipMemcpyHostToDevice, q->stream));
            HIPCK(hipStreamSynchronize(q->stream));
        }
        return 0;
    }
    if ((int)p->comms.size() != n_gpus) {
        for (ncclComm_t c : p->comms) (void)ncclCommDestroy(c);
        p->comms.assign(n_gpus, nullptr);
        std::vector<int> devs(n_gpus);
        for (int k = 0; k < n_gpus; k++) devs[k] = p->replicas[k]->device;
        if (ncclCommInitAll(p->comms.data(), n_gpus, devs.data()) != ncclSuccess) {
            p->comms.clear();
            return fail("ncclCommInitAll over %d devices failed", n_gpus);
        }
    }
    ncclResult_t r = ncclGroupStart();
    for (int k = 0; k < n_gpus && r == ncclSuccess; k++)
        r = ncclAllReduce(d_dP[k], d_dP[k], m, ncclDouble, ncclSum, p->comms[k], p->replicas[k]->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return fail("ncclAllReduce of dP_shell failed: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    for (int k = 0; k < n_gpus; k++) {
        HIPCK(hipSetDevice(p->replicas[k]->device));
        HIPCK(hipStreamSynchronize(p->replicas[k]->stream));
    }
    return 0;
}

// Contiguous shard k of S over n rays, boundaries on 64-ray (one wave, one
// work-queue group) multiples, so every shard holds the same 64-ray groups as
// the unsplit beam and per-ray results do not depend on the split.
static void beam_shard(int n, int S, int k, int &lo, int &cnt) {
    const long G = (n + 63) / 64;
    const long g0 = G * k / S, g1 = G * (k + 1) / S;
    lo = (int)std::min<long>(g0 * 64, n);
    cnt = (int)std::min<long>(g1 * 64, n) - lo;
}

// The staging of torj_trace_beam on replica q: device and host memory for
// `nslots` (1 or 2) shard slots of `slot` doubles each, the copy stream and the
// events.  The host side is pinned while it fits TORJ_BEAM_PIN_MB (default
// 2048 MiB per replica; the transfers then run at PCIe rate and overlap the
// trace), pageable above it (hipMemcpyAsync stages those copies itself: slower,
// but a beam of huge user shards never fails for want of pinnable memory).
static int beam_stage(torj_plasma_s *q, size_t slot, int nslots) {
    auto &b = q->stage;
    if (!b.sc) {
        HIPCK(hipStreamCreateWithFlags(&b.sc, hipStreamNonBlocking));
        for (int r = 0; r < 2; r++) {
            HIPCK(hipEventCreateWithFlags(&b.up[r], hipEventDisableTiming));
            HIPCK(hipEventCreateWithFlags(&b.tr[r], hipEventDisableTiming));
            HIPCK(hipEventCreateWithFlags(&b.dn[r], hipEventDisableTiming));
        }
    }
    const size_t bytes = (size_t)nslots * slot * sizeof(double);
    if (b.d_cap < bytes) {
        if (b.d) HIPCK(hipFree(b.d));
        b.d = nullptr, b.d_cap = 0;
        HIPCK(hipMalloc(&b.d, bytes));
        b.d_cap = bytes;
    }
    const char *pin_e = getenv("TORJ_BEAM_PIN_MB");
    const size_t pin_max = (size_t)(pin_e ? atol(pin_e) : 2048) << 20;
    const bool pin = bytes <= pin_max;
    if (b.h_cap < bytes || (b.h_pinned && !pin)) {
        if (b.h) {
            if (b.h_pinned)
                HIPCK(hipHostFree(b.h));
            else
                free(b.h);
        }
        b.h = nullptr, b.h_cap = 0;
        if (pin) {
            HIPCK(hipHostMalloc(&b.h, bytes, hipHostMallocDefault));
        } else {
            b.h = malloc(bytes);
            if (!b.h) return fail("torj_trace_beam: host staging of %zu bytes failed", bytes);
        }
        b.h_cap = bytes;
        b.h_pinned = pin;
    }
    return 0;
}

// One device's share of torj_trace_beam: its shards k0, k0 + dk, ... traced on
// the replica's stream from compact device buffers, with dP_shell accumulated
// on the device (d_dP, zeroed here) for the reduce.  Host arrays are the
// caller's (pageable); each shard goes through pinned staging in two slots on
// a copy stream, pipelined so that shard j + 1's upload and shard j - 1's
// download overlap shard j's trace:
//   copy stream  up(0) up(1) [tr 0] dn(0) up(2) [tr 1] dn(1) up(3) ...
//   trace stream        [up 0] trace(0) [up 1, dn of 2 shards back] trace(1) ...
// The host packs shard j + 1's inputs into its pinned slot while shard j
// traces, and unpacks shard j - 2's outputs (waiting for their download)
// before the slot's next download is queued.  A shard's rows are compact
// (row r of an array at r * cnt) on both sides, so each transfer is one copy;
// a slot's input and output blocks sit at fixed offsets (sized for the
// largest shard), so they never overlap across shards of different sizes.
static int beam_worker(torj_plasma_s *q, const torj_trace_cfg *cfg, int n, int S, int k0, int dk,
                       const double *x0, const double *N0, const double *w, int n_psi,
                       const double *grid, const double *xl, const double *s0, double *state,
                       int *status, int *steps, double *P_dep, double *traj, double *d_dP) {
    if (ensure_device(q)) return -1;
    hipStream_t s = q->stream;
    const bool depo = n_psi >= 2 && grid;
    const bool tr_out = traj && cfg->traj_stride > 0 && cfg->n_steps / cfg->traj_stride > 0;
    const int n_save = tr_out ? cfg->n_steps / cfg->traj_stride : 0;
    std::vector<int> los, cnts;  // this device's shards
    int m = 0;
    for (int k = k0; k < S; k += dk) {
        int lo, cnt;
        beam_shard(n, S, k, lo, cnt);
        if (cnt == 0) continue;
        los.push_back(lo), cnts.push_back(cnt);
        m = std::max(m, cnt);
    }
    if (depo) HIPCK(hipMemsetAsync(d_dP, 0, (n_psi + 1) * sizeof(double), s));
    if (m == 0) return 0;
    DevBufs B;
    double *dgrid = nullptr;
    if (depo && B.up(&dgrid, grid, n_psi, s)) return -1;
    // rows per shard: inputs x0 N0 [w] [x_launch] [s0]; outputs state [P_dep]
    // [traj], then status and steps (two int rows in one double row)
    const int n_in = 6 + (w ? 1 : 0) + (xl ? 3 : 0) + (s0 ? 1 : 0);
    const int n_out = 7 + (depo ? 1 : 0) + n_save * 5 + 1;
    const size_t slot = (size_t)(n_in + n_out) * m;
    const int nk = (int)los.size();
    if (beam_stage(q, slot, nk > 1 ? 2 : 1)) return -1;  // one shard: no second slot
    auto &bs = q->stage;
    double *dbase = (double *)bs.d, *hbase = (double *)bs.h;
    struct View {  // one slot's arrays for a shard of cnt rays
        double *x0, *N0, *w, *xl, *s0, *state, *Pdep, *traj;
        int *status, *steps;
        double *in, *out;  // the contiguous input / output blocks
        size_t n_in, n_out;  // their sizes in doubles
    };
    auto view = [&](double *base, int r, int cnt) {
        View v{};
        double *c = base + (size_t)r * slot;
        v.in = c;
        v.x0 = c, c += 3 * (size_t)cnt;
        v.N0 = c, c += 3 * (size_t)cnt;
        if (w) v.w = c, c += cnt;
        if (xl) v.xl = c, c += 3 * (size_t)cnt;
        if (s0) v.s0 = c, c += cnt;
        v.n_in = c - v.in;
        // outputs at a fixed offset (m rays' inputs), so a shard's outputs never
        // share bytes with the next shards' inputs in the same slot: shard
        // j - 2's download into the host slot can land while shard j's inputs
        // are packed there
        c = v.in + (size_t)n_in * m;
        v.out = c;
        v.state = c, c += 7 * (size_t)cnt;
        if (depo) v.Pdep = c, c += cnt;
        if (n_save) v.traj = c, c += (size_t)n_save * 5 * cnt;
        v.status = (int *)c, v.steps = (int *)c + cnt, c += cnt;
        v.n_out = c - v.out;
        return v;
    };
    const size_t D = sizeof(double);
    // rows x cnt sub-block of a (rows x n) SoA host array <-> compact rows
    auto pack = [&](double *dst, const double *src, int rows, int lo, int cnt) {
        if (!src) return;
#pragma omp parallel for if ((size_t)rows * cnt > (1u << 18)) num_threads(8)
        for (int r = 0; r < rows; r++) memcpy(dst + (size_t)r * cnt, src + (size_t)r * n + lo, cnt * D);
    };
    auto unpack = [&](double *dst, const double *src, int rows, int lo, int cnt) {
        if (!dst) return;
#pragma omp parallel for if ((size_t)rows * cnt > (1u << 18)) num_threads(8)
        for (int r = 0; r < rows; r++) memcpy(dst + (size_t)r * n + lo, src + (size_t)r * cnt, cnt * D);
    };
    auto stage_in = [&](int j) -> int {  // pack shard j and queue its upload
        const int r = j & 1, lo = los[j], cnt = cnts[j];
        if (j >= 2) HIPCK(hipEventSynchronize(bs.up[r]));  // shard j - 2's upload left the slot
        const View h = view(hbase, r, cnt), d = view(dbase, r, cnt);
        pack(h.x0, x0, 3, lo, cnt), pack(h.N0, N0, 3, lo, cnt), pack(h.w, w, 1, lo, cnt);
        pack(h.xl, xl, 3, lo, cnt), pack(h.s0, s0, 1, lo, cnt);
        HIPCK(hipMemcpyAsync(d.in, h.in, h.n_in * D, hipMemcpyHostToDevice, bs.sc));
        HIPCK(hipEventRecord(bs.up[r], bs.sc));
        return 0;
    };
    auto finish = [&](int j) -> int {  // wait for shard j's download, unpack it
        const int r = j & 1, lo = los[j], cnt = cnts[j];
        HIPCK(hipEventSynchronize(bs.dn[r]));
        const View h = view(hbase, r, cnt);
        unpack(state, h.state, 7, lo, cnt);
        if (depo) unpack(P_dep, h.Pdep, 1, lo, cnt);
        if (n_save) unpack(traj, h.traj, n_save * 5, lo, cnt);
        memcpy(status + lo, h.status, cnt * sizeof(int));
        memcpy(steps + lo, h.steps, cnt * sizeof(int));
        return 0;
    };
    // TORJ_BEAM_SYNC=1 (read per call; diagnosis): drain the device after every
    // queued step, so the pipeline runs in program order
    const char *sync_e = getenv("TORJ_BEAM_SYNC");
    const bool dbg_sync = sync_e && atoi(sync_e) != 0;
    auto dsync = [&]() -> int {
        if (dbg_sync) HIPCK(hipDeviceSynchronize());
        return 0;
    };
    if (stage_in(0) || dsync()) return -1;
    for (int j = 0; j < nk; j++) {
        const int r = j & 1, cnt = cnts[j];
        if (j + 1 < nk && (stage_in(j + 1) || dsync())) return -1;
        const View d = view(dbase, r, cnt);
        HIPCK(hipStreamWaitEvent(s, bs.up[r], 0));
        if (j >= 2) HIPCK(hipStreamWaitEvent(s, bs.dn[r], 0));  // the slot's previous outputs are out
        if (torj_trace_device_ex(q, cfg, cnt, d.x0, d.N0, d.w, depo ? n_psi : 0, dgrid, d.xl, d.s0,
                                 d.state, d.status, d.steps, depo ? d_dP : nullptr, d.Pdep, d.traj,
                                 nullptr, s))
            return -1;
        HIPCK(hipEventRecord(bs.tr[r], s));
        if (dsync()) return -1;
        if (j >= 2 && finish(j - 2)) return -1;  // before this slot's host buffer is reused
        const View h = view(hbase, r, cnt);
        HIPCK(hipStreamWaitEvent(bs.sc, bs.tr[r], 0));
        HIPCK(hipMemcpyAsync(h.out, d.out, d.n_out * D, hipMemcpyDeviceToHost, bs.sc));
        HIPCK(hipEventRecord(bs.dn[r], bs.sc));
    }
    for (int j = std::max(0, nk - 2); j < nk; j++)
        if (finish(j)) return -1;
    // every shard's queue / grid flags (sticky since the last check)
    return torj_trace_check(q, s);
}

// Shards of torj_trace_beam when the caller leaves n_shards = 0: each device's
// share in pieces of at most kBeamAutoRays rays (at least one per device), so
// the host transfers of one piece overlap the trace of the next (beam_worker)
// while every piece still fills the device (the split pipeline wants >= ~1e5
// rays: a 1e5-ray beam stays one piece).
constexpr long kBeamAutoRays = 131072;
static int beam_auto_shards(int n, int n_gpus) {
    const long per = ((long)n + n_gpus - 1) / n_gpus;
    return n_gpus * (int)std::max<long>(1, (per + kBeamAutoRays - 1) / kBeamAutoRays);
}

extern "C" {

int torj_trace_beam(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                    const double *N0, const double *weights, int n_psi, const double *grid,
                    const double *x_launch, const double *s0, double *state, int *status,
                    int *steps, double *dP, double *Pdep, double *traj, int n_gpus, int n_shards) {
    if (!p || !cfg) return fail("bad plasma handle or cfg");
    if (n < 0 || n_shards < 0) return fail("n and n_shards must be >= 0");
    if (n == 0) {
        if (dP && n_psi > 0) std::fill(dP, dP + n_psi + 1, 0.0);
        return 0;
    }
    if (!x0 || !N0 || !state || !status || !steps) return fail("x0, N0, state, status, steps required");
    const bool depo = n_psi >= 2 && grid;
    if (depo) {
        for (int k = 1; k < n_psi; k++)
            if (!(grid[k] > grid[k - 1])) return fail("psi_dP_dV must be strictly increasing");
        if (!dP || !Pdep) return fail("deposition needs dP_shell and P_dep");
    }
    const bool same = beam_same_device();
    if (beam_replicas(p, n_gpus, same)) return -1;
    const int S = n_shards > 0 ? std::max(n_shards, n_gpus) : beam_auto_shards(n, n_gpus);
    const char *rccl_e = getenv("TORJ_BEAM_RCCL");  // read per call (tests toggle it)
    const bool reduce = depo && (n_gpus > 1 || (rccl_e && atoi(rccl_e) != 0));
    // per-device partial dP_shell, then one all-reduce
    std::vector<double *> d_dP(n_gpus, nullptr);
    int out = beam_fanout(p, n_gpus, "torj_trace_beam", [&](int k) -> int {
        torj_plasma_s *q = p->replicas[k];
        if (depo) HIPCK(hipMalloc(&d_dP[k], (n_psi + 1) * sizeof(double)));
        return beam_worker(q, cfg, n, S, k, n_gpus, x0, N0, weights, n_psi, grid, x_launch, s0, state,
                           status, steps, depo ? Pdep : nullptr, traj, d_dP[k]);
    });
    if (!out && reduce) out = beam_reduce(p, n_gpus, d_dP, n_psi, same);
    if (!out && depo) {
        torj_plasma_s *q0 = p->replicas[0];
        if (hipSetDevice(q0->device) != hipSuccess ||
            hipMemcpyAsync(dP, d_dP[0], (n_psi + 1) * sizeof(double), hipMemcpyDeviceToHost,
                           q0->stream) != hipSuccess ||
            hipStreamSynchronize(q0->stream) != hipSuccess)
            out = fail("download of dP_shell failed");
    }
    for (int k = 0; k < n_gpus; k++)
        if (d_dP[k]) {
            (void)hipSetDevice(p->replicas[k]->device);
            (void)hipStreamSynchronize(p->replicas[k]->stream);
            (void)hipFree(d_dP[k]);
        }
    if (!out && !depo) {
        if (dP) std::fill(dP, dP + (n_psi > 0 ? n_psi + 1 : 1), 0.0);
        if (Pdep) std::fill(Pdep, Pdep + n, 0.0);
    }
    (void)hipSetDevice(p->device);
    return out;
}

int torj_trace_beam_device(torj_plasma_t p, const torj_trace_cfg *cfg, int n_gpus, int n_psi,
                           const torj_beam_shard *shards) {
    if (!p || !cfg || !shards) return fail("bad plasma handle, cfg or shards");
    const bool same = beam_same_device();
    if (beam_replicas(p, n_gpus, same)) return -1;
    bool depo = n_psi >= 2;
    for (int k = 0; k < n_gpus; k++) {
        if (shards[k].n < 0) return fail("shard %d: n < 0", k);
        depo = depo && shards[k].psi_grid && shards[k].dP_shell;
    }
    if (n_psi >= 2 && !depo) return fail("deposition needs psi_grid and dP_shell on every shard");
    const char *rccl_e = getenv("TORJ_BEAM_RCCL");
    const bool reduce = depo && (n_gpus > 1 || (rccl_e && atoi(rccl_e) != 0));
    int out = beam_fanout(p, n_gpus, "torj_trace_beam_device", [&](int k) -> int {
        torj_plasma_s *q = p->replicas[k];
        const torj_beam_shard &h = shards[k];
        if (ensure_device(q)) return -1;
        if (h.n > 0 &&
            torj_trace_device_ex(q, cfg, h.n, h.x0, h.N0, h.weights, depo ? n_psi : 0, h.psi_grid,
                                 h.x_launch, h.s0, h.state, h.status, h.steps, h.dP_shell, h.P_dep,
                                 h.traj, h.counters, q->stream))
            return -1;
        return torj_trace_check(q, q->stream);  // waits for the stream: queue / grid flags
    });
    if (!out && reduce) {
        std::vector<double *> d_dP(n_gpus);
        for (int k = 0; k < n_gpus; k++) d_dP[k] = shards[k].dP_shell;
        out = beam_reduce(p, n_gpus, d_dP, n_psi, same);
    }
    (void)hipSetDevice(p->device);
    return out;
}

int torj_trace_check(torj_plasma_t p, void *stream) {
    if (!p) return fail("bad plasma handle");
    if (!p->d_flags) return 0;  // no launch yet
    HIPCK(hipSetDevice(p->device));
    HIPCK(hipStreamSynchronize((hipStream_t)stream));
    int flags = 0;  // ORed by every launch on this handle since the last check
    HIPCK(hipMemcpy(&flags, p->d_flags, sizeof(int), hipMemcpyDeviceToHost));
    if (flags) HIPCK(hipMemset(p->d_flags, 0, sizeof(int)));
    if (flags & 1) return fail("psi_dP_dV must be strictly increasing");
    if (flags & 2) return fail("work-queue watchdog fired (ready-queue stalled)");
    if (flags & 4) return fail("work queue did not retire every ray group");
    return 0;
}

}  // extern "C"

#endif  // TORJ_TRAJ_TU
