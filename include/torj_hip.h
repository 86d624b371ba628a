/*
 * torj_hip.h -- C ABI of libtorj_hip.so, the MI355X-native replacement for the
 * ray-tracing hot path of TorJ.jl (make_ray / make_beam, src/solve.jl).
 *
 * The reference has no FFI: everything is Julia.  Each entry point below names
 * the Julia function whose behaviour it replaces (file:line in the TorJ.jl
 * repository); INTEGRATION.md shows the `ccall` bindings a TorJ maintainer
 * would add (torj.jl_amd/julia/TorJHIP.jl) and the Python ctypes mirror used by
 * this repository's tests (torj.jl_amd/torj_hip).
 *
 * Conventions
 *  - Plain C types only.  Return value: 0 = success, <0 = error; the message of
 *    the last error on the calling thread is returned by torj_last_error().
 *    No exception or longjmp ever crosses this boundary.
 *  - Per-ray 3-vectors are COMPONENT-MAJOR ("SoA"): v[c*n + i] is component c of
 *    ray i.  This is exactly the memory of a Julia `n x 3` Matrix{Float64}
 *    (column-major), e.g. the ray_positions returned by launch_peripheral_rays
 *    (src/launch.jl:84-86), so Julia passes them without copying.
 *  - 2-D maps are (nR x nZ) column-major (R fastest), i.e. Julia matrices.
 *  - Functions without the _device suffix take HOST pointers owned by the
 *    caller and valid only for the call (Julia: GC.@preserve); they copy to the
 *    GPU, run, copy back and synchronise.  *_device functions take device
 *    pointers and a hipStream_t (as void*), enqueue and return immediately.
 *  - All arithmetic is fp64.
 *  - Every compute entry point runs on the GPU (HIP, gfx950).  There is no
 *    CPU fallback: without a usable GPU they return an error.
 */
#ifndef TORJ_HIP_H
#define TORJ_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TORJ_ABI_VERSION 8  /* 3: torj_trace_beam, sticky launch flags; 4: 8 work counters;
                               5: torj_trace_beam_device, torj_power_deposition_profile;
                               6: torj_beam_timing_read, torj_trace_beam's automatic shards;
                               7: torj_build_id; 8: torj_beam_comm_info */

/* per-ray status codes (replace the reference's @assert / unhandled returns) */
enum torj_status {
    TORJ_RAY_OK = 0,          /* ran all steps */
    TORJ_RAY_LEFT_PLASMA = 1, /* psi > psi_exit at a chunk boundary (src/solve.jl:174) */
    TORJ_RAY_ABSORBED = 2,    /* P < P_min at a chunk boundary (src/solve.jl:176) */
    TORJ_RAY_NAN = 3,         /* non-finite state (e.g. upper-hybrid resonance) */
    TORJ_RAY_REFLECTED = 4,   /* N_s^2 <= 0 at the plasma edge (src/solve.jl:57-59) */
    TORJ_RAY_ENTRY_FAIL = 5,  /* first_point / refraction assertions (src/solve.jl:32,138,141) */
    TORJ_RAY_MAX_STEPS = 6    /* integrator 1: accepted-step capacity n_steps exhausted */
};

typedef struct torj_plasma_s *torj_plasma_t;

/* ---- library / device ---------------------------------------------------- */
int torj_abi_version(void);
/* identity of this build: 16 hex digits of a hash over the library's sources
 * and compile flags (csrc/Makefile).  Profiles record it, and bench.py uses a
 * committed profile only when its build id equals the loaded library's. */
const char *torj_build_id(void);
const char *torj_last_error(void);
int torj_device_count(int *n);

/* abs_Al_init(N_absz) (src/absorption.jl:1-7): Gauss-Legendre order of the
 * Albajar resonance-ellipse integral (process-global, like the reference's
 * module globals _int_absz/_int_weights, src/constants.jl:7-8).  1 <= n <= 64.
 * Absorption calls fail with the reference's ErrorException message
 * (src/absorption.jl:173-175) until this has been called.  Also reads
 * TORJ_TINY_ALPHA (m^-1, default 1e-20; 0 = off): fixed-step ray tracing skips
 * a harmonic integral whose rigorous bound on its share of alpha is below it
 * (tau moves by < 2 TORJ_TINY_ALPHA per metre of ray). */
int torj_abs_al_init(int n);

/* ---- Plasma (src/plasma.jl:2-58) ----------------------------------------- */
/* Plasma(R_coords, Z_coords, psi_norm_data, psi_prof, ne_prof, Te_prof, Br_data,
 *        Bz_data, Bϕ_data, eqt1d_psi_norm, eqt1d_volume)   (src/plasma.jl:30-58)
 * Builds the Interpolations.jl-equivalent cubic B-spline coefficients (Line()
 * boundary/extrapolation) on the host and uploads them to `device`. */
int torj_plasma_create(int nR, int nZ, const double *R_coords, const double *Z_coords,
                       const double *psi_norm_data, int n_prof, const double *psi_prof,
                       const double *ne_prof, const double *Te_prof, const double *Br_data,
                       const double *Bz_data, const double *Bphi_data, int n_eq,
                       const double *eqt1d_psi_norm, const double *eqt1d_volume, int device,
                       torj_plasma_t *out);
/* Same, from B-spline coefficient arrays already built by Interpolations.jl
 * (parent(spl.itp.itp.coefs): (nR+2) x (nZ+2) column-major each; field order
 * psi, ln ne, ln Te, Br, Bz, Bphi) and the 1-D volume spline coefficients
 * (n_vol+2 over the uniform psi range [vol_psi1, vol_psin]). */
int torj_plasma_create_from_coefs(int nR, int nZ, double R1, double Rn, double Z1, double Zn,
                                  const double *coef_psi, const double *coef_lnne,
                                  const double *coef_lnTe, const double *coef_Br,
                                  const double *coef_Bz, const double *coef_Bphi, int n_vol,
                                  double vol_psi1, double vol_psin, const double *vol_coefs,
                                  double psi_prof_max, int device, torj_plasma_t *out);
int torj_plasma_destroy(torj_plasma_t p);
/* field: 0 psi, 1 ln ne, 2 ln Te, 3 Br, 4 Bz, 5 Bphi.  out: (nR+2)*(nZ+2), column-major */
int torj_plasma_get_coefs(torj_plasma_t p, int field, double *out);
double torj_plasma_psi_prof_max(torj_plasma_t p);
/* plasma.volume_psi_spline at n points (host) */
int torj_plasma_volume(torj_plasma_t p, int n, const double *psi, double *vol);

/* ---- point evaluations (GPU; mirror the reference's unit-tested functions) -- */
/* Per point i (x, N component-major 3 x n), out is 13 x n component-major:
 *   0-2  B_spline(plasma, x)            (src/plasma.jl:73-81)
 *   3    n_e(plasma, x)                 (src/plasma.jl:83-85)
 *   4    T_e(plasma, x)                 (src/plasma.jl:87-89)
 *   5    evaluate(psi_norm_spline, x)   (src/plasma.jl:61-65)
 *   6-8  X, Y, N_par of eval_plasma     (src/dispersion.jl:7-15)
 *   9-11 b of eval_plasma
 *   12   |B|                                                             */
int torj_eval_plasma(torj_plasma_t p, int n, const double *x, const double *N, double omega,
                     double *out);
/* dispersion_relation (src/dispersion.jl:34-39), the normalised Hamiltonian
 * RHS of gradΛ! (src/solve.jl:85-93; du = dx/ds, dN/ds, 6 x n) and α_approx
 * (src/absorption.jl:228-235; pass alpha = NULL to skip). */
int torj_dispersion(torj_plasma_t p, int n, const double *x, const double *N, double omega,
                    int mode, double *D, double *du, double *alpha);
/* abs_Albajar_fast(omega, X, Y, N_abs, N_par, Te, mode) (src/absorption.jl:191-226),
 * batched over n tuples (arrays of length n). */
int torj_abs_albajar_fast(int n, const double *omega, const double *X, const double *Y,
                          const double *N_abs, const double *N_par, const double *Te, int mode,
                          double *alpha);
/* refractive_index_sq(X, Y, N_par, mode) (src/dispersion.jl:29-32), batched */
/* Warm-plasma absorption alpha (src/general_absorption.jl:1328-1337, repaired
 * as described in DESIGN.md): warmdisp's N_perp^2 with the weakly (iwarm 1) or
 * fully (iwarm 3) relativistic dielectric tensor, lrm = min(5, larmornumber),
 * alpha = 2 Im(N_perp^2) omega/c / |dD/dN| (inv_dDdN = 1/|dD/dN|); Nperp2 (may
 * be NULL) receives N_perp^2 as (re, im) pairs.  GPU, batched (host arrays). */
int torj_alpha_warm(int n, const double *omega, const double *X, const double *Y,
                    const double *N_abs, const double *N_par, const double *Te,
                    const double *inv_dDdN, int mode, int iwarm, double *alpha, double *Nperp2);

int torj_refractive_index_sq(int n, const double *X, const double *Y, const double *N_par,
                             int mode, double *out);

/* ---- launch (host) ------------------------------------------------------- */
/* IMAS.pol_tor_angles_2_vector(pol, tor) as called at src/solve.jl:211 */
void torj_pol_tor_angles_2_vector(double pol, double tor, double N[3]);
/* launch_peripheral_rays (src/launch.jl:24-132).  Call with pos == NULL to get
 * the ray count in *n_rays; then with arrays of that size (pos, dir
 * component-major 3 x n).  Returns -1 (ArgumentError) for N_rings < 2. */
int torj_launch_peripheral_rays(const double x0[3], const double N0[3], double w,
                                double inverse_curvature_radius, double f, int N_rings,
                                int min_azimuthal_points, int normalize_weight_sum, int *n_rays,
                                double *pos, double *dir, double *weights);

/* ---- ray entry: first_point + vacuum_plasma_refraction (src/solve.jl:7-74) --
 * x0, N0: vacuum launch points/directions (3 x n); outputs the in-plasma start
 * point, refracted N, vacuum path length s0 and a status per ray. */
int torj_ray_entry(torj_plasma_t p, int n, const double *x0, const double *N0, double omega,
                   int mode, double *x_plasma, double *N_plasma, double *s0, int *status);
/* Same computation on the GPU (one lane per ray), device pointers, async on
 * `stream` (hipStream_t or NULL).  Replaces the per-ray host bisection + NLsolve
 * of make_beam's ray loop (src/solve.jl:219-221 -> :137-141). */
int torj_ray_entry_device(torj_plasma_t p, int n, const double *x0, const double *N0,
                          double omega, int mode, double *x_plasma, double *N_plasma, double *s0,
                          int *status, void *stream);
/* Host pointers, GPU compute (upload, torj_ray_entry_device, download). */
int torj_ray_entry_gpu(torj_plasma_t p, int n, const double *x0, const double *N0, double omega,
                       int mode, double *x_plasma, double *N_plasma, double *s0, int *status);

/* ---- the hot path: ray stepping (src/solve.jl:144-177) ------------------- */
typedef struct {
    double omega;     /* 2 pi f */
    int mode;         /* +1 X-mode, -1 O-mode (src/solve.jl:110) */
    double ds;        /* fixed RK4 step [m]; the reference caps dtmax at 1e-4 (src/solve.jl:157) */
    int n_steps;      /* steps per ray (s_max / ds) */
    int chunk_steps;  /* termination checks every chunk_steps (reference: 100 chunks, src/solve.jl:145) */
    double psi_exit;  /* 1.0 in the reference (src/solve.jl:174) */
    double P_min;     /* 1e-6 in the reference (src/solve.jl:176) */
    int absorption;   /* optical depth model: 0 none; 1 abs_Albajar_fast (src/absorption.jl:191-226);
                         2 warm weakly relativistic, 3 warm fully relativistic (the repaired
                         src/general_absorption.jl alpha, :1328-1337; 3 is what it hard-codes,
                         2 is BASELINE's C5) -- see torj_alpha_warm */
    int traj_stride;  /* 0: no trajectory; else save (x,y,z,tau) every traj_stride steps */
    int deposition;   /* 0: in-kernel psi-shell binning of the RK4 steps (fast, default);
                         1: the reference's power_deposition_profile (src/plasma.jl:91-151):
                            not-a-knot cubic splines of psi(s) and dP/ds = P alpha through
                            make_ray's saved points, boundary roots paired per shell,
                            |integral| per pair, outside-in walk -- needs torj_trace_ex */
    int integrator;   /* 0: fixed-step classic RK4 of n_steps steps of ds (default);
                         1: adaptive, as the reference's solve() (src/solve.jl:144-162):
                            Tsit5 5(4) on u = (x, N, P) with DiffEq's PI step control and
                            initial-step heuristic, abstol/reltol below, dtmax = ds, over
                            n_chunks tspans of s_max/n_chunks starting at s0 (each chunk
                            restarts the integrator); n_steps is then the per-ray capacity
                            of accepted steps (status MAX_STEPS when exceeded) */
    double abstol, reltol;  /* integrator 1: 1e-6, 1e-6 in the reference (src/solve.jl:157) */
    double s_max;     /* integrator 1: path length in the plasma (make_ray's s_max) */
    int n_chunks;     /* integrator 1: 100 in the reference (src/solve.jl:145) */
} torj_trace_cfg;

/* Host-pointer form.  x0, N0: in-plasma start states (3 x n); weights (n, may
 * be NULL = all 1); psi_grid (n_psi, may be n_psi = 0: no deposition).
 * Outputs: state 7 x n (x, y, z, Nx, Ny, Nz, tau with P = exp(-tau)),
 * status n, steps n; dP_shell n_psi + 1: [j] = sum_rays w * (power deposited
 * in psi shell [psi_grid[j], psi_grid[j+1]]) for j < n_psi-1, [n_psi-1] = 0,
 * [n_psi] = sum_rays w * P_dep(ray); P_dep n (per ray, unweighted).  traj:
 * (n_steps/traj_stride) x 5 x n = (x, y, z, tau, s) every traj_stride (accepted)
 * steps, s the arc length from the vacuum launch point; NaN after a ray stops.  Any output may be
 * NULL.  Divide dP_shell[j] by the shell volume to get make_beam's dP_dV
 * (src/plasma.jl:141, src/solve.jl:237-240). */
int torj_trace(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
               const double *N0, const double *weights, int n_psi, const double *psi_grid,
               double *state, int *status, int *steps, double *dP_shell, double *P_dep,
               double *traj);

/* With the vacuum launch points x_launch (3 x n, make_ray's first point, s = 0)
 * and path lengths s0 (n) to the entry point -- what cfg->deposition = 1 needs
 * to rebuild make_ray's s / psi vectors.  With deposition = 1, dP_shell[j] is
 * sum_rays w dP_j of the reference profile, dP_shell[n_psi] = sum_rays w P and
 * P_dep[i] = the ray's deposited power P (src/plasma.jl:140-147). */
int torj_trace_ex(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                  const double *N0, const double *weights, int n_psi, const double *psi_grid,
                  const double *x_launch, const double *s0, double *state, int *status,
                  int *steps, double *dP_shell, double *P_dep, double *traj);

/* Device-pointer form (inputs resident in HBM; what bench.py times).
 * dP_shell (n_psi+1) is ACCUMULATED into (zero it first).  counters (may be
 * NULL): 8 x uint64 accumulated, the basis of the algorithmic FLOP count
 * (torj_hip/flops.py): [0] ray-steps, [1] RHS evaluations, then
 *   absorption 1 (Albajar): [2] calls reaching the harmonic sum, [3] harmonic
 *     integrals evaluated, [4] Bessel-series terms, [5] harmonic integrals found
 *     exactly zero without their node loop, [6] harmonic integrals skipped as
 *     provably below an ulp of the sum (alpha bit-identical), [7] harmonic
 *     integrals found exactly zero in calls settled before the polarisation
 *     vector (every harmonic present an exact zero: alpha = 0, no call
 *     reaches the harmonic sum);
 *   absorption 2 (warm, iwarm 1): [2] Faddeeva evaluations by the asymptotic
 *     series (|z| >= 16, of [3]), [3] Faddeeva evaluations, [4] warmdisp
 *     passes, [5] passes x Larmor order lrm,
 *     [6] sum lrm, [7] sum lrm^2 (one warm alpha per RHS evaluation);
 *   absorption 0 / 3: [2..7] 0.
 * stream: hipStream_t or NULL. */
int torj_trace_device(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                      const double *N0, const double *weights, int n_psi,
                      const double *psi_grid, double *state, int *status, int *steps,
                      double *dP_shell, double *P_dep, double *traj, uint64_t *counters,
                      void *stream);
int torj_trace_device_ex(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                         const double *N0, const double *weights, int n_psi,
                         const double *psi_grid, const double *x_launch, const double *s0,
                         double *state, int *status, int *steps, double *dP_shell, double *P_dep,
                         double *traj, uint64_t *counters, void *stream);

/* make_beam's fan-out and reduce across the GPUs of this process
 * (src/solve.jl:209-240: one task per ray, then sum_i w_i dP_dV_i and
 * sum_i w_i P_i).  Host pointers, the arguments and outputs of torj_trace_ex.
 * The rays are cut into n_shards contiguous shards (0: automatic -- each
 * device's share in pieces of at most 131 072 rays, at least one per device;
 * otherwise at least n_gpus), their boundaries on 64-ray multiples, dealt
 * round-robin to n_gpus devices: device (p's device + k) mod the device count
 * for k < n_gpus, each with its own copy of the plasma, stream and host thread.
 * A device runs its shards in turn through pinned staging in two slots on a
 * copy stream: shard j + 1's upload and shard j - 1's download overlap shard
 * j's trace (one torj_trace_check after the last), its
 * dP_shell partial accumulating on the device; the partials are summed over
 * the devices by one RCCL all-reduce of n_psi + 1 fp64 (single-process
 * communicator from ncclCommInitAll, kept on the handle; n_gpus = 1 needs no
 * reduce unless env TORJ_BEAM_RCCL=1).  Per-ray outputs equal torj_trace_ex's
 * for the same rays and scheduling; dP_shell differs by summation order only.
 * Errors name the failing device.  Test-only: env TORJ_BEAM_SAME_DEVICE=1 puts
 * every replica on p's own device (the threaded multi-replica branch on one
 * GPU; the partials are then summed on the host, RCCL refusing a device twice). */
int torj_trace_beam(torj_plasma_t p, const torj_trace_cfg *cfg, int n, const double *x0,
                    const double *N0, const double *weights, int n_psi, const double *psi_grid,
                    const double *x_launch, const double *s0, double *state, int *status,
                    int *steps, double *dP_shell, double *P_dep, double *traj, int n_gpus,
                    int n_shards);

/* make_beam's fan-out over DEVICE-RESIDENT shards (the serving / benchmark
 * form of torj_trace_beam: inputs already in HBM, no host staging).  Shard k
 * lives on replica k's device -- (p's device + k) mod the device count -- and
 * its pointers are that device's memory, laid out exactly as the arguments of
 * torj_trace_device_ex.  Each replica traces its shard on its own stream from
 * its own host thread (n = 0: nothing), waits and checks it (torj_trace_check);
 * then, with deposition (n_psi >= 2, psi_grid and dP_shell on every shard),
 * the (n_psi + 1) dP_shell vectors are all-reduced in place by RCCL, so every
 * shard's dP_shell holds the sum over the shards (zero them first: the trace
 * accumulates into them).  n_gpus = 1 skips the reduce unless env
 * TORJ_BEAM_RCCL=1.  Synchronous.  Same reference interface as torj_trace_beam
 * (src/solve.jl:209-240). */
typedef struct {
    int n;                                    /* rays in this shard */
    const double *x0, *N0;                    /* 3 x n */
    const double *weights;                    /* n or NULL */
    const double *psi_grid;                   /* n_psi (this device's copy) */
    const double *x_launch, *s0;              /* 3 x n, n (deposition = 1) or NULL */
    double *state;                            /* 7 x n */
    int *status, *steps;                      /* n */
    double *dP_shell;                         /* n_psi + 1, accumulated, then all-reduced */
    double *P_dep;                            /* n or NULL */
    double *traj;                             /* (n_steps / traj_stride) x 5 x n or NULL */
    uint64_t *counters;                       /* 8 or NULL (torj_trace_device) */
} torj_beam_shard;
int torj_trace_beam_device(torj_plasma_t p, const torj_trace_cfg *cfg, int n_gpus, int n_psi,
                           const torj_beam_shard *shards);

/* Scheduling of torj_trace / torj_trace_device launches on this plasma handle
 * (no reference counterpart: an MI355X tuning knob; results are independent
 * of it up to the summation order of dP_shell).  mode -1: default (env
 * TORJ_SCHED; else 1 when the beam has more
 * 64-ray groups than the device has SIMDs, otherwise 0); 0: one lane per ray for the whole trace; 1: persistent
 * waves pulling 64-ray groups chunk by chunk from a ready queue; 2: the whole
 * trace with 16 lanes per ray (Albajar absorption, no binning: the node pairs
 * of the absorption integral split between a ray's lanes, results equal to
 * rounding; mode -1 picks it for beams of at most 2 x 64 x SIMDs / 16 rays
 * unless env TORJ_LPR=1); 3: the split RK4 path (fixed steps, Albajar or
 * warm absorption): the trajectories' cold RK4 in one kernel, the 4 x n_steps
 * alpha evaluations per ray in a fully parallel one, the optical depth by an
 * in-order scan, blocks of steps pipelined over two streams (DESIGN.md 3.7;
 * mode -1 picks it for Albajar where it would pick 1, for the weakly
 * relativistic warm model always and for the fully relativistic one on beams
 * of fewer than 3 x 64-ray groups per CU, unless env TORJ_SPLIT=0;
 * TORJ_SPLIT_WARM=0 / 1 turns the warm choice off / on for every size).
 * waves: number of persistent waves for mode 1 (0 = default: min(8 per CU, G - G/16));
 * steps per pipeline block for mode 3 (0 = from the 1 GiB per alpha-input
 * buffer budget, env TORJ_SPLIT_MB; four buffers in flight). */
int torj_set_sched(torj_plasma_t p, int mode, int waves);

/* Waits for `stream` and checks every trace launched on this handle since
 * the previous check (the flags are sticky: each launch ORs its outcome in,
 * this call reads and clears them): that each psi_dP_dV grid was strictly
 * increasing (checked on the device, so the _device calls never read device
 * memory back or synchronise inside the launch; the host-pointer calls also
 * check their host copy up front), and for work-queue launches, that every ray
 * group retired and the stall watchdog (no progress anywhere in the grid for
 * 120 s) did not fire.  torj_trace[_ex] call it themselves; callers of the
 * asynchronous _device calls call it before trusting the outputs.  All
 * _device calls on one handle must use one stream: they share the handle's
 * scratch (work queue, deposition workspace). */
int torj_trace_check(torj_plasma_t p, void *stream);

/* Per-phase HIP-event timing of torj_trace[_device][_ex] calls on this handle
 * (measurement support, no reference counterpart).  torj_timing(p, 1) clears
 * and enables recording: events on the call's stream before the trace kernel,
 * after it, and after the deposition kernels.  torj_timing_read waits for the
 * recorded calls and returns their count and summed trace-kernel / post-
 * processing milliseconds, then clears. */
int torj_timing(torj_plasma_t p, int enable);
int torj_timing_read(torj_plasma_t p, int *calls, double *trace_ms, double *post_ms);

/* The same per replica of a torj_trace_beam[_device] fan-out (torj_timing(p, 1)
 * enables it on the handle and every replica): calls, trace_ms, post_ms are
 * arrays of n_gpus entries (replica k = device (p's device + k) mod count; k = 0
 * is p), each as torj_timing_read returns it, and reduce_ms the summed host-
 * clock time of make_beam's RCCL all-reduce (the grouped ncclAllReduce and its
 * stream waits).  Clears what it reads. */
int torj_beam_timing_read(torj_plasma_t p, int n_gpus, int *calls, double *trace_ms, double *post_ms,
                          double *reduce_ms);

/* Who took part in make_beam's reduce (src/solve.jl:233-240) of the last
 * torj_trace_beam[_device] fan-out over n_gpus replicas (measurement support,
 * no reference counterpart): per replica k, the HIP device it ran on
 * (device[k]), and its RCCL communicator's rank count (ncclCommCount) and
 * rank (ncclCommUserRank) in nranks[k] / rank[k] -- or 0 / -1 where no
 * communicator exists (one replica without TORJ_BEAM_RCCL=1: nothing to
 * reduce; the test-only same-device placement: partials summed on the host).  Arrays of n_gpus
 * entries; n_gpus may not exceed the handle's replicas. */
int torj_beam_comm_info(torj_plasma_t p, int n_gpus, int *device, int *nranks, int *rank);

/* power_deposition_profile(plasma, s, x, dP_ds, psi_dP_dV) (src/plasma.jl:91-151)
 * on the GPU for n_rays rays at once: ray r has n_points[r] >= 4 points with
 * strictly increasing s, concatenated ray after ray -- s and dP_ds (sum of
 * n_points), x component-major 3 x (sum of n_points).  psi at each point from
 * the plasma's psi spline; the not-a-knot cubic fits of psi(s) - psi_j and
 * dP/ds (Dierckx.Spline1D k = 3), their roots (Dierckx.roots, maxn = 8: the
 * first 8 per boundary in s order), the |integral| per root pair and the
 * outside-in walk, as torj_trace_ex's deposition = 1 applies to a trace.
 * Outputs: dP_dV n_rays x n_psi, row r = ray r's dP_dV (its last entry 0, as
 * the reference's), and P (n_rays).  Host pointers, synchronous.  Errors
 * mirror the reference's: too few points or non-increasing s (Dierckx), a
 * non-increasing psi_dP_dV. */
int torj_power_deposition_profile(torj_plasma_t p, int n_rays, const int *n_points, const double *s,
                                  const double *x, const double *dP_ds, int n_psi,
                                  const double *psi_dP_dV, double *dP_dV, double *P);

/* shell volumes dV[j] = V(psi_grid[j+1]) - V(psi_grid[j]), j < n_psi-1 (host;
 * src/plasma.jl:117-122) */
int torj_shell_volumes(torj_plasma_t p, int n_psi, const double *psi_grid, double *dV);

#ifdef __cplusplus
}
#endif
#endif /* TORJ_HIP_H */
