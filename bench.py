#!/usr/bin/env python3
"""Headline benchmark: ray-steps/s of the EC ray-tracing hot path on MI355X.

Workload (BASELINE.json configs[2]): a 100,203-ray EC beam
(launch_peripheral_rays with N_rings=92, min_azimuthal_points=11) per GPU,
X-mode, 92.5 GHz, 2,000 fixed RK4 steps of ds = 1e-4 m with Albajar absorption,
in-kernel psi-shell deposition on a 1,000-point psi grid and a x100-decimated
trajectory, through the synthetic circular-tokamak equilibrium (56 x 56 grid).
One "step" of this benchmark = one full pass of the hot path over the beam
(every ray integrated over its 2,000 RK4 steps) + the RCCL all-reduce of the
deposited-power profile across ranks.

value = ray-steps actually integrated by all ranks / wall time of the timed
steps (inputs resident in HBM; ray entry and upload are setup, outside).
Multi-GPU: one process per GPU (torchrun), each rank traces its own beam
(rotated toroidally by 2*pi*rank/world; the plasma is axisymmetric), no
data-path collective; one all_reduce of (n_psi+1) fp64 = make_beam's reduce
(src/solve.jl:233-240).  scaling = "weak".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))

# MI355X fp64 vector peak (spec): 256 CU x 2.4 GHz x 128 flop/clk (64 FMA lanes)
FP64_VECTOR_PEAK_TFLOPS = 78.6
HBM_PEAK_BPS = 8.0e12  # MI355X HBM3E (MI355X_MICROARCH.md)
# the C5 a-priori conditioning flag's relative input perturbation: 2^-45, at
# least the GPU Weideman Faddeeva's own relative error (2.5e-14), so the flag
# covers the implementation's error as well as the reference's rounding
WARM_FLAG_ETA = 2.0 ** -45
# parity's unfloored tau statistic covers the sampled rays with tau_cpu at least this
TAU_RESOLVABLE = 1e-12
# the library's default tiny-alpha threshold (torj_hip.hip kTinyAlpha; env TORJ_TINY_ALPHA)
TINY_ALPHA_DEFAULT = 1e-20
ABSORPTION = {"none": 0, "albajar": 1, "warm_wr": 2, "warm_fr": 3}
# the split RK4 pipeline's kernels (trajectory, alpha points, optical-depth scan, final)
SPLIT_KERNELS = "k_traj|k_alpha_pts|k_tau_scan|k_split_final"
# version of the FLOP model behind roofline.achieved (torj_hip/flops.py); bumped
# whenever a counter's meaning or a per-unit price changes, so figures of
# different rounds are compared only under the same model
FLOP_MODEL = {"albajar": "albajar-v5 (round 6: the node loop's gamma as the resonance condition's linear "
                         "form G0 +- G1 t, no square root; round 5: harmonics skipped below tiny_alpha = 1e-20 m^-1 priced as "
                         "negligible ones; round 3: exact-zero, negligible and settled-early harmonics "
                         "priced at their tests)",
              "none": "albajar-v5",
              "warm_wr": "warm-v4 (round 6: Weideman's polynomial and the asymptotic series by the real-coefficient "
                         "recurrence, 176 and 60 FLOP per evaluation instead of 278 and 84; round 5: warmdisp's breaking pass sums no tensor, its root by "
                         "the conjugate product, the asymptotic Faddeeva series by Horner; round 3: counter[2] = asymptotic Faddeeva "
                         "evaluations; larmornumber tests priced at one per call, a lower bound)"}
ALPHA_NAME = {"none": "no absorption (cold)", "albajar": "Albajar alpha (GL-24)",
              "warm_wr": "warm weakly-relativistic alpha (iwarm=1)",
              "warm_fr": "warm fully-relativistic alpha (iwarm=3)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n-rings", type=int, default=92)
    ap.add_argument("--min-az", type=int, default=11)
    ap.add_argument("--n-steps", type=int, default=2000)
    ap.add_argument("--ds", type=float, default=1e-4)
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--freq", type=float, default=92.5e9)
    ap.add_argument("--n-psi", type=int, default=1000)
    ap.add_argument("--traj-stride", type=int, default=100)
    ap.add_argument("--deposition", choices=["binned", "reference"], default="reference",
                    help="binned: in-kernel psi-shell binning; reference: "
                         "power_deposition_profile's FITPACK semantics (extra kernel)")
    ap.add_argument("--integrator", choices=["rk4", "adaptive"], default="rk4",
                    help="rk4: fixed steps of ds; adaptive: the reference's solve() semantics "
                         "(Tsit5, DiffEq step control, dtmax = ds, 100 chunks over n_steps*ds)")
    ap.add_argument("--absorption", choices=list(ABSORPTION), default="albajar",
                    help="albajar: abs_Albajar_fast (C3, the headline); warm_wr / warm_fr: the "
                         "repaired general_absorption.jl alpha, iwarm 1 (C5) / 3; none: cold")
    ap.add_argument("--shard", action="store_true",
                    help="C4 (strong scaling): split ONE fan across the ranks (contiguous ray "
                         "ranges) instead of one rotated fan per rank; e.g. --n-rings 291 --shard "
                         "for the ~1e6-ray beam over 8 GPUs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-api", action="store_true",
                    help="skip the host-pointer (PCIe-inclusive) calls and the library-path rate "
                         "(profiling passes)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target CPU time of the bounded cpu_baseline sample")
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the exact leg (the same timed loop with TORJ_TINY_ALPHA=0)")
    ap.add_argument("--no-beam-host", action="store_true",
                    help="skip the C4-scale torj_trace_beam host-pointer call (N = 1)")
    ap.add_argument("--parity-rays", type=int, default=128,
                    help="N > 1: rays of the oracle parity sample on rank 0 / device 0's shard")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}: launch one process per GPU "
                 f"with --nproc-per-node equal to --gpus")
    if world == 1 and args.gpus > 1:
        return main_library(args)  # one process, N devices: make_beam's library path
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus {args.gpus} < 1")
    import torch
    import torch.distributed as dist

    import torj_hip as T
    from torj_hip import flops as F
    from torj_hip import synthetic as S
    from torj_hip.parallel import allreduce_deposition

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test-only rehearsal of the multi-process path on a one-GPU box: every rank on
    # device 0 and the reduce over gloo (RCCL refuses two ranks on one device)
    same_dev = world > 1 and os.environ.get("TORJ_BENCH_SAME_DEVICE") == "1"
    if same_dev:
        local = 0
        dist.init_process_group("gloo")
    elif world > 1:
        if local >= torch.cuda.device_count():
            sys.exit(f"bench.py: LOCAL_RANK {local} but {torch.cuda.device_count()} HIP device(s) visible")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    # ---- setup (outside the timed region) ----
    eq = S.circular_tokamak()
    plasma = T.Plasma(*S.plasma_args(eq), device=local)
    T.abs_Al_init(24)
    f = args.freq
    omega = 2 * np.pi * f
    setup = S.SETUP
    N0 = T.pol_tor_angles_2_vector(setup["steering_angle_pol"], setup["steering_angle_tor"])
    x0 = np.array([setup["R0"], 0.0, setup["z0"]])
    pos, dirs, w = T.launch_peripheral_rays(x0, N0, setup["spot_size"],
                                            setup["inverse_curvature_radius"], f,
                                            N_rings=args.n_rings,
                                            min_azimuthal_points=args.min_az)
    n_fan = len(w)
    if args.shard:  # strong scaling: this rank's contiguous slice of the one fan
        lo, hi = rank * n_fan // world, (rank + 1) * n_fan // world
        pos, dirs, w = pos[lo:hi], dirs[lo:hi], w[lo:hi]
    else:  # weak scaling: each rank its own beam, rotated toroidally (axisymmetric plasma)
        phi = 2 * np.pi * rank / max(world, 1)
        rot = np.array([[np.cos(phi), -np.sin(phi), 0], [np.sin(phi), np.cos(phi), 0], [0, 0, 1]])
        pos, dirs = pos @ rot.T, dirs @ rot.T
    t_entry = time.perf_counter()
    xp, Np, s0, st = T.ray_entry(plasma, pos, dirs, omega, args.mode, gpu=True)
    t_entry = time.perf_counter() - t_entry  # first call: includes device setup
    if not (st == 0).all():
        raise RuntimeError(f"ray entry failed for {(st != 0).sum()} rays")
    n = len(w)
    grid = np.linspace(0.0, 1.0, args.n_psi)

    def dev_t(a, dtype=torch.float64):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype)

    d_x0, d_N0, d_w, d_grid = dev_t(xp.T), dev_t(Np.T), dev_t(w), dev_t(grid)
    d_state = torch.empty((7, n), dtype=torch.float64, device=dev)
    d_status = torch.empty(n, dtype=torch.int32, device=dev)
    d_steps = torch.empty(n, dtype=torch.int32, device=dev)
    d_dP = torch.zeros(args.n_psi + 1, dtype=torch.float64, device=dev)
    d_Pdep = torch.empty(n, dtype=torch.float64, device=dev)
    adaptive = args.integrator == "adaptive"
    cap = 2 * args.n_steps + 400 if adaptive else args.n_steps  # accepted-step capacity
    n_save = (cap if adaptive else args.n_steps) // args.traj_stride if args.traj_stride > 0 else 0
    d_traj = torch.empty((max(n_save, 1), 5, n), dtype=torch.float64, device=dev)
    d_cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    dep = 1 if args.deposition == "reference" else 0
    cfg = T._lib.TraceCfg(omega, args.mode, args.ds, cap, max(1, args.n_steps // 100),
                          1.0, 1e-6, ABSORPTION[args.absorption], args.traj_stride, dep,
                          int(adaptive), 1e-6, 1e-6,
                          args.n_steps * args.ds, 100)
    d_xl, d_s0 = dev_t(pos.T), dev_t(s0)
    L = T.lib()
    # the hot path's caller stream: a stream of its own (non-blocking, like the
    # library's internal ones), made torch's current stream so that the per-step
    # zeroing runs on it too; TORJ_BENCH_STREAM=default keeps torch's default
    # (legacy NULL) stream, which synchronises implicitly with blocking streams
    if os.environ.get("TORJ_BENCH_STREAM", "own") == "default":
        stream = torch.cuda.current_stream(dev)
    else:
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)

    def launch(counters=None):
        d_dP.zero_()
        T._lib.check(L.torj_trace_device_ex(
            plasma.handle, cfg, n, d_x0.data_ptr(), d_N0.data_ptr(), d_w.data_ptr(), args.n_psi,
            d_grid.data_ptr(), d_xl.data_ptr(), d_s0.data_ptr(), d_state.data_ptr(),
            d_status.data_ptr(), d_steps.data_ptr(), d_dP.data_ptr(), d_Pdep.data_ptr(),
            d_traj.data_ptr() if n_save else None, counters, stream.cuda_stream))

    def progress(msg):  # heartbeat on stderr (long warm-model launches), never on stdout
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    def one_step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        launch()
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            allreduce_deposition(d_dP)  # RCCL over xGMI: (n_psi+1) fp64, make_beam's reduce

    # counted launch (work counters for the algorithmic FLOP figure), also warms up
    d_cnt.zero_()
    launch(d_cnt.data_ptr())
    T._lib.check(L.torj_trace_check(plasma.handle, stream.cuda_stream))  # all groups retired
    progress("counted launch done")
    cnt = d_cnt.cpu().numpy().astype(np.int64)
    ray_steps_local = int(cnt[0])
    for k in range(args.warmup):
        one_step()
        torch.cuda.synchronize(dev)
        progress(f"warmup {k + 1}/{args.warmup} done")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    T._lib.check(L.torj_timing(plasma.handle, 1))  # library HIP events around each phase
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    T._lib.check(L.torj_trace_check(plasma.handle, stream.cuda_stream))
    progress(f"timed region done: {elapsed:.2f} s")
    hot_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))  # whole torj_trace_device_ex call
    import ctypes
    n_calls, t_trace, t_post = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    T._lib.check(L.torj_timing_read(plasma.handle, ctypes.byref(n_calls), ctypes.byref(t_trace),
                                    ctypes.byref(t_post)))
    T._lib.check(L.torj_timing(plasma.handle, 0))
    kern_ms = t_trace.value / max(n_calls.value, 1)  # the trace kernel alone
    post_ms = t_post.value / max(n_calls.value, 1)   # deposition kernels (reference mode)
    tot_steps = torch.tensor([ray_steps_local], dtype=torch.float64, device=dev)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    km = torch.tensor([kern_ms, post_ms, hot_ms], dtype=torch.float64, device=dev)
    per_rank = None
    if world > 1:
        # make_beam's reduce alone (outside the timed region): the RCCL all-reduce
        # of the (n_psi + 1) vector, timed over 20 calls on a scratch copy
        scratch = d_dP.clone()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t_r = time.perf_counter()
        for _ in range(20):
            allreduce_deposition(scratch)
        torch.cuda.synchronize(dev)
        reduce_ms = (time.perf_counter() - t_r) / 20 * 1e3
        mine = torch.tensor([kern_ms, post_ms, hot_ms, elapsed / args.steps * 1e3, float(n),
                             float(ray_steps_local), reduce_ms, float(torch.cuda.current_device()),
                             float(dist.get_rank()), float(dist.get_world_size())],
                            dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        rows = [a.cpu().numpy() for a in allr]
        per_rank = {"trace_ms": [float(r[0]) for r in rows], "deposition_ms": [float(r[1]) for r in rows],
                    "call_ms": [float(r[2]) for r in rows], "step_ms": [float(r[3]) for r in rows],
                    "rays": [int(r[4]) for r in rows], "ray_steps": [int(r[5]) for r in rows],
                    "rccl_allreduce_ms": [float(r[6]) for r in rows],
                    # who took part: each rank's HIP device (torch.cuda.current_device) and its
                    # rank / size in the process group the all_reduce ran over
                    "device": [int(r[7]) for r in rows], "pg_rank": [int(r[8]) for r in rows],
                    "pg_size": [int(r[9]) for r in rows], "backend": dist.get_backend()}
        dist.all_reduce(tot_steps)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ray_steps_all = float(tot_steps.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = ray_steps_all / (ms_per_step / 1e3)

    if rank == 0:
        status = d_status.cpu().numpy()
        # the headline launches' outputs (the parity sample's GPU side), before any
        # later leg reuses the buffers
        gpu_out = (d_state.cpu().numpy().T.copy(), status.copy(), d_steps.cpu().numpy())
        flop =(F.algorithmic_flops(cnt, n_gl=24) if args.absorption in ("albajar", "none")
                else F.algorithmic_flops_warm(cnt) if args.absorption == "warm_wr" else None)
        n_simd = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        sched = adaptive or (os.environ.get("TORJ_SCHED", "1") != "0" and (n + 63) // 64 > n_simd)
        dm = 2 if args.deposition == "reference" else 1
        at = ABSORPTION[args.absorption]  # ABS template: 0 cold, 1 Albajar, 2 / 3 warm iwarm 1 / 3
        # the library's default for a large fixed-step Albajar beam: the split
        # pipeline -- its kernels are timed together as the trace phase
        sw = os.environ.get("TORJ_SPLIT_WARM", "-1")
        split = (not adaptive and os.environ.get("TORJ_SPLIT", "1") == "1"
                 and ((sched and args.absorption == "albajar")
                      or (args.absorption == "warm_wr" and sw != "0")
                      or (args.absorption == "warm_fr" and (sw == "1" or (sw != "0" and (n + 63) // 64 < 3 * n_simd // 4)))))
        # small Albajar beams run 16 lanes per ray (the library's automatic choice)
        lpr16 = (not sched and at == 1 and dm == 2 and os.environ.get("TORJ_LPR", "0") != "1"
                 and n * 16 <= n_simd * 2 * 64)
        kname = ((SPLIT_KERNELS if at == 1 else SPLIT_KERNELS.replace("k_alpha_pts", "k_alpha_warm_pts"))
                 if split
                 else f"k_trace_sched<{at}, {dm}, true, {int(adaptive)}>" if sched
                 else f"k_trace<{at}, {dm}, true, 16>" if lpr16
                 else f"k_trace<{at}, {dm}, true>")  # rocprof's name of the instance
        traffic = measured_traffic(kname, n, args, L.torj_build_id().decode())
        kern_s = float(km[0].item()) / 1e3
        flop_source = ("algorithmic (torj_hip/flops.py algorithmic_flops_warm x the kernel's "
                       "8 work counters; a lower bound, oracle/flopcount_warm.py)"
                       if args.absorption == "warm_wr"
                       else "algorithmic (torj_hip/flops.py x the kernel's work counters)")
        if flop is None and traffic and traffic.get("fp64_flops_executed"):
            # warm_fr: no op-count model (its t-quadrature's expei branches);
            # executed fp64 VALU FLOPs of the same kernel and workload from the
            # committed PMC profile
            flop = traffic["fp64_flops_executed"]
            flop_source = f"executed: PMC SQ_INSTS_VALU_*_F64 x 64 lanes ({traffic['file']})"
        achieved = flop / kern_s / 1e12 if flop is not None else None
        out = {
            "metric": "ray-steps/sec, 1e5-ray EC fan on 1 MI355X (+ 2/4/8-GPU scaling)",
            "value": value,
            "unit": "ray-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if args.shard else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic circular-tokamak equilibrium (analytic, sampled on 56x56) + "
                    "launch_peripheral_rays fan",
            "config": {
                "workload": f"{'C5' if args.absorption.startswith('warm') else ('C4' if args.shard else 'C3')}: "
                            f"{(str(n_fan) + '-ray EC fan sharded over ' + str(world) + ' GPU(s)') if args.shard else (str(n) + '-ray EC fan per GPU')} (N_rings={args.n_rings}, "
                            f"min_az={args.min_az}), X-mode {f/1e9:.1f} GHz, {args.n_steps} RK4 "
                            f"steps ds={args.ds:g} m ({args.integrator}), {ALPHA_NAME[args.absorption]}, psi-shell deposition "
                            f"n_psi={args.n_psi} ({args.deposition}), traj stride {args.traj_stride}",
                "rays_per_gpu": n,
                "rays_total": n_fan if args.shard else n * world,
                "rk4_steps": args.n_steps,
                "n_psi": args.n_psi,
                "traj_stride": args.traj_stride,
                "absorption": args.absorption,
                # harmonics whose rigorous share of alpha is below this are not
                # integrated (m^-1; 0 = every integral, the reference's work)
                "tiny_alpha": tiny_alpha() if args.absorption == "albajar" else None,
                "build_id": L.torj_build_id().decode(),
                "torj_env": torj_env(),
                "parallelism": (f"ray-shard x{world} on ONE device (TORJ_BENCH_SAME_DEVICE rehearsal, "
                                f"gloo all_reduce of dP/dV)" if same_dev
                                else f"ray-shard x{world} + RCCL all_reduce of dP/dV"),
                "ray_status_counts": {T.STATUS_NAMES[i]: int(c)
                                      for i, c in enumerate(np.bincount(status, minlength=6)) if c},
            },
            "roofline": {
                "bound": "fp64-valu",
                "achieved": achieved,
                "peak": FP64_VECTOR_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / FP64_VECTOR_PEAK_TFLOPS if achieved is not None else None,
                "traffic": traffic["traffic_bytes"] if traffic else None,
                "traffic_source": traffic["file"] if traffic else None,
                "hbm_GBps": traffic["traffic_bytes"] / kern_s / 1e9 if traffic else None,
                "hbm_frac": traffic["traffic_bytes"] / kern_s / HBM_PEAK_BPS if traffic else None,
                "valu_busy": traffic.get("valu_busy") if traffic else None,
                "valu_busy_by_kernel": traffic.get("valu_busy_by_kernel") if traffic else None,
                "valu_active_per_wave": traffic.get("valu_active_per_wave") if traffic else None,
                # executed fp64 FLOPs of the same kernel and workload (PMC:
                # SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 x 64 lanes, FMA x 2)
                "executed_TFLOPs": (traffic["fp64_flops_executed"] / kern_s / 1e12
                                    if traffic and traffic.get("fp64_flops_executed") else None),
                "frac_executed": (traffic["fp64_flops_executed"] / kern_s / 1e12 / FP64_VECTOR_PEAK_TFLOPS
                                  if traffic and traffic.get("fp64_flops_executed") else None),
                "kernel": kname,
                "kernel_ms": kern_s * 1e3,
                "kernel_ms_note": ("the trace phase: the split pipeline's kernels (trajectory, alpha, "
                                   "tau scan and, for the reference profile, the deposition walk's "
                                   "streamed windows, whose work the FLOP count does not price) "
                                   "overlapped on three streams, HIP events on the launch stream "
                                   "around all of them"
                                   if split else "HIP events around the trace kernel"),
                "rocprof_per_launch_ms": traffic.get("rocprof_per_launch_ms") if traffic else None,
                "deposition_kernels_ms": float(km[1].item()),
                "hot_path_ms": float(km[2].item()),
                "flop_per_launch": flop,
                "flop_source": flop_source if flop is not None else None,
                "flop_per_ray_step": flop / max(cnt[0], 1) if flop is not None else None,
                "flop_model": FLOP_MODEL.get(args.absorption),
            },
            # NOT achieved hardware throughput: the same launch priced as the reference's
            # algorithm, which evaluates the integrals the kernel skips bit-identically
            # (exact zeros, negligible ones, the harmonics of calls settled before the
            # polarisation vector), over the measured time -- a work-equivalent rate
            "work_equivalent": ({
                "flop_per_launch_reference_algorithm": F.algorithmic_flops_reference(cnt, n_gl=24),
                "reference_algorithm_equivalent_TFLOPs":
                    F.algorithmic_flops_reference(cnt, n_gl=24) / kern_s / 1e12,
                "note": "the reference algorithm's op count over the measured trace phase; the "
                        "kernel skips part of that work (bit-identically, or below tiny_alpha = "
                        "1e-20 m^-1 of absorption with tau moved by < 2e-20 per metre), so this is "
                        "not achieved throughput (roofline.frac is)",
            } if args.absorption == "albajar" else None),
            "work_counters": (
                {"ray_steps": int(cnt[0]), "rhs_evals": int(cnt[1]),
                 "faddeeva_evals_asymptotic": int(cnt[2]), "faddeeva_evals": int(cnt[3]),
                 "warmdisp_passes": int(cnt[4]), "passes_x_lrm": int(cnt[5]),
                 "sum_lrm": int(cnt[6]), "sum_lrm2": int(cnt[7])}
                if args.absorption == "warm_wr" else
                {"ray_steps": int(cnt[0]), "rhs_evals": int(cnt[1]),
                 "alpha_active": int(cnt[2]), "harmonic_integrals": int(cnt[3]),
                 "bessel_series_terms": int(cnt[4]),
                 "harmonic_integrals_exact_zero": int(cnt[5]),
                 "harmonic_integrals_negligible": int(cnt[6]),
                 "harmonic_integrals_settled_early": int(cnt[7])}),
        }
        if per_rank is not None:
            out["multi_gpu"] = multi_gpu_block(per_rank, path="torchrun: one process per GPU, "
                                               "torj_trace_device_ex per rank + torch.distributed "
                                               "all_reduce of dP_shell")
        if world == 1 and not args.no_host_api:
            # the same beam through make_beam's library path (torj_trace_beam_device,
            # what `--gpus N` in one process times), so an N = 1 point of either path
            # compares with the N >= 2 lines of both
            out["library_path"] = library_path_rate(T, plasma, cfg, args, n, d_x0, d_N0, d_w, d_grid,
                                                    d_xl, d_s0, d_state, d_status, d_steps, d_dP,
                                                    d_Pdep, d_traj if n_save else None,
                                                    ray_steps_local, value)
            progress("library-path steps done")
        if world == 1 and not args.no_host_api:
            out["host_api"] = host_api_rate(T, plasma, cfg, xp, Np, w, grid, n_save, ray_steps_local,
                                            pos, s0)
            progress("host-pointer call done")
            if not args.no_beam_host and args.absorption == "albajar" and not adaptive:
                out["host_api_beam_c4"] = host_beam_c4(T, plasma, cfg, args, omega, n_save)
                progress("C4-scale torj_trace_beam call done")
            out["ray_entry"] = entry_timing(T, plasma, pos, dirs, omega, args.mode, t_entry)
        exact_out = None
        if (world == 1 and args.absorption == "albajar" and not adaptive and not args.no_exact
                and tiny_alpha() > 0.0):
            out["exact"], exact_out = exact_leg(T, L, plasma, launch, dev, args, value, kern_ms, post_ms,
                                                d_state, d_status, d_steps, gpu_out)
            progress("exact (TORJ_TINY_ALPHA=0) leg done")
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"], parity = cpu_baseline(eq, xp, Np, w, omega, args, grid, gpu_out,
                                                       exact_out)
            if parity is not None:
                if exact_out is not None:
                    out["exact"]["parity"] = parity.pop("exact")
                out["parity"] = parity
        elif world > 1 and args.parity_rays > 0 and args.integrator == "rk4":
            # rank 0's shard against the oracle (bounded sample, untimed)
            out["parity"] = parity_sample(eq, xp, Np, w, omega, args, grid, gpu_out, args.parity_rays)
            out["parity"]["shard"] = "rank 0"
        check_line(out)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_library(args):
    """`python bench.py --gpus N` in ONE process (no torchrun): make_beam's
    library path over N devices, torj_trace_beam_device -- device-resident ray
    shards (inputs in HBM before the timed region), one host thread + stream per
    device, then the RCCL all-reduce of the (n_psi + 1) deposition vector
    (src/solve.jl:209-240).  Weak scaling (default): each device its own beam,
    rotated toroidally by 2 pi k / N; --shard: ONE fan cut into N contiguous
    64-ray-aligned shards (C4, strong).  Exits non-zero before any GPU work when
    fewer than N devices are visible.  TORJ_BEAM_SAME_DEVICE=1 rehearses the
    N-replica path on device 0 (labelled in the line; not a scaling figure)."""
    import ctypes

    import torch

    same = os.environ.get("TORJ_BEAM_SAME_DEVICE", "0") not in ("", "0")
    n_vis = torch.cuda.device_count()  # does not initialise the GPU on this image
    if n_vis < args.gpus and not same:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible HIP devices, found {n_vis}",
              file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.init()  # torch's HIP runtime first, then the library's (tests/conftest.py)
    import torj_hip as T
    from torj_hip import flops as F
    from torj_hip import synthetic as S
    from torj_hip.parallel import beam_comm_info, group_shard, trace_beam_device

    N = args.gpus
    eq = S.circular_tokamak()
    plasma = T.Plasma(*S.plasma_args(eq), device=0)
    T.abs_Al_init(24)
    f = args.freq
    omega = 2 * np.pi * f
    setup = S.SETUP
    N0 = T.pol_tor_angles_2_vector(setup["steering_angle_pol"], setup["steering_angle_tor"])
    x0 = np.array([setup["R0"], 0.0, setup["z0"]])
    pos, dirs, w = T.launch_peripheral_rays(x0, N0, setup["spot_size"], setup["inverse_curvature_radius"],
                                            f, N_rings=args.n_rings, min_azimuthal_points=args.min_az)
    n_fan = len(w)
    parts = []  # per device: (launch points, directions, weights)
    for k in range(N):
        if args.shard:
            sl = group_shard(n_fan, N, k)
            parts.append((pos[sl], dirs[sl], w[sl]))
        else:
            phi = 2 * np.pi * k / N
            rot = np.array([[np.cos(phi), -np.sin(phi), 0], [np.sin(phi), np.cos(phi), 0], [0, 0, 1]])
            parts.append((pos @ rot.T, dirs @ rot.T, w))
    grid = np.linspace(0.0, 1.0, args.n_psi)
    adaptive = args.integrator == "adaptive"
    cap = 2 * args.n_steps + 400 if adaptive else args.n_steps
    n_save = cap // args.traj_stride if args.traj_stride > 0 else 0
    dep = 1 if args.deposition == "reference" else 0
    cfg = T._lib.TraceCfg(omega, args.mode, args.ds, cap, max(1, args.n_steps // 100), 1.0, 1e-6,
                          ABSORPTION[args.absorption], args.traj_stride, dep, int(adaptive), 1e-6,
                          1e-6, args.n_steps * args.ds, 100)
    shards = []
    for k, (p_k, d_k, w_k) in enumerate(parts):
        xp, Np, s0, st = T.ray_entry(plasma, p_k, d_k, omega, args.mode, gpu=True)
        if not (st == 0).all():
            raise RuntimeError(f"ray entry failed for {(st != 0).sum()} rays of shard {k}")
        dev = torch.device("cuda", 0 if same else k % n_vis)
        n = len(w_k)

        def d(a, dtype=torch.float64):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype)

        shards.append(dict(
            n=n, x0=d(xp.T), N0=d(Np.T), weights=d(w_k), psi_grid=d(grid), x_launch=d(p_k.T), s0=d(s0),
            state=torch.empty((7, n), dtype=torch.float64, device=dev),
            status=torch.empty(n, dtype=torch.int32, device=dev),
            steps=torch.empty(n, dtype=torch.int32, device=dev),
            dP_shell=torch.zeros(args.n_psi + 1, dtype=torch.float64, device=dev),
            P_dep=torch.empty(n, dtype=torch.float64, device=dev),
            traj=(torch.empty((n_save, 5, n), dtype=torch.float64, device=dev) if n_save else None),
            counters=torch.zeros(8, dtype=torch.int64, device=dev)))
    devs = sorted({sh["state"].device.index for sh in shards})

    def sync():
        for i in devs:
            torch.cuda.synchronize(i)

    def step(counted=False):
        for sh in shards:  # make_beam's sums start at 0 (the trace accumulates)
            sh["dP_shell"].zero_()
        sync()  # torch's zeroing before the library's own streams read them
        trace_beam_device(plasma, cfg, args.n_psi,
                          [dict(sh, counters=sh["counters"] if counted else None) for sh in shards])

    def progress(msg):
        print(f"[bench] {msg}", file=sys.stderr, flush=True)

    step(counted=True)
    cnt = [sh["counters"].cpu().numpy().astype(np.int64) for sh in shards]
    ray_steps = int(sum(c[0] for c in cnt))
    progress("counted launch done")
    for k in range(args.warmup):
        step()
        progress(f"warmup {k + 1}/{args.warmup} done")
    sync()
    L = T.lib()
    T._lib.check(L.torj_timing(plasma.handle, 1))  # the handle and every replica: per-device phases
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    progress(f"timed region done: {elapsed:.2f} s")
    calls = (ctypes.c_int * N)()
    t_trace, t_post = (ctypes.c_double * N)(), (ctypes.c_double * N)()
    t_red = ctypes.c_double()
    T._lib.check(L.torj_beam_timing_read(plasma.handle, N, calls, t_trace, t_post, ctypes.byref(t_red)))
    T._lib.check(L.torj_timing(plasma.handle, 0))
    trace_ms = [t_trace[k] / max(calls[k], 1) for k in range(N)]
    dep_ms = [t_post[k] / max(calls[k], 1) for k in range(N)]
    kern_ms, post_ms = trace_ms[0], dep_ms[0]
    rccl_ms = t_red.value / max(args.steps, 1)
    # the fan-out + reduce overhead alone: empty shards, the same deposition vectors
    empty = [dict(n=0, psi_grid=sh["psi_grid"], dP_shell=sh["dP_shell"]) for sh in shards]
    t1 = time.perf_counter()
    for _ in range(20):
        trace_beam_device(plasma, cfg, args.n_psi, empty)
    reduce_ms = (time.perf_counter() - t1) / 20 * 1e3
    ms_per_step = elapsed / args.steps * 1e3
    value = ray_steps / (ms_per_step / 1e3)
    flop0 = (F.algorithmic_flops(cnt[0], n_gl=24) if args.absorption in ("albajar", "none")
             else F.algorithmic_flops_warm(cnt[0]) if args.absorption == "warm_wr" else None)
    achieved = flop0 / (kern_ms / 1e3) / 1e12 if flop0 is not None and kern_ms > 0 else None
    # device 0's launch is the profiled single-device workload when each device
    # traces the whole fan (weak scaling): its HBM bytes per launch from the
    # profile of the same build, workload and switches (None otherwise, e.g. for
    # the C4 shards, which no profile covers)
    traffic0 = None
    if args.absorption in ("albajar", "warm_wr"):
        try:
            kn = SPLIT_KERNELS if args.absorption == "albajar" else SPLIT_KERNELS.replace("k_alpha_pts",
                                                                                            "k_alpha_warm_pts")
            traffic0 = measured_traffic(kn, int(shards[0]["n"]), args, L.torj_build_id().decode())
        except Exception:  # a missing or malformed profile leaves the field empty
            traffic0 = None
    dP0 = shards[0]["dP_shell"].cpu().numpy()
    agree = max(float(np.abs(sh["dP_shell"].cpu().numpy() - dP0).max()) for sh in shards)
    placement = ("same-device rehearsal (TORJ_BEAM_SAME_DEVICE=1): all replicas on device 0, partials "
                 "summed on the host -- not a scaling measurement" if same else
                 f"replica k on device k (of {n_vis} visible), RCCL all-reduce over xGMI")
    out = {
        "metric": "ray-steps/sec, 1e5-ray EC fan on 1 MI355X (+ 2/4/8-GPU scaling)",
        "value": value,
        "unit": "ray-steps/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.shard else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic circular-tokamak equilibrium (analytic, sampled on 56x56) + "
                "launch_peripheral_rays fan",
        "config": {
            "workload": (f"{'C4' if args.shard else 'C3'} via the library path torj_trace_beam_device: "
                         + (f"{n_fan}-ray EC fan sharded over {N} devices" if args.shard
                            else f"{n_fan}-ray EC fan per device") +
                         f" (N_rings={args.n_rings}, min_az={args.min_az}), X-mode {f/1e9:.1f} GHz, "
                         f"{args.n_steps} RK4 steps ds={args.ds:g} m ({args.integrator}), "
                         f"{ALPHA_NAME[args.absorption]}, psi-shell deposition n_psi={args.n_psi} "
                         f"({args.deposition}), traj stride {args.traj_stride}"),
            "rays_per_device": [sh["n"] for sh in shards],
            "rays_total": int(sum(sh["n"] for sh in shards)),
            "rk4_steps": args.n_steps,
            "n_psi": args.n_psi,
            "absorption": args.absorption,
            "parallelism": (f"one process, {N} replicas (host thread + stream each), device-resident "
                            f"ray shards, RCCL all-reduce of dP_shell"),
            "placement": placement,
            "n_devices_used": len(devs),
            "tiny_alpha": tiny_alpha(),
            "build_id": L.torj_build_id().decode(),
        },
        "roofline": {
            "bound": "fp64-valu",
            "achieved": achieved,
            "peak": FP64_VECTOR_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / FP64_VECTOR_PEAK_TFLOPS if achieved is not None else None,
            "traffic": traffic0["traffic_bytes"] if traffic0 else None,
            "traffic_source": ((traffic0["file"] + ": the single-device profile of device 0's launch "
                                "(same build, rays, steps and switches), not measured in this run")
                               if traffic0 else None),
            "note": "device 0's trace phase (library HIP events) and its shard's counted FLOPs",
            "kernel_ms": kern_ms,
            "deposition_kernels_ms": post_ms,
            "flop_per_launch": flop0,
        },
        "beam": {
            "call_ms": ms_per_step,
            "device0_trace_ms": kern_ms,
            "device0_deposition_ms": post_ms,
            "fanout_reduce_only_ms": reduce_ms,
            "dP_shell_max_diff_between_devices": agree,
            "deposited_power_sum": float(dP0[-1]),
        },
        "multi_gpu": multi_gpu_block(
            {"trace_ms": trace_ms, "deposition_ms": dep_ms, "call_ms": [ms_per_step] * N,
             "step_ms": [ms_per_step] * N, "rays": [sh["n"] for sh in shards],
             "ray_steps": [int(c[0]) for c in cnt], "rccl_allreduce_ms": [rccl_ms] * N,
             # torj_beam_comm_info: each replica's HIP device and its RCCL communicator's
             # rank count / rank (ncclCommCount / ncclCommUserRank; 0 / -1: no communicator)
             **beam_comm_info(plasma, N)},
            path="one process: torj_trace_beam_device, a host thread + stream per device, the "
                 "library's RCCL all-reduce (ncclCommInitAll)"),
    }
    if args.parity_rays > 0 and args.integrator == "rk4":
        sh0 = shards[0]
        p0 = parts[0]
        xp0, Np0, _, _ = T.ray_entry(plasma, p0[0], p0[1], omega, args.mode, gpu=True)
        gpu_out = (sh0["state"].cpu().numpy().T, sh0["status"].cpu().numpy(), sh0["steps"].cpu().numpy())
        out["parity"] = parity_sample(eq, xp0, Np0, p0[2], omega, args, grid, gpu_out, args.parity_rays)
        out["parity"]["shard"] = "device 0"
    check_line(out)
    print(json.dumps(out), flush=True)


# keys every bench line carries (the driver's contract), and those of an N >= 2
# line's multi_gpu block; tests/test_bench_cli.py pins both
LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
             "scaling", "vs_baseline", "dtype", "data", "config", "roofline")
MULTI_GPU_KEYS = ("path", "trace_ms_per_device", "deposition_ms_per_device", "call_ms_per_device",
                  "rays_per_device", "ray_steps_per_device", "trace_ms_max", "trace_ms_min",
                  "imbalance", "rccl_allreduce_ms", "device")
# and who took part in the reduce, per path: the library path's RCCL communicator
# (torj_beam_comm_info), torchrun's process group
MULTI_GPU_COMM_KEYS = {"library": ("rccl_nranks", "rccl_rank"), "torchrun": ("pg_rank", "pg_size", "backend")}


def multi_gpu_block(per, path):
    """The N >= 2 line's per-device figures: every device's trace-phase and
    deposition milliseconds (library HIP events), its call time, rays and
    ray-steps, the spread of the trace phase (max / min - 1) and the RCCL
    all-reduce of make_beam's reduce (src/solve.jl:233-240)."""
    tr = [float(v) for v in per["trace_ms"]]
    extra = {k: per[k] for k in ("device", "pg_rank", "pg_size", "backend", "rccl_nranks", "rccl_rank")
             if k in per}
    return {"path": path, **extra,
            "trace_ms_per_device": tr,
            "deposition_ms_per_device": [float(v) for v in per["deposition_ms"]],
            "call_ms_per_device": [float(v) for v in per["call_ms"]],
            "rays_per_device": [int(v) for v in per["rays"]],
            "ray_steps_per_device": [int(v) for v in per["ray_steps"]],
            "trace_ms_max": max(tr), "trace_ms_min": min(tr),
            "imbalance": max(tr) / max(min(tr), 1e-9) - 1.0,
            "rccl_allreduce_ms": float(max(per["rccl_allreduce_ms"]))}


def check_line(out):
    """The line's schema (raises before printing a malformed line)."""
    missing = [k for k in LINE_KEYS if k not in out]
    if missing:
        raise KeyError(f"bench line lacks {missing}")
    if out["n_gpus"] > 1:
        mg = out.get("multi_gpu")
        if mg is None or any(k not in mg for k in MULTI_GPU_KEYS):
            raise KeyError("an N >= 2 line needs the multi_gpu block with " + ", ".join(MULTI_GPU_KEYS))
        if len(mg["trace_ms_per_device"]) != out["n_gpus"] or len(mg["device"]) != out["n_gpus"]:
            raise ValueError("multi_gpu: one trace_ms and one device entry per device")
        if not any(all(k in mg for k in ks) for ks in MULTI_GPU_COMM_KEYS.values()):
            raise KeyError("multi_gpu: the reduce's participants (" + " or ".join(
                ", ".join(ks) for ks in MULTI_GPU_COMM_KEYS.values()) + ")")
    return out


def library_path_rate(T, plasma, cfg, args, n, d_x0, d_N0, d_w, d_grid, d_xl, d_s0, d_state, d_status,
                      d_steps, d_dP, d_Pdep, d_traj, ray_steps, value_main):
    """The N = 1 beam through torj_trace_beam_device (the library's make_beam
    fan-out, what `bench.py --gpus N` times in one process) on the same device
    buffers: min(steps, 10) timed calls after one warm one, host clock with the
    device drained on both sides, as the headline's timed region."""
    import torch
    from torj_hip.parallel import trace_beam_device

    sh = dict(n=n, x0=d_x0, N0=d_N0, weights=d_w, psi_grid=d_grid, x_launch=d_xl, s0=d_s0,
              state=d_state, status=d_status, steps=d_steps, dP_shell=d_dP, P_dep=d_Pdep, traj=d_traj)

    def call():
        d_dP.zero_()
        torch.cuda.synchronize()
        trace_beam_device(plasma, cfg, args.n_psi, [sh])

    call()
    k = max(1, min(args.steps, 10))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        call()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    v = ray_steps / dt
    return {"value": v, "unit": "ray-steps/s", "ms_per_step": dt * 1e3, "steps": k,
            "vs_headline": v / value_main,
            "note": "torj_trace_beam_device with one shard on this device (includes the per-call "
                    "zeroing of dP_shell and the library's synchronous return)"}


def host_beam_c4(T, plasma, cfg, args, omega, n_save):
    """make_beam's host-pointer form (torj_trace_beam, what the Julia shim's
    make_beam calls) at C4 scale on this device: the 1 005 293-ray fan
    (N_rings = 291) from pageable host arrays to pageable host arrays, the
    automatic shards (pinned staging, transfers overlapping the traces), one
    warm call then one timed.  PCIe-inclusive; reported beside the headline."""
    from torj_hip import synthetic as S

    setup = S.SETUP
    N0 = T.pol_tor_angles_2_vector(setup["steering_angle_pol"], setup["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays(np.array([setup["R0"], 0.0, setup["z0"]]), N0,
                                            setup["spot_size"], setup["inverse_curvature_radius"],
                                            args.freq, N_rings=291, min_azimuthal_points=args.min_az)
    xp, Np, s0, st = T.ray_entry(plasma, pos, dirs, omega, args.mode, gpu=True)
    n = len(w)
    xs, Ns, xl = (np.ascontiguousarray(a.T) for a in (xp, Np, pos))
    grid = np.linspace(0.0, 1.0, args.n_psi)
    state, status, steps = np.zeros((7, n)), np.zeros(n, np.int32), np.zeros(n, np.int32)
    dP, Pdep = np.zeros(args.n_psi + 1), np.zeros(n)
    traj = np.zeros((max(n_save, 1), 5, n))
    dp, ip = T._lib.dptr, T._lib.iptr
    L = T.lib()

    def call():
        T._lib.check(L.torj_trace_beam(plasma.handle, cfg, n, dp(xs), dp(Ns), dp(w), args.n_psi, dp(grid),
                                       dp(xl), dp(s0), dp(state), ip(status), ip(steps), dp(dP), dp(Pdep),
                                       dp(traj) if n_save else None, 1, 0))

    call()
    t0 = time.perf_counter()
    call()
    dt = time.perf_counter() - t0
    ray_steps = float(steps.sum())
    return {"value": ray_steps / dt, "unit": "ray-steps/s", "ms": dt * 1e3, "rays": n,
            "ray_steps": int(ray_steps), "shards": -(-n // 131072),
            "status_ok": int((status == 0).sum()),
            "d2h_bytes": int(state.nbytes + status.nbytes + steps.nbytes + Pdep.nbytes
                             + (traj.nbytes if n_save else 0)),
            "note": "torj_trace_beam, 1 device, n_shards = 0 (automatic), host arrays both ways "
                    "incl. PCIe (not the headline)"}


def host_api_rate(T, plasma, cfg, xp, Np, w, grid, n_save, ray_steps, pos, s0):
    """PCIe-inclusive rate of the host-pointer boundary (torj_trace: device
    allocation, H2D of the start states, the trace, D2H of state, status,
    steps, dP_shell, P_dep and the trajectory).  Reported beside `value`,
    never as it."""
    n = len(w)
    xs, Ns = np.ascontiguousarray(xp.T), np.ascontiguousarray(Np.T)
    state, status, steps = np.zeros((7, n)), np.zeros(n, np.int32), np.zeros(n, np.int32)
    dP, Pdep = np.zeros(len(grid) + 1), np.zeros(n)
    traj = np.zeros((max(n_save, 1), 5, n))
    dp, ip = T._lib.dptr, T._lib.iptr
    t0 = time.perf_counter()
    xl = np.ascontiguousarray(pos.T)
    T._lib.check(T.lib().torj_trace_ex(plasma.handle, cfg, n, dp(xs), dp(Ns), dp(w), len(grid),
                                       dp(grid), dp(xl), dp(s0), dp(state), ip(status), ip(steps),
                                       dp(dP), dp(Pdep), dp(traj) if n_save else None))
    dt = time.perf_counter() - t0
    return {"value": ray_steps / dt, "unit": "ray-steps/s", "ms": dt * 1e3,
            "d2h_bytes": int(state.nbytes + status.nbytes + steps.nbytes + dP.nbytes + Pdep.nbytes
                             + (traj.nbytes if n_save else 0)),
            "note": "torj_trace host-pointer path incl. PCIe transfers (not the headline)"}


def entry_timing(T, plasma, pos, dirs, omega, mode, t_first):
    """first_point + vacuum_plasma_refraction for the whole beam (setup, outside
    `value`): the GPU kernel through the host-pointer ABI, vs the host C++ path."""
    t0 = time.perf_counter()
    T.ray_entry(plasma, pos, dirs, omega, mode, gpu=True)
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    T.ray_entry(plasma, pos, dirs, omega, mode)
    t_host = time.perf_counter() - t0
    return {"gpu_ms": t_gpu * 1e3, "gpu_first_call_ms": t_first * 1e3, "host_ms": t_host * 1e3,
            "host_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or os.cpu_count())}


def tiny_alpha():
    """The tiny-alpha threshold the library reads at abs_Al_init (m^-1)."""
    v = os.environ.get("TORJ_TINY_ALPHA")
    return float(v) if v is not None else TINY_ALPHA_DEFAULT


def exact_leg(T, L, plasma, launch, dev, args, value_main, trace_ms_main, post_ms_main, d_state,
              d_status, d_steps, gpu_out_main):
    """The headline's timed loop again with TORJ_TINY_ALPHA=0: every harmonic
    integral with m >= m_0 evaluated, as the reference does (src/absorption.jl:
    213-223), so what the default's bounded tiny-alpha skip buys
    is visible beside it.  min(steps, 10) launches after one warm one, the host
    clock with the device drained on both sides (the headline's timed region) and
    the library's HIP events for the trace / deposition phases.  Returns the
    leg's figures and its outputs (state, status, steps) for the parity sample."""
    import ctypes

    import torch

    old = os.environ.get("TORJ_TINY_ALPHA")
    os.environ["TORJ_TINY_ALPHA"] = "0"
    try:
        T.abs_Al_init(24)
        launch()
        torch.cuda.synchronize(dev)
        k = max(1, min(args.steps, 10))
        T._lib.check(L.torj_timing(plasma.handle, 1))
        t0 = time.perf_counter()
        for _ in range(k):
            launch()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / k
        n_calls, t_trace, t_post = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        T._lib.check(L.torj_timing_read(plasma.handle, ctypes.byref(n_calls), ctypes.byref(t_trace),
                                        ctypes.byref(t_post)))
        T._lib.check(L.torj_timing(plasma.handle, 0))
        out = (d_state.cpu().numpy().T.copy(), d_status.cpu().numpy(), d_steps.cpu().numpy())
    finally:
        if old is None:
            del os.environ["TORJ_TINY_ALPHA"]
        else:
            os.environ["TORJ_TINY_ALPHA"] = old
        T.abs_Al_init(24)
    ray_steps = float(out[2].astype(np.int64).sum())
    trace_ms = t_trace.value / max(n_calls.value, 1)
    s0, s1 = gpu_out_main[0][:, 6], out[0][:, 6]
    return {"tiny_alpha": 0.0,
            "value": ray_steps / dt, "unit": "ray-steps/s", "ms_per_step": dt * 1e3, "steps": k,
            "trace_ms": trace_ms, "deposition_ms": t_post.value / max(n_calls.value, 1),
            "headline_over_exact": value_main / (ray_steps / dt),
            "trace_ms_saved_by_tiny_alpha": trace_ms - trace_ms_main,
            "status_equal_headline": bool(np.array_equal(out[1], gpu_out_main[1])),
            "steps_equal_headline": bool(np.array_equal(out[2], gpu_out_main[2])),
            "xN_equal_headline": bool(np.array_equal(out[0][:, :6], gpu_out_main[0][:, :6])),
            "max_abs_tau_diff_headline": float(np.abs(s1 - s0).max()),
            "note": "the same launches with TORJ_TINY_ALPHA=0 (every harmonic integral evaluated); "
                    "the headline skips a harmonic whose rigorous share of alpha is below "
                    "config.tiny_alpha m^-1"}, out


def torj_env():
    """The TORJ_* switches of this process (kernel variants, schedules): a
    profile is paired only with a run under the same switches."""
    return {k: v for k, v in sorted(os.environ.items())
            if k.startswith("TORJ_") and k != "TORJ_HIP_LIB"}  # the library: its build id


# switches that place replicas / ranks on devices without changing any kernel:
# not part of the match between a run and a profile
PLACEMENT_ENV = ("TORJ_BENCH_SAME_DEVICE", "TORJ_BEAM_SAME_DEVICE")


def kernel_env(env):
    return {k: v for k, v in env.items() if k not in PLACEMENT_ENV}


def measured_traffic(kname, n, args, build_id):
    """HBM bytes per launch of the hot kernel, measured offline by
    scripts/profile.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gfx950
    correction) and summarised by tools/prof_summary.py into
    profiles/<round>/traffic.json; used only if it was taken on this workload
    and kernel, by a library of the same build id (torj_build_id(): a hash of
    the sources and compile flags) under the same TORJ_* switches (PMC
    collection cannot run inside the timed process)."""
    import glob
    base = kname
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*traffic.json")), reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        wl = t.get("workload", {})
        if (wl.get("build_id") == build_id and kernel_env(wl.get("torj_env", {})) == kernel_env(torj_env())
                and base in (t.get("kernel") or "") and wl.get("rays") == n
                and wl.get("rk4_steps") == args.n_steps and wl.get("n_psi") == args.n_psi
                and wl.get("traj_stride") == args.traj_stride
                and wl.get("absorption", "albajar") == args.absorption):
            t["file"] = os.path.relpath(f, ROOT)
            # VALU-busy of the same profile, SIMD level: the quad-cycles the kernel's
            # waves issued VALU (SQ_ACTIVE_INST_VALU x 4 cycles) over the SIMD-cycles
            # of its dispatches (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024
            # SIMDs).  Overlapped pipeline dispatches each count the shared wall
            # cycles, so there the figure is a lower bound; per kernel beside it.
            # valu_active_per_wave: SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES.
            def simd_busy(c):
                return 4.0 * c["SQ_ACTIVE_INST_VALU"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8.0)
            try:
                summ = json.load(open(f.replace("traffic.json", "pmc_summary.json")))
                pmc = summ["avg"]
                t["valu_busy"] = simd_busy(pmc)
                t["valu_active_per_wave"] = pmc["SQ_ACTIVE_INST_VALU"] / pmc["SQ_WAVE_CYCLES"]
                if summ.get("by_kernel"):
                    t["valu_busy_by_kernel"] = {k: simd_busy(v) for k, v in summ["by_kernel"].items()
                                                if v.get("GRBM_GUI_ACTIVE")}
            except (OSError, ValueError, KeyError, ZeroDivisionError):
                t["valu_busy"] = None
            if "|" in base:  # pipeline: rocprof's per-launch kernel times of the same workload
                t["rocprof_per_launch_ms"] = pipeline_kernel_ms(
                    f.replace("traffic.json", "kernel_stats.csv"), base.split("|"))
            return t
    return None


def pipeline_kernel_ms(stats_csv, kernels):
    """Per-launch milliseconds of each pipeline kernel from a committed
    rocprofv3 --kernel-trace --stats summary (launches = calls of the last,
    once-per-launch kernel).  The pipeline overlaps them on two streams, so
    their sum exceeds the trace phase's wall time."""
    import csv
    try:
        rows = list(csv.DictReader(open(stats_csv)))
    except OSError:
        return None
    tot = {k: 0.0 for k in kernels}
    launches = 0
    for r in rows:
        for k in kernels:
            if k in r["Name"]:
                tot[k] += float(r["TotalDurationNs"]) / 1e6
                if k == kernels[-1]:
                    launches += int(r["Calls"])
    if not launches:
        return None
    return {k: v / launches for k, v in tot.items()}


def _parity(OP, r, idx, xp, Np, omega, args, gpu_out, threads):
    """GPU endpoints of the sampled rays (gpu_out: state, status, steps of the
    whole beam) against the oracle's run r on the same rays."""
    model = ABSORPTION[args.absorption]
    warm = model >= 2
    gs, gst, gk = (a[idx] for a in gpu_out)
    os_ = r["state"]
    ex = np.abs(gs[:, :3] - os_[:, :3]).max(1) / np.linalg.norm(os_[:, :3], axis=1)
    eN = np.abs(gs[:, 3:6] - os_[:, 3:6]).max(1) / np.linalg.norm(os_[:, 3:6], axis=1)
    # tau relative, floored at 1e-6 (tests/test_gpu_parity.py TAU_FLOOR): below
    # it the bar is 1e-16 absolute
    et = np.abs(gs[:, 6] - os_[:, 6]) / np.maximum(np.abs(os_[:, 6]), 1e-6)
    et_strict = np.abs(gs[:, 6] - os_[:, 6]) / np.maximum(np.abs(os_[:, 6]), 1e-300)
    # unfloored relative tau over the rays whose tau a result can resolve
    # (tau_cpu >= 1e-12): the tiny-alpha skip's share there is bounded by
    # 2e-20 per metre / 1e-12
    resolv = np.abs(os_[:, 6]) >= TAU_RESOLVABLE
    parity = {"rays": int(len(idx)), "vs": "oracle/torj_oracle.c (same RK4, same rays)",
              "status_equal": bool(np.array_equal(gst, r["status"])),
              "steps_equal": bool(np.array_equal(gk, r["steps"])),
              "max_rel_x": float(ex.max()), "max_rel_N": float(eN.max()),
              "max_rel_tau": float(et.max()), "tau_floor": 1e-6,
              "max_rel_tau_unfloored": float(et_strict.max()),
              "tau_resolvable": TAU_RESOLVABLE,
              "rays_tau_resolvable": int(resolv.sum()),
              "max_rel_tau_resolvable": float(et_strict[resolv].max()) if resolv.any() else None,
              # below the floor the bar is absolute: the largest |tau_gpu - tau_cpu| there
              # (the tiny-alpha skip moves tau by < 2e-20 per metre of ray)
              "max_abs_tau_below_floor": float(np.where(np.abs(os_[:, 6]) < 1e-6,
                                                        np.abs(gs[:, 6] - os_[:, 6]), 0.0).max()),
              "max_rel": float(max(ex.max(), eN.max(), et.max())),
              "rays_within_bar": int((np.maximum(np.maximum(ex, eN), et)
                                      <= {1: 1e-10, 2: 1e-8, 3: 1e-9}.get(model, 1e-10)).sum()),
              "p99_rel_tau": float(np.quantile(et, 0.99)),
              "worst_tau_ray": {"fan_index": int(idx[int(et.argmax())]),
                                "tau_gpu": float(gs[int(et.argmax()), 6]),
                                "tau_cpu": float(os_[int(et.argmax()), 6])},
              "bar_rel": {1: 1e-10, 2: 1e-8, 3: 1e-9}.get(model, 1e-10),
              "bar": (f"x, N: {dict({1: 1e-10, 2: 1e-8, 3: 1e-9}).get(model, 1e-10):g} relative to "
                      f"|x|, |N|; tau: {dict({1: 1e-10, 2: 1e-8, 3: 1e-9}).get(model, 1e-10):g} "
                      f"relative, i.e. {1e-6 * {1: 1e-10, 2: 1e-8, 3: 1e-9}.get(model, 1e-10):g} "
                      f"absolute below tau = 1e-6 (the floor: P moves by < 1 ulp there); status "
                      f"and steps exact")}
    if model == 1 and resolv.any():
        # the resolvable rays outside the bar unfloored: the oracle's a-priori
        # sensitivity (or_albajar_sensitivity, from the trajectory alone: tau's change
        # when every stage point's alpha inputs move by 2^-45 relative) for each;
        # flagged beyond half the bar, as the C5 line flags (tools/c3_tau_diag.py
        # runs it on every resolvable ray: DESIGN.md 3.7)
        out = np.nonzero(resolv & (et_strict > parity["bar_rel"]))[0]
        sens = (OP.albajar_sensitivity(xp[idx[out]], Np[idx[out]], omega, args.mode, args.ds,
                                       r["steps"][out], n_threads=threads) if len(out) else np.zeros(0))
        fl = ~(sens <= 0.5 * parity["bar_rel"] * np.abs(os_[out, 6]))
        keep = resolv.copy()
        keep[out[fl]] = False
        parity["tau_resolvable_conditioning"] = {
            "rays_out_of_bar": int(len(out)), "rays_out_of_bar_flagged": int(fl.sum()),
            "max_rel_tau_resolvable_excl_flagged": float(et_strict[keep].max()) if keep.any() else None,
            "out_of_bar": [{"fan_index": int(idx[k]), "tau_cpu": float(os_[k, 6]), "rel": float(et_strict[k]),
                            "sens_over_tau": float(sv / abs(os_[k, 6])), "flagged": bool(f)}
                           for k, sv, f in zip(out[:16], sens[:16], fl[:16])],
            "flag": "oracle or_albajar_sensitivity over the ray's stage points with inputs moved by "
                    "2^-45 relative exceeds half the bar: tau not determined to 1e-10 by a double-"
                    "precision restatement (a harmonic's threshold, alpha ~ sqrt(r^2 - 1))"}
    if warm:
        # a-priori conditioning flag: how far each sampled ray's tau
        # moves when every RK4 stage point's warm-alpha inputs move by 2^-45 relative
        # (oracle or_warm_sensitivity, untimed, from the trajectory alone --
        # independent of the GPU's answer); flagged when that exceeds half the bar
        bar = {2: 1e-8, 3: 1e-9}[model]
        t0 = time.perf_counter()
        sens = OP.warm_sensitivity(xp[idx], Np[idx], omega, args.mode, args.ds, r["steps"],
                                   iwarm=1 if model == 2 else 3, eta=WARM_FLAG_ETA,
                                   n_threads=threads)
        t_sens = time.perf_counter() - t0
        rel_sens = sens / np.maximum(np.abs(os_[:, 6]), 1e-6)
        flagged = rel_sens > 0.5 * bar
        ok = ~flagged
        e_all = np.maximum(np.maximum(ex, eN), et)
        parity["conditioning"] = {
            "flag": "tau sensitivity to 2^-45 relative (128-ulp; at least the GPU Weideman "
                    "Faddeeva's own 2.5e-14) perturbations of every stage point's alpha inputs "
                    "(Y up / down, X N_par Te jointly) > bar / 2 (relative, tau floor 1e-6); "
                    "oracle or_warm_sensitivity, a-priori",
            "eta": WARM_FLAG_ETA,
            "rays_flagged": int(flagged.sum()),
            "rays_unflagged": int(ok.sum()),
            "rays_within_bar_unflagged": int((e_all[ok] <= bar).sum()),
            "max_rel_tau_unflagged": float(et[ok].max()) if ok.any() else None,
            "p99_rel_tau_unflagged": float(np.quantile(et[ok], 0.99)) if ok.any() else None,
            "rays_out_of_bar_flagged": int((e_all[flagged] > bar).sum()),
            # the headline figure: every sampled ray, flagged or not
            "rays_within_bar_all": int((e_all <= bar).sum()),
            "rays_sampled": int(len(idx)),
            "seconds": t_sens,
            "flagged_fan_indices": [int(i) for i in idx[flagged][:64]],
        }
        parity["note"] = ("warm model: flagged rays have an optical depth that no double-"
                          "precision restatement determines to the bar (cold-edge harmonic "
                          "crossings: fsup's recurrence cancels, and warmdisp's root selector "
                          "is decided at the 1e-11 level, one ulp of Y picking the other root; "
                          "50-digit evidence in profiles/r03/c5_conditioning_evidence.json)")
    return parity


def parity_sample(eq, xp, Np, w, omega, args, grid, gpu_out, n_rays):
    """The oracle on n_rays rays evenly spaced over this beam (untimed): the
    N >= 2 lines' parity object, as the N = 1 line's cpu_baseline sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from torj_hip import synthetic as S

    OP = O.OraclePlasma(*S.plasma_args(eq))
    O.abs_al_init(24)
    threads = O.default_threads()
    idx = np.linspace(0, len(w) - 1, num=min(n_rays, len(w)), dtype=int)
    r = OP.trace(xp[idx], Np[idx], omega, args.mode, args.ds, args.n_steps, weights=w[idx],
                 psi_grid=grid, absorption=ABSORPTION[args.absorption], n_threads=threads)
    return _parity(OP, r, idx, xp, Np, omega, args, gpu_out, threads)


def cpu_baseline(eq, xp, Np, w, omega, args, grid, gpu_out, exact_out=None):
    """The CPU oracle (C restatement, OpenMP on every host core) on a bounded
    sample of the same rays, warm models included (oracle/torj_warm_oracle.c).
    Returns (cpu_baseline, parity): when the sample runs the full n_steps, parity
    compares its endpoints with the timed launches' GPU outputs for the same rays
    (status / steps exact, max relative error of x, N, tau; bar 1e-10, warm models
    the tests' 1e-8 / 1e-9 on tau, tests/test_gpu_warm.py); with exact_out (the
    TORJ_TINY_ALPHA=0 leg's outputs) parity["exact"] holds the same comparison
    for that leg against the same oracle run."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from torj_hip import synthetic as S

    OP = O.OraclePlasma(*S.plasma_args(eq))
    O.abs_al_init(24)
    model = ABSORPTION[args.absorption]
    warm = model >= 2
    threads = O.default_threads()
    kw = dict(psi_grid=grid, absorption=model, n_threads=threads)
    # calibration sample: one ray per thread over the full path
    idx = np.linspace(0, len(w) - 1, num=threads, dtype=int)
    t0 = time.perf_counter()
    OP.trace(xp[idx], Np[idx], omega, args.mode, args.ds, args.n_steps, weights=w[idx], **kw)
    t_cal = time.perf_counter() - t0
    scale = max(1.0, args.cpu_seconds / max(t_cal, 1e-3))
    n_steps = args.n_steps
    n_rays = int(max(threads, min(len(w), threads * round(scale))))
    idx = np.linspace(0, len(w) - 1, num=n_rays, dtype=int)
    t0 = time.perf_counter()
    r = OP.trace(xp[idx], Np[idx], omega, args.mode, args.ds, n_steps, weights=w[idx], **kw)
    dt = time.perf_counter() - t0
    steps = int(r["steps"].sum())
    parity = None
    if n_steps == args.n_steps and args.integrator == "rk4":
        parity = _parity(OP, r, idx, xp, Np, omega, args, gpu_out, threads)
        if exact_out is not None:
            parity["exact"] = _parity(OP, r, idx, xp, Np, omega, args, exact_out, threads)
    what =("oracle/torj_oracle.c RK4 + oracle/torj_warm_oracle.c warm alpha, OpenMP" if warm
            else "oracle/torj_oracle.c OpenMP")
    return {"value": steps / dt, "unit": "ray-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n_rays} rays (evenly spaced over the same fan) x {n_steps} RK4 steps, "
                      f"{what}, {steps} ray-steps in {dt:.1f} s (ray stepping "
                      f"+ binned deposition; the reference profile's FITPACK post-processing is "
                      f"not included on the CPU side)"}, parity


if __name__ == "__main__":
    main()
