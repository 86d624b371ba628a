"""The multi-process make_beam path with the HIP library in every rank: two
processes (world size 2, gloo -- RCCL refuses two ranks on one device, and the
boxes here have one GPU) each trace their ray shard through libtorj_hip on
device 0 and reduce the deposition vector with torj_hip.parallel's
all_reduce, as bench.py's torchrun path does (src/solve.jl:219-240).  Against
the one-process trace of the whole beam: per-ray outputs bit-identical, the
reduced dP_shell to rounding.  And bench.py itself under torch.distributed.run
(TORJ_BENCH_SAME_DEVICE=1): one JSON line with the multi_gpu block and rank 0's
parity sample within its bar."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _beam(T):
    from torj_hip import synthetic as S

    eq = S.circular_tokamak()
    P = T.Plasma(*S.plasma_args(eq), device=0)
    T.abs_Al_init(24)
    s = S.SETUP
    f = s["f_abs_test"]
    om = 2 * np.pi * f
    N0 = T.pol_tor_angles_2_vector(s["steering_angle_pol"], s["steering_angle_tor"])
    pos, dirs, w = T.launch_peripheral_rays([s["R0"], 0.0, s["z0"]], N0, s["spot_size"],
                                            s["inverse_curvature_radius"], f, N_rings=10,
                                            min_azimuthal_points=5)
    xp, Np, s0, st = T.ray_entry(P, pos, dirs, om, 1, gpu=True)
    return P, pos, xp, Np, s0, w, om


KW = dict(ds=1e-4, n_steps=1500, traj_stride=100, deposition="reference")


def _worker(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
    import torch
    import torj_hip as T
    from torj_hip.parallel import allreduce_deposition, shard_slice

    P, pos, xp, Np, s0, w, om = _beam(T)
    sl = shard_slice(len(w), rank, world)
    grid = np.linspace(0, 1, 400)
    g = T.trace(P, xp[sl], Np[sl], om, 1, psi_grid=grid, weights=w[sl], x_launch=pos[sl], s0=s0[sl], **KW)
    vec = torch.from_numpy(g.dP_shell.copy())
    allreduce_deposition(vec)
    np.savez(out + f".{rank}.npz", state=g.state, status=g.status, steps=g.steps, P_dep=g.P_dep,
             traj=g.traj, dP=vec.numpy(), lo=sl.start, hi=sl.stop)
    dist.barrier()
    dist.destroy_process_group()


def test_two_processes_hip_shards_and_reduce(gpu, T, tmp_path):
    import torch.multiprocessing as mp

    out = str(tmp_path / "rank")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    P, pos, xp, Np, s0, w, om = _beam(T)
    grid = np.linspace(0, 1, 400)
    ref = T.trace(P, xp, Np, om, 1, psi_grid=grid, weights=w, x_launch=pos, s0=s0, **KW)
    parts = [np.load(out + f".{r}.npz") for r in range(2)]
    assert parts[0]["hi"] == parts[1]["lo"] and parts[1]["hi"] == len(w)
    for p in parts:
        sl = slice(int(p["lo"]), int(p["hi"]))
        for f in ("state", "status", "steps", "P_dep"):
            assert np.array_equal(p[f], getattr(ref, f)[sl]), f
        assert np.array_equal(p["traj"], ref.traj[sl], equal_nan=True)
    dP = parts[0]["dP"]
    assert np.array_equal(dP, parts[1]["dP"])  # every rank holds the reduced vector
    assert np.abs(dP - ref.dP_shell).max() <= 1e-13 * np.abs(ref.dP_shell).max()


def test_bench_torchrun_two_ranks_same_device(gpu):
    env = dict(os.environ, TORJ_BENCH_SAME_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--n-rings", "20", "--parity-rays", "32"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    mg = d["multi_gpu"]
    assert len(mg["trace_ms_per_device"]) == 2 and min(mg["rays_per_device"]) > 0
    p = d["parity"]
    assert p["shard"] == "rank 0" and p["rays_within_bar"] == p["rays"], p
