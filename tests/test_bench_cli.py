"""bench.py's --gpus handling on CPU (no device work happens before these
checks): too few visible devices, a WORLD_SIZE that disagrees with --gpus and
--gpus < 1 all exit non-zero with a message instead of measuring something else."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("TORJ_BEAM_SAME_DEVICE", None)
    env["HIP_VISIBLE_DEVICES"] = ""  # hide any device (the CPU suite may run anywhere)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_gpus_more_than_visible_fails_loudly():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible HIP devices, found 0" in r.stderr
    assert r.stdout.strip() == ""  # no bench line


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE = 2" in r.stderr


def test_gpus_below_one_rejected():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus 0" in r.stderr


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)  # definitions only (main() is behind __name__)
    return m


def _line(n_gpus, **extra):
    out = {k: None for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step",
                             "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                             "roofline")}
    out["n_gpus"] = n_gpus
    out.update(extra)
    return out


def test_multi_gpu_line_schema():
    """The N >= 2 line (both launch paths): every device's trace / deposition /
    call milliseconds, rays and ray-steps, the spread, and the RCCL all-reduce;
    check_line refuses a line without them, or with a per-device list of the
    wrong length."""
    import pytest

    B = _bench_module()
    per = {"trace_ms": [50.0, 52.0], "deposition_ms": [1.0, 1.1], "call_ms": [55.0, 56.0],
           "step_ms": [56.0, 56.0], "rays": [100203, 100203], "ray_steps": [200406000, 200406000],
           "rccl_allreduce_ms": [0.05, 0.06], "device": [0, 1], "rccl_nranks": [2, 2],
           "rccl_rank": [0, 1]}
    mg = B.multi_gpu_block(per, path="test")
    # the reduce's participants pass through: each replica's device and its RCCL
    # communicator's rank count / rank (torj_beam_comm_info)
    assert mg["device"] == [0, 1] and mg["rccl_nranks"] == [2, 2] and mg["rccl_rank"] == [0, 1]
    assert set(B.MULTI_GPU_KEYS) <= set(mg)
    assert mg["trace_ms_max"] == 52.0 and mg["trace_ms_min"] == 50.0
    assert abs(mg["imbalance"] - 0.04) < 1e-12 and mg["rccl_allreduce_ms"] == 0.06
    B.check_line(_line(2, multi_gpu=mg))
    B.check_line(_line(1))  # N = 1 needs no multi_gpu block
    with pytest.raises(KeyError):
        B.check_line(_line(2))
    with pytest.raises(ValueError):
        B.check_line(_line(3, multi_gpu=mg))
    # torchrun's form: the process group's ranks instead of a library communicator
    tr = B.multi_gpu_block(dict(per, pg_rank=[0, 1], pg_size=[2, 2], backend="nccl"), path="t")
    for k in ("rccl_nranks", "rccl_rank"):
        tr.pop(k)
    B.check_line(_line(2, multi_gpu=tr))
    anon = dict(mg)
    for k in ("rccl_nranks", "rccl_rank"):
        anon.pop(k)
    with pytest.raises(KeyError):  # no participants named
        B.check_line(_line(2, multi_gpu=anon))
    bad = _line(2, multi_gpu=mg)
    del bad["roofline"]
    with pytest.raises(KeyError):
        B.check_line(bad)


def test_tiny_alpha_and_resolvable_tau_statistic(monkeypatch):
    """config.tiny_alpha follows TORJ_TINY_ALPHA (default 1e-20), and the parity
    object's unfloored tau statistic covers exactly the sampled rays with
    tau_cpu >= 1e-12 (a tiny-tau ray with a large relative error does not count,
    a resolvable one does)."""
    import numpy as np

    B = _bench_module()
    monkeypatch.delenv("TORJ_TINY_ALPHA", raising=False)
    assert B.tiny_alpha() == 1e-20 == B.TINY_ALPHA_DEFAULT
    monkeypatch.setenv("TORJ_TINY_ALPHA", "0")
    assert B.tiny_alpha() == 0.0

    class Args:
        absorption, mode, ds = "albajar", 1, 1e-4

    n = 4
    st = np.zeros((n, 7))
    st[:, :3], st[:, 3:6] = [2.0, 0.1, 0.3], [0.5, 0.6, 0.1]
    st[:, 6] = [1e-126, 3e-13, 2e-12, 0.5]
    gpu = st.copy()
    gpu[0, 6] = 0.0              # below any resolution: relative error 1, not counted
    gpu[2, 6] *= 1 + 4e-11       # resolvable: counted
    gpu[3, 6] *= 1 + 1e-12
    r = {"state": st, "status": np.zeros(n, np.int32), "steps": np.full(n, 2000, np.int32)}
    p = B._parity(None, r, np.arange(n), None, None, 0.0, Args,
                  (gpu, np.zeros(n, np.int32), np.full(n, 2000, np.int32)), 1)
    assert p["rays_tau_resolvable"] == 2 and p["tau_resolvable"] == 1e-12
    assert abs(p["max_rel_tau_resolvable"] - 4e-11) < 1e-15
    assert p["max_rel_tau_unfloored"] == 1.0
    assert p["rays_within_bar"] == n  # the floored bar holds for all four
    c = p["tau_resolvable_conditioning"]
    assert c["rays_out_of_bar"] == 0 and c["max_rel_tau_resolvable_excl_flagged"] == p["max_rel_tau_resolvable"]

    # a resolvable ray outside the bar unfloored: the oracle's a-priori
    # sensitivity decides whether it is flagged (beyond half the bar) and left
    # out of the excl_flagged statistic
    class OP:
        def __init__(self, sens):
            self.sens = sens

        def albajar_sensitivity(self, x0, N0, omega, mode, ds, steps, n_threads=None):
            assert len(x0) == len(steps) == 1
            return np.array([self.sens])

    gpu[2, 6] = st[2, 6] * (1 + 6e-10)
    xp = np.zeros((n, 3))
    for sens, flagged in ((1e-19, True), (1e-23, False)):
        p = B._parity(OP(sens), r, np.arange(n), xp, xp, 0.0, Args,
                      (gpu, np.zeros(n, np.int32), np.full(n, 2000, np.int32)), 1)
        c = p["tau_resolvable_conditioning"]
        assert c["rays_out_of_bar"] == 1 and c["rays_out_of_bar_flagged"] == int(flagged)
        assert c["out_of_bar"][0]["fan_index"] == 2
        want = 1e-12 if flagged else 6e-10
        assert abs(c["max_rel_tau_resolvable_excl_flagged"] - want) < 0.1 * want


def test_traffic_profile_match_ignores_placement_switches(monkeypatch):
    """measured_traffic pairs a run with a committed profile of the same build,
    workload and kernel switches; the placement-only switches of the same-device
    rehearsals (TORJ_BEAM_SAME_DEVICE, TORJ_BENCH_SAME_DEVICE) do not enter the
    match, any kernel switch does (CPU: the profile files only)."""
    import glob
    import importlib.util
    import json

    f = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")))[-1]
    wl = json.load(open(f))["workload"]
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)

    class A:
        n_steps, n_psi, traj_stride, absorption = wl["rk4_steps"], wl["n_psi"], wl["traj_stride"], "albajar"

    for k in list(os.environ):
        if k.startswith("TORJ_"):
            monkeypatch.delenv(k)
    for k, v in wl.get("torj_env", {}).items():
        monkeypatch.setenv(k, v)
    t = B.measured_traffic(B.SPLIT_KERNELS, wl["rays"], A, wl["build_id"])
    assert t is not None and t["traffic_bytes"] > 0
    monkeypatch.setenv("TORJ_BEAM_SAME_DEVICE", "1")
    monkeypatch.setenv("TORJ_BENCH_SAME_DEVICE", "1")
    assert B.measured_traffic(B.SPLIT_KERNELS, wl["rays"], A, wl["build_id"]) is not None
    monkeypatch.setenv("TORJ_ALPHA_ZFLAG", "0")  # a kernel switch: no match
    assert B.measured_traffic(B.SPLIT_KERNELS, wl["rays"], A, wl["build_id"]) is None
    assert B.measured_traffic(B.SPLIT_KERNELS, wl["rays"], A, "0" * 16) is None
