"""Multi-GPU layout of make_beam (src/solve.jl:209-242): one process per GPU.

Rays never interact (src/solve.jl:219-221), so a beam is split into contiguous
ray shards with no collective on the data path; the only exchange is
make_beam's weighted reduce (src/solve.jl:233-240) of the shell-binned
deposited power, one all_reduce of n_psi + 1 fp64 (RCCL over xGMI when the
process group backend is "nccl", gloo in the CPU tests).
"""
from __future__ import annotations


def shard_slice(n: int, rank: int, world: int) -> slice:
    """Contiguous, balanced shard of n rays for `rank` (sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return slice(start, start + base + (1 if rank < extra else 0))


def allreduce_deposition(dP_shell, group=None):
    """Sum the per-rank (n_psi + 1) deposition vector in place (torch tensor)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(dP_shell, op=dist.ReduceOp.SUM, group=group)
    return dP_shell


def group_shard(n: int, n_shards: int, k: int) -> slice:
    """Shard k of n_shards over n rays with boundaries on 64-ray multiples (one
    wave / one work-queue group), as torj_trace_beam cuts a beam (beam_shard in
    torj_hip.hip): every shard holds whole 64-ray groups of the unsplit beam, so
    per-ray results do not depend on the split."""
    if n_shards < 1 or not (0 <= k < n_shards):
        raise ValueError(f"bad shard {k} / {n_shards}")
    G = (n + 63) // 64
    lo = min(G * k // n_shards * 64, n)
    hi = min(G * (k + 1) // n_shards * 64, n)
    return slice(lo, hi)


_SHARD_FIELDS = ("x0", "N0", "weights", "psi_grid", "x_launch", "s0", "state", "status", "steps",
                 "dP_shell", "P_dep", "traj", "counters")


def trace_beam_device(plasma, cfg, n_psi: int, shards) -> None:
    """torj_trace_beam_device: make_beam's fan-out over device-resident shards
    (src/solve.jl:209-240).  shards[k] is a dict with "n" and any of the
    torj_beam_shard fields (torch tensors on replica k's device -- (plasma
    device + k) mod count -- or raw device pointers); each shard's dP_shell ends
    as the sum over all shards (RCCL all-reduce).  Synchronous."""
    from ._lib import BeamShard, TraceCfg, check, lib  # noqa: F401
    import ctypes as C

    arr = (BeamShard * len(shards))()
    for k, sh in enumerate(shards):
        arr[k].n = int(sh["n"])
        for f in _SHARD_FIELDS:
            v = sh.get(f)
            if v is not None and not isinstance(v, int):
                v = v.data_ptr()
            setattr(arr[k], f, v)
    check(lib().torj_trace_beam_device(plasma.handle, C.byref(cfg), len(shards), int(n_psi), arr))


def beam_comm_info(plasma, n_gpus: int) -> dict:
    """torj_beam_comm_info: per replica of the last fan-out over n_gpus, the HIP
    device it ran on and its RCCL communicator's rank count and rank
    (ncclCommCount / ncclCommUserRank; 0 / -1 without a communicator: one
    replica, or the test-only same-device placement)."""
    from ._lib import check, lib
    import ctypes as C

    dev, nr, rk = (C.c_int * n_gpus)(), (C.c_int * n_gpus)(), (C.c_int * n_gpus)()
    check(lib().torj_beam_comm_info(plasma.handle, int(n_gpus), dev, nr, rk))
    return {"device": list(dev), "rccl_nranks": list(nr), "rccl_rank": list(rk)}
