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
