"""world_size-2 gloo test of the multi-GPU layout (torj_hip/parallel.py, used by
bench.py): ray shards traced independently + one all_reduce of the deposition
vector reproduce the single-process beam.  The per-rank tracer here is the CPU
oracle (test infrastructure standing in for the GPU kernel, which the gpu tests
cover); what is under test is the sharding and the reduce."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _beam():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
    import oracle as O
    from torj_hip import synthetic as S

    O.abs_al_init(24)
    eq = S.circular_tokamak()
    P = O.OraclePlasma(*S.plasma_args(eq))
    om = 2 * np.pi * 92.5e9
    N0 = O.pol_tor_angles_2_vector(np.deg2rad(30), 0.0)
    pos, dirs, w = O.launch_peripheral_rays([2.5, 0, 0.4], N0, 0.0174, 1 / 3.99, 92.5e9)
    ent = [P.ray_entry(pos[i], dirs[i], om, 1) for i in range(len(w))]
    xs, Ns = np.array([e[1] for e in ent]), np.array([e[2] for e in ent])
    return P, xs, Ns, w, om


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
    from torj_hip.parallel import allreduce_deposition, shard_slice

    P, xs, Ns, w, om = _beam()
    sl = shard_slice(len(w), rank, world)
    grid = np.linspace(0, 1, 200)
    r = P.trace(xs[sl], Ns[sl], om, 1, 1e-4, 300, psi_grid=grid, weights=w[sl], n_threads=2)
    vec = torch.zeros(len(grid) + 1, dtype=torch.float64)
    vec[:-1] = torch.from_numpy(r["dP"])
    vec[-1] = float(np.sum(w[sl] * r["Pdep"]))
    allreduce_deposition(vec)
    if rank == 0:
        np.save(out, vec.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_slice_partitions():
    from torj_hip.parallel import shard_slice

    for n in (0, 1, 7, 46, 100203):
        for world in (1, 2, 3, 8):
            sl = [shard_slice(n, r, world) for r in range(world)]
            idx = np.concatenate([np.arange(n)[s] for s in sl])
            assert np.array_equal(idx, np.arange(n))
            sizes = [s.stop - s.start for s in sl]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_slice(10, 2, 2)


def test_two_rank_gloo_beam_reduce(tmp_path):
    out = str(tmp_path / "vec.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    vec = np.load(out)
    P, xs, Ns, w, om = _beam()
    grid = np.linspace(0, 1, 200)
    r = P.trace(xs, Ns, om, 1, 1e-4, 300, psi_grid=grid, weights=w, n_threads=2)
    assert np.abs(vec[:-1] - r["dP"]).max() <= 1e-14 * max(np.abs(r["dP"]).max(), 1e-300)
    assert abs(vec[-1] - np.sum(w * r["Pdep"])) < 1e-14
