"""World-size-2 gloo rehearsal of the multi-GPU z-slab path (CPU only).

Each rank builds its particle set exactly as bench.py does (own sphere-pack copy +
halo of the neighbouring copies), interpolates its z-slab with the oracle, and the
slabs are gathered over gloo.  The stitched field must equal a single-process
interpolation over the union of all copies: the slab decomposition with halos is
exact (no data-path collective is needed for the interpolation itself).
"""
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _args(G=24, N=3000, halo=12):
    return types.SimpleNamespace(grid=G, particles=N, halo=halo)


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import cpu_ref

    a = _args()
    P, Q = bench.rank_particles(a, rank, world, values="normal")
    ax = np.linspace(0, a.grid - 1, a.grid)
    az = ax + rank * a.grid
    U, V, W = cpu_ref.interp_grid(P, Q, ax, ax, az, "idw", 8, 2.0)
    slab = torch.from_numpy(np.stack([U, V, W]))
    parts = [torch.empty_like(slab) for _ in range(world)]
    dist.all_gather(parts, slab)
    if rank == 0:
        q.put(torch.cat(parts, dim=1).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_zslab_halo_decomposition_is_exact():
    from ptv_interpolation_amd import synth
    from oracle import cpu_ref

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    stitched = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = _args()
    allP, allQ = zip(*[synth.sphere_pack(a.particles, a.grid, values="normal", z_tiles=world, z_tile=t)
                       for t in range(world)])
    P = np.concatenate(allP); Q = np.concatenate(allQ)
    ax = np.linspace(0, a.grid - 1, a.grid)
    az = np.linspace(0, world * a.grid - 1, world * a.grid)
    U, V, W = cpu_ref.interp_grid(P, Q, ax, ax, az, "idw", 8, 2.0)
    assert np.array_equal(stitched[0], U) and np.array_equal(stitched[2], W)
