"""World-size-2 gloo rehearsal of the multi-GPU z-slab partition (CPU only).

Drives the partition code bench.py runs over RCCL (ptv_interpolation_amd/zslab.py): each
rank generates its own sphere-pack copy, ``replicate_columns`` all-gathers the replicated
particle set, ``rank_slab`` gives its planes of the ONE stacked grid, ``interp_slab`` runs the
culled interpolation with a deliberately small first halo (so the InexactError -> proven-halo
retry path runs), and ``gather_field`` reassembles the field.  The per-rank call is the oracle
restatement of the library's cull + exactness proof (oracle.cpu_ref.slab_cull_interp), since
the HIP library needs a GPU; the GPU side of the same proof is tests/test_gpu_zslab.py.

The stitched field must equal a single-process interpolation of the whole grid from all the
particles, bit for bit: the culled slab decomposition is exact.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = 8
SIZES = {"weak": (24, 3000), "strong": (48, 12000)}  # (G, particles per copy / in all)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib, synth, zslab

    G, N = SIZES[mode]
    if mode == "weak":  # bench.py headline: copy r per rank, replicated by all-gather
        P, Q = synth.sphere_pack(N, G, values="normal", z_tiles=world, z_tile=rank)
        cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])) for i in range(3)] + \
               [torch.from_numpy(np.ascontiguousarray(Q[:, i])) for i in range(3)]
        cols = zslab.replicate_columns(cols, dist)
        nz = G * world
        z0, z1 = rank * G, (rank + 1) * G
    else:  # strong: rank 0's set broadcast, the grid cut into even slabs
        cols = [torch.empty(N, dtype=torch.float64) for _ in range(6)]
        if rank == 0:
            P, Q = synth.sphere_pack(N, G, values="normal")
            for i in range(3):
                cols[i].copy_(torch.from_numpy(P[:, i]))
                cols[3 + i].copy_(torch.from_numpy(Q[:, i]))
        zslab.broadcast_columns(cols, dist)
        nz = G
        z0, z1 = zslab.rank_slab(nz, world, rank)
    Pr = torch.stack(cols[:3], 1).numpy()
    Qr = torch.stack(cols[3:], 1).numpy()
    ax = np.linspace(0, G - 1, G)
    az = np.linspace(0, nz - 1, nz)
    kept = {}

    def call(h):
        U, V, W, req, nk = cpu_ref.slab_cull_interp(Pr, Qr, ax, ax, az, z0, z1, "idw", K, 2.0, halo=h)
        if U is None:
            raise _lib.InexactError(_lib.PTV_E_INEXACT, "halo too small", req)
        kept.update(U=U, V=V, W=W, n=nk)
        return {"halo_required": req}

    state = zslab.HaloState(0.5)
    zslab.interp_slab(call, state)
    slab = torch.from_numpy(np.stack([kept["U"], kept["V"], kept["W"]], 1))  # (planes, 3, ny, nx)
    full = zslab.gather_field(slab, dist)
    info = torch.tensor([state.retries, kept["n"], len(Pr)], dtype=torch.float64)
    infos = [torch.empty_like(info) for _ in range(world)]
    dist.all_gather(infos, info)
    if rank == 0:
        q.put((full.numpy(), Pr, Qr, [i.numpy() for i in infos]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_zslab_partition_is_exact(mode):
    from oracle import cpu_ref

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    full, P, Q, infos = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nz = full.shape[0]
    G = SIZES[mode][0]
    ax = np.linspace(0, G - 1, G)
    az = np.linspace(0, nz - 1, nz)
    U, V, W = cpu_ref.interp_grid(P, Q, ax, ax, az, "idw", K, 2.0)
    assert np.array_equal(full[:, 0], U) and np.array_equal(full[:, 1], V) and np.array_equal(full[:, 2], W)
    for retries, n_kept, n_all in infos:
        assert retries >= 1            # the 0.5 first halo was refused and widened
        assert n_kept < n_all          # and the cull still dropped particles
