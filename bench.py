#!/usr/bin/env python3
"""Headline benchmark: k-NN IDW of 5M sphere-pack particles onto a 512^3 grid (fp64).

Metric (BASELINE.json): Mvoxels/s interpolated + achieved HBM GB/s, 512^3 grid /
5M particles IDW.  One *step* = one full pass of the hot path with every input
already resident in HBM: bounding box + particle binning + coarse-lattice bounds +
the k-NN IDW kernel writing U, V, W (the reference rebuilds its KDTree on every
call, interpolator.py:132, so the binning is inside the step).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Multi-GPU (weak scaling): rank r owns z-slab copy r of a stack of
sphere packs along z (grid 512 x 512 x 512N, 5M particles per copy); it bins its
own copy plus the particles of the neighbouring copies within `--halo` voxels of
its slab and interpolates its 512^3 slab.  No collective touches the data path;
the barrier + max-over-ranks timing uses torch.distributed (RCCL).
`value` = all voxels of all ranks / max rank time.

Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic bytes of the k-NN
kernel, V*(6k+3)*8 (SURVEY.md §8(d) gather model), / its hipEvent-timed average
duration.  `roofline.traffic` is read from profiles/traffic_*.json (rocprofv3
FETCH_SIZE/WRITE_SIZE passes, tools/collect_traffic.sh) when present.
`cpu_baseline` times the oracle restatement of interpolator.py:126-155
(scipy KDTree + numpy) over z-slabs on a ProcessPoolExecutor — the
interpolator.py:173-182 / test_parallel.py multiprocess pattern — on a bounded
sample of the same workload.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mvoxels/s interpolated + achieved HBM GB/s, 512³ grid / 5M particles IDW"
METRIC_DIV = "Mvoxels/s + achieved HBM GB/s, consistent divergence (physics.py:6-53) of a 512³ field"
METRIC_FILTER = "Mparticles/s filtered + achieved HBM GB/s, k-NN median/MAD outlier filter (filtering.py:5-58), 5M particles"
METRIC_MASK = ("Mvoxels/s + achieved HBM GB/s, pore-mask path (sample_mask_on_grid + extract_boundary_particles, "
               "interpolator.py:205-284), 512³ mask")
METRIC_RBF = "Mvoxels/s interpolated + achieved FP64 TFLOP/s, 512³ grid / 5M particles local RBF"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec (AMD); not listed in the guide


def rbf_resolved(args):
    """(kernel, epsilon, degree, m) with scipy's defaults (_rbfinterp.py:300-313)."""
    from math import comb

    from ptv_interpolation_amd import rbf

    kern = args.rbf_kernel
    eps = args.epsilon if args.epsilon is not None else 1.0
    deg = args.degree if args.degree is not None else max(rbf.NAME_TO_MIN_DEGREE.get(kern, -1), 0)
    m = args.k + (comb(deg + 3, 3) if deg >= 0 else 0)
    return kern, eps, deg, m


def rbf_flops_per_voxel(k, m):
    """distances 8 k(k-1)/2, LU (2/3) m^3, substitution + build 6 m^2, eval 8k + 6m."""
    return 8 * k * (k - 1) / 2 + (2.0 / 3.0) * m ** 3 + 6 * m ** 2 + 8 * k + 6 * m


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--grid", type=int, default=512)
    ap.add_argument("--particles", type=int, default=5_000_000)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--power", type=float, default=2.0)
    ap.add_argument("--method", default="idw", choices=["idw", "sibson", "nearest", "rbf", "div", "filter", "mask"])
    ap.add_argument("--div-dtype", default="f64", choices=["f64", "f32"],
                    help="--method div: field dtype (f32 = the C5 fp32 field, Python-float spacings)")
    ap.add_argument("--rbf-kernel", default="thin_plate_spline", help="--method rbf: scipy kernel name")
    ap.add_argument("--epsilon", type=float, default=None, help="--method rbf: shape parameter")
    ap.add_argument("--degree", type=int, default=None, help="--method rbf: polynomial degree")
    ap.add_argument("--out-dtype", default="f64", choices=["f64", "f32"],
                    help="k-NN methods: U, V, W stored as float32 (PTV_FLAG_OUT_F32, the fused main.py:230 "
                         "astype; arithmetic stays f64) — the C5 configuration's field")
    ap.add_argument("--mask", action="store_true",
                    help="k-NN methods: sphere-pack fluid mask + NaN fill fused (main.py:195-207; the C4 masked "
                         "geometry): solid voxels are skipped and written as 0")
    ap.add_argument("--r0-scale", type=float, default=0.0, help="dev: first search radius / expected k-NN radius")
    ap.add_argument("--halo", type=int, default=64, help="neighbour-copy halo (voxels) for N>1")
    ap.add_argument("--cpu-sample-planes", type=int, default=16)
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--allgather", action="store_true", help="also time an RCCL all-gather of U,V,W (reported apart)")
    return ap.parse_args()


def rank_particles(args, rank, world, values="reference"):
    """Particles of pack copy `rank` plus halo particles of copies rank+-1 (weak scaling)."""
    from ptv_interpolation_amd import synth

    G = args.grid
    P, Q = synth.sphere_pack(args.particles, G, values=values, z_tiles=world, z_tile=rank)
    if world == 1:
        return P, Q
    parts, vals = [P], [Q]
    z_lo, z_hi = rank * G, (rank + 1) * G
    for nb in (rank - 1, rank + 1):
        if 0 <= nb < world:
            Pn, Qn = synth.sphere_pack(args.particles, G, values=values, z_tiles=world, z_tile=nb)
            keep = (Pn[:, 2] >= z_lo - args.halo) & (Pn[:, 2] < z_hi + args.halo)
            parts.append(Pn[keep])
            vals.append(Qn[keep])
    return np.concatenate(parts), np.concatenate(vals)


def row_traffic(*keys):
    """Sum of HBM bytes per launch of the named row kernels (profiles/traffic_rows_*.json,
    tools/traffic_rows.py), or None when any is missing."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_rows_*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            t = json.load(f)
        return float(sum(t[k]["hbm_bytes"] for k in keys))
    except Exception:
        return None


def traffic_from_profiles(kernel_substr="k_knn_interp<"):
    """HBM bytes per k-NN launch from the newest profiles/traffic_*.json (or None)."""
    import re

    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json"))
                   if re.fullmatch(r"traffic_r\d+\.json", os.path.basename(f)))  # not traffic_rows_*
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            t = json.load(f)
        return float(t["hbm_bytes_per_launch"])
    except Exception:
        return None


def cpu_baseline(args, P, Q, ax):
    """Oracle restatement on a bounded z-slab sample, multiprocess (test_parallel.py pattern)."""
    from oracle import cpu_ref

    planes = min(args.cpu_sample_planes, len(ax))
    z0 = len(ax) // 2 - planes // 2
    workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
    t = time.perf_counter()
    cpu_ref.interp_grid_parallel(P, Q, ax, ax, ax, args.method, args.k, args.power,
                                 z0=z0, z1=z0 + planes, n_jobs=workers, slab=max(1, planes // workers))
    dt = time.perf_counter() - t
    nvox = planes * len(ax) * len(ax)
    return {"value": round(nvox / dt / 1e6, 4), "unit": "Mvoxels/s", "cores": workers, "kind": "port",
            "sample": f"{planes} central z-planes ({nvox} voxels) of the same {args.grid}^3/"
                      f"{args.particles} workload; scipy KDTree + numpy (oracle/cpu_ref.py), "
                      f"{workers} processes, each building its own tree (interpolator.py:173-182 pattern)",
            "seconds": round(dt, 2)}


def _rbf_cpu_worker(a):
    from oracle import cpu_ref

    P, Q, q, k, kern, eps, deg = a
    return cpu_ref.rbf_local_points(P, Q, q, k, kern, eps, deg)


def cpu_baseline_rbf(args, P, Q, ax):
    """Oracle local RBF (KDTree + per-voxel LAPACK gesv) on a bounded voxel sample, split over a
    ProcessPoolExecutor like interpolator.py:173-182 (each worker builds its own tree)."""
    from concurrent.futures import ProcessPoolExecutor

    kern, eps, deg, _ = rbf_resolved(args)
    workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
    nvox = 2048 * workers
    G = len(ax)
    rng = np.random.default_rng(0)
    sel = rng.integers(0, G ** 3, nvox)
    iz, iy, ix = np.unravel_index(sel, (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], -1)
    t = time.perf_counter()
    with ProcessPoolExecutor(max_workers=workers) as ex:
        list(ex.map(_rbf_cpu_worker, [(P, Q, c, args.k, kern, eps, deg) for c in np.array_split(q, workers)]))
    dt = time.perf_counter() - t
    return {"value": round(nvox / dt / 1e6, 6), "unit": "Mvoxels/s", "cores": workers, "kind": "port",
            "sample": f"{nvox} random voxels of the same {G}^3/{args.particles} workload; scipy KDTree + numpy "
                      f"LAPACK gesv per voxel (oracle/cpu_ref.rbf_local_points), {workers} processes, each "
                      f"building its own tree (interpolator.py:173-182 pattern)",
            "seconds": round(dt, 2)}


def cpu_baseline_div(args, fields, fluid):
    """Oracle divergence (numpy, one process — the reference's physics.py is single-threaded
    numpy) on a bounded z-slab sample of the same field."""
    from oracle import cpu_ref

    G = args.grid
    planes = min(64, G)
    sl = slice(G // 2 - planes // 2, G // 2 - planes // 2 + planes)
    u, v, w = (f[sl] for f in fields)
    t = time.perf_counter()
    cpu_ref.consistent_divergence(u, v, w, fluid[sl], 1.0, 1.0, 1.0)
    dt = time.perf_counter() - t
    nvox = planes * G * G
    return {"value": round(nvox / dt / 1e6, 3), "unit": "Mvoxels/s", "cores": 1, "kind": "port",
            "sample": f"{planes} central z-planes ({nvox} voxels) of the same {G}^3 field; numpy restatement "
                      f"of physics.compute_consistent_divergence (oracle/cpu_ref.py), 1 process",
            "seconds": round(dt, 2)}


def main_div(args):
    """--method div: one step = the consistent divergence of a resident (G, G, G) velocity field
    with the sphere-pack fluid mask (view_divergence.py:39).  Weak scaling: each rank owns a
    G^3 z-slab plus one halo plane per interior side (no collective on the data path)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from ptv_interpolation_amd import _lib, synth

    G = args.grid
    f32 = args.div_dtype == "f32"
    tdt = torch.float32 if f32 else torch.float64
    s = 4 if f32 else 8
    lo = 1 if rank > 0 else 0
    hi = 1 if rank < world - 1 else 0
    nzb = G + lo + hi
    fluid = synth.fluid_mask(G)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    fields = [torch.randn((nzb, G, G), generator=gen, dtype=tdt, device=dev) for _ in range(3)]
    mask_np = np.concatenate([fluid[-lo:] if lo else fluid[:0], fluid, fluid[:hi]])
    mask = torch.from_numpy(np.ascontiguousarray(mask_np).view(np.uint8)).to(dev)
    out = torch.empty((G, G, G), dtype=tdt, device=dev)
    ctx = _lib.Context(local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    dtc = _lib.F32 if f32 else _lib.F64

    def step():
        return ctx.divergence_dev(G, G, nzb, [f.data_ptr() for f in fields], mask.data_ptr(), out.data_ptr(),
                                  1.0, 1.0, 1.0, field_dtype=dtc, result_dtype=dtc, z_range=(lo, lo + G),
                                  edges=(lo == 0, hi == 0), stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    k_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        k_ms.append(ctx.last_stats()["ms_stencil"])
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    vox = G ** 3
    kavg = float(np.mean(k_ms))
    alg = vox * (3 * s + 1 + s)
    ach = alg / (kavg * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline_div(args, [f.cpu().numpy() for f in fields], fluid)
        except Exception as e:
            cpu = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        line = {
            "metric": METRIC_DIV, "value": round(vox * world / (elapsed / args.steps) / 1e6, 2),
            "unit": "Mvoxels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.div_dtype,
            "data": "synthetic: N(0,1) velocity field, generate_sphere_pack.py fluid mask at voxel centres",
            "config": {"workload": f"consistent divergence of a {G}^3 {args.div_dtype} field (z-slab per GPU)",
                       "grid": G, "method": "div", "parallelism": f"z-slab x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "traffic": row_traffic("div:k_divergence") if (G == 512 and not f32) else None,
                         "kernel": f"k_divergence<{'float' if f32 else 'double'}>",
                         "alg_bytes_per_launch": alg, "kernel_ms": round(kavg, 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def _dist_init():
    """One process per GPU (torchrun env); returns (world, rank, local, dist or None, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local, dist, torch.device("cuda", local)


def _timed(step, args, dist, dev, stat_key, ctx):
    """W warmup steps, then K steps between barriers + synchronize; (max-over-ranks seconds, kernel ms list)."""
    import torch

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    k_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        k_ms.append(ctx.last_stats()[stat_key] if stat_key else 0.0)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, k_ms


def main_filter(args):
    """--method filter: one step = remove_outliers_knn (filtering.py:5-58) over a resident particle set:
    binning + (k+1)-NN of every particle among the particles (slot mode) + median/MAD per particle.
    Weak scaling: each rank filters its own sphere-pack copy (independent particle sets)."""
    import torch

    world, rank, local, dist, dev = _dist_init()
    from ptv_interpolation_amd import _lib, synth

    k = 25 if args.k == 8 else args.k   # the reference default (main.py:44)
    P, _ = synth.sphere_pack(args.particles, args.grid)
    rng = np.random.default_rng(20260214 + rank)
    Q = rng.standard_normal((len(P), 3))
    Q[rng.choice(len(P), len(P) // 100, replace=False)] *= 8.0  # 1 % outliers
    n = len(P)
    cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).to(dev) for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).to(dev) for i in range(3)]
    keep = torch.empty(n, dtype=torch.uint8, device=dev)
    kth = torch.empty(n, dtype=torch.float64, device=dev)
    ctx = _lib.Context(local)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        return ctx.filter_outliers_knn_dev(n, [c.data_ptr() for c in cols], keep.data_ptr(), kth.data_ptr(), k=k,
                                           threshold=3.0, stream=stream)

    elapsed, k_ms = _timed(step, args, dist, dev, "ms_knn", ctx)
    st = ctx.last_stats()
    kavg = float(np.mean(k_ms))
    # gather model per particle: k+1 neighbour records {x,y,z,u,v,w} + keep byte + k-th distance
    alg = n * ((6 * (k + 1)) * 8 + 1 + 8)
    ach = alg / (kavg * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            from oracle import cpu_ref

            m = min(n, 400_000)
            t = time.perf_counter()
            cpu_ref.outlier_filter(P[:m], Q[:m], k, 3.0, workers=1)
            dt = time.perf_counter() - t
            cpu = {"value": round(m / dt / 1e6, 4), "unit": "Mparticles/s", "cores": 1, "kind": "port",
                   "sample": f"first {m} particles of the same cloud (a {m / n:.0%} subset at the same density "
                             "is not the same neighbourhoods; documented), scipy KDTree(k+1) + numpy median/MAD "
                             "(oracle/cpu_ref.outlier_filter = filtering.py:15-51), workers=1",
                   "seconds": round(dt, 2)}
        except Exception as e:
            cpu = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        print(json.dumps({
            "metric": METRIC_FILTER, "value": round(n * world / (elapsed / args.steps) / 1e6, 2),
            "unit": "Mparticles/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: generate_sphere_pack.py geometry, N(0,1) velocities with 1% x8 outliers",
            "config": {"workload": f"remove_outliers_knn k={k} threshold=3 over {n} particles", "k": k,
                       "particles": n, "method": "filter", "parallelism": f"independent particle sets x{world}"},
            "breakdown_ms": {"bin": round(st["ms_bin"], 3), "knn+stats": round(kavg, 3)},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "traffic": row_traffic("filter:k_knn_interp", "filter:k_outlier_stats")
                         if (k == 25 and n == 5_000_000) else None,
                         "kernel": f"k_knn_interp<{32 if k + 1 <= 32 else 64}> (slot mode) + k_outlier_stats",
                         "alg_bytes_per_launch": alg, "kernel_ms": round(kavg, 4)},
            "cpu_baseline": cpu}), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main_mask(args):
    """--method mask: one step = sample_mask_on_grid (a G^3 raw mask onto the G^3 grid, main.py:161
    at --downscale 1) + extract_boundary_particles(thickness=1, step=1) (main.py:168) on resident
    bytes.  Weak scaling: each rank processes its own mask copy."""
    import torch

    world, rank, local, dist, dev = _dist_init()
    from ptv_interpolation_amd import _lib, synth

    G = args.grid
    fluid = synth.fluid_mask(G)
    raw = torch.from_numpy(np.ascontiguousarray(fluid).view(np.uint8)).to(dev)
    ax_h = np.linspace(0, G - 1, G)
    axes = [torch.from_numpy(ax_h.copy()).to(dev) for _ in range(3)]
    out = torch.empty((G, G, G), dtype=torch.uint8, device=dev)
    ctx = _lib.Context(local)
    # a real (non-null) torch stream, so that the library's launches and the timing events share it
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    stream = torch.cuda.current_stream(dev).cuda_stream
    lo, span, den = [0.0] * 3, [float(G - 1)] * 3, [float(G - 1)] * 3
    nb = ctx.boundary_particles_dev(raw.data_ptr(), (G, G, G), 1, 1, lo, span, den, stream=stream)
    bxyz = torch.empty((3, max(nb, 1)), dtype=torch.float64, device=dev)
    optrs = [bxyz[i].data_ptr() for i in range(3)]
    ms = {"sample": [], "boundary": []}
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step():
        e[0].record()
        ctx.sample_mask_dev(raw.data_ptr(), (G, G, G), (ax_h, ax_h, ax_h), [a.data_ptr() for a in axes],
                            (G, G, G), out.data_ptr(), stream=stream)
        e[1].record()
        ctx.boundary_particles_dev(raw.data_ptr(), (G, G, G), 1, 1, lo, span, den, out_ptrs=optrs, cap=nb,
                                   stream=stream)
        e[2].record()

    def step_timed():
        step()
        torch.cuda.synchronize(dev)
        ms["sample"].append(e[0].elapsed_time(e[1]))
        ms["boundary"].append(e[1].elapsed_time(e[2]))

    elapsed, _ = _timed(step_timed, args, dist, dev, None, ctx)
    V = G ** 3
    t_s, t_b = float(np.mean(ms["sample"][args.warmup:] or ms["sample"])), float(np.mean(ms["boundary"][args.warmup:] or ms["boundary"]))
    alg_s = 2 * V            # read the raw byte, write the grid byte (same resolution)
    alg_b = V + 24 * nb      # read the mask once, write 3 doubles per boundary particle
    ach_s = alg_s / (t_s * 1e-3) / 1e9
    ach_b = alg_b / (t_b * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            from oracle import cpu_ref

            Gs = min(G, 256)
            f = synth.fluid_mask(Gs)
            (X, Y, Z) = np.meshgrid(np.linspace(0, Gs - 1, Gs), np.linspace(0, Gs - 1, Gs),
                                    np.linspace(0, Gs - 1, Gs), indexing="ij")[::-1]
            t = time.perf_counter()
            cpu_ref.sample_mask_nearest(f, ((0, Gs),) * 3, X, Y, Z)
            cpu_ref.boundary_particles(f, ((0, Gs),) * 3, 1, 1)
            dt = time.perf_counter() - t
            cpu = {"value": round(Gs ** 3 / dt / 1e6, 3), "unit": "Mvoxels/s", "cores": 1, "kind": "port",
                   "sample": f"{Gs}^3 sphere-pack mask, numpy restatement (oracle/cpu_ref.sample_mask_nearest + "
                             "boundary_particles of interpolator.py:205-284), 1 process",
                   "seconds": round(dt, 2)}
        except Exception as ex:
            cpu = {"value": None, "error": repr(ex)[:200]}
    if rank == 0:
        print(json.dumps({
            "metric": METRIC_MASK, "value": round(V * world / (elapsed / args.steps) / 1e6, 2),
            "unit": "Mvoxels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: generate_sphere_pack.py fluid mask at voxel centres",
            "config": {"workload": f"sample_mask_on_grid {G}^3 -> {G}^3 + extract_boundary_particles "
                                   f"(thickness 1, step 1, {nb} particles)", "grid": G, "method": "mask",
                       "parallelism": f"independent masks x{world}"},
            "breakdown_ms": {"sample": round(t_s, 4), "boundary": round(t_b, 4)},
            "roofline": {"bound": "hbm", "achieved": round(ach_b, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach_b / HBM_PEAK_GBPS, 4),
                         "traffic": row_traffic("mask:k_boundary_count16", "mask:k_boundary_emit16")
                         if G == 512 else None,
                         "kernel": "extract_boundary_particles (k_boundary_count + scan + k_boundary_emit)",
                         "alg_bytes_per_launch": alg_b, "kernel_ms": round(t_b, 4),
                         "sample_mask": {"achieved": round(ach_s, 1), "frac": round(ach_s / HBM_PEAK_GBPS, 4),
                                         "alg_bytes": alg_s, "kernel_ms": round(t_s, 4)}},
            "cpu_baseline": cpu}), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.method == "div":
        return main_div(args)
    if args.method == "filter":
        return main_filter(args)
    if args.method == "mask":
        return main_mask(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from ptv_interpolation_amd import _lib

    G = args.grid
    P, Q = rank_particles(args, rank, world)
    n = P.shape[0]
    ax_h = np.linspace(0, G - 1, G)
    az_h = ax_h + rank * G
    cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).to(dev) for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).to(dev) for i in range(3)]
    axes = [torch.from_numpy(ax_h).to(dev), torch.from_numpy(ax_h.copy()).to(dev), torch.from_numpy(az_h).to(dev)]
    out_f32 = args.out_dtype == "f32" and args.method != "rbf"
    mask_t = None
    if args.mask:
        from ptv_interpolation_amd import synth as _synth

        fm = _synth.fluid_mask(G)
        fluid_frac = float(fm.mean())
        mask_t = torch.from_numpy(np.ascontiguousarray(fm).view(np.uint8)).to(dev)
        del fm
    out = [torch.empty((G, G, G), dtype=torch.float32 if out_f32 else torch.float64, device=dev) for _ in range(3)]
    ctx = _lib.Context(local)
    method = {"idw": _lib.METHOD_IDW, "sibson": _lib.METHOD_SIBSON, "nearest": _lib.METHOD_NEAREST}.get(args.method)
    if args.method == "nearest":
        args.k = 1
    stream = torch.cuda.current_stream(dev).cuda_stream

    if args.method == "rbf":
        kern, eps, deg, m_sys = rbf_resolved(args)

        def step():
            return ctx.interp_rbf_dev(n, [c.data_ptr() for c in cols], G, G, G,
                                      axes_ptrs=[a.data_ptr() for a in axes],
                                      out_ptrs=[o.data_ptr() for o in out], k=args.k, kernel=kern, epsilon=eps,
                                      degree=deg, stream=stream)
    else:
        def step():
            return ctx.interp_knn_dev(n, [c.data_ptr() for c in cols], G, G, G,
                                      axes_ptrs=[a.data_ptr() for a in axes],
                                      out_ptrs=[o.data_ptr() for o in out], method=method, k=args.k,
                                      power=args.power, stream=stream,
                                      mask_ptr=mask_t.data_ptr() if mask_t is not None else 0,
                                      r0_scale=args.r0_scale,
                                      flags=(_lib.FLAG_OUT_F32 if out_f32 else 0) |
                                            (_lib.FLAG_NAN_TO_NUM if mask_t is not None else 0))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    knn_ms, lat_ms, bin_ms, solve_ms = [], [], [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = ctx.last_stats()  # synchronises on the step's events
        knn_ms.append(st["ms_knn"])
        lat_ms.append(st["ms_lattice"])
        bin_ms.append(st["ms_bin"])
        solve_ms.append(st["ms_solve"])
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    gather_ms = None
    if args.allgather and dist is not None:
        full = [torch.empty((G * world, G, G), dtype=out[0].dtype, device=dev) for _ in range(3)]
        torch.cuda.synchronize(dev)
        dist.barrier()
        tg = time.perf_counter()
        for c in range(3):
            dist.all_gather_into_tensor(full[c], out[c])
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - tg) * 1e3
        del full

    vox = G ** 3
    ms_step = elapsed / args.steps * 1e3
    value = vox * world / (elapsed / args.steps) / 1e6
    knn_avg = float(np.mean(knn_ms))
    alg_bytes = vox * ((6 * args.k) * 8 + 3 * (4 if out_f32 else 8))
    if args.mask:  # solid voxels are skipped, fluid V in the gather term; + the mask bytes
        alg_bytes = int(round(vox * fluid_frac)) * (6 * args.k) * 8 + vox * (3 * (4 if out_f32 else 8) + 1)
    achieved = alg_bytes / (knn_avg * 1e-3) / 1e9
    traffic = traffic_from_profiles()

    if args.method == "rbf":
        solve_avg = float(np.mean(solve_ms))
        flops = vox * rbf_flops_per_voxel(args.k, m_sys)
        tf = flops / (solve_avg * 1e-3) / 1e12
        roof = {"bound": "fp64", "achieved": round(tf, 2), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tf / FP64_PEAK_TFLOPS, 4), "traffic": None, "kernel": "k_rbf_local",
                "alg_flops_per_launch": flops, "kernel_ms": round(solve_avg, 3)}
    else:
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic, "kernel": f"k_knn_interp<{args.k}>",
                "alg_bytes_per_launch": alg_bytes, "kernel_ms": round(knn_avg, 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = (cpu_baseline_rbf if args.method == "rbf" else cpu_baseline)(args, P, Q, ax_h)
        except Exception as e:  # the baseline must never take the GPU line down
            cpu = {"value": None, "error": repr(e)[:200]}

    if rank == 0:
        line = {
            "metric": METRIC_RBF if args.method == "rbf" else METRIC,
            "value": round(value, 2),
            "unit": "Mvoxels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: generate_sphere_pack.py geometry scaled to voxel units, seeded, w=1 flow field",
            "config": {"workload": (f"{G}^3 grid / {args.particles} particles local RBF {kern} k={args.k} "
                                    f"eps={eps} degree={deg} (system {m_sys}) fp64 (z-slab per GPU)")
                       if args.method == "rbf" else
                       f"{G}^3 grid / {args.particles} particles {args.method.upper()} "
                       f"k={args.k} p={args.power} fp64" + (" (float32 U, V, W)" if out_f32 else "") +
                       (f" + sphere-pack fluid mask ({fluid_frac:.1%} fluid, solid skipped)" if args.mask else "") +
                       " (z-slab per GPU)",
                       "grid": G, "particles": args.particles, "particles_binned_rank0": n,
                       "method": args.method, "k": args.k, "power": args.power,
                       "parallelism": f"z-slab x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            **({"fluid_mvoxels_per_s": round(value * fluid_frac, 2)} if args.mask else {}),
            "breakdown_ms": {"bin": round(float(np.mean(bin_ms)), 3), "lattice": round(float(np.mean(lat_ms)), 3),
                             "knn": round(knn_avg, 3), "solve": round(float(np.mean(solve_ms)), 3)},
        }
        if gather_ms is not None:
            line["allgather_ms"] = round(gather_ms, 2)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
