#!/usr/bin/env python3
"""Benchmark of the MI355X scattered-to-grid interpolator (BASELINE.json metric and configs).

Headline (the default; BASELINE metric): k-NN IDW (k = 8, p = 2, fp64) of 5M sphere-pack
particles onto a 512^3 grid.  One *step* = one pass of the hot path with every input already
resident in HBM: bounding box + particle binning + coarse-lattice bounds + the k-NN IDW kernel
writing U, V, W (the reference rebuilds its KDTree on every call, interpolator.py:132, so the
binning is inside the step).

    python bench.py [--gpus N --steps K --warmup W] [--config headline|c2|c3|c4|c5|...]
    torchrun --nproc-per-node N bench.py --gpus N ...          (one process per GPU, RCCL)

``--gpus N`` with N > 1 and no torchrun environment starts the N ranks itself: the parent
process, which has not touched a GPU, runs ``python -m torch.distributed.run --nproc-per-node
N bench.py ...`` as a child and exits with its code; each rank checks that the world size it
was given equals ``--gpus`` and fails loudly otherwise.

Multi-GPU = the north_star partition (zslab.py): ONE grid cut into z-slabs,
rank r computing planes slab_bounds(nz, N)[r], the particle set replicated in every rank's HBM
(broadcast before the timed loop) and culled on device by a per-column map derived from the
slab's own lattice bounds, proven exact on the device before every main launch
(PTV_FLAG_SLAB_CULL_AUTO; the warmup's first call builds the map; a failed proof reruns the call
unculled, never changes a result).
No collective touches the timed step; an RCCL all-gather reassembly of the full field (slabs
padded to the largest one when they differ) is timed once after it and reported apart
(``allgather_ms``).

* headline (default): strong scaling of the named 512^3 / 5M workload: every N computes the
  same grid, rank r its 512/N planes.
* headline_weak: N stacked 512^3 sphere-pack copies along z (5M particles each, all 5M N
  replicated on every rank), rank r owns copy r's 512^3 planes.
* c2 (256^3 / 1M IDW), c3 (512^3 / 5M local Gaussian RBF 32 x 32), c4 (1024^3 / 10M IDW with
  the sphere-pack pore mask fused), c5 (2048^3 / 50M IDW, float32 field, + the consistent
  divergence of view_divergence.py over each slab with a one-plane halo interpolated
  redundantly): strong scaling of the named grid, the configs' N = 1 line being the whole grid
  on one GPU.

``--share R/N`` (one GPU, no collective) runs rank R's step of the N-rank strong partition:
the per-rank step time a rehearsal of the N-GPU run is built from (tools/share_balance.py).
``--dry-run`` (CPU, gloo) runs the launcher and the partition / broadcast / padded all-gather
with a plane-index fill in place of the kernel (tests/test_bench_launch.py).

Rank 0 prints ONE JSON line.  ``roofline.achieved`` = algorithmic bytes of the k-NN kernel
(SURVEY.md §8(d) gather model, V (6k 8 + 3 s_out) for this rank's slab) / its hipEvent-timed
average duration; ``roofline.frac_step`` divides the step's bytes (+ 48 B per binned particle)
by bin + cull + lattice + k-NN time.  ``cpu_baseline`` times the oracle restatement of
interpolator.py:126-155 (scipy KDTree + numpy) over z-slabs on a ProcessPoolExecutor — the
interpolator.py:173-182 / test_parallel.py pattern — on a bounded sample of the same workload,
with the CPU model and the calibration against the reference (profiles/cpu_calibration_*.json).
``--method div|filter|mask`` bench the rows next to the path (physics.py / filtering.py /
the pore-mask path) with their own metric lines; ``--method linear`` benches griddata(method=
'linear') (the reference default) with the host Delaunay build timed apart from the GPU step.
"""
from __future__ import annotations

import argparse
import contextlib
import glob
import io
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mvoxels/s interpolated + achieved HBM GB/s, 512³ grid / 5M particles IDW"
METRIC_C2 = "Mvoxels/s interpolated + achieved HBM GB/s, 256³ grid / 1M particles IDW"
METRIC_C2R = "Mvoxels/s interpolated + achieved HBM GB/s, 256³ grid / 1M particles IDW radius-search"
METRIC_RBF = "Mvoxels/s interpolated + achieved FP64 TFLOP/s, 512³ grid / 5M particles local RBF"
METRIC_C4 = "Mvoxels/s interpolated + achieved HBM GB/s, 1024³ grid / 10M particles masked IDW (z-slab partition)"
METRIC_C5 = ("Mvoxels/s interpolated + achieved HBM GB/s, 2048³ grid / 50M particles fp32 IDW + divergence "
             "(z-slab partition)")
METRIC_DIV = "Mvoxels/s + achieved HBM GB/s, consistent divergence (physics.py:6-53) of a 512³ field"
METRIC_FILTER = "Mparticles/s filtered + achieved HBM GB/s, k-NN median/MAD outlier filter (filtering.py:5-58), 5M particles"
METRIC_LINEAR = "Mvoxels/s interpolated + achieved HBM GB/s, griddata(method='linear') over a Delaunay triangulation"
METRIC_MASK = ("Mvoxels/s + achieved HBM GB/s, pore-mask path (sample_mask_on_grid + extract_boundary_particles, "
               "interpolator.py:205-284), 512³ mask")
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec (AMD); not listed in the guide
KMAX_EXACT = (1, 4, 8, 12)  # k_knn_interp list lengths (ptv_knn.hip kmax_for): pair lists serve k <= length,
KMAX_KEYS = (16, 24, 32, 40, 48, 56, 64, 96, 128)  # packed-key lists k + 1 <= length

# BASELINE.json configs; C1 (64^3 / 10k, CPU plumbing) is a parity test case
CONFIGS = {
    "headline": dict(grid=512, particles=5_000_000, method="idw", k=8, scaling="strong", metric=METRIC),
    "headline_weak": dict(grid=512, particles=5_000_000, method="idw", k=8, scaling="weak", metric=METRIC),
    "c2": dict(grid=256, particles=1_000_000, method="idw", k=8, scaling="strong", metric=METRIC_C2),
    # BASELINE config 2 as named ("IDW radius-search"): an extension, the reference has no radius
    # search (parity unpinned; tests/test_gpu_radius.py); r = 3 voxels ~ 6.8 particles per ball
    "c2r": dict(grid=256, particles=1_000_000, method="idw", k=8, radius=3.0, scaling="strong", metric=METRIC_C2R),
    "c3": dict(grid=512, particles=5_000_000, method="rbf", k=32, rbf_kernel="gaussian", epsilon=0.3, degree=-1,
               scaling="strong", metric=METRIC_RBF),
    "c4": dict(grid=1024, particles=10_000_000, method="idw", k=8, mask=True, scaling="strong", metric=METRIC_C4),
    "c5": dict(grid=2048, particles=50_000_000, method="idw", k=8, out_dtype="f32", div=True, scaling="strong",
               metric=METRIC_C5),
}


def kmax_for(k):
    return next((m for m in KMAX_EXACT if k <= m), 0) or next((m for m in KMAX_KEYS if k + 1 <= m), 0)


def rbf_resolved(args):
    """(kernel, epsilon, degree, m) with scipy's defaults (_rbfinterp.py:300-313)."""
    from math import comb

    from ptv_interpolation_amd import rbf

    kern = args.rbf_kernel
    eps = args.epsilon if args.epsilon is not None else 1.0
    deg = args.degree if args.degree is not None else max(rbf.NAME_TO_MIN_DEGREE.get(kern, -1), 0)
    m = args.k + (comb(deg + 3, 3) if deg >= 0 else 0)
    return kern, eps, deg, m


def rbf_kernel_label(kern, k, m, deg):
    """The solver launch_rbf (ptv_rbf.hip) picks: k_rbf_spd16 for the SPD kernels without a
    polynomial (M <= 32), the null-space k_rbf_ns for the scale-invariant kernels with degree >= their
    minimum and 1 or 4 monomials (k <= 32), else the pivoting k_rbf_local."""
    M = (m + 7) & ~7
    npoly = m - k
    if kern in ("gaussian", "inverse_multiquadric", "inverse_quadratic") and m == k and M <= 32:
        return f"k_rbf_spd16<{M}>"
    min_deg = {"linear": 0, "thin_plate_spline": 1, "cubic": 1, "quintic": 2}
    if kern in min_deg and deg >= min_deg[kern] and npoly in (1, 4) and npoly < k <= 32:
        nc = 16 if k <= 16 else 20 if k <= 20 else 24 if k <= 24 else 32
        return f"k_rbf_ns<{nc}, {npoly}>"
    return f"k_rbf_local<{M}>" if M <= 64 else "k_rbf_big"


def rbf_flops_per_voxel(k, m):
    """distances 8 k(k-1)/2, LU (2/3) m^3, substitution + build 6 m^2, eval 8k + 6m."""
    return 8 * k * (k - 1) / 2 + (2.0 / 3.0) * m ** 3 + 6 * m ** 2 + 8 * k + 6 * m


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="number of GPUs (ranks); > 1 without torchrun's env starts the ranks itself")
    ap.add_argument("--share", default=None, metavar="R/N",
                    help="one GPU: time rank R's step of the N-rank strong z-slab partition (rehearsal)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo: launcher + partition + padded all-gather, a plane-index fill for the kernel")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 20; 5 for c3, c5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 5; 2 for c3, c5)")
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--particles", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--power", type=float, default=2.0)
    ap.add_argument("--radius", type=float, default=None,
                    help="idw: fixed-radius search (PTV_METHOD_IDW_RADIUS, an extension) instead of k-NN")
    ap.add_argument("--method", default=None,
                    choices=["idw", "sibson", "nearest", "rbf", "linear", "div", "filter", "mask"])
    ap.add_argument("--div-dtype", default="f64", choices=["f64", "f32"],
                    help="--method div: field dtype (f32 = the C5 fp32 field, Python-float spacings)")
    ap.add_argument("--rbf-kernel", default=None, help="rbf: scipy kernel name (default thin_plate_spline)")
    ap.add_argument("--epsilon", type=float, default=None, help="rbf: shape parameter")
    ap.add_argument("--degree", type=int, default=None, help="rbf: polynomial degree")
    ap.add_argument("--out-dtype", default=None, choices=["f64", "f32"],
                    help="k-NN methods: U, V, W stored as float32 (PTV_FLAG_OUT_F32, the fused main.py:230 "
                         "astype; arithmetic stays f64)")
    ap.add_argument("--mask", action="store_true", default=None,
                    help="k-NN methods: sphere-pack fluid mask + NaN fill fused (main.py:195-207): solid voxels "
                         "are skipped and written as 0")
    ap.add_argument("--div", action="store_true", default=None,
                    help="k-NN methods: + consistent divergence of each slab (C5)")
    ap.add_argument("--slabs", default=None, metavar="b0,b1,...,bN",
                    help="strong scaling: explicit z-slab plane boundaries (N + 1 of them) instead of the even cut")
    ap.add_argument("--no-balance", action="store_true",
                    help="N>1: keep the even (or --slabs) cut; default: re-cut the slabs during the warmup from the "
                         "ranks' measured step times (zslab.balanced_bounds), fixed before the timed steps")
    ap.add_argument("--halo", type=float, default=None,
                    help="N>1: the scalar slab_halo cull starting at this halo (zslab.interp_slab retries) instead "
                         "of the per-column map (PTV_FLAG_SLAB_CULL_AUTO, default)")
    ap.add_argument("--r0-scale", type=float, default=0.0, help="dev: first search radius / expected k-NN radius")
    ap.add_argument("--cpu-sample-planes", type=int, default=None)
    ap.add_argument("--cpu-workers", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-allgather", action="store_true", help="N>1: skip the timed RCCL all-gather reassembly")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer end-to-end interpolate_field timing")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    defaults = dict(grid=cfg["grid"], particles=cfg["particles"], method=cfg["method"], k=cfg["k"],
                    rbf_kernel=cfg.get("rbf_kernel", "thin_plate_spline"), epsilon=cfg.get("epsilon"),
                    degree=cfg.get("degree"), out_dtype=cfg.get("out_dtype", "f64"), mask=cfg.get("mask", False),
                    div=cfg.get("div", False), radius=cfg.get("radius", 0.0))
    for key, v in defaults.items():
        if getattr(a, key) is None:
            setattr(a, key, v)
    heavy = a.config in ("c3", "c5")
    a.steps = a.steps if a.steps is not None else (5 if heavy else 20)
    a.warmup = a.warmup if a.warmup is not None else (2 if heavy else 5)
    a.scaling = cfg["scaling"]
    a.metric = cfg["metric"]
    return a


# ---------------------------------------------------------------------------------------------
# CPU baseline context: the host's CPU model, and the calibration of the oracle against the
# reference in the build container (tools/cpu_calibration.py)
# ---------------------------------------------------------------------------------------------
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_calibration():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "cpu_calibration_*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            c = json.load(f)
        return {"file": os.path.relpath(files[-1], ROOT), "ratios": c.get("ratios"), "within_15pct": c.get("within_15pct")}
    except Exception:
        return None


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


def emit_line(line):
    """Print one bench JSON line, stamped with the SHA-256 prefix of the library that ran it."""
    line.setdefault("lib_sha256", lib_sha256())
    print(json.dumps(line), flush=True)


def lib_sha256():
    """First 16 hex digits of the loaded library's SHA-256 (tools/traffic.py records the same)."""
    import hashlib

    from ptv_interpolation_amd import _lib

    try:
        with open(_lib.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def traffic_from_profiles():
    """(HBM bytes per main k-NN launch at the headline, its source) from the newest
    profiles/traffic_rNN.json: PMC counters cannot be collected inside the timed process
    (rocprofv3 wraps it), so the line cites the profile run and whether it profiled this very
    library (same SHA-256) or an earlier build."""
    import re

    def round_key(f):  # traffic_r03b.json -> (3, "b"): the round order, not the checkout's mtimes
        m = re.fullmatch(r"traffic_r(\d+)([a-z]?)\.json", os.path.basename(f))
        return (int(m.group(1)), m.group(2))

    files = sorted((f for f in glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json"))
                    if re.fullmatch(r"traffic_r\d+[a-z]?\.json", os.path.basename(f))),  # not traffic_rows_*
                   key=round_key)
    if not files:
        return None, None
    try:
        me = lib_sha256()
        shas = {}
        for f in files:
            with open(f) as fh:
                shas[f] = json.load(fh).get("lib_sha256")
        # the profile of this very library if there is one, else the latest round's
        pick = next((f for f in reversed(files) if shas[f] is not None and shas[f] == me), files[-1])
        files = [pick]
        with open(files[-1]) as f:
            t = json.load(f)
        sha = t.get("lib_sha256")
        src = {"file": os.path.relpath(files[-1], ROOT), "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes",
               "lib_sha256": sha, "this_build": sha is not None and sha == lib_sha256()}
        return float(t["hbm_bytes_per_launch"]), src
    except Exception:
        return None, None


def _cpu_line(value, unit, workers, sample, dt):
    return {"value": value, "unit": unit, "cores": workers, "kind": "port", "sample": sample, "seconds": round(dt, 2),
            "cpu_model": cpu_model(), "calibration": cpu_calibration()}


def cpu_baseline(args, P, Q, ax, az, z0_grid):
    """Oracle restatement on a bounded z-slab sample, multiprocess (test_parallel.py pattern)."""
    from oracle import cpu_ref

    big = args.particles > 20_000_000
    # a bounded sample (10-30 s of CPU work): fewer planes for 50M particles or k >= 30
    planes = min(args.cpu_sample_planes or (4 if big or args.k >= 30 else 16), len(az))
    workers = max(1, min(args.cpu_workers or (4 if big else 16), os.cpu_count() or 1))
    z0 = z0_grid + len(az) // 2 - planes // 2
    t = time.perf_counter()
    cpu_ref.interp_grid_parallel(P, Q, ax, ax, az, args.method, args.k, args.power,
                                 z0=z0, z1=z0 + planes, n_jobs=workers, slab=max(1, planes // workers))
    dt = time.perf_counter() - t
    nvox = planes * len(ax) * len(ax)
    return _cpu_line(round(nvox / dt / 1e6, 4), "Mvoxels/s", workers,
                     f"{planes} central z-planes ({nvox} voxels) of the same {args.grid}^3/{args.particles} workload "
                     f"(mask not applied); scipy KDTree + numpy (oracle/cpu_ref.py), {workers} processes, each "
                     f"building its own tree (interpolator.py:173-182 pattern)", dt)


_BALL = {}


def ball_population(P, ax, radius, nsample=20000):
    """Mean number of particles within `radius` of a grid voxel (seeded voxel sample)."""
    key = (id(P), radius)
    if key not in _BALL:
        from scipy.spatial import KDTree

        G = len(ax)
        rng = np.random.default_rng(1)
        iz, iy, ix = np.unravel_index(rng.integers(0, G ** 3, nsample), (G, G, G))
        q = np.stack([ax[ix], ax[iy], ax[iz]], 1)
        _BALL[key] = float(np.mean(KDTree(P).query_ball_point(q, radius, return_length=True)))
    return _BALL[key]


def cpu_baseline_radius(args, P, Q, ax, radius):
    """The fixed-radius IDW restatement (oracle/cpu_ref.idw_radius_points: KDTree
    query_ball_point + numpy per voxel) on a bounded random voxel sample, one process."""
    from oracle import cpu_ref

    G = len(ax)
    nvox = 100_000
    rng = np.random.default_rng(0)
    iz, iy, ix = np.unravel_index(rng.integers(0, G ** 3, nvox), (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], -1)
    t = time.perf_counter()
    cpu_ref.idw_radius_points(P, Q, q, radius, power=args.power)
    dt = time.perf_counter() - t
    return _cpu_line(round(nvox / dt / 1e6, 4), "Mvoxels/s", 1,
                     f"{nvox} random voxels of the same {G}^3/{args.particles} workload, radius {radius}; scipy "
                     f"KDTree query_ball_point + numpy (oracle/cpu_ref.idw_radius_points), 1 process "
                     f"(no reference counterpart: kind 'port')", dt)


def _rbf_cpu_worker(a):
    from oracle import cpu_ref

    P, Q, q, k, kern, eps, deg = a
    return cpu_ref.rbf_local_points(P, Q, q, k, kern, eps, deg)


def cpu_baseline_rbf(args, P, Q, ax):
    """Oracle local RBF (KDTree + per-voxel LAPACK gesv) on a bounded voxel sample, split over a
    ProcessPoolExecutor like interpolator.py:173-182 (each worker builds its own tree)."""
    from concurrent.futures import ProcessPoolExecutor

    kern, eps, deg, _ = rbf_resolved(args)
    workers = max(1, min(args.cpu_workers or 16, os.cpu_count() or 1))
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
    return _cpu_line(round(nvox / dt / 1e6, 6), "Mvoxels/s", workers,
                     f"{nvox} random voxels of the same {G}^3/{args.particles} workload; scipy KDTree + numpy "
                     f"LAPACK gesv per voxel (oracle/cpu_ref.rbf_local_points), {workers} processes, each "
                     f"building its own tree (interpolator.py:173-182 pattern)", dt)


def env_world():
    """(world, rank, local rank) from torchrun's environment (1, 0, 0 without one)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def check_world(args, world):
    """--gpus must name the world size the ranks were started with (fail loudly, never run
    a different N than the one the line would report)."""
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the world size is {world} "
                         f"(start N ranks with torchrun --nproc-per-node N, or --gpus N alone)")


def _dist_init(args=None):
    """One process per GPU (torchrun env); returns (world, rank, local, dist or None, device)."""
    world, rank, local = env_world()
    if args is not None:
        check_world(args, world)
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, expected {world}")
    return world, rank, local, dist, torch.device("cuda", local)


def launch_ranks(n):
    """Start n ranks of this script under torch.distributed.run (a child process: this process
    has not initialised the GPU and is not replaced) and return their exit code."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def allgather_padded(slab, counts, dist):
    """Reassemble the full (sum(counts), ...) field on every rank from the ranks' (counts[r], ...)
    slabs: one all_gather_into_tensor of slabs padded to max(counts) planes, then the padding
    dropped (zslab.gather_field; uneven slabs when N does not divide nz)."""
    from ptv_interpolation_amd import zslab

    return zslab.gather_field(slab, dist, counts=counts)


@contextlib.contextmanager
def pinned_device(device):
    """PTV_DEVICE=device for the drop-in calls inside the block, the previous value restored."""
    old = os.environ.get("PTV_DEVICE")
    os.environ["PTV_DEVICE"] = str(device)
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("PTV_DEVICE", None)
        else:
            os.environ["PTV_DEVICE"] = old


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


# ---------------------------------------------------------------------------------------------
# the interpolation benches (headline, c2-c5)
# ---------------------------------------------------------------------------------------------
def _device_fluid_mask(G, nz_grid, planes, dev):
    """uint8 (nz_grid, G, G) device tensor: the sphere-pack fluid mask (synth.fluid_mask; stacked
    copies repeat it along z) on planes [a, b), zero elsewhere (never read)."""
    import torch

    from ptv_interpolation_amd import synth

    m = torch.zeros((nz_grid, G, G), dtype=torch.uint8, device=dev)
    a, b = planes
    for z in range(a, b, 64):
        zz = min(b, z + 64)
        m[z:zz] = synth.fluid_mask_device(G, z, zz, dev)
    return m


def parse_share(share):
    """'R/N' -> (R, N) with 0 <= R < N."""
    try:
        r, n = (int(v) for v in share.split("/"))
    except ValueError:
        raise SystemExit(f"bench.py: --share wants R/N, got {share!r}")
    if not (n >= 1 and 0 <= r < n):
        raise SystemExit(f"bench.py: --share {share}: need 0 <= R < N")
    return r, n


def e2e_leg(args, P, Q, G, k, radius, local):
    """End to end through the drop-in, as main.py:151 + :184-192 call it: a host DataFrame
    in, dense float64 create_grid meshgrids (3 x 8 V bytes), host float64 U, V, W out: the
    separability check of the meshgrids, H2D, binning + kernels, D2H.  The first call also
    creates the context and its device buffers (what a one-shot main.py run pays); the second
    is the steady state.  Zero-stride create_grid(dense=False) views are timed as well."""
    import pandas as pd

    from ptv_interpolation_amd import _lib
    from ptv_interpolation_amd import interpolator as ip

    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
    kw = {"idw": dict(idw_neighbors=k, idw_power=args.power), "sibson": dict(sibson_neighbors=k),
          "nearest": {}}[args.method]
    if radius:
        kw["idw_radius"] = radius
    res = {}
    with pinned_device(local):  # this rank's GPU only (launcher.devices())
        for name, dense in (("dense", True), ("views", False)):
            grid, _ = ip.create_grid(((0, G), (0, G), (0, G)), G, dense=dense)
            walls = []
            for _ in range(2):
                t = time.perf_counter()
                with contextlib.redirect_stdout(io.StringIO()):
                    out = ip.interpolate_field(df, grid, method=args.method, **kw)
                walls.append(time.perf_counter() - t)
                del out
            hs = _lib.Context.get(local).stats
            res[name] = {"wall_s_first": round(walls[0], 3), "wall_s": round(walls[-1], 3),
                         "mvoxels_per_s": round(G ** 3 / walls[-1] / 1e6, 1),
                         "ms_h2d": round(hs["ms_h2d"], 2),
                         "ms_device": round(hs["ms_total"] - hs["ms_h2d"] - hs["ms_d2h"], 2),
                         "ms_d2h": round(hs["ms_d2h"], 2)}
            del grid
    d = res["dense"]
    d2h_floor = 3 * 8 * G ** 3 / 53e9 * 1e3  # measured pinned / touched D2H rate, 53 GB/s
    return {**d, "views": res["views"], "d2h_floor_ms": round(d2h_floor, 1),
            "what": "interpolate_field(DataFrame, create_grid() dense meshgrids as main.py:151) -> host float64 "
                    "U, V, W; wall_s = second call, wall_s_first includes context + buffer creation; "
                    "views = create_grid(dense=False)"}


def main_interp(args):
    import torch

    share = parse_share(args.share) if args.share else None
    if share is not None:
        # one GPU, no process group: rank R's step of the N-rank strong partition
        if env_world()[0] != 1 or args.scaling != "strong":
            raise SystemExit("bench.py: --share runs one process on one GPU, for a strong-scaling config")
        world0, rank0, local, dist, dev = _dist_init()
        rank, world = share
    else:
        world, rank, local, dist, dev = _dist_init(args)
    from ptv_interpolation_amd import _lib, synth, zslab

    G, k = args.grid, args.k
    rbf = args.method == "rbf"
    weak = args.scaling == "weak"
    if args.method == "nearest":
        k = args.k = 1
    nz = G * world if weak else G
    if args.slabs:
        bounds = [int(v) for v in args.slabs.split(",")]
        if weak or len(bounds) != world + 1 or bounds[0] != 0 or bounds[-1] != nz or \
                any(bounds[i] >= bounds[i + 1] for i in range(world)):
            raise SystemExit(f"bench.py: --slabs needs {world + 1} increasing boundaries from 0 to {nz}")
    else:
        bounds = [0] + [zslab.rank_slab(nz, world, r)[1] for r in range(world)] if not weak else None
    z0, z1 = (rank * G, (rank + 1) * G) if weak else (bounds[rank], bounds[rank + 1])
    za, zb, hlo, hhi = zslab.halo_slab(z0, z1, nz, 1 if args.div else 0)

    # particles: replicated on every rank (north_star); weak: copy r generated by rank r and
    # all-gathered; strong: generated by rank 0 and broadcast
    def cols_of(P, Q):
        return [torch.from_numpy(np.ascontiguousarray(P[:, i])).to(dev) for i in range(3)] + \
               [torch.from_numpy(np.ascontiguousarray(Q[:, i])).to(dev) for i in range(3)]

    P = Q = None
    if weak:
        P, Q = synth.sphere_pack(args.particles, G, z_tiles=world, z_tile=rank)
        cols = zslab.replicate_columns(cols_of(P, Q), dist)
    elif rank == 0 or dist is None:
        P, Q = synth.sphere_pack(args.particles, G)
        cols = zslab.broadcast_columns(cols_of(P, Q), dist)
    else:
        cols = zslab.broadcast_columns([torch.empty(args.particles, dtype=torch.float64, device=dev)
                                        for _ in range(6)], dist)
    n = cols[0].numel()
    ax_h = np.linspace(0, G - 1, G)
    az_h = np.linspace(0, nz - 1, nz)
    axes = [torch.from_numpy(ax_h).to(dev), torch.from_numpy(ax_h.copy()).to(dev), torch.from_numpy(az_h).to(dev)]
    out_f32 = args.out_dtype == "f32" and not rbf
    odt = torch.float32 if out_f32 else torch.float64
    out = [torch.empty((zb - za, G, G), dtype=odt, device=dev) for _ in range(3)]
    mask_t = None
    fluid_frac = None
    if args.mask or args.div:
        mask_t = _device_fluid_mask(G, nz, (za, zb), dev)
        fluid_frac = float(mask_t[z0:z1].float().mean().item())
    div_out = torch.empty((z1 - z0, G, G), dtype=odt, device=dev) if args.div else None
    ctx = _lib.Context(local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    method = {"idw": _lib.METHOD_IDW, "sibson": _lib.METHOD_SIBSON, "nearest": _lib.METHOD_NEAREST}.get(args.method)
    radius = args.radius if (args.radius and args.method == "idw") else 0.0
    if radius:
        method = _lib.METHOD_IDW_RADIUS
    cull = world > 1 and not rbf and not radius
    halo = zslab.HaloState(args.halo) if (cull and args.halo is not None) else None
    ptrs = [c.data_ptr() for c in cols]
    aptrs = [a.data_ptr() for a in axes]
    optrs = [o.data_ptr() for o in out]
    if rbf:
        kern, eps, deg, m_sys = rbf_resolved(args)

    def step():
        if rbf:
            ctx.interp_rbf_dev(n, ptrs, G, G, nz, axes_ptrs=aptrs, out_ptrs=optrs, k=k, kernel=kern, epsilon=eps,
                               degree=deg, z_range=(za, zb), stream=stream)
            return
        flags = ((_lib.FLAG_OUT_F32 if out_f32 else 0) | (_lib.FLAG_NAN_TO_NUM if args.mask else 0) |
                 (_lib.FLAG_SLAB_CULL_AUTO if cull and halo is None else 0))
        mptr = mask_t.data_ptr() if (mask_t is not None and args.mask) else 0

        def call(h):
            return ctx.interp_knn_dev(n, ptrs, G, G, nz, axes_ptrs=aptrs, out_ptrs=optrs, method=method, k=k,
                                      power=args.power, stream=stream, mask_ptr=mptr, r0_scale=args.r0_scale,
                                      flags=flags, z_range=(za, zb), slab_halo=h, radius=radius)

        zslab.interp_slab(call, halo) if halo is not None else call(0.0)
        if args.div:
            dtc = _lib.F32 if out_f32 else _lib.F64
            ctx.divergence_dev(G, G, zb - za, [o.data_ptr() for o in out], mask_t[za:zb].data_ptr(),
                               div_out.data_ptr(), 1.0, 1.0, 1.0, field_dtype=dtc, result_dtype=dtc,
                               z_range=(hlo, hlo + (z1 - z0)), edges=(hlo == 0, hhi == 0), stream=stream)

    # load balance (N > 1, strong k-NN configs): the sphere pack's void planes cost more per plane
    # than its packed ones, so the even cut leaves the void-heavy slabs last.  After warmup steps 1
    # and 3 every rank's device time of its step is all-gathered and the slabs are re-cut
    # (zslab.balanced_bounds); the next warmup step builds the new slab's cull map, and the cut is
    # fixed before the timed steps (the same grid, the same particles: strong scaling unchanged)
    balance = (dist is not None and world > 1 and not weak and not rbf and not args.div and not args.no_balance
               and not args.slabs)
    rebalances = []

    def rebalance():
        nonlocal z0, z1, za, zb, out, optrs, bounds, mask_t, fluid_frac
        st = ctx.last_stats()
        t = torch.tensor([st["ms_bin"] + st["ms_cull"] + st["ms_lattice"] + st["ms_knn"]], dtype=torch.float64,
                         device=dev)
        ts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(ts, t)
        times = [float(x.item()) for x in ts]
        new = zslab.balanced_bounds(bounds, times)
        rebalances.append({"bounds": bounds, "ms": [round(v, 3) for v in times]})
        if new != bounds:
            bounds = new
            z0, z1 = bounds[rank], bounds[rank + 1]
            za, zb = z0, z1
            out = [torch.empty((zb - za, G, G), dtype=odt, device=dev) for _ in range(3)]
            optrs = [o.data_ptr() for o in out]
            if mask_t is not None:
                mask_t = _device_fluid_mask(G, nz, (za, zb), dev)
                fluid_frac = float(mask_t[z0:z1].float().mean().item())

    cold = None
    for w in range(args.warmup):
        if w == 0:
            # the cold call (a one-shot interpolate_field: no cached cull map, every particle binned)
            torch.cuda.synchronize(dev)
            tc = time.perf_counter()
        step()
        if w == 0:
            torch.cuda.synchronize(dev)
            st0 = ctx.last_stats()
            cold = {"wall_ms": round((time.perf_counter() - tc) * 1e3, 3),
                    "device_ms": round(st0["ms_bin"] + st0["ms_cull"] + st0["ms_lattice"] + st0["ms_knn"] +
                                       st0["ms_solve"], 3), "n_binned": int(st0["n_binned"])}
        if balance and w in (1, 3) and w + 1 < args.warmup:
            rebalance()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    rec = {key: [] for key in ("ms_knn", "ms_lattice", "ms_bin", "ms_solve", "ms_cull", "ms_stencil", "n_binned",
                               "n_rbf_pivoted")}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = ctx.last_stats()  # synchronises on the step's events
        for key in rec:
            rec[key].append(st[key])
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    avg = {key: float(np.mean(v)) for key, v in rec.items()}

    # RCCL all-gather reassembly of the full field, once, reported apart from `value`
    gather_ms = None
    if dist is not None and not args.no_allgather:
        counts = [b - a for a, b in (((r * G, (r + 1) * G) if weak else (bounds[r], bounds[r + 1]))
                                     for r in range(world))]
        try:
            for it in range(2):  # the first all-gather sets RCCL's channels up: time the second
                torch.cuda.synchronize(dev)
                dist.barrier()
                tg = time.perf_counter()
                for o in out:
                    full = allgather_padded(o[hlo:hlo + (z1 - z0)], counts, dist)
                    del full
                torch.cuda.synchronize(dev)
                gather_ms = (time.perf_counter() - tg) * 1e3
            t = torch.tensor([gather_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            gather_ms = float(t.item())
        except Exception as e:  # the reassembly must never take the bench line down
            gather_ms = repr(e)[:200]

    # end-to-end through the drop-in (host DataFrame in, host float64 U, V, W out): H2D +
    # binning + kernels + D2H, what a main.py user pays (N = 1, unmasked k-NN configs)
    e2e = None
    if world == 1 and share is None and not rbf and not args.mask and not args.div and not args.no_e2e and P is not None:
        try:
            e2e = e2e_leg(args, P, Q, G, k, radius, local)
        except Exception as e:
            e2e = {"error": repr(e)[:200]}

    V_slab = (z1 - z0) * G * G
    s_out = 4 if out_f32 else 8
    if rbf:
        flops = (zb - za) * G * G * rbf_flops_per_voxel(k, m_sys)
        tf = flops / (avg["ms_solve"] * 1e-3) / 1e12
        roof = {"bound": "fp64", "achieved": round(tf, 2), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tf / FP64_PEAK_TFLOPS, 4), "traffic": None,
                "kernel": rbf_kernel_label(kern, k, m_sys, deg),
                "alg_flops_per_launch": flops, "kernel_ms": round(avg["ms_solve"], 3),
                "knn_slots_ms": round(avg["ms_knn"], 3),
                # voxels the null-space kernel handed to the pivoting kernel per step (max over steps)
                "n_rbf_pivoted": int(max(rec["n_rbf_pivoted"])) if rec["n_rbf_pivoted"] else 0}
    else:
        Vk = (zb - za) * G * G  # voxels the k-NN launch computes (slab + redundant halo planes)
        if radius:  # gather model with the measured mean ball population in place of k
            k_eff = ball_population(P, ax_h, radius) if P is not None else 0.0
            alg = int(round(Vk * (6 * k_eff * 8 + 3 * s_out)))
        elif args.mask:  # solid voxels are skipped: fluid V in the gather term, + the mask byte
            alg = int(round(Vk * fluid_frac)) * 6 * k * 8 + Vk * (3 * s_out + 1)
        else:
            alg = Vk * (6 * k * 8 + 3 * s_out)
        ach = alg / (avg["ms_knn"] * 1e-3) / 1e9
        t_step = avg["ms_bin"] + avg["ms_cull"] + avg["ms_lattice"] + avg["ms_knn"]
        alg_step = alg + 48 * avg["n_binned"]
        # the committed PMC traffic is the whole-grid one-GPU launch's: never a share's or a slab's
        headline_shape = (G == 512 and args.particles == 5_000_000 and k == 8 and not args.mask and not out_f32
                          and world == 1 and share is None and not radius)
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 4),
                "traffic": traffic_from_profiles()[0] if headline_shape else None,
                "traffic_source": traffic_from_profiles()[1] if headline_shape else None,
                "kernel": "k_knn_interp<4, radius>" if radius else f"k_knn_interp<{kmax_for(k)}>",
                "alg_bytes_per_launch": alg,
                "kernel_ms": round(avg["ms_knn"], 3),
                "frac_step": round(alg_step / (t_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "step_device_ms": round(t_step, 3)}
        if args.div:
            dalg = V_slab * (4 * s_out + 1)
            dach = dalg / (avg["ms_stencil"] * 1e-3) / 1e9
            roof["divergence"] = {"kernel": f"k_divergence<{'float' if out_f32 else 'double'}>",
                                  "achieved": round(dach, 1), "frac": round(dach / HBM_PEAK_GBPS, 4),
                                  "alg_bytes": dalg, "kernel_ms": round(avg["ms_stencil"], 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and P is not None:
        try:
            cpu = (cpu_baseline_rbf(args, P, Q, ax_h) if rbf else
                   cpu_baseline_radius(args, P, Q, ax_h, radius) if radius else
                   cpu_baseline(args, P, Q, ax_h, az_h, 0))
        except Exception as e:  # the baseline must never take the GPU line down
            cpu = {"value": None, "error": repr(e)[:200]}

    if rank == 0 or share is not None:
        vox_total = V_slab * world if weak else G ** 3
        value = vox_total / (elapsed / args.steps) / 1e6
        if share is not None:  # one rank's share: its own slab's rate; the N-rank value is the rehearsal's
            value = V_slab / (elapsed / args.steps) / 1e6
        if weak:
            wl = (f"{G}x{G}x{nz} grid = {world} stacked {G}^3 sphere-pack copies / {args.particles * world} "
                  f"particles (replicated), {G}^3 slab + {args.particles} particles' copy per GPU")
        else:
            sizes = [bounds[r + 1] - bounds[r] for r in range(world)] if bounds is not None else [G]
            per = (f"{sizes[0]} planes" if min(sizes) == max(sizes) else f"{min(sizes)}-{max(sizes)} planes")
            wl = f"{G}^3 grid / {args.particles} particles (replicated), z-slabs of {per} per GPU"
        if share is not None:
            wl = (f"rank {rank} of {world}: planes [{z0}, {z1}) ({z1 - z0} planes) of the " + wl +
                  " (one-GPU rehearsal, no collective)")
        if rbf:
            wl += f"; local RBF {kern} k={k} eps={eps} degree={deg} (system {m_sys}) fp64"
        else:
            wl += ((f"; IDW radius={radius} (mean ball {ball_population(P, ax_h, radius):.2f} particles) p={args.power} fp64"
                    if radius else f"; {args.method.upper()} k={k} p={args.power} fp64") +
                   (" (float32 U, V, W)" if out_f32 else "") +
                   (f" + sphere-pack fluid mask ({fluid_frac:.1%} fluid, solid skipped)" if args.mask else "") +
                   (" + consistent divergence (one-plane halo interpolated)" if args.div else ""))
        line = {
            "metric": args.metric, "value": round(value, 2), "unit": "Mvoxels/s",
            "n_gpus": 1 if share is not None else world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            # arithmetic type: every k-NN / weight / sum / solve is fp64; the C5 field is stored as f32
            "dtype": "f64", "field_dtype": "f32" if out_f32 else "f64",
            "data": "synthetic: generate_sphere_pack.py geometry scaled to voxel units, seeded, w=1 flow field",
            "config": {"workload": wl, "name": args.config, "grid": G, "grid_z": nz, "particles": args.particles,
                       "particles_replicated": n, "method": args.method, "k": k, "power": args.power,
                       "out_dtype": "f32" if out_f32 else "f64", "mask": bool(args.mask), "div": bool(args.div),
                       "planes": [z0, z1],
                       "parallelism": f"z-slab x{world}" + (" (particles replicated, per-slab cull)" if cull else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "breakdown_ms": {"bin": round(avg["ms_bin"], 3), "cull": round(avg["ms_cull"], 3),
                             "lattice": round(avg["ms_lattice"], 3), "knn": round(avg["ms_knn"], 3),
                             "solve": round(avg["ms_solve"], 3), "divergence": round(avg["ms_stencil"], 3)},
        }
        if share is not None:
            line["share"] = {"rank": rank, "world": world}
        if cold is not None:
            line["cold_call"] = dict(cold, note="first warmup step on a fresh context (includes one-time "
                                                "buffer allocation; N > 1: no cached cull map, every "
                                                "particle binned; before any re-cut)")
        if args.mask:
            line["fluid_mvoxels_per_s"] = round(value * fluid_frac, 2)
        if bounds is not None and world > 1:
            line["slabs"] = {"bounds": bounds, "rebalances": rebalances,
                             "how": ("re-cut from the ranks' measured step times during the warmup "
                                     "(zslab.balanced_bounds)" if balance else
                                     ("explicit --slabs" if args.slabs else "even cut"))}
        if cull:
            line["cull"] = ({"mode": "scalar slab_halo", **halo.as_dict()} if halo is not None else
                            {"mode": "per-column map (PTV_FLAG_SLAB_CULL_AUTO), proven on the device"})
            line["cull"]["particles_binned"] = int(avg["n_binned"])
        if gather_ms is not None:
            line["allgather_ms"] = round(gather_ms, 2) if isinstance(gather_ms, float) else gather_ms
        if e2e is not None:
            line["e2e"] = e2e
        emit_line(line)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


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
            "cpu_model": cpu_model(),
            "sample": f"{planes} central z-planes ({nvox} voxels) of the same {G}^3 field; numpy restatement "
                      f"of physics.compute_consistent_divergence (oracle/cpu_ref.py), 1 process",
            "seconds": round(dt, 2)}


def main_div(args):
    """--method div: one step = the consistent divergence of a resident (G, G, G) velocity field
    with the sphere-pack fluid mask (view_divergence.py:39).  Weak scaling: each rank owns a
    G^3 z-slab plus one halo plane per interior side (no collective on the data path)."""
    import torch

    world, rank, local, dist, dev = _dist_init(args)
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
        emit_line(line)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main_filter(args):
    """--method filter: one step = remove_outliers_knn (filtering.py:5-58) over a resident particle set:
    binning + (k+1)-NN of every particle among the particles with the median/MAD statistics fused
    into the search kernel's epilogue (filter mode).
    Weak scaling: each rank filters its own sphere-pack copy (independent particle sets)."""
    import torch

    world, rank, local, dist, dev = _dist_init(args)
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
            cpu = {"value": round(m / dt / 1e6, 4), "unit": "Mparticles/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                   "sample": f"first {m} particles of the same cloud (a {m / n:.0%} subset at the same density "
                             "is not the same neighbourhoods; documented), scipy KDTree(k+1) + numpy median/MAD "
                             "(oracle/cpu_ref.outlier_filter = filtering.py:15-51), workers=1",
                   "seconds": round(dt, 2)}
        except Exception as e:
            cpu = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        emit_line({
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
                         "traffic": row_traffic("filter:k_knn_interp", "filter:k_slot_speed")
                         if (k == 25 and n == 5_000_000) else None,
                         "kernel": f"k_knn_interp<{kmax_for(k + 1)}, filter> ((k+1)-NN + fused median/MAD)",
                         "alg_bytes_per_launch": alg, "kernel_ms": round(kavg, 4)},
            "cpu_baseline": cpu})
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main_mask(args):
    """--method mask: one step = sample_mask_on_grid (a G^3 raw mask onto the G^3 grid, main.py:161
    at --downscale 1) + extract_boundary_particles(thickness=1, step=1) (main.py:168) on resident
    bytes.  Weak scaling: each rank processes its own mask copy."""
    import torch

    world, rank, local, dist, dev = _dist_init(args)
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
                   "cpu_model": cpu_model(),
                   "sample": f"{Gs}^3 sphere-pack mask, numpy restatement (oracle/cpu_ref.sample_mask_nearest + "
                             "boundary_particles of interpolator.py:205-284), 1 process",
                   "seconds": round(dt, 2)}
        except Exception as ex:
            cpu = {"value": None, "error": repr(ex)[:200]}
    if rank == 0:
        emit_line({
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
            "cpu_baseline": cpu})
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main_linear(args):
    """--method linear: one step = griddata(method='linear') (interpolator.py:196-197, the reference
    default) on resident data: binning + the k = 1 slot search (walk starts) + the point-location walk
    and barycentric interpolation of every voxel (ptv_linear.hip).  The triangulation is built once on
    the host by scipy's Delaunay (Qhull, as LinearNDInterpolator does) before the timed region; its
    wall time is reported next to the step (`host_triangulation_s`).  Defaults 256^3 / 1M particles
    (--config c2 size).  Weak scaling: each rank interpolates its own copy."""
    import torch
    from scipy.spatial import Delaunay

    world, rank, local, dist, dev = _dist_init(args)
    from ptv_interpolation_amd import _lib, synth

    G = args.grid if args.config != "headline" or args.grid != 512 else 256
    n = args.particles if args.config != "headline" or args.particles != 5_000_000 else 1_000_000
    P, _ = synth.sphere_pack(n, G)
    Q = np.random.default_rng(20261017 + rank).standard_normal((n, 3))
    t0 = time.perf_counter()
    d = Delaunay(P)
    tri = _lib.Triangulation(d)  # includes scipy's transform (LinearNDInterpolator computes it too)
    t_host = time.perf_counter() - t0
    ax_h = np.linspace(0, G - 1, G)
    cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).to(dev) for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).to(dev) for i in range(3)]
    axes = [torch.from_numpy(ax_h.copy()).to(dev) for _ in range(3)]
    tarr = [torch.from_numpy(a).to(dev) for a in (tri.simplices, tri.neighbors, tri.transform, tri.vertex_to_simplex)]
    out = [torch.empty((G, G, G), dtype=torch.float64, device=dev) for _ in range(3)]
    ctx = _lib.Context(local)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        return ctx.interp_linear_dev(n, [c.data_ptr() for c in cols], G, G, G, [t.data_ptr() for t in tarr],
                                     tri.nsimplex, tri.min_bound, tri.max_bound,
                                     axes_ptrs=[a.data_ptr() for a in axes], out_ptrs=[o.data_ptr() for o in out],
                                     stream=stream)

    elapsed, w_ms = _timed(step, args, dist, dev, "ms_solve", ctx)
    st = ctx.last_stats()
    wavg = float(np.mean(w_ms))
    V = G ** 3
    inside = float((out[0] != 0).double().mean().item())
    # per voxel inside the hull: the containing simplex's transform (96 B) and vertex ids (16 B), the
    # 4 vertices' values (4 x 24 B); every voxel: its walk-start slot (4 B) + the 3 outputs (24 B)
    alg = int(V * inside) * (96 + 16 + 96) + V * (4 + 24)
    ach = alg / (wavg * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            from scipy.interpolate import LinearNDInterpolator

            ip = LinearNDInterpolator(d, Q, fill_value=0.0)  # reuses the triangulation and its transform
            nz_s = max(1, min(G, 2_000_000 // (G * G)))
            Z, Y, X = np.meshgrid(ax_h[G // 2 - nz_s // 2:G // 2 - nz_s // 2 + nz_s], ax_h, ax_h, indexing="ij")
            t = time.perf_counter()
            ip((X, Y, Z))
            dt = time.perf_counter() - t
            cpu = {"value": round(X.size / dt / 1e6, 4), "unit": "Mvoxels/s", "cores": 1, "kind": "port",
                   "cpu_model": cpu_model(),
                   "sample": f"{nz_s} central z-planes ({X.size} voxels) of the same workload: scipy "
                             "LinearNDInterpolator evaluation over the same prebuilt Delaunay (the reference's "
                             "griddata minus its Qhull build), 1 process", "seconds": round(dt, 2)}
        except Exception as e:
            cpu = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        emit_line({
            "metric": METRIC_LINEAR, "value": round(V * world / (elapsed / args.steps) / 1e6, 2),
            "unit": "Mvoxels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: generate_sphere_pack.py geometry scaled to voxel units, N(0,1) velocities",
            "config": {"workload": f"griddata(method='linear') {G}^3 grid / {n} particles ({tri.nsimplex} simplices, "
                                   f"{inside:.1%} of voxels inside the hull)", "grid": G, "particles": n,
                       "method": "linear", "parallelism": f"independent copies x{world}"},
            "host_triangulation_s": round(t_host, 2),
            "breakdown_ms": {"bin": round(st["ms_bin"], 3), "lattice": round(st["ms_lattice"], 3),
                             "nearest_slots": round(st["ms_knn"], 3), "walk": round(wavg, 3)},
            "brute_force_voxels": int(st["n_singular"]),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None, "kernel": "k_linear_walk",
                         "alg_bytes_per_launch": alg, "kernel_ms": round(wavg, 4)},
            "cpu_baseline": cpu})
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main_dryrun(args):
    """--dry-run: the N-rank strong partition on the CPU over gloo.  Rank 0 generates the
    particle set and broadcasts it, every rank computes its planes rank_slab(nz, N, r) (a fill
    with the global plane index stands in for the HIP kernel, which needs a GPU), the padded
    all-gather reassembles the field, and rank 0 checks that every plane arrived exactly once
    and in order.  Prints one JSON line: world size, partition, check."""
    import torch
    import torch.distributed as dist

    world, rank, _ = env_world()
    check_world(args, world)
    from ptv_interpolation_amd import synth, zslab

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    else:
        dist = None
    G = args.grid
    nz = G
    z0, z1 = zslab.rank_slab(nz, world, rank)
    if rank == 0:
        P, Q = synth.sphere_pack(args.particles, G)
        cols = [torch.from_numpy(np.ascontiguousarray(a[:, i])) for a in (P, Q) for i in range(3)]
    else:
        cols = [torch.empty(args.particles, dtype=torch.float64) for _ in range(6)]
    zslab.broadcast_columns(cols, dist)
    digest = torch.tensor([float(sum(float(c.sum()) for c in cols))], dtype=torch.float64)
    slab = torch.arange(z0, z1, dtype=torch.float64).view(-1, 1, 1).expand(z1 - z0, G, G).contiguous()
    counts = [b - a for a, b in (zslab.rank_slab(nz, world, r) for r in range(world))]
    full = zslab.gather_field(slab, dist, counts=counts)
    digests = [torch.empty_like(digest) for _ in range(world)] if dist else [digest]
    if dist:
        dist.all_gather(digests, digest)
    # the warmup re-cut of the GPU path (zslab.balanced_bounds over all-gathered step times), with a
    # synthetic cost of 1 per plane plus 2 per plane in the middle third standing in for the kernel's
    bounds = [0] + [zslab.rank_slab(nz, world, r)[1] for r in range(world)]
    cost = lambda a, b: float(sum(1.0 + (2.0 if nz // 3 <= z < 2 * nz // 3 else 0.0) for z in range(a, b)))  # noqa: E731
    spread = []
    for _ in range(2):
        t = torch.tensor([cost(bounds[rank], bounds[rank + 1])], dtype=torch.float64)
        ts = [torch.zeros_like(t) for _ in range(world)] if dist else [t]
        if dist:
            dist.all_gather(ts, t)
        times = [float(x.item()) for x in ts]
        spread.append(max(times) / min(times))
        bounds = zslab.balanced_bounds(bounds, times, min_planes=1)
    bt = torch.tensor(bounds, dtype=torch.float64)
    allb = [torch.zeros_like(bt) for _ in range(world)] if dist else [bt]
    if dist:
        dist.all_gather(allb, bt)
    if rank == 0:
        ok = (tuple(full.shape) == (nz, G, G) and
              bool(torch.equal(full[:, 0, 0], torch.arange(nz, dtype=torch.float64))) and
              bool(torch.equal(full, full[:, :1, :1].expand_as(full))))
        print(json.dumps({"dry_run": True, "n_gpus": world, "world_size": dist.get_world_size() if dist else 1,
                          "gpus_flag": args.gpus, "grid": G, "particles": args.particles,
                          "partition": [list(zslab.rank_slab(nz, world, r)) for r in range(world)],
                          "particles_agree": len({float(d.item()) for d in digests}) == 1,
                          "field_reassembled": ok,
                          "balanced": {"bounds": bounds, "ranks_agree": all(torch.equal(x, bt) for x in allb),
                                       "cost_spread": [round(v, 4) for v in spread]}}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        if args.share:
            raise SystemExit("bench.py: --share is a one-GPU run; drop --gpus")
        sys.exit(launch_ranks(args.gpus))
    if args.dry_run:
        return main_dryrun(args)
    if args.method == "linear":
        return main_linear(args)
    if args.method == "div":
        return main_div(args)
    if args.method == "filter":
        return main_filter(args)
    if args.method == "mask":
        return main_mask(args)
    return main_interp(args)


if __name__ == "__main__":
    main()
