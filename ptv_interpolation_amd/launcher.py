"""Multi-GPU z-slab launcher for the drop-in API (replaces the reference's
``ProcessPoolExecutor`` fan-out of interpolator.py:173-182 / test_parallel.py).

Every voxel depends only on the particle set and its own coordinate, and a z-slab call of
the kernels produces the same bits as the same planes of a whole-grid call, so the grid's
z planes are split into contiguous slabs, one per device, each device interpolates its slab
from the (replicated) particle set, and the slabs land in disjoint slices of the caller's
output.  The k-NN methods bin only the particles that can reach their slab (the per-column cull
map of PTV_FLAG_SLAB_CULL_AUTO, cached in each slab's context and proven exact on the device).
One host thread per device drives its own context and stream (ctypes releases the GIL during the C
calls); no collective touches the data path.

Devices: ``PTV_DEVICE=i`` pins one device; ``PTV_DEVICES=0,1,...`` lists them (a device
may repeat: several contexts, one per slab, on the same GPU); default all visible GPUs.

Slab bounds start even; callers that pass a ``balance_key`` (the k-NN methods) get them re-cut
from the slabs' measured device times (``zslab.balanced_bounds``, as bench.py's warmup does), at
most ``MAX_RECUTS`` times per (grid, devices, key), and only from calls whose slabs all ran culled
(a cold call's time is dominated by binning every particle, not by its planes).  A re-cut changes
the slabs' keys, so the next call of each slab builds its cull map again.

Each context is used by one thread at a time (a per-context lock held across ``fn``): concurrent
calls share the slab contexts, their buffers and their cached cull maps.
"""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib

_ctx_lock = threading.Lock()
_slab_ctx = {}
_use_locks = {}  # id(context) -> lock held while a slab runs on it
_balance = {}  # (nz, devices, balance_key) -> {"bounds": [...], "recuts": int}
MAX_RECUTS = 2
_tls = threading.local()  # per calling thread: what fn returned for each slab of its last run_slabs


def __getattr__(name):
    # launcher.last_results: the calling thread's last run_slabs results (slab order); thread-local,
    # so concurrent interpolate_field calls do not overwrite each other's per-slab stats
    if name == "last_results":
        return getattr(_tls, "results", [])
    raise AttributeError(name)


def devices():
    if "PTV_DEVICE" in os.environ:
        return [int(os.environ["PTV_DEVICE"])]
    if os.environ.get("PTV_DEVICES"):
        return [int(d) for d in os.environ["PTV_DEVICES"].split(",") if d.strip()]
    return list(range(max(1, _lib.device_count())))


def slab_bounds(nz: int, parts: int):
    """Contiguous [z0, z1) slabs, as even as possible, in order."""
    parts = max(1, min(parts, nz))
    edges = [nz * i // parts for i in range(parts + 1)]
    return [(edges[i], edges[i + 1]) for i in range(parts)]


def context(device: int, slot: int) -> "_lib.Context":
    """Context of slab `slot` on `device` (slot 0 is the shared per-device context)."""
    if slot == 0:
        return _lib.Context.get(device)
    with _ctx_lock:
        c = _slab_ctx.get((device, slot))
        if c is None:
            c = _lib.Context(device)
            _slab_ctx[(device, slot)] = c
    return c


def _use_lock(ctx):
    with _ctx_lock:
        lk = _use_locks.get(id(ctx))
        if lk is None:
            lk = _use_locks[id(ctx)] = threading.Lock()
    return lk


def _slab_cost(res, wall_ms):
    """A slab's cost for the re-cut: its device time when fn returned the call's stats, else wall."""
    if isinstance(res, dict) and all(k in res for k in ("ms_bin", "ms_cull", "ms_lattice", "ms_knn")):
        return res["ms_bin"] + res["ms_cull"] + res["ms_lattice"] + res["ms_knn"]
    return wall_ms


def _all_culled(res):
    return all(isinstance(r, dict) and 0 < r.get("n_binned", 0) < r.get("n_particles", 0) for r in res)


def current_bounds(nz: int, parts: int, balance_key=None, devs=None):
    """The N + 1 slab boundaries run_slabs uses for this grid (balanced ones once measured)."""
    even = [0] + [b for _, b in slab_bounds(nz, parts)]
    if balance_key is None:
        return even
    ent = _balance.get((nz, tuple(devs if devs is not None else devices()), balance_key))
    return list(ent["bounds"]) if ent is not None and len(ent["bounds"]) == len(even) else even


def run_slabs(nz: int, fn, out, results=None, balance_key=None):
    """Fill the preallocated C-contiguous (nz, ...) arrays ``out`` slab by slab.

    ``fn(ctx, z0, z1, views)`` writes planes [z0, z1) into ``views`` (the z-slices of ``out``,
    contiguous, written in place by the library's D2H: no per-slab arrays and no host
    concatenation).  One slab per device of ``devices()``, one host thread each; a single
    device runs fn(ctx, 0, nz, out) directly.  Returns ``out``; fn's per-slab results are
    ``last_results`` of the calling thread (or appended to ``results`` when given).
    ``balance_key``: re-cut the bounds of later calls with the same key from this call's slab
    costs (see the module docstring)."""
    out = tuple(out)
    for a in out:
        if not (a.flags.c_contiguous and a.shape[0] == nz):
            raise ValueError("run_slabs: outputs must be C-contiguous with nz leading planes")
    devs = devices()
    if len(devs) <= 1 or nz < 2:
        ctx = _lib.Context.get(devs[0])
        with _use_lock(ctx):
            res = [fn(ctx, 0, nz, out)]
        _tls.results = res
        if results is not None:
            results.extend(res)
        return out
    parts = min(len(devs), nz)
    bounds = current_bounds(nz, parts, balance_key, devs)
    seen = {}
    jobs = []
    for i, d in enumerate(devs[:parts]):
        z0, z1 = bounds[i], bounds[i + 1]
        slot = seen.get(d, 0)
        seen[d] = slot + 1
        jobs.append((context(d, slot), z0, z1, tuple(a[z0:z1] for a in out)))

    def run(job):
        with _use_lock(job[0]):
            t0 = time.perf_counter()
            r = fn(*job)
            return r, (time.perf_counter() - t0) * 1e3

    with ThreadPoolExecutor(len(jobs)) as ex:
        timed = list(ex.map(run, jobs))
    res = [r for r, _ in timed]
    _tls.results = res
    if results is not None:
        results.extend(res)
    if balance_key is not None and _all_culled(res):
        key = (nz, tuple(devs), balance_key)
        ent = _balance.setdefault(key, {"bounds": bounds, "recuts": 0})
        if ent["recuts"] < MAX_RECUTS:
            from .zslab import balanced_bounds

            costs = [_slab_cost(r, w) for r, w in timed]
            if max(costs) > 1.1 * min(costs):
                new = balanced_bounds(bounds, costs, min_planes=min(12, nz // parts))
                if new != bounds:
                    ent["bounds"] = new
                    ent["recuts"] += 1
    return out


def slab_count(nz: int) -> int:
    """How many slabs run_slabs cuts an nz-plane grid into."""
    n = len(devices())
    return 1 if n <= 1 or nz < 2 else min(n, nz)
