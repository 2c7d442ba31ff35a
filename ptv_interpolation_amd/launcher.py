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
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib

_ctx_lock = threading.Lock()
_slab_ctx = {}
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


def run_slabs(nz: int, fn, out, results=None):
    """Fill the preallocated C-contiguous (nz, ...) arrays ``out`` slab by slab.

    ``fn(ctx, z0, z1, views)`` writes planes [z0, z1) into ``views`` (the z-slices of ``out``,
    contiguous, written in place by the library's D2H: no per-slab arrays and no host
    concatenation).  One slab per device of ``devices()``, one host thread each; a single
    device runs fn(ctx, 0, nz, out) directly.  Returns ``out``; fn's per-slab results are
    ``last_results`` of the calling thread (or appended to ``results`` when given)."""
    out = tuple(out)
    for a in out:
        if not (a.flags.c_contiguous and a.shape[0] == nz):
            raise ValueError("run_slabs: outputs must be C-contiguous with nz leading planes")
    devs = devices()
    if len(devs) <= 1 or nz < 2:
        res = [fn(_lib.Context.get(devs[0]), 0, nz, out)]
        _tls.results = res
        if results is not None:
            results.extend(res)
        return out
    slabs = slab_bounds(nz, len(devs))
    seen = {}
    jobs = []
    for d, (z0, z1) in zip(devs, slabs):
        slot = seen.get(d, 0)
        seen[d] = slot + 1
        jobs.append((context(d, slot), z0, z1, tuple(a[z0:z1] for a in out)))
    with ThreadPoolExecutor(len(jobs)) as ex:
        res = list(ex.map(lambda j: fn(*j), jobs))
    _tls.results = res
    if results is not None:
        results.extend(res)
    return out


def slab_count(nz: int) -> int:
    """How many slabs run_slabs cuts an nz-plane grid into."""
    n = len(devices())
    return 1 if n <= 1 or nz < 2 else min(n, nz)
