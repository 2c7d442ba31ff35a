"""Multi-GPU z-slab launcher for the drop-in API (replaces the reference's
``ProcessPoolExecutor`` fan-out of interpolator.py:173-182 / test_parallel.py).

Every voxel depends only on the particle set and its own coordinate, and a z-slab call of
the kernels produces the same bits as the same planes of a whole-grid call, so the grid's
z planes are split into contiguous slabs, one per device, each device bins the full
(replicated) particle set and interpolates its slab, and the slabs land in disjoint
slices of the caller's output.  One host thread per device drives its own context and
stream (ctypes releases the GIL during the C calls); no collective touches the data path.

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


def run_slabs(nz: int, fn):
    """fn(ctx, z0, z1) -> tuple of (z1 - z0, ...) arrays; returns their z concatenation.

    One slab per device of ``devices()``; a single device runs fn(ctx, 0, nz) directly."""
    devs = devices()
    if len(devs) <= 1 or nz < 2:
        return fn(_lib.Context.get(devs[0]), 0, nz)
    slabs = slab_bounds(nz, len(devs))
    seen = {}
    jobs = []
    for d, (z0, z1) in zip(devs, slabs):
        slot = seen.get(d, 0)
        seen[d] = slot + 1
        jobs.append((context(d, slot), z0, z1))
    with ThreadPoolExecutor(len(jobs)) as ex:
        parts = list(ex.map(lambda j: fn(*j), jobs))
    return tuple(np.concatenate([p[c] for p in parts], axis=0) for c in range(len(parts[0])))
