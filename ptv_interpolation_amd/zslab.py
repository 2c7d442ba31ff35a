"""Multi-GPU z-slab partition of ONE grid with the particle set replicated (SURVEY.md §8(e),
BASELINE north_star; replaces the reference's process fan-out, interpolator.py:173-182).

One process per GPU.  Rank r of P computes planes ``slab_bounds(nz, P)[r]`` of the grid.
Every rank holds the whole particle set in HBM (replicated once with an RCCL all-gather or
broadcast, outside the timed step) and the library bins only the particles that can reach
its slab.  Default (bench.py, the drop-in launcher): the per-column cull map of
``PTV_FLAG_SLAB_CULL_AUTO``, which the library derives from the slab's own lattice bounds, caches
per context and proves exact on the device before every main launch.  The scalar
``ptv_knn_params.slab_halo`` path remains: on-device compaction to the particles within the halo
of the slab's z extent, then a proof from the coarse-lattice k-th distance bounds that no culled
particle can be among any slab voxel's k nearest; when it fails the call returns
``PTV_E_INEXACT`` with the halo it would have needed, and ``interp_slab`` retries with at least
1.25x the refused halo (the requirement is computed on a different particle set and lattice each
time, so it can grow over two or three retries) and, as a last resort, bins everything.  No
collective touches the interpolation itself; an all-gather reassembles the full field only when a
caller wants it on every device (``gather_field``).  ``balanced_bounds`` re-cuts the slabs from
measured step times (bench.py's warmup).

The functions take torch tensors / a ``torch.distributed`` module, so the same partition code
runs over RCCL on the GPUs (bench.py) and over gloo on the CPU (tests/test_distributed.py,
with an oracle-backed ``call``).
"""
from __future__ import annotations

import math

from . import _lib
from .launcher import slab_bounds

__all__ = ["rank_slab", "halo_slab", "replicate_columns", "broadcast_columns", "HaloState", "interp_slab",
           "halo_guess", "gather_field"]


def rank_slab(nz: int, world: int, rank: int):
    """[z0, z1) planes of rank `rank` (contiguous, as even as possible, in rank order)."""
    return slab_bounds(nz, world)[rank] if rank < min(world, nz) else (nz, nz)


def halo_slab(z0: int, z1: int, nz: int, planes: int = 1):
    """The slab grown by `planes` halo planes per interior side, clipped to the grid, and the
    (lo, hi) number of halo planes added (a stencil's one-plane halo, physics.py:6-53)."""
    a, b = max(0, z0 - planes), min(nz, z1 + planes)
    return a, b, z0 - a, b - z1


def replicate_columns(local, dist=None):
    """All-gather each rank's equal-length 1-D column tensors into the replicated columns
    (rank order).  ``local``: list of tensors; returns a list of tensors."""
    if dist is None or dist.get_world_size() == 1:
        return list(local)
    out = []
    for c in local:
        full = c.new_empty((dist.get_world_size() * c.numel(),))
        dist.all_gather_into_tensor(full, c.contiguous())
        out.append(full)
    return out


def broadcast_columns(cols, dist=None, src: int = 0):
    """Broadcast rank `src`'s column tensors in place (every rank allocated the same shapes)."""
    if dist is not None and dist.get_world_size() > 1:
        for c in cols:
            dist.broadcast(c, src)
    return cols


class HaloState:
    """The halo a rank uses for its slab cull; ``interp_slab`` widens it to the proven value."""

    def __init__(self, halo: float):
        self.halo = float(halo)
        self.retries = 0
        self.required = None

    def as_dict(self):
        return {"halo": self.halo, "required": self.required, "retries": self.retries}


def interp_slab(call, state: HaloState, max_tries: int = 4):
    """``call(halo) -> stats dict`` (a ``Context.interp_knn_dev`` bound to this rank's slab);
    on ``InexactError`` retry with the halo the library proved sufficient, at least 1.25x the one
    refused (the proof of a wider cull is computed on a different particle set and lattice, so its
    requirement can come out higher again: in sphere-pack voids the requirement grew over two or
    three retries by 1x steps), last resort 0 (every particle binned, nothing to prove)."""
    for _ in range(max_tries):
        try:
            st = call(state.halo)
            state.required = st.get("halo_required")
            return st
        except _lib.InexactError as e:
            state.retries += 1
            h = e.halo_required
            state.halo = (max(h * (1.0 + 1e-6), 1.25 * state.halo)
                          if (h is not None and math.isfinite(h) and h > 0) else 0.0)
            if state.halo == 0.0:
                break
    state.halo = 0.0
    st = call(0.0)
    state.required = None
    return st


def halo_guess(n_particles: int, extent, k: int, factor: float = 4.0) -> float:
    """First halo to try: `factor` x the radius of a ball holding k particles at the mean
    density over `extent` (x, y, z lengths)."""
    vol = 1.0
    for e in extent:
        vol *= max(float(e), 1e-300)
    r = (k * vol / (max(n_particles, 1) * 4.18879020478639)) ** (1.0 / 3.0)
    return factor * r


def gather_field(slab, dist=None, counts=None):
    """All-gather the ranks' (planes_r, ny, nx) slabs into the (sum planes_r, ny, nx) field on
    every rank (RCCL over xGMI on the GPUs): the reassembly step, never on the data path of the
    interpolation.  ``counts``: every rank's plane count in rank order (default: all equal to
    this slab's).  Unequal slabs are padded to the largest for one all_gather_into_tensor and
    the padding is dropped afterwards."""
    if dist is None or dist.get_world_size() == 1:
        return slab
    world = dist.get_world_size()
    counts = [slab.shape[0]] * world if counts is None else [int(c) for c in counts]
    if len(counts) != world or counts[dist.get_rank()] != slab.shape[0]:
        raise ValueError(f"gather_field: counts {counts} do not match world {world} / this slab {slab.shape[0]}")
    rest = tuple(slab.shape[1:])
    pmax = max(counts)
    if all(c == pmax for c in counts):
        full = slab.new_empty((world * pmax,) + rest)
        dist.all_gather_into_tensor(full, slab.contiguous())
        return full
    send = slab.new_zeros((pmax,) + rest)
    send[:slab.shape[0]] = slab
    padded = slab.new_empty((world * pmax,) + rest)
    dist.all_gather_into_tensor(padded, send)
    full = slab.new_empty((sum(counts),) + rest)
    off = 0
    for r, c in enumerate(counts):
        full[off:off + c] = padded[r * pmax:r * pmax + c]
        off += c
    return full


def balanced_bounds(bounds, times, min_planes: int = 12):
    """Re-cut a z-slab partition so that every rank gets the same share of the measured cost.

    ``bounds``: the current N + 1 plane boundaries (0 = b0 < b1 < ... < bN = nz); ``times``: each
    rank's measured step time on its slab.  The cost is modelled as uniform within each current
    slab (time / planes), the cumulative cost is cut at k / N of the total, and every slab keeps at
    least ``min_planes`` planes (the slab lattice needs >= 9; fewer would lose the cull proof).
    Repeated after each re-measure, the cut converges on slabs of varying cost density (the sphere
    pack's void planes cost more per plane than its packed ones)."""
    bounds = [int(b) for b in bounds]
    n = len(bounds) - 1
    nz = bounds[-1]
    if n <= 1 or len(times) != n:
        return bounds
    min_planes = max(1, min(int(min_planes), nz // n))
    dens = []
    for r in range(n):
        w = bounds[r + 1] - bounds[r]
        dens.append(max(float(times[r]), 0.0) / w if w > 0 else 0.0)
    cum = [0.0]
    for r in range(n):
        cum.append(cum[-1] + dens[r] * (bounds[r + 1] - bounds[r]))
    total = cum[-1]
    if not (total > 0.0):
        return bounds

    def plane_at(c):  # the (fractional) plane where the cumulative cost reaches c
        for r in range(n):
            if c <= cum[r + 1] or r == n - 1:
                d = dens[r]
                return bounds[r] + ((c - cum[r]) / d if d > 0 else 0.0)
        return float(nz)

    new = [0]
    for r in range(1, n):
        z = int(round(plane_at(total * r / n)))
        z = max(z, new[-1] + min_planes)
        z = min(z, nz - (n - r) * min_planes)
        new.append(z)
    new.append(nz)
    return new
