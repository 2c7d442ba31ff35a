"""Seeded synthetic sphere-pack particle sets (bench and test inputs).

Restates the geometry of the reference's ``generate_sphere_pack.py``:
six spheres of radius R=0.5 in a simple-hexagonal stack of two equilateral
triangles (generate_sphere_pack.py:8-32), a domain equal to the sphere-centre
bounding box grown by R+0.2 (:34-43), uniformly sampled particles with sphere
interiors rejected (:46-54, :95-97), and the reference flow field ``w = 1``,
``u = v = 0`` (:86-93).

Differences, all required by the measurement plan:

* exactly ``n`` particles are produced (rejection sampling is repeated until
  the count is reached) from ``numpy.random.default_rng(seed)``;
* coordinates are affinely mapped per axis to voxel units ``[0, G-1]`` so the
  grid ``create_grid(((0, G),)*3, G)`` has unit spacing;
* ``values="normal"`` draws iid N(0,1) u, v, w (parity runs) instead of the
  constant reference field (throughput runs).
"""
from __future__ import annotations

import math

import numpy as np

R = 0.5
_D = 2 * R
CENTERS = np.array(
    [
        (0.0, 0.0, 0.0),
        (_D, 0.0, 0.0),
        (_D / 2.0, math.sqrt(3.0) * _D / 2.0, 0.0),
        (0.0, 0.0, _D),
        (_D, 0.0, _D),
        (_D / 2.0, math.sqrt(3.0) * _D / 2.0, _D),
    ]
)
LO = CENTERS.min(axis=0) - R - 0.2
HI = CENTERS.max(axis=0) + R + 0.2

PARTICLE_SEED = 20260213
VALUE_SEED = 20260214


def inside_spheres(x, y, z) -> np.ndarray:
    """True where (x, y, z) (domain units) lies strictly inside any sphere."""
    m = np.zeros(np.broadcast(x, y, z).shape, dtype=bool)
    for cx, cy, cz in CENTERS:
        m |= ((x - cx) ** 2 + (y - cy) ** 2 + (z - cz) ** 2) < R * R
    return m


def sphere_pack(n: int, grid: int | tuple = 64, seed: int = PARTICLE_SEED,
                values: str = "reference", value_seed: int = VALUE_SEED, z_tiles: int = 1,
                z_tile: int = 0):
    """Return ``(points (n,3), vals (n,3))`` float64 in voxel units.

    ``grid`` is G (cube) or (gx, gy, gz).  ``z_tiles``/``z_tile`` place the
    pack copy ``z_tile`` of a stack of ``z_tiles`` copies along z (used by the
    weak-scaling multi-GPU bench: copy t occupies z in [t*gz, (t+1)*gz)).
    """
    gx, gy, gz = (grid, grid, grid) if isinstance(grid, int) else grid
    scale = np.array([gx - 1, gy - 1, gz - 1], dtype=np.float64) / (HI - LO)
    rng = np.random.default_rng([seed, z_tile])
    out = np.empty((0, 3))
    need = n
    chunks = []
    while need > 0:
        m = int(need / 0.7) + 1024
        p = rng.uniform(LO, HI, size=(m, 3))
        keep = ~inside_spheres(p[:, 0], p[:, 1], p[:, 2])
        p = p[keep][:need]
        chunks.append(p)
        need -= p.shape[0]
    out = np.concatenate(chunks)
    pts = (out - LO) * scale
    pts[:, 2] += z_tile * gz
    if values == "reference":
        vals = np.zeros((n, 3))
        vals[:, 2] = 1.0
    elif values == "normal":
        vals = np.random.default_rng([value_seed, z_tile]).standard_normal((n, 3))
    else:
        raise ValueError(values)
    return np.ascontiguousarray(pts), np.ascontiguousarray(vals)


def fluid_mask(grid: int | tuple) -> np.ndarray:
    """(gz, gy, gx) bool: True (fluid) where the voxel centre lies outside the spheres."""
    gx, gy, gz = (grid, grid, grid) if isinstance(grid, int) else grid
    ax = [LO[i] + np.arange(g) * (HI[i] - LO[i]) / (g - 1) for i, g in enumerate((gx, gy, gz))]
    # broadcast views (same elementwise arithmetic as a meshgrid, no 3 x 8 B/voxel temporaries)
    return ~inside_spheres(ax[0][None, None, :], ax[1][None, :, None], ax[2][:, None, None])


def fluid_mask_device(grid: int | tuple, z0: int, z1: int, device):
    """Planes [z0, z1) of ``fluid_mask(grid)`` as a torch uint8 (z1 - z0, gy, gx) tensor built
    on `device` (plane z is copy-local plane z % gz: stacked copies repeat the pack), with the
    same float64 arithmetic as ``fluid_mask`` (bit-identical; no (gz, gy, gx) float64 host
    temporaries, which reach 69 GB at 2048^3)."""
    import torch

    gx, gy, gz = (grid, grid, grid) if isinstance(grid, int) else grid
    f64 = dict(dtype=torch.float64, device=device)
    ax = [float(LO[i]) + (torch.arange(g, **f64) * float(HI[i] - LO[i])) / float(g - 1)
          for i, g in enumerate((gx, gy, gz))]
    x = ax[0][None, None, :]
    y = ax[1][None, :, None]
    z = ax[2][torch.arange(z0, z1, device=device) % gz][:, None, None]
    inside = torch.zeros((z1 - z0, gy, gx), dtype=torch.bool, device=device)
    for cx, cy, cz in CENTERS:
        inside |= ((x - float(cx)) ** 2 + (y - float(cy)) ** 2 + (z - float(cz)) ** 2) < R * R
    return (~inside).to(torch.uint8)
