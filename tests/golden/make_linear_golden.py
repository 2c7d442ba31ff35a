"""Generate the method='linear' parity fixtures by importing the reference interpolator.

The reference's default method, ``interpolate_field(..., method='linear')``, is
``griddata(points, values, grid_coords, method='linear', fill_value=0.0)``
(interpolator.py:196-197).  Runs only where the read-only reference checkout exists
(default ``/root/reference``); the GPU box only reads the committed ``linear_*.npz``.
Each fixture stores the inputs (particles, values, 1-D grid axes) and the reference
outputs ``U, V, W`` (C-order (nz, ny, nx) float64).

Cases: continuous random particles (general position: no voxel lies on a shared face, so
the result is unique and checked bit for bit) on grids reaching beyond the convex hull
(fill_value there), an anisotropic grid, the call without a ``method`` argument (the
default), and particles on a jittered lattice with duplicated positions (Qhull "coplanar"
points that are not vertices).

Usage:  python tests/golden/make_linear_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import _import_reference, _run, _save  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    ref = _import_reference(args.ref)
    rng = np.random.default_rng(20261017)

    # (1) general position, grid beyond the hull on every side
    P = rng.uniform(2.0, 21.0, (3000, 3)); Q = rng.standard_normal((3000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 24),) * 3, 24, method="linear")
    _save("linear_rand", points=P, values=Q, ax=x, ay=y, az=z, U=U, V=V, W=W)

    # (2) anisotropic grid (nx, ny, nz) = (30, 20, 12) over a slab-shaped particle cloud
    P = np.stack([rng.uniform(-1, 30, 4000), rng.uniform(0, 19, 4000), rng.uniform(1, 11, 4000)], -1)
    Q = rng.standard_normal((4000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 30), (0, 20), (0, 12)), (30, 20, 12), method="linear")
    _save("linear_aniso", points=P, values=Q, ax=x, ay=y, az=z, U=U, V=V, W=W)

    # (3) the reference default (no method argument: 'linear')
    P = rng.uniform(0, 15, (1500, 3)); Q = rng.standard_normal((1500, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 16),) * 3, 16)
    _save("linear_default", points=P, values=Q, ax=x, ay=y, az=z, U=U, V=V, W=W)

    # (4) a jittered 8^3 lattice plus 40 exact duplicates (coplanar points, not vertices)
    g = np.arange(8, dtype=float) * 2.0 + 1.0
    L = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    L = L + rng.uniform(-0.3, 0.3, L.shape)
    dup = L[rng.choice(len(L), 40, replace=False)]
    P = np.concatenate([L, dup]); Q = rng.standard_normal((len(P), 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 18),) * 3, 18, method="linear")
    _save("linear_dups", points=P, values=Q, ax=x, ay=y, az=z, U=U, V=V, W=W)


if __name__ == "__main__":
    main()
