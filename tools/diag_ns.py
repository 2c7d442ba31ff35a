"""Null-space RBF diagnostic: the huge-smoothing case of test_extreme_pivots_take_the_ieee_path,
per-voxel errors against the oracle and the pivot statistics (dev tool; PTV_LIB selects the build)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cpu_ref  # noqa: E402
from ptv_interpolation_amd.rbf import LocalRBFInterpolator  # noqa: E402

rng = np.random.default_rng(61)
n, G = 3000, 10
P = rng.uniform(-0.5, G - 0.5, (n, 3))
Q = rng.standard_normal((n, 3))
ax = np.linspace(0.0, G - 1.0, G)
sm = np.zeros(len(P))
sm[::5] = float(sys.argv[1]) if len(sys.argv) > 1 else 2e307
it = LocalRBFInterpolator(P, Q, neighbors=20, smoothing=sm)
U, V, W = it.evaluate_grid(ax, ax, ax)
ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, 20, smoothing=sm)
err = np.abs(U - ref[0])
print("lib", os.environ.get("PTV_LIB", "default"), "smoothing", sm[0])
print("finite", np.isfinite(U).all(), "max err", float(np.nanmax(err)), "n bad(>1e-8)", int((err > 1e-8).sum()),
      "nan", int(np.isnan(U).sum()))
try:
    from ptv_interpolation_amd import _lib
    print("stats", _lib.Context.get(0).last_stats)
except Exception as e:  # noqa: BLE001
    print("stats unavailable", e)
bad = np.argwhere(err > 1e-8)[:8]
for b in bad:
    print(tuple(int(x) for x in b), float(U[tuple(b)]), float(ref[0][tuple(b)]))
