"""Per-wave stamps of the lattice-level k-distance launch (dev build, PTV_STAMP_LATTICE=1):
mean and max cycles per phase, candidates, passes.  usage: PTV_LIB=ab/<dev>.so PTV_STAMP_LATTICE=1
python tools/lattice_stamps.py [G N k]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ptv_interpolation_amd import _lib, synth  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
for z0, z1 in ((0, G), (G // 4, G // 4 + G // 8), (0, G // 8)):
    ctx.debug_stamps(1)
    ctx.interp_knn(P, Q, axes=(ax, ax, ax[z0:z1]), k=k)
    st = ctx.stats
    c = ctx.debug_stamps(2)
    ctx.debug_stamps(0)
    print(f"planes {z0}..{z1}: lattice {st['ms_lattice']:.3f} ms, knn {st['ms_knn']:.3f} ms, waves {c['waves']:.0f}")
    print("   mean:", {a: round(b, 1) for a, b in c["mean"].items()})
    print("   max: ", {a: round(b, 1) for a, b in c["max"].items()})
