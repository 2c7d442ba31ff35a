"""Phase cycles of the null-space local-RBF kernel k_rbf_ns (dev tool; needs a PTV_NS_STAMP build:
PTV_EXTRA_FLAGS=-DPTV_NS_STAMP=1 PTV_BUILD_TAG=nsst python -m ptv_interpolation_amd.build, then
PTV_LIB=ab/libptv_nsst.so python tools/ns_stamps.py [G N k ...]).  Prints mean cycles per wave."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth
from ptv_interpolation_amd.rbf import LocalRBFInterpolator

args = [a for a in sys.argv[1:]]
G = int(args[0]) if args else 256
N = int(args[1]) if len(args) > 1 else 5_000_000 * 256 ** 3 // 512 ** 3
ks = [int(a) for a in args[2:]] or [20, 32]
names = ("gather+sort", "qr(P)", "build phi", "readback+Y", "rank-2r", "lu", "backsub+e", "eval")
P, Q = synth.sphere_pack(N, G, values="normal")
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
dump = "/tmp/ptv_ns_stamps.bin"
os.environ["PTV_STAMPS_DUMP"] = dump
for k in ks:
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel="thin_plate_spline")
    it.evaluate_grid(ax, ax, ax)
    ctx.debug_stamps(1)
    it.evaluate_grid(ax, ax, ax)
    print(f"k={k}: solve {ctx.stats['ms_solve']:.1f} ms, knn {ctx.stats['ms_knn']:.1f} ms")
    ctx.debug_stamps(2)
    ctx.debug_stamps(0)
    r = np.fromfile(dump, dtype=np.uint64).reshape(-1, 8).astype(np.float64)
    r = r[r.sum(axis=1) > 0]
    tot = r.sum(axis=1).mean()
    print(f"  waves {len(r)}, mean cycles per wave {tot:.0f}")
    for i, nme in enumerate(names):
        print(f"  {nme:12s} {r[:, i].mean():9.0f}  ({r[:, i].mean() / tot:.1%})")
