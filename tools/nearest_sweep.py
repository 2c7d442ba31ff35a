"""Dev tool: nearest (k = 1) or IDW main-launch time at 512^3 / 5M vs the binning cell shape
(PTV_CELL_OCC particles per cube cell, PTV_CELL_XREF x-refinement; both read per call).
usage: python tools/nearest_sweep.py k occ:xref [occ:xref ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth

k = int(sys.argv[1])
P, Q = synth.sphere_pack(5_000_000, 512)
ax = np.linspace(0, 511, 512)
ctx = _lib.Context.get(0)
method = _lib.METHOD_NEAREST if k == 1 else _lib.METHOD_IDW
for spec in sys.argv[2:]:
    occ, xref = spec.split(":")
    os.environ["PTV_CELL_OCC"], os.environ["PTV_CELL_XREF"] = occ, xref
    for it in range(3):
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=method, k=k)
    st = ctx.stats
    print(f"k {k} occ {occ} xref {xref}: bin {st['ms_bin']:.3f} lattice {st['ms_lattice']:.3f} "
          f"knn {st['ms_knn']:.3f} ms cells {list(st['cells'])}", flush=True)
