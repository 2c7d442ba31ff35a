"""Dev tool: outlier-filter (k = 25) search time at 5M sphere-pack particles vs the binning cell
shape (PTV_CELL_OCC particles per cube cell, PTV_CELL_XREF x-refinement; both read per call) and
the first search radius scale (PTV_R0_SCALE when the library reads it).
usage: python tools/filter_sweep.py occ:xref [occ:xref ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth

P, _ = synth.sphere_pack(5_000_000, 512)
Q = np.random.default_rng(1).standard_normal((len(P), 3))
ctx = _lib.Context.get(0)
for spec in sys.argv[1:]:
    occ, xref = spec.split(":")
    os.environ["PTV_CELL_OCC"], os.environ["PTV_CELL_XREF"] = occ, xref
    for it in range(3):
        keep, kth = ctx.filter_outliers_knn(P, Q, k=25, threshold=3.0)
    st = ctx.stats
    print(f"filter occ {occ} xref {xref}: bin {st['ms_bin']:.3f} knn {st['ms_knn']:.3f} ms cells {list(st['cells'])} "
          f"kept {int(keep.sum())}", flush=True)
