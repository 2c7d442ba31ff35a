"""Dev tool: SHA-256 of the U, V, W planes of one 512^3 / 5M sphere-pack interpolation, for
bit-identity A/B of library builds (PTV_LIB selects the build).
usage: PTV_LIB=ab/libptv_base.so python tools/out_hash.py sibson 30   (or: filter 25)"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth

method, k = sys.argv[1], int(sys.argv[2])
P, Q = synth.sphere_pack(5_000_000, 512)
ax = np.linspace(0, 511, 512)
ctx = _lib.Context.get(0)
if method == "filter":
    U, V = ctx.filter_outliers_knn(P, Q, k=k, threshold=3.0)
    W = np.zeros(1)
else:
    m = {"idw": _lib.METHOD_IDW, "sibson": _lib.METHOD_SIBSON}[method]
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=m, k=k)
h = hashlib.sha256()
for a in (U, V, W):
    h.update(np.ascontiguousarray(a).tobytes())
print(f"{os.environ.get('PTV_LIB', 'in-tree')} {method} k={k}: sha256 {h.hexdigest()[:16]} "
      f"repaired tiles {ctx.stats['n_repair_tiles']}", flush=True)
