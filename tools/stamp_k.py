"""Per-wave phase stamps of the main k-NN launch for any k / method (dev tool; needs a library
built with -DPTV_STAMP_ALL=1 for KMAX != 8, e.g. PTV_LIB=ab/libptv_stamp.so).

usage: stamp_k.py G N k [idw|sibson|filter]   (filter: PTV_STAMP_LATTICE=4 is set here)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth

G, N, k = (int(v) for v in sys.argv[1:4])
method = sys.argv[4] if len(sys.argv) > 4 else "idw"
m = _lib.METHOD_IDW if method == "idw" else _lib.METHOD_SIBSON
if method == "filter":
    os.environ["PTV_STAMP_LATTICE"] = "4"
P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
for it in range(2):
    if it == 1:
        ctx.debug_stamps(1)
    if method == "filter":
        ctx.filter_outliers_knn(P, Q, k=k)
    else:
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=m, k=k)
st = ctx.stats
c = ctx.debug_stamps(2)
ctx.debug_stamps(0)
print(f"{method} k={k} G={G} N={N}: lat {st.get('ms_lattice', 0):.2f} knn {st.get('ms_knn', 0):.2f} ms, waves {c['waves']:.0f}")
print("   mean per wave:", {k2: round(v, 1) for k2, v in c["mean"].items()})
print("   max per wave: ", {k2: round(v, 1) for k2, v in c["max"].items()}, flush=True)
