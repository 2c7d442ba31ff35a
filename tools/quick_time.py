"""Quick timing of a sphere-pack config through the host C-ABI (dev tool).

usage: quick_time.py G N k [occupancy] [--counters]
"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from ptv_interpolation_amd import _lib, synth

args = [a for a in sys.argv[1:] if not a.startswith("--")]
G = int(args[0]) if len(args) > 0 else 512
N = int(args[1]) if len(args) > 1 else 5_000_000
k = int(args[2]) if len(args) > 2 else 8
occ = float(args[3]) if len(args) > 3 else 0.0
t = time.time(); P, Q = synth.sphere_pack(N, G); print("synth", round(time.time() - t, 3), flush=True)
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
for it in range(3):
    if "--stamps" in sys.argv and it == 2:
        ctx.debug_stamps(1)
    t = time.time()
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k, cell_occupancy=occ)
    st = ctx.stats
    print(f"iter {it} G {G} N {N} k {k} occ {occ} wall {time.time()-t:.3f}s bin {st['ms_bin']:.2f} ms lat {st['ms_lattice']:.2f} ms knn {st['ms_knn']:.2f} ms "
          f"cells {st['cells']} r0 {st['r0']:.2f} Mvox/s(knn) {G**3/st['ms_knn']/1e3:.1f}", flush=True)
if "--stamps" in sys.argv:
    c = ctx.debug_stamps(2); ctx.debug_stamps(0)
    print("waves recorded", int(c["waves"]))
    print("mean per wave:", {k2: round(v, 1) for k2, v in c["mean"].items()})
    print("max  per wave:", {k2: round(v, 1) for k2, v in c["max"].items()})
