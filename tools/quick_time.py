"""Quick timing of the headline config through the host C-ABI (dev tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from ptv_interpolation_amd import _lib, synth

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
occ = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
t = time.time(); P, Q = synth.sphere_pack(N, G); print("synth", time.time() - t, flush=True)
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
for it in range(3):
    t = time.time()
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k, cell_occupancy=occ)
    st = ctx.stats
    print(f"iter {it} wall {time.time()-t:.3f}s bin {st['ms_bin']:.2f} ms knn {st['ms_knn']:.2f} ms "
          f"h2d {st['ms_h2d']:.1f} d2h {st['ms_d2h']:.1f} cells {st['cells']} L {st['levels']} "
          f"Mvox/s(knn) {G**3/st['ms_knn']/1e3:.1f}", flush=True)
print("U stats", np.nanmin(U), np.nanmax(U), np.isnan(U).sum())
