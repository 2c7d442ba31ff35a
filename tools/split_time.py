"""Time the k-NN kernel on fluid-only / solid-only voxels of the sphere pack (dev tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from ptv_interpolation_amd import _lib, synth

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
fl = synth.fluid_mask(G)
print("fluid fraction", fl.mean(), flush=True)
ctx = _lib.Context.get(0)
for name, m in (("all", None), ("fluid", fl), ("solid", ~fl)):
    for it in range(2):
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k, fluid_mask=m)
    st = ctx.stats
    print(f"{name:6s} lat {st['ms_lattice']:.2f} knn {st['ms_knn']:.2f} ms", flush=True)
