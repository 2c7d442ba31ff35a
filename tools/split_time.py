"""Time the k-NN kernel on fluid-only / solid-only voxels of the sphere pack (dev tool).

usage: split_time.py G N k [--stamps]
"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from ptv_interpolation_amd import _lib, synth

args = [a for a in sys.argv[1:] if not a.startswith("--")]
G = int(args[0]) if len(args) > 0 else 512
N = int(args[1]) if len(args) > 1 else 5_000_000
k = int(args[2]) if len(args) > 2 else 8
P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
fl = synth.fluid_mask(G)
print("fluid fraction", fl.mean(), flush=True)
ctx = _lib.Context.get(0)
for name, m in (("all", None), ("fluid", fl), ("solid", ~fl)):
    for it in range(2):
        if "--stamps" in sys.argv and it == 1:
            ctx.debug_stamps(1)
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k, fluid_mask=m)
    st = ctx.stats
    print(f"{name:6s} lat {st['ms_lattice']:.2f} knn {st['ms_knn']:.2f} ms", flush=True)
    if "--stamps" in sys.argv:
        c = ctx.debug_stamps(2); ctx.debug_stamps(0)
        print("   mean per wave:", {k2: round(v, 1) for k2, v in c["mean"].items()}, flush=True)
