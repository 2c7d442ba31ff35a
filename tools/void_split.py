"""Dev tool: bin / lattice / k-NN times of the headline shape on a sphere pack (voids) and on a
uniform cloud of the same particle density in the fluid (no voids), device-resident, to see
what the voids cost each phase.  usage: void_split.py [G] [N] [k]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ptv_interpolation_amd import _lib, synth  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
ctx = _lib.Context.get(0)
ax = torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda")
out = [torch.empty((G, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
P, Q = synth.sphere_pack(N, G)
fl = float(synth.fluid_mask(min(G, 256)).mean())
rng = np.random.default_rng(3)
Pu = rng.uniform(-0.5, G - 0.5, (int(N / fl), 3))
occs = [float(x) for x in os.environ.get("OCCS", "0").split(",")]
xrefs = [float(x) for x in os.environ.get("XREFS", "1").split(",")]
for occ, xref, (name, PP) in [(o, x, c) for o in occs for x in xrefs for c in (("spherepack", P),)]:
    if occ > 0:
        os.environ["PTV_CELL_OCC"] = str(occ)
    os.environ["PTV_CELL_XREF"] = str(xref)
    cols = [torch.from_numpy(np.ascontiguousarray(PP[:, i])).cuda() for i in range(3)] + \
           [torch.ones(len(PP), dtype=torch.float64, device="cuda") for _ in range(3)]
    acc = []
    for it in range(6):
        ctx.interp_knn_dev(len(PP), [c.data_ptr() for c in cols], G, G, G, axes_ptrs=[ax.data_ptr()] * 3,
                           out_ptrs=[o.data_ptr() for o in out], k=k)
        st = ctx.last_stats()
        if it >= 2:
            acc.append((st["ms_bin"], st["ms_lattice"], st["ms_knn"]))
    b, l, kk = np.mean(acc, axis=0)
    print(f"occ {occ} xref {xref} {name:11s} n {len(PP)} bin {b:.3f} lattice {l:.3f} knn {kk:.3f} ms  cells {st['cells']}", flush=True)
