"""Debug helper: the C5 rank-share pattern (f32 k-NN slab with one halo plane per side, then
the f32 divergence of the slab) at a reduced size, on the context's own stream and on torch's
stream, compared with the oracle divergence of the GPU field.  Prints what differs."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import cpu_ref  # noqa: E402
from ptv_interpolation_amd import _lib, synth, zslab  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
ctx = _lib.Context.get(0)
P, Q = synth.sphere_pack(n, G, values="normal")
cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).cuda() for i in range(3)] + \
       [torch.from_numpy(np.ascontiguousarray(Q[:, i])).cuda() for i in range(3)]
ax = torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda")
z0, z1 = zslab.rank_slab(G, 8, 3)
za, zb, hlo, hhi = zslab.halo_slab(z0, z1, G, 1)
for use_torch_stream in (False, True):
    stream = torch.cuda.current_stream().cuda_stream if use_torch_stream else 0
    out = [torch.empty((zb - za, G, G), dtype=torch.float32, device="cuda") for _ in range(3)]
    ctx.interp_knn_dev(n, [c.data_ptr() for c in cols], G, G, G, axes_ptrs=[ax.data_ptr()] * 3,
                       out_ptrs=[o.data_ptr() for o in out], k=8, flags=_lib.FLAG_OUT_F32, z_range=(za, zb),
                       stream=stream)
    mask = synth.fluid_mask_device(G, za, zb, torch.device("cuda", 0))
    torch.cuda.synchronize()
    div = torch.full((z1 - z0, G, G), 12345.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    st = ctx.divergence_dev(G, G, zb - za, [o.data_ptr() for o in out], mask.data_ptr(), div.data_ptr(), 1.0, 1.0,
                            1.0, field_dtype=_lib.F32, result_dtype=_lib.F32, z_range=(hlo, hlo + (z1 - z0)),
                            edges=(hlo == 0, hhi == 0), stream=stream)
    torch.cuda.synchronize()
    print("stream", "torch" if use_torch_stream else "ctx", "stats", {k: st[k] for k in ("n_voxels",)},
          "untouched", int((div == 12345.0).sum().item()), "of", div.numel(), flush=True)
    for p in (0, (z1 - z0) // 2, z1 - z0 - 1):
        b = hlo + p
        blk = [o[b - 1:b + 2].cpu().numpy() for o in out]
        mk = mask[b - 1:b + 2].cpu().numpy().view(bool)
        exp = cpu_ref.consistent_divergence(blk[0], blk[1], blk[2], mk, 1.0, 1.0, 1.0)[1]
        got = div[p].cpu().numpy()
        bad = ~((got == exp) | (np.isnan(got) & np.isnan(exp)))
        print(f"  plane {p}: mismatches {int(bad.sum())} / {bad.size}", flush=True)
        if bad.any():
            i = np.argwhere(bad)[:5]
            for yy, xx in i:
                print("    at", yy, xx, "got", got[yy, xx], "exp", exp[yy, xx])
