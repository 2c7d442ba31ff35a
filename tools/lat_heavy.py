"""Which lattice tiles are slow (dev build, no split, XCD order): per-tile stamp cycles of the
finest lattice level's k-distance launch against the tile's bounds.  usage (GPU, dev build):
PTV_LIB=abx/libptv_dbg.so python tools/lat_heavy.py [G N k]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
os.environ.update(PTV_LAT_SPLIT="0", PTV_NO_LAT_ORDER="1", PTV_STAMP_LATTICE="1",
                  PTV_STAMPS_DUMP="/tmp/stamps.bin", PTV_DBG_LATDK="/tmp/latdk.bin")
from ptv_interpolation_amd import _lib, synth  # noqa: E402

P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
ctx.debug_stamps(1)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
print("lattice ms", ctx.stats["ms_lattice"])
ctx.debug_stamps(2)
rec = np.fromfile("/tmp/stamps.bin", dtype=np.uint64).reshape(-1, 8)
with open("/tmp/latdk.bin", "rb") as f:
    n = np.frombuffer(f.read(12), dtype=np.int32)
    dk = np.frombuffer(f.read(), dtype=np.float64).reshape(n[2], n[1], n[0])
nx, ny, nz = int(n[0]), int(n[1]), int(n[2])
ntx, nty, ntz = (nx + 3) // 4, (ny + 3) // 4, (nz + 3) // 4
ntxb = (ntx + 3) // 4
nb = ntxb * nty * ntz


def xcd_block(b):
    q, r = nb >> 3, nb & 7
    x, i = b & 7, b >> 3
    return x * (q + 1) + i if x < r else r * (q + 1) + (x - r) * q + i


cyc = rec[:, :6].sum(1).astype(np.float64)
cand = (rec[:, 6] & 0xffffffff).astype(np.int64)
passes = ((rec[:, 7] >> 16) & 0xffff).astype(np.int64)
live = np.nonzero(cyc > 0)[0]
tmaxD = {}
for t in range(ntx * nty * ntz):
    tx, r = t % ntx, t // ntx
    ty, tz = r % nty, r // nty
    blk = dk[tz * 4:tz * 4 + 4, ty * 4:ty * 4 + 4, tx * 4:tx * 4 + 4]
    tmaxD[(tx, ty, tz)] = float(blk.max())
allD = np.array(sorted(tmaxD.values(), reverse=True))
order = np.argsort(-cyc[live])
print(f"tiles {ntx}x{nty}x{ntz}, waves recorded {len(live)}, mean cycles {cyc[live].mean():.0f}")
for i in order[:25]:
    gw = live[i]
    lb, wid = gw // 4, gw % 4
    b = xcd_block(lb)
    bx, rr = b % ntxb, b // ntxb
    ty, tz = rr % nty, rr // nty
    tx = bx * 4 + wid
    D = tmaxD.get((tx, ty, tz), -1)
    rank = int((allD > D).sum())
    c = (np.array([tx, ty, tz]) * 16 + 6) * (G - 1) / (4 * (nx - 1)) if nx > 1 else 0
    print(f"cycles {cyc[gw]:10.0f} cand {cand[gw]:7d} passes {passes[gw]} tile {(tx, ty, tz)} voxel~{np.round(c).astype(int)} "
          f"maxD {D:7.2f} rank by D {rank}")

# where the slow tiles' blocks sit in the longest-first order (the order dumped by a second run)
os.environ.pop("PTV_NO_LAT_ORDER")
os.environ["PTV_DBG_ORDER"] = "/tmp/order.bin"
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
with open("/tmp/order.bin", "rb") as f:
    cn = np.frombuffer(f.read(12), dtype=np.int32)
    cd = np.frombuffer(f.read(8 * int(np.prod(cn))), dtype=np.float64).reshape(cn[2], cn[1], cn[0])
    od = np.frombuffer(f.read(), dtype=np.int32)
pos = np.empty(nb, dtype=np.int64)
pos[od] = np.arange(nb)
print("coarse bounds: max", cd.max(), "min", cd.min(), "blocks", nb)
for i in order[:12]:
    gw = live[i]
    lb, wid = gw // 4, gw % 4
    b = xcd_block(lb)
    bx, rr = b % ntxb, b // ntxb
    ty, tz = rr % nty, rr // nty
    key = cd[tz:tz + 2, ty:ty + 2, 4 * bx:4 * bx + 5].max()
    print(f"slow tile block {b}: position in order {pos[b]}, coarse key {key:.2f}")
top = od[:10]
print("first blocks of the order and their keys:", [(int(b), round(float(cd[(b // ntxb) // nty:(b // ntxb) // nty + 2, (b // ntxb) % nty:(b // ntxb) % nty + 2, 4 * (b % ntxb):4 * (b % ntxb) + 5].max()), 2)) for b in top])
