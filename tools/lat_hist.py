"""Per-wave cost of the lattice-level k-NN launch against the tile's depth inside a sphere
(dev tool; needs a GPU).  usage: python tools/lat_hist.py [G N k]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

os.environ["PTV_STAMP_LATTICE"] = "1"
os.environ["PTV_NO_LAT_ORDER"] = "1"
os.environ["PTV_LAT_HEAVY"] = "0"
dump = "/tmp/ptv_stamps_raw_lat.bin"
os.environ["PTV_STAMPS_DUMP"] = dump
from ptv_interpolation_amd import _lib, synth

args = [a for a in sys.argv[1:] if not a.startswith("--")]
G = int(args[0]) if args else 512
N = int(args[1]) if len(args) > 1 else 5_000_000
k = int(args[2]) if len(args) > 2 else 8
P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context.get(0)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
ctx.debug_stamps(1)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
print("lattice ms", ctx.stats["ms_lattice"])
ctx.debug_stamps(2)
ctx.debug_stamps(0)
r = np.fromfile(dump, dtype=np.uint64).reshape(-1, 8)
n = (G - 1 + 3) // 4 + 1          # lattice points per axis
nt = (n + 3) // 4
ntxb = (nt + 3) // 4
nb = ntxb * nt * nt
bid = np.arange(r.shape[0]) // 4
wid = np.arange(r.shape[0]) % 4
q, rm = nb >> 3, nb & 7
x, i = bid & 7, bid >> 3
b = np.where(x < rm, x * (q + 1) + i, rm * (q + 1) + (x - rm) * q + i)
bx = b % ntxb
rr = b // ntxb
ty, tz = rr % nt, rr // nt
tx = bx * 4 + wid
ok = (tx < nt) & (bid < nb)
cyc = r[:, :6].sum(1).astype(np.float64)
cand = (r[:, 6] & 0xffffffff).astype(np.float64)
kept = (r[:, 7] >> 32).astype(np.float64)
# tile centre in voxel units -> sphere-pack units; depth inside the nearest sphere (>0 inside)
scale = (G - 1) / (synth.HI - synth.LO)
c = np.stack([(tx * 16 + 6.0), (ty * 16 + 6.0), (tz * 16 + 6.0)], 1) / scale + synth.LO
d = np.min(np.linalg.norm(c[:, None, :] - synth.CENTERS[None], axis=2), axis=1)
depth = (synth.R - d) * float(np.mean(scale))  # voxels (approx.)
tot = cyc[ok].sum()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/lat_hist.npz", cyc=cyc[ok], cand=cand[ok], kept=kept[ok], depth=depth[ok], tx=tx[ok], ty=ty[ok], tz=tz[ok])
print(f"waves {ok.sum()} mean cycles {cyc[ok].mean():.0f} max {cyc[ok].max():.0f}")
cs = np.sort(cyc[ok])[::-1]
for m in (1, 10, 100, 1000):
    print(f"  {m:5d}th slowest: {cs[m - 1]:.0f} cycles")
for lo, hi in ((-1e9, -10), (-10, 0), (0, 10), (10, 30), (30, 60), (60, 90), (90, 1e9)):
    s = ok & (depth >= lo) & (depth < hi)
    if s.any():
        print(f"depth [{lo:6.0f},{hi:6.0f}): waves {s.sum():6d} share {cyc[s].sum() / tot:.3f} mean {cyc[s].mean():9.0f} "
              f"max {cyc[s].max():9.0f} cand {cand[s].mean():8.0f} kept {kept[s].mean():7.0f}")
top = np.argsort(-np.where(ok, cyc, 0))[:10]
for t in top:
    print(f"  slow wave tile ({tx[t]},{ty[t]},{tz[t]}) depth {depth[t]:6.1f} cycles {cyc[t]:.0f} cand {cand[t]:.0f} kept {kept[t]:.0f}")
