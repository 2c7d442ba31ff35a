"""Per-wave cost distribution of the k-NN kernel (dev tool): which tiles dominate.

usage: python tools/stamp_hist.py [G N k]   (needs a GPU; writes gpurun_out/stamps_raw.npy)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth

args = [a for a in sys.argv[1:] if not a.startswith("--")]
G = int(args[0]) if len(args) > 0 else 512
N = int(args[1]) if len(args) > 1 else 5_000_000
k = int(args[2]) if len(args) > 2 else 8
os.makedirs("gpurun_out", exist_ok=True)
dump = "/tmp/ptv_stamps_raw.bin"
os.environ["PTV_STAMPS_DUMP"] = dump
P, Q = synth.sphere_pack(N, G)
ax = np.linspace(0, G - 1, G)
fl = synth.fluid_mask(G)
ctx = _lib.Context.get(0)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
ctx.debug_stamps(1)
ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
print("knn ms", ctx.stats["ms_knn"])
ctx.debug_stamps(2)
ctx.debug_stamps(0)
r = np.fromfile(dump, dtype=np.uint64).reshape(-1, 8)
nt = G // 4
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
# fluid fraction per tile
ff = fl.reshape(nt, 4, nt, 4, nt, 4).mean(axis=(1, 3, 5))  # [tz, ty, tx]
f = np.zeros(r.shape[0])
f[ok] = ff[tz[ok], ty[ok], tx[ok]]
cand = (r[:, 6] & 0xffffffff).astype(np.float64)
rounds = (r[:, 7] & 0xffff).astype(np.float64)
tot = cyc[ok].sum()
print(f"waves {ok.sum()}  mean cycles {cyc[ok].mean():.0f}")
for name, sel in (("fluid (f=1)", ok & (f == 1)), ("mixed", ok & (f > 0) & (f < 1)), ("solid (f=0)", ok & (f == 0))):
    print(f"{name:12s} waves {sel.sum():8d} ({sel.sum() / ok.sum():.3f})  cycles share {cyc[sel].sum() / tot:.3f}  "
          f"mean {cyc[sel].mean():8.0f}  cand {cand[sel].mean():7.1f}  rounds {rounds[sel].mean():5.2f}")
c = np.sort(cyc[ok])[::-1]
cs = np.cumsum(c) / tot
for frac in (0.001, 0.01, 0.05, 0.1, 0.25):
    n = int(frac * len(c))
    print(f"top {frac * 100:5.1f}% waves: {cs[n - 1]:.3f} of cycles (threshold {c[n - 1]:.0f})")
# solid tiles: cycles vs distance into the void (from the lattice k-distance proxy: candidates)
sol = ok & (f == 0)
for lo, hi in ((0, 200), (200, 500), (500, 1000), (1000, 3000), (3000, 1e9)):
    s = sol & (cand >= lo) & (cand < hi)
    print(f"solid cand [{lo},{hi}): waves {s.sum():7d} share {cyc[s].sum() / tot:.3f} mean cyc {cyc[s].mean() if s.any() else 0:.0f}")
