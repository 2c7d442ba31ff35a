"""Split lattice launch check (dev build, PTV_LIB=<a PTV_DEV_KNOBS build>): lattice bounds with and without the split
launch, and the per-column cull map's decisions.  usage: python tools/lattice_split_check.py"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lattice(G, N, k, split, out):
    code = f"""
import numpy as np, sys
sys.path.insert(0, {ROOT!r})
from ptv_interpolation_amd import _lib, synth
P, Q = synth.sphere_pack({N}, {G}, values="normal")
ax = np.linspace(0, {G} - 1, {G})
ctx = _lib.Context(0)
U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k={k})
np.save({out!r} + ".npy", U)
print("stats", ctx.stats["ms_lattice"], ctx.stats["ms_knn"])
"""
    env = dict(os.environ, PTV_LAT_SPLIT=str(split), PTV_DBG_LATDK=out + ".bin")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout.strip(), r.stderr.strip()[-2000:])
    with open(out + ".bin", "rb") as f:
        n = np.frombuffer(f.read(12), dtype=np.int32)
        dk = np.frombuffer(f.read(), dtype=np.float64).reshape(n[2], n[1], n[0])
    return dk, np.load(out + ".npy")


def main():
    os.makedirs("gpurun_out/dbg", exist_ok=True)
    for G, N, k in ((256, 1_000_000, 50), (256, 1_000_000, 8), (512, 5_000_000, 30)):
        d0, u0 = lattice(G, N, k, 0, f"gpurun_out/dbg/l{G}_{k}_s0")
        d1, u1 = lattice(G, N, k, 16, f"gpurun_out/dbg/l{G}_{k}_s16")
        diff = d0 != d1
        small = d1 < d0 * (1 - 1e-12)
        print(f"G={G} k={k}: lattice {d0.shape}, differ {diff.sum()}, split smaller {small.sum()}, "
              f"outputs differ {(u0 != u1).sum()}")
        idx = np.argwhere(diff)[:10]
        for z, y, x in idx:
            print("   ", (z, y, x), d0[z, y, x], d1[z, y, x])
    # cull map
    code = f"""
import numpy as np, sys
sys.path.insert(0, {ROOT!r})
from ptv_interpolation_amd import _lib, synth
G = 96
P, Q = synth.sphere_pack(150000, G, values="normal")
ax = np.linspace(0, G - 1, G)
ctx = _lib.Context(0)
for z0, z1 in ((0, 24), (24, 48)):
    for it in range(2):
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=8, z_range=(z0, z1), flags=_lib.FLAG_SLAB_CULL_AUTO)
        print("call", it, (z0, z1), "binned", ctx.stats["n_binned"])
"""
    env = dict(os.environ, PTV_DBG_CULL="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout.strip(), r.stderr.strip()[-3000:])


if __name__ == "__main__":
    main()
