"""Where the end-to-end drop-in call spends its time (dev tool): interpolate_field on a host
DataFrame with dense create_grid meshgrids (as main.py:151 passes them) or zero-stride views,
second call profiled with cProfile.

usage: e2e_profile.py G N k [dense|views]
"""
import contextlib
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pandas as pd

from ptv_interpolation_amd import _lib, synth
from ptv_interpolation_amd import interpolator as ip

G, N, k = (int(v) for v in sys.argv[1:4])
dense = (sys.argv[4] if len(sys.argv) > 4 else "dense") == "dense"
P, Q = synth.sphere_pack(N, G)
df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
t = time.perf_counter()
grid, _ = ip.create_grid(((0, G), (0, G), (0, G)), G, dense=dense)
print(f"create_grid(dense={dense}) {time.perf_counter() - t:.3f} s", flush=True)
for it in range(3):
    t = time.perf_counter()
    if it == 2:
        pr = cProfile.Profile()
        pr.enable()
    with contextlib.redirect_stdout(io.StringIO()):
        U, V, W = ip.interpolate_field(df, grid, method="idw", idw_neighbors=k)
    if it == 2:
        pr.disable()
    wall = time.perf_counter() - t
    st = _lib.Context.get(0).stats
    print(f"call {it}: wall {wall:.3f} s  h2d {st['ms_h2d']:.1f} ms  device {st['ms_total'] - st['ms_h2d'] - st['ms_d2h']:.1f} ms"
          f"  d2h {st['ms_d2h']:.1f} ms", flush=True)
    del U, V, W
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
print(s.getvalue())
