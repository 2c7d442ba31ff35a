"""Dev tool: headline (512^3 / 5M, IDW k = 8) bin / lattice / k-NN times under dev env knobs given
as NAME=VALUE[,NAME=VALUE] specs (read by the library per call), e.g. PTV_LAT_SEEDS=0.
usage: python tools/lattice_sweep.py '' PTV_LAT_SEEDS=0 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ptv_interpolation_amd import _lib, synth

P, Q = synth.sphere_pack(5_000_000, 512)
ax = np.linspace(0, 511, 512)
ctx = _lib.Context.get(0)
ref = None
for spec in sys.argv[1:]:
    env = dict(kv.split("=") for kv in spec.split(",") if kv)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    for it in range(3):
        U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=8)
    st = ctx.stats
    same = ref is None or all(np.array_equal(a, b) for a, b in zip((U, V, W), ref))
    if ref is None:
        ref = (U.copy(), V.copy(), W.copy())
    print(f"[{spec or 'default'}] bin {st['ms_bin']:.3f} lattice {st['ms_lattice']:.3f} knn {st['ms_knn']:.3f} ms "
          f"identical={same}", flush=True)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
