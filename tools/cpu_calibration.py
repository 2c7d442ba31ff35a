"""Calibrate the CPU baseline (oracle/cpu_ref.py) against the reference interpolator
(the restatement must be within +-15 % of the reference's time on C1 and C2).

Runs only where the read-only reference checkout exists (this container).  Both sides run the
same work on the same inputs, back to back:

* C1: 64^3 grid / 10k sphere-pack particles / IDW k = 8, one process: the reference
  ``interpolate_field`` (interpolator.py:126-155) vs ``cpu_ref.interp_grid``;
* C2: 256^3 / 1M / IDW k = 8 over z-slabs on a ProcessPoolExecutor of 8 workers (the
  interpolator.py:173-182 pattern): the reference per slab vs ``cpu_ref.interp_grid_parallel``.

Writes profiles/cpu_calibration_<tag>.json (bench.py attaches it to ``cpu_baseline``).
Usage: python tools/cpu_calibration.py [--tag r02] [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import platform
import sys
import time
import types
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
_REF = {}


def _ref_init(ref_path, P, Q, ax):
    import importlib.util

    sys.modules.setdefault("tifffile", types.ModuleType("tifffile"))
    spec = importlib.util.spec_from_file_location("ref_interpolator", os.path.join(ref_path, "interpolator.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    _REF.update(m=m, P=P, Q=Q, ax=ax)


def _ref_slab(z):
    import pandas as pd

    m, P, Q, ax = _REF["m"], _REF["P"], _REF["Q"], _REF["ax"]
    z0, z1 = z
    Z, Y, X = np.meshgrid(ax[z0:z1], ax, ax, indexing="ij")
    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
    with contextlib.redirect_stdout(io.StringIO()):
        U, V, W = m.interpolate_field(df, (X, Y, Z), method="idw", idw_neighbors=8, idw_power=2.0)
    return float(U.sum())


def _time_ref(ref_path, P, Q, ax, workers, slab):
    ranges = [(s, min(s + slab, len(ax))) for s in range(0, len(ax), slab)]
    if workers == 1:
        _ref_init(ref_path, P, Q, ax)  # module import outside the timed region
        t = time.perf_counter()
        for r in ranges:
            _ref_slab(r)
        return time.perf_counter() - t
    # worker start-up (imports) inside, as for the oracle's pool below
    t = time.perf_counter()
    with ProcessPoolExecutor(workers, initializer=_ref_init, initargs=(ref_path, P, Q, ax)) as ex:
        list(ex.map(_ref_slab, ranges))
    return time.perf_counter() - t


def _time_oracle(P, Q, ax, workers, slab):
    from oracle import cpu_ref

    t = time.perf_counter()
    if workers == 1:
        cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", 8, 2.0)
    else:
        cpu_ref.interp_grid_parallel(P, Q, ax, ax, ax, "idw", 8, 2.0, n_jobs=workers, slab=slab)
    return time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--tag", default="r02")
    a = ap.parse_args()
    from ptv_interpolation_amd import synth

    res = {}
    for name, G, n, workers, slab in (("C1", 64, 10_000, 1, 64), ("C2", 256, 1_000_000, 8, 8)):
        P, Q = synth.sphere_pack(n, G, values="normal")
        ax = np.linspace(0, G - 1, G)
        t_ref = _time_ref(a.ref, P, Q, ax, workers, slab)
        t_ora = _time_oracle(P, Q, ax, workers, slab)
        res[name] = {"grid": G, "particles": n, "workers": workers, "reference_s": round(t_ref, 3),
                     "oracle_s": round(t_ora, 3), "ratio": round(t_ora / t_ref, 3)}
        print(name, res[name], flush=True)
    ratios = {k: v["ratio"] for k, v in res.items()}
    out = {"what": "oracle/cpu_ref.py vs the reference interpolate_field, same inputs, same container, back to back",
           "host": platform.processor() or platform.machine(), "cpus": os.cpu_count(), "cases": res,
           "ratios": ratios, "within_15pct": all(0.85 <= r <= 1.15 for r in ratios.values())}
    path = os.path.join(ROOT, "profiles", f"cpu_calibration_{a.tag}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
