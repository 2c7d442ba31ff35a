"""The shipped N > 1 step at benchmark size, rehearsed share by share on one GPU (SURVEY.md §8(e);
bench.py's strong-scaling step; the reference's split, interpolator.py:126-155, 173-182).

bench.py's rank r of N runs ``interp_knn_dev(..., flags=FLAG_SLAB_CULL_AUTO, z_range=slab)`` on
the replicated device-resident particle set with slab bounds re-cut from measured step times.
Here every share of the committed 8-way cut of the 512^3 / 5M headline is run on its own fresh
context: one cold call (no cached cull map: every particle binned, the map built from the slab's
own lattice) and two warm calls (the map reused, the cull proven on the device before the gated
main launch).  Every call's planes must equal the whole-grid call's bit for bit; a voxel may differ
only where value-heterogeneous ties sit among its k nearest (another cell grid may order equal
distances differently; tests/_util.hetero_ties_points), and those are checked to be exactly that.
Each share's cold and warm step times are printed as ``SHARE {json}`` lines.
"""
import json
import time

import numpy as np
import pytest

from tests._util import hetero_ties_points

pytestmark = pytest.mark.gpu

G, N = 512, 5_000_000
CUT = [0, 79, 139, 186, 257, 327, 372, 432, 512]  # bench.py's balanced 8-way cut (profiles/r05e_balance)
WARM_BINNED_MAX = 1_200_000


@pytest.fixture(scope="module")
def pack():
    import torch

    from ptv_interpolation_amd import _lib, synth

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    P, Q = synth.sphere_pack(N, G)
    cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).cuda() for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).cuda() for i in range(3)]
    ax = torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda")
    return {"P": P, "Q": Q, "cols": cols, "ax": ax, "whole": {}}


def _whole(pack, k):
    import torch

    from ptv_interpolation_amd import _lib

    if k not in pack["whole"]:
        pack["whole"].clear()  # one k at a time (3.2 GB each)
        ctx = _lib.Context(0)
        out = [torch.empty((G, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
        ctx.interp_knn_dev(N, [c.data_ptr() for c in pack["cols"]], G, G, G, axes_ptrs=[pack["ax"].data_ptr()] * 3,
                           out_ptrs=[o.data_ptr() for o in out], k=k)
        torch.cuda.synchronize()
        assert ctx.last_stats()["n_binned"] == N
        ctx.close()
        pack["whole"][k] = out
    return pack["whole"][k]


def _mismatch(out, ref):
    """Flat indices (within the slab) where any component differs (NaNs equal)."""
    import torch

    bad = None
    for a, b in zip(out, ref):
        d = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
        bad = d if bad is None else (bad | d)
    return torch.nonzero(bad.reshape(-1)).reshape(-1).cpu().numpy()


def _check_share(pack, k, rank, calls=3):
    import torch

    from ptv_interpolation_amd import _lib

    whole = _whole(pack, k)
    z0, z1 = CUT[rank], CUT[rank + 1]
    ref = [w[z0:z1] for w in whole]
    ctx = _lib.Context(0)  # fresh: no cached cull map
    out = [torch.empty((z1 - z0, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
    rec = []
    try:
        for call in range(calls):
            for o in out:
                o.fill_(-7.0)  # a call that skipped its outputs must not pass on the previous call's
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.interp_knn_dev(N, [c.data_ptr() for c in pack["cols"]], G, G, G,
                               axes_ptrs=[pack["ax"].data_ptr()] * 3, out_ptrs=[o.data_ptr() for o in out], k=k,
                               flags=_lib.FLAG_SLAB_CULL_AUTO, z_range=(z0, z1))
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            st = ctx.last_stats()
            dev = st["ms_bin"] + st["ms_cull"] + st["ms_lattice"] + st["ms_knn"]
            bad = _mismatch(out, ref)
            het_frac = 0.0
            if len(bad):
                iz, iy, ix = np.unravel_index(bad, (z1 - z0, G, G))
                q = np.stack([ix, iy, iz + z0], -1).astype(np.float64)
                _, het = hetero_ties_points(pack["P"], pack["Q"], q, k)
                assert het.all(), f"share {rank} call {call}: {int((~het).sum())} differing voxels are not ties"
                het_frac = len(bad) / ((z1 - z0) * G * G)
            rec.append({"call": "cold" if call == 0 else "warm", "wall_ms": round(wall, 3),
                        "device_ms": round(dev, 3), "bin": round(st["ms_bin"], 3), "cull": round(st["ms_cull"], 3),
                        "lattice": round(st["ms_lattice"], 3), "knn": round(st["ms_knn"], 3),
                        "n_binned": int(st["n_binned"]), "hetero_tie_voxels": int(len(bad)),
                        "hetero_tie_frac": het_frac})
    finally:
        ctx.close()
    print("SHARE " + json.dumps({"k": k, "rank": rank, "world": 8, "planes": [z0, z1], "calls": rec}))
    assert rec[0]["n_binned"] == N  # cold: no map yet, every particle binned
    for r in rec[1:]:
        assert r["n_binned"] <= WARM_BINNED_MAX, r
    return rec


@pytest.mark.timeout(900)
def test_balanced_shares_k8_bit_identical(pack):
    """All eight shares of the balanced cut, IDW k = 8 (the headline): cold + two warm calls each."""
    worst = {"cold": 0.0, "warm": 0.0}
    for r in range(8):
        rec = _check_share(pack, 8, r)
        worst["cold"] = max(worst["cold"], rec[0]["device_ms"])
        worst["warm"] = max(worst["warm"], min(x["device_ms"] for x in rec[1:]))
    print("SHARE " + json.dumps({"k": 8, "worst_device_ms": worst}))


@pytest.mark.timeout(900)
def test_balanced_shares_k50_bit_identical(pack):
    """Two shares of the balanced cut at IDW k = 50 (the reference default k; packed-key lists)."""
    for r in (2, 5):
        _check_share(pack, 50, r)
