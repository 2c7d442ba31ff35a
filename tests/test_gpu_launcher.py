"""Multi-device z-slab launcher of the drop-in API (ptv_interpolation_amd/launcher.py,
SURVEY §8(e)): slabs on several contexts reproduce the single-call result bit for bit.
On a one-GPU box the devices are repeated (PTV_DEVICES=0,0,0: three contexts, three
streams, three host threads on the same GPU)."""
import contextlib
import io

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def _df(P, Q):
    return pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})


@pytest.mark.parametrize("method,kw", [("idw", {"idw_neighbors": 8}), ("idw", {"idw_neighbors": 50}),
                                       ("sibson", {"sibson_neighbors": 30}), ("nearest", {}),
                                       ("rbf", {"rbf_neighbors": 20})])
def test_slabs_on_three_contexts_equal_one_call(monkeypatch, method, kw):
    from ptv_interpolation_amd import interpolator as ip
    from ptv_interpolation_amd import synth

    G = 40 if method == "rbf" else 64
    P, Q = synth.sphere_pack(20000 if method != "rbf" else 6000, G, values="normal")
    (X, Y, Z), _ = ip.create_grid(((0, G),) * 3, (G, G, 37))  # 37 planes: uneven slabs
    with contextlib.redirect_stdout(io.StringIO()):
        monkeypatch.setenv("PTV_DEVICE", "0")
        one = ip.interpolate_field(_df(P, Q), (X, Y, Z), method=method, **kw)
        monkeypatch.delenv("PTV_DEVICE")
        monkeypatch.setenv("PTV_DEVICES", "0,0,0")
        three = ip.interpolate_field(_df(P, Q), (X, Y, Z), method=method, **kw)
    for a, b in zip(three, one):
        assert a.shape == X.shape and np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("method,kw", [("idw", {"idw_neighbors": 50}), ("idw", {"idw_neighbors": 8}),
                                       ("sibson", {"sibson_neighbors": 30})])
def test_slabs_cull_their_particles(monkeypatch, method, kw):
    """The drop-in multi-device path (main.py:184-192 -> interpolate_field -> launcher.run_slabs)
    culls each slab's particles with the per-column map of PTV_FLAG_SLAB_CULL_AUTO: the first call
    of each slab context bins every particle and builds the map from the slab's lattice bounds; the
    repeated call bins fewer than N per slab (the cull proven exact on the device) and both
    reproduce the one-call result bit for bit.  PTV_DEVICES=0,0,0,0: four slabs on four contexts."""
    from ptv_interpolation_amd import interpolator as ip
    from ptv_interpolation_amd import launcher, synth

    G = 96
    N = 150_000
    P, Q = synth.sphere_pack(N, G, values="normal")
    (X, Y, Z), _ = ip.create_grid(((0, G),) * 3, G)
    with contextlib.redirect_stdout(io.StringIO()):
        monkeypatch.setenv("PTV_DEVICE", "0")
        one = ip.interpolate_field(_df(P, Q), (X, Y, Z), method=method, **kw)
        assert launcher.last_results[0]["n_binned"] == N
        monkeypatch.delenv("PTV_DEVICE")
        monkeypatch.setenv("PTV_DEVICES", "0,0,0,0")
        first = ip.interpolate_field(_df(P, Q), (X, Y, Z), method=method, **kw)
        binned_first = [st["n_binned"] for st in launcher.last_results]
        again = ip.interpolate_field(_df(P, Q), (X, Y, Z), method=method, **kw)
        binned = [st["n_binned"] for st in launcher.last_results]
    print(f"{method} {kw}: particles binned per slab {binned_first} (first call), {binned} (again) of {N}")
    assert len(binned) == 4 and all(b < N for b in binned)
    for a, b, c in zip(first, again, one):
        assert np.array_equal(a, c, equal_nan=True) and np.array_equal(b, c, equal_nan=True)


def test_slab_cull_map_refreshes_when_particles_change(monkeypatch):
    """The cull map is cached per context and keyed by the particle set (arrays, n, a fingerprint):
    a call with different particles of the same count through the same host-path buffers does not
    reuse a stale map (or, if the fingerprint missed the change, its proof fails and the call reruns
    unculled), so the result stays bit-identical to the one-call result."""
    from ptv_interpolation_amd import interpolator as ip
    from ptv_interpolation_amd import synth

    G = 96
    N = 150_000
    P, Q = synth.sphere_pack(N, G, values="normal")
    P2 = P.copy()
    P2[:, 2] = (G - 1) - P2[:, 2]  # the same count, mirrored in z
    (X, Y, Z), _ = ip.create_grid(((0, G),) * 3, G)
    with contextlib.redirect_stdout(io.StringIO()):
        monkeypatch.setenv("PTV_DEVICE", "0")
        one = ip.interpolate_field(_df(P2, Q), (X, Y, Z), method="idw", idw_neighbors=8)
        monkeypatch.delenv("PTV_DEVICE")
        monkeypatch.setenv("PTV_DEVICES", "0,0,0")
        ip.interpolate_field(_df(P, Q), (X, Y, Z), method="idw", idw_neighbors=8)
        ip.interpolate_field(_df(P, Q), (X, Y, Z), method="idw", idw_neighbors=8)
        three = ip.interpolate_field(_df(P2, Q), (X, Y, Z), method="idw", idw_neighbors=8)
        # the same fingerprint (the 16 sampled particles kept) over changed data: the proof fails
        # and the call reruns with every particle binned
        P3 = P2.copy()
        keep = np.array([int(j * (N - 1) / 15) for j in range(16)])
        moved = np.setdiff1d(np.arange(N), keep)
        P3[moved, 2] = (G - 1) - P3[moved, 2]
        monkeypatch.setenv("PTV_DEVICE", "0")
        one3 = ip.interpolate_field(_df(P3, Q), (X, Y, Z), method="idw", idw_neighbors=8)
        monkeypatch.delenv("PTV_DEVICE")
        three3 = ip.interpolate_field(_df(P3, Q), (X, Y, Z), method="idw", idw_neighbors=8)
    for a, b in zip(three, one):
        assert np.array_equal(a, b, equal_nan=True)
    for a, b in zip(three3, one3):
        assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("change", ["shift", "scale"])
def test_slab_cull_map_keyed_by_axis_values(change):
    """The cull map's cache key holds the axis values, not only their pointers: the same particles,
    the same grid shape and the same axis buffers refilled in place with other coordinates (a
    recycled allocation) must not reuse the map built for the old lattice positions.  Three slabs,
    each a cold and a warm call on the old axes, then a call on the new ones; every slab equals the
    whole-grid call on the same axes bit for bit."""
    import torch

    from ptv_interpolation_amd import _lib, synth

    G, N = 96, 150_000
    P, Q = synth.sphere_pack(N, G, values="normal")
    cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).cuda() for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).cuda() for i in range(3)]
    ptrs = [c.data_ptr() for c in cols]
    axes = [torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda") for _ in range(3)]
    aptrs = [a.data_ptr() for a in axes]
    new = [a * 0.8 + 9.5 if change == "shift" else a * 0.55 for a in axes]

    def whole():
        ctx = _lib.Context(0)
        out = [torch.empty((G, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
        ctx.interp_knn_dev(N, ptrs, G, G, G, axes_ptrs=aptrs, out_ptrs=[o.data_ptr() for o in out], k=8)
        torch.cuda.synchronize()
        ctx.close()
        return out

    ref_old = whole()
    slabs = [(0, 30), (30, 61), (61, G)]
    ctxs = [_lib.Context(0) for _ in slabs]
    binned = []
    try:
        for phase in ("cold", "warm", "new axes"):
            if phase == "new axes":
                for a, b in zip(axes, new):
                    a.copy_(b)
                torch.cuda.synchronize()
                ref = whole()
            else:
                ref = ref_old
            for ctx, (z0, z1) in zip(ctxs, slabs):
                out = [torch.full((z1 - z0, G, G), -7.0, dtype=torch.float64, device="cuda") for _ in range(3)]
                torch.cuda.synchronize()
                ctx.interp_knn_dev(N, ptrs, G, G, G, axes_ptrs=aptrs, out_ptrs=[o.data_ptr() for o in out], k=8,
                                   flags=_lib.FLAG_SLAB_CULL_AUTO, z_range=(z0, z1))
                torch.cuda.synchronize()
                binned.append((phase, z0, ctx.last_stats()["n_binned"]))
                for a, b in zip(out, ref):
                    assert torch.equal(a, b[z0:z1]), (phase, z0, z1)
    finally:
        for c in ctxs:
            c.close()
    print(f"{change}: binned per (phase, slab) {binned}")
    # the new-axes call found no map for its key: every particle binned again
    assert all(b == N for ph, _, b in binned if ph != "warm") and all(b < N for ph, _, b in binned if ph == "warm")
