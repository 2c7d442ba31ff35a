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
    bins only the particles within a proven-exact halo of each slab (slab_halo +
    zslab.interp_slab), not the whole set on every device: PTV_DEVICES=0,0,0,0 (four slabs on
    four contexts) bins fewer particles than N per slab and reproduces the one-call result bit
    for bit."""
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
        four = ip.interpolate_field(_df(P, Q), (X, Y, Z), method=method, **kw)
    binned = [st["n_binned"] for st in launcher.last_results]
    print(f"{method} {kw}: particles binned per slab {binned} of {N}; halos "
          f"{[(round(st['halo_first'], 2), st['halo_state']) for st in launcher.last_results]}")
    assert len(binned) == 4 and all(b < N for b in binned)
    for a, b in zip(four, one):
        assert np.array_equal(a, b, equal_nan=True)
