"""GPU fixed-radius IDW (``PTV_METHOD_IDW_RADIUS``, ``interpolate_field(..., idw_radius=r)``).

This is an EXTENSION for BASELINE config 2 ("256^3 grid, 1M particles, IDW radius-search"):
the reference has no radius search (interpolator.py:139 is ``tree.query(k)`` only), so its
parity is UNPINNED.  The semantics are defined by ``oracle.cpu_ref.idw_radius_points``: every
particle with ``((dx*dx + dy*dy) + dz*dz) <= r*r`` (scipy ``query_ball_point``'s test), the
reference's weights ``1/(d**p + 1e-10)``, ``sum(w v) / sum(w)``, NaN for an empty ball.

Bar: the NaN pattern (empty balls) identical, and normwise <= 1e-12 (the GPU sums the ball in
its gather order, the oracle in particle-index order).  Voxels with a particle within 1e-9 of
the ball surface are excluded (membership there is a rounding decision).
"""
import numpy as np
import pandas as pd
import pytest

from oracle import cpu_ref
from tests._util import normwise

pytestmark = pytest.mark.gpu

TOL = 1e-12


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


def _surface_voxels(points, q, r):
    """(M,) bool: queries with a particle within 1e-9 of the radius-r sphere around them."""
    from scipy.spatial import KDTree

    t = KDTree(points)
    outer = t.query_ball_point(q, r + 1e-9, return_length=True)
    inner = t.query_ball_point(q, max(r - 1e-9, 0.0), return_length=True)
    return outer != inner


def _check(got, ref, skip):
    for c in range(3):
        a = got[c].reshape(-1)[~skip]
        b = ref[:, c][~skip]
        assert np.array_equal(np.isnan(a), np.isnan(b)), "empty-ball (NaN) pattern differs"
        assert normwise(a, b) <= TOL


@pytest.mark.parametrize("n,G,r,p", [(20000, 48, 3.0, 2.0), (20000, 48, 1.2, 2.0), (6000, 40, 6.5, 1.5),
                                     (20000, 48, 2.5, 1.0), (3000, 33, 9.0, 0.5)])
def test_random_vs_oracle(ctx, n, G, r, p):
    from ptv_interpolation_amd import _lib

    rng = np.random.default_rng(1000 + n + G)
    P = rng.uniform(-0.5, G - 0.5, (n, 3))
    Q = rng.standard_normal((n, 3))
    ax = np.linspace(0.0, G - 1.0, G)
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=_lib.METHOD_IDW_RADIUS, power=p, radius=r)
    q = cpu_ref.grid_queries(ax, ax, ax)
    ref = cpu_ref.idw_radius_points(P, Q, q, r, power=p)
    _check((U, V, W), ref, _surface_voxels(P, q, r))
    if r < 1.5:
        assert np.isnan(U).any()  # small balls: some voxels see no particle


def test_sphere_pack_voids_mask_and_nan_fill(ctx):
    """Sphere-pack voids (empty balls -> NaN), the fused mask + nan_to_num epilogue."""
    from ptv_interpolation_amd import _lib, synth

    G = 56
    P, Q = synth.sphere_pack(40000, G, values="normal")
    ax = np.linspace(0.0, G - 1.0, G)
    q = cpu_ref.grid_queries(ax, ax, ax)
    ref = cpu_ref.idw_radius_points(P, Q, q, 2.0)
    skip = _surface_voxels(P, q, 2.0)
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=_lib.METHOD_IDW_RADIUS, radius=2.0)
    _check((U, V, W), ref, skip)
    assert np.isnan(U).any()
    fl = synth.fluid_mask(G)
    Um, Vm, Wm = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=_lib.METHOD_IDW_RADIUS, radius=2.0,
                                fluid_mask=fl, flags=_lib.FLAG_NAN_TO_NUM)
    Ur, Vr, Wr = cpu_ref.nan_fill_and_mask(*(ref[:, c].reshape(U.shape) for c in range(3)), fluid_mask=fl)
    for a, b in ((Um, Ur), (Vm, Vr), (Wm, Wr)):
        assert not np.isnan(a).any()
        assert np.array_equal(a[~fl], b[~fl])  # solid voxels: exactly 0
        assert normwise(a.reshape(-1)[~skip], b.reshape(-1)[~skip]) <= TOL


def test_point_list_grid(ctx):
    from ptv_interpolation_amd import _lib

    rng = np.random.default_rng(7)
    P = rng.uniform(0, 20, (4000, 3))
    Q = rng.standard_normal((4000, 3))
    q = rng.uniform(0, 20, (3000, 3))
    U, V, W = ctx.interp_knn(P, Q, grid_points=[q[:, 0], q[:, 1], q[:, 2]], shape=(1, 1, len(q)),
                             method=_lib.METHOD_IDW_RADIUS, radius=2.2)
    ref = cpu_ref.idw_radius_points(P, Q, q, 2.2)
    _check((U, V, W), ref, _surface_voxels(P, q, 2.2))


def test_interpolate_field_option(capsys):
    """Drop-in extension keyword: interpolate_field(method='idw', idw_radius=r)."""
    from ptv_interpolation_amd import interpolator as ip

    rng = np.random.default_rng(3)
    P = rng.uniform(0, 31, (8000, 3))
    Q = rng.standard_normal((8000, 3))
    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
    (X, Y, Z), (x, y, z) = ip.create_grid(((0, 32),) * 3, 32)
    U, V, W = ip.interpolate_field(df, (X, Y, Z), method="idw", idw_power=2.0, idw_radius=3.5)
    assert capsys.readouterr().out.startswith("Using IDW Interpolation (power=2.0, radius=3.5)...")
    q = cpu_ref.grid_queries(x, y, z)
    _check((U, V, W), cpu_ref.idw_radius_points(P, Q, q, 3.5), _surface_voxels(P, q, 3.5))
    with pytest.raises(ValueError):
        ip.interpolate_field(df, (X, Y, Z), method="idw", idw_radius=-1.0)


def test_config2_sampled(ctx):
    """BASELINE config 2 shape: 256^3 grid, 1M sphere-pack particles, r = 3 voxels; 20k sampled
    voxels against the oracle."""
    from ptv_interpolation_amd import _lib, synth

    G = 256
    P, Q = synth.sphere_pack(1_000_000, G, values="normal")
    ax = np.linspace(0.0, G - 1.0, G)
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=_lib.METHOD_IDW_RADIUS, radius=3.0)
    rng = np.random.default_rng(11)
    sel = rng.choice(G ** 3, 20000, replace=False)
    iz, iy, ix = np.unravel_index(sel, (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], 1)
    ref = cpu_ref.idw_radius_points(P, Q, q, 3.0)
    skip = _surface_voxels(P, q, 3.0)
    got = tuple(a.reshape(-1)[sel] for a in (U, V, W))
    _check(got, ref, skip)
