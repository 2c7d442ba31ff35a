"""GPU parity for method='linear' (the reference default: griddata(method='linear',
fill_value=0.0), interpolator.py:196-197) through the C ABI (ptv_interp_linear) and the
drop-in interpolate_field.  Runs only on an MI355X (``-m gpu``).

Bar: the triangulation is scipy's own (the same Delaunay call LinearNDInterpolator makes), so
every voxel that lies inside one simplex is bit-identical to the reference (np.array_equal on
the golden fixtures, which are in general position).  Voxels within eps of a face shared by two
simplices (lattice inputs, degenerate simplices) may be located in either neighbour, whose
interpolants agree to rounding: those cases are checked normwise (<= 1e-12) and the number of
differing voxels is bounded.
"""
import numpy as np
import pandas as pd
import pytest

from tests._util import load, normwise

pytestmark = pytest.mark.gpu

NAMES = ["linear_rand", "linear_aniso", "linear_default", "linear_dups"]


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


def _grid(g):
    Z, Y, X = np.meshgrid(g["az"], g["ay"], g["ax"], indexing="ij")
    return X, Y, Z


@pytest.mark.parametrize("name", NAMES)
def test_golden_dropin_bit_exact(ctx, name, capsys):
    """interpolate_field(df, grid) with method='linear' (or the default) equals the reference."""
    from ptv_interpolation_amd.interpolator import interpolate_field

    g = load(name)
    df = pd.DataFrame({"x": g["points"][:, 0], "y": g["points"][:, 1], "z": g["points"][:, 2],
                       "u": g["values"][:, 0], "v": g["values"][:, 1], "w": g["values"][:, 2]})
    kw = {} if name == "linear_default" else {"method": "linear"}
    U, V, W = interpolate_field(df, _grid(g), **kw)
    assert capsys.readouterr().out == ""  # the reference prints nothing on this branch
    for c, a in zip("UVW", (U, V, W)):
        assert a.shape == g[c].shape and a.dtype == np.float64
        assert np.array_equal(a, g[c]), f"{name} {c}: max |d| {np.max(np.abs(a - g[c])):.3e}"


def test_random_vs_oracle_point_list_and_slabs(ctx):
    """64^3 grid / 40k particles (general position) against the oracle: whole grid, point-list
    grid, and three uneven z-slabs all bit-identical."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib
    from scipy.spatial import Delaunay

    rng = np.random.default_rng(7)
    P = rng.uniform(3, 60, (40000, 3))
    Q = rng.standard_normal((40000, 3))
    ax = np.linspace(0, 63, 64)
    tri = _lib.Triangulation(Delaunay(P))
    ref = cpu_ref.linear_grid(P, Q, ax, ax, ax)
    got = ctx.interp_linear(P, Q, tri, axes=(ax, ax, ax))
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    Z, Y, X = np.meshgrid(ax[:20], ax, ax, indexing="ij")
    pl = ctx.interp_linear(P, Q, tri, grid_points=(X, Y, Z), shape=X.shape)
    for a, b in zip(pl, ref):
        assert np.array_equal(a, b[:20])
    for z0, z1 in ((0, 9), (9, 40), (40, 64)):
        sl = ctx.interp_linear(P, Q, tri, axes=(ax, ax, ax), z_range=(z0, z1), chunk_planes=8)
        for a, b in zip(sl, ref):
            assert np.array_equal(a, b[z0:z1])


def test_mask_nan_to_num_and_fill_value(ctx):
    """Solid voxels are 0 (fused main.py:202-207), NaN values become 0 under NAN_TO_NUM, and
    fill_value is written outside the hull."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib
    from scipy.spatial import Delaunay

    rng = np.random.default_rng(8)
    P = rng.uniform(4, 27, (6000, 3))
    Q = rng.standard_normal((6000, 3))
    Q[::97, 1] = np.nan
    ax = np.linspace(0, 31, 32)
    tri = _lib.Triangulation(Delaunay(P))
    mask = rng.random((32, 32, 32)) < 0.7
    U, V, W = ctx.interp_linear(P, Q, tri, axes=(ax, ax, ax), fluid_mask=mask, flags=_lib.FLAG_NAN_TO_NUM,
                                fill_value=-5.0)
    ref = cpu_ref.linear_grid(P, Q, ax, ax, ax, fill_value=-5.0)
    for a, b in zip((U, V, W), ref):
        e = np.where(mask, np.nan_to_num(b), 0.0)
        assert np.array_equal(a, e)
    assert (U[mask] == -5.0).any()


def test_lattice_degenerate_simplices_take_the_brute_force(ctx):
    """An exact 6^3 lattice: Qhull returns flat simplices (NaN transforms), so some walks fall
    back to scipy's brute-force scan (counted in stats['n_singular']).  Query points off the
    lattice planes; agreement with the oracle to rounding (ties between neighbouring simplices)."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib
    from scipy.spatial import Delaunay

    g = np.arange(6.0)
    P = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    Q = np.random.default_rng(9).standard_normal((len(P), 3))
    tri = _lib.Triangulation(Delaunay(P))
    assert np.isnan(tri.transform[:, 0, 0]).any()
    ax = np.linspace(-0.37, 5.41, 23)
    got = ctx.interp_linear(P, Q, tri, axes=(ax, ax, ax))
    ref = cpu_ref.linear_grid(P, Q, ax, ax, ax)
    print("brute-force voxels:", ctx.stats["n_singular"])
    for a, b in zip(got, ref):
        assert normwise(a, b) <= 1e-12
        assert np.mean(a != b) < 0.05


def test_sphere_pack_sampled(ctx):
    """128^3 grid, 300k sphere-pack particles (voids: simplices spanning the solid spheres):
    20k random voxels against the oracle over the same Delaunay object, bit-identical."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib, synth
    from scipy.spatial import Delaunay

    G = 128
    P, Q = synth.sphere_pack(300_000, G, values="normal")
    ax = np.linspace(0, G - 1, G)
    d = Delaunay(P)
    U, V, W = ctx.interp_linear(P, Q, _lib.Triangulation(d), axes=(ax, ax, ax))
    print("brute-force voxels:", ctx.stats["n_singular"], "walk ms:", ctx.stats["ms_solve"])
    rng = np.random.default_rng(11)
    sel = rng.integers(0, G ** 3, 20000)
    iz, iy, ix = np.unravel_index(sel, (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], -1)
    ref = cpu_ref.linear_points(P, Q, q, tri=d)
    for c, a in enumerate((U, V, W)):
        assert np.array_equal(a.ravel()[sel], ref[:, c])
