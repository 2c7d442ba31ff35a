"""GPU parity for the pore-mask path and the k-NN outlier filter.

* ``sample_mask_on_grid`` (interpolator.py:205-238) -> ``ptv_sample_mask``;
* ``extract_boundary_particles`` (interpolator.py:240-284) -> ``ptv_boundary_particles``;
* ``filtering.remove_outliers_knn`` (filtering.py:5-58) -> ``ptv_filter_outliers_knn``.

All three are integer/index work (nearest-index lookups, a dilation, an ordered
compaction, a neighbour-set median) and are required bit-exact: against the reference
golden vectors (tests/golden/make_golden.py: mask_cases, filter_cases), against the
oracle on larger seeded inputs, and through size-independent properties at full size.
"""
import contextlib
import io

import numpy as np
import pandas as pd
import pytest

from oracle import cpu_ref
from tests._util import filter_ties, load, names

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


def _bounds(g, key):
    b = g[key]
    if int(g[key + "_int"]):
        b = b.astype(int)
    return tuple(tuple(v.tolist()) for v in b)


# ---------------------------------------------------------------- sample_mask_on_grid
@pytest.mark.parametrize("name", names(("mask_sample_",)))
def test_sample_mask_golden(ctx, name):
    from ptv_interpolation_amd import interpolator as ip

    g = load(name)
    Z, Y, X = np.meshgrid(g["az"], g["ay"], g["ax"], indexing="ij")
    got = ip.sample_mask_on_grid(g["raw"], (X, Y, Z), _bounds(g, "raw_bounds"))
    assert got.dtype == np.bool_ and got.shape == g["mask"].shape
    assert np.array_equal(got, g["mask"])
    # point-list mode (a grid that is not a meshgrid: flat coordinate arrays)
    flat = ip.sample_mask_on_grid(g["raw"], (X.ravel(), Y.ravel(), Z.ravel()), _bounds(g, "raw_bounds"))
    assert flat.shape == (X.size,) and np.array_equal(flat, g["mask"].ravel())


def test_sample_mask_descending_and_label_raw(ctx):
    from ptv_interpolation_amd import interpolator as ip

    rng = np.random.default_rng(3)
    raw = rng.integers(0, 3, (9, 11, 13)).astype(np.int16)  # astype(float) > 0.5 on a label mask
    bounds = ((20, 7), (0, 11), (0, 9))                       # descending x axis: linspace(20, 6, 13)
    (X, Y, Z), _ = ip.create_grid(((0, 22), (-2, 12), (0, 10)), (17, 14, 10))
    got = ip.sample_mask_on_grid(raw, (X, Y, Z), bounds)
    assert np.array_equal(got, cpu_ref.sample_mask_nearest(raw, bounds, X, Y, Z))


def test_sample_mask_full_size_vs_oracle(ctx):
    """512^3 grid from a 384^3 raw mask (main.py --downscale 0.75): every voxel against the oracle."""
    from ptv_interpolation_amd import interpolator as ip
    from ptv_interpolation_amd import synth

    raw = synth.fluid_mask(384)
    bounds = ((0, 384),) * 3
    (X, Y, Z), (x, y, z) = ip.create_grid(bounds, 512, dense=False)
    got = ip.sample_mask_on_grid(raw, (X, Y, Z), bounds)
    jx = cpu_ref.rgi_nearest_index(np.linspace(0, 383, 384), x)
    jy = cpu_ref.rgi_nearest_index(np.linspace(0, 383, 384), y)
    jz = cpu_ref.rgi_nearest_index(np.linspace(0, 383, 384), z)
    assert (jx >= 0).all() and (jy >= 0).all() and (jz >= 0).all()
    exp = raw[jz[:, None, None], jy[None, :, None], jx[None, None, :]]
    assert np.array_equal(got, exp)


# ---------------------------------------------------------------- extract_boundary_particles
@pytest.mark.parametrize("name", names(("boundary_",)))
def test_boundary_particles_golden(ctx, name):
    from ptv_interpolation_amd import interpolator as ip

    g = load(name)
    got = ip.extract_boundary_particles(g["mask"], _bounds(g, "bounds"), sampling_step=int(g["step"]),
                                        thickness=int(g["thickness"]))
    for a, e in zip(got, (g["bx"], g["by"], g["bz"])):
        assert a.dtype == e.dtype and np.array_equal(a, e)


def test_boundary_particles_edge_cases(ctx):
    from ptv_interpolation_amd import interpolator as ip

    assert [len(a) for a in ip.extract_boundary_particles(None, ((0, 4),) * 3)] == [0, 0, 0]
    allf = np.ones((5, 6, 7), dtype=bool)    # no solid voxel
    assert [len(a) for a in ip.extract_boundary_particles(allf, ((0, 7), (0, 6), (0, 5)))] == [0, 0, 0]
    alls = np.zeros((5, 6, 7), dtype=bool)   # no fluid voxel
    assert [len(a) for a in ip.extract_boundary_particles(alls, ((0, 7), (0, 6), (0, 5)))] == [0, 0, 0]
    with pytest.raises(TypeError):           # `~mask` of a float mask, as in the reference
        ip.extract_boundary_particles(np.ones((3, 3, 3)), ((0, 3),) * 3)


@pytest.mark.parametrize("thickness,step", [(1, 1), (2, 5), (4, 1)])
def test_boundary_particles_ragged_vs_oracle(ctx, thickness, step):
    from ptv_interpolation_amd import interpolator as ip
    from tests.golden.make_golden import _blob_mask

    m = _blob_mask((61, 77, 93), 40, 17 + thickness)
    b = ((1.5, 95.0), (0, 77), (-4, 60))
    got = ip.extract_boundary_particles(m, b, sampling_step=step, thickness=thickness)
    exp = cpu_ref.boundary_particles(m, b, step, thickness)
    for a, e in zip(got, exp):
        assert np.array_equal(a, e)


def test_boundary_particles_full_size_count_and_order(ctx):
    """512^3 sphere-pack mask: the GPU list equals the oracle's (sorted C order, every voxel)."""
    from ptv_interpolation_amd import interpolator as ip
    from ptv_interpolation_amd import synth

    m = synth.fluid_mask(512)
    b = ((0, 512),) * 3
    gx, gy, gz = ip.extract_boundary_particles(m, b, sampling_step=1, thickness=2)
    ex, ey, ez = cpu_ref.boundary_particles(m, b, 1, 2)
    assert len(gx) == len(ex) > 0
    assert np.array_equal(gx, ex) and np.array_equal(gy, ey) and np.array_equal(gz, ez)


# ---------------------------------------------------------------- remove_outliers_knn
def _df(P, Q):
    return pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})


@pytest.mark.parametrize("name", names(("filter_",)))
def test_outlier_filter_golden(ctx, name):
    from ptv_interpolation_amd import filtering

    g = load(name)
    df = _df(g["points"], g["values"])
    df["id"] = np.arange(len(df))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = filtering.remove_outliers_knn(df, k=int(g["k"]), threshold=float(g["threshold"]))
    keep = np.zeros(len(df), dtype=bool)
    keep[out["id"].values] = True
    ties = filter_ties(g["points"], int(g["k"]))
    if ties.any():
        # coincident particles (filter_dup_*): the tie-dependent decisions are excluded, the
        # rest must match; the radius line is tie-independent
        assert name.startswith("filter_dup"), "unexpected ties in a continuous fixture"
        assert np.array_equal(keep[~ties], g["keep"][~ties])
        assert buf.getvalue().splitlines()[0] == str(g["stdout"]).splitlines()[0]
    else:
        assert np.array_equal(keep, g["keep"])
        assert buf.getvalue() == str(g["stdout"])
    assert list(out.index) == list(range(len(out)))  # reset_index(drop=True)


def test_outlier_filter_small_and_clean(ctx):
    from ptv_interpolation_amd import filtering

    P = np.random.default_rng(1).uniform(0, 5, (20, 3))
    df = _df(P, np.ones_like(P))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = filtering.remove_outliers_knn(df, k=25)
    assert out is df and "too small (20)" in buf.getvalue()
    with contextlib.redirect_stdout(io.StringIO()):
        out = filtering.remove_outliers_knn(_df(P, np.ones_like(P)), k=5)  # uniform speed: MAD 0, z 0
    assert len(out) == 20


@pytest.mark.parametrize("k", [4, 16, 25, 40])
def test_outlier_filter_vs_oracle(ctx, k):
    """Larger seeded clouds (and sphere-pack voids) at several list lengths, bit-exact keep masks."""
    from ptv_interpolation_amd import synth

    P, _ = synth.sphere_pack(60000, 96)
    rng = np.random.default_rng(k)
    Q = rng.standard_normal((len(P), 3))
    Q[rng.choice(len(P), 600, replace=False)] *= 8.0
    keep, kth = ctx.filter_outliers_knn(P, Q, k=k, threshold=3.0)
    exp, radius = cpu_ref.outlier_filter(P, Q, k, 3.0, workers=-1)
    assert np.array_equal(keep.view(bool), exp)
    assert np.median(kth) == radius


def test_outlier_filter_full_size_properties(ctx):
    """5M particles (the headline particle count), k = 25: a sampled subset of particles
    against the oracle's per-particle statistics, and the radius median."""
    from scipy.spatial import KDTree

    from ptv_interpolation_amd import synth

    P, _ = synth.sphere_pack(5_000_000, 512)
    rng = np.random.default_rng(7)
    Q = rng.standard_normal((len(P), 3))
    keep, kth = ctx.filter_outliers_knn(P, Q, k=25, threshold=3.0)
    sel = rng.choice(len(P), 20000, replace=False)
    dist, idx = KDTree(P).query(P[sel], k=26, workers=-1)
    speed = np.sqrt(Q[:, 0] ** 2 + Q[:, 1] ** 2 + Q[:, 2] ** 2)
    ns = speed[idx[:, 1:]]
    med = np.median(ns, axis=1)
    mad = np.median(np.abs(ns - med[:, None]), axis=1)
    exp = np.abs(speed[sel] - med) / (mad + 1e-6) <= 3.0
    assert np.array_equal(keep.view(bool)[sel], exp)
    assert np.array_equal(kth[sel], dist[:, -1])


@pytest.mark.parametrize("thickness", [1, 2])
def test_boundary_particles_label_mask_aligned_rows(ctx, thickness):
    """Integer label mask with 16-aligned rows (the 16-voxel SWAR kernels) and the numpy
    `bool & ~int` low-bit rule, against the oracle; also a bool mask of the same shape."""
    from ptv_interpolation_amd import interpolator as ip

    rng = np.random.default_rng(40 + thickness)
    lab = rng.integers(0, 4, (12, 10, 32)).astype(np.uint8)
    lab[:, :, 8:20] = 0
    b = ((0, 32), (0, 10), (0, 12))
    for m in (lab, lab == 2):
        got = ip.extract_boundary_particles(m, b, sampling_step=1, thickness=thickness)
        exp = cpu_ref.boundary_particles(m, b, 1, thickness)
        for a, e in zip(got, exp):
            assert np.array_equal(a, e)
