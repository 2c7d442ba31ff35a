"""GPU parity of the large-k path (k >= 128 for IDW / Sibson, k >= 127 for the outlier filter;
ptv_knn_big.hip): the reference's KDTree.query takes any k (interpolator.py:97, :139;
filtering.py:26), so these k run a list-free search -- per-query ball bound, candidate gather,
segmented radix sort -- and the reference's epilogue, including numpy's pairwise-sum recursion past
128 terms (oracle.cpu_ref.pairwise_sum).  Checked against the oracle (scipy KDTree + numpy):
IDW p = 2 bit-exact, Sibson and pow-path powers within the normwise bar, the filter's keep
masks and k-th distances bit-exact.
"""
import contextlib
import io

import numpy as np
import pandas as pd
import pytest

from tests._util import hetero_ties, hetero_ties_points, normwise

pytestmark = pytest.mark.gpu

TOL = 1e-10


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


def _random_case(seed, n, G):
    rng = np.random.default_rng(seed)
    P = rng.uniform(-0.5, G - 0.5, (n, 3))
    Q = rng.standard_normal((n, 3))
    ax = np.arange(G, dtype=np.float64)
    return P, Q, ax


@pytest.mark.parametrize("method,k,power", [("idw", 128, 2.0), ("idw", 129, 2.0), ("idw", 200, 2.0),
                                            ("idw", 333, 2.0), ("idw", 1000, 2.0), ("idw", 256, 1.0),
                                            ("idw", 150, 1.5), ("sibson", 128, 2.0), ("sibson", 257, 2.0)])
def test_large_k_vs_oracle(ctx, method, k, power):
    """Random cloud, 16^3 grid: IDW p in {2, 1} bit-exact (every pairwise-sum split: 128 = one
    leaf, 129 = 64 + 65, 1000 = a three-level tree), p = 1.5 and Sibson within the normwise bar."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib

    P, Q, ax = _random_case(k, 6000, 16)
    m = _lib.METHOD_IDW if method == "idw" else _lib.METHOD_SIBSON
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=m, k=k, power=power)
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, method, k, power)
    exact = method == "idw" and power in (1.0, 2.0)
    for a, b in zip((U, V, W), ref):
        if exact:
            assert np.array_equal(a, b), f"{np.sum(a != b)} voxels differ"
        else:
            e = normwise(a, b)
            print(f"{method} k={k} p={power}: normwise {e:.2e}, bit-identical {np.mean(a == b):.4f}")
            assert e <= TOL


def test_large_k_sphere_pack_voids_and_slabs(ctx):
    """Sphere pack (void voxels far from every particle: the ball bound grows over several steps),
    IDW k = 200 on a 40^3 grid: bit-exact against the oracle except value-heterogeneous ties, and
    three z-slab calls equal to the whole-grid call."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import synth

    G = 40
    P, Q = synth.sphere_pack(30000, G, values="normal")
    ax = np.linspace(0, G - 1, G)
    whole = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=200)
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", 200, 2.0)
    tie, het = hetero_ties(P, Q, ax, ax, ax, 200)
    print(f"ties {tie.mean():.4%}, value-heterogeneous (excluded) {het.mean():.4%}")
    assert het.mean() < 0.01
    for a, b in zip(whole, ref):
        assert np.array_equal(a[~het], b[~het])
    for z0, z1 in ((0, 13), (13, 27), (27, G)):
        part = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=200, z_range=(z0, z1))
        for a, b in zip(part, whole):
            assert np.array_equal(a, b[z0:z1])


def test_large_k_mask_f32_points_and_lattice_ties(ctx):
    """The fused epilogue options (fluid mask: solid voxels 0; NaN fill; float32 outputs), point-list
    queries, and a particle lattice whose every distance boundary is a tie (one value per particle
    set: value-homogeneous, so bit-exact whatever the order)."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib

    P, Q, ax = _random_case(3, 5000, 12)
    k = 150
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", k, 2.0)
    mask = np.random.default_rng(2).uniform(size=(12, 12, 12)) < 0.6
    m = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k, fluid_mask=mask, flags=_lib.FLAG_NAN_TO_NUM)
    f = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k, flags=_lib.FLAG_OUT_F32)
    Z, Y, X = np.meshgrid(ax, ax, ax, indexing="ij")
    pts = ctx.interp_knn(P, Q, grid_points=[X.ravel(), Y.ravel(), Z.ravel()], shape=X.shape, k=k)
    for c in range(3):
        assert np.array_equal(m[c][mask], ref[c][mask]) and (m[c][~mask] == 0).all()
        assert f[c].dtype == np.float32 and np.array_equal(f[c], ref[c].astype(np.float32))
        assert np.array_equal(pts[c].reshape(ref[c].shape), ref[c])
    # lattice: 8^3 particles on integers, values constant -> every tie value-homogeneous
    g = np.arange(8, dtype=np.float64)
    Pl = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    Ql = np.tile([[0.25, -1.5, 3.0]], (len(Pl), 1))
    axl = np.arange(0, 7.5, 0.5)
    out = ctx.interp_knn(Pl, Ql, axes=(axl, axl, axl), k=140)
    refl = cpu_ref.interp_grid(Pl, Ql, axl, axl, axl, "idw", 140, 2.0)
    for a, b in zip(out, refl):
        assert np.array_equal(a, b)


def test_large_k_dropin_and_launcher(monkeypatch):
    """interpolate_field(method='idw', idw_neighbors=300) through the drop-in (one device and three
    slab contexts) equals the oracle; the reference's default path takes any k."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import interpolator as ip

    P, Q, ax = _random_case(9, 8000, 14)
    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
    (X, Y, Z), _ = ip.create_grid(((0, 13),) * 3, 14)
    ref = cpu_ref.interp_points(P, Q, np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1), "idw", 300, 2.0)
    with contextlib.redirect_stdout(io.StringIO()):
        monkeypatch.setenv("PTV_DEVICE", "0")
        one = ip.interpolate_field(df, (X, Y, Z), method="idw", idw_neighbors=300)
        monkeypatch.delenv("PTV_DEVICE")
        monkeypatch.setenv("PTV_DEVICES", "0,0,0")
        three = ip.interpolate_field(df, (X, Y, Z), method="idw", idw_neighbors=300)
    for c in range(3):
        assert np.array_equal(one[c].ravel(), ref[:, c])
        assert np.array_equal(three[c], one[c])


@pytest.mark.parametrize("k", [127, 160, 300])
def test_large_k_outlier_filter_vs_oracle(ctx, k):
    """The outlier filter's (k+1)-NN at k >= 127 (filtering.py:26): keep masks and the (k+1)-th
    neighbour distances bit-exact against the oracle, on a sphere pack with planted outliers."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import synth
    from scipy.spatial import KDTree

    P, _ = synth.sphere_pack(20000, 48)
    rng = np.random.default_rng(k)
    Q = rng.standard_normal((len(P), 3))
    Q[rng.choice(len(P), 300, replace=False)] *= 8.0
    keep, kth = ctx.filter_outliers_knn(P, Q, k=k, threshold=3.0)
    exp, radius = cpu_ref.outlier_filter(P, Q, k, 3.0, workers=-1)
    d, _ = KDTree(P).query(P, k=k + 1, workers=-1)
    print(f"k={k}: removed {np.sum(~exp)}")
    assert np.array_equal(keep.view(bool), exp)
    assert np.array_equal(kth, d[:, -1])
    assert np.median(kth) == radius


def test_large_k_hetero_ties_points_helper_consistent(ctx):
    """A voxel exactly between particles with different values at k >= 128 is reported as a
    value-heterogeneous tie by the helper the other tests use (sanity of the exclusion)."""
    P = np.array([[float(i), 0.0, 0.0] for i in range(-100, 101)])
    Q = np.arange(len(P), dtype=np.float64)[:, None].repeat(3, 1)
    tie, het = hetero_ties_points(P, Q, np.array([[0.5, 0.0, 0.0]]), 130)
    assert tie[0] and het[0]
