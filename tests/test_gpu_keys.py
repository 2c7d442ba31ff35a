"""GPU parity of the packed-key k-NN lists (k >= 13; ptv_knn_impl.hpp insert_key) and their
near-tie repair, against the oracle (scipy KDTree + numpy restatement of
interpolator.py:83-155) and the reference fixtures.

The key lists order candidates by (d2 truncated to 52 - B mantissa bits, slot); the epilogue
recomputes the exact d2, and tiles whose order or k-th/(k+1)-th boundary the truncation could
not prove go to an exact rerun (ptv_stats.n_repair_tiles).  These tests cover k beyond the old
64 limit (interpolator.py:139 accepts any k), exact ties everywhere (a particle lattice: every
boundary is a tie, so the repair path runs), coincident particles (d2 = 0 keys are subnormal
doubles) and the outlier filter's (k+1)-NN (filtering.py:26) through the same lists.
"""
import numpy as np
import pytest

from tests._util import hetero_ties, load, normwise

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


@pytest.mark.parametrize("method,k", [("idw", 13), ("idw", 15), ("idw", 16), ("idw", 31), ("idw", 32),
                                      ("idw", 80), ("idw", 100), ("idw", 127),
                                      ("sibson", 24), ("sibson", 96), ("sibson", 127)])
def test_key_lists_vs_oracle(ctx, method, k):
    """Every key-list length (16 .. 128 slots) against KDTree + numpy on a random 20^3 case;
    IDW p = 2 bit-exact, Sibson within the normwise bar (numpy's SIMD exp)."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib

    P, Q, ax = _random_case(11 + k, 3000, 20)
    m = _lib.METHOD_IDW if method == "idw" else _lib.METHOD_SIBSON
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=m, k=k)
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, method, k, 2.0)
    print(f"{method} k={k}: repaired tiles {ctx.stats['n_repair_tiles']}")
    for a, b in zip((U, V, W), ref):
        if method == "idw":
            assert np.array_equal(a, b), f"{np.sum(a != b)} voxels differ"
        else:
            assert normwise(a, b) <= TOL


def test_k_above_n_raises(ctx):
    P, Q, ax = _random_case(3, 100, 6)
    with pytest.raises(ValueError):
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=101)
    # k >= 128 is served by the large-k path (tests/test_gpu_bigk.py), k > n still raises there
    with pytest.raises(ValueError):
        ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=200)


@pytest.mark.parametrize("k", [14, 20, 50])
def test_lattice_ties_repair(ctx, k):
    """Particles on an integer lattice with one value per component, voxels on the lattice and
    between it: exact distance ties at (almost) every k-th/(k+1)-th boundary, so the near-tie
    repair reruns the tiles; every tie is value-homogeneous, so the result is bit-exact
    everywhere whatever the tie order (a wrong distance multiset would not be)."""
    from oracle import cpu_ref

    g = np.arange(0.0, 14.0)
    Z, Y, X = np.meshgrid(g, g, g, indexing="ij")
    P = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    Q = np.tile([1.5, -2.0, 0.25], (len(P), 1))
    for ax in (np.arange(0.0, 13.0, 1.0), np.arange(0.5, 13.0, 1.0)):
        U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
        rep = ctx.stats["n_repair_tiles"]
        ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", k, 2.0)
        print(f"lattice k={k} axis offset {ax[0]}: repaired tiles {rep}")
        assert rep > 0  # the repair path ran
        for a, b in zip((U, V, W), ref):
            assert np.array_equal(a, b), f"{np.sum(a != b)} voxels differ"


def test_lattice_ties_whole_launch_rerun(ctx):
    """The repair list past its capacity (PTV_FLAG_KNN_REPAIR_ALL: a one-entry list) reruns the
    whole launch with the exact pair lists: the result is bit-identical to the listed-tile rerun and
    to the oracle, with more tiles to repair than the list holds."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib

    g = np.arange(0.0, 14.0)
    Z, Y, X = np.meshgrid(g, g, g, indexing="ij")
    P = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    Q = np.tile([1.5, -2.0, 0.25], (len(P), 1))
    ax = np.arange(0.5, 13.0, 1.0)
    listed = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=20)
    whole = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=20, flags=_lib.FLAG_KNN_REPAIR_ALL)
    rep = ctx.stats["n_repair_tiles"]
    print(f"whole-launch rerun: tiles to repair {rep}")
    assert rep > 1
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", 20, 2.0)
    for a, b, c in zip(listed, whole, ref):
        assert np.array_equal(a, b) and np.array_equal(b, c)


@pytest.mark.parametrize("k", [16, 40])
def test_lattice_plus_random_ties(ctx, k):
    """A spacing-4 particle lattice mixed with random particles (random values): exact ties
    where only lattice particles decide; value-heterogeneous tie voxels excluded (counted),
    every other voxel bit-exact vs the oracle."""
    from oracle import cpu_ref

    g = np.arange(0.0, 24.0, 4.0)
    Z, Y, X = np.meshgrid(g, g, g, indexing="ij")
    rng = np.random.default_rng(k)
    P = np.concatenate([np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1), rng.uniform(0, 22, (6000, 3))])
    Q = rng.standard_normal((len(P), 3))
    ax = np.arange(0.0, 23.0, 1.0)
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=k)
    rep = ctx.stats["n_repair_tiles"]
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", k, 2.0)
    tie, het = hetero_ties(P, Q, ax, ax, ax, k)
    print(f"lattice+random k={k}: ties {tie.mean():.2%}, value-heterogeneous (excluded) {het.mean():.2%}, "
          f"repaired tiles {rep}")
    keep = ~het
    assert keep.mean() > 0.5
    for a, b in zip((U, V, W), ref):
        assert np.array_equal(a[keep], b[keep]), f"{np.sum(a[keep] != b[keep])} voxels differ"


def test_coincident_particles_subnormal_keys(ctx):
    """Voxels that coincide with particles (d2 = 0: the key is the slot as a subnormal double)
    and duplicated particles at k = 20: bit-exact vs the oracle where no tie decides."""
    from oracle import cpu_ref

    rng = np.random.default_rng(4)
    ax = np.arange(10, dtype=np.float64)
    Zg, Yg, Xg = np.meshgrid(ax, ax, ax, indexing="ij")
    on = np.stack([Xg.ravel(), Yg.ravel(), Zg.ravel()], -1)[rng.choice(1000, 150, replace=False)]
    P = np.concatenate([on, rng.uniform(0, 9, (1500, 3))])
    Q = rng.standard_normal((len(P), 3))
    U, V, W = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=20)
    ref = cpu_ref.interp_grid(P, Q, ax, ax, ax, "idw", 20, 2.0)
    _, het = hetero_ties(P, Q, ax, ax, ax, 20)
    keep = ~het
    for a, b in zip((U, V, W), ref):
        assert np.array_equal(a[keep], b[keep])
        assert np.isfinite(a).all()


@pytest.mark.parametrize("name", ["idw_small_k16_p2.0", "idw_small_k33_p2.0", "idw_small_k64_p2.0",
                                  "idw_default_k50", "sibson_k30", "sibson_small_k64"])
def test_key_lists_reference_fixtures(ctx, name):
    """The reference's own outputs for k >= 13 (tests/golden/make_golden.py)."""
    from ptv_interpolation_amd import _lib

    g = load(name)
    m = _lib.METHOD_IDW if str(g["method"]) == "idw" else _lib.METHOD_SIBSON
    U, V, W = ctx.interp_knn(g["points"], g["values"], axes=(g["ax"], g["ay"], g["az"]), method=m,
                             k=int(g["k"]), power=float(g["power"]))
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        assert normwise(a, b) <= TOL
        if m == _lib.METHOD_IDW and float(g["power"]) == 2.0:
            assert np.array_equal(a, b)


@pytest.mark.parametrize("k", [12, 25, 63, 100])
def test_filter_key_lists_vs_oracle(ctx, k):
    """remove_outliers_knn's (k+1)-NN (filtering.py:26) through the key lists (k + 1 >= 13)
    and beyond the old k = 63 limit: keep masks bit-exact vs the oracle's KDTree restatement."""
    from oracle import cpu_ref

    rng = np.random.default_rng(100 + k)
    P = rng.uniform(0, 30, (6000, 3))
    Q = rng.standard_normal((6000, 3))
    Q[rng.choice(6000, 60, replace=False)] *= 25.0  # outliers
    keep, kth = ctx.filter_outliers_knn(P, Q, k=k, threshold=3.0)
    ref_keep, ref_radius = cpu_ref.outlier_filter(P, Q, k, 3.0, workers=-1)
    assert np.array_equal(keep.view(bool), ref_keep)
    assert np.median(kth) == ref_radius
