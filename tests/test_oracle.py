"""The oracle (oracle/cpu_ref.py) pinned against the reference's own outputs.

Golden vectors come from importing the reference interpolator.py
(tests/golden/make_golden.py).  IDW/Sibson with p=2 are required bit-exact;
pow/exp paths and tied inputs are normwise (<= 1e-10).
"""
import numpy as np
import pytest

from oracle import cpu_ref
from tests._util import load, names, normwise


def _bit_exact_expected(g):
    return int(g.get("tied", 0)) == 0 and str(g["method"]) == "idw" and float(g["power"]) in (2.0, 1.0, 0.5, -1.0)


@pytest.mark.parametrize("name", names(("idw", "sibson", "edge")))
def test_oracle_matches_reference(name):
    g = load(name)
    U, V, W = cpu_ref.interp_grid(g["points"], g["values"], g["ax"], g["ay"], g["az"],
                                  method=str(g["method"]), k=int(g["k"]), power=float(g["power"]))
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        if _bit_exact_expected(g) or str(g["method"]) == "sibson" and not int(g.get("tied", 0)):
            # Sibson uses np.exp on the same machine class; exact here, normwise elsewhere.
            assert normwise(a, b) <= 1e-13
        if _bit_exact_expected(g):
            assert np.array_equal(a, b, equal_nan=True)
        assert normwise(a, b) <= 1e-10


def test_oracle_masked_pipeline():
    g = load("masked_spherepack_idw")
    U, V, W = cpu_ref.interp_grid(g["points"], g["values"], g["ax"], g["ay"], g["az"], "idw", 8, 2.0)
    assert normwise(U, g["U_raw"]) <= 1e-12
    U, V, W = cpu_ref.nan_fill_and_mask(U, V, W, g["mask"])
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        assert normwise(a, b) <= 1e-12


@pytest.mark.parametrize("k", [1, 3, 7, 8, 9, 16, 30, 50, 64, 127, 128, 129, 300])
def test_pairwise_sum_matches_numpy(k):
    rng = np.random.default_rng(k)
    A = rng.standard_normal((300, k)) * np.exp(rng.uniform(-30, 30, (300, k)))
    ref = A.sum(axis=1)
    mine = np.array([cpu_ref.pairwise_sum(r) for r in A])
    assert np.array_equal(ref, mine)


def test_bruteforce_matches_kdtree():
    rng = np.random.default_rng(3)
    P = rng.uniform(0, 20, (3000, 3)); Qp = rng.uniform(-2, 22, (2000, 3))
    d1, i1 = cpu_ref.knn_kdtree(P, Qp, 17)
    d2, i2 = cpu_ref.knn_bruteforce(P, Qp, 17)
    assert np.array_equal(d1, d2)
    assert np.array_equal(i1, i2)


def test_parallel_driver_equals_whole_grid():
    g = load("idw_k8_p2")
    U0, V0, W0 = cpu_ref.interp_grid(g["points"], g["values"], g["ax"], g["ay"], g["az"], "idw", 8, 2.0)
    U1, V1, W1 = cpu_ref.interp_grid_parallel(g["points"], g["values"], g["ax"], g["ay"], g["az"], "idw", 8, 2.0, n_jobs=2)
    assert np.array_equal(U0, U1) and np.array_equal(V0, V1) and np.array_equal(W0, W1)


def _rbf_args(g):
    eps = float(g["epsilon"]) if "epsilon" in g else None
    deg = int(g["degree"]) if "degree" in g else None
    return int(g["k"]), str(g["kernel"]), eps, deg, float(g["smoothing"])


@pytest.mark.parametrize("name", names(("rbf",)))
def test_rbf_oracle_matches_reference(name):
    """The local-RBF restatement (scipy RBFInterpolator(neighbors=k) via numpy's LAPACK gesv)
    against the reference's own outputs.  The Gaussian eps=0.3 systems reach cond 6e8: two
    LAPACK builds differ there by 1.6e-9, so those fixtures get 1e-8 (tests/test_gpu_rbf.py)."""
    g = load(name)
    k, kern, eps, deg, s = _rbf_args(g)
    U, V, W = cpu_ref.rbf_local_grid(g["points"], g["values"], g["ax"], g["ay"], g["az"], k, kern, eps, deg, s)
    tol = 1e-8 if kern == "gaussian" else 1e-11
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        assert normwise(a, b) <= tol


def test_rbf_monomial_powers_match_scipy():
    from scipy.interpolate._rbfinterp import _monomial_powers

    for deg in range(-1, 4):
        assert np.array_equal(cpu_ref.monomial_powers(deg), _monomial_powers(3, deg))


@pytest.mark.parametrize("kernel", sorted(cpu_ref.RBF_PHI))
def test_rbf_kernel_formulas_match_scipy(kernel):
    """phi(r) against scipy's compiled kernel matrix builder on one small point set."""
    from scipy.interpolate._rbfinterp_pythran import _kernel_matrix

    rng = np.random.default_rng(1)
    y = rng.uniform(0, 3, (20, 3))
    ref = _kernel_matrix(y, kernel)
    r = np.sqrt(((y[:, None, :] - y[None, :, :]) ** 2).sum(-1))
    assert np.allclose(cpu_ref.RBF_PHI[kernel](r), ref, rtol=1e-13, atol=1e-14)


@pytest.mark.parametrize("name", names(("div_",)))
def test_divergence_oracle_matches_reference(name):
    """physics.compute_consistent_divergence golden vectors: bit-exact, same dtype."""
    g = load(name)
    sp = [g[k] if int(g["spacing_np64"]) else float(g[k]) for k in ("dx", "dy", "dz")]
    d = cpu_ref.consistent_divergence(g["u"], g["v"], g["w"], g["mask"], *sp)
    assert d.dtype == g["div"].dtype
    assert np.array_equal(d, g["div"])


def test_nearest_oracle_matches_reference():
    g = load("nearest_small")
    U, V, W = cpu_ref.interp_grid(g["points"], g["values"], g["ax"], g["ay"], g["az"], "nearest")
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        assert np.array_equal(a, b)


# ------------------------------------------------ pore-mask path + outlier filter (§8(f) rows 2-3)
def _bounds(g, key):
    b = g[key]
    if int(g[key + "_int"]):
        b = b.astype(int)
    return tuple(tuple(v.tolist()) for v in b)


@pytest.mark.parametrize("name", names(("mask_sample_",)))
def test_oracle_sample_mask_matches_reference(name):
    g = load(name)
    Z, Y, X = np.meshgrid(g["az"], g["ay"], g["ax"], indexing="ij")
    assert np.array_equal(cpu_ref.sample_mask_nearest(g["raw"], _bounds(g, "raw_bounds"), X, Y, Z), g["mask"])


@pytest.mark.parametrize("name", names(("boundary_",)))
def test_oracle_boundary_particles_match_reference(name):
    g = load(name)
    got = cpu_ref.boundary_particles(g["mask"], _bounds(g, "bounds"), int(g["step"]), int(g["thickness"]))
    for a, e in zip(got, (g["bx"], g["by"], g["bz"])):
        assert a.dtype == e.dtype and np.array_equal(a, e)


@pytest.mark.parametrize("name", names(("filter_",)))
def test_oracle_outlier_filter_matches_reference(name):
    g = load(name)
    keep, radius = cpu_ref.outlier_filter(g["points"], g["values"], int(g["k"]), float(g["threshold"]))
    assert np.array_equal(keep, g["keep"])
    assert f"= {radius:.4f}\n" in str(g["stdout"])


def test_oracle_rgi_nearest_tie_and_bounds():
    g = np.array([0.0, 1.0, 2.0, 3.0])
    x = np.array([-0.1, 0.0, 0.5, 0.5000001, 1.5, 2.9, 3.0, 3.1])
    assert cpu_ref.rgi_nearest_index(g, x).tolist() == [-1, 0, 0, 1, 1, 3, 3, -1]
    assert cpu_ref.rgi_nearest_index(g[::-1], x).tolist() == [-1, 3, 3, 2, 2, 0, 0, -1]
    assert cpu_ref.rgi_nearest_index(np.array([2.0]), np.array([2.0, 2.5])).tolist() == [0, -1]


def test_idw_radius_oracle_matches_bruteforce():
    """The fixed-radius IDW restatement (an extension; parity unpinned) against a brute-force
    evaluation of its definition: d2 <= r*r, w = 1/(d**p + 1e-10), sum(w v)/sum(w), NaN if empty."""
    rng = np.random.default_rng(5)
    P = rng.uniform(0, 10, (500, 3))
    Q = rng.standard_normal((500, 3))
    q = rng.uniform(0, 10, (300, 3))
    for r, p in ((1.0, 2.0), (2.5, 1.5), (0.3, 2.0)):
        got = cpu_ref.idw_radius_points(P, Q, q, r, power=p)
        for i in range(len(q)):
            dd = q[i] - P
            d2 = (dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]) + dd[:, 2] * dd[:, 2]
            sel = d2 <= r * r
            if not sel.any():
                assert np.isnan(got[i]).all()
                continue
            w = 1.0 / (np.sqrt(d2[sel]) ** p + 1e-10)
            np.testing.assert_allclose(got[i], (w[:, None] * Q[sel]).sum(0) / w.sum(), rtol=1e-13, atol=1e-15)


@pytest.mark.parametrize("name", names(("linear_",)))
def test_linear_oracle_matches_reference(name):
    """method='linear' restatement (Delaunay.find_simplex + interpnd arithmetic) against the
    reference interpolate_field fixtures, bit for bit."""
    from oracle import cpu_ref

    g = load(name)
    out = cpu_ref.linear_grid(g["points"], g["values"], g["ax"], g["ay"], g["az"])
    for a, c in zip(out, "UVW"):
        assert np.array_equal(a, g[c])
