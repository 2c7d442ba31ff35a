"""GPU parity of the local-RBF path (``method='rbf'``, interpolator.py:157-195) through the
C ABI (``ptv_interp_rbf_local``), against the reference golden vectors and the oracle
(``oracle.cpu_ref.rbf_local_points``).  Runs only on an MI355X (``-m gpu``).

Bar: normwise max|d|/max|ref| per component.  The per-voxel solve is a
dense LU with partial pivoting; the GPU factors unblocked (one row per lane) where
scipy's LAPACK dgetrf is blocked, so the results agree to the conditioning of the
systems, not bit for bit:

* TOL = 1e-10 for every case whose systems have cond <= 1e8 (all reference-reachable
  kernels at the fixture sizes: TPS, cubic, quintic, linear; cond 4e2 .. 2e7);
* TOL_ILL = 1e-8 for the Gaussian eps=0.3 fixtures (cond up to 6e8), where two CPU
  LAPACK builds (numpy's and scipy's OpenBLAS) already differ by 1.6e-9.
"""
import numpy as np
import pandas as pd
import pytest

from tests._util import load, names, normwise

pytestmark = pytest.mark.gpu

TOL = 1e-10
TOL_ILL = 1e-8
TRUTH_FACTOR = 1.0  # GPU distance to the exact answer vs the CPU LAPACKs' (see the Gaussian test)


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


def _df(points, values):
    return pd.DataFrame({c: points[:, i] for i, c in enumerate("xyz")} | {c: values[:, i] for i, c in enumerate("uvw")})


def _tol(g):
    return TOL_ILL if str(g["kernel"]) == "gaussian" else TOL


@pytest.mark.parametrize("name", [n for n in names(("rbf",)) if "gaussian" not in n])
def test_golden_dropin(ctx, name, capsys):
    """interpolate_field(method='rbf') on the reference's own fixtures (reachable kernels)."""
    from ptv_interpolation_amd import interpolator as ip

    g = load(name)
    n = len(g["ax"])
    (X, Y, Z), _ = ip.create_grid(((0, n),) * 3, n)
    assert np.array_equal(X[0, 0], g["ax"])
    U, V, W = ip.interpolate_field(_df(g["points"], g["values"]), (X, Y, Z), method="rbf",
                                   rbf_neighbors=int(g["k"]), rbf_kernel=str(g["kernel"]),
                                   smoothing=float(g["smoothing"]))
    out = capsys.readouterr().out
    assert out.startswith(f"Using RBF Interpolation ({g['kernel']}) with {int(g['k'])} neighbors, "
                          f"smoothing={float(g['smoothing'])} and n_jobs=1...")
    assert f"Interpolating {n ** 3} points serially..." in out
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        assert a.shape == b.shape and a.dtype == np.float64
        assert normwise(a, b) <= _tol(g)


@pytest.mark.parametrize("name", [n for n in names(("rbf",)) if "gaussian" in n])
def test_golden_gaussian_scipy_oracle(ctx, name):
    """RBFInterpolator(kernel='gaussian', epsilon=0.3, degree=0/-1) — scipy oracle cases.

    These systems have cond up to 6e8, and no float64 solver reaches the 1e-10 bar on them:
    tests/golden/make_golden.py (rbf_truth_cases) solved the same float64 systems in
    extended precision and measured scipy's own dgesv result (the golden U, V, W) 0.8e-9 to
    2.4e-9 normwise away from that exact answer, numpy's LAPACK 1.0e-9 to 1.7e-9
    (``gap_scipy`` / ``gap_numpy`` in truth_<name>.npz).  The bar for the GPU is therefore
    the reference's own accuracy: its distance to the exact answer must stay within
    TRUTH_FACTOR x the worse of the two CPU LAPACK distances, per component (and within
    TOL_ILL of scipy's result).  The achieved errors are printed (pytest -s / the log)."""
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    g = load(name)
    t = load("truth_" + name)
    it = LocalRBFInterpolator(g["points"], g["values"], neighbors=int(g["k"]), kernel="gaussian",
                              epsilon=float(g["epsilon"]), degree=int(g["degree"]),
                              smoothing=float(g["smoothing"]))
    U, V, W = it.evaluate_grid(g["ax"], g["ay"], g["az"])
    for i, (c, a) in enumerate(zip("UVW", (U, V, W))):
        e_ref, e_exact = normwise(a, g[c]), normwise(a, t[c])
        gap = max(float(t["gap_scipy"][i]), float(t["gap_numpy"][i]))
        print(f"{name} {c}: gpu-vs-scipy {e_ref:.3e}  gpu-vs-exact {e_exact:.3e}  "
              f"scipy-vs-exact {float(t['gap_scipy'][i]):.3e}  numpy-vs-exact {float(t['gap_numpy'][i]):.3e}")
        assert e_exact <= max(TOL, TRUTH_FACTOR * gap)
        assert e_ref <= TOL_ILL


def _rand_case(seed, n, G, lo=0.0, hi=None):
    rng = np.random.default_rng(seed)
    hi = float(G - 1) if hi is None else hi
    P = rng.uniform(lo - 0.5, hi + 0.5, (n, 3))
    Q = rng.standard_normal((n, 3))
    ax = np.linspace(lo, hi, G)
    return P, Q, ax


@pytest.mark.parametrize("kernel,k,degree,eps", [
    ("thin_plate_spline", 20, None, None),
    ("thin_plate_spline", 32, None, None),
    ("cubic", 8, None, None),
    ("quintic", 30, None, None),
    ("linear", 50, None, None),
    ("multiquadric", 24, None, 0.8),
    ("inverse_multiquadric", 24, None, 0.8),
    ("inverse_quadratic", 24, 1, 0.8),
    ("gaussian", 32, -1, 1.0),
    ("gaussian", 60, 0, 1.5),
    ("thin_plate_spline", 54, 2, None),
])
def test_random_vs_oracle(ctx, kernel, k, degree, eps):
    """Every scipy kernel, system sizes 12..64 (each padded size class), against the oracle."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(k * 7 + len(kernel), 6000, 16)
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel, epsilon=eps, degree=degree)
    U, V, W = it.evaluate_grid(ax, ax, ax)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, k, kernel, eps, degree)
    for a, b in zip((U, V, W), ref):
        assert normwise(a, b) <= TOL


@pytest.mark.parametrize("kernel,k,degree,eps", [
    ("thin_plate_spline", 64, None, None),   # m = 68: the reference default kernel past 64
    ("quintic", 60, None, None),             # m = 70
    ("cubic", 100, None, None),              # m = 104
    ("linear", 124, None, None),             # m = 128, the largest system
    ("inverse_multiquadric", 90, -1, 0.8),   # SPD kernel past the register kernels' 32
])
def test_large_systems_vs_oracle(ctx, kernel, k, degree, eps):
    """Systems of 64 < m <= 128 (k_rbf_big: one wave per voxel, the system in LDS) against the
    oracle; RBFInterpolator(neighbors=k) accepts any k (interpolator.py:162-167)."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(k * 11 + len(kernel), 5000, 8)
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel, epsilon=eps, degree=degree)
    U, V, W = it.evaluate_grid(ax, ax, ax)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, k, kernel, eps, degree)
    for a, b in zip((U, V, W), ref):
        err = normwise(a, b)
        print(f"{kernel} k={k}: normwise {err:.2e}")
        assert err <= TOL


@pytest.mark.parametrize("kernel,k,degree,eps", [
    ("thin_plate_spline", 126, None, None),  # m = 130: past the LDS kernel
    ("quintic", 126, None, None),            # m = 136
    ("linear", 150, None, None),             # m = 154, k >= 128: the large-k slot search too
    ("inverse_multiquadric", 200, -1, 0.8),  # m = 200
])
def test_huge_systems_vs_oracle(ctx, kernel, k, degree, eps):
    """Systems of m > 128 (k_rbf_huge: the system in a global-memory slice per workgroup) and
    neighbour counts k >= 128 (the large-k slot search, ptv_knn_big.hip) against the oracle:
    RBFInterpolator(neighbors=k) takes any k (interpolator.py:162-167)."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(k * 13 + len(kernel), 4000, 6)
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel, epsilon=eps, degree=degree)
    U, V, W = it.evaluate_grid(ax, ax, ax)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, k, kernel, eps, degree)
    # the larger systems are worse conditioned: the bar is the exact answer of the same systems
    # (extended precision), gpu-vs-exact <= max(1e-10, TRUTH_FACTOR x lapack-vs-exact), as for C3
    Z, Y, X = np.meshgrid(ax, ax, ax, indexing="ij")
    q = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    ext = cpu_ref.rbf_local_points(P, Q, q, k, kernel, eps, degree, solver="extended")
    for c, (a, b) in enumerate(zip((U, V, W), ref)):
        e_ref = normwise(a, b)
        e_exact = normwise(a.ravel(), ext[:, c])
        gap = normwise(b.ravel(), ext[:, c])
        print(f"{kernel} k={k} m={k + it.nmonos}: gpu-vs-lapack {e_ref:.2e}, "
              f"gpu-vs-exact {e_exact:.2e}, lapack-vs-exact {gap:.2e}")
        assert e_exact <= max(TOL, TRUTH_FACTOR * gap)


def test_smoothing_scalar_and_per_point(ctx):
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(11, 4000, 12)
    sm = np.random.default_rng(12).uniform(0.0, 3.0, len(P))
    for s in (5.0, sm):
        U, V, W = LocalRBFInterpolator(P, Q, neighbors=24, smoothing=s).evaluate_grid(ax, ax, ax)
        ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, 24, smoothing=s)
        for a, b in zip((U, V, W), ref):
            assert normwise(a, b) <= TOL


def test_point_list_call_and_extra_components(ctx):
    """__call__ on an (Q, 3) list; 5 value components go through in groups of three."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(21)
    P = rng.uniform(0, 10, (3000, 3))
    D = rng.standard_normal((3000, 5))
    X = rng.uniform(-1, 11, (777, 3))
    out = LocalRBFInterpolator(P, D, neighbors=16, kernel="cubic")(X)
    assert out.shape == (777, 5)
    ref = cpu_ref.rbf_local_points(P, D, X, 16, "cubic")
    for c in range(5):
        assert normwise(out[:, c], ref[:, c]) <= TOL


def test_z_slab_and_chunking_equal_whole(ctx):
    """Chunked k-NN + solve launches and z-slab calls give the whole-grid result bit for bit."""
    P, Q, ax = _rand_case(31, 5000, 20)
    k = 20
    whole = ctx.interp_rbf(P, Q, axes=(ax, ax, ax), k=k)
    chunked = ctx.interp_rbf(P, Q, axes=(ax, ax, ax), k=k, chunk_planes=4)
    slab = ctx.interp_rbf(P, Q, axes=(ax, ax, ax), k=k, z_range=(8, 16))
    for a, b, c in zip(whole, chunked, slab):
        assert np.array_equal(a, b)
        assert np.array_equal(a[8:16], c)


def test_mask_and_nan_to_num(ctx):
    from ptv_interpolation_amd import _lib

    P, Q, ax = _rand_case(41, 4000, 12)
    mask = np.random.default_rng(42).uniform(size=(12, 12, 12)) < 0.6
    full = ctx.interp_rbf(P, Q, axes=(ax, ax, ax), k=20)
    m = ctx.interp_rbf(P, Q, axes=(ax, ax, ax), k=20, fluid_mask=mask, flags=_lib.FLAG_NAN_TO_NUM)
    for a, b in zip(full, m):
        assert np.array_equal(a[mask], b[mask])
        assert (b[~mask] == 0).all()


def test_singular_system_raises_linalgerror(ctx):
    """Coplanar particles leave the TPS linear-polynomial block rank deficient (an exactly
    zero column): scipy's dgesv reports info > 0 and RBFInterpolator raises LinAlgError."""
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(5)
    P = rng.uniform(0, 4, (40, 3))
    P[:, 2] = 1.0
    Q = rng.standard_normal((40, 3))
    ax = np.linspace(0, 3, 4)
    with pytest.raises(np.linalg.LinAlgError, match="Singular matrix"):
        LocalRBFInterpolator(P, Q, neighbors=20).evaluate_grid(ax, ax, ax)


def test_singular_count_once_after_list_overflow(ctx):
    """Every voxel of a coplanar particle set is singular (TPS degree 1): the null-space kernel flags
    all 32^3 voxels of the one chunk, more than its list holds, and the chunk is re-solved by the
    pivoting kernel.  The singular voxels must be counted once (the rerun used to add its counts to
    the first pass's), so the reported count is exactly the voxel count."""
    import re

    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(15)
    P = rng.uniform(0, 31, (4000, 3))
    P[:, 2] = 15.5
    Q = rng.standard_normal((len(P), 3))
    ax = np.linspace(0, 31, 32)
    with pytest.raises(np.linalg.LinAlgError, match="Singular matrix") as ei:
        LocalRBFInterpolator(P, Q, neighbors=20).evaluate_grid(ax, ax, ax)
    m = re.search(r"\((\d+) voxel system", str(ei.value))
    print("reported:", str(ei.value)[:120], "| pivoted:", ctx.last_stats()["n_rbf_pivoted"])
    assert m is not None and int(m.group(1)) == 32 ** 3


def test_full_size_sampled(ctx):
    """C3 shape at a reduced grid: 128^3 over a 5M-particle-density sphere pack slice, TPS k=32,
    checked on 3000 random voxels against the oracle."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(77)
    G = 128
    n = 5_000_000 * G ** 3 // 512 ** 3
    P = rng.uniform(-0.5, G - 0.5, (n, 3))
    Q = rng.standard_normal((n, 3))
    ax = np.arange(G, dtype=np.float64)
    it = LocalRBFInterpolator(P, Q, neighbors=32, kernel="thin_plate_spline")
    U, V, W = it.evaluate_grid(ax, ax, ax)
    sel = rng.integers(0, G ** 3, 3000)
    iz, iy, ix = np.unravel_index(sel, (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], -1)
    ref = cpu_ref.rbf_local_points(P, Q, q, 32, "thin_plate_spline")
    for c, a in enumerate((U, V, W)):
        assert normwise(a.ravel()[sel], ref[:, c]) <= TOL


def test_extreme_pivots_take_the_ieee_path(ctx):
    """Pivots outside the v_rcp_f64 + Newton range (|p| >= 2^1020: smoothing 2e307 on every
    fifth diagonal) take LAPACK dgetf2's IEEE reciprocal; results stay finite and match the
    oracle.  (At 1e308 LAPACK itself overflows to NaN on some voxels.)"""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(61, 3000, 10)
    sm = np.zeros(len(P))
    sm[::5] = 2e307
    U, V, W = LocalRBFInterpolator(P, Q, neighbors=20, smoothing=sm).evaluate_grid(ax, ax, ax)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, 20, smoothing=sm)
    for a, b in zip((U, V, W), ref):
        assert np.isfinite(a).all()
        assert normwise(a, b) <= TOL


def test_c3_full_size_gaussian_sampled(ctx):
    """C3 (BASELINE configs[2]): 512^3 grid, 5M sphere-pack particles, local Gaussian RBF
    eps = 0.3, degree -1 (32 x 32 systems), k = 32, the whole grid on the GPU, 3000 random
    voxels against the oracle (scipy KDTree + LAPACK gesv per voxel) and against the exact
    answer of the same systems (extended precision).  Bar: gpu-vs-exact within
    max(1e-10, TRUTH_FACTOR x lapack-vs-exact); the achieved errors are printed."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import synth
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    G = 512
    P, Q = synth.sphere_pack(5_000_000, G, values="normal")
    ax = np.linspace(0, G - 1, G)
    it = LocalRBFInterpolator(P, Q, neighbors=32, kernel="gaussian", epsilon=0.3, degree=-1)
    out = it.evaluate_grid(ax, ax, ax)
    rng = np.random.default_rng(2024)
    sel = rng.integers(0, G ** 3, 3000)
    iz, iy, ix = np.unravel_index(sel, (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], -1)
    lap = cpu_ref.rbf_local_points(P, Q, q, 32, "gaussian", 0.3, -1)
    ext = cpu_ref.rbf_local_points(P, Q, q, 32, "gaussian", 0.3, -1, solver="extended")
    for c, a in enumerate(out):
        got = a.ravel()[sel]
        e_ref, e_exact, gap = normwise(got, lap[:, c]), normwise(got, ext[:, c]), normwise(lap[:, c], ext[:, c])
        print(f"C3 {'UVW'[c]}: gpu-vs-lapack {e_ref:.3e}  gpu-vs-exact {e_exact:.3e}  lapack-vs-exact {gap:.3e}")
        assert e_exact <= max(TOL, TRUTH_FACTOR * gap)


def test_spd_register_kernel_rerun_matches_lds_kernel(ctx, monkeypatch):
    """SPD systems (gaussian, degree -1) run k_rbf_spd16 (v_rcp_f64 + Newton reciprocals only);
    a pivot outside that range (here: scalar smoothing 2e307 puts every diagonal pivot above
    2^1020) makes the host rerun the launch with k_rbf_spd, which adds the IEEE division for such
    pivots.  Both kernels eliminate in the same order with the same reciprocals wherever the
    fast one serves; their evaluation sums differ in order (16-lane rows of two entries vs a
    32-lane segment sum), so on these ill-conditioned systems they agree to TOL_ILL (checked on
    a normal case with PTV_FLAG_RBF_SPD_LDS forcing the LDS kernel), and the rerun matches the oracle."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(63, 4000, 12)
    fast = LocalRBFInterpolator(P, Q, neighbors=32, kernel="gaussian", epsilon=0.3, degree=-1).evaluate_grid(ax, ax, ax)
    lds = LocalRBFInterpolator(P, Q, neighbors=32, kernel="gaussian", epsilon=0.3, degree=-1).evaluate_grid(
        ax, ax, ax, flags=_lib.FLAG_RBF_SPD_LDS)
    assert any(not np.array_equal(a, b) for a, b in zip(fast, lds))  # two different kernels ran
    for a, b in zip(fast, lds):
        assert normwise(a, b) <= TOL_ILL
    big = LocalRBFInterpolator(P, Q, neighbors=32, kernel="gaussian", epsilon=0.3, degree=-1,
                               smoothing=2e307).evaluate_grid(ax, ax, ax)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, 32, kernel="gaussian", epsilon=0.3, degree=-1, smoothing=2e307)
    for a, b in zip(big, ref):
        assert np.isfinite(a).all()
        assert normwise(a, b) <= TOL


@pytest.mark.parametrize("kernel,k,degree", [
    ("thin_plate_spline", 20, None),  # main.py:34-35 default: 24 x 24 systems, 20 row slots
    ("thin_plate_spline", 32, None),  # C3's reachable half: 32 row slots
    ("thin_plate_spline", 23, None),  # 24 row slots, one padded row
    ("cubic", 14, None),              # 16 row slots
    ("linear", 30, None),             # one monomial
])
def test_nullspace_vs_pivoting_and_oracle(ctx, kernel, k, degree):
    """The scale-invariant kernels run the null-space solver k_rbf_ns (static elimination order:
    Householder QR of the polynomial block, LU without pivoting of the projected SPD block); the
    partial-pivoting kernel (PTV_FLAG_RBF_PIVOTING) and the oracle's LAPACK gesv solve the same
    systems.  Both GPU kernels must meet the bar against the oracle, and they must differ somewhere
    (two different solvers ran).  The achieved errors are printed."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(k * 13 + len(kernel), 5000, 14)
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel, degree=degree)
    ns = it.evaluate_grid(ax, ax, ax)
    assert ctx.stats["n_rbf_pivoted"] == 0
    piv = it.evaluate_grid(ax, ax, ax, flags=_lib.FLAG_RBF_PIVOTING)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, k, kernel, None, degree)
    gz, gy, gx = np.meshgrid(ax, ax, ax, indexing="ij")
    ext = cpu_ref.rbf_local_points(P, Q, np.stack([gx.ravel(), gy.ravel(), gz.ravel()], -1), k, kernel,
                                   degree=degree, solver="extended")
    assert any(not np.array_equal(a, b) for a, b in zip(ns, piv))
    for c, (a, b, r) in enumerate(zip(ns, piv, ref)):
        e_ns, e_piv = normwise(a, r), normwise(b, r)
        x = ext[:, c]
        t_ns, t_piv, t_lap = normwise(a.ravel(), x), normwise(b.ravel(), x), normwise(r.ravel(), x)
        print(f"{kernel} k={k} {'UVW'[c]}: null-space vs oracle {e_ns:.2e}, pivoting vs oracle {e_piv:.2e}; "
              f"vs exact: null-space {t_ns:.2e}, pivoting {t_piv:.2e}, lapack {t_lap:.2e}")
        assert e_ns <= TOL and e_piv <= TOL


@pytest.mark.parametrize("kernel,k,degree", [("quintic", 22, None), ("thin_plate_spline", 18, 2)])
def test_ten_monomials_take_the_pivoting_kernel(ctx, kernel, k, degree):
    """Degree-2 polynomial tails (ten monomials: the quintic's minimum, or a raised TPS degree) are
    solved by the partial-pivoting kernel: the null-space route lost 100x LAPACK's accuracy on the
    sphere pack's void voxels (1.2e-10 from the exact answer).  The default path is the pivoting
    path bit for bit and meets the bar against the oracle."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(k * 13 + len(kernel), 5000, 14)
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel, degree=degree)
    dflt = it.evaluate_grid(ax, ax, ax)
    piv = it.evaluate_grid(ax, ax, ax, flags=_lib.FLAG_RBF_PIVOTING)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, k, kernel, None, degree)
    for a, b, r in zip(dflt, piv, ref):
        assert np.array_equal(a, b)
        assert normwise(a, r) <= TOL


def test_nullspace_hands_rank_deficient_voxels_to_pivoting(ctx):
    """A neighbourhood whose particles are coplanar has a rank-deficient polynomial block: the
    null-space solver flags it and the pivoting kernel re-solves it (list mode).  Here a plane of
    particles sits inside a random cloud: voxels near the plane whose k nearest all lie in it are
    handed over (singular: LinAlgError, as scipy); with smoothing and a cloud dense enough that
    no voxel's neighbourhood is planar, nothing is handed over."""
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(8)
    cloud = rng.uniform(0, 12, (3000, 3))
    g = np.arange(0, 12, 0.25)
    px, py = np.meshgrid(g, g, indexing="ij")
    plane = np.stack([px.ravel(), py.ravel(), np.full(px.size, 6.0)], -1)
    P = np.concatenate([cloud, plane])
    Q = rng.standard_normal((len(P), 3))
    ax = np.linspace(0, 11, 12)
    with pytest.raises(np.linalg.LinAlgError, match="Singular matrix"):
        LocalRBFInterpolator(P, Q, neighbors=20).evaluate_grid(ax, ax, ax)
    n = ctx.last_stats()["n_rbf_pivoted"]
    print("voxels handed to the pivoting kernel:", n)
    assert 0 < n < 12 ** 3


def test_nullspace_list_overflow_reruns_with_pivoting(ctx):
    """Extreme smoothing on every particle puts every pivot of the projected block outside the
    Newton reciprocal's range: every voxel is flagged, more than the 16384 the list holds per
    launch, and the host reruns the launch on the pivoting kernel; the result matches the oracle
    and the stats report every voxel as pivoted."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q, ax = _rand_case(71, 6000, 27)
    sm = np.full(len(P), 2e307)
    U, V, W = LocalRBFInterpolator(P, Q, neighbors=20, smoothing=sm).evaluate_grid(ax, ax, ax)
    assert ctx.stats["n_rbf_pivoted"] == 27 ** 3
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ax, ax, 20, smoothing=sm)
    for a, b in zip((U, V, W), ref):
        assert np.isfinite(a).all()
        assert normwise(a, b) <= TOL


def test_nullspace_overflow_reruns_only_its_chunk(ctx):
    """Two z-chunks (chunk_planes=20 over 40 planes): smoothing above the null-space kernel's 2^26
    limit on the particles below z = 18 makes the first chunk flag more voxels than the 16384-entry
    list holds, so that chunk
    alone is re-solved by the pivoting kernel; the second keeps the null-space solve.  The stats
    count every voxel of the rerun chunk plus the second chunk's flagged ones.  The mixed smoothing
    (1e8 next to 0) leaves the systems ill-conditioned, so the bar is the C3 one: gpu-vs-exact within
    max(1e-10, lapack-vs-exact) per component (extended-precision truth of the same systems)."""
    from oracle import cpu_ref

    rng = np.random.default_rng(72)
    P = rng.uniform(-0.5, 32.5, (40000, 3))
    P[:, 2] = rng.uniform(-0.5, 40.5, 40000)
    Q = rng.standard_normal((40000, 3))
    sm = np.where(P[:, 2] < 18.0, 1e8, 0.0)
    ax, az = np.arange(32, dtype=np.float64), np.arange(40, dtype=np.float64)
    U, V, W = ctx.interp_rbf(P, Q, axes=(ax, ax, az), k=20, smoothing=sm, chunk_planes=20)
    npiv = ctx.stats["n_rbf_pivoted"]
    print("voxels solved by the pivoting kernel:", npiv)
    assert 20 * 32 * 32 <= npiv < 40 * 32 * 32
    rng2 = np.random.default_rng(3)
    sel = rng2.integers(0, 40 * 32 * 32, 2000)
    iz, iy, ix = np.unravel_index(sel, (40, 32, 32))
    q = np.stack([ax[ix], ax[iy], az[iz]], -1)
    lap = cpu_ref.rbf_local_points(P, Q, q, 20, smoothing=sm)
    ext = cpu_ref.rbf_local_points(P, Q, q, 20, smoothing=sm, solver="extended")
    for c, a in enumerate((U, V, W)):
        assert np.isfinite(a).all()
        got = a.ravel()[sel]
        e_exact, gap = normwise(got, ext[:, c]), normwise(lap[:, c], ext[:, c])
        print(f"{'UVW'[c]}: gpu-vs-exact {e_exact:.3e}  lapack-vs-exact {gap:.3e}")
        assert e_exact <= max(TOL, gap)


@pytest.mark.parametrize("shape", [(1, 1, 1), (1, 1, 3), (2, 3, 5), (1, 7, 1)])
@pytest.mark.parametrize("kernel,k,eps,degree", [
    ("thin_plate_spline", 20, None, None),  # k_rbf_ns<20, 4>
    ("gaussian", 32, 1.5, -1),              # k_rbf_spd16<32>
])
def test_persistent_kernels_on_tiny_grids(ctx, shape, kernel, k, eps, degree):
    """The persistent null-space and SPD kernels take quads (4 voxels) from per-XCD ranges of an
    occupancy-sized grid: grids of fewer voxels than one quad, one block or one XCD's share (most
    waves and whole XCDs idle, a partial last quad) match the oracle."""
    from oracle import cpu_ref
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(sum(shape) * 7 + k)
    P = rng.uniform(0, 6, (400, 3))
    Q = rng.standard_normal((400, 3))
    nz, ny, nx = shape
    ax, ay, az = (np.linspace(1.0, 5.0, n) for n in (nx, ny, nz))
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel, epsilon=eps, degree=degree)
    got = it.evaluate_grid(ax, ay, az)
    ref = cpu_ref.rbf_local_grid(P, Q, ax, ay, az, k, kernel, eps, degree)
    for a, b in zip(got, ref):
        assert a.shape == (nz, ny, nx)
        assert normwise(a, b) <= TOL_ILL if kernel == "gaussian" else normwise(a, b) <= TOL


def _interior_biased_voxels(G, n, rng, frac_inside=0.4):
    """n voxel indices of a G^3 sphere-pack grid, at least `frac_inside` of them inside the solid
    spheres (void voxels: their neighbourhoods come from a sphere shell), the rest uniform."""
    from ptv_interpolation_amd import synth

    scale = (G - 1) / (synth.HI - synth.LO)
    inside = np.empty(0, dtype=np.int64)
    while inside.size < int(n * frac_inside):
        c = rng.integers(0, G ** 3, 20 * n)
        iz, iy, ix = np.unravel_index(c, (G, G, G))
        dom = synth.LO + np.stack([ix, iy, iz], -1) / scale
        inside = np.concatenate([inside, c[synth.inside_spheres(dom[:, 0], dom[:, 1], dom[:, 2])]])
    inside = inside[: int(n * frac_inside)]
    return np.concatenate([inside, rng.integers(0, G ** 3, n - inside.size)])


@pytest.mark.parametrize("kernel,k,G,n", [
    ("thin_plate_spline", 20, 512, 5_000_000),  # main.py:34-35 default, the rbf_tps20 bench line
    ("thin_plate_spline", 32, 512, 5_000_000),  # the rbf_tps32 bench line
    ("quintic", 22, 256, 1_000_000),            # ten monomials, the worst-conditioned family
    ("cubic", 14, 256, 1_000_000),              # 16 row slots
])
def test_nullspace_sphere_pack_sampled(ctx, kernel, k, G, n):
    """k_rbf_ns on the geometry it is benched on: the whole sphere-pack grid on the GPU, 3000
    voxels (40 % inside the solid spheres, where the neighbourhoods are sphere-shell caps) against
    the oracle's LAPACK gesv and the extended-precision solve of the same systems.  Bar per
    component: gpu-vs-exact <= max(1e-10, lapack-vs-exact).  The voxels handed to the pivoting
    kernel (n_rbf_pivoted) are printed and bounded."""
    from oracle import cpu_ref
    from ptv_interpolation_amd import synth
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    P, Q = synth.sphere_pack(n, G, values="normal")
    ax = np.linspace(0, G - 1, G)
    it = LocalRBFInterpolator(P, Q, neighbors=k, kernel=kernel)
    out = it.evaluate_grid(ax, ax, ax)
    npiv = ctx.stats["n_rbf_pivoted"]
    print(f"{kernel} k={k} {G}^3/{n}: voxels handed to the pivoting kernel {npiv} ({npiv / G ** 3:.2e})")
    assert npiv <= 1e-4 * G ** 3
    rng = np.random.default_rng(4242 + k)
    sel = _interior_biased_voxels(G, 3000, rng)
    iz, iy, ix = np.unravel_index(sel, (G, G, G))
    q = np.stack([ax[ix], ax[iy], ax[iz]], -1)
    lap = cpu_ref.rbf_local_points(P, Q, q, k, kernel)
    ext = cpu_ref.rbf_local_points(P, Q, q, k, kernel, solver="extended")
    for c, a in enumerate(out):
        got = a.ravel()[sel]
        e_ref, e_exact, gap = normwise(got, lap[:, c]), normwise(got, ext[:, c]), normwise(lap[:, c], ext[:, c])
        print(f"{kernel} k={k} {'UVW'[c]}: gpu-vs-lapack {e_ref:.3e}  gpu-vs-exact {e_exact:.3e}  "
              f"lapack-vs-exact {gap:.3e}")
        assert e_exact <= max(TOL, gap)


def test_nullspace_coincident_neighbours_take_pivoting_verdict(ctx):
    """A particle duplicated at the same position makes every system whose k nearest hold both
    copies exactly singular (e_i - e_j lies in the null space of P^T and of Phi).  The null-space
    solver's last pivot then comes out ~1e-16 relative with either sign; the relative pivot test
    hands such voxels to the pivoting kernel, so the default path reaches the same verdict as
    PTV_FLAG_RBF_PIVOTING (LAPACK's: an exactly zero pivot, LinAlgError)."""
    from ptv_interpolation_amd import _lib
    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(99)
    cloud = rng.uniform(0, 12, (3000, 3))
    P = np.concatenate([cloud, cloud[:1]])
    P[-1] = P[0]
    Q = rng.standard_normal((len(P), 3))
    ax = np.linspace(0, 11, 12)
    verdicts = []
    for flags in (0, _lib.FLAG_RBF_PIVOTING):
        try:
            LocalRBFInterpolator(P, Q, neighbors=20).evaluate_grid(ax, ax, ax, flags=flags)
            verdicts.append("solved")
        except np.linalg.LinAlgError:
            verdicts.append("singular")
        if flags == 0:
            npiv = ctx.last_stats()["n_rbf_pivoted"]
            print("voxels handed to the pivoting kernel:", npiv)
            assert npiv > 0
    assert verdicts == ["singular", "singular"]
    # without the duplicate (the same cloud) nothing is handed over and the result is finite
    U, V, W = LocalRBFInterpolator(cloud, Q[:-1], neighbors=20).evaluate_grid(ax, ax, ax)
    assert ctx.last_stats()["n_rbf_pivoted"] == 0 and np.isfinite(U).all()
