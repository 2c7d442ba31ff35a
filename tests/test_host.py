"""Host-side logic of the drop-in module (no GPU): grid construction and
introspection, argument validation mirroring the reference's exceptions,
I/O helpers, mask resampling and boundary particles vs the reference's outputs."""
import numpy as np
import pandas as pd
import pytest

from ptv_interpolation_amd import interpolator as ip
from ptv_interpolation_amd import synth
from tests._util import load


def test_create_grid_matches_reference_axes():
    g = load("idw_aniso_k13")
    (X, Y, Z), (x, y, z) = ip.create_grid(((-3.2, 5.1), (10.0, 14.0), (0.5, 2.0)), (20, 12, 9))
    assert np.array_equal(x, g["ax"]) and np.array_equal(y, g["ay"]) and np.array_equal(z, g["az"])
    assert X.shape == (9, 12, 20)
    assert np.array_equal(X[3, 4, :], x) and np.array_equal(Y[2, :, 5], y) and np.array_equal(Z[:, 1, 1], z)


def test_create_grid_views_equal_dense():
    (Xd, Yd, Zd), _ = ip.create_grid(((0, 7), (1, 9), (2, 6)), (7, 8, 4))
    (Xv, Yv, Zv), _ = ip.create_grid(((0, 7), (1, 9), (2, 6)), (7, 8, 4), dense=False)
    for a, b in ((Xd, Xv), (Yd, Yv), (Zd, Zv)):
        assert a.shape == b.shape and np.array_equal(a, b)


def test_separable_axes_detection():
    (X, Y, Z), (x, y, z) = ip.create_grid(((0, 10), (0, 6), (0, 4)), (10, 6, 4))
    ax, ay, az = ip.separable_axes(X, Y, Z)
    assert np.array_equal(ax, x) and np.array_equal(ay, y) and np.array_equal(az, z)
    (Xv, Yv, Zv), _ = ip.create_grid(((0, 10), (0, 6), (0, 4)), (10, 6, 4), dense=False)
    assert ip.separable_axes(Xv, Yv, Zv) is not None
    X2 = X.copy(); X2[1, 2, 3] += 0.5
    assert ip.separable_axes(X2, Y, Z) is None
    assert ip.separable_axes(X.ravel(), Y.ravel(), Z.ravel()) is None
    # a zero-stride view varying along the WRONG axis (x values along z) is not separable
    (Xc, Yc, Zc), (xc, _, _) = ip.create_grid(((0, 5), (0, 5), (0, 5)), 5, dense=False)
    assert ip.separable_axes(Xc, Yc, Zc) is not None
    assert ip.separable_axes(np.broadcast_to(xc[:, None, None], Xc.shape), Yc, Zc) is None


def _df(n=20, seed=0):
    r = np.random.default_rng(seed)
    P = r.uniform(0, 5, (n, 3)); Q = r.standard_normal((n, 3))
    return pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})


def test_reference_exceptions_before_any_gpu_call(capsys):
    """k=1 -> AxisError, k>N -> IndexError, as the reference raises (interpolator.py:139-153)."""
    grid, _ = ip.create_grid(((0, 4),) * 3, 4)
    df = _df(10)
    with pytest.raises(np.exceptions.AxisError):
        ip.interpolate_field(df, grid, method="idw", idw_neighbors=1)
    with pytest.raises(IndexError):
        ip.interpolate_field(df, grid, method="idw", idw_neighbors=11)
    with pytest.raises(np.exceptions.AxisError):
        ip.interpolate_field(df, grid, method="sibson", sibson_neighbors=1)
    out = capsys.readouterr().out
    assert "Using IDW Interpolation (power=2.0, neighbors=1)..." in out
    assert "Using Sibson (Natural Neighbor) Interpolation (neighbors=1)..." in out


def test_griddata_methods_pass_through():
    """'cubic' stays scipy griddata (interpolator.py:196-197), which rejects 3-D data exactly as
    in the reference; 'linear' runs on the GPU (tests/test_gpu_linear.py) and, with no GPU
    visible, fails loudly instead of falling back to the CPU."""
    grid, _ = ip.create_grid(((0, 4),) * 3, 4)
    with pytest.raises(ValueError, match="cubic"):
        ip.interpolate_field(_df(60), grid, method="cubic")
    from ptv_interpolation_amd import _lib

    if _lib.device_count() == 0:
        with pytest.raises((ValueError, _lib.PtvError)):
            ip.interpolate_field(_df(60), grid, method="linear")


def test_load_ptv_data_renames(tmp_path):
    p = tmp_path / "p.csv"
    pd.DataFrame({"x": [0.0, 1.0], "y": [0.0, 1.0], "z": [0.0, 1.0], "vx": [1.0, 2.0], "vy": [0.0, 0.0],
                  "vz": [3.0, 4.0]}).to_csv(p, index=False)
    df = ip.load_ptv_data(str(p))
    assert list(df["u"]) == [1.0, 2.0] and list(df["w"]) == [3.0, 4.0]
    bad = tmp_path / "b.csv"
    pd.DataFrame({"x": [0.0]}).to_csv(bad, index=False)
    with pytest.raises(IOError):
        ip.load_ptv_data(str(bad))


@pytest.mark.gpu
def test_mask_sampling_and_boundary_particles_match_reference():
    g = load("masked_spherepack_idw")
    fluid = g["fluid_raw"]
    G = fluid.shape[0]
    bounds = ((0, G),) * 3
    (X, Y, Z), _ = ip.create_grid(bounds, (32, 32, 32))
    assert np.array_equal(ip.sample_mask_on_grid(fluid, (X, Y, Z), bounds), g["mask"])
    bx, by, bz = ip.extract_boundary_particles(fluid, bounds, sampling_step=3, thickness=1)
    nb = len(bx)
    P = g["points"]
    assert np.array_equal(P[-nb:, 0], bx) and np.array_equal(P[-nb:, 1], by) and np.array_equal(P[-nb:, 2], bz)


def test_sphere_pack_is_seeded_and_exact_count():
    P1, Q1 = synth.sphere_pack(5000, 40)
    P2, Q2 = synth.sphere_pack(5000, 40)
    assert P1.shape == (5000, 3) and np.array_equal(P1, P2)
    assert (P1 >= 0).all() and (P1 <= 39).all()
    assert (Q1[:, 2] == 1.0).all() and (Q1[:, :2] == 0.0).all()
    # no particle inside a sphere (generate_sphere_pack.py:50-54, :95-97)
    lo, hi = synth.LO, synth.HI
    D = lo + P1 / 39.0 * (hi - lo)
    assert not synth.inside_spheres(D[:, 0], D[:, 1], D[:, 2]).any()


def test_rbf_argument_resolution_matches_scipy():
    """LocalRBFInterpolator raises what scipy's RBFInterpolator raises (_rbfinterp.py:258-345),
    before any GPU call."""
    import warnings

    from scipy.interpolate import RBFInterpolator

    from ptv_interpolation_amd.rbf import LocalRBFInterpolator

    rng = np.random.default_rng(0)
    P, D = rng.uniform(0, 5, (30, 3)), rng.standard_normal((30, 3))
    bad = [dict(kernel="nope"), dict(kernel="gaussian"), dict(degree=-2), dict(neighbors=3, degree=1),
           dict(smoothing=np.ones(7))]
    for kw in bad:
        kw.setdefault("neighbors", 10)
        with pytest.raises(Exception) as ref:
            RBFInterpolator(P, D, **kw)
        with pytest.raises(type(ref.value)) as mine:
            LocalRBFInterpolator(P, D, **kw)
        assert str(mine.value)[:24] == str(ref.value)[:24]
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        LocalRBFInterpolator(P, D, neighbors=10, kernel="thin_plate_spline", degree=0)
    assert any(issubclass(x.category, UserWarning) for x in w)
    it = LocalRBFInterpolator(P, D, neighbors=50)  # k clamps to n (_rbfinterp.py:322)
    assert it.neighbors == 30 and it.degree == 1 and it.epsilon == 1.0


def test_divergence_host_rules_before_any_gpu_call():
    """physics mirror: the reference's exceptions and numpy's promotion, decided on the host."""
    from ptv_interpolation_amd import physics

    f = np.zeros((3, 4, 5))
    with pytest.raises(np.exceptions.AxisError):
        physics.compute_consistent_divergence(f, f, f, None, 1.0, 1.0, 1.0)
    with pytest.raises(NotImplementedError):
        physics.compute_consistent_divergence(f, f.astype(np.float32), f, f > 0, 1.0, 1.0, 1.0)
    f32 = np.empty(0, np.float32).dtype
    assert physics._result_dtype(f32, 0.5) == np.float32
    assert physics._result_dtype(f32, np.float64(0.5)) == np.float64
    assert physics._result_dtype(np.dtype(np.float64), np.float32(0.5)) == np.float64
    x = np.linspace(0, 9, 10)
    assert physics._result_dtype(f32, x[1] - x[0]) == np.float64  # view_divergence.py:22


def test_launcher_slabs_and_device_list(monkeypatch):
    from ptv_interpolation_amd import launcher

    assert launcher.slab_bounds(10, 3) == [(0, 3), (3, 6), (6, 10)]
    assert launcher.slab_bounds(2, 8) == [(0, 1), (1, 2)]
    assert launcher.slab_bounds(512, 8)[-1] == (448, 512)
    monkeypatch.setenv("PTV_DEVICES", "0, 2,3")
    assert launcher.devices() == [0, 2, 3]
    monkeypatch.setenv("PTV_DEVICE", "5")
    assert launcher.devices() == [5]


def test_launcher_recuts_slabs_from_measured_costs(monkeypatch):
    """launcher.run_slabs re-cuts the slab bounds of later calls with the same balance key from the
    slabs' device times (zslab.balanced_bounds), only after calls whose slabs all ran culled, at
    most MAX_RECUTS times; a call without a key keeps even slabs.  (No GPU: contexts are stubbed.)"""
    import numpy as np

    from ptv_interpolation_amd import launcher

    monkeypatch.setenv("PTV_DEVICES", "0,0,0,0")
    monkeypatch.delenv("PTV_DEVICE", raising=False)
    monkeypatch.setattr(launcher, "context", lambda d, slot: ("ctx", d, slot))
    monkeypatch.setattr(launcher, "_balance", {})
    nz = 128
    dens = np.where(np.arange(nz) < 32, 4.0, 1.0)  # the first quarter of the planes costs 4x
    cold = [True]

    def fn(ctx, z0, z1, views):
        for v in views:
            v[...] = z0
        n = 1000
        return {"ms_bin": 0.0, "ms_cull": 0.0, "ms_lattice": 0.0, "ms_knn": float(dens[z0:z1].sum()),
                "n_particles": n, "n_binned": n if cold[0] else n // 4}

    out = [np.empty((nz, 2, 2)) for _ in range(3)]
    even = [0, 32, 64, 96, 128]
    launcher.run_slabs(nz, fn, out, balance_key="k")
    assert launcher.current_bounds(nz, 4, "k") == even  # a cold call measures binning, not planes
    cold[0] = False
    launcher.run_slabs(nz, fn, out, balance_key="k")
    b1 = launcher.current_bounds(nz, 4, "k")
    assert b1 != even and b1[0] == 0 and b1[-1] == nz and b1[1] < 32
    costs = lambda b: [dens[b[i]:b[i + 1]].sum() for i in range(4)]  # noqa: E731
    assert max(costs(b1)) < max(costs(even))
    launcher.run_slabs(nz, fn, out, balance_key="k")
    b2 = launcher.current_bounds(nz, 4, "k")
    launcher.run_slabs(nz, fn, out, balance_key="k")
    assert launcher.current_bounds(nz, 4, "k") == b2  # MAX_RECUTS = 2 reached
    assert launcher.current_bounds(nz, 4, "other") == even
    # the slabs written follow the bounds in use
    assert [out[0][z, 0, 0] for z in b2[:-1]] == b2[:-1]
