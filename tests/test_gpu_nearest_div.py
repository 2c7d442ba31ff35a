"""GPU parity for the two §8(f) rows built on the hot path:

* ``interpolate_field(method='nearest')`` (interpolator.py:196-197: griddata ->
  NearestNDInterpolator, a k = 1 KDTree query) on the k-NN kernel: bit-exact against
  the reference golden vector and the oracle (voxels whose two nearest particles are
  equidistant are tie-order dependent and excluded, as in test_gpu_parity.py);
* ``physics.compute_consistent_divergence`` (physics.py:6-53) on the stencil kernel:
  bit-exact, same dtype, against the reference golden vectors, the oracle at ragged
  sizes, and z-slab launches with one-plane halos against the whole field.
"""
import numpy as np
import pandas as pd
import pytest

from oracle import cpu_ref
from tests._util import boundary_ties, load, names

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


# ---------------------------------------------------------------- nearest
def test_nearest_golden(ctx):
    from ptv_interpolation_amd import _lib

    g = load("nearest_small")
    axes = (g["ax"], g["ay"], g["az"])
    U, V, W = ctx.interp_knn(g["points"], g["values"], axes=axes, method=_lib.METHOD_NEAREST, k=1)
    keep = ~boundary_ties(g["points"], *axes, 1)
    for a, b in ((U, g["U"]), (V, g["V"]), (W, g["W"])):
        assert np.array_equal(a[keep], b[keep])


def test_nearest_interpolate_field_sphere_pack():
    """Host mirror, sphere-pack geometry (voids exercise the coarse-lattice bounds)."""
    from ptv_interpolation_amd import interpolator as ip
    from ptv_interpolation_amd import synth

    P, Q = synth.sphere_pack(30000, 64, values="normal")
    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
    (X, Y, Z), (x, y, z) = ip.create_grid(((0, 64),) * 3, 64)
    U, V, W = ip.interpolate_field(df, (X, Y, Z), method="nearest")
    Ur, Vr, Wr = cpu_ref.interp_grid(P, Q, x, y, z, "nearest")
    keep = ~boundary_ties(P, x, y, z, 1)
    for a, b in ((U, Ur), (V, Vr), (W, Wr)):
        assert np.array_equal(a[keep], b[keep])


def test_nearest_point_list_grid():
    """Non-separable grid (point-list mode) through interpolate_field."""
    from ptv_interpolation_amd import interpolator as ip

    rng = np.random.default_rng(5)
    P = rng.uniform(0, 10, (2000, 3)); Q = rng.standard_normal((2000, 3))
    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "u": Q[:, 0], "v": Q[:, 1], "w": Q[:, 2]})
    G = rng.uniform(0, 10, (3, 7, 9, 11))
    U, V, W = ip.interpolate_field(df, (G[0], G[1], G[2]), method="nearest")
    ref = cpu_ref.interp_points(P, Q, np.stack([G[0].ravel(), G[1].ravel(), G[2].ravel()], -1), "nearest")
    assert np.array_equal(U.ravel(), ref[:, 0]) and np.array_equal(W.ravel(), ref[:, 2])


# ---------------------------------------------------------------- divergence
def _spacings(g):
    return [g[k] if int(g["spacing_np64"]) else float(g[k]) for k in ("dx", "dy", "dz")]


@pytest.mark.parametrize("name", names(("div_",)))
def test_divergence_golden(ctx, name):
    from ptv_interpolation_amd import physics

    g = load(name)
    d = physics.compute_consistent_divergence(g["u"], g["v"], g["w"], g["mask"], *_spacings(g))
    assert d.dtype == g["div"].dtype
    assert np.array_equal(d, g["div"]), f"{np.sum(d != g['div'])} voxels differ"


@pytest.mark.parametrize("shape,dt,h", [((33, 70, 129), np.float64, (0.7, 1.3, 0.9)),
                                        ((17, 65, 67), np.float32, (1.1, 0.6, 2.5)),
                                        ((2, 1, 300), np.float64, (1.0, 1.0, 1.0)),
                                        ((40, 48, 64), np.float32, (np.float64(0.25),) * 3)])
def test_divergence_ragged_vs_oracle(ctx, shape, dt, h):
    from ptv_interpolation_amd import physics

    rng = np.random.default_rng(hash(shape) % 2**32)
    u, v, w = (rng.standard_normal(shape).astype(dt) for _ in range(3))
    m = rng.uniform(size=shape) < 0.6
    d = physics.compute_consistent_divergence(u, v, w, m, *h)
    r = cpu_ref.consistent_divergence(u, v, w, m, *h)
    assert d.dtype == r.dtype and np.array_equal(d, r)


def test_divergence_zslabs_with_halos_equal_whole(ctx):
    """each z-slab computed from its planes plus a one-plane halo on each
    interior side equals the whole-field result (what each rank does)."""
    rng = np.random.default_rng(3)
    shape = (37, 40, 72)
    u, v, w = (rng.standard_normal(shape) for _ in range(3))
    m = rng.uniform(size=shape) < 0.7
    whole = cpu_ref.consistent_divergence(u, v, w, m, 0.5, 0.5, 0.5)
    P = 4
    cuts = np.linspace(0, shape[0], P + 1).astype(int)
    for r in range(P):
        s, e = cuts[r], cuts[r + 1]
        lo, hi = max(s - 1, 0), min(e + 1, shape[0])
        sl = slice(lo, hi)
        out = ctx.divergence(u[sl], v[sl], w[sl], m[sl], 0.5, 0.5, 0.5, z_range=(s - lo, e - lo),
                             edges=(lo == 0 and s == 0, hi == shape[0] and e == shape[0]))
        assert np.array_equal(out, whole[s:e]), r


def test_divergence_rejects_missing_halo(ctx):
    u = np.zeros((6, 4, 4))
    with pytest.raises(ValueError, match="halo"):
        ctx.divergence(u, u, u, u > 0, 1.0, 1.0, 1.0, z_range=(0, 6), edges=(False, True))


def test_divergence_device_pointers(ctx):
    """ptv_divergence_dev on HBM-resident torch tensors (the bench path)."""
    import torch

    from ptv_interpolation_amd import _lib

    rng = np.random.default_rng(8)
    shape = (24, 40, 96)
    f = [rng.standard_normal(shape).astype(np.float32) for _ in range(3)]
    m = rng.uniform(size=shape) < 0.5
    dev = [torch.from_numpy(a).cuda() for a in f]
    dm = torch.from_numpy(m.view(np.uint8)).cuda()
    out = torch.empty(shape, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.divergence_dev(shape[2], shape[1], shape[0], [t.data_ptr() for t in dev], dm.data_ptr(), out.data_ptr(),
                       0.5, 0.25, 2.0, field_dtype=_lib.F32, result_dtype=_lib.F32,
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    r = cpu_ref.consistent_divergence(*f, m, 0.5, 0.25, 2.0)
    assert np.array_equal(out.cpu().numpy(), r)
