"""PTV_FLAG_OUT_F32: U, V, W written as float32 by the k-NN kernel — the fused
`U.astype(np.float32)` of main.py:230 applied after the float64 result, the nan_to_num
(main.py:195-199) and the mask (main.py:202-207).  Required bit-exact against the float64
outputs cast with numpy (SURVEY §8(d) C5 stores the field in float32)."""
import numpy as np
import pytest

from tests._util import load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


@pytest.mark.parametrize("method,k", [("idw", 8), ("idw", 50), ("sibson", 30), ("nearest", 1)])
def test_out_f32_is_astype_of_f64(ctx, method, k):
    from ptv_interpolation_amd import _lib, synth

    P, Q = synth.sphere_pack(30000, 64, values="normal")
    Q[::97] *= 1e40  # values beyond float32 range: astype gives inf, as numpy does
    ax = np.linspace(0, 63, 64)
    m = {"idw": _lib.METHOD_IDW, "sibson": _lib.METHOD_SIBSON, "nearest": _lib.METHOD_NEAREST}[method]
    ref = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=m, k=k)
    got = ctx.interp_knn(P, Q, axes=(ax, ax, ax), method=m, k=k, flags=_lib.FLAG_OUT_F32)
    for a, b in zip(got, ref):
        assert a.dtype == np.float32
        with np.errstate(over="ignore"):
            assert np.array_equal(a, b.astype(np.float32), equal_nan=True)


def test_out_f32_masked_epilogue(ctx):
    """The masked sphere-pack fixture (main.py epilogue: NaN fill + solid zeroing) in float32:
    the cast of the float64 fused-epilogue output, zeros on solid voxels."""
    from ptv_interpolation_amd import _lib

    g = load("masked_spherepack_idw")
    axes = (g["ax"], g["ay"], g["az"])
    ref = ctx.interp_knn(g["points"], g["values"], axes=axes, k=8, fluid_mask=g["mask"], flags=_lib.FLAG_NAN_TO_NUM)
    got = ctx.interp_knn(g["points"], g["values"], axes=axes, k=8, fluid_mask=g["mask"],
                         flags=_lib.FLAG_NAN_TO_NUM | _lib.FLAG_OUT_F32)
    for a, b in zip(got, ref):
        assert a.dtype == np.float32 and np.array_equal(a, b.astype(np.float32))
        assert (a[~g["mask"]] == 0).all()


def test_out_f32_device_path(ctx):
    import torch

    from ptv_interpolation_amd import _lib, synth

    P, Q = synth.sphere_pack(20000, 48, values="normal")
    ax = np.linspace(0, 47, 48)
    ref = ctx.interp_knn(P, Q, axes=(ax, ax, ax), k=8)
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(np.ascontiguousarray(P[:, i])).to(dev) for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).to(dev) for i in range(3)]
    axes = [torch.from_numpy(ax.copy()).to(dev) for _ in range(3)]
    out = [torch.empty((48, 48, 48), dtype=torch.float32, device=dev) for _ in range(3)]
    ctx.interp_knn_dev(len(P), [c.data_ptr() for c in cols], 48, 48, 48, axes_ptrs=[a.data_ptr() for a in axes],
                       out_ptrs=[o.data_ptr() for o in out], k=8, flags=_lib.FLAG_OUT_F32)
    torch.cuda.synchronize(dev)
    for o, r in zip(out, ref):
        assert np.array_equal(o.cpu().numpy(), r.astype(np.float32))


def test_rbf_rejects_out_f32(ctx):
    from ptv_interpolation_amd import _lib

    g = load("rbf_thin_plate_spline_k20_s0.0")
    with pytest.raises(NotImplementedError):
        ctx.interp_rbf(g["points"], g["values"], axes=(g["ax"], g["ay"], g["az"]), k=20, kernel="thin_plate_spline", epsilon=1.0,
                       degree=1, flags=_lib.FLAG_OUT_F32)
