"""Drop-in replacement for the reference ``interpolator`` module (MI355X path).

Same public names and signatures as tombultreys/ptv_interpolation
``interpolator.py`` so ``main.py``, ``test_parallel.py`` and the dataset run
scripts import it unchanged (put this repo first on ``PYTHONPATH``; the repo
root ``interpolator.py`` re-exports this module):

    load_ptv_data        interpolator.py:9-26
    load_mask            interpolator.py:28-39
    create_grid          interpolator.py:41-60
    interpolate_field    interpolator.py:65-203   <- idw / sibson run on the GPU
    sample_mask_on_grid  interpolator.py:205-238
    extract_boundary_particles  interpolator.py:240-284

``interpolate_field(method='idw'|'sibson'|'nearest'|'rbf'|'linear')`` runs the k-NN search
and the weighted average (or the local RBF solve) as HIP kernels through the C ABI
(include/ptv_api.h).  There is no CPU fallback for these methods: a missing library
or GPU raises.  Results reproduce the reference arithmetic (see
ptv_interpolation_amd/csrc/ptv_knn.hip); ``n_jobs`` is accepted and ignored by the
GPU methods (the reference uses it only for RBF, interpolator.py:173).  ``nearest``
is a scipy ``griddata`` call in the reference (interpolator.py:196-197), i.e. a k = 1
KDTree query, and runs on the same k-NN kernel here.  ``linear`` (the reference default,
griddata -> LinearNDInterpolator) triangulates with the same scipy Delaunay (Qhull) call on
the host and locates / interpolates every voxel on the GPU (ptv_linear.hip).  ``cubic``
stays a scipy ``griddata`` call (it raises for 3-D data, as in the reference).
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib, launcher

__all__ = [
    "load_ptv_data",
    "load_mask",
    "create_grid",
    "interpolate_field",
    "sample_mask_on_grid",
    "extract_boundary_particles",
]

_EPS = 1e-10  # interpolator.py:102, :142


# ---------------------------------------------------------------------------
# I/O and grid helpers (host side, same behaviour as the reference)
# ---------------------------------------------------------------------------
def load_ptv_data(filepath):
    """CSV -> DataFrame with columns x, y, z, u, v, w (vx/vy/vz renamed); interpolator.py:9-26."""
    import pandas as pd

    try:
        df = pd.read_csv(filepath)
        df.rename(columns={"vx": "u", "vy": "v", "vz": "w"}, inplace=True)
        need = {"x", "y", "z", "u", "v", "w"}
        if not need.issubset(df.columns):
            raise ValueError(f"CSV must contain columns: {need}")
        return df
    except Exception as e:  # the reference wraps every failure as IOError
        raise IOError(f"Error reading {filepath}: {e}")


def load_mask(filepath):
    """3-D TIFF -> bool (True = fluid, i.e. > 0); interpolator.py:28-39."""
    try:
        import tifffile

        return tifffile.imread(filepath) > 0
    except Exception as e:
        raise IOError(f"Error reading mask {filepath}: {e}")


def create_grid(bounds, resolution, dense=True):
    """Regular grid: axes ``linspace(min, max-1, n)``; (X, Y, Z) of shape (nz, ny, nx).

    interpolator.py:41-60.  ``dense=False`` returns read-only zero-stride
    broadcast views with identical shape and values (no 3*8*V-byte meshgrids);
    ``interpolate_field`` recognises either form as a separable grid.
    """
    (xmin, xmax), (ymin, ymax), (zmin, zmax) = bounds
    if isinstance(resolution, int):
        nx = ny = nz = resolution
    else:
        nx, ny, nz = resolution
    x = np.linspace(xmin, xmax - 1, nx)
    y = np.linspace(ymin, ymax - 1, ny)
    z = np.linspace(zmin, zmax - 1, nz)
    if dense:
        Z, Y, X = np.meshgrid(z, y, x, indexing="ij")
    else:
        shape = (nz, ny, nx)
        X = np.broadcast_to(x[None, None, :], shape)
        Y = np.broadcast_to(y[None, :, None], shape)
        Z = np.broadcast_to(z[:, None, None], shape)
    return (X, Y, Z), (x, y, z)


def sample_mask_on_grid(mask_raw, grid_tuple, bounds_raw):
    """Nearest-neighbour resampling of a raw mask onto the grid; interpolator.py:205-238.

    The reference builds ``RegularGridInterpolator((z, y, x), mask_raw.astype(float),
    method='nearest', bounds_error=False, fill_value=0)`` over the raw axes
    ``linspace(min, max-1, n)`` and thresholds the samples at 0.5.  Here the raw mask goes
    to the GPU as bytes (1 = value > 0.5; a bool mask as is) and ``ptv_sample_mask`` does
    the per-voxel nearest lookup (scipy's interval search + ``t <= 0.5`` rule, out of
    bounds -> 0) and the gather (ptv_interpolation_amd/csrc/ptv_mask.hip).
    """
    raw = np.asarray(mask_raw)
    nz, ny, nx = raw.shape
    (xmin, xmax), (ymin, ymax), (zmin, zmax) = bounds_raw
    X, Y, Z = grid_tuple
    axes = []
    for lo, hi, n in ((xmin, xmax, nx), (ymin, ymax, ny), (zmin, zmax, nz)):
        axes.append(np.linspace(lo, hi - 1, n) if n > 1 else np.array([lo], dtype=np.float64))
    if raw.dtype == np.bool_:
        raw_bytes = raw.view(np.uint8)
    else:
        raw_bytes = (raw.astype(float) > 0.5).view(np.uint8)
    ctx = _lib.Context.get(_gpu_device())
    sep = separable_axes(X, Y, Z)
    shape = np.shape(X)
    if sep is not None:
        out = ctx.sample_mask(raw_bytes, axes, axes=sep)
    else:
        n = int(np.size(X))
        out = ctx.sample_mask(raw_bytes, axes, grid_points=(np.ravel(X), np.ravel(Y), np.ravel(Z)),
                              shape=(1, 1, n))
    return out.view(np.bool_).reshape(shape)


def extract_boundary_particles(mask, bounds, sampling_step=1, thickness=1):
    """Solid voxels within `thickness` 6-connected steps of fluid -> coordinates; interpolator.py:240-284.

    ``binary_dilation(mask, generate_binary_structure(3, 1), iterations=thickness) & ~mask``,
    ``np.where`` (C order), ``[::sampling_step]`` and ``lo + idx * (hi - 1 - lo) / (n - 1)``
    run on the GPU (``ptv_boundary_particles``: dilation passes, a fused last pass with a
    per-block count, a scan, and an ordered emit).
    """
    if mask is None:
        return np.array([]), np.array([]), np.array([])
    m = np.asarray(mask)
    nz, ny, nx = m.shape
    (xmin, xmax), (ymin, ymax), (zmin, zmax) = bounds
    if m.dtype == np.bool_:
        mb, enc = m.view(np.uint8), _lib.MASK_BOOL
    else:
        _ = ~m.reshape(-1)[:1]  # the reference's `~mask` (TypeError for float masks)
        mb = ((m != 0).astype(np.uint8) << 1) | (m & 1).astype(np.uint8)
        enc = _lib.MASK_BITS
    # scipy: iterations < 1 repeats the dilation until nothing changes; nx + ny + nz
    # passes reach every voxel of the box
    t = int(thickness) if thickness >= 1 else nx + ny + nz
    step = int(sampling_step) if sampling_step > 1 else 1
    lo = (xmin, ymin, zmin)
    span = (xmax - 1 - xmin, ymax - 1 - ymin, zmax - 1 - zmin)
    ns = (nx, ny, nz)
    den = tuple(float(n - 1) if n > 1 else 1.0 for n in ns)
    ctx = _lib.Context.get(_gpu_device())
    coords = ctx.boundary_particles(mb, enc, t, step, [float(v) for v in lo], [float(v) for v in span], den)
    if len(coords[0]) == 0:
        return np.array([]), np.array([]), np.array([])
    out = []
    for c, n, l in zip(coords, ns, lo):
        # n == 1: np.full_like(int64 indices, min) in the reference
        out.append(c if n > 1 else np.full_like(np.empty(len(c), dtype=np.int64), l))
    return tuple(out)


# ---------------------------------------------------------------------------
# grid introspection
# ---------------------------------------------------------------------------
def separable_axes(X, Y, Z):
    """Return (ax, ay, az) if (X, Y, Z) is an (nz, ny, nx) meshgrid(z, y, x, 'ij'), else None."""
    X, Y, Z = np.asarray(X), np.asarray(Y), np.asarray(Z)
    if X.ndim != 3 or X.shape != Y.shape or X.shape != Z.shape or X.size == 0:
        return None
    ax = np.ascontiguousarray(X[0, 0, :], dtype=np.float64)
    ay = np.ascontiguousarray(Y[0, :, 0], dtype=np.float64)
    az = np.ascontiguousarray(Z[:, 0, 0], dtype=np.float64)

    def zero_stride(A, axis):
        # zero-stride broadcast view (create_grid(dense=False)): constant along the two other
        # axes by construction, provided the one nonzero stride sits on `axis`
        return all(A.strides[d] == 0 for d in range(3) if d != axis)

    checks = [(A, ref) for A, ref, axis in ((X, ax[None, None, :], 2), (Y, ay[None, :, None], 1),
                                            (Z, az[:, None, None], 0)) if not zero_stride(A, axis)]
    if not checks:
        return ax, ay, az
    # dense meshgrids (main.py:151 passes create_grid's): every element must match its axis
    # value.  Cheap rejections first (corner planes), then the full comparison over z-chunks
    # on a thread pool (numpy releases the GIL): 3 x 1 GiB at 512^3 read once, in parallel.
    nz = X.shape[0]
    for A, ref in checks:
        for z in {0, nz - 1}:
            if not np.array_equal(A[z], np.broadcast_to(ref[min(z, ref.shape[0] - 1)], A.shape[1:])):
                return None
    return (ax, ay, az) if _all_match(checks, nz) else None


def _all_match(checks, nz):
    """Whether every (A, ref) pair has A == broadcast(ref) elementwise, checked over z-chunks
    on up to 16 threads with an early stop."""
    from concurrent.futures import ThreadPoolExecutor

    plane = int(np.prod(checks[0][0].shape[1:]))
    step = max(1, (1 << 21) // max(plane, 1))  # ~2M elements per task
    chunks = [(a, min(nz, a + step)) for a in range(0, nz, step)]
    bad = []

    def run(ch):
        if bad:
            return
        a, b = ch
        for A, ref in checks:
            r = ref[a:b] if ref.shape[0] > 1 else ref
            if not np.array_equal(A[a:b], np.broadcast_to(r, A[a:b].shape)):
                bad.append(ch)
                return

    if len(chunks) == 1:
        run(chunks[0])
    else:
        with ThreadPoolExecutor(min(16, len(chunks), os.cpu_count() or 1)) as ex:
            list(ex.map(run, chunks))
    return not bad


def _gpu_device():
    """The device of single-device calls (mask path): PTV_DEVICE, else the first of launcher.devices()."""
    return launcher.devices()[0]


def _knn_field(points, values, grid_tuple, method, k, power, radius=0.0):
    """GPU k-NN IDW/Sibson (or fixed-radius IDW) over the caller's grid; returns (U, V, W)
    with X's shape."""
    X, Y, Z = grid_tuple
    shape = np.shape(X)
    n = points.n if isinstance(points, _lib.ParticleColumns) else points.shape[0]
    if method == "idw_radius":
        # extension (no reference counterpart): k is not used
        if not (np.isfinite(radius) and radius > 0):
            raise ValueError(f"idw_radius must be a positive finite number, got {radius}")
        if n == 0:
            raise ValueError("no particles to interpolate from")
        k = 1
    else:
        if k < 1:
            raise ValueError(f"k must be a positive integer, got {k}")
        if n == 0:
            raise ValueError("no particles to interpolate from")
        if k == 1 and method != "nearest":
            # the reference's KDTree.query(k=1) squeezes to (V,), then .sum(axis=1) fails
            raise np.exceptions.AxisError("axis 1 is out of bounds for array of dimension 1")
        if k > n:
            # KDTree pads missing neighbours with index n; values[indices] then fails
            raise IndexError(f"index {n} is out of bounds for axis 0 with size {n}")
    m = {"idw": _lib.METHOD_IDW, "sibson": _lib.METHOD_SIBSON, "nearest": _lib.METHOD_NEAREST,
         "idw_radius": _lib.METHOD_IDW_RADIUS}[method]
    axes = separable_axes(X, Y, Z)
    if axes is not None:
        # z-slab per device (launcher.py); bit-identical to one whole-grid call.  With several
        # slabs each one bins only the particles that can reach its planes (PTV_FLAG_SLAB_CULL_AUTO:
        # a per-column cull map the slab's context derives from its own lattice bounds on the first
        # call and proves exact on the device on every later call with the same particles), as the
        # north_star z-slab partition does (zslab.py)
        nz = len(axes[2])
        flags = _lib.FLAG_SLAB_CULL_AUTO if (launcher.slab_count(nz) > 1 and method != "idw_radius") else 0

        def slab(ctx, z0, z1, views):
            ctx.interp_knn(points, values, axes=axes, method=m, k=k, power=power, eps=_EPS, z_range=(z0, z1),
                           out=views, radius=radius, flags=flags)
            return dict(ctx.stats)

        full = [np.empty((nz, len(axes[1]), len(axes[0]))) for _ in range(3)]
        # later calls on this grid re-cut the slabs from these slabs' measured device times
        U, V, W = launcher.run_slabs(nz, slab, full, balance_key=("knn", m, k) if flags else None)
    else:
        ctx = _lib.Context.get(launcher.devices()[0])
        size = int(np.prod(shape))
        g = [np.ascontiguousarray(np.asarray(A, dtype=np.float64)).reshape(-1) for A in (X, Y, Z)]
        sh = tuple(shape) if len(shape) == 3 else (1, 1, size)
        U, V, W = ctx.interp_knn(points, values, grid_points=g, shape=sh, method=m, k=k, power=power, eps=_EPS,
                                 radius=radius)
    return U.reshape(shape), V.reshape(shape), W.reshape(shape)


def interpolate_field(df, grid_tuple, method="linear", rbf_neighbors=20, rbf_kernel="thin_plate_spline",
                      smoothing=0.0, n_jobs=1, idw_power=2.0, idw_neighbors=50, sibson_neighbors=30,
                      idw_radius=None):
    """Interpolate PTV particles onto the grid (interpolator.py:65-203 signature and semantics).

    Returns ``(U, V, W)`` float64 arrays of the grid's shape.

    ``idw_radius`` (extension, not in the reference): with ``method='idw'``, weight every particle
    within this distance of the voxel (scipy ``query_ball_point``'s ``d**2 <= r*r`` test) instead
    of the ``idw_neighbors`` nearest; same weights ``1/(d**idw_power + 1e-10)``; a voxel with no
    particle in its ball is NaN.  Parity unpinned (the reference has no radius search); tested
    against ``oracle.cpu_ref.idw_radius_points`` to 1e-12 normwise.
    """
    X, Y, Z = grid_tuple
    # interpolator.py:78-79 (float64 coercion); the k-NN methods take the DataFrame's columns
    # as they are (a float64 block's rows are contiguous: no (N, 3) gathers or column copies)
    cols = _lib.ParticleColumns.from_frame(df)

    if method == "sibson":
        print(f"Using Sibson (Natural Neighbor) Interpolation (neighbors={sibson_neighbors})...")
        return _knn_field(cols, None, grid_tuple, "sibson", int(sibson_neighbors), 2.0)
    if method == "idw" and idw_radius is not None:
        print(f"Using IDW Interpolation (power={idw_power}, radius={idw_radius})...")
        return _knn_field(cols, None, grid_tuple, "idw_radius", 1, float(idw_power), float(idw_radius))
    if method == "idw":
        print(f"Using IDW Interpolation (power={idw_power}, neighbors={idw_neighbors})...")
        return _knn_field(cols, None, grid_tuple, "idw", int(idw_neighbors), float(idw_power))
    points, values = cols.points, cols.values
    if method == "rbf":
        print(f"Using RBF Interpolation ({rbf_kernel}) with {rbf_neighbors} neighbors, "
              f"smoothing={smoothing} and n_jobs={n_jobs}...")
        from . import rbf as _rbf

        return _rbf.rbf_field(points, values, grid_tuple, int(rbf_neighbors), rbf_kernel, smoothing,
                              n_jobs=int(n_jobs))
    if method == "nearest":
        # griddata(method='nearest') (interpolator.py:196-197) is NearestNDInterpolator: the
        # k = 1 query of the same GPU k-NN kernel, values of the nearest particle
        return _knn_field(cols, None, grid_tuple, "nearest", 1, 2.0)
    if method == "linear":
        return _linear_field(points, values, grid_tuple)
    # 'cubic' (and anything else) goes to griddata as in the reference, which raises for 3-D data
    from scipy.interpolate import griddata

    out = griddata(points, values, (X, Y, Z), method=method, fill_value=0.0)
    return out[..., 0], out[..., 1], out[..., 2]


def _linear_field(points, values, grid_tuple, fill_value=0.0):
    """griddata(points, values, (X, Y, Z), method='linear', fill_value=0.0) (interpolator.py:197).

    The triangulation is ``scipy.spatial.Delaunay(points)`` -- the same Qhull call
    LinearNDInterpolator makes, so the simplices and barycentric transforms are the reference's
    own (and Qhull's errors for degenerate inputs are raised unchanged); every voxel's point
    location and barycentric interpolation run on the GPU (ptv_linear.hip), z-slabs over the
    devices like the k-NN methods."""
    from scipy.spatial import Delaunay

    X, Y, Z = np.broadcast_arrays(*grid_tuple)
    shape = np.shape(X)
    tri = _lib.Triangulation(Delaunay(np.ascontiguousarray(points, dtype=np.float64)))
    axes = separable_axes(X, Y, Z)
    if axes is not None:
        full = [np.empty((len(axes[2]), len(axes[1]), len(axes[0]))) for _ in range(3)]
        U, V, W = launcher.run_slabs(len(axes[2]), lambda ctx, z0, z1, views: ctx.interp_linear(
            points, values, tri, axes=axes, fill_value=fill_value, z_range=(z0, z1), out=views), full)
    else:
        ctx = _lib.Context.get(launcher.devices()[0])
        size = int(np.prod(shape))
        g = [np.ascontiguousarray(np.asarray(A, dtype=np.float64)).reshape(-1) for A in (X, Y, Z)]
        sh = tuple(shape) if len(shape) == 3 else (1, 1, size)
        U, V, W = ctx.interp_linear(points, values, tri, grid_points=g, shape=sh, fill_value=fill_value)
    return U.reshape(shape), V.reshape(shape), W.reshape(shape)
