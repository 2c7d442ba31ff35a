"""CPU restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the MI355X k-NN interpolation path.  Only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it.  Nothing under ``ptv_interpolation_amd/`` imports
it, and the shipped path never falls back to it.

What it restates (reference = tombultreys/ptv_interpolation, read-only):

* ``interpolator.interpolate_field`` IDW branch  (interpolator.py:126-155)
* ``interpolator.interpolate_field`` Sibson branch (interpolator.py:83-124)
* ``interpolator.interpolate_field`` local-RBF branch (interpolator.py:157-195)
  through scipy's ``RBFInterpolator(neighbors=k)`` evaluation
  (``_rbfinterp.py:463-556``, ``_build_system`` / ``dgesv`` :82-127): see
  ``rbf_local_points`` below
* ``interpolate_field(method='nearest')`` (interpolator.py:196-197: griddata ->
  NearestNDInterpolator, a k=1 KDTree query, values[idx]) in ``interp_points``
* ``physics.compute_consistent_divergence`` (physics.py:6-53) as
  ``consistent_divergence`` below (an independent per-axis index restatement,
  not the reference's np.roll formulation)
* ``interpolator.sample_mask_on_grid`` (interpolator.py:205-238, scipy
  ``RegularGridInterpolator(method='nearest')`` restated as a per-axis interval
  search) and ``interpolator.extract_boundary_particles`` (interpolator.py:240-284,
  ``binary_dilation`` restated as padded face shifts) as ``sample_mask_nearest`` /
  ``boundary_particles`` below
* ``filtering.remove_outliers_knn`` (filtering.py:5-58) as ``outlier_filter``
* the RBF process fan-out pattern (interpolator.py:173-182,
  test_parallel.py:6-28) as a z-slab ``ProcessPoolExecutor`` driver used as the
  same-box CPU baseline.

The k-NN search itself lives in the reference's third-party dependency
``scipy.spatial.KDTree`` (cKDTree, unpinned in requirements.txt:2; this image
ships scipy 1.15.3).  ``knn_kdtree`` calls it exactly as the reference does
(interpolator.py:132,139).  ``knn_bruteforce`` is an independent numpy
restatement of the same contract — Euclidean k nearest, ascending distance,
``d = sqrt((dx*dx + dy*dy) + dz*dz)`` (the cKDTree p=2 accumulation order,
verified bit-exact against cKDTree in this container) — used to cross-check
the tree on small cases.

Numerics pinned here (each verified bit-exact against numpy 2.2.6 in
``tests/test_oracle.py``):

* ``x.sum(axis=1)`` over a C-contiguous (V, k) array is ``0.0 + pairwise(row)``
  where ``pairwise`` is numpy's 8-accumulator blocked pairwise summation
  (``pairwise_sum`` below).
* ``d ** p`` takes numpy's scalar fast paths: p=2 -> d*d, p=1 -> d,
  p=0.5 -> sqrt(d), p=-1 -> 1/d; otherwise ``np.power``.
* ``x.std(axis=1)`` = sqrt(pairwise((x - pairwise(x)/k)**2) / k).

Parity is pinned by the golden vectors in ``tests/golden/`` that were produced
by importing the reference ``interpolator.py`` itself
(``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import math
import os
from concurrent.futures import ProcessPoolExecutor

import numpy as np

EPS = 1e-10  # interpolator.py:102 and :142


# ----------------------------------------------------------------------------
# numpy's reduction order, restated (used by the GPU epilogue contract)
# ----------------------------------------------------------------------------
def pairwise_sum(a) -> float:
    """numpy ``@TYPE@_pairwise_sum`` for a contiguous 1-D float64 run.

    n < 8: sequential from 0.0; 8 <= n <= 128: eight strided accumulators,
    ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the n%8 tail sequentially;
    n > 128: split at n/2 rounded down to a multiple of 8 and recurse.
    The reduction result is ``0.0 + pairwise_sum(row)`` (identity first).
    """
    n = len(a)
    if n < 8:
        res = 0.0
        for v in a:
            res += float(v)
        return res
    if n <= 128:
        r = [float(a[j]) for j in range(8)]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                r[j] += float(a[i + j])
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += float(a[i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise_sum(a[:n2]) + pairwise_sum(a[n2:])


def numpy_power(d: np.ndarray, p: float) -> np.ndarray:
    """``d ** p`` exactly as ndarray.__pow__ evaluates it (scalar fast paths)."""
    if p == 2.0:
        return d * d
    if p == 1.0:
        return d.copy()
    if p == 0.5:
        return np.sqrt(d)
    if p == -1.0:
        with np.errstate(divide="ignore"):
            return 1.0 / d
    return np.power(d, p)


# ----------------------------------------------------------------------------
# k-NN
# ----------------------------------------------------------------------------
def knn_kdtree(points: np.ndarray, queries: np.ndarray, k: int):
    """scipy KDTree query, as interpolator.py:132 (build) and :139 (query)."""
    from scipy.spatial import KDTree

    tree = KDTree(points)
    return tree.query(queries, k=k)


def knn_bruteforce(points: np.ndarray, queries: np.ndarray, k: int, chunk: int = 2048):
    """Exact brute-force k-NN (small cases only): ties broken by lower index.

    Distances use the cKDTree p=2 order ``(dx*dx + dy*dy) + dz*dz`` then sqrt.
    """
    points = np.ascontiguousarray(points, dtype=np.float64)
    queries = np.ascontiguousarray(queries, dtype=np.float64)
    nq = queries.shape[0]
    dist = np.empty((nq, k))
    idx = np.empty((nq, k), dtype=np.int64)
    for s in range(0, nq, chunk):
        q = queries[s : s + chunk]
        dx = q[:, None, 0] - points[None, :, 0]
        dy = q[:, None, 1] - points[None, :, 1]
        dz = q[:, None, 2] - points[None, :, 2]
        d2 = (dx * dx + dy * dy) + dz * dz
        order = np.argsort(d2, axis=1, kind="stable")[:, :k]
        idx[s : s + chunk] = order
        dist[s : s + chunk] = np.sqrt(np.take_along_axis(d2, order, axis=1))
    return dist, idx


# ----------------------------------------------------------------------------
# weights + gather-sum (the per-voxel epilogue)
# ----------------------------------------------------------------------------
def idw_weights(dist: np.ndarray, power: float, eps: float = EPS) -> np.ndarray:
    """interpolator.py:142-147 — w = 1/(d**p + eps), normalised by its row sum."""
    w = 1.0 / (numpy_power(dist, power) + eps)
    return w / w.sum(axis=1, keepdims=True)


def sibson_weights(dist: np.ndarray, eps: float = EPS) -> np.ndarray:
    """interpolator.py:102-116 — inverse-distance weights damped by exp(-d/std(d))."""
    inv = 1.0 / (dist + eps)
    w = inv / inv.sum(axis=1, keepdims=True)
    sigma = dist.std(axis=1, keepdims=True)
    with np.errstate(invalid="ignore", over="ignore", under="ignore"):
        w = w * np.exp(-dist / (sigma + eps))
        return w / w.sum(axis=1, keepdims=True)


def gather_sum(weights: np.ndarray, values: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """interpolator.py:150-153 (and :119-122): per component sum_k w * values[idx]."""
    out = np.zeros((weights.shape[0], 3))
    for c in range(3):
        out[:, c] = (weights * values[idx, c]).sum(axis=1)
    return out


def interp_points(points, values, queries, method="idw", k=8, power=2.0, knn="kdtree"):
    """Interpolate at an (M,3) query list; returns (M,3) float64 (AoS like the reference)."""
    points = np.asarray(points, dtype=np.float64)
    values = np.asarray(values, dtype=np.float64)
    queries = np.asarray(queries, dtype=np.float64).reshape(-1, 3)
    if method == "nearest":
        k = 1
    if knn == "kdtree":
        dist, idx = knn_kdtree(points, queries, k)
    else:
        dist, idx = knn_bruteforce(points, queries, k)
    if method == "nearest":
        # NearestNDInterpolator.__call__: values[i] for the single nearest particle
        return values[np.asarray(idx).reshape(-1)]
    if method == "idw":
        w = idw_weights(dist, power)
    elif method == "sibson":
        w = sibson_weights(dist)
    else:
        raise ValueError(method)
    with np.errstate(invalid="ignore"):
        return gather_sum(w, values, idx)


def idw_radius_points(points, values, queries, radius, power=2.0, eps=EPS):
    """Fixed-radius IDW -- an EXTENSION with no reference counterpart (the reference only has
    the k-NN ``tree.query``, interpolator.py:139), so parity is unpinned: this restatement
    defines it for the GPU's PTV_METHOD_IDW_RADIUS.  Per query: every particle with
    ``((dx*dx + dy*dy) + dz*dz) <= r*r`` (scipy ``KDTree.query_ball_point``'s test), weights
    ``1/(d**p + eps)`` with numpy's scalar power (as interpolator.py:142-147), and
    ``sum(w * v) / sum(w)``; an empty ball gives NaN.  Returns (M, 3) float64."""
    from scipy.spatial import KDTree

    points = np.asarray(points, dtype=np.float64)
    values = np.asarray(values, dtype=np.float64)
    q = np.asarray(queries, dtype=np.float64).reshape(-1, 3)
    out = np.full((len(q), 3), np.nan)
    for i, idx in enumerate(KDTree(points).query_ball_point(q, radius, return_sorted=True)):
        if not idx:
            continue
        dd = q[i] - points[idx]
        d = np.sqrt((dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]) + dd[:, 2] * dd[:, 2])
        w = 1.0 / (numpy_power(d, power) + eps)
        out[i] = (w[:, None] * values[idx]).sum(axis=0) / w.sum()
    return out


def grid_queries(ax, ay, az, z0=0, z1=None):
    """Voxel coordinates of the C-order (nz, ny, nx) grid, x fastest (interpolator.py:59,135)."""
    z1 = len(az) if z1 is None else z1
    Z, Y, X = np.meshgrid(np.asarray(az)[z0:z1], ay, ax, indexing="ij")
    return np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=-1)


def interp_grid(points, values, ax, ay, az, method="idw", k=8, power=2.0, z0=0, z1=None, knn="kdtree"):
    """Whole-grid (or z-slab) interpolation -> (U, V, W) each (nz', ny, nx)."""
    z1 = len(az) if z1 is None else z1
    q = grid_queries(ax, ay, az, z0, z1)
    out = interp_points(points, values, q, method, k, power, knn)
    shape = (z1 - z0, len(ay), len(ax))
    return tuple(np.ascontiguousarray(out[:, c].reshape(shape)) for c in range(3))


# ----------------------------------------------------------------------------
# local RBF (interpolator.py:157-195 -> scipy RBFInterpolator(neighbors=k))
# ----------------------------------------------------------------------------
# scipy/interpolate/_rbfinterp_pythran.py kernel functions of r = ||eps*x - eps*y||
RBF_PHI = {
    "linear": lambda r: -r,
    "thin_plate_spline": lambda r: np.where(r == 0.0, 0.0, r * r * np.log(np.where(r == 0.0, 1.0, r))),
    "cubic": lambda r: r * r * r,
    "quintic": lambda r: -(r * r * r * r * r),
    "multiquadric": lambda r: -np.sqrt(r * r + 1.0),
    "inverse_multiquadric": lambda r: 1.0 / np.sqrt(r * r + 1.0),
    "inverse_quadratic": lambda r: 1.0 / (r * r + 1.0),
    "gaussian": lambda r: np.exp(-(r * r)),
}
RBF_SCALE_INVARIANT = {"linear", "thin_plate_spline", "cubic", "quintic"}
RBF_MIN_DEGREE = {"multiquadric": 0, "linear": 0, "thin_plate_spline": 1, "cubic": 1, "quintic": 2}


def monomial_powers(degree: int, ndim: int = 3) -> np.ndarray:
    """_rbfinterp.py ``_monomial_powers``: exponents in combinations_with_replacement order."""
    from itertools import combinations_with_replacement

    rows = []
    for deg in range(degree + 1):
        for mono in combinations_with_replacement(range(ndim), deg):
            r = [0] * ndim
            for v in mono:
                r[v] += 1
            rows.append(r)
    return np.array(rows, dtype=np.int64).reshape(-1, ndim)


def _poly(xhat, powers):
    """(..., 3) -> (..., R): prod over axes of xhat ** powers[j] (``_polynomial_matrix``)."""
    return np.prod(xhat[..., None, :] ** powers, axis=-1)


def solve_extended(lhs, rhs):
    """Batched Gaussian elimination with partial pivoting in x87 extended precision
    (``np.longdouble``, 64-bit significand) of float64 systems (C, m, m) x (C, m, S).

    An accuracy reference, not the reference's algorithm: its error against the exact
    solution of the float64 system is ~cond * 2^-64, about 2000x below that of a float64
    LAPACK solve, so ``normwise(x_solver, x_extended)`` measures how far a float64 solver
    (scipy's dgesv, numpy's, the GPU's) lands from the exact answer of the same system."""
    A = np.array(lhs, dtype=np.longdouble)
    B = np.array(rhs, dtype=np.longdouble)
    C, m, _ = A.shape
    ar = np.arange(C)
    for c in range(m):
        p = c + np.argmax(np.abs(A[:, c:, c]), axis=1)
        if np.any(A[ar, p, c] == 0):
            raise np.linalg.LinAlgError("Singular matrix")
        A[:, [c], :], A[ar, p, :] = A[ar, p, :][:, None, :], A[:, c, :].copy()
        B[:, [c], :], B[ar, p, :] = B[ar, p, :][:, None, :], B[:, c, :].copy()
        l = A[:, c + 1:, c] / A[:, c, c][:, None]
        A[:, c + 1:, c:] -= l[:, :, None] * A[:, c, c:][:, None, :]
        B[:, c + 1:, :] -= l[:, :, None] * B[:, c, :][:, None, :]
    X = np.empty_like(B)
    for c in range(m - 1, -1, -1):
        acc = B[:, c, :] - np.einsum("cj,cjs->cs", A[:, c, c + 1:], X[:, c + 1:, :])
        X[:, c, :] = acc / A[:, c, c][:, None]
    return X


def rbf_local_points(points, values, queries, k, kernel="thin_plate_spline", epsilon=None, degree=None,
                     smoothing=0.0, chunk=2048, solver="lapack"):
    """RBFInterpolator(points, values, neighbors=k, kernel, epsilon, degree, smoothing)(queries).

    Per query: KDTree k nearest (``_rbfinterp.py:513``), indices sorted ascending
    (:521), system built per ``_build_system`` -- kernel block
    ``phi(||eps*y_i - eps*y_j||)`` + smoothing on the diagonal, polynomial block
    ``P((y - shift)/scale)`` with shift = (max+min)/2, scale = (max-min)/2 (0 -> 1)
    over the neighbourhood -- solved with LAPACK gesv (numpy batched solve, the same
    dgesv scipy calls at :113), evaluated as ``[phi(||eps*x - eps*y_j||), P((x -
    shift)/scale)] @ coeffs`` (:404-418).  scipy solves each *unique* neighbourhood
    once; solving it once per query gives the same coefficients.
    Returns (Q, S) float64.  Singular systems raise numpy.linalg.LinAlgError.
    """
    from scipy.spatial import KDTree

    y = np.asarray(points, dtype=np.float64)
    d = np.asarray(values, dtype=np.float64).reshape(len(y), -1)
    x = np.asarray(queries, dtype=np.float64).reshape(-1, 3)
    if epsilon is None:
        if kernel not in RBF_SCALE_INVARIANT:
            raise ValueError("`epsilon` must be specified if `kernel` is not one of scale-invariant kernels.")
        epsilon = 1.0
    if degree is None:
        degree = max(RBF_MIN_DEGREE.get(kernel, -1), 0)
    powers = monomial_powers(degree)
    k = int(min(k, len(y)))
    sm = np.broadcast_to(np.asarray(smoothing, dtype=np.float64), (len(y),))
    phi = RBF_PHI[kernel]
    R = powers.shape[0]
    m = k + R
    _, idx = KDTree(y).query(x, k)
    idx = np.sort(np.asarray(idx).reshape(len(x), k), axis=1)
    out = np.empty((len(x), d.shape[1]))
    for c0 in range(0, len(x), chunk):
        ii = idx[c0:c0 + chunk]
        yn = y[ii]  # (C, k, 3)
        mins, maxs = yn.min(axis=1), yn.max(axis=1)
        shift = (maxs + mins) / 2
        scale = (maxs - mins) / 2
        scale[scale == 0.0] = 1.0
        ye = yn * epsilon
        diff = ye[:, :, None, :] - ye[:, None, :, :]
        r = np.sqrt((diff[..., 0] ** 2 + diff[..., 1] ** 2) + diff[..., 2] ** 2)
        lhs = np.zeros((len(ii), m, m))
        lhs[:, :k, :k] = phi(r)
        lhs[:, np.arange(k), np.arange(k)] += sm[ii]
        P = _poly((yn - shift[:, None, :]) / scale[:, None, :], powers)
        lhs[:, :k, k:] = P
        lhs[:, k:, :k] = np.swapaxes(P, 1, 2)
        rhs = np.zeros((len(ii), m, d.shape[1]))
        rhs[:, :k] = d[ii]
        xq = x[c0:c0 + chunk]
        dq = xq[:, None, :] * epsilon - ye
        rq = np.sqrt((dq[..., 0] ** 2 + dq[..., 1] ** 2) + dq[..., 2] ** 2)
        vec = np.concatenate([phi(rq), _poly((xq - shift) / scale, powers)], axis=1)
        if solver == "extended":
            coeffs = solve_extended(lhs, rhs)
            out[c0:c0 + chunk] = np.einsum("qm,qms->qs", vec.astype(np.longdouble), coeffs).astype(np.float64)
        else:
            coeffs = np.linalg.solve(lhs, rhs)
            out[c0:c0 + chunk] = np.einsum("qm,qms->qs", vec, coeffs)
    return out


def rbf_local_grid(points, values, ax, ay, az, k, kernel="thin_plate_spline", epsilon=None, degree=None,
                   smoothing=0.0, z0=0, z1=None):
    """Whole-grid (or z-slab) local RBF -> (U, V, W) each (nz', ny, nx)."""
    z1 = len(az) if z1 is None else z1
    q = grid_queries(ax, ay, az, z0, z1)
    out = rbf_local_points(points, values, q, k, kernel, epsilon, degree, smoothing)
    shape = (z1 - z0, len(ay), len(ax))
    return tuple(np.ascontiguousarray(out[:, c].reshape(shape)) for c in range(3))


# ----------------------------------------------------------------------------
# multiprocess z-slab driver (interpolator.py:173-182 pattern) — CPU baseline
# ----------------------------------------------------------------------------
_W = {}


def _worker_init(points, values, ax, ay, az, method, k, power):
    _W.update(points=points, values=values, ax=ax, ay=ay, az=az, method=method, k=k, power=power)


def _worker_slab(z_range):
    z0, z1 = z_range
    w = _W
    return z0, interp_grid(w["points"], w["values"], w["ax"], w["ay"], w["az"], w["method"], w["k"], w["power"], z0, z1)


def interp_grid_parallel(points, values, ax, ay, az, method="idw", k=8, power=2.0,
                         z0=0, z1=None, n_jobs=None, slab=None):
    """Fan z-slabs over a ProcessPoolExecutor, each worker holding its own KDTree.

    Z-slab results are bit-identical to the whole-grid call for IDW/Sibson
    (each voxel depends only on its coordinate and the full particle set).
    """
    z1 = len(az) if z1 is None else z1
    n_jobs = n_jobs or os.cpu_count() or 1
    planes = z1 - z0
    slab = slab or max(1, math.ceil(planes / (4 * n_jobs)))
    ranges = [(s, min(s + slab, z1)) for s in range(z0, z1, slab)]
    shape = (planes, len(ay), len(ax))
    U, V, W = (np.empty(shape) for _ in range(3))
    with ProcessPoolExecutor(max_workers=n_jobs, initializer=_worker_init,
                             initargs=(points, values, ax, ay, az, method, k, power)) as ex:
        for s, (u, v, w) in ex.map(_worker_slab, ranges):
            U[s - z0 : s - z0 + u.shape[0]] = u
            V[s - z0 : s - z0 + u.shape[0]] = v
            W[s - z0 : s - z0 + u.shape[0]] = w
    return U, V, W


# ---------------------------------------------------------------------------
# method='linear': griddata(points, values, xi, method='linear', fill_value=0.0)
# (interpolator.py:196-197) = scipy LinearNDInterpolator: Delaunay (Qhull) + point location
# (spatial/_qhull.pyx _find_simplex) + barycentric interpolation (interpolate/interpnd.pyx
# _do_evaluate).  scipy 1.15.3 (the reference container's) is a third-party dependency; its
# published algorithm restated: Delaunay.find_simplex runs the same walk from the same start
# sequence (eps = 100 DBL_EPSILON), then
#   c_i = ((0 + T_i0 (x_0 - r_0)) + T_i1 (x_1 - r_1)) + T_i2 (x_2 - r_2), c_3 = ((1 - c_0) - c_1) - c_2
#   out = (((0 + c_0 v_s0) + c_1 v_s1) + c_2 v_s2) + c_3 v_s3,  fill_value where no simplex.
# Pinned bit-exactly by tests/golden/linear_*.npz (the reference interpolate_field itself).
# ---------------------------------------------------------------------------
def linear_points(points, values, queries, fill_value=0.0, tri=None):
    from scipy.spatial import Delaunay

    points = np.ascontiguousarray(points, dtype=np.float64)
    values = np.asarray(values, dtype=np.float64)
    q = np.ascontiguousarray(queries, dtype=np.float64).reshape(-1, 3)
    tri = Delaunay(points) if tri is None else tri
    s = tri.find_simplex(q)
    ok = s >= 0
    T = tri.transform[np.where(ok, s, 0)]
    d = q - T[:, 3, :]
    c = []
    for i in range(3):
        ci = np.zeros(len(q))
        for j in range(3):
            ci = ci + T[:, i, j] * d[:, j]
        c.append(ci)
    c.append(((1.0 - c[0]) - c[1]) - c[2])
    vv = values[tri.simplices[np.where(ok, s, 0)]]  # (m, 4, 3)
    out = np.zeros((len(q), values.shape[1]))
    for j in range(4):
        out = out + c[j][:, None] * vv[:, j]
    out[~ok] = fill_value
    return out


def linear_grid(points, values, ax, ay, az, fill_value=0.0, z0=0, z1=None):
    """(U, V, W) each (nz', ny, nx) of griddata(method='linear') on the separable grid."""
    q = grid_queries(ax, ay, az, z0, z1)
    z1 = len(az) if z1 is None else z1
    out = linear_points(points, values, q, fill_value)
    shp = (z1 - z0, len(ay), len(ax))
    return tuple(out[:, c].reshape(shp) for c in range(3))


def lattice_axis(a, step=4):
    """The library's coarse-lattice axis (ptv_api.cpp prepare / k_subsample): every `step`-th
    value of `a` plus the last."""
    a = np.asarray(a, dtype=np.float64)
    n = len(a)
    m = 1 if n <= 1 else (n - 1 + step - 1) // step + 1
    return a[np.minimum(np.arange(m) * step, n - 1)]


def slab_cull_interp(points, values, ax, ay, az, z0, z1, method="idw", k=8, power=2.0, halo=0.0):
    """Restatement of the library's slab cull (ptv_knn_params.slab_halo) for the CPU tests of the
    multi-GPU partition (tests/test_distributed.py): keep the particles with z within `halo` of
    the slab's z extent (order kept), prove exactness from the lattice k-th distances D(c) of the
    kept set (need(c) = D(c) + diag(c) + dz(c) - m(c), ptv_knn.hip k_halo_need, with exact D),
    and interpolate planes [z0, z1) from the kept set.  Returns (U, V, W, halo_required,
    n_kept); the interpolation is skipped (None) when halo_required > halo."""
    from scipy.spatial import KDTree

    P = np.asarray(points, dtype=np.float64)
    Q = np.asarray(values, dtype=np.float64)
    zs = np.asarray(az, dtype=np.float64)[z0:z1]
    zmin, zmax = zs.min(), zs.max()
    keep = (P[:, 2] >= zmin - halo) & (P[:, 2] <= zmax + halo)
    Pk, Qk = P[keep], Q[keep]
    lax, lay, laz = lattice_axis(ax), lattice_axis(ay), lattice_axis(zs)

    def step(a):
        d = np.abs(np.diff(a))
        left = np.concatenate([[0.0], d])
        right = np.concatenate([d, [0.0]])
        return np.maximum(left, right)

    Zc, Yc, Xc = np.meshgrid(laz, lay, lax, indexing="ij")
    D, _ = KDTree(Pk).query(np.stack([Xc.ravel(), Yc.ravel(), Zc.ravel()], -1), k=k)
    D = np.asarray(D).reshape(len(laz), len(lay), len(lax), -1)[..., -1]
    sz, sy, sx = np.meshgrid(step(laz), step(lay), step(lax), indexing="ij")
    diag = np.sqrt(sx ** 2 + sy ** 2 + sz ** 2)
    m = np.maximum(np.minimum(Zc - zmin, zmax - Zc), 0.0)
    required = float(max(np.max(D + diag + sz - m), 0.0))
    if required > halo:
        return None, None, None, required, int(keep.sum())
    U, V, W = interp_grid(Pk, Qk, ax, ay, az, method, k, power, z0, z1)
    return U, V, W, required, int(keep.sum())


def nan_fill_and_mask(U, V, W, fluid_mask=None):
    """main.py:195-207 caller epilogue: nan_to_num if U has a NaN, zero solid voxels."""
    if np.isnan(U).any():
        U, V, W = np.nan_to_num(U), np.nan_to_num(V), np.nan_to_num(W)
    if fluid_mask is not None:
        solid = ~fluid_mask
        U, V, W = U.copy(), V.copy(), W.copy()
        U[solid] = 0
        V[solid] = 0
        W[solid] = 0
    return U, V, W


# ----------------------------------------------------------------------------
# consistent divergence (physics.py:6-53)
# ----------------------------------------------------------------------------
def _faces(vel, fluid, axis):
    """(f_next, f_prev) of get_face_vel (physics.py:26-48) along ``axis``, by index:
    f_next[i] = (vel[i] + vel[i+1]) / 2 if fluid[i+1] else 0, = vel[i] at i = n-1;
    f_prev[i] = f_next[i-1] = (vel[i-1] + vel[i]) / 2 if fluid[i] else 0, = vel[i] at i = 0."""
    v = np.moveaxis(vel, axis, -1)
    m = np.moveaxis(fluid, axis, -1)
    zero = np.zeros((), dtype=vel.dtype)
    fn = np.empty_like(v)
    fp = np.empty_like(v)
    fn[..., :-1] = np.where(m[..., 1:], (v[..., :-1] + v[..., 1:]) / 2.0, zero)
    fn[..., -1] = v[..., -1]
    fp[..., 1:] = np.where(m[..., 1:], (v[..., :-1] + v[..., 1:]) / 2.0, zero)
    fp[..., 0] = v[..., 0]
    return np.moveaxis(fn, -1, axis), np.moveaxis(fp, -1, axis)


def consistent_divergence(u, v, w, mask, dx, dy, dz):
    """div = ((ufn - ufp)/dx + (vfn - vfp)/dy) + (wfn - wfp)/dz (physics.py:53), numpy's
    evaluation order and dtype promotion (the spacing scalars are passed through as given)."""
    fluid = np.asarray(mask).astype(bool)
    ufn, ufp = _faces(np.asarray(u), fluid, 2)
    vfn, vfp = _faces(np.asarray(v), fluid, 1)
    wfn, wfp = _faces(np.asarray(w), fluid, 0)
    return (ufn - ufp) / dx + (vfn - vfp) / dy + (wfn - wfp) / dz


# ----------------------------------------------------------------------------
# pore-mask path (interpolator.py:205-284) and the k-NN outlier filter (filtering.py:5-58)
# ----------------------------------------------------------------------------
def rgi_nearest_index(grid, x):
    """RegularGridInterpolator 'nearest' index along one axis (scipy 1.15 _rgi.py
    _find_indices / _evaluate_nearest / _find_out_of_bounds), -1 = out of bounds."""
    g = np.asarray(grid, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    n = len(g)
    flip = n > 1 and g[0] > g[-1]
    if flip:
        g = g[::-1]
    oob = (x < g[0]) | (x > g[-1]) | np.isnan(x)
    if n == 1:
        j = np.zeros(x.shape, dtype=np.int64)
    else:
        i = np.clip(np.searchsorted(g, x, side="right") - 1, 0, n - 2)
        t = (x - g[i]) / (g[i + 1] - g[i])
        j = np.where(t <= 0.5, i, i + 1)
    if flip:
        j = n - 1 - j
    return np.where(oob, -1, j)


def sample_mask_nearest(mask_raw, bounds_raw, X, Y, Z):
    """sample_mask_on_grid (interpolator.py:205-238): nearest raw voxel, 0 outside, > 0.5."""
    raw = np.asarray(mask_raw).astype(float) > 0.5
    nz, ny, nx = raw.shape
    (xmin, xmax), (ymin, ymax), (zmin, zmax) = bounds_raw
    axes = [np.linspace(lo, hi - 1, n) if n > 1 else np.array([lo], dtype=np.float64)
            for lo, hi, n in ((zmin, zmax, nz), (ymin, ymax, ny), (xmin, xmax, nx))]
    jz = rgi_nearest_index(axes[0], np.ravel(Z))
    jy = rgi_nearest_index(axes[1], np.ravel(Y))
    jx = rgi_nearest_index(axes[2], np.ravel(X))
    ok = (jz >= 0) & (jy >= 0) & (jx >= 0)
    out = np.zeros(jz.shape, dtype=bool)
    out[ok] = raw[jz[ok], jy[ok], jx[ok]]
    return out.reshape(np.shape(X))


def _dilate6(a):
    """One binary_dilation pass with the 6-connected cross and border_value 0."""
    p = np.pad(a, 1, constant_values=False)
    return (p[1:-1, 1:-1, 1:-1] | p[:-2, 1:-1, 1:-1] | p[2:, 1:-1, 1:-1] | p[1:-1, :-2, 1:-1]
            | p[1:-1, 2:, 1:-1] | p[1:-1, 1:-1, :-2] | p[1:-1, 1:-1, 2:])


def boundary_particles(mask, bounds, sampling_step=1, thickness=1):
    """extract_boundary_particles (interpolator.py:240-284), dilation restated."""
    if mask is None:
        return np.array([]), np.array([]), np.array([])
    m = np.asarray(mask)
    nz, ny, nx = m.shape
    (xmin, xmax), (ymin, ymax), (zmin, zmax) = bounds
    g = m != 0
    if thickness >= 1:
        for _ in range(thickness):
            g = _dilate6(g)
    else:  # scipy: iterate until nothing changes
        while True:
            h = _dilate6(g)
            if np.array_equal(h, g):
                break
            g = h
    iz, iy, ix = np.nonzero(g & (~m))
    if len(ix) == 0:
        return np.array([]), np.array([]), np.array([])
    if sampling_step > 1:
        iz, iy, ix = iz[::sampling_step], iy[::sampling_step], ix[::sampling_step]

    def phys(idx, lo, hi, n):
        return lo + idx * (hi - 1 - lo) / (n - 1) if n > 1 else np.full_like(idx, lo)

    return phys(ix, xmin, xmax, nx), phys(iy, ymin, ymax, ny), phys(iz, zmin, zmax, nz)


def outlier_filter(points, values, k=25, threshold=3.0, workers=1):
    """remove_outliers_knn (filtering.py:5-58) -> (keep mask, median k-th radius).

    KDTree(points).query(points, k+1) with column 0 dropped, speed median and MAD over the
    k neighbours, z = |speed - median| / (MAD + 1e-6) <= threshold."""
    from scipy.spatial import KDTree

    points = np.asarray(points, dtype=np.float64)
    u, v, w = (np.asarray(values, dtype=np.float64)[:, c] for c in range(3))
    speed = np.sqrt(u**2 + v**2 + w**2)
    dist, idx = KDTree(points).query(points, k=k + 1, workers=workers)
    nb = idx[:, 1:]
    radius = np.median(dist[:, 1:][:, -1])
    ns = speed[nb]
    med = np.median(ns, axis=1)
    mad = np.median(np.abs(ns - med[:, None]), axis=1)
    z = np.abs(speed - med) / (mad + 1e-6)
    return z <= threshold, radius
