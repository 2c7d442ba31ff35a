"""Generate the golden parity fixtures by importing the reference interpolator.

Runs only where the read-only reference checkout exists (default
``/root/reference``); the GPU box never runs it, it only reads the committed
``*.npz`` files.  ``tifffile`` is not installed in this image and is only used
by the reference's TIFF I/O (interpolator.py:35, main.py:230), so a stub module
is placed in ``sys.modules`` before the import.

Every fixture stores its inputs (particles, values, 1-D grid axes, parameters)
and the reference outputs ``U, V, W`` (C-order (nz, ny, nx) float64), plus the
numpy/scipy versions they were produced with.  Particle coordinates are
continuous random draws so that no two particles tie at the k-th distance
(cKDTree's tie order is traversal dependent) except in the
explicitly-tied edge cases, which are checked normwise only.

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import contextlib
import io
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference(path):
    sys.modules.setdefault("tifffile", types.ModuleType("tifffile"))
    sys.path.insert(0, path)
    import interpolator  # noqa: E402  (the reference module)

    return interpolator


def _df(points, values):
    import pandas as pd

    return pd.DataFrame({"x": points[:, 0], "y": points[:, 1], "z": points[:, 2],
                         "u": values[:, 0], "v": values[:, 1], "w": values[:, 2]})


def _save(name, **arrays):
    import scipy

    arrays.setdefault("numpy_version", np.array(np.__version__))
    arrays.setdefault("scipy_version", np.array(scipy.__version__))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    print("wrote", name)


def _run(ref, points, values, bounds, res, **kw):
    (X, Y, Z), (x, y, z) = ref.create_grid(bounds, res)
    with contextlib.redirect_stdout(io.StringIO()):
        U, V, W = ref.interpolate_field(_df(points, values), (X, Y, Z), **kw)
    return x, y, z, np.ascontiguousarray(U), np.ascontiguousarray(V), np.ascontiguousarray(W)


def knn_cases(ref):
    rng = np.random.default_rng(20260213)

    # (1) headline-shaped IDW: k=8, p=2, unit-spaced 32^3 grid, 5k particles
    P = rng.uniform(-0.5, 31.5, (5000, 3)); Q = rng.standard_normal((5000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 32),) * 3, 32, method="idw", idw_neighbors=8, idw_power=2.0)
    _save("idw_k8_p2", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=8, power=2.0, U=U, V=V, W=W)

    # (2) IDW k=50, p=1.5 (pow path)
    P = rng.uniform(0, 23, (4000, 3)); Q = rng.standard_normal((4000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 24),) * 3, 24, method="idw", idw_neighbors=50, idw_power=1.5)
    _save("idw_k50_p1.5", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=50, power=1.5, U=U, V=V, W=W)

    # (3) reference defaults (idw_neighbors=50, idw_power=2.0; interpolator.py:65)
    P = rng.uniform(0, 19, (3000, 3)); Q = rng.standard_normal((3000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 20),) * 3, 20, method="idw")
    _save("idw_default_k50", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=50, power=2.0, U=U, V=V, W=W)

    # (4) Sibson k=30
    P = rng.uniform(0, 23, (4000, 3)); Q = rng.standard_normal((4000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 24),) * 3, 24, method="sibson", sibson_neighbors=30)
    _save("sibson_k30", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("sibson"), k=30, power=2.0, U=U, V=V, W=W)

    # (5) anisotropic grid in physical units, particles beyond the grid box, odd k
    P = np.stack([rng.uniform(-4.0, 6.0, 3000), rng.uniform(9.0, 15.0, 3000), rng.uniform(0.0, 2.5, 3000)], 1)
    Q = rng.standard_normal((3000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((-3.2, 5.1), (10.0, 14.0), (0.5, 2.0)), (20, 12, 9),
                            method="idw", idw_neighbors=13, idw_power=2.0)
    _save("idw_aniso_k13", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=13, power=2.0, U=U, V=V, W=W)

    # (6) Sibson on the same anisotropic set with the reference default k
    x, y, z, U, V, W = _run(ref, P, Q, ((-3.2, 5.1), (10.0, 14.0), (0.5, 2.0)), (20, 12, 9), method="sibson")
    _save("sibson_aniso_k30", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("sibson"), k=30, power=2.0, U=U, V=V, W=W)

    # (7) small k values and p = 1, 0.5, -1, 3 (numpy fast paths and pow)
    P = rng.uniform(0, 11, (600, 3)); Q = rng.standard_normal((600, 3))
    for k, p in ((2, 1.0), (5, 0.5), (7, -1.0), (9, 3.0), (16, 2.0), (33, 2.0), (64, 2.0)):
        x, y, z, U, V, W = _run(ref, P, Q, ((0, 12),) * 3, 12, method="idw", idw_neighbors=k, idw_power=p)
        _save(f"idw_small_k{k}_p{p}", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=k, power=p, U=U, V=V, W=W)
    for k in (2, 7, 8, 17, 64):
        x, y, z, U, V, W = _run(ref, P, Q, ((0, 12),) * 3, 12, method="sibson", sibson_neighbors=k)
        _save(f"sibson_small_k{k}", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("sibson"), k=k, power=2.0, U=U, V=V, W=W)


def edge_cases(ref):
    rng = np.random.default_rng(7)
    # voxel coincident with a particle: weight 1/(0 + 1e-10) dominates
    P = rng.uniform(0, 9, (400, 3)); P[:40] = np.round(P[:40]); Q = rng.standard_normal((400, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 10),) * 3, 10, method="idw", idw_neighbors=8)
    _save("edge_coincident_idw", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=8, power=2.0, U=U, V=V, W=W, tied=1)
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 10),) * 3, 10, method="sibson", sibson_neighbors=8)
    _save("edge_coincident_sibson", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("sibson"), k=8, power=2.0, U=U, V=V, W=W, tied=1)
    # k == N
    P = rng.uniform(0, 7, (12, 3)); Q = rng.standard_normal((12, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 8),) * 3, 8, method="idw", idw_neighbors=12)
    _save("edge_k_eq_n", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=12, power=2.0, U=U, V=V, W=W)
    # Sibson sigma = 0: the 8 corners of a cube around voxel (2,2,2) -> all distances equal -> NaN
    c = np.array([[2 + sx, 2 + sy, 2 + sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], float)
    P = np.concatenate([c, rng.uniform(6, 9, (20, 3))]); Q = rng.standard_normal((28, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 10),) * 3, 10, method="sibson", sibson_neighbors=8)
    assert np.isnan(U[2, 2, 2])
    _save("edge_sibson_sigma0", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("sibson"), k=8, power=2.0, U=U, V=V, W=W, tied=1)


def masked_case(ref):
    """main.py:78-207 masked pipeline, reproduced with the reference functions."""
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from ptv_interpolation_amd import synth

    G = 48
    fluid = synth.fluid_mask(G)                        # mask_raw (True = fluid), interpolator.py:37
    pts, _ = synth.sphere_pack(6000, G, seed=11)
    vals = np.random.default_rng(12).standard_normal((6000, 3))
    bounds = ((0, G), (0, G), (0, G))                  # main.py:105-106
    keep = (pts >= 0).all(1) & (pts < G).all(1)        # main.py:140-142
    pts, vals = pts[keep], vals[keep]
    res = (32, 32, 32)                                 # --downscale 1.5 -> round(48/1.5), main.py:115-119
    (X, Y, Z), (x, y, z) = ref.create_grid(bounds, res)
    mask = ref.sample_mask_on_grid(fluid, (X, Y, Z), bounds_raw=bounds)
    bx, by, bz = ref.extract_boundary_particles(fluid, bounds, sampling_step=3, thickness=1)
    P = np.concatenate([pts, np.stack([bx, by, bz], 1)])
    Q = np.concatenate([vals, np.zeros((len(bx), 3))])
    with contextlib.redirect_stdout(io.StringIO()):
        U, V, W = ref.interpolate_field(_df(P, Q), (X, Y, Z), method="idw", idw_neighbors=8)
    Ur, Vr, Wr = (np.ascontiguousarray(a) for a in (U, V, W))
    if np.isnan(U).any():                               # main.py:195-199
        U, V, W = np.nan_to_num(U), np.nan_to_num(V), np.nan_to_num(W)
    U, V, W = U.copy(), V.copy(), W.copy()
    U[~mask] = 0; V[~mask] = 0; W[~mask] = 0            # main.py:202-207
    _save("masked_spherepack_idw", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("idw"), k=8, power=2.0,
          mask=mask, fluid_raw=fluid, U_raw=Ur, V_raw=Vr, W_raw=Wr, U=U, V=V, W=W, tied=1)


def rbf_cases(ref):
    """Local RBF fixtures (interpolator.py:157-195 and scipy RBFInterpolator directly)."""
    from scipy.interpolate import RBFInterpolator

    rng = np.random.default_rng(99)
    P = rng.uniform(0, 11, (1500, 3)); Q = rng.standard_normal((1500, 3))
    for kern, k, s in (("thin_plate_spline", 20, 0.0), ("thin_plate_spline", 32, 5.0), ("cubic", 20, 0.0),
                       ("quintic", 24, 0.0), ("linear", 16, 0.0)):
        x, y, z, U, V, W = _run(ref, P, Q, ((0, 12),) * 3, 12, method="rbf", rbf_neighbors=k, rbf_kernel=kern, smoothing=s)
        _save(f"rbf_{kern}_k{k}_s{s}", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("rbf"),
              kernel=np.array(kern), k=k, smoothing=s, U=U, V=V, W=W)
    # Gaussian is not reachable through interpolate_field (no epsilon pass-through, interpolator.py:162-167):
    # scipy oracle only, degree 0 (33x33 at k=32) and degree -1 (32x32).
    (X, Y, Z), (x, y, z) = ref.create_grid(((0, 12),) * 3, 12)
    flat = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    for deg in (0, -1):
        out = RBFInterpolator(P, Q, neighbors=32, kernel="gaussian", epsilon=0.3, degree=deg)(flat)
        U, V, W = (np.ascontiguousarray(out[:, c].reshape(X.shape)) for c in range(3))
        _save(f"rbf_gaussian_eps0.3_k32_deg{deg}", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("rbf"),
              kernel=np.array("gaussian"), k=32, smoothing=0.0, epsilon=0.3, degree=deg, U=U, V=V, W=W)
    # test_parallel.py:6-28 input (5 particles, neighbors clamps to N)
    P5 = np.array([[0, 0, 0], [10, 0, 0], [0, 10, 0], [10, 10, 0], [5, 5, 5]], float)
    Q5 = np.array([[1, 0, 0], [1, 0, 0], [1, 0, 0], [1, 0, 0], [2, 0, 0]], float)
    x, y, z, U, V, W = _run(ref, P5, Q5, ((0, 10),) * 3, 10, method="rbf", n_jobs=1)
    _save("rbf_test_parallel", points=P5, values=Q5, ax=x, ay=y, az=z, method=np.array("rbf"),
          kernel=np.array("thin_plate_spline"), k=20, smoothing=0.0, U=U, V=V, W=W)


def nearest_cases(ref):
    """method='nearest' (interpolator.py:196-197: griddata -> NearestNDInterpolator, a k=1
    KDTree query).  Continuous draws: no two particles tie as a voxel's nearest."""
    rng = np.random.default_rng(31)
    P = rng.uniform(-0.5, 20.5, (3000, 3)); Q = rng.standard_normal((3000, 3))
    x, y, z, U, V, W = _run(ref, P, Q, ((0, 21), (0, 18), (0, 15)), (21, 18, 15), method="nearest")
    _save("nearest_small", points=P, values=Q, ax=x, ay=y, az=z, method=np.array("nearest"), k=1, power=2.0,
          U=U, V=V, W=W)


def div_cases(ref_path):
    """physics.compute_consistent_divergence (physics.py:6-53), the divergence view_divergence.py:39
    reads: float64 fields; float32 fields with Python-float spacings (float32 result) and with
    numpy float64 spacings (float64 result, view_divergence.py:22-24); a one-plane axis; and the
    masked sphere-pack IDW field of masked_case() with its grid spacing."""
    sys.path.insert(0, ref_path)
    import physics  # noqa: E402  (the reference module)

    rng = np.random.default_rng(41)
    shape = (20, 24, 28)
    f = rng.standard_normal((3,) + shape)
    m = rng.uniform(size=shape) < 0.7
    cases = [("div_f64", f, m, (0.5, 1.25, 2.0)),
             ("div_f32", f.astype(np.float32), m, (0.5, 1.25, 2.0)),
             ("div_f32_np64", f.astype(np.float32), m, tuple(np.float64(h) for h in (0.75, 1.5, 0.3))),
             ("div_flat", rng.standard_normal((3, 1, 5, 7)), rng.uniform(size=(1, 5, 7)) < 0.6, (1.0, 1.0, 1.0))]
    g = np.load(os.path.join(HERE, "masked_spherepack_idw.npz"))
    x = g["ax"]
    h = x[1] - x[0]
    cases.append(("div_masked_spherepack", np.stack([g["U"], g["V"], g["W"]]), g["mask"], (h, h, h)))
    for name, F, M, (dx, dy, dz) in cases:
        D = physics.compute_consistent_divergence(F[0], F[1], F[2], M, dx, dy, dz)
        _save(name, u=F[0], v=F[1], w=F[2], mask=M, dx=np.float64(dx), dy=np.float64(dy), dz=np.float64(dz),
              spacing_np64=int(isinstance(dx, np.floating)), div=D)


def _blob_mask(shape, n_spheres, seed):
    """Random union of solid spheres (False) in fluid (True), any shape."""
    rng = np.random.default_rng(seed)
    nz, ny, nx = shape
    Z, Y, X = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    fluid = np.ones(shape, dtype=bool)
    for _ in range(n_spheres):
        c = rng.uniform(0, 1, 3) * np.array([nx, ny, nz])
        r = rng.uniform(2.0, 0.25 * min(shape) + 2.0)
        fluid &= (X - c[0]) ** 2 + (Y - c[1]) ** 2 + (Z - c[2]) ** 2 > r * r
    return fluid


def mask_cases(ref):
    """Pore-mask path: sample_mask_on_grid (interpolator.py:205-238) and
    extract_boundary_particles (interpolator.py:240-284) on bool, non-cubic and integer masks."""
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from ptv_interpolation_amd import synth

    sphere = synth.fluid_mask(48)
    blob = _blob_mask((20, 27, 33), 9, 5)
    labels = np.random.default_rng(6).integers(0, 4, (14, 17, 19)).astype(np.uint8)
    labels[:, :, :6] = 0
    raws = {"sphere48": (sphere, ((0, 48),) * 3), "blob": (blob, ((0, 33), (0, 27), (0, 20))),
            "blob_off": (blob, ((2.5, 40.25), (-3.0, 30.0), (10, 30)))}
    # (raw, grid bounds, grid resolution (nx, ny, nz)); wider grid bounds put voxels out of bounds,
    # 95 points on [0, 47] put grid points exactly half way between raw voxels (t = 0.5 ties)
    samples = [("sphere48", ((0, 48),) * 3, (32, 32, 32)),
               ("sphere48", ((0, 48),) * 3, (95, 40, 24)),
               ("sphere48", ((-6, 55),) * 3, (30, 30, 30)),
               ("blob", ((0, 33), (0, 27), (0, 20)), (50, 13, 20)),
               ("blob_off", ((0, 45), (-5, 32), (5, 35)), (24, 31, 17))]
    for i, (rk, gb, res) in enumerate(samples):
        raw, rb = raws[rk]
        (X, Y, Z), (x, y, z) = ref.create_grid(gb, res)
        m = ref.sample_mask_on_grid(raw, (X, Y, Z), bounds_raw=rb)
        _save(f"mask_sample_{i}", raw=raw, raw_bounds=np.array(rb, dtype=np.float64),
              raw_bounds_int=int(all(isinstance(v, int) for b in rb for v in b)), ax=x, ay=y, az=z, mask=m)
    bnd = [("sphere48", 1, 1), ("sphere48", 2, 3), ("blob", 3, 7), ("blob_off", 1, 2), ("blob", 0, 5)]
    for i, (rk, t, st) in enumerate(bnd):
        raw, rb = raws[rk]
        bx, by, bz = ref.extract_boundary_particles(raw, rb, sampling_step=st, thickness=t)
        _save(f"boundary_{i}", mask=raw, bounds=np.array(rb, dtype=np.float64),
              bounds_int=int(all(isinstance(v, int) for b in rb for v in b)), thickness=t, step=st,
              bx=bx, by=by, bz=bz)
    bx, by, bz = ref.extract_boundary_particles(labels, ((0, 19), (0, 17), (0, 14)), sampling_step=1, thickness=1)
    _save("boundary_labels", mask=labels, bounds=np.array(((0, 19), (0, 17), (0, 14)), dtype=np.float64),
          bounds_int=1, thickness=1, step=1, bx=bx, by=by, bz=bz)
    flat = _blob_mask((1, 20, 30), 3, 8)
    bx, by, bz = ref.extract_boundary_particles(flat, ((0, 30), (0, 20), (4, 9)), sampling_step=1, thickness=1)
    _save("boundary_flat", mask=flat, bounds=np.array(((0, 30), (0, 20), (4, 9)), dtype=np.float64),
          bounds_int=1, thickness=1, step=1, bx=bx, by=by, bz=bz)


def filter_cases(ref_path):
    """remove_outliers_knn (filtering.py:5-58): which particles survive, and the printed radius."""
    import importlib.util

    # load the reference file explicitly: the repo root holds a `filtering` shim of the same name
    spec = importlib.util.spec_from_file_location("ref_filtering", os.path.join(ref_path, "filtering.py"))
    filtering = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(filtering)

    rng = np.random.default_rng(31)
    n = 4000
    P = rng.uniform(0, 20, (n, 3))
    Q = np.stack([np.sin(P[:, 0] / 3), np.cos(P[:, 1] / 4), 0.2 * P[:, 2] / 20], 1) + 0.05 * rng.standard_normal((n, 3))
    bad = rng.choice(n, 80, replace=False)
    Q[bad] *= rng.uniform(3, 10, (80, 1))
    for k, thr in ((25, 3.0), (8, 2.0), (10, 3.0), (63, 3.0)):
        df = _df(P, Q)
        df["id"] = np.arange(n)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            out = filtering.remove_outliers_knn(df, k=k, threshold=thr)
        keep = np.zeros(n, dtype=bool)
        keep[out["id"].values] = True
        _save(f"filter_k{k}_t{thr}", points=P, values=Q, k=k, threshold=thr, keep=keep,
              stdout=np.array(buf.getvalue()))


def filter_dup_case(ref_path):
    """remove_outliers_knn with coincident particles (duplicated positions, different
    velocities): cKDTree's column 0 of query(k+1) (filtering.py:26-30) is then any of the
    coincident points, traversal dependent, so the keep mask of those points and of
    particles whose (k+1)-th / (k+2)-th neighbours tie is tie-dependent (the tests exclude
    them, tests/test_gpu_mask_filter.py)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_filtering", os.path.join(ref_path, "filtering.py"))
    filtering = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(filtering)
    rng = np.random.default_rng(57)
    n = 3000
    P = rng.uniform(0, 15, (n, 3))
    src = rng.choice(n, 200, replace=False)
    dst = rng.choice(np.setdiff1d(np.arange(n), src), 200, replace=False)
    P[dst] = P[src]                                   # 200 coincident pairs
    P[dst[:20]] = P[src[0]]                           # and one 21-fold cluster
    Q = np.stack([np.sin(P[:, 0] / 3), np.cos(P[:, 1] / 4), 0.1 * P[:, 2]], 1) + 0.05 * rng.standard_normal((n, 3))
    Q[dst[::7]] *= 6.0                                # twins with outlying velocities
    k, thr = 10, 3.0
    df = _df(P, Q)
    df["id"] = np.arange(n)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = filtering.remove_outliers_knn(df, k=k, threshold=thr)
    keep = np.zeros(n, dtype=bool)
    keep[out["id"].values] = True
    _save(f"filter_dup_k{k}_t{thr}", points=P, values=Q, k=k, threshold=thr, keep=keep, stdout=np.array(buf.getvalue()))


def rbf_truth_cases():
    """Accuracy reference for the ill-conditioned Gaussian fixtures (cond up to 6e8): the same
    float64 systems solved in extended precision (oracle.cpu_ref.solve_extended).  Stores the
    exact-answer field plus how far the two CPU LAPACK paths land from it (scipy's dgesv =
    the golden U, V, W; numpy's batched gesv = the oracle), so the GPU bound in
    tests/test_gpu_rbf.py is the reference's own distance to the exact answer."""
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from oracle import cpu_ref

    for deg in (0, -1):
        name = f"rbf_gaussian_eps0.3_k32_deg{deg}"
        g = np.load(os.path.join(HERE, name + ".npz"))
        q = cpu_ref.grid_queries(g["ax"], g["ay"], g["az"])
        ext = cpu_ref.rbf_local_points(g["points"], g["values"], q, 32, "gaussian", 0.3, deg, solver="extended")
        npl = cpu_ref.rbf_local_points(g["points"], g["values"], q, 32, "gaussian", 0.3, deg)
        shape = g["U"].shape
        truth = [np.ascontiguousarray(ext[:, c].reshape(shape)) for c in range(3)]

        def nw(a, b):
            return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))

        gap_scipy = [nw(g[c], t) for c, t in zip("UVW", truth)]
        gap_numpy = [nw(npl[:, i].reshape(shape), t) for i, t in enumerate(truth)]
        _save("truth_" + name, U=truth[0], V=truth[1], W=truth[2], gap_scipy=np.array(gap_scipy),
              gap_numpy=np.array(gap_numpy))
        print("  scipy-vs-exact", gap_scipy, "numpy-vs-exact", gap_numpy)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="knn,edge,masked,rbf,nearest,div,mask,filter,filterdup,rbftruth")
    a = ap.parse_args()
    ref = _import_reference(a.ref)
    only = a.only.split(",")
    if "knn" in only:
        knn_cases(ref)
    if "edge" in only:
        edge_cases(ref)
    if "masked" in only:
        masked_case(ref)
    if "rbf" in only:
        rbf_cases(ref)
    if "nearest" in only:
        nearest_cases(ref)
    if "div" in only:
        div_cases(a.ref)
    if "mask" in only:
        mask_cases(ref)
    if "filter" in only:
        filter_cases(a.ref)
    if "filterdup" in only:
        filter_dup_case(a.ref)
    if "rbftruth" in only:
        rbf_truth_cases()


if __name__ == "__main__":
    main()
