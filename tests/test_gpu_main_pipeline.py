"""End-to-end pin of ``main.py`` (main.py:21-246) through the drop-in modules, on the GPU.

tests/golden/make_main_golden.py ran the reference ``main.py`` itself on C1 (10k sphere-pack
particles, voxel units): an unmasked IDW run and a masked run with the outlier filter, the
pore-mask path and virtual boundary particles.  This test replays the same steps with the
MI355X implementations — ``load_ptv_data``, the domain crop (main.py:137-143),
``filtering.apply_filters``, ``create_grid``, ``sample_mask_on_grid``,
``extract_boundary_particles``, ``interpolate_field`` and the main.py:194-207 epilogue — and
compares what main.py saves (main.py:220-226): x, y, z and mask bit for bit, u, v, w bit for
bit except at tie voxels (k-th and (k+1)-th neighbours equidistant: the boundary particles
sit on the integer voxel lattice), and the status lines the library functions print.  The
reference's own source never travels here: only its inputs and outputs (the fixtures).
"""
import argparse
import contextlib
import io

import numpy as np
import pytest

from tests._util import hetero_ties, load

pytestmark = pytest.mark.gpu

# main.py's argparse defaults for the options the pipeline reads (main.py:23-52)
DEFAULTS = dict(mask=None, downscale=1.0, crop=None, method="linear", rbf_neighbors=20,
                rbf_kernel="thin_plate_spline", smoothing=0.0, idw_power=2.0, idw_neighbors=50,
                sibson_neighbors=30, boundary_particles=False, boundary_sampling=1, boundary_thickness=1,
                filter_outliers=False, filter_neighbors=25, filter_threshold=3.0, filter_max_speed=10.0,
                n_jobs=1)


def _args(argv, masked):
    a = dict(DEFAULTS)
    it = iter(argv)
    for tok in it:
        key = tok[2:].replace("-", "_")
        if isinstance(DEFAULTS.get(key), bool):
            a[key] = True
        else:
            a[key] = type(DEFAULTS[key])(next(it)) if DEFAULTS.get(key) is not None else next(it)
    a["mask"] = masked
    return argparse.Namespace(**a)


def _replay(csv_path, args, mask_raw):
    """main.py:55-207 with the drop-in modules (no crop / offset / swap / transpose options)."""
    from ptv_interpolation_amd import filtering
    from ptv_interpolation_amd import interpolator as ip

    df = ip.load_ptv_data(csv_path)
    if args.mask:
        nz, ny, nx = mask_raw.shape
        bounds = ((0, nx), (0, ny), (0, nz))
        xmin, xmax, ymin, ymax, zmin, zmax = 0, nx, 0, ny, 0, nz
        resolution = (max(1, int(round(nx / args.downscale))), max(1, int(round(ny / args.downscale))),
                      max(1, int(round(nz / args.downscale))))
    else:
        xmin, xmax = df.x.min(), df.x.max()
        ymin, ymax = df.y.min(), df.y.max()
        zmin, zmax = df.z.min(), df.z.max()
        bounds = ((xmin, xmax + 1), (ymin, ymax + 1), (zmin, zmax + 1))
        resolution = max(1, int(round(64 / args.downscale)))
    df = df[(df.x >= xmin) & (df.x < xmax) & (df.y >= ymin) & (df.y < ymax) &
            (df.z >= zmin) & (df.z < zmax)].reset_index(drop=True)
    if args.filter_outliers:
        df = filtering.apply_filters(df, args)
    (X, Y, Z), (x, y, z) = ip.create_grid(bounds, resolution)
    mask = ip.sample_mask_on_grid(mask_raw, (X, Y, Z), bounds_raw=bounds) if args.mask else np.zeros(X.shape, bool)
    if args.boundary_particles and args.mask:
        import pandas as pd

        bx, by, bz = ip.extract_boundary_particles(mask_raw, bounds, sampling_step=args.boundary_sampling,
                                                   thickness=args.boundary_thickness)
        if len(bx) > 0:
            b_df = pd.DataFrame({"x": bx, "y": by, "z": bz, "u": np.zeros_like(bx), "v": np.zeros_like(by),
                                 "w": np.zeros_like(bz)})
            df = pd.concat([df, b_df], ignore_index=True)
    U, V, W = ip.interpolate_field(df, (X, Y, Z), method=args.method, rbf_neighbors=args.rbf_neighbors,
                                   rbf_kernel=args.rbf_kernel, smoothing=args.smoothing, idw_power=args.idw_power,
                                   idw_neighbors=args.idw_neighbors, sibson_neighbors=args.sibson_neighbors,
                                   n_jobs=args.n_jobs)
    if np.isnan(U).any():
        U, V, W = np.nan_to_num(U), np.nan_to_num(V), np.nan_to_num(W)
    if args.mask:
        solid = ~mask
        U[solid] = 0
        V[solid] = 0
        W[solid] = 0
    return dict(x=x, y=y, z=z, u=U, v=V, w=W, mask=mask), df


@pytest.mark.parametrize("name", ["main_c1_idw", "main_c1_masked"])
def test_main_pipeline_matches_reference(name, tmp_path):
    g = load(name)
    csv_path = tmp_path / "c1.csv"
    csv_path.write_text(str(g["csv"]))
    args = _args([str(t) for t in g["args"]], bool(int(g["masked"])))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out, df = _replay(str(csv_path), args, g["mask_raw"] if args.mask else None)
    for key in ("x", "y", "z", "mask"):
        assert out[key].dtype == g["out_" + key].dtype and np.array_equal(out[key], g["out_" + key]), key
    P = df[["x", "y", "z"]].values
    tie, het = hetero_ties(P, df[["u", "v", "w"]].values, out["x"], out["y"], out["z"], args.idw_neighbors)
    if args.mask:
        het &= out["mask"]  # solid voxels are zeroed by main.py:202-207 whatever the neighbours
    print(f"{name}: k-th-distance ties {tie.mean():.4%} of voxels, value-heterogeneous (excluded) {het.mean():.4%}")
    assert het.mean() < 0.005
    for key in ("u", "v", "w"):
        a, b = out[key], g["out_" + key]
        assert a.shape == b.shape and a.dtype == b.dtype == np.float64
        assert np.array_equal(a[~het], b[~het]), key
    ref_lines = str(g["stdout"]).splitlines()
    for line in buf.getvalue().splitlines():
        assert line in ref_lines, f"status line not printed by the reference: {line!r}"
