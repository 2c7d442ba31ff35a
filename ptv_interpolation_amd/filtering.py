"""Drop-in replacement for the reference ``filtering`` module (MI355X path).

Same names and behaviour as tombultreys/ptv_interpolation ``filtering.py``:

    remove_outliers_knn        filtering.py:5-58   <- (k+1)-NN + median/MAD on the GPU
    remove_outliers_threshold  filtering.py:60-74
    apply_filters              filtering.py:76-90

``remove_outliers_knn`` runs the particle-to-particle k-NN query and the per-particle
median / MAD / z-score on the GPU through ``ptv_filter_outliers_knn``
(include/ptv_api.h; kernels in ptv_interpolation_amd/csrc/ptv_filter.hip and the
slot mode of ptv_knn.hip).  There is no CPU fallback.  Coordinates and velocities are
taken as float64 (the CSV loader's dtype).
"""
from __future__ import annotations

import numpy as np

from . import _lib

__all__ = ["remove_outliers_knn", "remove_outliers_threshold", "apply_filters"]

_MAD_EPS = 1e-6  # filtering.py:46


def _device():
    from . import launcher

    return launcher.devices()[0]


def remove_outliers_knn(df, k=25, threshold=3.0):
    """Neighbourhood median/MAD filter on speed; filtering.py:5-58."""
    if len(df) <= k:
        print(f"  Warning: DataFrame too small ({len(df)}) for k-NN filter (k={k}). Skipping.")
        return df
    points = df[["x", "y", "z"]].values
    values = df[["u", "v", "w"]].values
    ctx = _lib.Context.get(_device())
    keep, kth = ctx.filter_outliers_knn(points, values, k=k, threshold=threshold, mad_eps=_MAD_EPS)
    median_filter_radius = np.median(kth)
    print(f"  Filtering radius: median voxel distance to {k}-th neighbor = {median_filter_radius:.4f}")
    keep_mask = keep.view(np.bool_)
    n_removed = np.sum(~keep_mask)
    if n_removed > 0:
        print(f"  Outlier Filter: Removed {n_removed} points ({n_removed/len(df)*100:.2f}%).")
        return df[keep_mask].reset_index(drop=True)
    print("  Outlier Filter: No outliers detected.")
    return df


def remove_outliers_threshold(df, max_speed=10.0):
    """Global speed cut; filtering.py:60-74 (a single elementwise pass, kept on the host)."""
    u, v, w = df["u"].values, df["v"].values, df["w"].values
    speed = np.sqrt(u**2 + v**2 + w**2)
    keep_mask = speed <= max_speed
    n_removed = np.sum(~keep_mask)
    if n_removed > 0:
        print(f"  Threshold Filter: Removed {n_removed} points with speed > {max_speed}.")
        return df[keep_mask].reset_index(drop=True)
    return df


def apply_filters(df, args):
    """filtering.py:76-90."""
    if not args.filter_outliers:
        return df
    df = remove_outliers_threshold(df, max_speed=args.filter_max_speed)
    if len(df) > 0:
        df = remove_outliers_knn(df, k=args.filter_neighbors, threshold=args.filter_threshold)
    return df
