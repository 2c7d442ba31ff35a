"""Local RBF interpolation on the GPU: the ``method='rbf'`` branch of
``interpolate_field`` (interpolator.py:157-195) and the scipy object it builds.

The reference constructs ``scipy.interpolate.RBFInterpolator(points, values,
neighbors=rbf_neighbors, kernel=rbf_kernel, smoothing=smoothing)``
(interpolator.py:162-167) and evaluates it on the flattened grid, serially in
chunks of 10 000 points (:184-193) or fanned out over ``n_jobs`` processes
(:173-182).  ``LocalRBFInterpolator`` keeps that constructor's argument
resolution and errors (scipy ``_rbfinterp.py:258-345``: kernel names, the
epsilon requirement, the default polynomial degree, the minimum number of
points) and evaluates with the HIP kernels behind ``ptv_interp_rbf_local``
(k-NN in slot mode, then one (k + r)-square solve per voxel).  There is no CPU
fallback: a missing library or GPU raises.

Supported: ``neighbors`` set (the only way interpolate_field calls it), three
value components (u, v, w; fewer are zero-padded, more are evaluated in groups
of three), ``k + #monomials <= 128``.  ``neighbors=None`` (one global system
over all particles) is not a GPU path and raises NotImplementedError.
"""
from __future__ import annotations

import warnings
from math import comb

import numpy as np

from . import _lib

# scipy/interpolate/_rbfinterp.py:19-45
AVAILABLE = {"linear", "thin_plate_spline", "cubic", "quintic", "multiquadric", "inverse_multiquadric",
             "inverse_quadratic", "gaussian"}
SCALE_INVARIANT = {"linear", "thin_plate_spline", "cubic", "quintic"}
NAME_TO_MIN_DEGREE = {"multiquadric": 0, "linear": 0, "thin_plate_spline": 1, "cubic": 1, "quintic": 2}
MAX_SYSTEM = 128  # systems up to this size are solved in LDS; larger ones in global memory (k_rbf_huge)


def _device():
    from . import launcher

    return launcher.devices()[0]


class LocalRBFInterpolator:
    """``RBFInterpolator(y, d, neighbors=k, smoothing, kernel, epsilon, degree)`` on the GPU.

    Argument handling follows ``_rbfinterp.py:258-345`` line for line (same
    exception types and messages for bad kernels, a missing epsilon, a too-low
    degree, too few points for the polynomial).
    """

    def __init__(self, y, d, neighbors=None, smoothing=0.0, kernel="thin_plate_spline", epsilon=None,
                 degree=None):
        y = np.asarray(y, dtype=float, order="C")
        if y.ndim != 2:
            raise ValueError("`y` must be a 2-dimensional array.")
        ny, ndim = y.shape
        if ndim != 3:
            raise NotImplementedError("the GPU local RBF path is three-dimensional (interpolator.py:78)")
        if np.iscomplexobj(d):
            raise NotImplementedError("complex data values are not supported on the GPU path")
        d = np.asarray(d, dtype=float, order="C")
        if d.shape[0] != ny:
            raise ValueError(f"Expected the first axis of `d` to have length {ny}.")
        self.d_shape = d.shape[1:]
        d = d.reshape((ny, -1))
        if np.isscalar(smoothing):
            smoothing = float(smoothing)
        else:
            smoothing = np.asarray(smoothing, dtype=float, order="C")
            if smoothing.shape != (ny,):
                raise ValueError(f"Expected `smoothing` to be a scalar or have shape ({ny},).")
        kernel = kernel.lower()
        if kernel not in AVAILABLE:
            raise ValueError(f"`kernel` must be one of {AVAILABLE}.")
        if epsilon is None:
            if kernel in SCALE_INVARIANT:
                epsilon = 1.0
            else:
                raise ValueError("`epsilon` must be specified if `kernel` is not one of "
                                 f"{SCALE_INVARIANT}.")
        else:
            epsilon = float(epsilon)
        min_degree = NAME_TO_MIN_DEGREE.get(kernel, -1)
        if degree is None:
            degree = max(min_degree, 0)
        else:
            degree = int(degree)
            if degree < -1:
                raise ValueError("`degree` must be at least -1.")
            elif -1 < degree < min_degree:
                warnings.warn(f"`degree` should not be below {min_degree} except -1 when `kernel` is '{kernel}'."
                              f"The interpolant may not be uniquely solvable, and the smoothing parameter may "
                              f"have an unintuitive effect.", UserWarning, stacklevel=2)
        if neighbors is None:
            nobs = ny
        else:
            neighbors = int(min(neighbors, ny))
            nobs = neighbors
        nmonos = comb(degree + ndim, ndim) if degree >= 0 else 0
        if nmonos > nobs:
            raise ValueError(f"At least {nmonos} data points are required when `degree` is {degree} and the "
                             f"number of dimensions is {ndim}.")
        if neighbors is None:
            raise NotImplementedError("RBFInterpolator(neighbors=None) builds one global system; only the local "
                                      "(neighbors=k) form used by interpolate_field runs on the GPU")
        self.y, self.d = y, d
        self.neighbors = neighbors
        self.smoothing = smoothing
        self.kernel = kernel
        self.epsilon = epsilon
        self.degree = degree
        self.nmonos = nmonos
        self.stats = None

    def _groups(self):
        """Value components in groups of three (the kernel solves for u, v, w together)."""
        S = self.d.shape[1]
        for c0 in range(0, S, 3):
            g = np.zeros((self.d.shape[0], 3))
            g[:, : min(3, S - c0)] = self.d[:, c0:c0 + 3]
            yield c0, min(3, S - c0), g

    def _run(self, ctx=None, out=None, **grid):
        """``out``: optional three arrays for a three-component evaluation, written in place."""
        ctx = ctx if ctx is not None else _lib.Context.get(_device())
        outs = []
        for c0, w, g in self._groups():
            res = ctx.interp_rbf(self.y, g, k=self.neighbors, kernel=self.kernel, epsilon=self.epsilon,
                                 degree=self.degree, smoothing=self.smoothing,
                                 out=out if self.d.shape[1] == 3 else None, **grid)
            self.stats = ctx.stats
            outs.extend(res[:w])
        return outs

    def __call__(self, x):
        """Evaluate at (Q, 3) points (``_rbfinterp.py:463-556``); returns (Q, ...) float64."""
        x = np.asarray(x, dtype=float, order="C")
        if x.ndim != 2:
            raise ValueError("`x` must be a 2-dimensional array.")
        nx, ndim = x.shape
        if ndim != self.y.shape[1]:
            raise ValueError(f"Expected the second axis of `x` to have length {self.y.shape[1]}.")
        if nx == 0:
            return np.empty((0,) + self.d_shape)
        comps = self._run(grid_points=(x[:, 0], x[:, 1], x[:, 2]), shape=(1, 1, nx))
        out = np.stack([c.reshape(-1) for c in comps], axis=-1)
        return out.reshape((nx,) + self.d_shape)

    def evaluate_grid(self, ax, ay, az, fluid_mask=None, flags=0, z_range=None, ctx=None, out=None):
        """Evaluate on the separable grid meshgrid(az, ay, ax, 'ij') (create_grid axes) without
        materialising the (V, 3) query list; returns one (nz', ny, nx) array per component
        (``out``: three preallocated arrays for three components, filled in place)."""
        return self._run(ctx=ctx, out=out, axes=(ax, ay, az), fluid_mask=fluid_mask, flags=flags, z_range=z_range)


def rbf_field(points, values, grid_tuple, k, kernel, smoothing, n_jobs=1):
    """interpolator.py:157-195 without the Python loop: (U, V, W) with the grid's shape.

    The status lines of the reference (:174, :187, :193) are printed with the same
    text; ``n_jobs`` only selects which ones (the GPU evaluates every voxel in one call).
    """
    from .interpolator import separable_axes

    X, Y, Z = grid_tuple
    shape = np.shape(X)
    interp = LocalRBFInterpolator(points, values, neighbors=k, kernel=kernel, smoothing=smoothing)
    n_points = int(np.prod(shape))
    if n_jobs > 1:
        print(f"Parallelizing evaluation across {n_jobs} processes...")
    else:
        print(f"Interpolating {n_points} points serially...")
    axes = separable_axes(X, Y, Z)
    if axes is not None:
        from . import launcher

        # z-slab per device (launcher.py), as interpolator.py:173-182 fans out over processes
        if interp.d.shape[1] != 3:
            raise ValueError("interpolate_field values must have three components (u, v, w)")
        full = [np.empty((len(axes[2]), len(axes[1]), len(axes[0]))) for _ in range(3)]
        U, V, W = launcher.run_slabs(len(axes[2]), lambda ctx, z0, z1, views: interp.evaluate_grid(
            *axes, z_range=(z0, z1), ctx=ctx, out=views), full)
    else:
        flat = np.stack([np.ravel(X), np.ravel(Y), np.ravel(Z)], axis=-1)
        out = interp(flat)
        U, V, W = out[:, 0], out[:, 1], out[:, 2]
    if n_jobs <= 1:
        chunk = 10000
        for i in range(0, n_points, chunk):
            end = min(i + chunk, n_points)
            if (i // chunk) % 10 == 0 or end == n_points:
                print(f"  Progress: {end / n_points * 100:.1f}% ({end}/{n_points})")
    return U.reshape(shape), V.reshape(shape), W.reshape(shape)
