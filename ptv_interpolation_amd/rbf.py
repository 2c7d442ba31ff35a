"""Local RBF (interpolator.py:157-195) on the GPU — not built yet in this revision."""


def rbf_field(points, values, grid_tuple, k, kernel, smoothing):
    raise NotImplementedError(
        "method='rbf' (local RBF, interpolator.py:157-195) has no GPU kernel in this build yet; "
        "no CPU fallback is provided")
