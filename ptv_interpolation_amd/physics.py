"""Drop-in for the reference ``physics.compute_consistent_divergence`` (MI355X path).

``compute_consistent_divergence(u, v, w, mask, dx, dy, dz)`` (physics.py:6-53) is the
divergence ``view_divergence.py:39,42`` evaluates on the interpolated field and the
divergence-cleaning loop re-evaluates every iteration (physics.py:173, :193-194).  Here it
is one HIP stencil kernel (csrc/ptv_div.hip) behind ``ptv_divergence`` (include/ptv_api.h);
no CPU fallback.  Results are bit-identical to the reference, including numpy's dtype
rules: float32 fields with Python-float spacings give float32; a numpy float64 spacing
(``x[1] - x[0]``, view_divergence.py:22) gives float64 quotients.

The sparse Poisson / variational cleaning solvers (physics.py:55-464) are outside the hot
path (SURVEY.md §8(f) names only the divergence).
"""
from __future__ import annotations

import numpy as np

from . import _lib, launcher

__all__ = ["compute_consistent_divergence"]


def _result_dtype(ft, h):
    """dtype of ``(float array of dtype ft) / h`` under numpy's promotion (NEP 50: Python
    scalars are weak, numpy scalars and 0-d arrays are not)."""
    return np.result_type(np.empty(0, dtype=ft), h)


def compute_consistent_divergence(u, v, w, mask, dx, dy, dz):
    """physics.py:6-53 on the GPU.  ``mask``: True = fluid (required, as in the reference,
    whose np.roll of ``None`` raises AxisError)."""
    if mask is None:
        raise np.exceptions.AxisError("axis 2 is out of bounds for array of dimension 0")
    u, v, w = (np.asarray(a) for a in (u, v, w))
    if not (u.shape == v.shape == w.shape == np.shape(mask)) or u.ndim != 3:
        raise ValueError(f"u, v, w and mask must share one 3-D shape, got {u.shape}, {v.shape}, "
                         f"{w.shape}, {np.shape(mask)}")
    fts = {a.dtype for a in (u, v, w)}
    if len(fts) != 1:
        raise NotImplementedError(f"fields of mixed dtypes {sorted(map(str, fts))} (numpy computes each "
                                  "axis in its own dtype) are not supported on the GPU path")
    ft = fts.pop()
    if ft.kind in "biu":
        # (int + int) / 2.0 is float64 in the reference; exact for |values| < 2**52
        ft = np.dtype(np.float64)
    if ft not in (np.float32, np.float64):
        raise NotImplementedError(f"field dtype {ft} (GPU path: float32 / float64)")
    rts = {_result_dtype(ft, h) for h in (dx, dy, dz)}
    if len(rts) != 1:
        raise NotImplementedError("spacings that promote float32 fields differently per axis "
                                  f"({sorted(map(str, rts))}) are not supported on the GPU path")
    rt = rts.pop()
    ctx = _lib.Context.get(launcher.devices()[0])  # PTV_DEVICE, else the first of PTV_DEVICES / all
    return ctx.divergence(u.astype(ft, copy=False), v.astype(ft, copy=False), w.astype(ft, copy=False),
                          np.asarray(mask).astype(bool, copy=False), float(dx), float(dy), float(dz),
                          result_dtype=rt)
