"""Shared helpers for the parity tests."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def names(prefixes=("idw", "sibson", "edge", "masked")):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        n = os.path.basename(p)[:-4]
        if n.startswith(prefixes):
            out.append(n)
    return out


def normwise(a, b):
    """max|a-b| / max|b| per SURVEY.md §8(c), NaNs must coincide."""
    a = np.asarray(a); b = np.asarray(b)
    na, nb = np.isnan(a), np.isnan(b)
    assert (na == nb).all(), "NaN pattern differs"
    m = ~nb
    if not m.any():
        return 0.0
    den = np.max(np.abs(b[m]))
    num = np.max(np.abs(a[m] - b[m]))
    return num / den if den > 0 else num
