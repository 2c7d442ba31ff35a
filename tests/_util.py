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


def boundary_ties(points, ax, ay, az, k):
    """(nz, ny, nx) bool: voxels whose k-th and (k+1)-th nearest particles are equidistant.

    At such voxels the neighbour SET depends on the search's tie order (cKDTree's is
    traversal dependent), so no implementation can be held to the reference there.
    """
    from scipy.spatial import KDTree

    Z, Y, X = np.meshgrid(az, ay, ax, indexing="ij")
    q = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    kk = min(k + 1, len(points))
    d, _ = KDTree(points).query(q, k=kk)
    d = d.reshape(len(q), -1)
    if kk <= k:
        return np.zeros(X.shape, bool)
    return (d[:, k - 1] == d[:, k]).reshape(X.shape)


def hetero_ties_points(points, values, q, k, extra=8):
    """(Q,) bool pair (tie, hetero) for query points q.

    ``tie``: two of the k + 1 nearest particles are equidistant (at the k-th distance the
    neighbour SET depends on the search's tie order; below it the rank ORDER does, and numpy's
    pairwise sum rounds differently in another order).  ``hetero``: such a voxel where some
    run of equidistant neighbours touching the first k does not carry one (u, v, w); only there
    can two correct searches give different bits.  At value-homogeneous ties every choice
    gives identical terms (equal distances -> equal weights, equal values) in the same rank
    order, so the result is bit-identical and the voxel stays in the comparison.  Tie runs
    longer than the columns queried are re-queried with more neighbours (up to 1024 beyond k;
    longer runs are counted heterogeneous, conservatively)."""
    from scipy.spatial import KDTree

    P = np.asarray(points, dtype=np.float64)
    Vv = np.asarray(values, dtype=np.float64).reshape(len(P), -1)
    q = np.asarray(q, dtype=np.float64).reshape(-1, 3)
    kk = min(k + extra, len(P))
    tree = KDTree(P)
    d, i = tree.query(q, k=kk, workers=-1)
    d = d.reshape(len(q), -1)
    # any two of the first min(k + 1, n) neighbours at exactly the same distance: the order of
    # equidistant neighbours (and, at the k-th, the set) is the search's choice
    kb = min(k + 1, kk)
    tie = (d[:, :kb - 1] == d[:, 1:kb]).any(axis=1)
    hetero = np.zeros(len(q), bool)
    rows = np.nonzero(tie)[0]
    while len(rows):
        dd, ii = tree.query(q[rows], k=kk, workers=-1)
        dd = dd.reshape(len(rows), -1)
        ii = ii.reshape(len(rows), -1)
        again = []
        for j, r in enumerate(rows):
            if kk < len(P) and dd[j, -1] == dd[j, k - 1]:  # the k-th's tie run may continue
                again.append(r)
                continue
            # every run of equal distances touching ranks < k must carry one value: then any
            # order (and any choice at the k-th) gives the same terms in the same rank order
            bad = False
            s = 0
            while s < min(k, dd.shape[1]) and not bad:
                e = s
                while e + 1 < dd.shape[1] and dd[j, e + 1] == dd[j, s]:
                    e += 1
                if e > s:
                    vals = Vv[ii[j, s:e + 1]]
                    bad = not (vals == vals[0]).all()
                s = e + 1
            hetero[r] = bad
        if not again or kk >= min(len(P), k + 1024):
            hetero[np.asarray(again, dtype=np.int64)] = True
            break
        rows = np.asarray(again)
        kk = min(len(P), k + 4 * (kk - k))
    return tie, hetero


def hetero_ties(points, values, ax, ay, az, k):
    """(tie, hetero) as (nz, ny, nx) bool over a separable grid (see hetero_ties_points)."""
    Z, Y, X = np.meshgrid(az, ay, ax, indexing="ij")
    q = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    tie, het = hetero_ties_points(points, values, q, k)
    return tie.reshape(X.shape), het.reshape(X.shape)


def tie_value_bounds(points, values, ax, ay, az, k, extra=64):
    """Per-voxel (lo, hi), each (C, nz, ny, nx): min / max of every value component over the
    particles any correct k-NN search may pick (the first k plus the whole run tied with the k-th
    distance).  IDW and Sibson outputs are positive-weight averages of their neighbours' values, so
    whatever the tie order they lie in [lo, hi] (up to rounding)."""
    from scipy.spatial import KDTree

    P = np.asarray(points, dtype=np.float64)
    Vv = np.asarray(values, dtype=np.float64).reshape(len(P), -1)
    Z, Y, X = np.meshgrid(az, ay, ax, indexing="ij")
    q = np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)
    kk = min(k + extra, len(P))
    d, i = KDTree(P).query(q, k=kk, workers=-1)
    d = d.reshape(len(q), -1)
    i = i.reshape(len(q), -1)
    cand = d <= d[:, k - 1:k]  # (Q, kk): within the k-th distance
    vals = Vv[i]  # (Q, kk, C)
    lo = np.where(cand[..., None], vals, np.inf).min(axis=1).T.reshape((-1,) + X.shape)
    hi = np.where(cand[..., None], vals, -np.inf).max(axis=1).T.reshape((-1,) + X.shape)
    return lo, hi


def filter_ties(points, k):
    """(n,) bool: particles whose remove_outliers_knn decision depends on cKDTree's tie order.

    The reference drops column 0 of ``KDTree.query(points, k + 1)`` (filtering.py:26-30) as
    "the point itself"; with a coincident twin that column may be the twin (a different
    speed).  A tie between the (k+1)-th and (k+2)-th neighbour distances changes the
    neighbour set.  Either makes the keep decision traversal dependent."""
    from scipy.spatial import KDTree

    P = np.asarray(points, dtype=np.float64)
    d, _ = KDTree(P).query(P, k=min(k + 2, len(P)))
    twin = d[:, 1] == 0.0
    tie = d[:, k] == d[:, k + 1] if d.shape[1] > k + 1 else np.zeros(len(P), bool)
    return twin | tie
