"""Accuracy study (CPU, numpy): the local-RBF saddle-point systems solved by the null-space
method the k_rbf_ns kernel uses, against the reference's LAPACK answers (golden fixtures)
and the extended-precision truth.

    [Phi  P] [c]   [d]      P = Q [R; 0] (Householder, r reflectors)
    [P^T  0] [e] = [0]      B = (Q^T Phi Q)[r:, r:]  is SPD for a conditionally positive
                            definite kernel with degree >= its minimum: c~2 = B^-1 (Q^T d)[r:]
                            c = Q [0; c~2],  e = R^-1 ((Q^T d)[:r] - (Q^T Phi Q)[:r, r:] c~2)

Run: python tools/rbf_nullspace_proto.py            (fixtures + random clouds)
     python tools/rbf_nullspace_proto.py --refine   (one step of iterative refinement)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cpu_ref  # noqa: E402
from tests._util import load, normwise  # noqa: E402


def householder_vectors(P):
    """LAPACK dgeqr2/dlarfg-style reflectors of P (C, k, r): v (C, r, k) with v[t, t] = 1,
    tau (C, r), R diag beta (C, r); P is overwritten with R on top."""
    C, k, r = P.shape
    P = P.copy()
    V = np.zeros((C, r, k))
    tau = np.zeros((C, r))
    beta = np.zeros((C, r))
    for t in range(r):
        x = P[:, t:, t]
        alpha = x[:, 0]
        xn = np.sqrt(np.sum(x[:, 1:] ** 2, axis=1))
        b = -np.copysign(np.sqrt(alpha * alpha + xn * xn), alpha)
        tt = (b - alpha) / b
        v = x / (alpha - b)[:, None]
        v[:, 0] = 1.0
        V[:, t, t:] = v
        tau[:, t] = tt
        beta[:, t] = b
        # apply H = I - tau v v^T to P[:, t:, t:]
        w = np.einsum("ci,cij->cj", v, P[:, t:, t:])
        P[:, t:, t:] -= tt[:, None, None] * v[:, :, None] * w[:, None, :]
    return V, tau, beta, P


def apply_left(V, tau, X, reverse=False):
    """Q^T X (forward) or Q X (reverse) for X (C, k, s)."""
    C, r, k = V.shape
    order = range(r - 1, -1, -1) if reverse else range(r)
    for t in order:
        v = V[:, t]
        w = np.einsum("ci,cis->cs", v, X)
        X = X - tau[:, t, None, None] * v[:, :, None] * w[:, None, :]
    return X


def solve_nullspace(lhs, rhs, k):
    C, m, _ = lhs.shape
    r = m - k
    Phi = lhs[:, :k, :k]
    P = lhs[:, :k, k:]
    d = rhs[:, :k]
    V, tau, beta, PR = householder_vectors(P)
    # two-sided transform Q^T Phi Q
    T = apply_left(V, tau, Phi)
    T = np.swapaxes(apply_left(V, tau, np.swapaxes(T, 1, 2)), 1, 2)
    dt = apply_left(V, tau, d)
    B = T[:, r:, r:]
    # LU without pivoting (the SPD path)
    c2 = np.linalg.solve(B, dt[:, r:])  # numpy (pivoting) -- accuracy study stand-in
    c2 = lu_nopiv_solve(B, dt[:, r:])
    Rm = PR[:, :r, :r]
    e = np.linalg.solve(Rm, dt[:, :r] - np.einsum("cij,cjs->cis", T[:, :r, r:], c2))
    ct = np.concatenate([np.zeros((C, r, rhs.shape[2])), c2], axis=1)
    c = apply_left(V, tau, ct, reverse=True)
    return np.concatenate([c, e], axis=1), beta, B


def lu_nopiv_solve(B, b):
    A = B.copy()
    x = b.copy()
    n = A.shape[1]
    for c in range(n):
        l = A[:, c + 1:, c] / A[:, c, c][:, None]
        A[:, c + 1:, c:] -= l[:, :, None] * A[:, c, c:][:, None, :]
        x[:, c + 1:] -= l[:, :, None] * x[:, c, None, :]
    out = np.empty_like(x)
    for c in range(n - 1, -1, -1):
        acc = x[:, c] - np.einsum("cj,cjs->cs", A[:, c, c + 1:], out[:, c + 1:])
        out[:, c] = acc / A[:, c, c][:, None]
    return out


def ns_kernel_order(lhs, rhs, k, vec):
    """The k_rbf_ns kernel's step order for one batch (vectorised over systems): dlarfg
    reflectors of P (applied to P and the right-hand sides), y_t = Phi v_t, the z recurrence
    Phi_t v_t = y_t - sum_{s<t} (v_s (z_s.v_t) + z_s (v_s.v_t)), z_t = p - tau (v.p)/2 v with
    p = tau Phi_t v_t, one rank-2r update Phi - sum_t (v_t z_t^T + z_t v_t^T) of the columns >= r,
    LU without pivoting of B, a back substitution that also forms the e right-hand side
    (rows < r), Rt e = rhs, and the evaluation (Q^T phi(x))[r:] . c~2 + P(x)^T e."""
    C, m, _ = lhs.shape
    r = m - k
    A = lhs[:, :k, :k].copy()
    P = lhs[:, :k, k:].copy()
    d = rhs[:, :k].copy()
    ph = vec[:, :k].copy()
    Vs, taus, betas = [], [], []
    rows = np.arange(k)
    for t in range(r):
        alpha = P[:, t, t]
        x = np.where(rows[None, :] > t, P[:, :, t], 0.0)
        s = np.sum(x * x, axis=1)
        b = -np.copysign(np.sqrt(alpha * alpha + s), alpha)
        tau = np.where(s == 0.0, 0.0, (b - alpha) / b)
        scal = np.where(s == 0.0, 0.0, 1.0 / (alpha - b))
        v = np.where(rows[None, :] > t, P[:, :, t] * scal[:, None], np.where(rows[None, :] == t, 1.0, 0.0))
        b = np.where(s == 0.0, alpha, b)
        for u in range(t + 1, r):
            w = np.sum(v * P[:, :, u], axis=1)
            P[:, :, u] -= (tau * w)[:, None] * v
        w = np.einsum("ci,cis->cs", v, d)
        d -= tau[:, None, None] * v[:, :, None] * w[:, None, :]
        Vs.append(v); taus.append(tau); betas.append(b)
    Z = [np.einsum("cij,cj->ci", A, Vs[t]) for t in range(r)]
    for t in range(r):
        for s2 in range(t):
            zv = np.sum(Z[s2] * Vs[t], axis=1)
            vv = np.sum(Vs[s2] * Vs[t], axis=1)
            Z[t] = Z[t] - Z[s2] * vv[:, None] - Vs[s2] * zv[:, None]
        Z[t] = Z[t] * taus[t][:, None]
        kk = 0.5 * taus[t] * np.sum(Vs[t] * Z[t], axis=1)
        Z[t] = Z[t] - kk[:, None] * Vs[t]
    for t in range(r):
        A[:, :, r:] -= Vs[t][:, :, None] * Z[t][:, None, r:] + Z[t][:, :, None] * Vs[t][:, None, r:]
    # LU without pivoting of rows/cols r..k-1; rows < r untouched (multiplier 0)
    for c in range(r, k):
        piv = A[:, c, c]
        l = np.where(rows[None, :] > c, A[:, :, c] / piv[:, None], 0.0)
        A[:, :, c + 1:] -= l[:, :, None] * A[:, c, None, c + 1:]
        d -= l[:, :, None] * d[:, c, None, :]
    # back substitution: x_c = d_c / U_cc, every row above c (including rows < r) updated
    x = np.zeros_like(d)
    for c in range(k - 1, r - 1, -1):
        x[:, c] = d[:, c] / A[:, c, c][:, None]
        above = rows[None, :] < c
        d -= np.where(above[:, :, None], A[:, :, c, None] * x[:, c, None, :], 0.0)
    # R e = d[:r]  (R row t: P[t, u] for u > t, diag beta_t)
    e = np.zeros((C, r, d.shape[2]))
    rhs_e = d[:, :r].copy()
    for t in range(r - 1, -1, -1):
        e[:, t] = rhs_e[:, t] / betas[t][:, None]
        rhs_e[:, :t] -= P[:, :t, t, None] * e[:, t, None, :]
    # Q^T phi(x)
    for t in range(r):
        w = np.sum(Vs[t] * ph, axis=1)
        ph -= (taus[t] * w)[:, None] * Vs[t]
    out = np.einsum("ci,cis->cs", ph[:, r:], x[:, r:]) + np.einsum("ct,cts->cs", vec[:, k:], e)
    return out


def ns_kernel_coeffs(lhs, rhs, k):
    """The kernel's step order (ns_kernel_order) returning the coefficients (c, e) instead of the
    evaluated value: c = Q [0; c~2]."""
    C, m, _ = lhs.shape
    r = m - k
    A = lhs[:, :k, :k].copy()
    P = lhs[:, :k, k:].copy()
    d = rhs[:, :k].copy()
    Vs, taus, betas = [], [], []
    rows = np.arange(k)
    for t in range(r):
        alpha = P[:, t, t]
        x = np.where(rows[None, :] > t, P[:, :, t], 0.0)
        s = np.sum(x * x, axis=1)
        b = -np.copysign(np.sqrt(alpha * alpha + s), alpha)
        tau = np.where(s == 0.0, 0.0, (b - alpha) / b)
        scal = np.where(s == 0.0, 0.0, 1.0 / (alpha - b))
        v = np.where(rows[None, :] > t, P[:, :, t] * scal[:, None], np.where(rows[None, :] == t, 1.0, 0.0))
        b = np.where(s == 0.0, alpha, b)
        for u in range(t + 1, r):
            w = np.sum(v * P[:, :, u], axis=1)
            P[:, :, u] -= (tau * w)[:, None] * v
        w = np.einsum("ci,cis->cs", v, d)
        d -= tau[:, None, None] * v[:, :, None] * w[:, None, :]
        Vs.append(v); taus.append(tau); betas.append(b)
    Z = [np.einsum("cij,cj->ci", A, Vs[t]) for t in range(r)]
    for t in range(r):
        for s2 in range(t):
            zv = np.sum(Z[s2] * Vs[t], axis=1)
            vv = np.sum(Vs[s2] * Vs[t], axis=1)
            Z[t] = Z[t] - Z[s2] * vv[:, None] - Vs[s2] * zv[:, None]
        Z[t] = Z[t] * taus[t][:, None]
        kk = 0.5 * taus[t] * np.sum(Vs[t] * Z[t], axis=1)
        Z[t] = Z[t] - kk[:, None] * Vs[t]
    for t in range(r):
        A[:, :, r:] -= Vs[t][:, :, None] * Z[t][:, None, r:] + Z[t][:, :, None] * Vs[t][:, None, r:]
    for c in range(r, k):
        piv = A[:, c, c]
        l = np.where(rows[None, :] > c, A[:, :, c] / piv[:, None], 0.0)
        A[:, :, c + 1:] -= l[:, :, None] * A[:, c, None, c + 1:]
        d -= l[:, :, None] * d[:, c, None, :]
    x = np.zeros_like(d)
    for c in range(k - 1, r - 1, -1):
        x[:, c] = d[:, c] / A[:, c, c][:, None]
        above = rows[None, :] < c
        d -= np.where(above[:, :, None], A[:, :, c, None] * x[:, c, None, :], 0.0)
    e = np.zeros((C, r, d.shape[2]))
    rhs_e = d[:, :r].copy()
    for t in range(r - 1, -1, -1):
        e[:, t] = rhs_e[:, t] / betas[t][:, None]
        rhs_e[:, :t] -= P[:, :t, t, None] * e[:, t, None, :]
    c = apply_left(np.stack(Vs, 1), np.stack(taus, 1), x, reverse=True)
    return np.concatenate([c, e], axis=1)


def ns_refined(lhs, rhs, k):
    """One step of fixed-precision iterative refinement on top of the kernel's solve: the float64
    residual of the first k rows (the constraint rows' residual is dropped: P^T c = 0 holds to
    rounding by construction) re-solved with the same method, the correction added."""
    c0 = ns_kernel_coeffs(lhs, rhs, k)
    res = rhs - np.einsum("cij,cjs->cis", lhs, c0)
    res[:, k:] = 0.0
    return c0 + ns_kernel_coeffs(lhs, res, k)


def refinement_study():
    """Null-space error against the extended-precision truth, without and with one refinement
    step, next to LAPACK's, on uniform clouds (the kernel's voxel-centred isotropic coordinates)."""
    from scipy.spatial import KDTree

    rng = np.random.default_rng(7)
    for kern, k in (("thin_plate_spline", 20), ("thin_plate_spline", 32), ("cubic", 14), ("linear", 30)):
        n, G = 5000, 14
        y = rng.uniform(-0.5, G - 0.5, (n, 3))
        vals = rng.standard_normal((n, 3))
        ax = np.linspace(0, G - 1, G)
        x = grid_q(ax, ax, ax)
        degree = max(cpu_ref.RBF_MIN_DEGREE.get(kern, -1), 0)
        powers = cpu_ref.monomial_powers(degree)
        phi = cpu_ref.RBF_PHI[kern]
        m = k + powers.shape[0]
        _, idx = KDTree(y).query(x, k)
        idx = np.sort(idx, axis=1)
        yn = y[idx]
        diff = yn[:, :, None, :] - yn[:, None, :, :]
        lhs = np.zeros((len(x), m, m))
        lhs[:, :k, :k] = phi(np.sqrt((diff[..., 0] ** 2 + diff[..., 1] ** 2) + diff[..., 2] ** 2))
        rel = yn - x[:, None, :]
        P = cpu_ref._poly(rel / np.abs(rel).max(axis=(1, 2))[:, None, None], powers)
        lhs[:, :k, k:] = P
        lhs[:, k:, :k] = np.swapaxes(P, 1, 2)
        rhs = np.zeros((len(x), m, 3))
        rhs[:, :k] = vals[idx]
        dq = x[:, None, :] - yn
        vec = np.concatenate([phi(np.sqrt((dq[..., 0] ** 2 + dq[..., 1] ** 2) + dq[..., 2] ** 2)),
                              cpu_ref._poly(np.zeros_like(x), powers)], axis=1)
        ext = np.einsum("qm,qms->qs", vec.astype(np.longdouble), cpu_ref.solve_extended(lhs, rhs)).astype(float)
        err = lambda c: max(normwise(np.einsum("qm,qms->qs", vec, c)[:, i], ext[:, i]) for i in range(3))
        e_lap = err(np.linalg.solve(lhs, rhs))
        e_ns = err(ns_kernel_coeffs(lhs, rhs, k))
        e_ir = err(ns_refined(lhs, rhs, k))
        print(f"{kern:18s} k={k:3d}: vs exact  lapack {e_lap:.2e}  null-space {e_ns:.2e} ({e_ns / e_lap:.1f}x)  "
              f"+1 refinement step {e_ir:.2e} ({e_ir / e_lap:.1f}x)")


def rbf_points(points, values, queries, k, kernel, epsilon=None, degree=None, smoothing=0.0, solver="ns"):
    from scipy.spatial import KDTree

    y = np.asarray(points, float)
    d = np.asarray(values, float).reshape(len(y), -1)
    x = np.asarray(queries, float).reshape(-1, 3)
    epsilon = 1.0 if epsilon is None else epsilon
    if degree is None:
        degree = max(cpu_ref.RBF_MIN_DEGREE.get(kernel, -1), 0)
    powers = cpu_ref.monomial_powers(degree)
    k = int(min(k, len(y)))
    sm = np.broadcast_to(np.asarray(smoothing, float), (len(y),))
    phi = cpu_ref.RBF_PHI[kernel]
    R = powers.shape[0]
    m = k + R
    _, idx = KDTree(y).query(x, k)
    idx = np.sort(np.asarray(idx).reshape(len(x), k), axis=1)
    yn = y[idx]
    mins, maxs = yn.min(axis=1), yn.max(axis=1)
    shift = (maxs + mins) / 2
    scale = (maxs - mins) / 2
    scale[scale == 0.0] = 1.0
    ye = yn * epsilon
    diff = ye[:, :, None, :] - ye[:, None, :, :]
    rr = np.sqrt((diff[..., 0] ** 2 + diff[..., 1] ** 2) + diff[..., 2] ** 2)
    lhs = np.zeros((len(x), m, m))
    lhs[:, :k, :k] = phi(rr)
    lhs[:, np.arange(k), np.arange(k)] += sm[idx]
    P = cpu_ref._poly((yn - shift[:, None, :]) / scale[:, None, :], powers)
    lhs[:, :k, k:] = P
    lhs[:, k:, :k] = np.swapaxes(P, 1, 2)
    rhs = np.zeros((len(x), m, d.shape[1]))
    rhs[:, :k] = d[idx]
    dq = x[:, None, :] * epsilon - ye
    rq = np.sqrt((dq[..., 0] ** 2 + dq[..., 1] ** 2) + dq[..., 2] ** 2)
    vec = np.concatenate([phi(rq), cpu_ref._poly((x - shift) / scale, powers)], axis=1)
    info = {}
    if solver == "ns":
        coeffs, beta, B = solve_nullspace(lhs, rhs, k)
        info["min_rdiag_rel"] = float(np.min(np.abs(beta) / np.sqrt(k)))
        ev = np.linalg.eigvalsh(B)
        info["B_min_eig"] = float(ev[:, 0].min())
        info["B_cond_max"] = float(np.max(ev[:, -1] / ev[:, 0]))
        info["A_cond_max"] = float(np.max(np.linalg.cond(lhs)))
    elif solver == "kernel":
        return ns_kernel_order(lhs, rhs, k, vec), info
    elif solver == "lapack":
        coeffs = np.linalg.solve(lhs, rhs)
    else:
        coeffs = cpu_ref.solve_extended(lhs, rhs)
        return np.einsum("qm,qms->qs", vec.astype(np.longdouble), coeffs).astype(float), info
    return np.einsum("qm,qms->qs", vec, coeffs), info


def grid_q(ax, ay, az):
    Z, Y, X = np.meshgrid(az, ay, ax, indexing="ij")
    return np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)


def main():
    import glob

    for p in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "rbf_*.npz"))):
        name = os.path.basename(p)[:-4]
        if "gaussian" in name or "parallel" in name:
            continue
        g = load(name)
        q = grid_q(g["ax"], g["ay"], g["az"])
        kern = str(g["kernel"])
        out, info = rbf_points(g["points"], g["values"], q, int(g["k"]), kern,
                               smoothing=float(g["smoothing"]))
        ext, _ = rbf_points(g["points"], g["values"], q, int(g["k"]), kern,
                            smoothing=float(g["smoothing"]), solver="ext")
        ko, _ = rbf_points(g["points"], g["values"], q, int(g["k"]), kern,
                           smoothing=float(g["smoothing"]), solver="kernel")
        ref = np.stack([g["U"].ravel(), g["V"].ravel(), g["W"].ravel()], -1)
        print(f"{name:40s} kernel-order-vs-ref {max(normwise(ko[:, i], ref[:, i]) for i in range(3)):.2e}")
        e_ref = max(normwise(out[:, i], ref[:, i]) for i in range(3))
        e_ex = max(normwise(out[:, i], ext[:, i]) for i in range(3))
        l_ex = max(normwise(ref[:, i], ext[:, i]) for i in range(3))
        print(f"{name:40s} ns-vs-ref {e_ref:.2e}  ns-vs-exact {e_ex:.2e}  lapack-vs-exact {l_ex:.2e}  {info}")
    rng = np.random.default_rng(1)
    for kern, k, G in (("thin_plate_spline", 20, 12), ("thin_plate_spline", 32, 12), ("cubic", 20, 10),
                       ("quintic", 30, 10), ("linear", 16, 10), ("thin_plate_spline", 50, 8)):
        n = 3000
        P = rng.uniform(-0.5, G - 0.5, (n, 3))
        Q = rng.standard_normal((n, 3))
        ax = np.linspace(0, G - 1, G)
        q = grid_q(ax, ax, ax)
        out, info = rbf_points(P, Q, q, k, kern)
        ref, _ = rbf_points(P, Q, q, k, kern, solver="lapack")
        ext, _ = rbf_points(P, Q, q, k, kern, solver="ext")
        e_ref = max(normwise(out[:, i], ref[:, i]) for i in range(3))
        e_ex = max(normwise(out[:, i], ext[:, i]) for i in range(3))
        l_ex = max(normwise(ref[:, i], ext[:, i]) for i in range(3))
        print(f"rand {kern:18s} k={k:3d}                  ns-vs-lapack {e_ref:.2e}  ns-vs-exact {e_ex:.2e}  lapack-vs-exact {l_ex:.2e}  {info}")


if __name__ == "__main__":
    if "--refine" in sys.argv:
        refinement_study()
    else:
        main()
