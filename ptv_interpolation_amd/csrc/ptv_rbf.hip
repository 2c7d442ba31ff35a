// ptv_rbf.hip — local RBF interpolation onto a voxel grid (gfx950): one small dense
// solve per voxel.
//
// Replaces, per voxel q, what scipy's RBFInterpolator(neighbors=k) does inside
// interpolate_field(method='rbf') (interpolator.py:157-195):
//   _, yindices = tree.query(x, k); yindices = np.sort(yindices, axis=1)   _rbfinterp.py:513-521
//   lhs, rhs, shift, scale = _build_system(y[idx], d[idx], smoothing, kernel, epsilon, powers)
//   coeffs = dgesv(lhs, rhs)                                                _rbfinterp.py:113
//   out = [phi(eps*|x - y_j|) ..., P((x - shift)/scale) ...] @ coeffs       _rbfinterp.py:404-418
// The k-NN lists come from k_knn_interp in slot mode (ptv_knn.hip); this kernel gathers
// the k particle records, orders them by particle index (the np.sort above, so the
// system rows are in the reference's order), builds the (k + r) x (k + r) system
//   [ phi(eps*||y_i - y_j||) + s_i*delta_ij   P(yhat_i) ]   [c]   [d]
//   [ P(yhat_j)^T                             0        ] . [e] = [0]
// with yhat = (y - shift)/scale, shift = (max + min)/2, scale = (max - min)/2 (0 -> 1)
// over the neighbourhood, factors it by Gaussian elimination with partial pivoting and
// evaluates the interpolant at q.
//
// MI355X mapping (fp64 vector ALU bound, no MFMA: the work is k^3/3 dependent rank-1
// updates of a <= 64 x 64 system per voxel, not a contraction):
//   * one system per L-lane segment of a wave64 (L = 16, 32 or 64 >= M, the system size
//     padded to a multiple of 8 with an identity block), so two to four voxels share a
//     wave when M <= 32;
//   * lane i of a segment holds ROW i of the system in registers (M doubles), the
//     pivot search is a segment max-reduction over the lanes (cross-lane shuffles), the
//     pivot row is broadcast through a per-segment LDS row, and rows are never moved:
//     partial pivoting is a per-lane "done" flag plus the LAPACK row position (idamax
//     tie order: the lowest current position wins);
//   * the right-hand sides (u, v, w) ride along in three more registers, back
//     substitution is column-oriented through LDS, and the evaluation is a segment
//     dot product.
// Numerics: the same formulas as scipy's Pythran kernels (phi on eps-scaled
// coordinates, r = sqrt((dx^2 + dy^2) + dz^2), monomials as products of integer
// powers); elimination uses fused multiply-adds like the OpenBLAS dger kernels.  The
// factorisation order differs from LAPACK's blocked dgetrf, so results agree with the
// reference to the conditioning of the system (see tests/test_gpu_rbf.py and DESIGN.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"
#include "ptv_rbf_math.hpp"

namespace ptv {

// Entries j in [j0, j0 + n) of system row li, into the lane's column of the per-wave LDS
// scratch (sc[jj * 64 + lane]).  A rolled loop: the phi / monomial code is emitted once, so
// the kernel stays small (a fully unrolled build is M copies of log/exp/sqrt and thrashes
// the instruction cache).
template <int KERN>
__device__ __forceinline__ void build_entries(double *__restrict__ sc, int lane, int j0, int n, int k, int m, int li,
                                              const double4 *__restrict__ ye, const double4 *__restrict__ yh,
                                              double4 yi, double4 hi, double si, const int *__restrict__ pw,
                                              int tcode) {
#pragma unroll 1
    for (int jj = 0; jj < n; ++jj) {
        const int j = j0 + jj;
        double e = 0.0;
        if (li < k) {
            if (j < k) {
                const double4 yj = ye[j];
                const double dx = yi.x - yj.x, dy = yi.y - yj.y, dz = yi.z - yj.z;
                e = rbf_phi<KERN>(sqrt((dx * dx + dy * dy) + dz * dz));
                if (j == li) e = e + si;
            } else if (j < m) {
                e = mono(hi.x, hi.y, hi.z, pw[j - k]);
            }
        } else if (li < m) {
            if (j < k) {
                const double4 hj = yh[j];
                e = mono(hj.x, hj.y, hj.z, tcode);
            }
        } else {
            e = j == li ? 1.0 : 0.0;  // identity padding up to M
        }
        sc[jj * 64 + lane] = e;
    }
}

constexpr int kBuildCols = 8;  // system columns built per LDS round (8: 44 KB of LDS per block, 3 blocks per CU)

template <int M, int L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(M <= 32 ? 3 : 1))) void k_rbf_local(RbfKernelArgs a, const double4 *__restrict__ prec,
                                                   const double4 *__restrict__ pval,
                                                   const uint32_t *__restrict__ slots,
                                                   const double *__restrict__ ax, const double *__restrict__ ay,
                                                   const double *__restrict__ az, const double *__restrict__ qpx,
                                                   const double *__restrict__ qpy, const double *__restrict__ qpz,
                                                   const double *__restrict__ smooth, const int *__restrict__ pw,
                                                   const uint8_t *__restrict__ mask, double *__restrict__ U,
                                                   double *__restrict__ V, double *__restrict__ W,
                                                   int *__restrict__ status) {
    static_assert(M <= L && L <= 64 && (64 % L) == 0, "segment must hold the system");
    constexpr int SPW = 64 / L;
    __shared__ double4 s_ye[4][64];   // eps-scaled coordinates (x, y, z, particle id) in id order
    __shared__ double4 s_yh[4][64];   // normalised coordinates yhat in id order
    __shared__ double4 s_val[4][64];  // data values (u, v, w) in id order; later the solution
    __shared__ double s_row[4][SPW][M + 4];
    __shared__ uint32_t s_id[4][64];
    __shared__ double s_build[4][kBuildCols * 64];  // row build scratch, [column][lane]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int seg = lane / L, li = lane % L, sb = seg * L;
    double4 *ye = s_ye[wid] + sb;
    double4 *yh = s_yh[wid] + sb;
    double4 *sv = s_val[wid] + sb;
    double *prow_buf = s_row[wid][seg];

    const long long plane = (long long)a.nx * a.ny;
    const long long nvox = (long long)(a.z1 - a.z0) * plane;
    long long v = ((long long)blockIdx.x * 4 + wid) * SPW + seg;  // chunk-local voxel
    bool valid = v < nvox;
    if (a.vlist != nullptr) {  // list mode: the voxels k_rbf_ns handed over (count on the device)
        const long long n = min((long long)*a.vcount, (long long)a.ns_cap);
        valid = v < n;
        // the grid is sized for the whole list: waves past the count leave at once (the solve below
        // is branch-free, and 16384 voxels of it cost ~0.1 ms per chunk when the list is empty)
        if (__builtin_amdgcn_ballot_w64(valid) == 0) return;
        v = valid ? (long long)a.vlist[v] : 0;
    }
    const long long vc = valid ? v : nvox - 1;
    const int iz = a.z0 + (int)(vc / plane);
    const long long rem = vc % plane;
    const int iy = (int)(rem / a.nx), ix = (int)(rem % a.nx);
    const size_t vfull = (size_t)iz * plane + rem;
    const bool active = valid && (mask == nullptr || mask[vfull] != 0);
    const int k = a.k, m = a.m;
    const double eps = a.epsilon;

    // ---- 1. the k neighbours, ranked by particle index (np.sort(yindices), _rbfinterp.py:521) ----
    const bool nb = active && li < k;
    double4 r = make_double4(0.0, 0.0, 0.0, 0.0), d = make_double4(0.0, 0.0, 0.0, 0.0);
    uint32_t id = 0xffffffffu;
    if (nb) {
        const uint32_t s = slots[(size_t)v * k + li];
        r = prec[s];
        d = pval[s];
        id = (uint32_t)r.w;
    }
    s_id[wid][lane] = id;
    double mnx = seg_min<L>(nb ? r.x : INFINITY), mxx = seg_max<L>(nb ? r.x : -INFINITY);
    double mny = seg_min<L>(nb ? r.y : INFINITY), mxy = seg_max<L>(nb ? r.y : -INFINITY);
    double mnz = seg_min<L>(nb ? r.z : INFINITY), mxz = seg_max<L>(nb ? r.z : -INFINITY);
    // _build_system: shift = (maxs + mins)/2, scale = (maxs - mins)/2, zero scale -> 1
    double shx = 0.0, shy = 0.0, shz = 0.0, scx = 1.0, scy = 1.0, scz = 1.0;
    if (active) {
        shx = (mxx + mnx) / 2.0;
        shy = (mxy + mny) / 2.0;
        shz = (mxz + mnz) / 2.0;
        scx = (mxx - mnx) / 2.0;
        scy = (mxy - mny) / 2.0;
        scz = (mxz - mnz) / 2.0;
        if (scx == 0.0) scx = 1.0;
        if (scy == 0.0) scy = 1.0;
        if (scz == 0.0) scz = 1.0;
    }
    rbf_wave_sync();
    int rank = 0;
    for (int j = 0; j < k; ++j) {
        const uint32_t o = s_id[wid][sb + j];
        rank += (o < id || (o == id && j < li)) ? 1 : 0;
    }
    if (li < k) {
        ye[rank] = make_double4(r.x * eps, r.y * eps, r.z * eps, (double)id);
        yh[rank] = make_double4((r.x - shx) / scx, (r.y - shy) / scy, (r.z - shz) / scz, 0.0);
        sv[rank] = d;
    }
    rbf_wave_sync();

    // ---- 2. row li of the system: [phi + s_i delta | P(yhat_i)] for kernel rows, [P(yhat_j)^T | 0]
    // for the polynomial rows, identity padding up to M; built BH columns at a time through LDS ----
    const bool krow = li < k;
    double A[M];
    const double4 yi = krow ? ye[li] : make_double4(0.0, 0.0, 0.0, 0.0);
    const double4 hi = krow ? yh[li] : make_double4(0.0, 0.0, 0.0, 0.0);
    const int tcode = (li >= k && li < m) ? pw[li - k] : 0;
    double si = 0.0;
    if (krow && active) si = smooth != nullptr ? smooth[(size_t)yi.w] : a.smoothing;
    double *sc = s_build[wid];
#pragma unroll
    for (int g = 0; g < M; g += kBuildCols) {
        const int n = M - g < kBuildCols ? M - g : kBuildCols;
        switch (a.kernel) {
#define PTV_BCASE(KK) \
    case KK: build_entries<KK>(sc, lane, g, n, k, m, li, ye, yh, yi, hi, si, pw, tcode); break;
            PTV_BCASE(PTV_RBF_LINEAR)
            PTV_BCASE(PTV_RBF_THIN_PLATE_SPLINE)
            PTV_BCASE(PTV_RBF_CUBIC)
            PTV_BCASE(PTV_RBF_QUINTIC)
            PTV_BCASE(PTV_RBF_MULTIQUADRIC)
            PTV_BCASE(PTV_RBF_INVERSE_MULTIQUADRIC)
            PTV_BCASE(PTV_RBF_INVERSE_QUADRATIC)
            default: build_entries<PTV_RBF_GAUSSIAN>(sc, lane, g, n, k, m, li, ye, yh, yi, hi, si, pw, tcode);
#undef PTV_BCASE
        }
        // each lane reads back only its own column of the scratch: no cross-lane hazard
#pragma unroll
        for (int jj = 0; jj < kBuildCols; ++jj)
            if (g + jj < M) A[g + jj] = sc[jj * 64 + lane];
    }
    double b0 = 0.0, b1 = 0.0, b2 = 0.0;
    if (krow) {
        const double4 dv = sv[li];
        b0 = dv.x;
        b1 = dv.y;
        b2 = dv.z;
    }

    // ---- 3. Gaussian elimination with partial pivoting; rows stay in their lanes ----
    // Pivot choice as one u32 segment max: the key is the top bits of |A[c]| (exponent and 13
    // mantissa bits; a nonzero value never maps to class 0) above (64 - pos), so the largest
    // |a| wins and, among keys equal in those bits, the lowest LAPACK row position (idamax's
    // first index).  The pivot row goes to the segment through LDS; every other row updates
    // branch-free (l = 0 for finished rows).
    bool done = li >= M;  // lanes beyond the padded system never pivot
    int pos = li;         // LAPACK row position
    int mystep = -1;      // the elimination step that used this row as pivot
    double diag = 1.0;    // this row's pivot (U diagonal entry)
    bool singular = false;
#pragma unroll
    for (int c = 0; c < M; ++c) {
        const unsigned long long ab = (unsigned long long)__double_as_longlong(fabs(A[c]));
        unsigned hi = (unsigned)(ab >> 32);
        hi = (ab != 0ull && hi < 128u) ? 128u : hi;
        const unsigned key = done ? 0u : ((hi & ~127u) | (unsigned)(64 - pos));
        const unsigned mk = seg_max_u32<L>(key);
        const bool isP = key == mk;
        singular = singular || (mk >> 7) == 0u;
        if (isP) {
#pragma unroll
            for (int j = c; j < M; ++j) prow_buf[j] = A[j];
            prow_buf[M] = b0;
            prow_buf[M + 1] = b1;
            prow_buf[M + 2] = b2;
            prow_buf[M + 3] = (double)pos;
            diag = A[c];
            mystep = c;
        }
        rbf_wave_sync();
        const double piv = prow_buf[c];
        const bool upd = !done && !isP;
        if (upd && pos == c) pos = (int)prow_buf[M + 3];  // the swap moves this row to the pivot's position
        const double l = (upd && piv != 0.0) ? elim_multiplier(A[c], piv) : 0.0;
#pragma unroll
        for (int j = c + 1; j < M; ++j) A[j] = fma(-l, prow_buf[j], A[j]);
        b0 = fma(-l, prow_buf[M], b0);
        b1 = fma(-l, prow_buf[M + 1], b1);
        b2 = fma(-l, prow_buf[M + 2], b2);
        done = done || isP;
        rbf_wave_sync();
    }

    // ---- 4. back substitution (column oriented, dtrsm order); solution in LDS ----
    const double rdiag = 1.0 / diag;
#pragma unroll
    for (int c = M - 1; c >= 0; --c) {
        if (mystep == c) sv[c] = make_double4(b0 * rdiag, b1 * rdiag, b2 * rdiag, 0.0);
        rbf_wave_sync();
        const double4 xc = sv[c];
        const double u = (mystep >= 0 && mystep < c) ? A[c] : 0.0;
        b0 = fma(-u, xc.x, b0);
        b1 = fma(-u, xc.y, b1);
        b2 = fma(-u, xc.z, b2);
    }

    // ---- 5. evaluate at the voxel: [phi(eps*|x - y_j|), P(xhat)] . coeffs ----
    double qx, qy, qz;
    if (a.separable) {
        qx = ax[ix];
        qy = ay[iy];
        qz = az[iz];
    } else {
        qx = qpx[vfull];
        qy = qpy[vfull];
        qz = qpz[vfull];
    }
    double e = 0.0;
    if (li < k) {
        const double dx = qx * eps - yi.x, dy = qy * eps - yi.y, dz = qz * eps - yi.z;
        e = rbf_phi_rt(a.kernel, sqrt((dx * dx + dy * dy) + dz * dz));
    } else if (li < m) {
        e = mono((qx - shx) / scx, (qy - shy) / scy, (qz - shz) / scz, pw[li - k]);
    }
    double4 cf = make_double4(0.0, 0.0, 0.0, 0.0);
    if (li < m) cf = sv[li];
    double o0 = seg_sum<L>(e * cf.x), o1 = seg_sum<L>(e * cf.y), o2 = seg_sum<L>(e * cf.z);
    if (!valid || li != 0) return;
    const size_t vo = (size_t)(iz - a.out_z0) * plane + rem;
    if (!active) {
        U[vo] = 0.0;
        V[vo] = 0.0;
        W[vo] = 0.0;
        return;
    }
    if (singular) {
        atomicAdd(&status[0], 1);
        atomicMin(&status[1], (int)min((long long)vfull, 0x7fffffffLL));
    }
    if (a.flags & PTV_FLAG_NAN_TO_NUM) {
        auto fix = [](double x) { return x != x ? 0.0 : (x == INFINITY ? DBL_MAX : (x == -INFINITY ? -DBL_MAX : x)); };
        o0 = fix(o0);
        o1 = fix(o1);
        o2 = fix(o2);
    }
    U[vo] = o0;
    V[vo] = o1;
    W[vo] = o2;
}

// ---------------------------------------------------------------------------
// Systems of 64 < m <= 128 (k_rbf_local keeps a row per lane, so 64 rows at most): one wave
// per voxel with the m x (m + 3) augmented matrix in (dynamic) LDS and explicit row swaps.
// The same entries (build_entries' formulas), LAPACK's idamax pivot (largest |a|, lowest row
// among equal ones), dgetf2's reciprocal multipliers (elim_multiplier), fma updates, the
// reciprocal back substitution and the segment-sum evaluation of k_rbf_local.  A rare
// configuration (k >= ~60 with a polynomial, or k >= 65): correctness over speed.
// ---------------------------------------------------------------------------
constexpr int kRbfBigRows = 128;

size_t rbf_big_lds_bytes(int m) {
    return (size_t)m * (m + 3) * sizeof(double) + 3 * kRbfBigRows * sizeof(double4) + kRbfBigRows * sizeof(uint32_t);
}

__global__ __launch_bounds__(64) void k_rbf_big(RbfKernelArgs a, const double4 *__restrict__ prec,
                                                const double4 *__restrict__ pval, const uint32_t *__restrict__ slots,
                                                const double *__restrict__ ax, const double *__restrict__ ay,
                                                const double *__restrict__ az, const double *__restrict__ qpx,
                                                const double *__restrict__ qpy, const double *__restrict__ qpz,
                                                const double *__restrict__ smooth, const int *__restrict__ pw,
                                                const uint8_t *__restrict__ mask, double *__restrict__ U,
                                                double *__restrict__ V, double *__restrict__ W,
                                                int *__restrict__ status) {
    extern __shared__ double lds_big[];
    const int lane = threadIdx.x;
    const int k = a.k, m = a.m, ld = m + 3;
    double *A = lds_big;                                             // row i at A + i * ld
    double4 *ye = reinterpret_cast<double4 *>(A + (size_t)m * ld);   // eps-scaled (x, y, z, id), id order
    double4 *yh = ye + kRbfBigRows;                                  // yhat, id order
    double4 *sv = yh + kRbfBigRows;                                  // values, later the solution
    uint32_t *sid = reinterpret_cast<uint32_t *>(sv + kRbfBigRows);  // ids in list order

    const long long plane = (long long)a.nx * a.ny;
    const long long v = blockIdx.x;  // chunk-local voxel (the grid is exactly the chunk)
    const int iz = a.z0 + (int)(v / plane);
    const long long rem = v % plane;
    const int iy = (int)(rem / a.nx), ix = (int)(rem % a.nx);
    const size_t vfull = (size_t)iz * plane + rem;
    const size_t vo = (size_t)(iz - a.out_z0) * plane + rem;
    if (mask != nullptr && mask[vfull] == 0) {  // wave-uniform (one voxel per wave)
        if (lane == 0) {
            U[vo] = 0.0;
            V[vo] = 0.0;
            W[vo] = 0.0;
        }
        return;
    }
    const double eps = a.epsilon;

    // ---- 1. the k neighbours (two per lane), ranked by particle index ----
    double4 r[2], d[2];
    uint32_t id[2];
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        r[h] = make_double4(0.0, 0.0, 0.0, 0.0);
        d[h] = r[h];
        id[h] = 0xffffffffu;
        if (j < k) {
            const uint32_t s = slots[(size_t)v * k + j];
            r[h] = prec[s];
            d[h] = pval[s];
            id[h] = (uint32_t)r[h].w;
            mn[0] = fmin(mn[0], r[h].x);
            mn[1] = fmin(mn[1], r[h].y);
            mn[2] = fmin(mn[2], r[h].z);
            mx[0] = fmax(mx[0], r[h].x);
            mx[1] = fmax(mx[1], r[h].y);
            mx[2] = fmax(mx[2], r[h].z);
        }
        if (j < kRbfBigRows) sid[j] = id[h];
    }
    double sh[3], scl[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double lo = seg_min<64>(mn[c]), hi = seg_max<64>(mx[c]);
        sh[c] = (hi + lo) / 2.0;  // _build_system: shift = (max + min)/2, scale = (max - min)/2 (0 -> 1)
        scl[c] = (hi - lo) / 2.0;
        if (scl[c] == 0.0) scl[c] = 1.0;
    }
    rbf_wave_sync();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        if (j < k) {
            int rank = 0;
            for (int t = 0; t < k; ++t) {
                const uint32_t o = sid[t];
                rank += (o < id[h] || (o == id[h] && t < j)) ? 1 : 0;
            }
            ye[rank] = make_double4(r[h].x * eps, r[h].y * eps, r[h].z * eps, (double)id[h]);
            yh[rank] = make_double4((r[h].x - sh[0]) / scl[0], (r[h].y - sh[1]) / scl[1], (r[h].z - sh[2]) / scl[2], 0.0);
            sv[rank] = d[h];
        }
    }
    rbf_wave_sync();

    // ---- 2. the augmented system, row by row (lanes over the columns and the 3 right-hand sides) ----
    for (int i = 0; i < m; ++i) {
        const bool krow = i < k;
        const double4 yi = krow ? ye[i] : make_double4(0.0, 0.0, 0.0, 0.0);
        const double4 hi = krow ? yh[i] : make_double4(0.0, 0.0, 0.0, 0.0);
        const int tcode = krow ? 0 : pw[i - k];
        double si = 0.0;
        if (krow) si = smooth != nullptr ? smooth[(size_t)yi.w] : a.smoothing;
        for (int j = lane; j < ld; j += 64) {
            double e = 0.0;
            if (j < m) {
                if (krow) {
                    if (j < k) {
                        const double4 yj = ye[j];
                        const double dx = yi.x - yj.x, dy = yi.y - yj.y, dz = yi.z - yj.z;
                        e = rbf_phi_rt(a.kernel, sqrt((dx * dx + dy * dy) + dz * dz));
                        if (j == i) e = e + si;
                    } else {
                        e = mono(hi.x, hi.y, hi.z, pw[j - k]);
                    }
                } else if (j < k) {
                    const double4 hj = yh[j];
                    e = mono(hj.x, hj.y, hj.z, tcode);
                }
            } else if (krow) {
                const double4 dv = sv[i];
                e = j == m ? dv.x : (j == m + 1 ? dv.y : dv.z);
            }
            A[(size_t)i * ld + j] = e;
        }
    }
    rbf_wave_sync();

    // ---- 3. LU with partial pivoting (explicit row swaps), the right-hand sides along ----
    bool singular = false;
    for (int c = 0; c < m; ++c) {
        double best = -1.0;
        int brow = m;
        for (int i = c + lane; i < m; i += 64) {
            const double q = fabs(A[(size_t)i * ld + c]);
            if (q > best) {  // rows ascend per lane: the first maximum is the lowest row
                best = q;
                brow = i;
            }
        }
        const double bmax = seg_max<64>(best);
        const int p = -(int)seg_max<64>(best == bmax ? -(double)brow : -(double)m);  // lowest row holding it
        singular = singular || !(bmax > 0.0);
        if (p != c) {
            for (int j = lane; j < ld; j += 64) {
                const double t = A[(size_t)c * ld + j];
                A[(size_t)c * ld + j] = A[(size_t)p * ld + j];
                A[(size_t)p * ld + j] = t;
            }
        }
        rbf_wave_sync();
        const double piv = A[(size_t)c * ld + c];
        for (int i = c + 1 + lane; i < m; i += 64) {
            const double aic = A[(size_t)i * ld + c];
            A[(size_t)i * ld + c] = piv != 0.0 ? elim_multiplier(aic, piv) : 0.0;
        }
        rbf_wave_sync();
        for (int j = c + 1 + lane; j < ld; j += 64) {
            const double pj = A[(size_t)c * ld + j];
            for (int i = c + 1; i < m; ++i) {
                const double l = A[(size_t)i * ld + c];
                A[(size_t)i * ld + j] = fma(-l, pj, A[(size_t)i * ld + j]);
            }
        }
        rbf_wave_sync();
    }

    // ---- 4. back substitution (column oriented), x_c = b_c * (1 / u_cc) into sv ----
    for (int c = m - 1; c >= 0; --c) {
        if (lane == 0) {
            const double rd = 1.0 / A[(size_t)c * ld + c];
            sv[c] = make_double4(A[(size_t)c * ld + m] * rd, A[(size_t)c * ld + m + 1] * rd, A[(size_t)c * ld + m + 2] * rd, 0.0);
        }
        rbf_wave_sync();
        const double4 xc = sv[c];
        for (int i = lane; i < c; i += 64) {
            const double u = A[(size_t)i * ld + c];
            A[(size_t)i * ld + m] = fma(-u, xc.x, A[(size_t)i * ld + m]);
            A[(size_t)i * ld + m + 1] = fma(-u, xc.y, A[(size_t)i * ld + m + 1]);
            A[(size_t)i * ld + m + 2] = fma(-u, xc.z, A[(size_t)i * ld + m + 2]);
        }
        rbf_wave_sync();
    }

    // ---- 5. evaluate at the voxel ----
    double qx, qy, qz;
    if (a.separable) {
        qx = ax[ix];
        qy = ay[iy];
        qz = az[iz];
    } else {
        qx = qpx[vfull];
        qy = qpy[vfull];
        qz = qpz[vfull];
    }
    double o[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        double e = 0.0;
        if (j < k) {
            const double4 yj = ye[j];
            const double dx = qx * eps - yj.x, dy = qy * eps - yj.y, dz = qz * eps - yj.z;
            e = rbf_phi_rt(a.kernel, sqrt((dx * dx + dy * dy) + dz * dz));
        } else if (j < m) {
            e = mono((qx - sh[0]) / scl[0], (qy - sh[1]) / scl[1], (qz - sh[2]) / scl[2], pw[j - k]);
        }
        if (j < m) {
            const double4 cf = sv[j];
            o[0] += e * cf.x;
            o[1] += e * cf.y;
            o[2] += e * cf.z;
        }
    }
    double o0 = seg_sum<64>(o[0]), o1 = seg_sum<64>(o[1]), o2 = seg_sum<64>(o[2]);
    if (lane != 0) return;
    if (singular) {
        atomicAdd(&status[0], 1);
        atomicMin(&status[1], (int)min((long long)vfull, 0x7fffffffLL));
    }
    if (a.flags & PTV_FLAG_NAN_TO_NUM) {
        auto fix = [](double x) { return x != x ? 0.0 : (x == INFINITY ? DBL_MAX : (x == -INFINITY ? -DBL_MAX : x)); };
        o0 = fix(o0);
        o1 = fix(o1);
        o2 = fix(o2);
    }
    U[vo] = o0;
    V[vo] = o1;
    W[vo] = o2;
}

// ---------------------------------------------------------------------------
// Systems of m > 128 (k >= 125 with a linear polynomial, any k >= 129): k_rbf_big's algorithm --
// the same entries, idamax pivots with explicit row swaps, dgetf2's reciprocal multipliers, fma
// updates, the reciprocal back substitution -- with the augmented matrix and the neighbour tables
// in a global-memory slice per workgroup of a persistent grid (they outgrow the LDS).  The LU
// streams its trailing matrix through L2 / HBM each column: correctness over speed, for a
// configuration the reference's RBFInterpolator(neighbors=k) also takes (interpolator.py:157-195).
// ---------------------------------------------------------------------------
// order this wave's global stores before its later loads (one wave per workgroup)
__device__ __forceinline__ void huge_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

size_t rbf_huge_slice_doubles(int m, int k) {
    // A (m x (m + 3)); ye, yh, rec, val (k double4 each); sv (m double4); sid (k u32)
    return (size_t)m * (m + 3) + 4 * (4 * (size_t)k + (size_t)m) + ((size_t)k + 1) / 2 + 8;
}

__global__ __launch_bounds__(64) void k_rbf_huge(RbfKernelArgs a, const double4 *__restrict__ prec,
                                                 const double4 *__restrict__ pval, const uint32_t *__restrict__ slots,
                                                 const double *__restrict__ ax, const double *__restrict__ ay,
                                                 const double *__restrict__ az, const double *__restrict__ qpx,
                                                 const double *__restrict__ qpy, const double *__restrict__ qpz,
                                                 const double *__restrict__ smooth, const int *__restrict__ pw,
                                                 const uint8_t *__restrict__ mask, double *__restrict__ U,
                                                 double *__restrict__ V, double *__restrict__ W,
                                                 int *__restrict__ status, double *__restrict__ scratch, size_t slice,
                                                 long long nvox) {
    const int lane = threadIdx.x;
    const int k = a.k, m = a.m, ld = m + 3;
    double *A = scratch + (size_t)blockIdx.x * slice;                // row i at A + i * ld
    double4 *ye = reinterpret_cast<double4 *>(A + (size_t)m * ld);   // eps-scaled (x, y, z, id), id order
    double4 *yh = ye + k;                                            // yhat, id order
    double4 *rec = yh + k;                                           // records, list order
    double4 *val = rec + k;                                          // values, list order
    double4 *sv = val + k;                                           // values (id order), later the solution
    uint32_t *sid = reinterpret_cast<uint32_t *>(sv + m);            // ids, list order
    const long long plane = (long long)a.nx * a.ny;
    const double eps = a.epsilon;
    for (long long v = blockIdx.x; v < nvox; v += gridDim.x) {
        const int iz = a.z0 + (int)(v / plane);
        const long long rem = v % plane;
        const int iy = (int)(rem / a.nx), ix = (int)(rem % a.nx);
        const size_t vfull = (size_t)iz * plane + rem;
        const size_t vo = (size_t)(iz - a.out_z0) * plane + rem;
        if (mask != nullptr && mask[vfull] == 0) {  // wave-uniform (one voxel per wave)
            if (lane == 0) {
                U[vo] = 0.0;
                V[vo] = 0.0;
                W[vo] = 0.0;
            }
            continue;
        }
        // ---- 1. the k neighbours, ranked by particle index ----
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int j = lane; j < k; j += 64) {
            const uint32_t s = slots[(size_t)v * k + j];
            const double4 r = prec[s];
            rec[j] = r;
            val[j] = pval[s];
            sid[j] = (uint32_t)r.w;
            mn[0] = fmin(mn[0], r.x);
            mn[1] = fmin(mn[1], r.y);
            mn[2] = fmin(mn[2], r.z);
            mx[0] = fmax(mx[0], r.x);
            mx[1] = fmax(mx[1], r.y);
            mx[2] = fmax(mx[2], r.z);
        }
        double sh[3], scl[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double lo = seg_min<64>(mn[c]), hi = seg_max<64>(mx[c]);
            sh[c] = (hi + lo) / 2.0;  // _build_system: shift = (max + min)/2, scale = (max - min)/2 (0 -> 1)
            scl[c] = (hi - lo) / 2.0;
            if (scl[c] == 0.0) scl[c] = 1.0;
        }
        huge_sync();
        for (int j = lane; j < k; j += 64) {
            const uint32_t idj = sid[j];
            int rank = 0;
            for (int t = 0; t < k; ++t) {
                const uint32_t o = sid[t];
                rank += (o < idj || (o == idj && t < j)) ? 1 : 0;
            }
            const double4 r = rec[j];
            ye[rank] = make_double4(r.x * eps, r.y * eps, r.z * eps, (double)idj);
            yh[rank] = make_double4((r.x - sh[0]) / scl[0], (r.y - sh[1]) / scl[1], (r.z - sh[2]) / scl[2], 0.0);
            sv[rank] = val[j];
        }
        huge_sync();
        // ---- 2. the augmented system, row by row ----
        for (int i = 0; i < m; ++i) {
            const bool krow = i < k;
            const double4 yi = krow ? ye[i] : make_double4(0.0, 0.0, 0.0, 0.0);
            const double4 hi = krow ? yh[i] : make_double4(0.0, 0.0, 0.0, 0.0);
            const int tcode = krow ? 0 : pw[i - k];
            double si = 0.0;
            if (krow) si = smooth != nullptr ? smooth[(size_t)yi.w] : a.smoothing;
            for (int j = lane; j < ld; j += 64) {
                double e = 0.0;
                if (j < m) {
                    if (krow) {
                        if (j < k) {
                            const double4 yj = ye[j];
                            const double dx = yi.x - yj.x, dy = yi.y - yj.y, dz = yi.z - yj.z;
                            e = rbf_phi_rt(a.kernel, sqrt((dx * dx + dy * dy) + dz * dz));
                            if (j == i) e = e + si;
                        } else {
                            e = mono(hi.x, hi.y, hi.z, pw[j - k]);
                        }
                    } else if (j < k) {
                        const double4 hj = yh[j];
                        e = mono(hj.x, hj.y, hj.z, tcode);
                    }
                } else if (krow) {
                    const double4 dv = sv[i];
                    e = j == m ? dv.x : (j == m + 1 ? dv.y : dv.z);
                }
                A[(size_t)i * ld + j] = e;
            }
        }
        huge_sync();
        // ---- 3. LU with partial pivoting (explicit row swaps), the right-hand sides along ----
        bool singular = false;
        for (int c = 0; c < m; ++c) {
            double best = -1.0;
            int brow = m;
            for (int i = c + lane; i < m; i += 64) {
                const double q = fabs(A[(size_t)i * ld + c]);
                if (q > best) {  // rows ascend per lane: the first maximum is the lowest row
                    best = q;
                    brow = i;
                }
            }
            const double bmax = seg_max<64>(best);
            const int p = -(int)seg_max<64>(best == bmax ? -(double)brow : -(double)m);  // lowest row holding it
            singular = singular || !(bmax > 0.0);
            if (p != c) {
                for (int j = lane; j < ld; j += 64) {
                    const double t = A[(size_t)c * ld + j];
                    A[(size_t)c * ld + j] = A[(size_t)p * ld + j];
                    A[(size_t)p * ld + j] = t;
                }
            }
            huge_sync();
            const double piv = A[(size_t)c * ld + c];
            for (int i = c + 1 + lane; i < m; i += 64) {
                const double aic = A[(size_t)i * ld + c];
                A[(size_t)i * ld + c] = piv != 0.0 ? elim_multiplier(aic, piv) : 0.0;
            }
            huge_sync();
            for (int j = c + 1 + lane; j < ld; j += 64) {
                const double pj = A[(size_t)c * ld + j];
                for (int i = c + 1; i < m; ++i) {
                    const double l = A[(size_t)i * ld + c];
                    A[(size_t)i * ld + j] = fma(-l, pj, A[(size_t)i * ld + j]);
                }
            }
            huge_sync();
        }
        // ---- 4. back substitution (column oriented), x_c = b_c * (1 / u_cc) into sv ----
        for (int c = m - 1; c >= 0; --c) {
            if (lane == 0) {
                const double rd = 1.0 / A[(size_t)c * ld + c];
                sv[c] = make_double4(A[(size_t)c * ld + m] * rd, A[(size_t)c * ld + m + 1] * rd,
                                     A[(size_t)c * ld + m + 2] * rd, 0.0);
            }
            huge_sync();
            const double4 xc = sv[c];
            for (int i = lane; i < c; i += 64) {
                const double u = A[(size_t)i * ld + c];
                A[(size_t)i * ld + m] = fma(-u, xc.x, A[(size_t)i * ld + m]);
                A[(size_t)i * ld + m + 1] = fma(-u, xc.y, A[(size_t)i * ld + m + 1]);
                A[(size_t)i * ld + m + 2] = fma(-u, xc.z, A[(size_t)i * ld + m + 2]);
            }
            huge_sync();
        }
        // ---- 5. evaluate at the voxel ----
        double qx, qy, qz;
        if (a.separable) {
            qx = ax[ix];
            qy = ay[iy];
            qz = az[iz];
        } else {
            qx = qpx[vfull];
            qy = qpy[vfull];
            qz = qpz[vfull];
        }
        double o[3] = {0.0, 0.0, 0.0};
        for (int j = lane; j < m; j += 64) {
            double e;
            if (j < k) {
                const double4 yj = ye[j];
                const double dx = qx * eps - yj.x, dy = qy * eps - yj.y, dz = qz * eps - yj.z;
                e = rbf_phi_rt(a.kernel, sqrt((dx * dx + dy * dy) + dz * dz));
            } else {
                e = mono((qx - sh[0]) / scl[0], (qy - sh[1]) / scl[1], (qz - sh[2]) / scl[2], pw[j - k]);
            }
            const double4 cf = sv[j];
            o[0] += e * cf.x;
            o[1] += e * cf.y;
            o[2] += e * cf.z;
        }
        double o0 = seg_sum<64>(o[0]), o1 = seg_sum<64>(o[1]), o2 = seg_sum<64>(o[2]);
        if (lane == 0) {
            if (singular) {
                atomicAdd(&status[0], 1);
                atomicMin(&status[1], (int)min((long long)vfull, 0x7fffffffLL));
            }
            if (a.flags & PTV_FLAG_NAN_TO_NUM) {
                auto fix = [](double x) { return x != x ? 0.0 : (x == INFINITY ? DBL_MAX : (x == -INFINITY ? -DBL_MAX : x)); };
                o0 = fix(o0);
                o1 = fix(o1);
                o2 = fix(o2);
            }
            U[vo] = o0;
            V[vo] = o1;
            W[vo] = o2;
        }
        huge_sync();  // the slice is rewritten by the next voxel
    }
}

// ---------------------------------------------------------------------------
// Symmetric positive definite systems: kernel gaussian / inverse_multiquadric /
// inverse_quadratic with degree -1 (no polynomial block, m = k) and smoothing >= 0.  The
// matrix [phi(eps |y_i - y_j|) + s delta_ij] is SPD for distinct points, so Gaussian
// elimination needs no pivoting (stable, growth factor 1; measured on the reference's
// Gaussian eps=0.3 fixtures: 2.2e-10 .. 3.6e-10 normwise from the exact answer against
// LAPACK dgesv's 1.1e-9 .. 2.4e-9).  That removes the pivot search, the pivot-row
// bookkeeping and the dynamic back-substitution order; the build computes each
// symmetric pair once.
//   * build: segment lane i (row i) evaluates phi for the columns (i + d) mod L, d = 1..L/2,
//     into scratch[d - 1][lane]; entry (i, j) is then scratch[(j - i) mod L - 1][i] when
//     (j - i) mod L <= L/2, else scratch[(i - j) mod L - 1][j] (the partner's); L/2 phi
//     evaluations per row instead of k;
//   * elimination: step c's pivot row is row c (lane c of each segment), broadcast through a
//     double-buffered LDS row (one barrier per step);
//   * back substitution in the same fixed order (lane c holds x_c).
// ---------------------------------------------------------------------------
#ifndef PTV_RBF_SPD_WAVES
#define PTV_RBF_SPD_WAVES 3  // 4 fits the LDS (40 KB per block) but spills 48 VGPRs: 1006 vs 990 ms
#endif
template <int M, int L, int KERN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PTV_RBF_SPD_WAVES))) void k_rbf_spd(
    RbfKernelArgs a, const double4 *__restrict__ prec, const double4 *__restrict__ pval,
    const uint32_t *__restrict__ slots, const double *__restrict__ ax, const double *__restrict__ ay,
    const double *__restrict__ az, const double *__restrict__ qpx, const double *__restrict__ qpy,
    const double *__restrict__ qpz, const uint8_t *__restrict__ mask, double *__restrict__ U,
    double *__restrict__ V, double *__restrict__ W, int *__restrict__ status) {
    static_assert(M <= L && L <= 32 && (64 % L) == 0, "segment must hold the system (two or more per wave)");
    constexpr int SPW = 64 / L;
    constexpr int H = L / 2;  // phi evaluations per row
    __shared__ double4 s_ye[4][64];            // eps-scaled coordinates (x, y, z, particle id) in id order
    // per wave: the sorted values + ids, then the symmetric build scratch, then the pivot rows
    // (double buffered) and the back-substitution broadcasts: 40 KB per block, 4 blocks per CU
    __shared__ double s_sc[4][H * 64];
    static_assert(2 * SPW * (M + 3) <= H * 64, "pivot rows must fit the build scratch");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int seg = lane / L, li = lane % L, sb = seg * L;
    double4 *ye = s_ye[wid] + sb;
    double *sc = s_sc[wid];
    double4 *sv = reinterpret_cast<double4 *>(sc) + sb;  // sorted values (before the build)
    uint32_t *sid = reinterpret_cast<uint32_t *>(sc + 4 * 64);  // after the 64 double4 values

    const long long plane = (long long)a.nx * a.ny;
    const long long nvox = (long long)(a.z1 - a.z0) * plane;
    const long long v = ((long long)blockIdx.x * 4 + wid) * SPW + seg;  // chunk-local voxel
    const bool valid = v < nvox;
    const long long vc = valid ? v : nvox - 1;
    const int iz = a.z0 + (int)(vc / plane);
    const long long rem = vc % plane;
    const int iy = (int)(rem / a.nx), ix = (int)(rem % a.nx);
    const size_t vfull = (size_t)iz * plane + rem;
    const bool active = valid && (mask == nullptr || mask[vfull] != 0);
    const int k = a.k;
    const double eps = a.epsilon;

    // ---- 1. the k neighbours ranked by particle index (np.sort(yindices), _rbfinterp.py:521) ----
    const bool nb = active && li < k;
    double4 r = make_double4(0.0, 0.0, 0.0, 0.0), d = make_double4(0.0, 0.0, 0.0, 0.0);
    uint32_t id = 0xffffffffu;
    if (nb) {
        const uint32_t s = slots[(size_t)v * k + li];
        r = prec[s];
        d = pval[s];
        id = (uint32_t)r.w;
    }
    sid[lane] = id;
    rbf_wave_sync();
    int rank = 0;
    for (int j = 0; j < k; ++j) {
        const uint32_t o = sid[sb + j];
        rank += (o < id || (o == id && j < li)) ? 1 : 0;
    }
    rbf_wave_sync();
    if (li < k) {
        ye[rank] = make_double4(r.x * eps, r.y * eps, r.z * eps, (double)id);
        sv[rank] = d;
    }
    rbf_wave_sync();
    const bool krow = li < k;
    const double4 yi = krow ? ye[li] : make_double4(0.0, 0.0, 0.0, 0.0);
    double b0 = 0.0, b1 = 0.0, b2 = 0.0;
    if (krow) {
        const double4 dv = sv[li];
        b0 = dv.x;
        b1 = dv.y;
        b2 = dv.z;
    }
    rbf_wave_sync();  // the values' LDS is the build scratch next

    // ---- 2. symmetric build ----
#pragma unroll 1
    for (int dd = 1; dd <= H; ++dd) {
        const int j = (li + dd) & (L - 1);
        double e = 0.0;
        if (krow && j < k) {
            const double4 yj = ye[j];
            const double dx = yi.x - yj.x, dy = yi.y - yj.y, dz = yi.z - yj.z;
            e = rbf_phi_d2<KERN>((dx * dx + dy * dy) + dz * dz);
        }
        sc[(dd - 1) * 64 + lane] = e;
    }
    rbf_wave_sync();
    const double diag = rbf_phi<KERN>(0.0) + a.smoothing;
    double A[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const int dj = (j - li) & (L - 1);
        // own entry (dj <= H) or the partner row j's entry (i - j) mod L
        const int addr = dj <= H ? (dj - 1) * 64 + lane : (L - dj - 1) * 64 + sb + j;
        const double e = sc[max(addr, 0)];
        A[j] = li >= k ? (j == li ? 1.0 : 0.0) : (j >= k ? 0.0 : (j == li ? diag : e));
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // at most 8 reads in flight (registers)
    }

    rbf_wave_sync();  // every lane has read its row before the pivot rows overwrite the scratch
    // ---- 3. elimination without pivoting (row c is step c's pivot row) ----
    bool singular = false;
#pragma unroll
    for (int c = 0; c < M; ++c) {
        double *prow = sc + ((c & 1) * SPW + seg) * (M + 3);
        if (li == c) {
#pragma unroll
            for (int j = c; j < M; ++j) prow[j] = A[j];
            prow[M] = b0;
            prow[M + 1] = b1;
            prow[M + 2] = b2;
        }
        rbf_wave_sync();
        const double piv = prow[c];
        singular = singular || piv == 0.0;
        const double rp = spd_recip(piv);
        const double l = (li > c && li < M && piv != 0.0) ? A[c] * rp : 0.0;
#pragma unroll
        for (int j = c + 1; j < M; ++j) A[j] = fma(-l, prow[j], A[j]);
        b0 = fma(-l, prow[M], b0);
        b1 = fma(-l, prow[M + 1], b1);
        b2 = fma(-l, prow[M + 2], b2);
    }

    // ---- 4. back substitution: x_c = b_c / U_cc on lane c, broadcast through LDS (the
    //      pivot-row buffers, free now; double buffered, one barrier per step) ----
    double dg = 1.0;
#pragma unroll
    for (int j = 0; j < M; ++j)
        if (j == li) dg = A[j];
    const double rd = spd_recip(dg);  // = k_rbf_spd16's rcp_nr wherever that one is valid
    double x0 = 0.0, x1 = 0.0, x2 = 0.0;
#pragma unroll
    for (int c = M - 1; c >= 0; --c) {
        double *xb = sc + ((c & 1) * SPW + seg) * (M + 3);
        if (li == c) {
            x0 = b0 * rd;
            x1 = b1 * rd;
            x2 = b2 * rd;
            xb[0] = x0;
            xb[1] = x1;
            xb[2] = x2;
        }
        rbf_wave_sync();
        const double xc0 = xb[0], xc1 = xb[1], xc2 = xb[2];
        const double u = li < c ? A[c] : 0.0;
        b0 = fma(-u, xc0, b0);
        b1 = fma(-u, xc1, b1);
        b2 = fma(-u, xc2, b2);
    }

    // ---- 5. evaluate at the voxel: sum_j phi(eps |x - y_j|) c_j ----
    double qx, qy, qz;
    if (a.separable) {
        qx = ax[ix];
        qy = ay[iy];
        qz = az[iz];
    } else {
        qx = qpx[vfull];
        qy = qpy[vfull];
        qz = qpz[vfull];
    }
    double e = 0.0;
    if (krow) {
        const double dx = qx * eps - yi.x, dy = qy * eps - yi.y, dz = qz * eps - yi.z;
        e = rbf_phi_d2<KERN>((dx * dx + dy * dy) + dz * dz);
    }
    double o0 = seg_sum<L>(e * x0), o1 = seg_sum<L>(e * x1), o2 = seg_sum<L>(e * x2);
    if (!valid || li != 0) return;
    const size_t vo = (size_t)(iz - a.out_z0) * plane + rem;
    if (!active) {
        U[vo] = 0.0;
        V[vo] = 0.0;
        W[vo] = 0.0;
        return;
    }
    if (singular) {
        atomicAdd(&status[0], 1);
        atomicMin(&status[1], (int)min((long long)vfull, 0x7fffffffLL));
    }
    if (a.flags & PTV_FLAG_NAN_TO_NUM) {
        auto fix = [](double x) { return x != x ? 0.0 : (x == INFINITY ? DBL_MAX : (x == -INFINITY ? -DBL_MAX : x)); };
        o0 = fix(o0);
        o1 = fix(o1);
        o2 = fix(o2);
    }
    U[vo] = o0;
    V[vo] = o1;
    W[vo] = o2;
}

// ---------------------------------------------------------------------------
// SPD systems, register-only factorisation: four systems per wave, one per 16-lane row, lane
// li holding rows li and li + 16 (R = 2 for M <= 32).  Every broadcast of the elimination and
// the back substitution is the DPP row_newbcast of the pivot lane's register
// (v_mov_b64_dpp row_newbcast:n, within each 16-lane row): no LDS round trip, no barrier.
// The LDS-broadcast kernel above was LDS-issue bound (SQ_WAIT_INST_LDS 35 % of wave cycles,
// one 8-cycle ds_read_b128 per two pivot-row values).  Same arithmetic and order as k_rbf_spd
// (no pivoting, fma updates, the multiplier a * spd_recip(p)), so the two agree bit for bit.
// ---------------------------------------------------------------------------


template <int M, int KERN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_rbf_spd16(
    RbfKernelArgs a, const double4 *__restrict__ prec, const double4 *__restrict__ pval,
    const uint32_t *__restrict__ slots, const double *__restrict__ ax, const double *__restrict__ ay,
    const double *__restrict__ az, const double *__restrict__ qpx, const double *__restrict__ qpy,
    const double *__restrict__ qpz, const uint8_t *__restrict__ mask, double *__restrict__ U,
    double *__restrict__ V, double *__restrict__ W, int *__restrict__ status) {
    static_assert(M <= 32, "two rows per lane");
    constexpr int R = (M + 15) / 16;  // rows per lane
    __shared__ double4 s_ye[4][4][32];  // per wave and system: eps-scaled coordinates + id, id order
    // per wave: the sorted values and ids, then the symmetric build scratch (4 systems x 16R
    // rows x 8R entries): 80 KB per block at R = 2, two blocks (the register budget's 2 waves
    // per SIMD) per CU
    constexpr int SC = 4 * (16 * R) * (8 * R) > 4 * 32 * 4 + 4 * 32 / 2 ? 4 * (16 * R) * (8 * R) : 4 * 32 * 4 + 4 * 32 / 2;
    __shared__ double s_sc[4][SC];  // (80 KB per block with s_ye: two blocks per CU, not a byte more)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: the quad loop is scalar
    const long long plane = (long long)a.nx * a.ny;
    const long long nvox = (long long)(a.z1 - a.z0) * plane;
    const int k = a.k;
    const double eps = a.epsilon;
    // Persistent, XCD-aware quads (4 voxels, one per 16-lane system) with the next quad's slots,
    // mask byte and coordinates loaded after step 1 and its particle records after the read-back
    // (k_rbf_ns does the same; the arithmetic of a quad is unchanged: bit-identical to k_rbf_spd)
    const long long nquad = (nvox + 3) / 4;
    const int xcd = (int)(blockIdx.x & 7u);
    const long long qend = nquad * (xcd + 1) / 8;
    const long long qstep = (long long)(gridDim.x >> 3) * 4;
    long long qd = nquad * xcd / 8 + (long long)(blockIdx.x >> 3) * 4 + wid;
    uint32_t nsl[R];
    double4 nr[R], nd[R];
    bool nvv;
    uint32_t nmb;
    int nz;
    long long nrem;
    double nq[3];
    auto stage1 = [&](long long qn, int seg, int li) {
        const long long vn = qn * 4 + seg;
        nvv = qn < qend && vn < nvox;
        const long long vc = nvv ? vn : nvox - 1;
        nz = a.z0 + (int)(vc / plane);
        nrem = vc - (long long)(nz - a.z0) * plane;
        const int iy = (int)(nrem / a.nx), ix = (int)(nrem - (long long)iy * a.nx);
        const size_t vfull = (size_t)nz * plane + nrem;
        nmb = *(mask != nullptr ? mask + vfull : &kNsMaskOn);
        const bool sep = a.separable != 0;
        nq[0] = *(sep ? ax + ix : qpx + vfull);
        nq[1] = *(sep ? ay + iy : qpy + vfull);
        nq[2] = *(sep ? az + nz : qpz + vfull);
#pragma unroll
        for (int q = 0; q < R; ++q) nsl[q] = slots[(size_t)vc * k + (li + 16 * q < k ? li + 16 * q : k - 1)];
    };
    auto stage2 = [&](int li) {
        const bool act = nvv && nmb != 0u;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const uint32_t sl = act && li + 16 * q < k ? nsl[q] : 0u;
            nr[q] = prec[sl];
            nd[q] = pval[sl];
        }
    };
    // records in flight cost 16 VGPRs per row set: at 32 rows the elimination leaves no room, and
    // only the slots are prefetched (the records then load at the top of the quad)
    constexpr bool PFR = M <= 24;
    {
        const int seg = (threadIdx.x & 63) >> 4, li = threadIdx.x & 15;
        stage1(qd, seg, li);
        if constexpr (PFR) stage2(li);
    }
    bool pend = false;  // a quad's outputs are stored once the next quad's records are in use
    size_t pvo = 0;
    double po[3] = {0.0, 0.0, 0.0};
    auto flush = [&]() {
        if (pend) {
            U[pvo] = po[0];
            V[pvo] = po[1];
            W[pvo] = po[2];
        }
        pend = false;
    };
    for (; qd < qend; qd += qstep) {
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));  // nothing lane-dependent is hoisted out of the quad loop
    const int seg = lane >> 4, li = lane & 15;
    double4 *ye = s_ye[wid][seg];
    double *sc = s_sc[wid];
    double4 *sv = reinterpret_cast<double4 *>(sc) + seg * 32;
    uint32_t *sid = reinterpret_cast<uint32_t *>(sc + 4 * 32 * 4) + seg * 32;
    const long long v = qd * 4 + seg;  // chunk-local voxel
    const bool valid = v < nvox;
    const int iz = nz;
    const long long rem = nrem;
    const size_t vfull = (size_t)iz * plane + rem;
    const bool active = nvv && nmb != 0u;
    const double qx = nq[0], qy = nq[1], qz = nq[2];
    if constexpr (!PFR) stage2(li);

    // ---- 1. neighbours li and li + 16, ranked by particle index (np.sort(yindices)) ----
    double4 r[R], d[R];
    uint32_t id[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int nbr = li + 16 * q;
        const bool ld = active && nbr < k;
        r[q] = ld ? nr[q] : make_double4(0.0, 0.0, 0.0, 0.0);
        d[q] = ld ? nd[q] : make_double4(0.0, 0.0, 0.0, 0.0);
        id[q] = ld ? (uint32_t)nr[q].w : 0xffffffffu;
        if (nbr < 32) sid[nbr] = id[q];
    }
    flush();
    rbf_wave_sync();
    int rank[R];
#pragma unroll
    for (int q = 0; q < R; ++q) rank[q] = 0;
    for (int j = 0; j < k; ++j) {
        const uint32_t o = sid[j];
#pragma unroll
        for (int q = 0; q < R; ++q) rank[q] += (o < id[q] || (o == id[q] && j < li + 16 * q)) ? 1 : 0;
    }
    rbf_wave_sync();
#pragma unroll
    for (int q = 0; q < R; ++q) {
        if (li + 16 * q < k) {
            ye[rank[q]] = make_double4(r[q].x * eps, r[q].y * eps, r[q].z * eps, (double)id[q]);
            sv[rank[q]] = d[q];
        }
    }
    rbf_wave_sync();
    double4 yi[R];
    double B[R][3];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int row = li + 16 * q;
        const bool kr = row < k;
        yi[q] = kr ? ye[row] : make_double4(0.0, 0.0, 0.0, 0.0);
        const double4 dv = kr ? sv[row] : make_double4(0.0, 0.0, 0.0, 0.0);
        B[q][0] = dv.x;
        B[q][1] = dv.y;
        B[q][2] = dv.z;
    }
    rbf_wave_sync();  // the values' LDS is the build scratch next
    stage1(qd + qstep, seg, li);  // the next quad's slots, mask byte and coordinates

    // ---- 2. symmetric build of rows li and li + 16: row i evaluates phi for the columns
    //      (i + d) mod NR, d = 1..H, into a row-swizzled slot of its segment's scratch
    //      (conflict-free stores); entry (i, j) is then its own (d = (j - i) mod NR <= H) or its
    //      partner row j's (d' = NR - d).  H phi per row instead of k. ----
    constexpr int NR = 16 * R, H = NR / 2;
    double *ss = sc + seg * (NR * H);
    const double diag = rbf_phi<KERN>(0.0) + a.smoothing;
    // branch-free and unrolled (the entries' LDS reads and phi chains overlap): slots past k hold
    // stale coordinates, their phi is computed and dropped (same arithmetic as k_rbf_spd)
#pragma unroll 4
    for (int dd = 1; dd <= H; ++dd) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            const int j = (row + dd) & (NR - 1);
            const double4 yj = ye[j];
            const double dx = yi[q].x - yj.x, dy = yi[q].y - yj.y, dz = yi[q].z - yj.z;
            const double f = rbf_phi_d2<KERN>((dx * dx + dy * dy) + dz * dz);
            ss[row * H + ((dd - 1) ^ (row & (H - 1)))] = row < k && j < k ? f : 0.0;
        }
    }
    rbf_wave_sync();  // the partner rows' entries are read next
    double dg[R];  // the diagonal: phi(0) + smoothing, 1 on padded rows (identity block)
#pragma unroll
    for (int q = 0; q < R; ++q) dg[q] = li + 16 * q < k ? diag : 1.0;
    double A[R][M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            // branch-free addresses: own slot (dj in 1..H) or the partner row j's (dj in H+1..NR-1);
            // dj = 0 (the diagonal) reads a stale slot of the row and takes dg instead.
            // Padded rows and columns hold 0 (the build writes e = 0 there).
            const int dj = (j - row) & (NR - 1);
            const int own = row * H + (((dj - 1) & (H - 1)) ^ (row & (H - 1)));
            const int par = j * H + ((NR - 1 - dj) ^ (j & (H - 1)));
            const double e = ss[dj <= H ? own : par];
            A[q][j] = dj == 0 ? dg[q] : e;
        }
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // bounded reads in flight
    }
    if constexpr (PFR) stage2(li);  // the next quad's particle records

    // ---- 3. elimination without pivoting; pivot row c = lane c % 16, row set c / 16.
    //      Row set q is finished once c >= 16 q + 15 (all its rows are above the pivot): its
    //      updates are skipped at compile time.  The next column's pivot and reciprocal are
    //      formed inside this column's step, right after its update of column c + 1, so that
    //      their dependent chain overlaps the remaining updates (look-ahead by one column). ----
    //      The reciprocal is v_rcp_f64 + two Newton steps alone (rcp_nr): a pivot outside
    //      (2^-1020, 2^1020) sets `slow`, and the host reruns the launch with k_rbf_spd, whose
    //      spd_recip adds the IEEE division for exactly those pivots (rare: a NaN or infinite
    //      input, or a condition number near 1e300).  Each lane keeps the reciprocal of its own
    //      rows' pivots (rd) for the back substitution. ----
    bool singular = false, slow = false;
#define PTV_BC(X) rowbcast_n(c, X)
    double piv, rp, rd[R];
#pragma unroll
    for (int q = 0; q < R; ++q) rd[q] = 1.0;
    {
        constexpr int c = 0;
        piv = PTV_BC(A[0][0]);
        rp = rcp_nr(piv);
    }
#pragma unroll
    for (int c = 0; c < M; ++c) {
        const int pq = c / 16;
        // c is a constant in the unrolled loop, so the row_newbcast lane folds to one
        singular = singular | (piv == 0.0);
        rd[pq] = li == (c & 15) ? rp : rd[pq];
        // multipliers: a row set wholly below the pivot needs no test, a finished one none at all
        // (a zero pivot leaves garbage multipliers: the call then fails with PTV_E_SINGULAR)
        // negated multipliers: A += u (-l) is one v_fmac_f64_dpp with the pivot row's u broadcast
        // inside it (fma(-l, u, a) and fma(u, -l, a) round alike: bit-identical to k_rbf_spd)
        double l[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            if (16 * q + 15 <= c) l[q] = 0.0;
            else if (16 * q > c) l[q] = -(A[q][c] * rp);
            else l[q] = row > c ? -(A[q][c] * rp) : 0.0;
        }
        double pivn = 0.0, rpn = 1.0;
#pragma unroll
        for (int j = c + 1; j < M; ++j) {
            if (R == 2 && pq == 0) fmac_bc_piv_n(c, A[R - 1][j], A[0][j], l[R - 1], l[0]);
            else fmac_bc_self_n(c, A[pq][j], l[pq]);
            if (j == c + 1) {
                pivn = rowbcast_n(c + 1, A[(c + 1) / 16][c + 1]);
                rpn = rcp_nr(pivn);
            }
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (R == 2 && pq == 0) fmac_bc_piv_n(c, B[R - 1][t], B[0][t], l[R - 1], l[0]);
            else fmac_bc_self_n(c, B[pq][t], l[pq]);
        }
        piv = pivn;
        rp = rpn;
        __builtin_amdgcn_sched_barrier(0);  // keep the steps apart (register pressure)
    }

    // a pivot outside the Newton reciprocal's range shows in the reciprocals this lane kept
    // (huge pivot: |1/p| tiny or 0; tiny or subnormal: overflow; NaN: NaN)
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const double ar = fabs(rd[q]);
        slow = slow | !(ar >= 0x1p-1020 && ar <= 0x1p1020);
    }
    slow = slow & !singular;

    // ---- 4. back substitution: x_c = b_c * (1 / U_cc) from lane c % 16.  Row r's b no longer
    //      changes after step r (only rows above c are updated), so every lane scales its own
    //      rows once at the end instead of taking x_r by a select at step r. ----
#pragma unroll
    for (int c = M - 1; c >= 0; --c) {
        const int pq = c / 16;
        double u[R];  // this lane's U entries of column c (rows above c), the rest 0
#pragma unroll
        for (int q = 0; q < R; ++q) u[q] = li + 16 * q < c ? A[q][c] : 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            // B -= u x_c as B += (-x_c) u, the solution broadcast inside the fmac (same rounding)
            const double nx = -(B[pq][t] * rd[pq]);
            if (R == 2 && c > 16) {  // both row sets have rows above c (at c = 16 only set 0)
                double bb[2] = {B[0][t], B[R - 1][t]};
                const double uu[2] = {u[0], u[R - 1]};
                fmac_bc_n<2>(c, bb, nx, uu);
                B[0][t] = bb[0];
                B[R - 1][t] = bb[1];
            } else {
                double bb[1] = {B[0][t]};
                const double uu[1] = {u[0]};
                fmac_bc_n<1>(c, bb, nx, uu);
                B[0][t] = bb[0];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < R; ++q)
#pragma unroll
        for (int t = 0; t < 3; ++t) B[q][t] = B[q][t] * rd[q];
#undef PTV_BC

    // ---- 5. evaluate at the voxel: sum_j phi(eps |x - y_j|) c_j ----
    double o0 = 0.0, o1 = 0.0, o2 = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q) {  // branch-free (rows past k: yi = 0, dropped)
        const double dx = qx * eps - yi[q].x, dy = qy * eps - yi[q].y, dz = qz * eps - yi[q].z;
        const double f = rbf_phi_d2<KERN>((dx * dx + dy * dy) + dz * dz);
        const double e = li + 16 * q < k ? f : 0.0;
        o0 += e * B[q][0];
        o1 += e * B[q][1];
        o2 += e * B[q][2];
    }
    o0 = seg_sum<16>(o0);
    o1 = seg_sum<16>(o1);
    o2 = seg_sum<16>(o2);
    if (valid && li == 0) {
        if (active) {
            if (singular) {
                atomicAdd(&status[0], 1);
                atomicMin(&status[1], (int)min((long long)vfull, 0x7fffffffLL));
            }
            if (slow) atomicOr(&status[2], 1);  // the host reruns this launch with k_rbf_spd
            if (a.flags & PTV_FLAG_NAN_TO_NUM) {
                auto fix = [](double x) { return x != x ? 0.0 : (x == INFINITY ? DBL_MAX : (x == -INFINITY ? -DBL_MAX : x)); };
                o0 = fix(o0);
                o1 = fix(o1);
                o2 = fix(o2);
            }
        }
        pend = true;
        pvo = (size_t)(iz - a.out_z0) * plane + rem;
        po[0] = active ? o0 : 0.0;
        po[1] = active ? o1 : 0.0;
        po[2] = active ? o2 : 0.0;
    }
    rbf_wave_sync();  // the next quad reuses this wave's LDS
    }  // quads
    flush();
}

template <int M, int KERN>
static void launch_spd_t(const RbfKernelArgs &ka, long long nvox, hipStream_t s, const double4 *prec,
                         const double4 *pval, const uint32_t *slots, const double *ax, const double *ay,
                         const double *az, const double *qx, const double *qy, const double *qz, const uint8_t *mask,
                         double *U, double *V, double *W, int *status) {
    constexpr int L = M <= 16 ? 16 : 32;
    constexpr int SPW = 64 / L;
    const long long waves = (nvox + SPW - 1) / SPW;
    const long long blocks = (waves + 3) / 4;
    hipLaunchKernelGGL((k_rbf_spd<M, L, KERN>), dim3((unsigned)blocks), dim3(256), 0, s, ka, prec, pval, slots, ax, ay,
                       az, qx, qy, qz, mask, U, V, W, status);
}

template <int M>
static void launch_spd_m(const RbfKernelArgs &ka, long long nvox, hipStream_t s, const double4 *prec,
                         const double4 *pval, const uint32_t *slots, const double *ax, const double *ay,
                         const double *az, const double *qx, const double *qy, const double *qz, const uint8_t *mask,
                         double *U, double *V, double *W, int *status) {
    switch (ka.kernel) {
        case PTV_RBF_INVERSE_MULTIQUADRIC:
            launch_spd_t<M, PTV_RBF_INVERSE_MULTIQUADRIC>(ka, nvox, s, prec, pval, slots, ax, ay, az, qx, qy, qz, mask,
                                                          U, V, W, status);
            break;
        case PTV_RBF_INVERSE_QUADRATIC:
            launch_spd_t<M, PTV_RBF_INVERSE_QUADRATIC>(ka, nvox, s, prec, pval, slots, ax, ay, az, qx, qy, qz, mask, U,
                                                       V, W, status);
            break;
        default:
            launch_spd_t<M, PTV_RBF_GAUSSIAN>(ka, nvox, s, prec, pval, slots, ax, ay, az, qx, qy, qz, mask, U, V, W,
                                              status);
    }
}

// whether the system is symmetric positive definite (see k_rbf_spd) and of a size it serves
static bool rbf_spd(const RbfKernelArgs &ka, const double *smooth) {
    if (const char *e = dev_knob("PTV_RBF_SPD"))  // dev knob: 0 = always the pivoting kernel
        if (e[0] == '0') return false;  // (1 = the LDS-broadcast SPD kernel, see launch_rbf)
    const bool pd_kernel = ka.kernel == PTV_RBF_GAUSSIAN || ka.kernel == PTV_RBF_INVERSE_MULTIQUADRIC ||
                           ka.kernel == PTV_RBF_INVERSE_QUADRATIC;
    return pd_kernel && ka.m == ka.k && smooth == nullptr && ka.smoothing >= 0.0 && rbf_system_size(ka.m) <= 32;
}

// whether k_rbf_ns (ptv_rbf_ns.hpp) serves the launch: a scale-invariant conditionally positive
// definite kernel (the kernels interpolate_field can reach, interpolator.py:162-167: no epsilon
// there) with degree >= its order - 1 (then (Q^T Phi Q)[r:, r:] is positive definite), 1 or 4
// monomials, k <= 32 row slots.  The scale-dependent kernels stay on the pivoting kernel: for the
// flat gaussian eps = 0.3 systems (cond 6e8) the projected system lost 20x LAPACK's accuracy
// (tools/rbf_nullspace_proto.py).  So do 10 monomials (degree 2, the quintic's minimum): on the
// sphere pack's void voxels (neighbourhoods on a sphere-shell cap, a nearly degenerate quadratic
// fit) the null-space solve landed 1.2e-10 from the exact answer against LAPACK's 8.7e-13
// (tests/test_gpu_rbf.py::test_nullspace_sphere_pack_sampled, round 5); the dev knob
// PTV_RBF_NS=10 re-enables it.
static bool rbf_ns(const RbfKernelArgs &ka, const double *smooth, long long nvox) {
    if (const char *e = dev_knob("PTV_RBF_NS"))  // dev knob: 0 = the pivoting kernel throughout
        if (e[0] == '0') return false;
    if (ka.ns_list == nullptr || ka.ns_cap <= 0 || nvox > 0xffffffffLL || (ka.flags & PTV_FLAG_RBF_PIVOTING)) return false;
    const int np = ka.m - ka.k;
    bool ns10 = false;
    if (const char *e = dev_knob("PTV_RBF_NS"))
        ns10 = std::atoi(e) == 10;
    if (!(np == 1 || np == 4 || (ns10 && np == 10 && ka.k <= 24))) return false;
    if (ka.k <= np || ka.k > 32) return false;
    // scalar smoothing the kernel would flag on every voxel (negative, or > 2^26: k_rbf_ns step 1)
    if (smooth == nullptr && !(ka.smoothing >= 0.0 && ka.smoothing <= 0x1p26)) return false;
    const int degree = np == 1 ? 0 : (np == 4 ? 1 : 2);
    switch (ka.kernel) {
        case PTV_RBF_LINEAR: return degree >= 0;             // -r: order 1
        case PTV_RBF_THIN_PLATE_SPLINE: return degree >= 1;  // r^2 log r: order 2
        case PTV_RBF_CUBIC: return degree >= 1;              // r^3: order 2
        case PTV_RBF_QUINTIC: return degree >= 2;            // -r^5: order 3
        default: return false;
    }
}

int rbf_system_size(int m) {
    if (m < 1) return 0;
    return m <= 64 ? (m + 7) & ~7 : m;  // k_rbf_local pads to a multiple of 8; k_rbf_big / k_rbf_huge take m
}

template <int M>
static void launch_rbf_t(const RbfKernelArgs &ka, long long nvox, hipStream_t s, const double4 *prec,
                         const double4 *pval, const uint32_t *slots, const double *ax, const double *ay,
                         const double *az, const double *qx, const double *qy, const double *qz,
                         const double *smooth, const int *pw, const uint8_t *mask, double *U, double *V, double *W,
                         int *status) {
    constexpr int L = M <= 16 ? 16 : (M <= 32 ? 32 : 64);
    constexpr int SPW = 64 / L;
    const long long waves = (nvox + SPW - 1) / SPW;
    const long long blocks = (waves + 3) / 4;
    hipLaunchKernelGGL((k_rbf_local<M, L>), dim3((unsigned)blocks), dim3(256), 0, s, ka, prec, pval, slots, ax, ay, az,
                       qx, qy, qz, smooth, pw, mask, U, V, W, status);
}

int launch_rbf(const RbfKernelArgs &ka, const Binned &b, const uint32_t *slots, const double *ax, const double *ay,
               const double *az, const double *qx, const double *qy, const double *qz, const double *smooth,
               const int *pw, const uint8_t *mask, double *U, double *V, double *W, int *status, hipStream_t s) {
    const int M = rbf_system_size(ka.m);
    if (M == 0) {
        set_error("local RBF system size " + std::to_string(ka.m) + " exceeds the GPU limit (" +
                  std::to_string(kRbfMaxSystem) + ")");
        return PTV_E_UNSUPPORTED;
    }
    const long long nvox = (long long)(ka.z1 - ka.z0) * ka.nx * ka.ny;
    if (nvox <= 0) return PTV_OK;
    if ((nvox + 3) / 4 > 0x7fffffffLL) {
        set_error("grid chunk too large for one launch");
        return PTV_E_ARG;
    }
    if (M > kRbfMaxSystem) {
        // persistent 64-lane workgroups, each with its global-memory slice (ka.huge_scratch, sized by
        // the host: ka.huge_blocks slices of rbf_huge_slice_doubles(m, k))
        if (ka.huge_scratch == nullptr || ka.huge_blocks <= 0) {
            set_error("local RBF: the m > 128 kernel needs its scratch");
            return PTV_E_ARG;
        }
        const long long blocks = std::min<long long>(ka.huge_blocks, nvox);
        hipLaunchKernelGGL(k_rbf_huge, dim3((unsigned)blocks), dim3(64), 0, s, ka, b.prec, b.pval, slots, ax, ay, az,
                           qx, qy, qz, smooth, pw, mask, U, V, W, status, ka.huge_scratch,
                           rbf_huge_slice_doubles(ka.m, ka.k), nvox);
        PTV_HIP(hipGetLastError());
        return PTV_OK;
    }
    if (M > 64) {
        // one 64-lane block per voxel: sub-launches of whole planes, at most 2^26 voxels (2^32 work
        // items) each, with the slots of each sub-launch's first plane
        const long long plane = (long long)ka.nx * ka.ny;
        if (plane > (1LL << 26)) {
            set_error("local RBF: grid plane too large for the m > 64 kernel");
            return PTV_E_UNSUPPORTED;
        }
        const size_t bytes = rbf_big_lds_bytes(ka.m);
        PTV_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rbf_big),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        const int step = (int)std::max<long long>(1, (1LL << 26) / plane);
        for (int za = ka.z0; za < ka.z1; za += step) {
            RbfKernelArgs sa = ka;
            sa.z0 = za;
            sa.z1 = std::min(ka.z1, za + step);
            const uint32_t *sl = slots + (size_t)(za - ka.z0) * plane * ka.k;
            hipLaunchKernelGGL(k_rbf_big, dim3((unsigned)((long long)(sa.z1 - sa.z0) * plane)), dim3(64), bytes, s, sa,
                               b.prec, b.pval, sl, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status);
            PTV_HIP(hipGetLastError());
        }
        return PTV_OK;
    }
    if (rbf_spd(ka, smooth)) {
        const char *e = dev_knob("PTV_RBF_SPD");  // dev knob: 1 = the LDS-broadcast SPD kernel
        if (!(e && e[0] == '1') && !ka.spd_lds && !(ka.flags & PTV_FLAG_RBF_SPD_LDS)) {
#define PTV_S16(MM, KK)                                                                                 \
    do {                                                                                                \
        static int occ = 0;                                                                             \
        hipLaunchKernelGGL((k_rbf_spd16<MM, KK>), dim3(persistent_grid(k_rbf_spd16<MM, KK>, (nvox + 3) / 4, occ)), \
                           dim3(256), 0, s, ka, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, mask, U, V, W, status); \
    } while (0)
#define PTV_S16K(MM) \
    switch (ka.kernel) { \
        case PTV_RBF_INVERSE_MULTIQUADRIC: PTV_S16(MM, PTV_RBF_INVERSE_MULTIQUADRIC); break; \
        case PTV_RBF_INVERSE_QUADRATIC: PTV_S16(MM, PTV_RBF_INVERSE_QUADRATIC); break; \
        default: PTV_S16(MM, PTV_RBF_GAUSSIAN); \
    }
            switch (M) {
                case 8: PTV_S16K(8) break;
                case 16: PTV_S16K(16) break;
                case 24: PTV_S16K(24) break;
                default: PTV_S16K(32)
            }
#undef PTV_S16K
#undef PTV_S16
            PTV_HIP(hipGetLastError());
            return PTV_OK;
        }
        switch (M) {
            case 8: launch_spd_m<8>(ka, nvox, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, mask, U, V, W, status); break;
            case 16: launch_spd_m<16>(ka, nvox, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, mask, U, V, W, status); break;
            case 24: launch_spd_m<24>(ka, nvox, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, mask, U, V, W, status); break;
            default: launch_spd_m<32>(ka, nvox, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, mask, U, V, W, status);
        }
        PTV_HIP(hipGetLastError());
        return PTV_OK;
    }
    RbfKernelArgs pa = ka;
    long long pn = nvox;
    if (rbf_ns(ka, smooth, nvox)) {
        PTV_HIP(hipMemsetAsync(status + 3, 0, sizeof(int), s));
        RbfKernelArgs na = ka;
        na.stamps = g_dbg;  // diagnostics: only PTV_NS_STAMP builds write them
        na.stamp_cap = g_dbg_cap;
        const int np = ka.m - ka.k;
        if (ka.k <= 16)
            launch_rbf_ns16(na, nvox, np, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status);
        else if (ka.k <= 20)
            launch_rbf_ns20(na, nvox, np, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status);
        else if (ka.k <= 24)
            launch_rbf_ns24(na, nvox, np, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status);
        else
            launch_rbf_ns32(na, nvox, np, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status);
        PTV_HIP(hipGetLastError());
        // the voxels it flagged: the pivoting kernel over the list (grid sized for ns_cap; waves past the
        // device count exit at once)
        pa.vlist = ka.ns_list;
        pa.vcount = status + 3;
        pn = ka.ns_cap;
    } else {
        pa.vlist = nullptr;
    }
    switch (M) {
#define PTV_RCASE(X) \
    case X: launch_rbf_t<X>(pa, pn, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status); break;
        PTV_RCASE(8)
        PTV_RCASE(16)
        PTV_RCASE(24)
        PTV_RCASE(32)
        PTV_RCASE(40)
        PTV_RCASE(48)
        PTV_RCASE(56)
        PTV_RCASE(64)
#undef PTV_RCASE
        default:
            return PTV_E_UNSUPPORTED;
    }
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
