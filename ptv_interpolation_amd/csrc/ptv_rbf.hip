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
// reference to the conditioning of the system (see tests/test_rbf.py and DESIGN.md).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

__device__ __forceinline__ void rbf_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// scipy/interpolate/_rbfinterp_pythran.py kernel functions (r >= 0)
template <int KERN>
__device__ __forceinline__ double rbf_phi(double r) {
    if constexpr (KERN == PTV_RBF_LINEAR) return -r;
    if constexpr (KERN == PTV_RBF_THIN_PLATE_SPLINE) return r == 0.0 ? 0.0 : (r * r) * log(r);
    if constexpr (KERN == PTV_RBF_CUBIC) return (r * r) * r;
    if constexpr (KERN == PTV_RBF_QUINTIC) return -((((r * r) * r) * r) * r);
    if constexpr (KERN == PTV_RBF_MULTIQUADRIC) return -sqrt(r * r + 1.0);
    if constexpr (KERN == PTV_RBF_INVERSE_MULTIQUADRIC) return 1.0 / sqrt(r * r + 1.0);
    if constexpr (KERN == PTV_RBF_INVERSE_QUADRATIC) return 1.0 / (r * r + 1.0);
    if constexpr (KERN == PTV_RBF_GAUSSIAN) return exp(-(r * r));
    return 0.0;
}

__device__ double rbf_phi_rt(int kern, double r) {
    switch (kern) {
        case PTV_RBF_LINEAR: return rbf_phi<PTV_RBF_LINEAR>(r);
        case PTV_RBF_THIN_PLATE_SPLINE: return rbf_phi<PTV_RBF_THIN_PLATE_SPLINE>(r);
        case PTV_RBF_CUBIC: return rbf_phi<PTV_RBF_CUBIC>(r);
        case PTV_RBF_QUINTIC: return rbf_phi<PTV_RBF_QUINTIC>(r);
        case PTV_RBF_MULTIQUADRIC: return rbf_phi<PTV_RBF_MULTIQUADRIC>(r);
        case PTV_RBF_INVERSE_MULTIQUADRIC: return rbf_phi<PTV_RBF_INVERSE_MULTIQUADRIC>(r);
        case PTV_RBF_INVERSE_QUADRATIC: return rbf_phi<PTV_RBF_INVERSE_QUADRATIC>(r);
        default: return rbf_phi<PTV_RBF_GAUSSIAN>(r);
    }
}

// x ** p for the small integer monomial exponents (np.prod(x ** powers[j]))
__device__ __forceinline__ double ipow(double x, int p) {
    if (p == 0) return 1.0;
    if (p == 1) return x;
    if (p == 2) return x * x;
    if (p == 3) return (x * x) * x;
    return pow(x, (double)p);
}

// monomial with exponents packed as px | py << 8 | pz << 16
__device__ __forceinline__ double mono(double hx, double hy, double hz, int code) {
    return (ipow(hx, code & 255) * ipow(hy, (code >> 8) & 255)) * ipow(hz, code >> 16);
}

template <int L>
__device__ __forceinline__ double seg_sum(double v) {
#pragma unroll
    for (int o = 1; o < L; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int L>
__device__ __forceinline__ double seg_min(double v) {
#pragma unroll
    for (int o = 1; o < L; o <<= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
template <int L>
__device__ __forceinline__ double seg_max(double v) {
#pragma unroll
    for (int o = 1; o < L; o <<= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <int L>
__device__ __forceinline__ int seg_min_i(int v) {
#pragma unroll
    for (int o = 1; o < L; o <<= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

// kernel block of row i: A[j] = phi(eps*|y_i - y_j|) (+ s_i on the diagonal) for j < k
template <int M, int KERN>
__device__ __forceinline__ void build_kernel_block(double (&A)[M], const double4 *__restrict__ ye, double4 yi,
                                                   int k, int li, bool krow, double si) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
        if (j < k) {
            const double4 yj = ye[j];
            const double dx = yi.x - yj.x, dy = yi.y - yj.y, dz = yi.z - yj.z;
            const double r = sqrt((dx * dx + dy * dy) + dz * dz);
            double p = rbf_phi<KERN>(r);
            if (j == li) p = p + si;
            if (krow) A[j] = p;
        }
    }
}

template <int M, int L>
__global__ __launch_bounds__(256) void k_rbf_local(RbfKernelArgs a, const double4 *__restrict__ prec,
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
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int seg = lane / L, li = lane % L, sb = seg * L;
    double4 *ye = s_ye[wid] + sb;
    double4 *yh = s_yh[wid] + sb;
    double4 *sv = s_val[wid] + sb;
    double *prow_buf = s_row[wid][seg];

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

    // ---- 2. row li of the system ----
    const bool krow = li < k;
    const bool prow = li >= k && li < m;
    double A[M];
#pragma unroll
    for (int j = 0; j < M; ++j) A[j] = 0.0;
    const double4 yi = krow ? ye[li] : make_double4(0.0, 0.0, 0.0, 0.0);
    double si = 0.0;
    if (krow && active) si = smooth != nullptr ? smooth[(size_t)yi.w] : a.smoothing;
    switch (a.kernel) {
        case PTV_RBF_LINEAR: build_kernel_block<M, PTV_RBF_LINEAR>(A, ye, yi, k, li, krow, si); break;
        case PTV_RBF_THIN_PLATE_SPLINE: build_kernel_block<M, PTV_RBF_THIN_PLATE_SPLINE>(A, ye, yi, k, li, krow, si); break;
        case PTV_RBF_CUBIC: build_kernel_block<M, PTV_RBF_CUBIC>(A, ye, yi, k, li, krow, si); break;
        case PTV_RBF_QUINTIC: build_kernel_block<M, PTV_RBF_QUINTIC>(A, ye, yi, k, li, krow, si); break;
        case PTV_RBF_MULTIQUADRIC: build_kernel_block<M, PTV_RBF_MULTIQUADRIC>(A, ye, yi, k, li, krow, si); break;
        case PTV_RBF_INVERSE_MULTIQUADRIC:
            build_kernel_block<M, PTV_RBF_INVERSE_MULTIQUADRIC>(A, ye, yi, k, li, krow, si);
            break;
        case PTV_RBF_INVERSE_QUADRATIC: build_kernel_block<M, PTV_RBF_INVERSE_QUADRATIC>(A, ye, yi, k, li, krow, si); break;
        default: build_kernel_block<M, PTV_RBF_GAUSSIAN>(A, ye, yi, k, li, krow, si); break;
    }
    if (m > k) {
        // polynomial blocks: P(yhat_i) in the columns k..m-1 of the kernel rows, P(yhat_j)^T in
        // the rows k..m-1, zeros in the bottom-right corner
        const double4 hi = krow ? yh[li] : make_double4(0.0, 0.0, 0.0, 0.0);
        const int tcode = prow ? pw[li - k] : 0;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            if (j < k) {
                const double4 hj = yh[j];
                const double p = mono(hj.x, hj.y, hj.z, tcode);
                if (prow) A[j] = p;
            } else if (j < m) {
                const double p = mono(hi.x, hi.y, hi.z, pw[j - k]);
                if (krow) A[j] = p;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < M; ++j)
        if (j >= m && li == j) A[j] = 1.0;  // identity padding up to M
    double b0 = 0.0, b1 = 0.0, b2 = 0.0;
    if (krow) {
        const double4 dv = sv[li];
        b0 = dv.x;
        b1 = dv.y;
        b2 = dv.z;
    }

    // ---- 3. Gaussian elimination with partial pivoting; rows stay in their lanes ----
    bool done = li >= M;  // lanes beyond the padded system never pivot
    int pos = li;         // LAPACK row position (idamax tie order)
    int mystep = -1;      // the elimination step that used this row as pivot
    bool singular = false;
#pragma unroll
    for (int c = 0; c < M; ++c) {
        const double key = done ? -1.0 : fabs(A[c]);
        const double mx = seg_max<L>(key);
        const bool cand = !done && key == mx;
        unsigned long long bal = __builtin_amdgcn_ballot_w64(cand);
        unsigned long long sbal = L == 64 ? bal : ((bal >> sb) & ((1ull << (L & 63)) - 1ull));
        if (__builtin_amdgcn_ballot_w64(__builtin_popcountll(sbal) > 1) != 0) {
            // ties: the lowest current row position wins (first index of idamax)
            const int pk = seg_min_i<L>(cand ? pos : 0x7fffffff);
            bal = __builtin_amdgcn_ballot_w64(cand && pos == pk);
            sbal = L == 64 ? bal : ((bal >> sb) & ((1ull << (L & 63)) - 1ull));
        }
        const int P = (int)__builtin_ctzll(sbal | (1ull << 63));
        const bool isP = li == P;
        singular = singular || !(mx > 0.0);
        if (isP) {
#pragma unroll
            for (int j = c; j < M; ++j) prow_buf[j] = A[j];
            prow_buf[M] = b0;
            prow_buf[M + 1] = b1;
            prow_buf[M + 2] = b2;
            prow_buf[M + 3] = (double)pos;
        }
        rbf_wave_sync();
        const double piv = prow_buf[c];
        if (isP) {
            done = true;
            mystep = c;
        } else if (!done) {
            if (pos == c) pos = (int)prow_buf[M + 3];  // the swap moves this row to the pivot's position
            if (piv != 0.0) {
                const double l = A[c] * (1.0 / piv);
#pragma unroll
                for (int j = c + 1; j < M; ++j) A[j] = fma(-l, prow_buf[j], A[j]);
                b0 = fma(-l, prow_buf[M], b0);
                b1 = fma(-l, prow_buf[M + 1], b1);
                b2 = fma(-l, prow_buf[M + 2], b2);
            }
        }
        rbf_wave_sync();
    }

    // ---- 4. back substitution (column oriented, dtrsm order); solution in LDS ----
#pragma unroll
    for (int c = M - 1; c >= 0; --c) {
        if (mystep == c) sv[c] = make_double4(b0 / A[c], b1 / A[c], b2 / A[c], 0.0);
        rbf_wave_sync();
        if (mystep >= 0 && mystep < c) {
            const double4 xc = sv[c];
            b0 = fma(-A[c], xc.x, b0);
            b1 = fma(-A[c], xc.y, b1);
            b2 = fma(-A[c], xc.z, b2);
        }
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

int rbf_system_size(int m) {
    if (m < 1 || m > kRbfMaxSystem) return 0;
    return (m + 7) & ~7;
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
    switch (M) {
#define PTV_RCASE(X) \
    case X: launch_rbf_t<X>(ka, nvox, s, b.prec, b.pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status); break;
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
