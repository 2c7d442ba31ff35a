// ptv_filter.hip — the k-NN median/MAD outlier filter on the GPU.
//
// Reference: filtering.py:5-58 remove_outliers_knn(df, k=25, threshold=3.0):
//   speed = sqrt(u**2 + v**2 + w**2)                                   (:16-17)
//   dist, idx = KDTree(points).query(points, k=k+1); drop column 0    (:20-30)
//   radius = median(dist[:, -1])                                       (:33-35, printed)
//   med = median(speed[idx], axis=1); mad = median(|speed[idx] - med|) (:38-44)
//   keep = |speed - med| / (mad + 1e-6) <= threshold                   (:47-51)
//
// The (k+1)-NN query runs on the same k-NN kernel as the grid path (slot mode, the
// particles themselves as a point-list "grid").  The query order is a second counting
// sort of the particles into coarse bricks of ~64 particles, so that a wave's 64 queries
// form a compact blob (the search-cell order would make them a thin strip along x, whose
// gather box is ~10x larger).  This file holds the two thin kernels either side of the
// search: building the query list, and the per-particle statistics.
#include "ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

// queries in brick order, padded to `npad` with the last record
__global__ __launch_bounds__(256) void k_binned_queries(const double4 *__restrict__ prec, int64_t n, int64_t npad,
                                                        double *__restrict__ qx, double *__restrict__ qy,
                                                        double *__restrict__ qz) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= npad) return;
    const double4 r = prec[i < n ? i : n - 1];
    qx[i] = r.x;
    qy[i] = r.y;
    qz[i] = r.z;
}

// the original-order particle coordinates, padded (bounding-box input of the binning pass)
__global__ __launch_bounds__(256) void k_pad_queries(const double *__restrict__ x, const double *__restrict__ y,
                                                     const double *__restrict__ z, int64_t n, int64_t npad,
                                                     double *__restrict__ qx, double *__restrict__ qy,
                                                     double *__restrict__ qz) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= npad) return;
    const int64_t j = i < n ? i : n - 1;
    qx[i] = x[j];
    qy[i] = y[j];
    qz[i] = z[j];
}

// value at sorted position `pos` of s[0..n): the element whose [#less, #less-or-equal) holds pos
template <int KMAX>
__device__ __forceinline__ double select_pos(const double (&s)[KMAX], int n, int pos) {
    double out = 0.0;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if (j < n) {
            int lt = 0, le = 0;
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                if (i < n) {
                    lt += s[i] < s[j] ? 1 : 0;
                    le += s[i] <= s[j] ? 1 : 0;
                }
            }
            if (lt <= pos && pos < le) out = s[j];
        }
    }
    return out;
}

// np.median of n values (n odd: the middle one; n even: mean of the two middle ones, i.e.
// (a + b) / 2); any NaN gives NaN (numpy's _median_nancheck)
template <int KMAX>
__device__ __forceinline__ double median_of(const double (&s)[KMAX], int n) {
    bool nan = false;
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
        if (j < n) nan = nan || (s[j] != s[j]);
    if (nan) return __longlong_as_double(0x7ff8000000000000LL);
    if (n & 1) return select_pos(s, n, n >> 1);
    const double a = select_pos(s, n, (n >> 1) - 1), b = select_pos(s, n, n >> 1);
    return (a + b) / 2.0;
}

__device__ __forceinline__ double speed_of(const double4 v) {
    return sqrt((v.x * v.x + v.y * v.y) + v.z * v.z);  // u**2 + v**2 + w**2, left to right
}

// one particle (binned order) per lane: its k+1 neighbour slots -> keep flag and the
// distance to the (k+1)-th neighbour, written at the particle's original index
template <int KMAX>
__global__ __launch_bounds__(256) void k_outlier_stats(FilterArgs a, const double4 *__restrict__ prec,
                                                       const double4 *__restrict__ pval,
                                                       const double4 *__restrict__ qrec,
                                                       const double4 *__restrict__ qval,
                                                       const uint32_t *__restrict__ slots, uint8_t *__restrict__ keep,
                                                       double *__restrict__ kth) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const int k1 = a.k + 1;
    const double4 q = qrec[i];  // query i (brick order); .w = original index
    const uint32_t *sl = slots + (size_t)i * k1;
    // the point itself is column 0 of the reference query (distance 0); when several
    // particles coincide with it, the query point's own record is the one dropped
    int drop = -1;
    double dmin = INFINITY, dmax = 0.0;
    int self = -1;
#pragma unroll
    for (int j = 0; j < KMAX + 1; ++j) {
        if (j < k1) {
            const uint32_t s = sl[j];
            const double4 r = prec[s];
            const double dx = r.x - q.x, dy = r.y - q.y, dz = r.z - q.z;
            const double d = sqrt((dx * dx + dy * dy) + dz * dz);  // cKDTree p=2 accumulation
            if (d < dmin) {
                dmin = d;
                drop = j;
            }
            dmax = fmax(dmax, d);
            if (r.w == q.w) self = j;  // the same particle (original index)
        }
    }
    if (self >= 0) drop = self;  // at distance 0 == dmin whenever it is in the list
    double sp[KMAX];
#pragma unroll
    for (int t = 0; t < KMAX; ++t) sp[t] = 0.0;
    int m = 0;
#pragma unroll
    for (int j = 0; j < KMAX + 1; ++j) {
        if (j < k1 && j != drop) {
            const double v = speed_of(pval[sl[j]]);
#pragma unroll
            for (int t = 0; t < KMAX; ++t)
                if (t == m) sp[t] = v;
            ++m;
        }
    }
    const double med = median_of(sp, a.k);
    double dev[KMAX];
#pragma unroll
    for (int t = 0; t < KMAX; ++t) dev[t] = fabs(sp[t] - med);
    const double mad = median_of(dev, a.k);
    const double z = fabs(speed_of(qval[i]) - med) / (mad + a.mad_eps);
    const int64_t orig = (int64_t)q.w;
    keep[orig] = z <= a.threshold ? 1 : 0;
    if (kth) kth[orig] = dmax;
}

int filter_kmax(int k) {
    if (k <= 8) return 8;
    if (k <= 16) return 16;
    if (k <= 32) return 32;
    if (k <= 63) return 64;
    return 0;
}

int launch_binned_queries(const double4 *prec, int64_t n, int64_t npad, double *qx, double *qy, double *qz,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_binned_queries, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, prec, n, npad, qx, qy,
                       qz);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_pad_queries(const double *x, const double *y, const double *z, int64_t n, int64_t npad, double *qx,
                       double *qy, double *qz, hipStream_t s) {
    hipLaunchKernelGGL(k_pad_queries, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, x, y, z, n, npad, qx, qy,
                       qz);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_outlier_stats(const FilterArgs &a, const Binned &b, const double4 *qrec, const double4 *qval,
                         const uint32_t *slots, uint8_t *keep, double *kth, hipStream_t s) {
    const dim3 grid((unsigned)((a.n + 255) / 256));
    switch (filter_kmax(a.k)) {
        case 8: hipLaunchKernelGGL(k_outlier_stats<8>, grid, dim3(256), 0, s, a, b.prec, b.pval, qrec, qval, slots, keep, kth); break;
        case 16: hipLaunchKernelGGL(k_outlier_stats<16>, grid, dim3(256), 0, s, a, b.prec, b.pval, qrec, qval, slots, keep, kth); break;
        case 32: hipLaunchKernelGGL(k_outlier_stats<32>, grid, dim3(256), 0, s, a, b.prec, b.pval, qrec, qval, slots, keep, kth); break;
        case 64: hipLaunchKernelGGL(k_outlier_stats<64>, grid, dim3(256), 0, s, a, b.prec, b.pval, qrec, qval, slots, keep, kth); break;
        default:
            set_error("outlier filter: k must be <= 63 (k + 1 neighbours on the GPU k-NN list)");
            return PTV_E_UNSUPPORTED;
    }
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
