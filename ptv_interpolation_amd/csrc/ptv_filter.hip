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
// particles themselves as a point-list "grid").  Query order: the particles sorted by a
// 30-bit Morton code (hipCUB radix sort, stable: ties keep index order), so that 64
// consecutive queries are a compact blob and 8 consecutive ones a compact sub-blob.  Each
// wave tile of 64 is then laid out like a 4x4x4 voxel tile: the 8 queries of Morton
// sub-group s go to the lanes whose bits (1, 3, 5) spell s, which is how the k-NN kernel
// groups lanes into its 8 sub-balls (ptv_knn.hip), so the sub-ball candidate filter
// works on particle queries too.  The per-particle statistics (speeds of the k neighbours,
// median, MAD, keep test) run in the search kernel's epilogue (kModeFilter, ptv_knn.hip), so
// no neighbour list goes through HBM.  This file holds the kernels before the search: the
// Morton sort, the query layout and the slot-order speeds.
#include <hipcub/hipcub.hpp>

#include "ptv_api.h"
#include "ptv_kernels.hpp"
#include "ptv_median.hpp"

namespace ptv {

// queries in record order, padded to `npad` with the last record
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

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(256) void k_morton(const double *__restrict__ x, const double *__restrict__ y,
                                                const double *__restrict__ z, int64_t n, double ox, double oy,
                                                double oz, double sx, double sy, double sz,
                                                uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    auto q = [](double v, double o, double sc) {
        const double f = (v - o) * sc;
        return (uint32_t)(f < 0.0 ? 0.0 : (f > 1023.0 ? 1023.0 : f));
    };
    keys[i] = spread10(q(x[i], ox, sx)) | (spread10(q(y[i], oy, sy)) << 1) | (spread10(q(z[i], oz, sz)) << 2);
    ids[i] = (uint32_t)i;
}

// query q of a 64-tile (Morton rank within the tile) <-> lane: sub-group s = q >> 3 sits on
// lane bits (1, 3, 5), member j = q & 7 on bits (0, 2, 4)
__device__ __forceinline__ int lane_of_query(int q) {
    const int s = q >> 3, j = q & 7;
    return (j & 1) | ((s & 1) << 1) | (((j >> 1) & 1) << 2) | (((s >> 1) & 1) << 3) | (((j >> 2) & 1) << 4) |
           (((s >> 2) & 1) << 5);
}
__device__ __forceinline__ int query_of_lane(int l) {
    const int s = ((l >> 1) & 1) | (((l >> 3) & 1) << 1) | (((l >> 5) & 1) << 2);
    const int j = (l & 1) | (((l >> 2) & 1) << 1) | (((l >> 4) & 1) << 2);
    return (s << 3) | j;
}

// Point-list "grid" of the search: nx = 16, ny = 4, nz = npad / 64, so a 256-thread block
// holds 4 wave tiles along x (all four waves busy; with nx = 4 three of them idled).  Tile
// g = 4 tz + tx covers lanes l at ((4 tz + l / 16) * 4 + (l / 4) % 4) * 16 + 4 tx + l % 4.
__device__ __forceinline__ int64_t pos_of(int64_t g, int l) {
    const int64_t tz = g >> 2, tx = g & 3;
    return ((tz * 4 + (l >> 4)) * 4 + ((l >> 2) & 3)) * 16 + tx * 4 + (l & 3);
}

// position of tile g / lane l holds Morton query 64 g + query_of_lane(l) (the last particle
// pads the final tiles); q_orig[position] = the query's original index (~0 for the pads)
__global__ __launch_bounds__(256) void k_query_layout(const uint32_t *__restrict__ perm, const double *__restrict__ x,
                                                      const double *__restrict__ y, const double *__restrict__ z,
                                                      int64_t n, int64_t npad, double *__restrict__ qx,
                                                      double *__restrict__ qy, double *__restrict__ qz,
                                                      uint32_t *__restrict__ q_orig) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (tile, lane) = (t / 64, t % 64)
    if (t >= npad) return;
    const int64_t q = (t & ~(int64_t)63) + query_of_lane((int)(t & 63));
    const uint32_t src = perm[q < n ? q : n - 1];
    const int64_t p = pos_of(t >> 6, (int)(t & 63));
    qx[p] = x[src];
    qy[p] = y[src];
    qz[p] = z[src];
    if (q_orig) q_orig[p] = q < n ? src : 0xffffffffu;
}

// speed of every binned particle, slot order (filtering.py:16-17)
__global__ __launch_bounds__(256) void k_slot_speed(const double4 *__restrict__ pval, int64_t n,
                                                    double *__restrict__ spd) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) spd[i] = speed_of(pval[i]);
}

int launch_slot_speed(const double4 *pval, int64_t n, double *spd, hipStream_t s) {
    hipLaunchKernelGGL(k_slot_speed, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pval, n, spd);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// the (k+1)-NN list length serving the filter's k (0: unsupported)
int filter_kmax(int k) { return k >= 1 ? kmax_for(k + 1) : 0; }

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

size_t morton_sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                       (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, 0, 30, nullptr);
    return bytes;
}

int launch_morton_order(const double *x, const double *y, const double *z, int64_t n, const double lo[3],
                        const double hi[3], uint32_t *keys, uint32_t *keys_out, uint32_t *ids, uint32_t *perm,
                        void *temp, size_t temp_bytes, hipStream_t s) {
    double sc[3];
    for (int d = 0; d < 3; ++d) {
        const double e = hi[d] - lo[d];
        sc[d] = e > 0.0 ? 1024.0 / e : 0.0;
    }
    hipLaunchKernelGGL(k_morton, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, y, z, n, lo[0], lo[1], lo[2],
                       sc[0], sc[1], sc[2], keys, ids);
    size_t bytes = temp_bytes;
    PTV_HIP(hipcub::DeviceRadixSort::SortPairs(temp, bytes, (const uint32_t *)keys, keys_out, (const uint32_t *)ids,
                                               perm, (int)n, 0, 30, s));
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_query_layout(const uint32_t *perm, const double *x, const double *y, const double *z, int64_t n,
                        int64_t npad, double *qx, double *qy, double *qz, uint32_t *q_orig, hipStream_t s) {
    hipLaunchKernelGGL(k_query_layout, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, perm, x, y, z, n, npad,
                       qx, qy, qz, q_orig);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
