// ptv_bin.hip — spatial-hash particle binning for the k-NN interpolator (gfx950).
//
// Replaces the role of the per-call cKDTree build in the reference
// (interpolator.py:90 and :132, scipy KDTree(points), leafsize 10): particles
// are sorted into a uniform cell grid in linear (z, y, x) order, so that every
// x-run of cells in a row is one contiguous particle range.
//
//   bbox        per-axis min/max of particles and queries (grid-stride, LDS reduce)
//   from 2.5M particles (launch_bin_sort):
//     cell_key      linear cell id per particle, no atomics
//     radix sort    stable hipCUB sort of (cell, index) pairs: in-cell order = index order
//     sorted_starts inverse permutation + cell starts at the code changes (fix-up for
//                   runs of > 65536 empty cells)
//   below (the atomic counting sort):
//     cell_code   linear cell id per particle + atomic histogram
//     scan        exclusive prefix sum of the cell histogram (3-phase, 4096 cells/block)
//     scatter     particle -> slot (atomic fill from the back of each cell)
//     seg_sort    ascending original index inside each cell (deterministic order)
//   place       AoS records for the scalar-load k-NN kernel, in original order through
//               the inverse permutation: prec[slot] = (x, y, z, id), pval[slot] = (u, v, w, 0)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

// ---------------------------------------------------------------------------
// bounding box
// ---------------------------------------------------------------------------
struct BBoxArgs {
    const double *p[3];
    const double *q[3];
    int64_t n;
    int64_t qn[3];
    const uint32_t *dn;  // particle count on the device (the slab cull's), or NULL: n
};

__global__ __launch_bounds__(256) void k_bbox(BBoxArgs a, double *partials) {
    double lo[3], hi[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        lo[d] = INFINITY;
        hi[d] = -INFINITY;
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t np = a.dn != nullptr ? (int64_t)*a.dn : a.n;
    for (int64_t i = t0; i < np; i += stride) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            double v = a.p[d][i];
            lo[d] = fmin(lo[d], v);
            hi[d] = fmax(hi[d], v);
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        for (int64_t i = t0; i < a.qn[d]; i += stride) {
            double v = a.q[d][i];
            lo[d] = fmin(lo[d], v);
            hi[d] = fmax(hi[d], v);
        }
    }
    __shared__ double red[6][256];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        red[d][threadIdx.x] = lo[d];
        red[3 + d][threadIdx.x] = hi[d];
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                red[d][threadIdx.x] = fmin(red[d][threadIdx.x], red[d][threadIdx.x + s]);
                red[3 + d][threadIdx.x] = fmax(red[3 + d][threadIdx.x], red[3 + d][threadIdx.x + s]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) partials[(size_t)blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// 256 threads: strided partial min/max per dimension, then an LDS tree (was 6 serial lanes)
__global__ __launch_bounds__(256) void k_bbox_final(const double *partials, int nblk, double *out) {
    double r[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) r[d] = d < 3 ? INFINITY : -INFINITY;
    for (int b = threadIdx.x; b < nblk; b += 256) {
#pragma unroll
        for (int d = 0; d < 6; ++d) {
            const double v = partials[(size_t)b * 6 + d];
            r[d] = d < 3 ? fmin(r[d], v) : fmax(r[d], v);
        }
    }
    __shared__ double red[6][256];
#pragma unroll
    for (int d = 0; d < 6; ++d) red[d][threadIdx.x] = r[d];
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) {
#pragma unroll
            for (int d = 0; d < 6; ++d)
                red[d][threadIdx.x] = d < 3 ? fmin(red[d][threadIdx.x], red[d][threadIdx.x + st])
                                            : fmax(red[d][threadIdx.x], red[d][threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) out[threadIdx.x] = red[threadIdx.x][0];
}

int launch_bbox(const double *const px[3], int64_t n, const double *const qa[3], const int64_t qn[3],
                double *d_partials, int max_blocks, double *d_out6, hipStream_t s, const uint32_t *d_n) {
    BBoxArgs a;
    a.dn = d_n;
    int64_t m = n;
    for (int d = 0; d < 3; ++d) {
        a.p[d] = px[d];
        a.q[d] = qa[d];
        a.qn[d] = qn[d];
        m = std::max(m, qn[d]);
    }
    a.n = n;
    int nblk = (int)std::min<int64_t>((m + 255) / 256, max_blocks);
    nblk = std::max(nblk, 1);
    hipLaunchKernelGGL(k_bbox, dim3(nblk), dim3(256), 0, s, a, d_partials);
    hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(256), 0, s, (const double *)d_partials, nblk, d_out6);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// ---------------------------------------------------------------------------
// cell codes + histogram
// ---------------------------------------------------------------------------
__device__ __forceinline__ int cell_coord(double v, double o, double ic, int nc) {
    double f = floor((v - o) * ic);
    int c = (f < 0.0) ? 0 : (f >= (double)nc ? nc - 1 : (int)f);
    return c;
}

// cell code + histogram; the atomic's return value is the particle's arrival rank in its
// cell (any order: k_seg_sort makes the in-cell order deterministic), so the scatter needs no
// second round of atomics
__global__ __launch_bounds__(256) void k_cell_code(CellGrid cg, const double *__restrict__ x,
                                                   const double *__restrict__ y, const double *__restrict__ z,
                                                   int64_t n, uint32_t *__restrict__ code,
                                                   uint32_t *__restrict__ count, uint32_t *__restrict__ rank) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int cx = cell_coord(x[i], cg.o[0], cg.ic[0], cg.nc[0]);
    int cy = cell_coord(y[i], cg.o[1], cg.ic[1], cg.nc[1]);
    int cz = cell_coord(z[i], cg.o[2], cg.ic[2], cg.nc[2]);
    uint32_t c = (uint32_t)(((long long)cz * cg.nc[1] + cy) * cg.nc[0] + cx);
    code[i] = c;
    rank[i] = atomicAdd(&count[c], 1u);
}

// ---------------------------------------------------------------------------
// exclusive scan of m uint32 counts -> start[0..m] (start[m] = total)
// ---------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;  // 4096

size_t scan_partials_needed(size_t m) { return (m + kScanTile - 1) / kScanTile + 1; }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint32_t *__restrict__ in, size_t m,
                                                              uint32_t *__restrict__ partials) {
    size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        size_t i = base + j;
        s += (i < m) ? in[i] : 0u;
    }
    // block reduce
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ uint32_t ws[kScanThreads / 64];
    if (lane == 0) ws[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) t += ws[w];
        partials[blockIdx.x] = t;
    }
}

// single-block exclusive scan of the block partials (in place), total -> partials[nb]
__global__ __launch_bounds__(1024) void k_scan_partials(uint32_t *partials, int nb) {
    __shared__ uint32_t ws[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < nb; base += 1024) {
        int i = base + threadIdx.x;
        uint32_t v = (i < nb) ? partials[i] : 0u;
        uint32_t inc = wave_incl_scan(v);
        if (lane == 63) ws[wid] = inc;
        __syncthreads();
        if (threadIdx.x < 64) {
            uint32_t t = (threadIdx.x < 16) ? ws[threadIdx.x] : 0u;
            uint32_t ti = wave_incl_scan(t);
            if (threadIdx.x < 16) ws[threadIdx.x] = ti - t;
        }
        __syncthreads();
        uint32_t excl = carry + ws[wid] + inc - v;
        __syncthreads();
        if (i < nb) partials[i] = excl;
        if (threadIdx.x == 1023) carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[nb] = carry;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_final(const uint32_t *__restrict__ in, size_t m,
                                                             const uint32_t *__restrict__ partials, int nb,
                                                             uint32_t *__restrict__ out) {
    size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        size_t i = base + j;
        v[j] = (i < m) ? in[i] : 0u;
        s += v[j];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(s);
    __shared__ uint32_t ws[kScanThreads / 64];
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    uint32_t off = partials[blockIdx.x];
    for (int w = 0; w < wid; ++w) off += ws[w];
    uint32_t run = off + inc - s;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        size_t i = base + j;
        if (i < m) out[i] = run;
        run += v[j];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[m] = partials[nb];
}

// ---------------------------------------------------------------------------
// scatter + deterministic in-cell order
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_scatter(const uint32_t *__restrict__ code, int64_t n,
                                                 const uint32_t *__restrict__ start,
                                                 const uint32_t *__restrict__ rank, uint32_t *__restrict__ perm) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    perm[start[code[i]] + rank[i]] = (uint32_t)i;
}

__device__ void sift_down(uint32_t *a, int root, int n) {
    while (true) {
        int child = 2 * root + 1;
        if (child >= n) return;
        if (child + 1 < n && a[child + 1] > a[child]) child++;
        if (a[root] >= a[child]) return;
        uint32_t t = a[root];
        a[root] = a[child];
        a[child] = t;
        root = child;
    }
}

// sorts each cell's slots by original index and records every particle's final slot
// (inv[original] = slot) for the placement pass
__global__ __launch_bounds__(256) void k_seg_sort(const uint32_t *__restrict__ start, size_t m,
                                                  uint32_t *__restrict__ perm, uint32_t *__restrict__ inv) {
    size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= m) return;
    uint32_t s = start[c], e = start[c + 1];
    int n = (int)(e - s);
    if (n <= 0) return;
    uint32_t *a = perm + s;
    if (n == 1) {
        inv[a[0]] = s;
        return;
    }
    if (n <= 48) {
        for (int i = 1; i < n; ++i) {
            uint32_t v = a[i];
            int j = i - 1;
            while (j >= 0 && a[j] > v) {
                a[j + 1] = a[j];
                --j;
            }
            a[j + 1] = v;
        }
    } else {  // pathological clustering: heap sort, O(n log n), still deterministic
        for (int r = n / 2 - 1; r >= 0; --r) sift_down(a, r, n);
        for (int end = n - 1; end > 0; --end) {
            uint32_t t = a[0];
            a[0] = a[end];
            a[end] = t;
            sift_down(a, 0, end);
        }
    }
    for (int j = 0; j < n; ++j) inv[a[j]] = s + (uint32_t)j;
}

// placement in original order: coalesced 48-B reads per particle, two full 32-B record
// writes at its slot (the slot-order gather read six scattered 8-B values per particle)
__global__ __launch_bounds__(256) void k_place(const uint32_t *__restrict__ inv, int64_t n,
                                               const double *__restrict__ x, const double *__restrict__ y,
                                               const double *__restrict__ z, const double *__restrict__ u,
                                               const double *__restrict__ v, const double *__restrict__ w,
                                               double4 *__restrict__ prec, double4 *__restrict__ pval) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = inv[i];
    prec[s] = make_double4(x[i], y[i], z[i], (double)i);
    pval[s] = make_double4(u[i], v[i], w[i], 0.0);
}

// ---------------------------------------------------------------------------
// slab cull (multi-GPU z-slab with replicated particles, ptv_knn_params.slab_halo):
// keep the particles with z in [min(az[z0..z1)) - halo, max(az[z0..z1)) + halo], in their
// original relative order (order-preserving compaction: per-block counts, scan, write)
// ---------------------------------------------------------------------------
constexpr int kCullItems = 4;  // particles per thread (16 measured 87 us for the write pass at 5M, latency-bound)
constexpr int kCullTile = 256 * kCullItems;  // particles per block

// win[0..3] = (zlo, zhi, slab z min, slab z max)
__global__ __launch_bounds__(256) void k_slab_window(const double *__restrict__ az, int z0, int z1, double halo,
                                                     double *__restrict__ win) {
    double lo = INFINITY, hi = -INFINITY;
    for (int i = z0 + (int)threadIdx.x; i < z1; i += 256) {
        lo = fmin(lo, az[i]);
        hi = fmax(hi, az[i]);
    }
    __shared__ double rl[256], rh[256];
    rl[threadIdx.x] = lo;
    rh[threadIdx.x] = hi;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            rl[threadIdx.x] = fmin(rl[threadIdx.x], rl[threadIdx.x + s]);
            rh[threadIdx.x] = fmax(rh[threadIdx.x], rh[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        win[0] = rl[0] - halo;
        win[1] = rh[0] + halo;
        win[2] = rl[0];
        win[3] = rh[0];
    }
}

__device__ __forceinline__ bool in_window(double z, const double *win) { return z >= win[0] && z <= win[1]; }

// the cull test of particle i: z inside the window [win[0], win[1]], or (per-column map) above it
// up to the top of its (x, y) cell / below it down to the bottom
__device__ __forceinline__ bool cull_keep(const double *__restrict__ x, const double *__restrict__ y,
                                          const double *__restrict__ z, int64_t i, double lo, double hi,
                                          const CullMap &m) {
    const double v = z[i];
    if (v >= lo && v <= hi) return true;
    if (m.top == nullptr) return false;
    const int cx = (int)fmin(fmax(floor((x[i] - m.x0) * m.icw), 0.0), (double)(m.mx - 1));
    const int cy = (int)fmin(fmax(floor((y[i] - m.y0) * m.ich), 0.0), (double)(m.my - 1));
    const int c = cy * m.mx + cx;
    return v > hi ? v <= m.top[c] : v >= m.bot[c];  // NaN coordinates: never kept
}

// pass 1: the keep test of every particle, one ballot mask per (block item, wave) and the block's count
__global__ __launch_bounds__(256) void k_cull_count(const double *__restrict__ x, const double *__restrict__ y,
                                                    const double *__restrict__ z, int64_t n,
                                                    const double *__restrict__ win, CullMap m,
                                                    uint32_t *__restrict__ bcount,
                                                    unsigned long long *__restrict__ masks) {
    const double lo = win[0], hi = win[1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kCullTile + threadIdx.x;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kCullItems; ++j) {
        const int64_t i = base + (int64_t)j * 256;
        const unsigned long long bm = __builtin_amdgcn_ballot_w64(i < n && cull_keep(x, y, z, i, lo, hi, m));
        if (lane == 0) masks[((size_t)blockIdx.x * kCullItems + j) * 4 + wid] = bm;
        c += (uint32_t)__builtin_popcountll(bm);
    }
    __shared__ uint32_t ws[4];
    if (lane == 0) ws[wid] = c;
    __syncthreads();
    if (threadIdx.x == 0) bcount[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

struct Cols6 {
    const double *src[6];
    double *dst[6];
};

// pass 2 (after the scan of the counts): the kept particles' six columns from pass 1's masks.
// Item (j, thread) of a block is particle base + j*256 + thread: j-major, thread-minor is index
// order, so the ranks below preserve it
__global__ __launch_bounds__(256) void k_cull_write(Cols6 c, int64_t n, const unsigned long long *__restrict__ masks,
                                                    const uint32_t *__restrict__ boff) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kCullTile + threadIdx.x;
    const unsigned long long *bm = masks + (size_t)blockIdx.x * kCullItems * 4;
    uint32_t off = boff[blockIdx.x];
#pragma unroll
    for (int j = 0; j < kCullItems; ++j) {
        const unsigned long long w0 = bm[j * 4], w1 = bm[j * 4 + 1], w2 = bm[j * 4 + 2], w3 = bm[j * 4 + 3];
        const unsigned long long m = wid == 0 ? w0 : (wid == 1 ? w1 : (wid == 2 ? w2 : w3));
        uint32_t pre = off;
        if (wid > 0) pre += (uint32_t)__builtin_popcountll(w0);
        if (wid > 1) pre += (uint32_t)__builtin_popcountll(w1);
        if (wid > 2) pre += (uint32_t)__builtin_popcountll(w2);
        if ((m >> lane) & 1ull) {
            const uint32_t r = pre + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            const int64_t i = base + (int64_t)j * 256;
#pragma unroll
            for (int a = 0; a < 6; ++a) c.dst[a][r] = c.src[a][i];
        }
        off += (uint32_t)(__builtin_popcountll(w0) + __builtin_popcountll(w1) + __builtin_popcountll(w2) +
                          __builtin_popcountll(w3));
    }
    (void)n;
}

size_t cull_blocks(int64_t n) { return (size_t)((n + kCullTile - 1) / kCullTile); }

size_t cull_mask_words(int64_t n) { return cull_blocks(n) * kCullItems * 4; }

int launch_cull(const double *const src[6], int64_t n, const double *az, int z0, int z1, double halo, double *win,
                uint32_t *bcount, unsigned long long *masks, double *const dst[6], uint32_t *h_total, hipStream_t s,
                const CullMap *map) {
    const int nb = (int)cull_blocks(n);
    const CullMap m = map != nullptr ? *map : CullMap{};
    hipLaunchKernelGGL(k_slab_window, dim3(1), dim3(256), 0, s, az, z0, z1, map != nullptr ? 0.0 : halo, win);
    hipLaunchKernelGGL(k_cull_count, dim3(nb), dim3(256), 0, s, src[0], src[1], src[2], n, (const double *)win, m,
                       bcount, masks);
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, bcount, nb);  // total -> bcount[nb]
    Cols6 c;
    for (int a = 0; a < 6; ++a) {
        c.src[a] = src[a];
        c.dst[a] = dst[a];
    }
    hipLaunchKernelGGL(k_cull_write, dim3(nb), dim3(256), 0, s, c, n, (const unsigned long long *)masks,
                       (const uint32_t *)bcount);
    PTV_HIP(hipGetLastError());
    if (h_total != nullptr) PTV_HIP(hipMemcpyAsync(h_total, bcount + nb, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    return PTV_OK;
}

// ---------------------------------------------------------------------------
// Per-column cull map (PTV_FLAG_SLAB_CULL_AUTO).  Every slab voxel v lies in a cell Q of the
// slab's finest lattice, and with the cell's corner bounds D(c) (k-th distance of the lattice
// point c, from the particles binned) d_k(v) <= D(c*) + |v - c*| for its nearest corner c*, so
// d_k(v) <= U(Q) = max_c D(c) + diag(Q) / 2 over the whole cell.  A particle p that is among
// v's k nearest therefore lies within U(Q) of the box Q.  Above the slab (z > Q's top z1) that
// means z <= z1 + sqrt(U^2 - gap_xy(p, Q)^2): the map keeps, for each (x, y) cell, the largest
// such height over every lattice cell that reaches it (and the lowest depth below the slab).
// Per lattice column (i, j) the cells l are folded into T = max_l (z1 + U), B = min_l (z0 - U)
// and Rm = max_l U; since r - sqrt(r^2 - g^2) decreases in r, T - Rm + sqrt(Rm^2 - g^2) bounds
// every cell's height of the column (B + Rm - sqrt(...) every depth).  A culled particle is then
// strictly farther than U(Q) from every cell, so it is neither among any voxel's k nearest nor
// tied with the k-th.  Margins: relative 1e-9 on every distance plus the binning margin.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long ord_key(double v) {  // monotone double -> u64
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double ord_val(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

constexpr int kColFields = 7;  // x lo, x hi, y lo, y hi, T, B, Rm

__global__ __launch_bounds__(256) void k_cull_columns(const double *__restrict__ lax, const double *__restrict__ lay,
                                                      const double *__restrict__ laz, int n0, int n1, int n2,
                                                      const double *__restrict__ dk, double mg, double slack,
                                                      double *__restrict__ cols) {
    const int c0 = max(n0 - 1, 1), c1 = max(n1 - 1, 1), c2 = max(n2 - 1, 1);
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= c0 * c1) return;
    const int i = t % c0, j = t / c0;
    const int i1 = min(i + 1, n0 - 1), j1 = min(j + 1, n1 - 1);
    const double xa = lax[i], xb = lax[i1], ya = lay[j], yb = lay[j1];
    const double dx = fabs(xb - xa), dy = fabs(yb - ya);
    auto D = [&](int a, int b, int l) { return dk[((size_t)l * n1 + b) * n0 + a]; };
    double T = -INFINITY, B = INFINITY, Rm = 0.0;
    for (int l = 0; l < c2; ++l) {
        const int l1 = min(l + 1, n2 - 1);
        const double za = laz[l], zb = laz[l1];
        const double dz = fabs(zb - za);
        const double dmax = fmax(fmax(fmax(D(i, j, l), D(i1, j, l)), fmax(D(i, j1, l), D(i1, j1, l))),
                                 fmax(fmax(D(i, j, l1), D(i1, j, l1)), fmax(D(i, j1, l1), D(i1, j1, l1))));
        const double U = (dmax + 0.5 * sqrt((dx * dx + dy * dy) + dz * dz)) * (1.0 + 1e-9 + slack) + mg;
        T = fmax(T, fmax(za, zb) + U);
        B = fmin(B, fmin(za, zb) - U);
        Rm = fmax(Rm, U);
    }
    if (!(Rm < INFINITY)) Rm = INFINITY;  // NaN bounds: reach everything
    double *o = cols + (size_t)t * kColFields;
    o[0] = fmin(xa, xb);
    o[1] = fmax(xa, xb);
    o[2] = fmin(ya, yb);
    o[3] = fmax(ya, yb);
    o[4] = T;
    o[5] = B;
    o[6] = Rm;
}

__global__ __launch_bounds__(256) void k_cull_map_init(unsigned long long *__restrict__ kt,
                                                       unsigned long long *__restrict__ kb, int nm) {
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t < nm) {
        kt[t] = ord_key(-INFINITY);
        kb[t] = ord_key(INFINITY);
    }
}

// map cell (thread) x a chunk of kMapChunk lattice columns (blockIdx.y): the chunk's largest height
// and lowest depth into the cell's ordered keys
constexpr int kMapChunk = 256;
__global__ __launch_bounds__(256) void k_cull_map(const double *__restrict__ cols, int ncol, CullMap m,
                                                  unsigned long long *__restrict__ kt,
                                                  unsigned long long *__restrict__ kb) {
    __shared__ double sc[kMapChunk * kColFields];
    const int c0 = (int)blockIdx.y * kMapChunk;
    const int nc = min(kMapChunk, ncol - c0);
    for (int e = (int)threadIdx.x; e < nc * kColFields; e += 256) sc[e] = cols[(size_t)c0 * kColFields + e];
    __syncthreads();
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= m.mx * m.my) return;
    const int cx = t % m.mx, cy = t / m.mx;
    // the cell's rectangle, widened for the particles' floor() assignment
    const double ex = 1e-9 * (fabs(m.x0) + m.mx * m.cw) + 1e-300, ey = 1e-9 * (fabs(m.y0) + m.my * m.ch) + 1e-300;
    // (edge cells reach out to infinity: particles beyond the grid are clamped into them)
    const double x0 = cx == 0 ? -INFINITY : m.x0 + cx * m.cw - ex;
    const double x1 = cx == m.mx - 1 ? INFINITY : m.x0 + (cx + 1) * m.cw + ex;
    const double y0 = cy == 0 ? -INFINITY : m.y0 + cy * m.ch - ey;
    const double y1 = cy == m.my - 1 ? INFINITY : m.y0 + (cy + 1) * m.ch + ey;
    double top = -INFINITY, bot = INFINITY;
    for (int q = 0; q < nc; ++q) {
        const double *o = sc + q * kColFields;
        const double gx = fmax(fmax(o[0] - x1, x0 - o[1]), 0.0), gy = fmax(fmax(o[2] - y1, y0 - o[3]), 0.0);
        const double g2 = gx * gx + gy * gy, R = o[6];
        if (!(R < INFINITY)) {  // an unbounded lattice cell: keep the whole column
            top = INFINITY;
            bot = -INFINITY;
        } else if (g2 <= R * R) {
            const double h = sqrt(R * R - g2);
            const double mgn = 1e-9 * (fabs(o[4]) + fabs(o[5]) + R);
            top = fmax(top, (o[4] - R) + h + mgn);
            bot = fmin(bot, (o[5] + R) - h - mgn);
        }
    }
    if (top > -INFINITY) atomicMax(kt + t, ord_key(top));
    if (bot < INFINITY) atomicMin(kb + t, ord_key(bot));
}

// decode the keys into the map (top / bot doubles); with `used`, the proof that the cull ran with
// a map at least as wide everywhere (*fail: 0 = proven; any cell short sets +inf's bits)
__global__ __launch_bounds__(256) void k_cull_map_final(const unsigned long long *__restrict__ kt,
                                                        const unsigned long long *__restrict__ kb, int nm,
                                                        double *__restrict__ top, double *__restrict__ bot,
                                                        const double *__restrict__ utop,
                                                        const double *__restrict__ ubot,
                                                        unsigned long long *__restrict__ fail) {
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    bool short_ = false;
    if (t < nm) {
        const double a = ord_val(kt[t]), b = ord_val(kb[t]);
        top[t] = a;
        bot[t] = b;
        if (utop != nullptr) short_ = !(a <= utop[t]) || !(b >= ubot[t]);
    }
    if (utop != nullptr && __builtin_amdgcn_ballot_w64(short_) != 0 && (threadIdx.x & 63) == 0)
        atomicMax(fail, (unsigned long long)__double_as_longlong(INFINITY));
}

// the cull proof of a call with the cached map: the map is monotone in the lattice bounds, so
// every bound of this call within `factor` of the bound the map was built from proves it (the
// lattice points are the same: the cache key holds the grid and the slab).  *fail as launch_cull_need.
__global__ __launch_bounds__(256) void k_bounds_within(const double *__restrict__ dk, const double *__restrict__ ref,
                                                       long long n, double factor, unsigned long long *__restrict__ fail) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const bool bad = i < n && !(dk[i] <= ref[i] * factor);
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && (threadIdx.x & 63) == 0)
        atomicMax(fail, (unsigned long long)__double_as_longlong(INFINITY));
}

// the cached cull map's speculative reuse: *fail = +inf's bits unless key[0..n) equals ref bitwise and
// the kept count equals the cached one (atomicMax: it only ever raises the word)
__global__ __launch_bounds__(256) void k_key_check(const double *__restrict__ key, const double *__restrict__ ref,
                                                   int n, const uint32_t *__restrict__ count, uint32_t expect,
                                                   unsigned long long *__restrict__ fail) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool bad = (i < n && __double_as_longlong(key[i]) != __double_as_longlong(ref[i])) ||
                     (i == 0 && *count != expect);
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && (threadIdx.x & 63) == 0)
        atomicMax(fail, (unsigned long long)__double_as_longlong(INFINITY));
}

int launch_key_check(const double *key, const double *ref, int n, const uint32_t *count, uint32_t expect,
                     unsigned long long *fail, hipStream_t s) {
    hipLaunchKernelGGL(k_key_check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, key, ref, n, count, expect,
                       fail);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_bounds_within(const double *dk, const double *ref, long long n, double factor, unsigned long long *fail,
                         hipStream_t s, bool reset) {
    if (reset) PTV_HIP(hipMemsetAsync(fail, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_bounds_within, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dk, ref, n, factor, fail);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_cull_need(const double *lax, const double *lay, const double *laz, const int n[3], const double *dk,
                     double mg, double slack, const CullMap &m, double *top, double *bot, double *cols,
                     unsigned long long *keys, const CullMap *used, unsigned long long *fail, hipStream_t s) {
    const int ncol = std::max(n[0] - 1, 1) * std::max(n[1] - 1, 1);
    const int nm = m.mx * m.my;
    hipLaunchKernelGGL(k_cull_columns, dim3((ncol + 255) / 256), dim3(256), 0, s, lax, lay, laz, n[0], n[1], n[2], dk, mg,
                       slack, cols);
    hipLaunchKernelGGL(k_cull_map_init, dim3((nm + 255) / 256), dim3(256), 0, s, keys, keys + nm, nm);
    hipLaunchKernelGGL(k_cull_map, dim3((nm + 255) / 256, (ncol + kMapChunk - 1) / kMapChunk), dim3(256), 0, s,
                       (const double *)cols, ncol, m, keys, keys + nm);
    if (used != nullptr) PTV_HIP(hipMemsetAsync(fail, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_cull_map_final, dim3((nm + 255) / 256), dim3(256), 0, s, (const unsigned long long *)keys,
                       (const unsigned long long *)(keys + nm), nm, top, bot, used ? used->top : nullptr,
                       used ? used->bot : nullptr, fail);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// a fingerprint of a particle set: the six values of kFingerprint evenly spaced particles
__global__ void k_fingerprint(Cols6 c, int64_t n, double *__restrict__ out) {
    const int t = (int)threadIdx.x;
    if (t < 6 * kFingerprint) {
        const int a = t / kFingerprint, j = t % kFingerprint;
        out[t] = c.src[a][(int64_t)((double)j * (double)(n - 1) / (double)(kFingerprint - 1))];
    }
}

int launch_fingerprint(const double *const src[6], int64_t n, double *out, hipStream_t s) {
    Cols6 c;
    for (int a = 0; a < 6; ++a) {
        c.src[a] = src[a];
        c.dst[a] = nullptr;
    }
    hipLaunchKernelGGL(k_fingerprint, dim3(1), dim3(6 * kFingerprint), 0, s, c, n, out);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// ---------------------------------------------------------------------------
// sort-based binning: cell codes without atomics, a stable radix sort of (code, index) pairs
// (in-cell order = ascending original index, as k_seg_sort makes it), cell starts by binary
// search, the inverse permutation, then k_place
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_cell_key(CellGrid cg, const double *__restrict__ x,
                                                  const double *__restrict__ y, const double *__restrict__ z,
                                                  int64_t n, uint32_t *__restrict__ code, uint32_t *__restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int cx = cell_coord(x[i], cg.o[0], cg.ic[0], cg.nc[0]);
    const int cy = cell_coord(y[i], cg.o[1], cg.ic[1], cg.nc[1]);
    const int cz = cell_coord(z[i], cg.o[2], cg.ic[2], cg.nc[2]);
    code[i] = (uint32_t)(((long long)cz * cg.nc[1] + cy) * cg.nc[0] + cx);
    idx[i] = (uint32_t)i;
}

// inv[perm[j]] = j (the placement pass writes each particle's records at its slot), and
// start[c] = first sorted position whose code is >= c, c in [0, m]: thread j at a code change
// (codes c' < c at j - 1, j) writes the start of cells (c', c] -- up to kStartGap of them (the
// pack's solid spheres leave runs of hundreds of empty x-thin cells); a longer run of empty cells
// raises *flag and k_start_fixup then binary-searches every cell
constexpr int kStartGap = 1 << 16;
__global__ __launch_bounds__(256) void k_sorted_starts(const uint32_t *__restrict__ skey, const uint32_t *__restrict__ perm,
                                                       int64_t n, size_t m, uint32_t *__restrict__ start,
                                                       uint32_t *__restrict__ inv, uint32_t *__restrict__ flag) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    if (j < n) inv[perm[j]] = (uint32_t)j;
    const int64_t prev = j == 0 ? -1 : (int64_t)skey[j - 1];
    const int64_t cur = j == n ? (int64_t)m : (int64_t)skey[j];
    if (cur - prev > kStartGap) {
        atomicOr(flag, 1u);
        return;
    }
    for (int64_t c = prev + 1; c <= cur; ++c) start[c] = (uint32_t)j;
}

__global__ __launch_bounds__(256) void k_start_fixup(const uint32_t *__restrict__ skey, int64_t n, size_t m,
                                                     uint32_t *__restrict__ start, const uint32_t *__restrict__ flag) {
    if (*flag == 0u) return;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c <= (int64_t)m;
         c += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)skey[mid] < c) lo = mid + 1;
            else hi = mid;
        }
        start[c] = (uint32_t)lo;
    }
}

static int cell_key_bits(size_t m) {
    int b = 1;
    while (b < 32 && ((size_t)1 << b) < m) ++b;
    return b;
}

size_t bin_sort_temp_bytes(int64_t n, size_t m) {
    size_t tb = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, 0,
                                           cell_key_bits(m)) != hipSuccess)
        return 0;
    return tb;
}

static int launch_bin_sort(const CellGrid &cg, const double *const px[3], const double *const pv[3], int64_t n,
                           uint32_t *d_code, uint32_t *d_perm, uint32_t *d_count, uint32_t *d_start,
                           double4 *d_prec, double4 *d_pval, const BinSortScratch &ss, hipStream_t s) {
    const size_t m = (size_t)cg.ncells;
    const int nb = (int)((n + 255) / 256);
    uint32_t *d_idx = d_code + n;
    hipLaunchKernelGGL(k_cell_key, dim3(nb), dim3(256), 0, s, cg, px[0], px[1], px[2], n, d_code, d_idx);
    size_t tb = ss.temp_bytes;
    PTV_HIP(hipcub::DeviceRadixSort::SortPairs(ss.temp, tb, (const uint32_t *)d_code, ss.keys, (const uint32_t *)d_idx,
                                               d_perm, (int)n, 0, cell_key_bits(m), s));
    // d_code is dead after the sort: it holds the inverse permutation from here on; the flag word
    // is the first of the (unused) count buffer
    PTV_HIP(hipMemsetAsync(d_count, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_sorted_starts, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s,
                       (const uint32_t *)ss.keys, (const uint32_t *)d_perm, n, m, d_start, d_code, d_count);
    hipLaunchKernelGGL(k_start_fixup, dim3(1024), dim3(256), 0, s, (const uint32_t *)ss.keys, n, m, d_start,
                       (const uint32_t *)d_count);
    hipLaunchKernelGGL(k_place, dim3(nb), dim3(256), 0, s, (const uint32_t *)d_code, n, px[0], px[1], px[2],
                       pv[0], pv[1], pv[2], d_prec, d_pval);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_bin(const CellGrid &cg, const double *const px[3], const double *const pv[3], int64_t n,
               uint32_t *d_code, uint32_t *d_perm, uint32_t *d_count, uint32_t *d_start,
               uint32_t *d_scan_partials, double4 *d_prec, double4 *d_pval, hipStream_t s,
               const BinSortScratch *ss) {
    if (ss != nullptr && ss->keys != nullptr && ss->temp != nullptr)
        return launch_bin_sort(cg, px, pv, n, d_code, d_perm, d_count, d_start, d_prec, d_pval, *ss, s);
    const size_t m = (size_t)cg.ncells;
    PTV_HIP(hipMemsetAsync(d_count, 0, m * sizeof(uint32_t), s));
    const int nb = (int)((n + 255) / 256);
    uint32_t *d_rank = d_code + n;  // in-cell arrival ranks: the second half of the code buffer (2n)
    hipLaunchKernelGGL(k_cell_code, dim3(nb), dim3(256), 0, s, cg, px[0], px[1], px[2], n, d_code, d_count, d_rank);
    const int sb = (int)((m + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(k_scan_reduce, dim3(sb), dim3(kScanThreads), 0, s, (const uint32_t *)d_count, m,
                       d_scan_partials);
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, d_scan_partials, sb);
    hipLaunchKernelGGL(k_scan_final, dim3(sb), dim3(kScanThreads), 0, s, (const uint32_t *)d_count, m,
                       (const uint32_t *)d_scan_partials, sb, d_start);
    hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(256), 0, s, (const uint32_t *)d_code, n,
                       (const uint32_t *)d_start, (const uint32_t *)d_rank, d_perm);
    // d_code is dead after the scatter: it holds the inverse permutation from here on
    hipLaunchKernelGGL(k_seg_sort, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, (const uint32_t *)d_start, m,
                       d_perm, d_code);
    hipLaunchKernelGGL(k_place, dim3(nb), dim3(256), 0, s, (const uint32_t *)d_code, n, px[0], px[1], px[2],
                       pv[0], pv[1], pv[2], d_prec, d_pval);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
