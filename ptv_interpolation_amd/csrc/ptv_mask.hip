// ptv_mask.hip — the pore-mask path on the GPU.
//
//   sample_mask_on_grid          interpolator.py:205-238  RegularGridInterpolator(method='nearest',
//                                bounds_error=False, fill_value=0) of the raw mask at every grid
//                                voxel, then `> 0.5`
//   extract_boundary_particles   interpolator.py:240-284  binary_dilation(fluid, 6-connected,
//                                iterations=thickness) & ~mask -> np.where (C order) -> [::step]
//                                -> physical coordinates
//
// Both are byte streams (1 B per voxel in, 1 B or a few sparse 24 B records out): HBM bound,
// one coalesced byte per lane, neighbour bytes from L1/L2 (the 6-point stencil re-reads each
// byte 7 times; only the first read reaches HBM).
#include "ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

// ---------------------------------------------------------------------------
// nearest-index lookup of RegularGridInterpolator (scipy _rgi.py _find_indices +
// _evaluate_nearest + _find_out_of_bounds, scipy 1.15):
//   i = interval with g[i] <= x < g[i+1] (clamped to [0, n-2]), t = (x - g[i]) / (g[i+1] - g[i]),
//   index = t <= 0.5 ? i : i + 1;  x < g[0] or x > g[n-1] -> fill (returned as -1).
//   A length-one axis maps every in-bounds x (x == g[0]) to 0.  `g` is ascending; a
//   descending caller axis is passed reversed with flip = 1 (scipy flips it the same way).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int rgi_nearest(const double *__restrict__ g, int n, int flip, double x) {
    const double g0 = g[0], gl = g[n - 1];
    if (x < g0 || x > gl) return -1;
    if (x != x) return -1;  // NaN coordinate: never > 0.5 in the reference either (parity unpinned)
    int j;
    if (n == 1) {
        j = 0;
    } else {
        int lo = 0, hi = n - 2;  // largest i in [0, n-2] with g[i] <= x
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (g[mid] <= x) lo = mid;
            else hi = mid - 1;
        }
        const double t = (x - g[lo]) / (g[lo + 1] - g[lo]);
        j = t <= 0.5 ? lo : lo + 1;
    }
    return flip ? n - 1 - j : j;
}

struct MaskSampleArgs {
    int rn[3];          // raw mask extents x, y, z
    int flip[3];
    const double *ra[3];  // raw axes (ascending)
    const uint8_t *raw;   // (rn[2], rn[1], rn[0]), 1 = value > 0.5
    int nx, ny;           // grid plane
    int z0, z1;           // planes of this launch
    int separable;
};

// per-axis tables for separable grids: tab[i] = raw index of grid axis point i, -1 = outside
__global__ __launch_bounds__(256) void k_mask_axis_table(const double *__restrict__ g, int n, int flip,
                                                         const double *__restrict__ q, int nq, int *__restrict__ tab) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < nq) tab[i] = rgi_nearest(g, n, flip, q[i]);
}

// 8 consecutive x voxels per lane: two 16-byte table loads, 8 raw-byte gathers (L1/L2: a raw
// row is shared by neighbouring lanes and by every grid row that maps to it), one 8-byte
// store when the run is 8-aligned inside the row (otherwise per-byte, row tails included)
__global__ __launch_bounds__(256) void k_mask_sample_sep(MaskSampleArgs a, const int *__restrict__ tx,
                                                         const int *__restrict__ ty, const int *__restrict__ tz,
                                                         uint8_t *__restrict__ out) {
    // flat lane index -> (row, 8-voxel segment); rows = (z, y) pairs of this launch
    const int segs = (a.nx + 7) >> 3;
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = g / segs;
    if (row >= (int64_t)a.ny * (a.z1 - a.z0)) return;
    const int ix0 = (int)(g - row * segs) * 8;
    const int iy = (int)(row % a.ny);
    const int iz = a.z0 + (int)(row / a.ny);
    const int jy = ty[iy], jz = tz[iz];
    const size_t orow = ((size_t)(iz - a.z0) * a.ny + iy) * a.nx;
    const bool row_ok = (jy | jz) >= 0;
    const uint8_t *rrow = a.raw + ((size_t)(row_ok ? jz : 0) * a.rn[1] + (row_ok ? jy : 0)) * a.rn[0];
    int jx[8];
    if (ix0 + 8 <= a.nx) {  // tx is 16-byte aligned (hipMalloc) and ix0 % 8 == 0
        const int4 t0 = *reinterpret_cast<const int4 *>(tx + ix0);
        const int4 t1 = *reinterpret_cast<const int4 *>(tx + ix0 + 4);
        jx[0] = t0.x; jx[1] = t0.y; jx[2] = t0.z; jx[3] = t0.w;
        jx[4] = t1.x; jx[5] = t1.y; jx[6] = t1.z; jx[7] = t1.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) jx[j] = tx[min(ix0 + j, a.nx - 1)];
    }
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t v = (row_ok && jx[j] >= 0) ? rrow[jx[j]] : 0u;
        if (j < 4) lo |= v << (8 * j);
        else hi |= v << (8 * (j - 4));
    }
    if (ix0 + 8 <= a.nx && ((orow + ix0) & 7) == 0) {
        *reinterpret_cast<uint2 *>(out + orow + ix0) = make_uint2(lo, hi);
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (ix0 + j < a.nx) out[orow + ix0 + j] = (uint8_t)((j < 4 ? lo >> (8 * j) : hi >> (8 * (j - 4))) & 0xff);
    }
}

// point-list grids: the three lookups per voxel
__global__ __launch_bounds__(256) void k_mask_sample_pts(MaskSampleArgs a, const double *__restrict__ px,
                                                         const double *__restrict__ py, const double *__restrict__ pz,
                                                         int64_t nvox, uint8_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nvox) return;
    const int64_t v = (int64_t)a.z0 * a.nx * a.ny + i;
    const int jx = rgi_nearest(a.ra[0], a.rn[0], a.flip[0], px[v]);
    const int jy = rgi_nearest(a.ra[1], a.rn[1], a.flip[1], py[v]);
    const int jz = rgi_nearest(a.ra[2], a.rn[2], a.flip[2], pz[v]);
    uint8_t r = 0;
    if ((jx | jy | jz) >= 0) r = a.raw[((size_t)jz * a.rn[1] + jy) * a.rn[0] + jx];
    out[i] = r;
}

int launch_mask_sample(const MaskSampleLaunch &m, const double *ax, const double *ay, const double *az,
                       const double *px, const double *py, const double *pz, int *tabs, uint8_t *out,
                       hipStream_t s) {
    MaskSampleArgs a;
    for (int d = 0; d < 3; ++d) {
        a.rn[d] = m.rn[d];
        a.flip[d] = m.flip[d];
        a.ra[d] = m.ra[d];
    }
    a.raw = m.raw;
    a.nx = m.nx;
    a.ny = m.ny;
    a.z0 = m.z0;
    a.z1 = m.z1;
    a.separable = ax != nullptr;
    if (m.z1 <= m.z0) return PTV_OK;
    if (a.separable) {
        int *tx = tabs, *ty = tabs + m.nx, *tz = tabs + m.nx + m.ny;
        const double *q[3] = {ax, ay, az};
        const int nq[3] = {m.nx, m.ny, m.nz};
        int *t[3] = {tx, ty, tz};
        for (int d = 0; d < 3; ++d)
            hipLaunchKernelGGL(k_mask_axis_table, dim3((nq[d] + 255) / 256), dim3(256), 0, s, m.ra[d], m.rn[d],
                               m.flip[d], q[d], nq[d], t[d]);
        const int64_t lanes = (int64_t)((m.nx + 7) / 8) * m.ny * (m.z1 - m.z0);
        hipLaunchKernelGGL(k_mask_sample_sep, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, a,
                           (const int *)tx, (const int *)ty, (const int *)tz, out);
    } else {
        const int64_t nvox = (int64_t)(m.z1 - m.z0) * m.nx * m.ny;
        hipLaunchKernelGGL(k_mask_sample_pts, dim3((unsigned)((nvox + 255) / 256)), dim3(256), 0, s, a, px, py, pz,
                           nvox, out);
    }
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// ---------------------------------------------------------------------------
// boundary particles
//
// Mask bytes: bit 1 = "nonzero" (what binary_dilation sees), bit 0 = the low bit of the
// value (what `dilated & ~mask` keeps: for a bool mask `~mask` is logical not, for an
// integer mask numpy's bitwise not leaves only the low bit in `bool & ~int`).  For a bool
// mask both bits are the value itself (flag `is_bool`).
// Dilation (scipy.ndimage.binary_dilation, 6-connected cross, border_value=0): a voxel is
// set if it or one of its in-bounds face neighbours is set.  thickness - 1 iterations run
// as ping-pong passes; the last one is fused into the count / emit passes.
// ---------------------------------------------------------------------------
struct BoundaryArgs {
    int nx, ny, nz;
    int64_t nvox;
    int is_bool;           // mask bytes are 0/1 (bool)
    const uint8_t *mask;   // the caller's mask
    const uint8_t *grown;  // dilation after thickness-1 passes (0/1), NULL: use the mask itself
    int64_t step;          // sampling_step
    double lo[3], span[3], den[3];
};

__device__ __forceinline__ bool nonzero_at(const BoundaryArgs &a, const uint8_t *__restrict__ src, int64_t v) {
    const uint8_t b = src[v];
    return (src == a.mask && !a.is_bool) ? ((b >> 1) & 1) != 0 : b != 0;
}

__device__ __forceinline__ bool dilated_at(const BoundaryArgs &a, const uint8_t *__restrict__ src, int ix, int iy,
                                           int iz, int64_t v) {
    const int64_t sy = a.nx, sz = (int64_t)a.nx * a.ny;
    bool g = nonzero_at(a, src, v);
    g = g || (ix > 0 && nonzero_at(a, src, v - 1));
    g = g || (ix + 1 < a.nx && nonzero_at(a, src, v + 1));
    g = g || (iy > 0 && nonzero_at(a, src, v - sy));
    g = g || (iy + 1 < a.ny && nonzero_at(a, src, v + sy));
    g = g || (iz > 0 && nonzero_at(a, src, v - sz));
    g = g || (iz + 1 < a.nz && nonzero_at(a, src, v + sz));
    return g;
}

__global__ __launch_bounds__(256) void k_dilate(BoundaryArgs a, const uint8_t *__restrict__ src,
                                                uint8_t *__restrict__ dst) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= a.nvox) return;
    const int ix = (int)(v % a.nx);
    const int64_t r = v / a.nx;
    const int iy = (int)(r % a.ny), iz = (int)(r / a.ny);
    dst[v] = dilated_at(a, src, ix, iy, iz, v) ? 1 : 0;
}

constexpr int kBndThreads = 256;
constexpr int kBndWaves = kBndThreads / 64;
constexpr int kBndIters = 16;
constexpr int kBndChunk = kBndThreads * kBndIters;  // voxels per block

// boundary flag of voxel v (C-order linear index): solid (low bit clear) and within one
// face step of the (thickness-1 times dilated) fluid
template <typename IDX>
__device__ __forceinline__ bool boundary_at(const BoundaryArgs &a, const uint8_t *__restrict__ src, int64_t v) {
    if (v >= a.nvox) return false;
    if (a.mask[v] & 1) return false;
    const IDX nx = (IDX)a.nx, ny = (IDX)a.ny;
    const IDX r = (IDX)v / nx;
    const int ix = (int)((IDX)v - r * nx);
    const IDX iz = r / ny;
    const int iy = (int)(r - iz * ny);
    return dilated_at(a, src, ix, iy, (int)iz, v);
}

// Iteration j of a block covers voxels base + j*256 + [0, 256): one byte per lane, lane
// contiguous (coalesced), and (j, wave, lane) order is C order, so wave ballots ranked in
// that order give each voxel its position in np.where's output.
template <typename IDX>
__global__ __launch_bounds__(kBndThreads) void k_boundary_count(BoundaryArgs a, unsigned long long *__restrict__ counts) {
    const uint8_t *src = a.grown ? a.grown : a.mask;
    const int64_t base = (int64_t)blockIdx.x * kBndChunk + threadIdx.x;
    uint32_t c = 0;
#pragma unroll 4
    for (int j = 0; j < kBndIters; ++j) {
        const bool f = boundary_at<IDX>(a, src, base + j * kBndThreads);
        c += (uint32_t)__popcll(__ballot(f));
    }
    __shared__ uint32_t ws[kBndWaves];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBndWaves; ++w) t += ws[w];
        counts[blockIdx.x] = t;
    }
}
__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// single-block exclusive scan of the per-block counts (in place); total -> counts[nb]
__global__ __launch_bounds__(1024) void k_boundary_scan(unsigned long long *counts, int64_t nb) {
    __shared__ unsigned long long ws[16];
    __shared__ unsigned long long carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t base = 0; base < nb; base += 1024) {
        const int64_t i = base + threadIdx.x;
        const unsigned long long v = i < nb ? counts[i] : 0ull;
        const unsigned long long inc = wave_incl_scan_u64(v);
        if (lane == 63) ws[wid] = inc;
        __syncthreads();
        if (threadIdx.x < 64) {
            const unsigned long long t = threadIdx.x < 16 ? ws[threadIdx.x] : 0ull;
            const unsigned long long ti = wave_incl_scan_u64(t);
            if (threadIdx.x < 16) ws[threadIdx.x] = ti - t;
        }
        __syncthreads();
        const unsigned long long excl = carry + ws[wid] + inc - v;
        __syncthreads();
        if (i < nb) counts[i] = excl;
        if (threadIdx.x == 1023) carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[nb] = carry;
}

// physical coordinate of interpolator.py:278-280: lo + idx * (hi - 1 - lo) / (n - 1)
__device__ __forceinline__ double phys(const BoundaryArgs &a, int d, int idx) {
    return a.lo[d] + ((double)idx * a.span[d]) / a.den[d];
}

// every boundary voxel of rank r (C order) with r % step == 0 becomes record r / step
template <typename IDX>
__global__ __launch_bounds__(kBndThreads) void k_boundary_emit(BoundaryArgs a,
                                                               const unsigned long long *__restrict__ offsets,
                                                               double *__restrict__ ox, double *__restrict__ oy,
                                                               double *__restrict__ oz) {
    const uint8_t *src = a.grown ? a.grown : a.mask;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kBndChunk + threadIdx.x;
    __shared__ uint32_t pre[kBndIters * kBndWaves];
    uint32_t bits = 0;  // this lane's flags, bit j = iteration j
#pragma unroll 4
    for (int j = 0; j < kBndIters; ++j) {
        const bool f = boundary_at<IDX>(a, src, base + j * kBndThreads);
        bits |= (f ? 1u : 0u) << j;
        const unsigned long long b = __ballot(f);
        if (lane == 0) pre[j * kBndWaves + wid] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    if (wid == 0) {  // exclusive scan of the 64 (iteration, wave) counts, in C order
        const uint32_t v = pre[lane];
        uint32_t inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        pre[lane] = inc - v;
    }
    __syncthreads();
    if (bits == 0) return;
    const unsigned long long off = offsets[blockIdx.x];
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll 4
    for (int j = 0; j < kBndIters; ++j) {
        const bool f = (bits >> j) & 1u;
        const unsigned long long b = __ballot(f);
        if (!f) continue;
        const unsigned long long rank = off + pre[j * kBndWaves + wid] + (unsigned long long)__popcll(b & below);
        if (rank % (unsigned long long)a.step != 0) continue;
        const int64_t v = base + j * kBndThreads;
        const IDX nx = (IDX)a.nx, ny = (IDX)a.ny;
        const IDX r = (IDX)v / nx;
        const int ix = (int)((IDX)v - r * nx);
        const IDX iz = r / ny;
        const int iy = (int)(r - iz * ny);
        const int64_t o = (int64_t)(rank / (unsigned long long)a.step);
        ox[o] = phys(a, 0, ix);
        oy[o] = phys(a, 1, iy);
        oz[o] = phys(a, 2, (int)iz);
    }
}

// ---- rows of 16-aligned length (nx % 16 == 0): 16 consecutive x voxels per lane, every
// neighbour plane as one 16-byte load, the x neighbours by byte shifts inside the two u64
// words (SWAR); lane order is C order, so ranks come from a block scan of lane counts.
constexpr uint64_t kOnes = 0x0101010101010101ull;

__device__ __forceinline__ void nz16(const BoundaryArgs &a, const uint8_t *src, int64_t v, uint64_t &w0,
                                     uint64_t &w1) {
    const uint4 q = *reinterpret_cast<const uint4 *>(src + v);
    w0 = (uint64_t)q.x | ((uint64_t)q.y << 32);
    w1 = (uint64_t)q.z | ((uint64_t)q.w << 32);
    if (src == a.mask && !a.is_bool) {
        w0 >>= 1;
        w1 >>= 1;
    }
    w0 &= kOnes;
    w1 &= kOnes;
}

__device__ __forceinline__ uint32_t boundary16(const BoundaryArgs &a, int64_t v0, int &ix0, int &iy, int &iz) {
    const uint8_t *src = a.grown ? a.grown : a.mask;
    const int64_t r = v0 / a.nx;
    ix0 = (int)(v0 - r * a.nx);
    iy = (int)(r % a.ny);
    iz = (int)(r / a.ny);
    const int64_t sy = a.nx, sz = (int64_t)a.nx * a.ny;
    uint64_t c0, c1, t0, t1;
    nz16(a, src, v0, c0, c1);
    uint64_t d0 = c0, d1 = c1;
    if (iy > 0) { nz16(a, src, v0 - sy, t0, t1); d0 |= t0; d1 |= t1; }
    if (iy + 1 < a.ny) { nz16(a, src, v0 + sy, t0, t1); d0 |= t0; d1 |= t1; }
    if (iz > 0) { nz16(a, src, v0 - sz, t0, t1); d0 |= t0; d1 |= t1; }
    if (iz + 1 < a.nz) { nz16(a, src, v0 + sz, t0, t1); d0 |= t0; d1 |= t1; }
    const bool enc = src == a.mask && !a.is_bool;
    uint64_t lb = 0, rb = 0;
    if (ix0 > 0) lb = (uint64_t)((enc ? (src[v0 - 1] >> 1) : src[v0 - 1]) & 1);
    if (ix0 + 16 < a.nx) rb = (uint64_t)((enc ? (src[v0 + 16] >> 1) : src[v0 + 16]) & 1);
    d0 |= (c0 << 8) | lb;                // left neighbours
    d1 |= (c1 << 8) | (c0 >> 56);
    d0 |= (c0 >> 8) | (c1 << 56);        // right neighbours
    d1 |= (c1 >> 8) | (rb << 56);
    const uint4 m = *reinterpret_cast<const uint4 *>(a.mask + v0);
    const uint64_t l0 = ((uint64_t)m.x | ((uint64_t)m.y << 32)) & kOnes;
    const uint64_t l1 = ((uint64_t)m.z | ((uint64_t)m.w << 32)) & kOnes;
    const uint64_t f0 = d0 & ~l0 & kOnes, f1 = d1 & ~l1 & kOnes;
    constexpr uint64_t kGather = 0x0102040810204080ull;  // byte i (0/1) -> bit i of the top byte
    return (uint32_t)((f0 * kGather) >> 56) | ((uint32_t)((f1 * kGather) >> 56) << 8);
}

__global__ __launch_bounds__(kBndThreads) void k_boundary_count16(BoundaryArgs a,
                                                                  unsigned long long *__restrict__ counts) {
    const int64_t v0 = ((int64_t)blockIdx.x * kBndThreads + threadIdx.x) * 16;
    uint32_t c = 0;
    if (v0 < a.nvox) {
        int ix0, iy, iz;
        c = __popc(boundary16(a, v0, ix0, iy, iz));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ uint32_t ws[kBndWaves];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBndWaves; ++w) t += ws[w];
        counts[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kBndThreads) void k_boundary_emit16(BoundaryArgs a,
                                                                 const unsigned long long *__restrict__ offsets,
                                                                 double *__restrict__ ox, double *__restrict__ oy,
                                                                 double *__restrict__ oz) {
    const int64_t v0 = ((int64_t)blockIdx.x * kBndThreads + threadIdx.x) * 16;
    uint32_t bits = 0;
    int ix0 = 0, iy = 0, iz = 0;
    if (v0 < a.nvox) bits = boundary16(a, v0, ix0, iy, iz);
    const uint32_t c = __popc(bits);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    __shared__ uint32_t ws[kBndWaves];
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    unsigned long long rank = offsets[blockIdx.x] + inc - c;
    for (int w = 0; w < wid; ++w) rank += ws[w];
    const double y = phys(a, 1, iy), z = phys(a, 2, iz);
    while (bits) {
        const int j = __ffs(bits) - 1;
        bits &= bits - 1;
        if (rank % (unsigned long long)a.step == 0) {
            const int64_t o = (int64_t)(rank / (unsigned long long)a.step);
            ox[o] = phys(a, 0, ix0 + j);
            oy[o] = y;
            oz[o] = z;
        }
        ++rank;
    }
}

size_t boundary_blocks(int64_t nvox) { return (size_t)((nvox + kBndChunk - 1) / kBndChunk); }

int launch_boundary_count(const BoundaryLaunch &m, uint8_t *ping, uint8_t *pong, unsigned long long *counts,
                          const uint8_t **grown_out, hipStream_t s) {
    BoundaryArgs a{};
    a.nx = m.nx;
    a.ny = m.ny;
    a.nz = m.nz;
    a.nvox = (int64_t)m.nx * m.ny * m.nz;
    a.is_bool = m.is_bool;
    a.mask = m.mask;
    a.grown = nullptr;
    a.step = 1;
    const unsigned nb1 = (unsigned)((a.nvox + 255) / 256);
    const uint8_t *src = m.mask;
    uint8_t *bufs[2] = {ping, pong};
    for (int it = 1; it < m.thickness; ++it) {
        uint8_t *dst = bufs[(it - 1) & 1];
        hipLaunchKernelGGL(k_dilate, dim3(nb1), dim3(256), 0, s, a, src, dst);
        src = dst;
        a.grown = dst;  // later passes read plain 0/1 bytes
    }
    *grown_out = a.grown;
    const int64_t nb = (int64_t)boundary_blocks(a.nvox);
    if (a.nx % 16 == 0 && ((uintptr_t)a.mask & 15) == 0)
        hipLaunchKernelGGL(k_boundary_count16, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, counts);
    else if (a.nvox < (int64_t)1 << 32)
        hipLaunchKernelGGL(k_boundary_count<uint32_t>, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, counts);
    else
        hipLaunchKernelGGL(k_boundary_count<uint64_t>, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, counts);
    hipLaunchKernelGGL(k_boundary_scan, dim3(1), dim3(1024), 0, s, counts, nb);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_boundary_emit(const BoundaryLaunch &m, const uint8_t *grown, const unsigned long long *offsets,
                         double *ox, double *oy, double *oz, hipStream_t s) {
    BoundaryArgs a{};
    a.nx = m.nx;
    a.ny = m.ny;
    a.nz = m.nz;
    a.nvox = (int64_t)m.nx * m.ny * m.nz;
    a.is_bool = m.is_bool;
    a.mask = m.mask;
    a.grown = grown;
    a.step = m.step;
    for (int d = 0; d < 3; ++d) {
        a.lo[d] = m.lo[d];
        a.span[d] = m.span[d];
        a.den[d] = m.den[d];
    }
    const int64_t nb = (int64_t)boundary_blocks(a.nvox);
    if (a.nx % 16 == 0 && ((uintptr_t)a.mask & 15) == 0)
        hipLaunchKernelGGL(k_boundary_emit16, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, offsets, ox, oy, oz);
    else if (a.nvox < (int64_t)1 << 32)
        hipLaunchKernelGGL(k_boundary_emit<uint32_t>, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, offsets, ox, oy,
                           oz);
    else
        hipLaunchKernelGGL(k_boundary_emit<uint64_t>, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, offsets, ox, oy,
                           oz);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
