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

// one voxel per lane, x fastest: coalesced byte stores; the raw bytes are a gather through
// three tiny tables (rows of the raw mask are reused by every grid row that maps to them)
__global__ __launch_bounds__(256) void k_mask_sample_sep(MaskSampleArgs a, const int *__restrict__ tx,
                                                         const int *__restrict__ ty, const int *__restrict__ tz,
                                                         uint8_t *__restrict__ out) {
    const int ix = blockIdx.x * 256 + threadIdx.x;
    const int iy = blockIdx.y;
    const int iz = a.z0 + (int)blockIdx.z;
    if (ix >= a.nx) return;
    const int jx = tx[ix], jy = ty[iy], jz = tz[iz];
    uint8_t v = 0;
    if ((jx | jy | jz) >= 0) v = a.raw[((size_t)jz * a.rn[1] + jy) * a.rn[0] + jx];
    out[((size_t)(iz - a.z0) * a.ny + iy) * a.nx + ix] = v;
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
        if (m.ny > 65535 || m.z1 - m.z0 > 65535) {
            set_error("sample_mask: grid y/z extent above 65535");
            return PTV_E_UNSUPPORTED;
        }
        hipLaunchKernelGGL(k_mask_sample_sep, dim3((m.nx + 255) / 256, m.ny, m.z1 - m.z0), dim3(256), 0, s, a,
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
constexpr int kBndItems = 16;
constexpr int kBndChunk = kBndThreads * kBndItems;  // voxels per block

// 16 consecutive voxels per lane -> bit mask of boundary voxels
__device__ __forceinline__ uint32_t boundary_bits(const BoundaryArgs &a, int64_t base) {
    const uint8_t *src = a.grown ? a.grown : a.mask;
    uint32_t bits = 0;
    if (base >= a.nvox) return 0;
    int ix = (int)(base % a.nx);
    const int64_t r = base / a.nx;
    int iy = (int)(r % a.ny), iz = (int)(r / a.ny);
#pragma unroll 4
    for (int j = 0; j < kBndItems; ++j) {
        const int64_t v = base + j;
        if (v < a.nvox) {
            const bool low = (a.mask[v] & 1) != 0;
            if (!low && dilated_at(a, src, ix, iy, iz, v)) bits |= 1u << j;
        }
        if (++ix == a.nx) {
            ix = 0;
            if (++iy == a.ny) {
                iy = 0;
                ++iz;
            }
        }
    }
    return bits;
}

__global__ __launch_bounds__(kBndThreads) void k_boundary_count(BoundaryArgs a, unsigned long long *__restrict__ counts) {
    const int64_t base = (int64_t)blockIdx.x * kBndChunk + (int64_t)threadIdx.x * kBndItems;
    uint32_t c = __popc(boundary_bits(a, base));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ uint32_t ws[kBndThreads / 64];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBndThreads / 64; ++w) t += ws[w];
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
__global__ __launch_bounds__(kBndThreads) void k_boundary_emit(BoundaryArgs a,
                                                               const unsigned long long *__restrict__ offsets,
                                                               double *__restrict__ ox, double *__restrict__ oy,
                                                               double *__restrict__ oz) {
    const int64_t base = (int64_t)blockIdx.x * kBndChunk + (int64_t)threadIdx.x * kBndItems;
    uint32_t bits = boundary_bits(a, base);
    const unsigned long long c = __popc(bits);
    const unsigned long long inc = wave_incl_scan_u64(c);
    __shared__ unsigned long long ws[kBndThreads / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    unsigned long long rank = offsets[blockIdx.x] + inc - c;
    for (int w = 0; w < wid; ++w) rank += ws[w];
    while (bits) {
        const int j = __ffs(bits) - 1;
        bits &= bits - 1;
        if (rank % (unsigned long long)a.step == 0) {
            const int64_t v = base + j;
            const int ix = (int)(v % a.nx);
            const int64_t r = v / a.nx;
            const int iy = (int)(r % a.ny), iz = (int)(r / a.ny);
            const int64_t o = (int64_t)(rank / (unsigned long long)a.step);
            ox[o] = phys(a, 0, ix);
            oy[o] = phys(a, 1, iy);
            oz[o] = phys(a, 2, iz);
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
    hipLaunchKernelGGL(k_boundary_count, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, counts);
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
    hipLaunchKernelGGL(k_boundary_emit, dim3((unsigned)nb), dim3(kBndThreads), 0, s, a, offsets, ox, oy, oz);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
