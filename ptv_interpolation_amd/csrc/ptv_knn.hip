// ptv_knn.hip — host side of the k-NN launches (list-length dispatch, near-tie repair) and the
// lattice helper kernels; the k-NN kernel itself is ptv_knn_impl.hpp.
#include "ptv_knn_impl.hpp"

namespace ptv {

unsigned long long *g_dbg = nullptr;
long long g_dbg_cap = 0;  // records

// ---------------------------------------------------------------------------
// Count-only k-th distance UPPER bound (coarsest lattice).  One wave per grid point;
// the lanes share the cell rows of a ball of radius R around it and count only the
// particles of cells lying entirely inside the ball (at most the particles within R),
// so count(R) >= k proves d_k <= R.  R grows by 1.5x until that holds, then a
// bisection tightens it.  No particle record is read.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int count_inside(const CellGrid &g, const uint32_t *__restrict__ cstart, double qx,
                                            double qy, double qz, double R, int lane) {
    const double Ri = R - g.mg;  // conservative: shrink by the binning margin
    if (Ri <= 0.0) return 0;
    const double R2 = Ri * Ri;
    const int ry0 = clampi(floor((qy - Ri - g.o[1]) * g.ic[1]), g.nc[1]);
    const int ry1 = clampi(floor((qy + Ri - g.o[1]) * g.ic[1]), g.nc[1]);
    const int rz0 = clampi(floor((qz - Ri - g.o[2]) * g.ic[2]), g.nc[2]);
    const int rz1 = clampi(floor((qz + Ri - g.o[2]) * g.ic[2]), g.nc[2]);
    const int nyr = ry1 - ry0 + 1;
    const int nrows = nyr * (rz1 - rz0 + 1);
    int cnt = 0;
    for (int row = lane; row < nrows; row += 64) {
        const int ccy = ry0 + row % nyr, ccz = rz0 + row / nyr;
        const double y0 = g.o[1] + (double)ccy * g.cs[1], y1 = g.o[1] + (double)(ccy + 1) * g.cs[1];
        const double z0 = g.o[2] + (double)ccz * g.cs[2], z1 = g.o[2] + (double)(ccz + 1) * g.cs[2];
        const double fy = fmax(fabs(y0 - qy), fabs(y1 - qy)), fz = fmax(fabs(z0 - qz), fabs(z1 - qz));
        const double h2 = fy * fy + fz * fz;
        if (h2 >= R2) continue;
        const double rx = sqrt(R2 - h2) * (1.0 - 1e-12);
        // cells [a, b] whose x-extent lies inside [qx - rx, qx + rx]
        const int a = (int)ceil((qx - rx - g.o[0]) * g.ic[0] + 1e-9);
        const int b = (int)floor((qx + rx - g.o[0]) * g.ic[0] - 1e-9) - 1;
        const int aa = max(a, 0), bb = min(b, g.nc[0] - 1);
        if (aa > bb) continue;
        const long long base = ((long long)ccz * g.nc[1] + ccy) * g.nc[0];
        cnt += (int)(cstart[base + bb + 1] - cstart[base + aa]);
    }
    return group_reduce<0x3f>(cnt, OpAdd{});
}

__global__ __launch_bounds__(256) void k_count_bound(CellGrid g, const uint32_t *__restrict__ cstart,
                                                     const double *__restrict__ ax, const double *__restrict__ ay,
                                                     const double *__restrict__ az, int nx, int ny, int nz, int k,
                                                     double r0, double rall, double *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const long long gp = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gp >= (long long)nx * ny * nz) return;  // wave-uniform
    const int ix = (int)(gp % nx), iy = (int)((gp / nx) % ny), iz = (int)(gp / ((long long)nx * ny));
    const double qx = ax[ix], qy = ay[iy], qz = az[iz];
    double lo = 0.0, hi = r0;
    while (hi < rall && count_inside(g, cstart, qx, qy, qz, hi, lane) < k) {
        lo = hi;
        hi *= 1.5;
    }
    if (hi >= rall) {
        hi = rall;
    } else {
        for (int it = 0; it < 6; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (count_inside(g, cstart, qx, qy, qz, mid, lane) >= k)
                hi = mid;
            else
                lo = mid;
        }
    }
    if (lane == 0) out[gp] = hi * (1.0 + 1e-12) + g.mg;
}

int launch_count_bound(const CellGrid &g, const uint32_t *cstart, const double *ax, const double *ay,
                       const double *az, int nx, int ny, int nz, int k, double r0, double *out, hipStream_t s) {
    double diag2 = 0.0;
    for (int d = 0; d < 3; ++d) {
        const double e = g.cs[d] * g.nc[d];
        diag2 += e * e;
    }
    const double rall = sqrt(diag2) * (1.0 + 1e-9) + g.mg;
    const long long pts = (long long)nx * ny * nz;
    hipLaunchKernelGGL(k_count_bound, dim3((unsigned)((pts + 3) / 4)), dim3(256), 0, s, g, cstart, ax, ay, az, nx, ny,
                       nz, k, r0, rall, out);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

__global__ void k_subsample(const double *__restrict__ in, int n, int step, double *__restrict__ out, int nout) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nout) out[j] = in[min(j * step, n - 1)];
}

__global__ void k_subsample_levels(SubsampleBatch b, int step) {
    const int l = blockIdx.y / 3, d = blockIdx.y % 3;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= b.n[l][d]) return;
    long long idx = j;
    for (int lev = l; lev >= 0; --lev) idx = min(idx * step, (long long)(lev == 0 ? b.n0[d] : b.n[lev - 1][d]) - 1);
    b.out[l][d][j] = b.base[d][idx];
}

int launch_subsample_levels(const SubsampleBatch &b, int step, hipStream_t s) {
    if (b.nlev <= 0) return PTV_OK;
    if (b.nlev > kMaxSubsampleLevels) {
        set_error("lattice: too many levels");
        return PTV_E_ARG;
    }
    int mx = 1;
    for (int l = 0; l < b.nlev; ++l)
        for (int d = 0; d < 3; ++d) mx = std::max(mx, b.n[l][d]);
    hipLaunchKernelGGL(k_subsample_levels, dim3((mx + 255) / 256, 3 * b.nlev), dim3(256), 0, s, b, step);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

__global__ void k_concat3(const double *__restrict__ a, int na, const double *__restrict__ b, int nb,
                          const double *__restrict__ c, int nc, double *__restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < na) out[j] = a[j];
    else if (j < na + nb) out[j] = b[j - na];
    else if (j < na + nb + nc) out[j] = c[j - na - nb];
}

int launch_concat3(const double *a, int na, const double *b, int nb, const double *c, int nc, double *out,
                   hipStream_t s) {
    const int n = na + nb + nc;
    if (n <= 0) return PTV_OK;
    hipLaunchKernelGGL(k_concat3, dim3((n + 255) / 256), dim3(256), 0, s, a, na, b, nb, c, nc, out);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_subsample(const double *in, int n, int step, double *out, int nout, hipStream_t s) {
    hipLaunchKernelGGL(k_subsample, dim3((nout + 255) / 256), dim3(256), 0, s, in, n, step, out, nout);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// ---------------------------------------------------------------------------
// Exactness of a slab-culled particle set (ptv_knn_params.slab_halo).  For lattice point c
// and any voxel v of a lattice cell with corner c: d_k(v) <= D(c) + |v - c| <= D(c) +
// diag(c), and v's distance to the nearer slab face is >= m(c) - dz(c); a culled particle is
// farther than halo + that distance.  So halo >= D(c) + diag(c) + dz(c) - m(c) for every c
// proves every voxel's k nearest are inside the window (strictly nearer, so no tie either).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double axis_step(const double *a, int j, int n) {
    // the larger of the two lattice intervals adjacent to point j (0 on a one-point axis)
    const double l = j > 0 ? fabs(a[j] - a[j - 1]) : 0.0;
    const double r = j + 1 < n ? fabs(a[j + 1] - a[j]) : 0.0;
    return fmax(l, r);
}

__global__ __launch_bounds__(256) void k_halo_need(const double *__restrict__ lax, const double *__restrict__ lay,
                                                   const double *__restrict__ laz, int nx, int ny, int nz,
                                                   const double *__restrict__ dk, const double *__restrict__ win,
                                                   double mg, unsigned long long *__restrict__ out) {
    const long long np = (long long)nx * ny * nz;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    double need = 0.0;
    if (i < np) {
        const int ix = (int)(i % nx), iy = (int)((i / nx) % ny), iz = (int)(i / ((long long)nx * ny));
        const double sx = axis_step(lax, ix, nx), sy = axis_step(lay, iy, ny), sz = axis_step(laz, iz, nz);
        const double diag = sqrt((sx * sx + sy * sy) + sz * sz);
        const double zc = laz[iz];
        const double m = fmax(fmin(zc - win[2], win[3] - zc), 0.0);
        const double D = dk[i];
        // rounding margin: relative 1e-9 on the distance terms plus the binning margin
        need = fmax(((D + diag + sz) * (1.0 + 1e-9) + mg) - m * (1.0 - 1e-12), 0.0);
        if (!(need < INFINITY)) need = INFINITY;
    }
    need = group_reduce<0x3f>(need, OpMax{});
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(need));
}

int launch_halo_need(const double *lax, const double *lay, const double *laz, int nx, int ny, int nz,
                     const double *dk, const double *win, double mg, unsigned long long *out, hipStream_t s) {
    const long long np = (long long)nx * ny * nz;
    PTV_HIP(hipMemsetAsync(out, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_halo_need, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, lax, lay, laz, nx, ny, nz, dk,
                       win, mg, out);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// ---------------------------------------------------------------------------
// Longest-first block order of a lattice-level launch.  k_block_keys (one thread per block,
// many workgroups) computes each block's key once, and their maximum; k_block_order (one
// workgroup of 1024 threads) buckets the keys in LDS, scans, and places the blocks by LDS atomics
// (the order inside a bucket is arbitrary, which changes nothing but the dispatch order).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_block_keys(const double *__restrict__ dkc, int cnx, int cny, int cnz,
                                                    int ntxb, int nty, int nblocks, double *__restrict__ keys,
                                                    unsigned long long *__restrict__ kmax) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    double D = 0.0;
    if (b < nblocks) {
        // block b: tiles (bx*4 .. bx*4+3, ty, tz) = points x [16 bx, 16 bx + 15], y [4 ty, 4 ty + 3],
        // z [4 tz, 4 tz + 3]; coarser point j sits at point 4 j (kLatticeStep), so the block lies in
        // the coarser cells spanned by x [4 bx, 4 bx + 4], y [ty, ty + 1], z [tz, tz + 1]
        const int bx = b % ntxb, rr = b / ntxb, ty = rr % nty, tz = rr / nty;
        for (int z = tz; z <= tz + 1; ++z)
            for (int y = ty; y <= ty + 1; ++y)
                for (int x = 4 * bx; x <= 4 * bx + 4; ++x)
                    D = fmax(D, dkc[((size_t)min(z, cnz - 1) * cny + min(y, cny - 1)) * cnx + min(x, cnx - 1)]);
        keys[b] = D;
    }
    // non-negative doubles (and +inf) order as their bit patterns
    const double m = group_reduce<0x3f>(D, OpMax{});
    if ((threadIdx.x & 63) == 0) atomicMax(kmax, (unsigned long long)__double_as_longlong(m));
}

__global__ __launch_bounds__(1024) void k_block_order(const double *__restrict__ keys,
                                                      const unsigned long long *__restrict__ kmax, int nblocks,
                                                      double inv_unit, int *__restrict__ order) {
    __shared__ int cnt[256];
    __shared__ int base[256];
    // buckets of the largest key / 256 (a fixed unit saturated: at 512^3 every block near a sphere
    // centre fell into the top bucket, in arbitrary order, and the slowest void tile could start last)
    const double mx = __longlong_as_double((long long)*kmax);
    const double scale = mx > 0.0 && mx < INFINITY ? 255.99 / mx : inv_unit;
    auto bucket = [&](int b) -> int {
        const double q = keys[b] * scale;
        return 255 - (q < 255.0 ? (int)q : 255);  // descending bound -> ascending bucket
    };
    for (int i = threadIdx.x; i < 256; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    for (int b = threadIdx.x; b < nblocks; b += blockDim.x) atomicAdd(&cnt[bucket(b)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int i = 0; i < 256; ++i) {
            base[i] = run;
            run += cnt[i];
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nblocks; b += blockDim.x) order[atomicAdd(&base[bucket(b)], 1)] = b;
}

int launch_block_order(const double *dk_coarse, const int nc[3], int nx, int ny, int nz, double unit, int *order,
                       double *keys, hipStream_t s) {
    const int ntxb = ((nx + 3) / 4 + 3) / 4, nty = (ny + 3) / 4, ntz = (nz + 3) / 4;
    const long long nblocks = (long long)ntxb * nty * ntz;
    if (nblocks > 0x7fffffffLL || !(unit > 0.0)) {
        set_error("lattice block order: bad launch shape");
        return PTV_E_ARG;
    }
    // keys[nblocks] holds the maximum's bits
    unsigned long long *kmax = reinterpret_cast<unsigned long long *>(keys + nblocks);
    PTV_HIP(hipMemsetAsync(kmax, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_block_keys, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, s, dk_coarse, nc[0],
                       nc[1], nc[2], ntxb, nty, (int)nblocks, keys, kmax);
    PTV_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_block_order, dim3(1), dim3(1024), 0, s, keys, kmax, (int)nblocks, 8.0 / unit, order);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// list lengths: exact (d2, slot) pair lists serve k <= 12 (length >= k); packed-key lists
// serve 13 <= k <= 127 (length >= k + 1: the near-tie slot)
static const int kKmaxExact[] = {1, 4, 8, 12};
static const int kKmaxKeys[] = {16, 24, 32, 40, 48, 56, 64, 96, 128};

int kmax_for(int k) {
    if (k < 1) return 0;
    for (int km : kKmaxExact)
        if (k <= km) return km;
    for (int km : kKmaxKeys)
        if (k + 1 <= km) return km;
    return 0;
}

// the list-length instantiations live in ptv_knn_k*.hip (parallel compilation)
#define PTV_KNN_EXTERN(K, E)                                                                           \
    extern template void launch_t<K, E>(dim3, hipStream_t, const KnnKernelArgs &, const Binned &, const double *, \
                                        const double *, const double *, const double *, const double *,        \
                                        const double *, const uint8_t *, double *, double *, double *);
PTV_KNN_EXTERN(1, false)
PTV_KNN_EXTERN(4, false)
PTV_KNN_EXTERN(8, false)
PTV_KNN_EXTERN(12, false)
PTV_KNN_EXTERN(16, false)
PTV_KNN_EXTERN(16, true)
PTV_KNN_EXTERN(24, false)
PTV_KNN_EXTERN(24, true)
PTV_KNN_EXTERN(32, false)
PTV_KNN_EXTERN(32, true)
PTV_KNN_EXTERN(40, false)
PTV_KNN_EXTERN(40, true)
PTV_KNN_EXTERN(48, false)
PTV_KNN_EXTERN(48, true)
PTV_KNN_EXTERN(56, false)
PTV_KNN_EXTERN(56, true)
PTV_KNN_EXTERN(64, false)
PTV_KNN_EXTERN(64, true)
PTV_KNN_EXTERN(96, false)
PTV_KNN_EXTERN(96, true)
PTV_KNN_EXTERN(128, false)
PTV_KNN_EXTERN(128, true)
#undef PTV_KNN_EXTERN

static int launch_kmax(int km, bool exact, dim3 grid, hipStream_t s, const KnnKernelArgs &ka, const Binned &b,
                       const double *ax, const double *ay, const double *az, const double *qx, const double *qy,
                       const double *qz, const uint8_t *mask, double *U, double *V, double *W) {
    switch (km) {
#define PTV_CASE(K)                                                                          \
    case K:                                                                                  \
        if constexpr (K >= 16) {                                                             \
            if (exact) {                                                                     \
                launch_t<K, true>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);    \
                break;                                                                       \
            }                                                                                \
        }                                                                                    \
        launch_t<K, false>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);           \
        break;
        PTV_CASE(1)
        PTV_CASE(4)
        PTV_CASE(8)
        PTV_CASE(12)
        PTV_CASE(16)
        PTV_CASE(24)
        PTV_CASE(32)
        PTV_CASE(40)
        PTV_CASE(48)
        PTV_CASE(56)
        PTV_CASE(64)
        PTV_CASE(96)
        PTV_CASE(128)
#undef PTV_CASE
        default:
            set_error("no k-NN list of length " + std::to_string(km));
            return PTV_E_UNSUPPORTED;
    }
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

static dim3 grid_for(long long nblocks) {
    // a dispatch holds < 2^32 work-items per dimension: above 2^23 blocks of 256 the grid is
    // 2-D, x a multiple of 8 so that the linear order still deals blocks round-robin over XCDs
    constexpr long long kMaxGridX = 1LL << 23;
    return dim3(nblocks <= kMaxGridX ? (unsigned)nblocks : (unsigned)kMaxGridX,
                nblocks <= kMaxGridX ? 1u : (unsigned)((nblocks + kMaxGridX - 1) / kMaxGridX));
}

int launch_knn(const KnnLaunch &a, const Binned &b, const double *ax, const double *ay, const double *az,
               const double *qx, const double *qy, const double *qz, const uint8_t *mask, double *U, double *V,
               double *W, hipStream_t s) {
    const int km = a.mode == kModeRadius ? 4 : kmax_for(a.k);
    if (km == 0) {
        set_error("k=" + std::to_string(a.k) + " exceeds the GPU k-NN list limit (127)");
        return PTV_E_UNSUPPORTED;
    }
    const bool keys = km >= 16;
    if (a.z1 <= a.z0) return PTV_OK;
    KnnKernelArgs ka;
    ka.cg = a.cg;
    ka.nx = a.nx;
    ka.ny = a.ny;
    ka.nz = a.nz;
    ka.z0 = a.z0;
    ka.z1 = a.z1;
    ka.ntx = (a.nx + 3) / 4;
    ka.nty = (a.ny + 3) / 4;
    ka.ntz = (a.z1 - a.z0 + 3) / 4;
    ka.ntxb = (ka.ntx + 3) / 4;
    ka.separable = a.separable;
    ka.method = a.method;
    ka.k = a.k;
    ka.kpad = km - a.k - (keys ? 1 : 0);
    ka.power = a.power;
    ka.eps = a.eps;
    ka.flags = a.flags;
    ka.r0 = a.r0;
    ka.mode = a.mode;
    ka.cb = a.cb;
    ka.kd_recs = a.kd_recs;
    ka.lz0 = a.lz0 < 0 ? a.z0 : a.lz0;
    ka.slots = a.slots;
    ka.radius = a.radius;
    ka.fe = a.fe;
    if (a.mode == kModeFilter && (a.fe.q_orig == nullptr || a.fe.inv == nullptr || a.fe.spd == nullptr ||
                                  a.fe.keep == nullptr || a.k < 2)) {
        set_error("filter-mode k-NN launch needs its epilogue buffers and k + 1 >= 2");
        return PTV_E_ARG;
    }
    if (a.mode == kModeRadius && !(a.radius > 0.0 && a.radius < INFINITY)) {
        set_error("radius search needs a positive finite radius");
        return PTV_E_ARG;
    }
    ka.order = a.order;
    ka.gate = a.gate;
    ka.gate_halo = a.gate_halo;
    // union seeds (k > 8): the first ~3/4 of each corner's list; the 8 corners' union still holds
    // k distinct particles (else the lattice bound): 512^3 / 5M same-box, IDW k = 50 115.4 ->
    // 114.1 ms at 36 of 50, Sibson k = 30 58.4 -> 57.5 ms at 22 of 30
    ka.seed_n = a.k > 8 ? (3 * a.k + 3) / 4 : a.k;
    if (const char *e = dev_knob("PTV_SEED_N")) ka.seed_n = std::max(1, std::min(a.k, std::atoi(e)));  // dev knob
    if (a.mode == kModeSlots && (a.slots == nullptr || (a.z0 - ka.lz0) % 4 != 0)) {
        set_error("slot-mode k-NN launch needs an output buffer and a tile-aligned first plane");
        return PTV_E_ARG;
    }
    double diag2 = 0.0;
    for (int d = 0; d < 3; ++d) {
        const double e = a.cg.cs[d] * a.cg.nc[d];
        diag2 += e * e;
    }
    ka.rall = sqrt(diag2) * (1.0 + 1e-9) + a.cg.mg;
    const long long nblocks = (long long)ka.ntxb * ka.nty * ka.ntz;
    if (nblocks > 0x7fffffffLL || (keys && nblocks >= (1LL << 30))) {
        set_error("grid too large for one launch");
        return PTV_E_ARG;
    }
    ka.nblocks = (int)nblocks;
    // packed keys: slot bits B (the largest slot is n - 1) and the key -> d2 bound factor
    int B = 1;
    while (B < 31 && (1LL << B) < b.n) ++B;
    ka.smask = (uint32_t)((1ULL << B) - 1ULL);
    ka.kscale = 1.0 + std::ldexp(1.0, B - 51);
    ka.rep_cnt = nullptr;
    ka.rep_list = nullptr;
    ka.rep_cap = 0;
    ka.tiles = nullptr;
    ka.ntiles = 0;
    ka.split = 0;
    ka.split_tiles = 0;
    ka.split_out = nullptr;
    ka.split_lb = 0;
    ka.order_skip = 0;
    if (a.mode == kModeKDist && a.split > 1 && a.split_blocks > 0 && a.order != nullptr && a.split_out != nullptr) {
        // lattice level: the first split_blocks blocks of the longest-first order (the void tiles)
        // with `split` waves per tile, the rest of the order as usual, then the merge of the split
        // tiles' partial lists (k_kdist_merge); parts that find no bound leave their lists cleared
        const int nsb = (int)std::min<long long>(a.split_blocks, nblocks);
        KnnKernelArgs ks = ka;
        ks.split = a.split;
        ks.split_tiles = nsb * 4;
        ks.split_out = a.split_out;
        PTV_HIP(hipMemsetAsync(a.split_out, 0xff, kdist_split_slots(a.split, nsb, km) * sizeof(uint32_t), s));
        const long long sblocks = ((long long)ks.split_tiles * a.split + 3) / 4;
        // one launch: the split waves first (the void tiles lead the longest-first order), then
        // the rest of the order as ordinary blocks (two launches serialised the split part)
        const long long total = sblocks + (nblocks - nsb);
        if (total > 0x7fffffffLL) {
            set_error("split lattice launch too large");
            return PTV_E_ARG;
        }
        ks.nblocks = (int)total;
        ks.split_lb = (int)sblocks;
        ks.order_skip = (int)(nsb - sblocks);
        int rc = launch_kmax(km, false, grid_for(total), s, ks, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
        if (rc != PTV_OK) return rc;
        ks.mode = kModeKDistMerge;
        return launch_kmax(km, false, grid_for(nsb), s, ks, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
    }
    const bool repair = keys && a.mode != kModeKDist && a.mode != kModeRadius;
    if (repair) {
        if (a.rep_cnt == nullptr || a.rep_list == nullptr || a.h_rep == nullptr) {
            set_error("key-list k-NN launch needs its near-tie repair buffers");
            return PTV_E_ARG;
        }
        ka.rep_cnt = a.rep_cnt;
        ka.rep_list = a.rep_list;
        ka.rep_cap = a.rep_cap;
        PTV_HIP(hipMemsetAsync(a.rep_cnt, 0, sizeof(unsigned int), s));
    }
    const int rc = launch_kmax(km, false, grid_for(nblocks), s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
    if (rc != PTV_OK || !repair) return rc;
    // near-tie repair: the listed tiles again with the exact (d2, slot) pair lists
    PTV_HIP(hipMemcpyAsync(a.h_rep, a.rep_cnt, sizeof(unsigned int), hipMemcpyDeviceToHost, s));
    PTV_HIP(hipStreamSynchronize(s));
    const unsigned int nrep = *a.h_rep;
    if (a.n_repair != nullptr) *a.n_repair += nrep;
    if (nrep == 0) return PTV_OK;
    KnnKernelArgs kr = ka;
    kr.kpad = km - a.k;
    kr.rep_cnt = nullptr;
    if ((long long)nrep <= (long long)a.rep_cap) {
        kr.tiles = a.rep_list;
        kr.ntiles = (int)nrep;
        kr.nblocks = (int)((nrep + 3) / 4);
        return launch_kmax(km, true, grid_for(kr.nblocks), s, kr, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
    }
    // more than the list holds: the whole launch again
    return launch_kmax(km, true, grid_for(nblocks), s, kr, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
}

}  // namespace ptv
