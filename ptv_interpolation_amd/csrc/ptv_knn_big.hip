// ptv_knn_big.hip — exact k-NN for k beyond the register lists (IDW / Sibson k >= 128, the outlier
// filter's k >= 127): the reference's KDTree.query takes any k (interpolator.py:97, :139;
// filtering.py:26), so these k take a separate, list-free path instead of PTV_E_UNSUPPORTED.
//
// Per chunk of queries (voxels of a slab, or particles for the filter):
//   1. k_big_bound (one thread per query): a radius R whose ball around the query certainly holds
//      k particles -- the binning cells lying entirely inside the ball of radius R' < R hold >= k
//      of them -- grown from the density radius; and ub = the particles of every cell the ball of
//      radius R + mg touches (the gather below visits exactly those cells).
//   2. inclusive scan of ub (hipCUB); the host splits the chunk into sub-chunks whose candidate
//      lists fit the buffers.
//   3. k_big_gather (one wave per query): the candidates with d2 <= R'^2 of the touched cells, in
//      ascending slot order (cell rows in linear order, ordered wave compaction), as (d2 bits, slot)
//      pairs -- every particle at or below the k-th distance is among them.
//   4. hipCUB segmented radix sort of each query's pairs by d2 (stable: equal d2 keep slot order).
//   5. the epilogue on the first k (k + 1 for the filter) entries of each sorted segment, in the
//      reference's arithmetic: IDW interpolator.py:141-153, Sibson :102-122 (numpy's pairwise sums,
//      including its recursive split past 128 terms), the filter's median / MAD filtering.py:20-51
//      (two more segmented sorts for the medians).
// Correctness over speed: k >= 128 is a rare configuration (the register-list kernels serve k <= 127).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "ptv_api.h"
#include "ptv_kernels.hpp"
#include "ptv_knn_big.hpp"

namespace ptv {

namespace {

__device__ __forceinline__ int big_clampi(double f, int n) {
    return f < 0.0 ? 0 : (f >= (double)(n - 1) ? n - 1 : (int)f);
}

// distance between coordinate q and cell c of an axis (0 inside)
__device__ __forceinline__ double big_gap(int c, double o, double cs, double q) {
    const double c0 = o + (double)c * cs, c1 = o + (double)(c + 1) * cs;
    return fmax(fmax(c0 - q, q - c1), 0.0);
}

// distance between coordinate q and the far side of cell c
__device__ __forceinline__ double big_far(int c, double o, double cs, double q) {
    const double c0 = o + (double)c * cs, c1 = o + (double)(c + 1) * cs;
    return fmax(fabs(c0 - q), fabs(c1 - q));
}

// the query's coordinates; active = computes an output (grid queries: inside the fluid mask)
__device__ __forceinline__ void big_query(const BigQueries &q, int64_t i, double &x, double &y, double &z, bool &active) {
    active = true;
    if (q.particles) {  // the filter: query i = particle i (original order)
        x = q.px[i];
        y = q.py[i];
        z = q.pz[i];
        return;
    }
    const int64_t plane = (int64_t)q.nx * q.ny;
    const int64_t iz = q.z0 + i / plane, r = i - (i / plane) * plane;
    const int64_t iy = r / q.nx, ix = r - iy * q.nx;
    const size_t vfull = ((size_t)iz * q.ny + iy) * q.nx + ix;
    if (q.ax != nullptr) {
        x = q.ax[ix];
        y = q.ay[iy];
        z = q.az[iz];
    } else {
        x = q.px[vfull];
        y = q.py[vfull];
        z = q.pz[vfull];
    }
    if (q.mask != nullptr) active = q.mask[vfull] != 0;
}

// the cells a ball of radius R around (x, y, z) touches: rows [y0, y1] x [z0, z1], each row's x-run
struct BallRows {
    int y0, z0, ny, nrows;
};
__device__ __forceinline__ BallRows ball_rows(const CellGrid &g, double y, double z, double R) {
    BallRows b;
    b.y0 = big_clampi(floor((y - R - g.o[1]) * g.ic[1]), g.nc[1]);
    const int y1 = big_clampi(floor((y + R - g.o[1]) * g.ic[1]), g.nc[1]);
    b.z0 = big_clampi(floor((z - R - g.o[2]) * g.ic[2]), g.nc[2]);
    const int z1 = big_clampi(floor((z + R - g.o[2]) * g.ic[2]), g.nc[2]);
    b.ny = y1 - b.y0 + 1;
    b.nrows = b.ny * (z1 - b.z0 + 1);
    return b;
}
// row r of the ball's rows: its particle range [start, start + count) (count 0 if untouched)
__device__ __forceinline__ void ball_row_run(const CellGrid &g, const uint32_t *__restrict__ cstart, const BallRows &b,
                                             int r, double x, double y, double z, double R, uint32_t &start,
                                             uint32_t &count) {
    const int cy = b.y0 + r % b.ny, cz = b.z0 + r / b.ny;
    const double gy = big_gap(cy, g.o[1], g.cs[1], y), gz = big_gap(cz, g.o[2], g.cs[2], z);
    const double h2 = gy * gy + gz * gz, R2 = R * R;
    start = 0;
    count = 0;
    if (h2 > R2) return;
    const double rx = sqrt(R2 - h2) * (1.0 + 1e-12);
    const int a = big_clampi(floor((x - rx - g.o[0]) * g.ic[0]), g.nc[0]);
    const int e = big_clampi(floor((x + rx - g.o[0]) * g.ic[0]), g.nc[0]);
    const uint32_t *rp = cstart + ((long long)cz * g.nc[1] + cy) * g.nc[0];
    start = rp[a];
    count = rp[e + 1] - start;
}

// particles in the cells lying entirely inside the ball of radius Ri (each such particle is within
// Ri + the binning margin of the query)
__device__ uint64_t count_inside(const CellGrid &g, const uint32_t *__restrict__ cstart, double x, double y, double z,
                                 double Ri) {
    if (!(Ri > 0.0)) return 0;
    const BallRows b = ball_rows(g, y, z, Ri);
    uint64_t cnt = 0;
    for (int r = 0; r < b.nrows; ++r) {
        const int cy = b.y0 + r % b.ny, cz = b.z0 + r / b.ny;
        const double fy = big_far(cy, g.o[1], g.cs[1], y), fz = big_far(cz, g.o[2], g.cs[2], z);
        const double h2 = fy * fy + fz * fz;
        if (h2 >= Ri * Ri) continue;
        const double hx = sqrt(Ri * Ri - h2) * (1.0 - 1e-12);
        // cells c with o + c cs >= x - hx and o + (c + 1) cs <= x + hx
        int a = (int)fmax(ceil((x - hx - g.o[0]) * g.ic[0]), 0.0);
        int e = (int)fmin(floor((x + hx - g.o[0]) * g.ic[0]) - 1.0, (double)(g.nc[0] - 1));
        if (a > e) continue;
        const uint32_t *rp = cstart + ((long long)cz * g.nc[1] + cy) * g.nc[0];
        cnt += rp[e + 1] - rp[a];
    }
    return cnt;
}

__global__ __launch_bounds__(256) void k_big_bound(BigQueries q, CellGrid g, const uint32_t *__restrict__ cstart,
                                                    int k, double r0, double rall, int64_t q0, int64_t nq,
                                                    double *__restrict__ R, unsigned long long *__restrict__ ub) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    double x, y, z;
    bool active;
    big_query(q, q0 + i, x, y, z, active);
    if (!active) {
        R[i] = -1.0;
        ub[i] = 0;
        return;
    }
    double Rc = fmin(r0, rall);
    for (int it = 0; it < 4096; ++it) {
        // shrunk for the binning margin (a binned particle lies within mg of its cell) and rounding
        const double Ri = Rc * (1.0 - 1e-12) - 2.0 * g.mg;
        const uint64_t c = count_inside(g, cstart, x, y, z, Ri);
        if (c >= (uint64_t)k || Rc >= rall) break;
        double f = c > 0 ? cbrt((double)k / (double)c) * 1.05 : 2.0;
        f = fmin(fmax(f, 1.1), 2.0);
        Rc = fmin(Rc * f, rall);
    }
    R[i] = Rc;
    const double Rg = Rc + g.mg;
    const BallRows b = ball_rows(g, y, z, Rg);
    uint64_t n = 0;
    for (int r = 0; r < b.nrows; ++r) {
        uint32_t s, c;
        ball_row_run(g, cstart, b, r, x, y, z, Rg, s, c);
        n += c;
    }
    ub[i] = n;
}

// one wave per query: the candidates with d2 <= (R + mg)^2 (1 + 1e-12), ascending slot order
__global__ __launch_bounds__(256) void k_big_gather(BigQueries q, CellGrid g, const double4 *__restrict__ prec,
                                                     const uint32_t *__restrict__ cstart, const double *__restrict__ R,
                                                     const unsigned long long *__restrict__ incl, int64_t q0,
                                                     int64_t qa, int64_t nq, unsigned long long *__restrict__ keys,
                                                     uint32_t *__restrict__ vals, int *__restrict__ seg_b,
                                                     int *__restrict__ seg_e) {
    __shared__ uint32_t lds_excl[4][64];
    __shared__ uint32_t lds_start[4][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * 4 + wid;  // query of the sub-chunk
    if (j >= nq) return;
    const int64_t i = qa + j;  // query of the chunk
    const unsigned long long base = qa > 0 ? incl[qa - 1] : 0ull;
    const long long off = (long long)((i > 0 ? incl[i - 1] : 0ull) - base);
    const double Rq = R[i];
    if (!(Rq >= 0.0)) {
        if (lane == 0) {
            seg_b[j] = (int)off;
            seg_e[j] = (int)off;
        }
        return;
    }
    double x, y, z;
    bool active;
    big_query(q, q0 + i, x, y, z, active);
    const double Rg = Rq + g.mg;
    const double thr = Rg * Rg * (1.0 + 1e-12);
    const BallRows b = ball_rows(g, y, z, Rg);
    uint32_t *ex = lds_excl[wid], *st = lds_start[wid];
    long long pos = 0;
    for (int rb = 0; rb < b.nrows; rb += 64) {
        uint32_t s = 0, c = 0;
        if (rb + lane < b.nrows) ball_row_run(g, cstart, b, rb + lane, x, y, z, Rg, s, c);
        // inclusive prefix sum of the run lengths over the wave
        uint32_t inc = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        const uint32_t total = __shfl(inc, 63, 64);
        ex[lane] = inc - c;
        st[lane] = s;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t src = 0; src < total; src += 64) {
            const uint32_t t = src + (uint32_t)lane;
            bool keep = false;
            uint32_t slot = 0;
            double e2 = 0.0;
            if (t < total) {
                // the last run whose first candidate is <= t (runs of length 0 share the next one's start)
                int lo = 0;
#pragma unroll
                for (int h = 32; h > 0; h >>= 1)
                    if (lo + h < 64 && ex[lo + h] <= t) lo += h;
                slot = st[lo] + (t - ex[lo]);
                const double4 p = prec[slot];
                const double dx = x - p.x, dy = y - p.y, dz = z - p.z;
                e2 = (dx * dx + dy * dy) + dz * dz;
                keep = e2 <= thr;
            }
            const unsigned long long m = __builtin_amdgcn_ballot_w64(keep);
            if (keep) {
                const long long r = off + pos + (long long)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                keys[r] = (unsigned long long)__double_as_longlong(e2);
                vals[r] = slot;
            }
            pos += __builtin_popcountll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) {
        seg_b[j] = (int)off;
        seg_e[j] = (int)(off + pos);
    }
}

// numpy's pairwise sum of f(0 .. n): n < 8 sequential from 0.0; n <= 128 eight accumulators, their
// tree, then the n % 8 tail; larger n split at n / 2 rounded down to a multiple of 8, recursively
// (the reduction adds the identity 0.0 first, which changes nothing for these sums)
template <class F>
__device__ double pw_leaf(const F &f, long long b, long long n) {
    if (n < 8) {
        double r = 0.0;
        for (long long i = 0; i < n; ++i) r += f(b + i);
        return r;
    }
    double r0 = f(b), r1 = f(b + 1), r2 = f(b + 2), r3 = f(b + 3), r4 = f(b + 4), r5 = f(b + 5), r6 = f(b + 6),
           r7 = f(b + 7);
    const long long stop = n - (n & 7);
    for (long long i = 8; i < stop; i += 8) {
        r0 += f(b + i);
        r1 += f(b + i + 1);
        r2 += f(b + i + 2);
        r3 += f(b + i + 3);
        r4 += f(b + i + 4);
        r5 += f(b + i + 5);
        r6 += f(b + i + 6);
        r7 += f(b + i + 7);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (long long i = stop; i < n; ++i) res += f(b + i);
    return res;
}
template <class F>
__device__ double pw_sum(const F &f, long long n) {
    struct Frame {
        long long b, n;
        int st;
        double left;
    };
    Frame s[48];  // depth <= log2(n / 64) + 1
    int sp = 0;
    s[0] = Frame{0, n, 0, 0.0};
    double ret = 0.0;
    while (true) {
        Frame &t = s[sp];
        if (t.n <= 128) {
            ret = pw_leaf(f, t.b, t.n);
        } else if (t.st == 0) {
            long long n2 = t.n / 2;
            n2 -= n2 % 8;
            t.st = 1;
            s[sp + 1] = Frame{t.b, n2, 0, 0.0};
            ++sp;
            continue;
        } else if (t.st == 1) {
            long long n2 = t.n / 2;
            n2 -= n2 % 8;
            t.left = ret;
            t.st = 2;
            s[sp + 1] = Frame{t.b + n2, t.n - n2, 0, 0.0};
            ++sp;
            continue;
        } else {
            ret = t.left + ret;
        }
        if (sp == 0) return ret;
        --sp;
    }
}

__device__ __forceinline__ double big_pow(double d, double p) {
    if (p == 2.0) return d * d;
    if (p == 1.0) return d;
    if (p == 0.5) return sqrt(d);
    if (p == -1.0) return 1.0 / d;
    return pow(d, p);
}

__device__ __forceinline__ double big_nan_to_num(double v) {
    if (v != v) return 0.0;
    if (v == INFINITY) return DBL_MAX;
    if (v == -INFINITY) return -DBL_MAX;
    return v;
}

// IDW / Sibson on the first k entries of each query's sorted segment; w (the unsorted key buffer,
// free after the sort) holds the per-neighbour weights, ds (the sorted keys, in place) the distances
__global__ __launch_bounds__(256) void k_big_interp(BigQueries q, const double4 *__restrict__ pval,
                                                     unsigned long long *__restrict__ ds,
                                                     const uint32_t *__restrict__ sv, double *__restrict__ w,
                                                     const int *__restrict__ seg_b, const int *__restrict__ seg_e,
                                                     int64_t q0, int64_t nq, int k, int method, double power,
                                                     double eps, uint32_t flags, double *__restrict__ U,
                                                     double *__restrict__ V, double *__restrict__ W) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nq) return;
    const int64_t vo = q0 + j;  // slab-relative voxel = output index
    const long long b = seg_b[j];
    double out[3] = {0.0, 0.0, 0.0};
    if (seg_e[j] - b >= k) {
        double *d = reinterpret_cast<double *>(ds) + b;
        const uint32_t *sl = sv + b;
        double *wb = w + b;
        for (int t = 0; t < k; ++t) d[t] = sqrt(__longlong_as_double((long long)ds[b + t]));
        if (method == PTV_METHOD_SIBSON) {
            // interpolator.py:106-116
            for (int t = 0; t < k; ++t) wb[t] = 1.0 / (d[t] + eps);
            const double s_inv = pw_sum([&](long long t) { return wb[t]; }, k);
            const double mean = pw_sum([&](long long t) { return d[t]; }, k) / (double)k;
            const double var = pw_sum([&](long long t) {
                const double c = d[t] - mean;
                return c * c;
            }, k) / (double)k;
            const double den = sqrt(var) + eps;
            for (int t = 0; t < k; ++t) wb[t] = (wb[t] / s_inv) * exp(-d[t] / den);
            const double s2 = pw_sum([&](long long t) { return wb[t]; }, k);
            for (int t = 0; t < k; ++t) wb[t] = wb[t] / s2;
        } else {
            // interpolator.py:141-147
            for (int t = 0; t < k; ++t) wb[t] = 1.0 / (big_pow(d[t], power) + eps);
            const double s = pw_sum([&](long long t) { return wb[t]; }, k);
            for (int t = 0; t < k; ++t) wb[t] = wb[t] / s;
        }
        // interpolator.py:150-153
        const double *vb = reinterpret_cast<const double *>(pval);
        for (int c = 0; c < 3; ++c)
            out[c] = pw_sum([&](long long t) { return wb[t] * vb[(size_t)sl[t] * 4 + c]; }, k);
        if (flags & PTV_FLAG_NAN_TO_NUM)
            for (int c = 0; c < 3; ++c) out[c] = big_nan_to_num(out[c]);
    }
    // inactive (masked) voxels: 0, as the register-list kernels write them
    if (flags & PTV_FLAG_OUT_F32) {
        reinterpret_cast<float *>(U)[vo] = (float)out[0];
        reinterpret_cast<float *>(V)[vo] = (float)out[1];
        reinterpret_cast<float *>(W)[vo] = (float)out[2];
    } else {
        U[vo] = out[0];
        V[vo] = out[1];
        W[vo] = out[2];
    }
}

// the local-RBF slot search (kModeSlots of the register lists): query j's k nearest slots
__global__ __launch_bounds__(256) void k_big_slots(const uint32_t *__restrict__ sv, const int *__restrict__ seg_b,
                                                    const int *__restrict__ seg_e, int64_t q0, int64_t nq, int k,
                                                    uint32_t *__restrict__ slots) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nq) return;
    const long long b = seg_b[j];
    if (seg_e[j] - b < k) return;  // inactive (masked) voxel: the solve skips it
    uint32_t *o = slots + (size_t)(q0 + j) * k;
    for (int t = 0; t < k; ++t) o[t] = sv[b + t];
}

// a speed's sort key: non-negative doubles order as their bits; every NaN becomes the canonical
// quiet NaN, which sorts after +inf
__device__ __forceinline__ unsigned long long spd_key(double s) {
    if (s != s) return 0x7ff8000000000000ull;
    return (unsigned long long)__double_as_longlong(s);
}
__device__ __forceinline__ double key_spd(unsigned long long k) { return __longlong_as_double((long long)k); }

// np.median of a sorted run of n keys (NaNs last: any NaN gives NaN, numpy's _median_nancheck)
__device__ __forceinline__ double sorted_median(const unsigned long long *s, int n) {
    const double last = key_spd(s[n - 1]);
    if (last != last) return last;
    if (n & 1) return key_spd(s[n >> 1]);
    return (key_spd(s[(n >> 1) - 1]) + key_spd(s[n >> 1])) / 2.0;
}

// filter step 1: the neighbour speeds (entries 1 .. k of the sorted (k+1)-NN, filtering.py:29,38)
// into a[j * k ..], and the distance to the (k+1)-th neighbour
__global__ __launch_bounds__(256) void k_big_filter_spd(const unsigned long long *__restrict__ ds,
                                                         const uint32_t *__restrict__ sv, const int *__restrict__ seg_b,
                                                         const double *__restrict__ spd, int64_t q0, int64_t nq, int k,
                                                         unsigned long long *__restrict__ a, double *__restrict__ kth) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nq) return;
    const long long b = seg_b[j];
    for (int t = 0; t < k; ++t) a[j * (long long)k + t] = spd_key(spd[sv[b + 1 + t]]);
    if (kth != nullptr) kth[q0 + j] = sqrt(__longlong_as_double((long long)ds[b + k]));
}

// filter step 2: the median of the sorted speeds, then |speed - median| per neighbour into a2
__global__ __launch_bounds__(256) void k_big_filter_dev(const unsigned long long *__restrict__ a, int64_t nq, int k,
                                                         double *__restrict__ med,
                                                         unsigned long long *__restrict__ a2) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nq) return;
    const unsigned long long *s = a + j * (long long)k;
    const double m = sorted_median(s, k);
    med[j] = m;
    for (int t = 0; t < k; ++t) a2[j * (long long)k + t] = spd_key(fabs(key_spd(s[t]) - m));
}

// filter step 3: MAD, z-score, keep (filtering.py:43-51)
__global__ __launch_bounds__(256) void k_big_filter_keep(const unsigned long long *__restrict__ a2,
                                                          const double *__restrict__ med, BigQueries q, int64_t q0,
                                                          int64_t nq, int k, double threshold, double mad_eps,
                                                          uint8_t *__restrict__ keep) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nq) return;
    const double mad = sorted_median(a2 + j * (long long)k, k);
    const int64_t i = q0 + j;
    const double u = q.pu[i], v = q.pv[i], w = q.pw[i];
    const double sp = sqrt((u * u + v * v) + w * w);  // filtering.py:16-17
    const double zs = fabs(sp - med[j]) / (mad + mad_eps);
    keep[i] = zs <= threshold ? 1 : 0;
}

inline unsigned grid1(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// The big-k path on prepared (binned) particles: `nq_total` queries (BigQueries), k neighbours
// (k + 1 for the filter, whose outputs then go to keep / kth).  Buffers are the caller's BigScratch.
int run_big_knn(BigScratch &sc, const BigQueries &q, const Binned &b, const CellGrid &cg, int64_t nq_total, int k,
                const BigEpilogue &ep, hipStream_t s) {
    if (nq_total <= 0) return PTV_OK;
    // the density radius for k particles and a radius that reaches every particle from any query
    const double ext[3] = {cg.cs[0] * cg.nc[0], cg.cs[1] * cg.nc[1], cg.cs[2] * cg.nc[2]};
    double vol = 1.0, diag2 = 0.0;
    int dims = 0;
    for (int a = 0; a < 3; ++a) {
        diag2 += ext[a] * ext[a];
        if (cg.nc[a] > 1 || ext[a] > 0.0) {
            vol *= std::max(ext[a], 1e-300);
            ++dims;
        }
    }
    const double rall = std::sqrt(diag2) * 1.01 + 8.0 * cg.mg + 1e-300;
    double r0 = std::cbrt((double)k * vol / ((double)std::max<int64_t>(b.n, 1) * 4.18879020478639));
    if (!(r0 > 0.0) || !std::isfinite(r0)) r0 = rall * 1e-3;
    // queries per chunk: about 6 k candidates each into the entry budget
    const int64_t budget = kBigEntryBudget;
    const int64_t per = std::max<int64_t>(1024, std::min<int64_t>(nq_total, budget / (6 * (int64_t)k + 64)));
    PTV_TRY(sc.R.ensure((size_t)per));
    PTV_TRY(sc.ub.ensure((size_t)per));
    PTV_TRY(sc.incl.ensure((size_t)per));
    PTV_TRY(sc.seg_b.ensure((size_t)per));
    PTV_TRY(sc.seg_e.ensure((size_t)per));
    std::vector<unsigned long long> h_incl;
    for (int64_t q0 = 0; q0 < nq_total; q0 += per) {
        const int64_t nq = std::min(per, nq_total - q0);
        hipLaunchKernelGGL(k_big_bound, dim3(grid1(nq, 256)), dim3(256), 0, s, q, cg, b.cstart, k, r0, rall, q0, nq,
                           sc.R.p, sc.ub.p);
        PTV_HIP(hipGetLastError());
        size_t tb = 0;
        PTV_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, sc.ub.p, sc.incl.p, (int)nq, s));
        PTV_TRY(sc.temp.ensure(tb / 8 + 1));
        PTV_HIP(hipcub::DeviceScan::InclusiveSum(sc.temp.p, tb, sc.ub.p, sc.incl.p, (int)nq, s));
        h_incl.resize((size_t)nq);
        PTV_HIP(hipMemcpyAsync(h_incl.data(), sc.incl.p, nq * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipStreamSynchronize(s));
        // sub-chunks whose entries fit the budget (a single query may exceed it: then alone)
        int64_t qa = 0;
        while (qa < nq) {
            const unsigned long long base = qa > 0 ? h_incl[qa - 1] : 0ull;
            int64_t qb = qa + 1;
            while (qb < nq && (int64_t)(h_incl[qb] - base) <= budget) ++qb;
            const int64_t nsub = qb - qa;
            const long long ent = (long long)(h_incl[qb - 1] - base);
            if (ent >= (1LL << 31)) {
                set_error("k-NN (large k): one query's candidate list exceeds 2^31 entries");
                return PTV_E_UNSUPPORTED;
            }
            const size_t ne = (size_t)std::max<long long>(ent, 1);
            PTV_TRY(sc.keys.ensure(ne));
            PTV_TRY(sc.keys2.ensure(ne));
            PTV_TRY(sc.vals.ensure(ne));
            PTV_TRY(sc.vals2.ensure(ne));
            hipLaunchKernelGGL(k_big_gather, dim3(grid1(nsub, 4)), dim3(256), 0, s, q, cg, b.prec, b.cstart, sc.R.p,
                               sc.incl.p, q0, qa, nsub, sc.keys.p, sc.vals.p, sc.seg_b.p, sc.seg_e.p);
            PTV_HIP(hipGetLastError());
            size_t sb = 0;
            PTV_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, sb, sc.keys.p, sc.keys2.p, sc.vals.p,
                                                                 sc.vals2.p, (int)ne, (int)nsub, sc.seg_b.p,
                                                                 sc.seg_e.p, 0, 64, s));
            PTV_TRY(sc.temp.ensure(sb / 8 + 1));
            PTV_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(sc.temp.p, sb, sc.keys.p, sc.keys2.p, sc.vals.p,
                                                                 sc.vals2.p, (int)ne, (int)nsub, sc.seg_b.p,
                                                                 sc.seg_e.p, 0, 64, s));
            if (ep.slots != nullptr) {
                hipLaunchKernelGGL(k_big_slots, dim3(grid1(nsub, 256)), dim3(256), 0, s, sc.vals2.p, sc.seg_b.p,
                                   sc.seg_e.p, q0 + qa, nsub, k, ep.slots);
                PTV_HIP(hipGetLastError());
            } else if (ep.filter) {
                // (k + 1)-NN of particle i = q0 + qa + j: neighbours 1 .. k, then the two medians
                const size_t na = (size_t)nsub * (size_t)(k - 1);
                const int kk = k - 1;  // the reference's k
                PTV_TRY(sc.fa.ensure(na));
                PTV_TRY(sc.fa2.ensure(na));
                PTV_TRY(sc.fb.ensure(na));
                PTV_TRY(sc.fmed.ensure((size_t)nsub));
                PTV_TRY(sc.fseg.ensure((size_t)nsub + 1));
                std::vector<int> hs((size_t)nsub + 1);
                for (int64_t t = 0; t <= nsub; ++t) hs[t] = (int)(t * kk);
                PTV_HIP(hipMemcpyAsync(sc.fseg.p, hs.data(), hs.size() * sizeof(int), hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL(k_big_filter_spd, dim3(grid1(nsub, 256)), dim3(256), 0, s, sc.keys2.p, sc.vals2.p,
                                   sc.seg_b.p, ep.spd, q0 + qa, nsub, kk, sc.fa.p, ep.kth);
                PTV_HIP(hipGetLastError());
                size_t fb = 0;
                PTV_HIP(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, fb, sc.fa.p, sc.fa2.p, (int)na, (int)nsub,
                                                                    sc.fseg.p, sc.fseg.p + 1, 0, 64, s));
                PTV_TRY(sc.temp.ensure(fb / 8 + 1));
                PTV_HIP(hipcub::DeviceSegmentedRadixSort::SortKeys(sc.temp.p, fb, sc.fa.p, sc.fa2.p, (int)na,
                                                                    (int)nsub, sc.fseg.p, sc.fseg.p + 1, 0, 64, s));
                hipLaunchKernelGGL(k_big_filter_dev, dim3(grid1(nsub, 256)), dim3(256), 0, s, sc.fa2.p, nsub, kk,
                                   sc.fmed.p, sc.fb.p);
                PTV_HIP(hipGetLastError());
                PTV_HIP(hipcub::DeviceSegmentedRadixSort::SortKeys(sc.temp.p, fb, sc.fb.p, sc.fa.p, (int)na,
                                                                    (int)nsub, sc.fseg.p, sc.fseg.p + 1, 0, 64, s));
                hipLaunchKernelGGL(k_big_filter_keep, dim3(grid1(nsub, 256)), dim3(256), 0, s, sc.fa.p, sc.fmed.p, q,
                                   q0 + qa, nsub, kk, ep.threshold, ep.mad_eps, ep.keep);
                PTV_HIP(hipGetLastError());
                // the host's copies of hs must outlive the upload
                PTV_HIP(hipStreamSynchronize(s));
            } else {
                hipLaunchKernelGGL(k_big_interp, dim3(grid1(nsub, 256)), dim3(256), 0, s, q, b.pval, sc.keys2.p,
                                   sc.vals2.p, reinterpret_cast<double *>(sc.keys.p), sc.seg_b.p, sc.seg_e.p, q0 + qa,
                                   nsub, k, ep.method, ep.power, ep.eps, ep.flags, ep.U, ep.V, ep.W);
                PTV_HIP(hipGetLastError());
            }
            qa = qb;
        }
    }
    return PTV_OK;
}

}  // namespace ptv
