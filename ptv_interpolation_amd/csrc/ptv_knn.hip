// ptv_knn.hip — exact k-nearest-neighbour IDW / Sibson interpolation onto a voxel grid (gfx950).
//
// Replaces, per voxel, the reference hot loop
//   distances, indices = tree.query(flat_coords, k)                 interpolator.py:139 (:97)
//   weights = 1/(d**p + 1e-10); weights /= weights.sum(axis=1)       interpolator.py:142-147
//   (Sibson: inv-distance * exp(-d/std(d)), renormalised            interpolator.py:102-116)
//   out[:, c] = (weights * values[indices, c]).sum(axis=1)          interpolator.py:150-153 (:119-122)
//
// Work decomposition: one wave64 = one 4x4x4 voxel tile (lane = voxel), a 256-thread
// workgroup = 4 tiles along x (16x4x4 voxels: 128-B output rows).  Each wave walks the
// Morton octree of particle cells front-to-back with a wave-uniform stack kept in one
// VGPR (lane i = stack slot i; v_readlane pops, a lane-select pushes); a node is visited iff some
// lane's voxel is closer to the node box than that lane's current k-th distance, so
// voids (sphere interiors) cost a few node tests instead of a shell of empty cells.
// Particle records are read with wave-uniform addresses (scalar loads), so each
// candidate is one s_load shared by 64 voxels; per lane a sorted register list of the
// KMAX best (d2, slot) is kept by a branch-free insertion network.
//
// Bit-level contract with the reference (compiled with -ffp-contract=off):
//   d2 = (dx*dx + dy*dy) + dz*dz, d = sqrt(d2)      (cKDTree p=2 accumulation, then sqrt)
//   d**p: p=2 -> d*d, 1 -> d, 0.5 -> sqrt, -1 -> 1/d, else pow (numpy scalar fast paths)
//   row sums: numpy pairwise order from identity 0.0 (8 accumulators, n%8 tail)
// Ties at equal d2 keep the earlier candidate in the fixed traversal order
// (cKDTree's tie order is traversal dependent too).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

constexpr int kLeafMax = 16;  // a node with <= kLeafMax particles is scanned directly

struct KnnKernelArgs {
    CellGrid cg;
    int nx, ny, nz, z0, z1;
    int ntx, nty, ntz, ntxb;
    int separable, method, k, kpad;
    double power, eps;
    uint32_t flags;
};

// numpy pairwise sum of a[0..n) (n <= KMAX <= 128), from identity 0.0.
template <int KMAX>
__device__ __forceinline__ double pairwise(const double (&a)[KMAX], int n) {
    if (KMAX < 8 || n < 8) {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (j < n) r += a[j];
        return r;
    }
    if constexpr (KMAX >= 8) {
        double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
        const int stop = n - (n & 7);
#pragma unroll
        for (int i = 8; i + 8 <= KMAX; i += 8) {
            if (i < stop) {
                r0 += a[i + 0];
                r1 += a[i + 1];
                r2 += a[i + 2];
                r3 += a[i + 3];
                r4 += a[i + 4];
                r5 += a[i + 5];
                r6 += a[i + 6];
                r7 += a[i + 7];
            }
        }
        double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
#pragma unroll
        for (int j = 8; j < KMAX; ++j)
            if (j >= stop && j < n) res += a[j];
        return res;
    }
    return 0.0;
}

// d ** p with numpy's scalar fast paths (p uniform).
__device__ __forceinline__ double np_pow(double d, double p) {
    if (p == 2.0) return d * d;
    if (p == 1.0) return d;
    if (p == 0.5) return sqrt(d);
    if (p == -1.0) return 1.0 / d;
    return pow(d, p);
}

__device__ __forceinline__ double nan_to_num(double v) {
    if (v != v) return 0.0;
    if (v == INFINITY) return DBL_MAX;
    if (v == -INFINITY) return -DBL_MAX;
    return v;
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

template <int KMAX>
__device__ __forceinline__ void insert(double (&bd)[KMAX], int (&bp)[KMAX], double d2, int p) {
    // descending sweep: slot j takes slot j-1 if the candidate beats j-1, else the
    // candidate if it beats j, else keeps its value (two live compare masks only)
    bool lt_j = d2 < bd[KMAX - 1];
#pragma unroll
    for (int j = KMAX - 1; j > 0; --j) {
        const bool lt_m = d2 < bd[j - 1];
        const double nd = lt_m ? bd[j - 1] : (lt_j ? d2 : bd[j]);
        const int np = lt_m ? bp[j - 1] : (lt_j ? p : bp[j]);
        bd[j] = nd;
        bp[j] = np;
        lt_j = lt_m;
    }
    if (lt_j) {
        bd[0] = d2;
        bp[0] = p;
    }
}

template <int KMAX>
__global__ __launch_bounds__(256) void k_knn_interp(KnnKernelArgs a, const double4 *__restrict__ prec,
                                                    const double4 *__restrict__ pval,
                                                    const uint32_t *__restrict__ cstart,
                                                    const double *__restrict__ ax, const double *__restrict__ ay,
                                                    const double *__restrict__ az, const double *__restrict__ qpx,
                                                    const double *__restrict__ qpy, const double *__restrict__ qpz,
                                                    const uint8_t *__restrict__ mask, double *__restrict__ U,
                                                    double *__restrict__ V, double *__restrict__ W) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const int bx = b % a.ntxb;
    const int rr = b / a.ntxb;
    const int ty = rr % a.nty;
    const int tz = rr / a.nty;
    const int tx = bx * 4 + wid;
    if (tx >= a.ntx) return;  // wave-uniform

    const int ix = tx * 4 + (lane & 3);
    const int iy = ty * 4 + ((lane >> 2) & 3);
    const int iz = a.z0 + tz * 4 + (lane >> 4);
    const bool valid = ix < a.nx && iy < a.ny && iz < a.z1;
    const int cx = min(ix, a.nx - 1), cy = min(iy, a.ny - 1), cz = min(iz, a.z1 - 1);
    const size_t vfull = ((size_t)cz * a.ny + cy) * a.nx + cx;
    double qx, qy, qz;
    if (a.separable) {
        qx = ax[cx];
        qy = ay[cy];
        qz = az[cz];
    } else {
        qx = qpx[vfull];
        qy = qpy[vfull];
        qz = qpz[vfull];
    }
    const bool active = valid && (mask == nullptr || mask[vfull] != 0);

    // sorted list: KMAX-k front sentinels (-1) so bd[KMAX-1] is the k-th best
    double bd[KMAX];
    int bp[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        bd[j] = (j < a.kpad) ? -1.0 : INFINITY;
        bp[j] = -1;
    }
    double thr = active ? INFINITY : -1.0;

    if (__builtin_amdgcn_ballot_w64(active) != 0) {
        // tile centre (front-to-back child order)
        const double tcx = 0.5 * (wave_min(active ? qx : INFINITY) + wave_max(active ? qx : -INFINITY));
        const double tcy = 0.5 * (wave_min(active ? qy : INFINITY) + wave_max(active ? qy : -INFINITY));
        const double tcz = 0.5 * (wave_min(active ? qz : INFINITY) + wave_max(active ? qz : -INFINITY));
        const int L = a.cg.L;
        int stack = 0;
        stack = (lane == 0) ? (int)((uint32_t)L << 27) : stack;
        int sp = 1;
        while (sp > 0) {
            --sp;
            const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(stack, sp);
            const int l = (int)(e >> 27);
            const uint32_t code = e & ((1u << 27) - 1u);
            const uint32_t s0 = cstart[code << (3 * l)];
            const uint32_t s1 = cstart[(code + 1u) << (3 * l)];
            if (s0 == s1) continue;
            const uint32_t ci = compact3(code), cj = compact3(code >> 1), ck = compact3(code >> 2);
            const double x0 = a.cg.o[0] + (double)(ci << l) * a.cg.cs[0] - a.cg.mg[0];
            const double x1 = a.cg.o[0] + (double)((ci + 1u) << l) * a.cg.cs[0] + a.cg.mg[0];
            const double y0 = a.cg.o[1] + (double)(cj << l) * a.cg.cs[1] - a.cg.mg[1];
            const double y1 = a.cg.o[1] + (double)((cj + 1u) << l) * a.cg.cs[1] + a.cg.mg[1];
            const double z0 = a.cg.o[2] + (double)(ck << l) * a.cg.cs[2] - a.cg.mg[2];
            const double z1 = a.cg.o[2] + (double)((ck + 1u) << l) * a.cg.cs[2] + a.cg.mg[2];
            const double ddx = fmax(fmax(x0 - qx, qx - x1), 0.0);
            const double ddy = fmax(fmax(y0 - qy, qy - y1), 0.0);
            const double ddz = fmax(fmax(z0 - qz, qz - z1), 0.0);
            const double md2 = (ddx * ddx + ddy * ddy) + ddz * ddz;
            if (__builtin_amdgcn_ballot_w64(md2 < thr) == 0) continue;
            if (l == 0 || s1 - s0 <= (uint32_t)kLeafMax) {
                for (uint32_t p = s0; p < s1; ++p) {
                    const double4 r = prec[p];
                    const double dx = qx - r.x, dy = qy - r.y, dz = qz - r.z;
                    const double d2 = (dx * dx + dy * dy) + dz * dz;
                    if (d2 < thr) {
                        insert<KMAX>(bd, bp, d2, (int)p);
                        thr = bd[KMAX - 1];
                    }
                }
            } else {
                const double mx = 0.5 * (x0 + x1), my = 0.5 * (y0 + y1), mz = 0.5 * (z0 + z1);
                const uint32_t oct = (tcx >= mx ? 1u : 0u) | (tcy >= my ? 2u : 0u) | (tcz >= mz ? 4u : 0u);
                const uint32_t lc = (uint32_t)(l - 1) << 27;
#pragma unroll
                for (int c = 7; c >= 0; --c) {
                    stack = (lane == sp) ? (int)(lc | ((code << 3) | (oct ^ (uint32_t)c))) : stack;
                    ++sp;
                }
            }
        }
    }

    if (!valid) return;
    const size_t vo = ((size_t)(iz - a.z0) * a.ny + iy) * a.nx + ix;
    if (!active) {
        U[vo] = 0.0;
        V[vo] = 0.0;
        W[vo] = 0.0;
        return;
    }

    // left-shift the list by kpad so real entries occupy slots 0..k-1 (kpad uniform)
#pragma unroll
    for (int sh = 1; sh < KMAX; sh <<= 1) {
        if (a.kpad & sh) {
#pragma unroll
            for (int j = 0; j + sh < KMAX; ++j) {
                bd[j] = bd[j + sh];
                bp[j] = bp[j + sh];
            }
        }
    }
    const int k = a.k;
    double w[KMAX];
    if (a.method == PTV_METHOD_SIBSON) {
        // interpolator.py:106-116
        double d[KMAX], t[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            d[j] = (j < k) ? sqrt(bd[j]) : 0.0;
            t[j] = (j < k) ? 1.0 / (d[j] + a.eps) : 0.0;
        }
        const double s_inv = pairwise<KMAX>(t, k);
        const double mean = pairwise<KMAX>(d, k) / (double)k;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            w[j] = t[j] / s_inv;
            const double c = d[j] - mean;
            t[j] = c * c;
        }
        const double sd = sqrt(pairwise<KMAX>(t, k) / (double)k);
        const double den = sd + a.eps;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) w[j] = (j < k) ? w[j] * exp(-d[j] / den) : 0.0;
        const double s2 = pairwise<KMAX>(w, k);
#pragma unroll
        for (int j = 0; j < KMAX; ++j) w[j] = w[j] / s2;
    } else {
        // interpolator.py:143-147
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            const double d = sqrt(bd[j]);
            w[j] = (j < k) ? 1.0 / (np_pow(d, a.power) + a.eps) : 0.0;
        }
        const double s = pairwise<KMAX>(w, k);
#pragma unroll
        for (int j = 0; j < KMAX; ++j) w[j] = w[j] / s;
    }

    // interpolator.py:150-153: per component, sum_k w * values[idx, c]
    const double *vb = reinterpret_cast<const double *>(pval);
    double out[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double t[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) t[j] = (j < k) ? w[j] * vb[(size_t)bp[j] * 4 + c] : 0.0;
        out[c] = pairwise<KMAX>(t, k);
    }
    if (a.flags & PTV_FLAG_NAN_TO_NUM) {
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = nan_to_num(out[c]);
    }
    U[vo] = out[0];
    V[vo] = out[1];
    W[vo] = out[2];
}

static const int kKmaxList[] = {4, 8, 12, 16, 24, 32, 40, 48, 56, 64};

int kmax_for(int k) {
    for (int km : kKmaxList)
        if (k <= km) return km;
    return 0;
}

template <int KMAX>
static void launch_t(dim3 grid, hipStream_t s, const KnnKernelArgs &ka, const Binned &b, const double *ax,
                     const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
                     const uint8_t *mask, double *U, double *V, double *W) {
    hipLaunchKernelGGL(k_knn_interp<KMAX>, grid, dim3(256), 0, s, ka, b.prec, b.pval, b.cstart, ax, ay, az, qx, qy,
                       qz, mask, U, V, W);
}

int launch_knn(const KnnLaunch &a, const Binned &b, const double *ax, const double *ay, const double *az,
               const double *qx, const double *qy, const double *qz, const uint8_t *mask, double *U, double *V,
               double *W, hipStream_t s) {
    const int km = kmax_for(a.k);
    if (km == 0) {
        set_error("k=" + std::to_string(a.k) + " exceeds the GPU k-NN list limit (64)");
        return PTV_E_UNSUPPORTED;
    }
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
    ka.kpad = km - a.k;
    ka.power = a.power;
    ka.eps = a.eps;
    ka.flags = a.flags;
    const long long nblocks = (long long)ka.ntxb * ka.nty * ka.ntz;
    if (nblocks > 0x7fffffffLL) {
        set_error("grid too large for one launch");
        return PTV_E_ARG;
    }
    dim3 grid((unsigned)nblocks);
    switch (km) {
#define PTV_CASE(K) \
    case K: launch_t<K>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W); break;
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
#undef PTV_CASE
        default:
            return PTV_E_UNSUPPORTED;
    }
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
