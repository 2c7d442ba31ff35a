// ptv_div.hip — consistent finite-volume divergence of an interpolated velocity field.
//
// Restates physics.compute_consistent_divergence (physics.py:6-53), the divergence
// view_divergence.py:39,42 reads after interpolation, as one
// HBM-bound stencil pass.  Per axis a with cell velocity c = vel[i] (get_face_vel,
// physics.py:26-48):
//     f_next = (i == n-1) ? c : (fluid[i+1] ? (c + vel[i+1]) / 2 : 0)      (:35-41)
//     f_prev = (i == 0)   ? c : (fluid[i]   ? (vel[i-1] + c) / 2 : 0)      (:44-46: roll of f_next)
// and div = ((ufn - ufp)/dx + (vfn - vfp)/dy) + (wfn - wfp)/dz             (:53)
// in numpy's evaluation order and types: the face values and their difference are in
// the field dtype T; the division and the sums in R = result_type(T, spacing) (a Python
// float spacing keeps float32 fields in float32, a numpy float64 scalar — view_divergence.py:22
// takes x[1] - x[0] — promotes the quotients to float64).  No np.roll wrap survives: the
// edge overwrites replace every wrapped face.  The cell's own fluid flag does not zero
// its divergence (the reference does not either).
//
// Layout: T fields (nz, ny, nx) C order in HBM, uint8 mask, R output.  A z-slab launch
// computes planes [z_begin, z_end) of a buffer whose plane 0 / nz-1 are either the domain's
// z edges (edge_lo / edge_hi) or one-plane halos from the neighbouring slab.
//
// Kernel shape: 64 x 4 lanes, each owning VEC consecutive x (16-byte loads and stores when
// rows are 16-byte aligned) of one y row, march kDivPlanes z-planes in batches of
// kDivBatch whose loads (clamped at the faces, so unconditional) all issue before the
// arithmetic: the z stencil of a batch is read once; the x neighbours come from the same
// cache lines and the y neighbours from the adjacent waves of the block (L1/L2).
// Algorithmic bytes per voxel: 3 sizeof(T) + 1 + sizeof(R).
#include <cstdlib>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

namespace {

constexpr int kDivPlanes = 32;  // z-planes per thread column
constexpr int kDivBatch = 4;    // planes whose loads are all issued before any arithmetic

// VEC consecutive elements per lane: one 16-byte load per lane when VEC * sizeof(T) == 16
template <typename T, int VEC>
struct Vec {
    T e[VEC];
};
template <typename T, int VEC>
__device__ __forceinline__ Vec<T, VEC> ldv(const T *p) {
    Vec<T, VEC> r;
    if constexpr (VEC * sizeof(T) == 16) {
        const uint4 q = *reinterpret_cast<const uint4 *>(p);
        __builtin_memcpy(r.e, &q, 16);
    } else if constexpr (VEC * sizeof(T) == 8) {
        const uint2 q = *reinterpret_cast<const uint2 *>(p);
        __builtin_memcpy(r.e, &q, 8);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) r.e[i] = p[i];
    }
    return r;
}
template <int VEC>
__device__ __forceinline__ Vec<uint8_t, VEC> ldm(const uint8_t *p) {
    Vec<uint8_t, VEC> r;
    if constexpr (VEC == 4) {
        const uint32_t q = *reinterpret_cast<const uint32_t *>(p);
        __builtin_memcpy(r.e, &q, 4);
    } else if constexpr (VEC == 2) {
        const uint16_t q = *reinterpret_cast<const uint16_t *>(p);
        __builtin_memcpy(r.e, &q, 2);
    } else {
        r.e[0] = p[0];
    }
    return r;
}

// One lane = VEC consecutive x of one (y, z-chunk) column; a block is 64 lanes x 4 rows.
template <typename T, typename R, int VEC>
__global__ __launch_bounds__(256) void k_divergence(DivArgs a, const T *__restrict__ U, const T *__restrict__ V,
                                                    const T *__restrict__ W, const uint8_t *__restrict__ M,
                                                    R *__restrict__ out) {
    int t = blockIdx.x;
    if (a.xcd) {
        // XCD-aware tile order: hardware block b runs on XCD b % 8, so logical tile
        // (b % 8) * per + b / 8 hands each XCD a contiguous run of tiles (x fastest, then y,
        // then z chunk) whose shared x / y halo lines stay in that XCD's L2
        const int per = (a.ntiles + 7) >> 3;
        t = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    }
    if (t >= a.ntiles) return;
    const int tx = t % a.ntx, ty = (t / a.ntx) % a.nty, tz = t / (a.ntx * a.nty);
    const int x0 = (tx * 64 + threadIdx.x) * VEC;
    const int y = ty * 4 + threadIdx.y;
    if (x0 >= a.nx || y >= a.ny) return;
    const int zb = a.z_begin + tz * kDivPlanes;
    const int ze = min(zb + kDivPlanes, a.z_end);
    const int64_t plane = (int64_t)a.nx * a.ny;
    const int64_t col = (int64_t)y * a.nx + x0;
    const R dx = (R)a.dx, dy = (R)a.dy, dz = (R)a.dz;
    const T half = (T)0.5;  // (c + n) / 2.0 == (c + n) * 0.5 exactly
    const int xl = x0 + VEC - 1;  // the lane's last x
    const bool ylo = y == 0, yhi = y == a.ny - 1;
    // neighbour offsets clamped at the domain faces: every load below is in bounds and
    // unconditional (the face rules then pick the cell value), so a batch's loads issue
    // back to back and overlap their HBM latency
    const int oxm = x0 == 0 ? 0 : 1, oxp = xl == a.nx - 1 ? 0 : 1;
    const int64_t oym = ylo ? 0 : a.nx, oyp = yhi ? 0 : a.nx;
    auto row = [&](int zz) { return (int64_t)min(max(zz, 0), a.nz - 1) * plane + col; };

    // w[t] = W(z0 - 1 + t), m[t] = fluid(z0 + t): the z stencil of the batch's planes; the
    // last two w and the last m carry into the next batch
    Vec<T, VEC> w[kDivBatch + 2];
    Vec<uint8_t, VEC> m[kDivBatch + 1];
    w[0] = ldv<T, VEC>(W + row(zb - 1));
    w[1] = ldv<T, VEC>(W + row(zb));
    m[0] = ldm<VEC>(M + row(zb));
    for (int z0 = zb; z0 < ze; z0 += kDivBatch) {
#pragma unroll
        for (int q = 2; q < kDivBatch + 2; ++q) w[q] = ldv<T, VEC>(W + row(z0 - 1 + q));
#pragma unroll
        for (int q = 1; q < kDivBatch + 1; ++q) m[q] = ldm<VEC>(M + row(z0 + q));
        Vec<T, VEC> uc[kDivBatch], vc[kDivBatch], vm[kDivBatch], vp[kDivBatch];
        Vec<uint8_t, VEC> my[kDivBatch];
        T ul[kDivBatch], ur[kDivBatch];
        uint8_t mr[kDivBatch];
#pragma unroll
        for (int j = 0; j < kDivBatch; ++j) {
            const int64_t r = row(z0 + j);
            uc[j] = ldv<T, VEC>(U + r);
            ul[j] = U[r - oxm];
            ur[j] = U[r + VEC - 1 + oxp];
            mr[j] = M[r + VEC - 1 + oxp];
            vc[j] = ldv<T, VEC>(V + r);
            vm[j] = ldv<T, VEC>(V + r - oym);
            vp[j] = ldv<T, VEC>(V + r + oyp);
            my[j] = ldm<VEC>(M + r + oyp);
        }
#pragma unroll
        for (int j = 0; j < kDivBatch; ++j) {
            const int z = z0 + j;
            if (z >= ze) break;
            const bool zlo = z == 0 && a.edge_lo, zhi = z == a.nz - 1 && a.edge_hi;
            Vec<R, VEC> o;
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const bool own = m[j].e[e] != 0;
                const bool xlo = x0 + e == 0, xhi = x0 + e == a.nx - 1;
                const T c = uc[j].e[e];
                const T un = e + 1 < VEC ? uc[j].e[e + 1 < VEC ? e + 1 : e] : ur[j];
                const T up = e > 0 ? uc[j].e[e > 0 ? e - 1 : 0] : ul[j];
                const bool mxn = (e + 1 < VEC ? m[j].e[e + 1 < VEC ? e + 1 : e] : mr[j]) != 0;
                const T ufn = xhi ? c : (mxn ? (c + un) * half : (T)0);
                const T ufp = xlo ? c : (own ? (up + c) * half : (T)0);
                const T vcc = vc[j].e[e];
                const T vfn = yhi ? vcc : (my[j].e[e] ? (vcc + vp[j].e[e]) * half : (T)0);
                const T vfp = ylo ? vcc : (own ? (vm[j].e[e] + vcc) * half : (T)0);
                const T wc = w[j + 1].e[e];
                const T wfn = zhi ? wc : (m[j + 1].e[e] ? (wc + w[j + 2].e[e]) * half : (T)0);
                const T wfp = zlo ? wc : (own ? (w[j].e[e] + wc) * half : (T)0);
                const R tx = (R)(ufn - ufp) / dx;
                const R ty = (R)(vfn - vfp) / dy;
                const R tz = (R)(wfn - wfp) / dz;
                o.e[e] = (tx + ty) + tz;
            }
            R *dst = out + (int64_t)(z - a.z_begin) * plane + col;
            if constexpr (VEC * sizeof(R) == 16) {
                uint4 q;
                __builtin_memcpy(&q, o.e, 16);
                *reinterpret_cast<uint4 *>(dst) = q;
            } else if constexpr (VEC * sizeof(R) == 32) {
                uint4 q[2];
                __builtin_memcpy(q, o.e, 32);
                reinterpret_cast<uint4 *>(dst)[0] = q[0];
                reinterpret_cast<uint4 *>(dst)[1] = q[1];
            } else {
#pragma unroll
                for (int e = 0; e < VEC; ++e) dst[e] = o.e[e];
            }
        }
        w[0] = w[kDivBatch];
        w[1] = w[kDivBatch + 1];
        m[0] = m[kDivBatch];
    }
}

template <typename T, typename R, int VEC>
int launch_v(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
             hipStream_t s) {
    DivArgs b = a;
    b.ntx = (a.nx + 64 * VEC - 1) / (64 * VEC);
    b.nty = (a.ny + 3) / 4;
    const int64_t nt = (int64_t)b.ntx * b.nty * ((a.z_end - a.z_begin + kDivPlanes - 1) / kDivPlanes);
    if (nt > 0x7fffff00LL) {
        set_error("divergence: grid too large for one launch");
        return PTV_E_ARG;
    }
    b.ntiles = (int)nt;
    const dim3 grid((unsigned)(((nt + 7) >> 3) << 3));
    hipLaunchKernelGGL((k_divergence<T, R, VEC>), grid, dim3(64, 4), 0, s, b, (const T *)U, (const T *)V,
                       (const T *)W, M, (R *)out);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

// 16-byte lanes (VEC = 16 / sizeof(T)) when every row starts 16-byte aligned, else one
// element per lane
template <typename T, typename R>
int launch_t(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
             hipStream_t s) {
    constexpr int VEC = 16 / sizeof(T);
    auto al = [](const void *p, size_t n) { return ((uintptr_t)p % n) == 0; };
    const bool vec_ok = a.nx % VEC == 0 && al(U, 16) && al(V, 16) && al(W, 16) && al(M, VEC) &&
                        al(out, VEC * sizeof(R));
    if (vec_ok) return launch_v<T, R, VEC>(a, U, V, W, M, out, s);
    return launch_v<T, R, 1>(a, U, V, W, M, out, s);
}

}  // namespace

int launch_typed(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
                 hipStream_t s);

int launch_divergence(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
                      hipStream_t s) {
    if (a.z_end <= a.z_begin) return PTV_OK;
    DivArgs b = a;
    if (const char *e = dev_knob("PTV_DIV_XCD")) b.xcd = std::atoi(e);  // dev knob
    return launch_typed(b, U, V, W, M, out, s);
}

int launch_typed(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
                 hipStream_t s) {
    if (a.field_f32 == 0 && a.result_f32 == 0) return launch_t<double, double>(a, U, V, W, M, out, s);
    if (a.field_f32 == 1 && a.result_f32 == 1) return launch_t<float, float>(a, U, V, W, M, out, s);
    if (a.field_f32 == 1 && a.result_f32 == 0) return launch_t<float, double>(a, U, V, W, M, out, s);
    set_error("divergence: float64 fields with float32 results are not a numpy promotion");
    return PTV_E_ARG;
}

}  // namespace ptv
