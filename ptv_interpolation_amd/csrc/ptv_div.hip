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
// Kernel shape: 64 x 4 threads own (x, y) columns and march kDivPlanes z-planes, keeping
// w(z), w(z+1) and fluid(z+1) in registers, so w and the z mask are read once; the x
// neighbours come from the same cache lines and the y neighbours from the adjacent
// waves of the block (L2).  Algorithmic bytes per voxel: 3 sizeof(T) + 1 + sizeof(R).
#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

namespace {

constexpr int kDivPlanes = 16;

template <typename T, typename R>
__global__ __launch_bounds__(256) void k_divergence(DivArgs a, const T *__restrict__ U, const T *__restrict__ V,
                                                    const T *__restrict__ W, const uint8_t *__restrict__ M,
                                                    R *__restrict__ out) {
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    if (x >= a.nx || y >= a.ny) return;
    const int zb = a.z_begin + blockIdx.z * kDivPlanes;
    const int ze = min(zb + kDivPlanes, a.z_end);
    const int64_t plane = (int64_t)a.nx * a.ny;
    const int64_t col = (int64_t)y * a.nx + x;
    const R dx = (R)a.dx, dy = (R)a.dy, dz = (R)a.dz;
    const T half = (T)0.5;  // (c + n) / 2.0 == (c + n) * 0.5 exactly
    const bool xlo = x == 0, xhi = x == a.nx - 1, ylo = y == 0, yhi = y == a.ny - 1;

    int64_t i = zb * plane + col;
    T wc = W[i];
    uint8_t mc = M[i];
    for (int z = zb; z < ze; ++z, i += plane) {
        const bool zlo = z == 0 && a.edge_lo, zhi = z == a.nz - 1 && a.edge_hi;
        // z: w(z+1) and fluid(z+1) slide into the next iteration (never read past a domain edge)
        T wn = wc;
        uint8_t mn = 0;
        if (!zhi) {
            wn = W[i + plane];
            mn = M[i + plane];
        }
        const T uc = U[i], vc = V[i];
        T ufn = uc, ufp = uc, vfn = vc, vfp = vc;
        if (!xhi) ufn = M[i + 1] ? (uc + U[i + 1]) * half : (T)0;
        if (!xlo) ufp = mc ? (U[i - 1] + uc) * half : (T)0;
        if (!yhi) vfn = M[i + a.nx] ? (vc + V[i + a.nx]) * half : (T)0;
        if (!ylo) vfp = mc ? (V[i - a.nx] + vc) * half : (T)0;
        T wfn = wc, wfp = wc;
        if (!zhi) wfn = mn ? (wc + wn) * half : (T)0;
        if (!zlo) wfp = mc ? (W[i - plane] + wc) * half : (T)0;
        const R tx = (R)(ufn - ufp) / dx;
        const R ty = (R)(vfn - vfp) / dy;
        const R tz = (R)(wfn - wfp) / dz;
        out[(int64_t)(z - a.z_begin) * plane + col] = (tx + ty) + tz;
        wc = wn;
        mc = mn;
    }
}

template <typename T, typename R>
int launch_t(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
             hipStream_t s) {
    const dim3 grid((a.nx + 63) / 64, (a.ny + 3) / 4, (a.z_end - a.z_begin + kDivPlanes - 1) / kDivPlanes);
    hipLaunchKernelGGL((k_divergence<T, R>), grid, dim3(64, 4), 0, s, a, (const T *)U, (const T *)V, (const T *)W, M,
                       (R *)out);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace

int launch_divergence(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
                      hipStream_t s) {
    if (a.z_end <= a.z_begin) return PTV_OK;
    if (a.field_f32 == 0 && a.result_f32 == 0) return launch_t<double, double>(a, U, V, W, M, out, s);
    if (a.field_f32 == 1 && a.result_f32 == 1) return launch_t<float, float>(a, U, V, W, M, out, s);
    if (a.field_f32 == 1 && a.result_f32 == 0) return launch_t<float, double>(a, U, V, W, M, out, s);
    set_error("divergence: float64 fields with float32 results are not a numpy promotion");
    return PTV_E_ARG;
}

}  // namespace ptv
