// ptv_linear.hip — method='linear' on the GPU (gfx950): point location in scipy's own
// Delaunay triangulation and barycentric interpolation, per voxel.
//
// Replaces, per voxel, what the reference's
//   interpolated = griddata(points, values, grid_coords, method='linear', fill_value=0.0)
// (interpolator.py:196-197) does inside LinearNDInterpolator's evaluation
// (scipy interpolate/interpnd.pyx _do_evaluate, spatial/_qhull.pyx _find_simplex):
//   * a point outside [min_bound - eps, max_bound + eps] (eps = 100 DBL_EPSILON) -> fill_value;
//   * a directed walk through the simplices: at simplex s the barycentric coordinates
//       c_i = ((0 + T_i0 (x_0 - r_0)) + T_i1 (x_1 - r_1)) + T_i2 (x_2 - r_2),  i < 3
//       c_3 = ((1 - c_0) - c_1) - c_2
//     (T = transform[s, :3], r = transform[s, 3]) are taken in order; the first c_k < -eps
//     moves to neighbour k (-1: outside the hull -> fill_value); all in [-eps, 1 + eps] ->
//     found; otherwise (a degenerate simplex: NaN transform) scipy falls back to a brute-force
//     scan, as here (k_linear_brute, first simplex index that accepts the point);
//   * out_k = (((0 + c_0 v[s_0, k]) + c_1 v[s_1, k]) + c_2 v[s_2, k]) + c_3 v[s_3, k].
// The triangulation (simplices, neighbors, transform) is scipy's own (Qhull, computed on the
// host exactly as LinearNDInterpolator does), so for every voxel that lies in one simplex the
// result is bit-identical; a voxel within eps of a shared face may be assigned to either
// simplex (scipy's choice depends on the previous voxel's simplex), where both agree to rounding.
//
// MI355X mapping: one lane per voxel, x fastest (a wave = 64 consecutive voxels of a row, whose
// walks visit the same few simplices: their transform rows stay in L2/L1).  The walk starts at a
// simplex incident to the voxel's nearest particle (the k = 1 search of ptv_knn.hip in slot
// mode), so it is a few steps long; scipy starts from the previous voxel's simplex after a walk
// over the lifted paraboloid.  Compiled with -ffp-contract=off (no fused multiply-adds).
#include <hip/hip_runtime.h>

#include <cfloat>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"

namespace ptv {

constexpr double kLinEps = 100.0 * DBL_EPSILON;  // interpnd: eps = 100 * DBL_EPSILON

// block b (dispatched to XCD b % 8) -> a contiguous range of rows per XCD (each XCD has its own L2)
__device__ __forceinline__ long long lin_xcd_block(long long b, long long nb) {
    const long long q = nb >> 3, r = nb & 7;
    const long long x = b & 7, i = b >> 3;
    return (x < r) ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// c_i of simplex s (interpnd _barycentric_coordinate_single, i < 3)
__device__ __forceinline__ double bary(const double *__restrict__ T, int i, double x0, double x1, double x2) {
    double c = 0.0;
    c = c + T[3 * i + 0] * (x0 - T[9]);
    c = c + T[3 * i + 1] * (x1 - T[10]);
    c = c + T[3 * i + 2] * (x2 - T[11]);
    return c;
}

__device__ __forceinline__ void lin_store(const LinearKernelArgs &a, double *U, double *V, double *W, size_t vo,
                                          double u, double v, double w) {
    if (a.flags & PTV_FLAG_NAN_TO_NUM) {
        auto fix = [](double t) { return t != t ? 0.0 : (t == INFINITY ? DBL_MAX : (t == -INFINITY ? -DBL_MAX : t)); };
        u = fix(u);
        v = fix(v);
        w = fix(w);
    }
    U[vo] = u;
    V[vo] = v;
    W[vo] = w;
}

// sum_j c_j values[simplices[s, j]] in interpnd's order (from 0.0)
__device__ __forceinline__ void lin_interp(const LinearKernelArgs &a, int s, const double (&c)[4], double &u,
                                           double &v, double &w) {
    const int4 vs = reinterpret_cast<const int4 *>(a.simplices)[s];
    const int id[4] = {vs.x, vs.y, vs.z, vs.w};
    double ou = 0.0, ov = 0.0, ow = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ou = ou + c[j] * a.pu[id[j]];
        ov = ov + c[j] * a.pv[id[j]];
        ow = ow + c[j] * a.pw[id[j]];
    }
    u = ou;
    v = ov;
    w = ow;
}

__device__ __forceinline__ void lin_point(const LinearKernelArgs &a, long long v, const double *__restrict__ ax,
                                          const double *__restrict__ ay, const double *__restrict__ az,
                                          const double *__restrict__ qx, const double *__restrict__ qy,
                                          const double *__restrict__ qz, int &iz, size_t &vfull, double &x0,
                                          double &x1, double &x2) {
    const long long plane = (long long)a.nx * a.ny;
    iz = a.z0 + (int)(v / plane);
    const long long rem = v % plane;
    const int iy = (int)(rem / a.nx), ix = (int)(rem % a.nx);
    vfull = (size_t)iz * plane + rem;
    if (a.separable) {
        x0 = ax[ix];
        x1 = ay[iy];
        x2 = az[iz];
    } else {
        x0 = qx[vfull];
        x1 = qy[vfull];
        x2 = qz[vfull];
    }
}

// _is_point_fully_outside (spatial/_qhull.pyx)
__device__ __forceinline__ bool lin_outside(const LinearKernelArgs &a, double x0, double x1, double x2) {
    return x0 < a.lo[0] - kLinEps || x0 > a.hi[0] + kLinEps || x1 < a.lo[1] - kLinEps || x1 > a.hi[1] + kLinEps ||
           x2 < a.lo[2] - kLinEps || x2 > a.hi[2] + kLinEps;
}

__global__ __launch_bounds__(256) void k_linear_walk(LinearKernelArgs a, const double4 *__restrict__ prec,
                                                     const uint32_t *__restrict__ slots, const double *__restrict__ ax,
                                                     const double *__restrict__ ay, const double *__restrict__ az,
                                                     const double *__restrict__ qx, const double *__restrict__ qy,
                                                     const double *__restrict__ qz, const uint8_t *__restrict__ mask,
                                                     double *__restrict__ U, double *__restrict__ V,
                                                     double *__restrict__ W) {
    const long long nvox = (long long)(a.z1 - a.z0) * a.nx * a.ny;
    const long long nb = (nvox + 255) / 256;
    const long long b = lin_xcd_block((long long)blockIdx.y * gridDim.x + blockIdx.x, nb);
    if (b >= nb) return;
    const long long v = b * 256 + threadIdx.x;  // chunk-local voxel
    if (v >= nvox) return;
    int iz;
    size_t vfull;
    double x0, x1, x2;
    lin_point(a, v, ax, ay, az, qx, qy, qz, iz, vfull, x0, x1, x2);
    const size_t vo = (size_t)(iz - a.out_z0) * a.nx * a.ny + (size_t)(vfull % ((size_t)a.nx * a.ny));
    if (mask != nullptr && mask[vfull] == 0) {  // solid voxel: 0, not computed (main.py:202-207 fused)
        lin_store(a, U, V, W, vo, 0.0, 0.0, 0.0);
        return;
    }
    if (lin_outside(a, x0, x1, x2)) {
        lin_store(a, U, V, W, vo, a.fill, a.fill, a.fill);
        return;
    }
    // start: a simplex incident to the nearest particle
    const int orig = (int)prec[slots[v]].w;
    int s = a.v2s[orig];
    if (s < 0 || (long long)s >= a.nsimplex) s = 0;
    int res = -3;  // -3: brute force, -1: outside the hull, >= 0: the simplex
    double c[4];
    for (int it = 0; it < a.max_walk; ++it) {
        const double *T = a.transform + (size_t)s * 12;
        int hop = -1;
        bool inside = true;
        double acc = 1.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < 3) {
                c[k] = bary(T, k, x0, x1, x2);
                acc = acc - c[k];
            } else {
                c[3] = acc;
            }
            if (c[k] < -kLinEps) {
                hop = k;
                break;
            }
            inside = inside && (c[k] <= 1.0 + kLinEps);  // NaN (degenerate simplex) -> not inside
        }
        if (hop >= 0) {
            const int m = a.neighbors[(size_t)s * 4 + hop];
            if (m == -1) {
                res = -1;
                break;
            }
            s = m;
            continue;
        }
        res = inside ? s : -3;
        break;
    }
    if (res >= 0) {
        double u, vv, w;
        lin_interp(a, res, c, u, vv, w);
        lin_store(a, U, V, W, vo, u, vv, w);
        return;
    }
    lin_store(a, U, V, W, vo, a.fill, a.fill, a.fill);
    if (res == -3) {  // degenerate simplex on the way, or no convergence: brute force (rare)
        const int at = atomicAdd(a.flag_count, 1);
        if (at < a.flag_cap) a.flag_list[at] = v + (long long)(a.z0 - a.out_z0) * a.nx * a.ny;
    }
}

// scipy _find_simplex_bruteforce for the flagged voxels: the first simplex (index order) that
// accepts the point -- a valid one by _barycentric_inside, or, for a degenerate (NaN transform)
// simplex, its first valid neighbour that contains the point within eps (eps_broad towards the
// degenerate one).  One block per flagged voxel, 256 simplices per round, stop at the first hit.
__global__ __launch_bounds__(256) void k_linear_brute(LinearKernelArgs a, const double *__restrict__ ax,
                                                      const double *__restrict__ ay, const double *__restrict__ az,
                                                      const double *__restrict__ qx, const double *__restrict__ qy,
                                                      const double *__restrict__ qz, double *__restrict__ U,
                                                      double *__restrict__ V, double *__restrict__ W) {
    __shared__ int s_hit, s_res;
    const int nflag = min(*a.flag_count, a.flag_cap);
    const double eps_broad = 1.4901161193847656e-08;  // sqrt(DBL_EPSILON)
    for (int f = blockIdx.x; f < nflag; f += gridDim.x) {
        const long long vs = a.flag_list[f];  // slab-relative voxel
        LinearKernelArgs b = a;
        b.z0 = a.out_z0;
        int iz;
        size_t vfull;
        double x0, x1, x2;
        lin_point(b, vs, ax, ay, az, qx, qy, qz, iz, vfull, x0, x1, x2);
        const size_t vo = (size_t)vs;
        int bestr = -1;  // the result simplex of the first accepting simplex
        for (long long base = 0; base < a.nsimplex; base += 256) {
            const long long i = base + threadIdx.x;
            int r = -1;
            if (i < a.nsimplex) {
                const double *T = a.transform + (size_t)i * 12;
                if (T[0] == T[0]) {  // valid transform: _barycentric_inside
                    double acc = 1.0;
                    bool in = true;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const double ck = bary(T, k, x0, x1, x2);
                        acc = acc - ck;
                        in = in && (-kLinEps <= ck && ck <= 1.0 + kLinEps);
                    }
                    in = in && (-kLinEps <= acc && acc <= 1.0 + kLinEps);
                    if (in) r = (int)i;
                } else {
                    for (int k = 0; k < 4 && r < 0; ++k) {
                        const int nbh = a.neighbors[(size_t)i * 4 + k];
                        if (nbh == -1) continue;
                        const double *Tn = a.transform + (size_t)nbh * 12;
                        if (Tn[0] != Tn[0]) continue;
                        double cn[4];
                        double acc = 1.0;
                        for (int m = 0; m < 3; ++m) {
                            cn[m] = bary(Tn, m, x0, x1, x2);
                            acc = acc - cn[m];
                        }
                        cn[3] = acc;
                        bool in = true;
                        for (int m = 0; m < 4; ++m) {
                            const double lo = a.neighbors[(size_t)nbh * 4 + m] == (int)i ? -eps_broad : -kLinEps;
                            in = in && (lo <= cn[m] && cn[m] <= 1.0 + kLinEps);
                        }
                        if (in) r = nbh;
                    }
                }
            }
            if (threadIdx.x == 0) s_hit = 0x7fffffff;
            __syncthreads();
            if (r >= 0) atomicMin(&s_hit, (int)threadIdx.x);
            __syncthreads();
            const int h = s_hit;  // uniform: the lowest accepting simplex of this round, if any
            if (h != 0x7fffffff) {
                if ((int)threadIdx.x == h) s_res = r;
                __syncthreads();
                bestr = s_res;
                break;
            }
            __syncthreads();  // s_hit is reset next round
        }
        if (threadIdx.x == 0) {
            if (bestr >= 0) {
                const double *T = a.transform + (size_t)bestr * 12;
                double c[4];
                double acc = 1.0;
                for (int k = 0; k < 3; ++k) {
                    c[k] = bary(T, k, x0, x1, x2);
                    acc = acc - c[k];
                }
                c[3] = acc;
                double u, vv, w;
                lin_interp(a, bestr, c, u, vv, w);
                lin_store(a, U, V, W, vo, u, vv, w);
            }  // else: no simplex -> the fill value written by the walk stays
        }
        __syncthreads();
    }
}

int launch_linear(const LinearKernelArgs &a, const double4 *prec, const uint32_t *slots, const double *ax,
                  const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
                  const uint8_t *mask, double *U, double *V, double *W, hipStream_t s) {
    const long long nvox = (long long)(a.z1 - a.z0) * a.nx * a.ny;
    if (nvox <= 0) return PTV_OK;
    const long long nb = (nvox + 255) / 256;
    const unsigned gx = (unsigned)std::min<long long>(nb, 1 << 20);
    const unsigned gy = (unsigned)((nb + gx - 1) / gx);
    hipLaunchKernelGGL(k_linear_walk, dim3(gx, gy), dim3(256), 0, s, a, prec, slots, ax, ay, az, qx, qy, qz, mask, U,
                       V, W);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

int launch_linear_brute(const LinearKernelArgs &a, int nflag, const double *ax, const double *ay, const double *az,
                        const double *qx, const double *qy, const double *qz, double *U, double *V, double *W,
                        hipStream_t s) {
    if (nflag <= 0) return PTV_OK;
    hipLaunchKernelGGL(k_linear_brute, dim3((unsigned)std::min(nflag, 4096)), dim3(256), 0, s, a, ax, ay, az, qx, qy,
                       qz, U, V, W);
    PTV_HIP(hipGetLastError());
    return PTV_OK;
}

}  // namespace ptv
