// ptv_rbf_ns.hpp — local RBF by the null-space method (gfx950): the per-voxel saddle-point
// systems of the reference-reachable kernels (thin-plate spline, cubic, quintic, linear) and of
// every other kernel with a polynomial tail, solved with a STATIC elimination order.
//
// The system scipy builds per voxel (RBFInterpolator(neighbors=k), _rbfinterp.py:82-127, called
// from interpolator.py:162-167) is
//     [Phi  P] [c]   [d]        Phi = phi(eps |y_i - y_j|) + s_i delta_ij   (k x k, symmetric)
//     [P^T  0] [e] = [0]        P   = monomials of yhat                      (k x r, r = 1, 4, 10)
// and scipy factors it with LAPACK dgesv (partial pivoting).  Partial pivoting needs a
// data-dependent pivot row, and a 16-lane segment can only broadcast a COMPILE-TIME lane in
// registers (v_mov_b64_dpp row_newbcast): the pivoting kernel k_rbf_local pays an LDS round trip
// and two wave syncs per column for it (0.02-0.03 of FP64 peak).  For a
// conditionally positive definite kernel of order o with degree >= o - 1 (linear, multiquadric:
// o = 1; thin-plate spline, cubic: o = 2; quintic: o = 3; the positive definite gaussian /
// inverse multiquadric / inverse quadratic: o = 0) the same solution is, exactly in real
// arithmetic:
//     P = Q [Rt; 0]               Householder QR (r reflectors, LAPACK dlarfg form)
//     B = (Q^T Phi Q)[r:, r:]     symmetric positive definite: no pivoting needed
//     c~2 = B^-1 (Q^T d)[r:],  c = Q [0; c~2],  e = Rt^-1 ((Q^T d)[:r] - (Q^T Phi Q)[:r, r:] c~2)
// and every step of it has a fixed pivot / broadcast lane.  Measured against the reference
// fixtures and the extended-precision truth (tools/rbf_nullspace_proto.py, the same step order
// in numpy): 7e-14 (TPS k=20), 4e-13 (cubic), 1.1e-11 (quintic, cond 3.6e7) normwise from
// scipy's answers, within 1-8x of LAPACK's own distance to the exact solution.
//
// Anything outside that regime is flagged per voxel and re-solved by the pivoting kernel
// (k_rbf_local in list mode, the host launches it right after this kernel): a rank-deficient
// polynomial block (|Rt_tt| < 1e-9 sqrt(k): coplanar / collinear neighbourhoods, where LAPACK
// decides singularity), a pivot of B at or below 2^-40 of B's largest diagonal entry (singular to
// working precision: coincident neighbours) or outside the Newton reciprocal's range, a negative
// per-point smoothing, non-finite inputs.  So singular systems keep the pivoting kernel's (and
// LAPACK's) verdict.
//
// Layout (per wave: four systems, one per 16-lane row; lane li holds system rows li + 16 q,
// q < R, in registers):
//   A[R][NC]  rows of Phi, later Q^T Phi Q, later its LU;  P[R][NP] the polynomial block;
//   B[R][3]   right-hand sides (u, v, w);  V[NP][R] the reflectors (kept for Q^T phi(x)).
// Every cross-lane operand is a row_newbcast of a lane fixed at compile time (the loops are
// unrolled, rowbcast_n folds) or a segment sum (DPP + v_permlane*_swap-free 16-lane reduce).
#pragma once

#include "ptv_kernels.hpp"
#include "ptv_rbf_math.hpp"
#include "ptv_log_table.hpp"

namespace ptv {

// Symmetric build scratch: row i evaluates phi for the columns (i + d) mod NC, d = 1..H, into
// slot d - 1 of its scratch row; entry (i, j) is then row i's slot (j - i) mod NC - 1 when that
// is < H, else row j's slot (i - j) mod NC - 1.  Rows are HS doubles apart: H itself with an XOR
// swizzle when H is a power of two (the 16-lane stores and reads land in distinct banks), else
// the next odd number (an odd stride is conflict-free for 16 lanes of 8-byte accesses).
template <int NC>
struct NsBuild {
    static constexpr int H = NC / 2;
    static constexpr bool POW2 = (H & (H - 1)) == 0;
    static constexpr int HS = POW2 ? H : (H | 1);
    __device__ static __forceinline__ int addr(int row, int slot) {
        if constexpr (POW2) return row * HS + (slot ^ (row & (H - 1)));
        else return row * HS + slot;
    }
};

// _monomial_powers(3, degree) (_rbfinterp.py:48-79; monomial_powers in ptv_api.cpp) packed px | py
// << 8 | pz << 16: degree 0 is the first entry, degree 1 the first 4, degree 2 all 10 (the order is
// by degree, so NP alone fixes every exponent)
constexpr int kNsPow[10] = {0, 1, 256, 65536, 2, 1 | 256, 1 | 65536, 512, 256 | 65536, 131072};
template <int C>
__device__ __forceinline__ double ipow_c(double x) {
    if constexpr (C == 0) return 1.0;
    else if constexpr (C == 1) return x;
    else return x * x;
}
template <int T, int NP>
__device__ __forceinline__ void ns_prow(double (&row)[NP], const double4 &h, bool kr) {
    if constexpr (T < NP) {
        constexpr int c = kNsPow[T];
        if constexpr (T == 0) row[T] = kr ? 1.0 : 0.0;
        else row[T] = (ipow_c<(c & 255)>(h.x) * ipow_c<((c >> 8) & 255)>(h.y)) * ipow_c<(c >> 16)>(h.z);
        ns_prow<T + 1, NP>(row, h, kr);
    }
}



#ifndef PTV_NS_STAMP
#define PTV_NS_STAMP 0  // dev builds: per-wave s_memtime phase cycles into RbfKernelArgs::stamps
#endif
#if PTV_NS_STAMP
#define PTV_NS_MARK(i)                                         \
    do {                                                       \
        __builtin_amdgcn_sched_barrier(0);                     \
        ts[i] = __builtin_amdgcn_s_memtime();                  \
        __builtin_amdgcn_sched_barrier(0);                     \
    } while (0)
#else
#define PTV_NS_MARK(i) \
    do {               \
    } while (0)
#endif

// log(x) for finite x > 0 within ~3 ulp by table reduction (tools/gen_log_table.py): x = m 2^e,
// the bin of m's top 9 fraction bits gives y = f m in [3/4, 3/2) with exponent e' and (s = f/c, T =
// log c); r = m s - 1 (|r| <= 2^-10, one fma), log x = e' ln 2 + T + log1p(r), log1p by its degree-6
// Taylor polynomial.  ~12 VALU and one 16-byte table read where fdlibm's reduction (a division)
// takes ~25.  The two bins that touch y = 1 have c = 1, so near x = 1 the result is log1p(r) alone.
__device__ __forceinline__ double log_tab(double x, const double2 *__restrict__ lt) {
    const double m = __builtin_amdgcn_frexp_mant(x);
    const int e = __builtin_amdgcn_frexp_exp(x);
    const int i = (__double2hiint(m) >> 11) & 511;
    const double2 st = lt[i];
    const double r = fma(m, st.x, -1.0);
    const double t = fma((double)(i < 256 ? e - 1 : e), 0x1.62e42fefa39efp-1, st.y);
    double h = fma(r, -1.0 / 6.0, 0.2);
    h = fma(r, h, -0.25);
    h = fma(r, h, 1.0 / 3.0);
    h = fma(r, h, -0.5);
    return t + fma(r * r, h, r);
}

// phi of the scale-invariant kernels from the squared distance d2 = r^2 (scipy's
// _rbfinterp_pythran forms up to rounding: the thin-plate spline as d2 log(d2) / 2, which needs no
// square root; r^3 = d2 r, -r^5 = -(d2 d2) r).  A few ulps from scipy's r**2*log(r), far inside
// what the solve amplifies (cond <= ~1e7 for these systems: 1e-9 relative at worst, 1e-13 typical).
template <int KERN>
__device__ __forceinline__ double phi_ns_t(double d2, const double2 *__restrict__ lt) {
    // log_tab(0) is finite (m = 0: r = -1), so d2 = 0 gives 0 with no test
    if constexpr (KERN == PTV_RBF_THIN_PLATE_SPLINE) return (0.5 * d2) * log_tab(d2, lt);
    if constexpr (KERN == PTV_RBF_CUBIC) return d2 * sqrt_spd(d2);
    if constexpr (KERN == PTV_RBF_QUINTIC) return -((d2 * d2) * sqrt_spd(d2));
    return -sqrt_spd(d2);  // linear
}
__device__ __forceinline__ double phi_ns(int kern, double d2, const double2 *__restrict__ lt) {
    switch (kern) {
        case PTV_RBF_THIN_PLATE_SPLINE: return phi_ns_t<PTV_RBF_THIN_PLATE_SPLINE>(d2, lt);
        case PTV_RBF_CUBIC: return phi_ns_t<PTV_RBF_CUBIC>(d2, lt);
        case PTV_RBF_QUINTIC: return phi_ns_t<PTV_RBF_QUINTIC>(d2, lt);
        default: return phi_ns_t<PTV_RBF_LINEAR>(d2, lt);
    }
}

#ifndef PTV_NS_LDS_PAD
#define PTV_NS_LDS_PAD 1  // dev builds: 0 = the round-4 build scratch layout (stride NC + 1, unpadded systems)
#endif
// LDS banks (MI355X_MICROARCH.md §LDS): ds_read_b64 serves 32 lanes (two systems) per cycle on 64
// dword banks, ds_write_b64 16 lanes on 32, ds_read_b128 16-lane groups mixing two systems.  The
// full-matrix build scratch (<= 20 row slots) has an EVEN row stride NC + 2: the build's writes of
// (i, i + d) and (i + d, i) step 2 (MS + 1) dwords per lane, distinct banks for 16 lanes (NC + 1 put
// lanes i and i + 8 on one bank); the read-back's rows MS doubles apart land on the 16 even double
// positions mod 32, and the next system starts an ODD number of doubles later, so the two systems of
// one 32-lane group read disjoint banks.  The half scheme's odd row stride (24 slots) takes 16 of the
// 32 positions, its complement 16 doubles on.  The eps-scaled coordinates of the next system start
// 16 bytes (an odd bank quad) further on, so the ds_read_b128 groups' two systems meet no common quad.
// 32 slots stay as they were: two blocks per CU already take the whole LDS.
template <int NC>
constexpr int ns_full_stride() { return PTV_NS_LDS_PAD ? NC + 2 : NC + 1; }
template <int NC, bool FULL>
constexpr int ns_sys_stride() {
    const int base = FULL ? NC * ns_full_stride<NC>() : NC * NsBuild<NC>::HS;
    if (!PTV_NS_LDS_PAD || (!FULL && !(NsBuild<NC>::HS & 1))) return base;  // pow2 half scheme: LDS-bound, as is
    const int want = FULL ? 1 : 16;                                          // offset mod 32 doubles
    return base + ((want - base % 32) + 32) % 32;
}
template <int NC>
constexpr int ns_ye_stride() { return PTV_NS_LDS_PAD && NC <= 24 ? 2 * NC + 1 : 2 * NC; }  // in double2 (16 B); 32 slots: LDS full

// The symmetric build's phi entries: the NC x H (row i, column (i + d) mod NC) entries as one list
// dealt round-robin over the 16 lanes of a system (ceil(NC H / 16) phi per lane: 13 at 20 slots, 18
// at 24, where one row per lane-set costs R H = 20, 24), each written where the read-back finds it
// (the full matrix, or NsBuild's half scheme).  One instantiation per kernel function, the loop
// unrolled by 4 so that independent phi chains (and their LDS loads) overlap.
template <int KERN, int NC, bool FULL>
__device__ __forceinline__ void ns_build(double *__restrict__ ss, const double4 *__restrict__ ye, int li, int k,
                                         const double2 *__restrict__ lt) {
    using Bd = NsBuild<NC>;
    constexpr int H = Bd::H, MS = ns_full_stride<NC>();
    constexpr int NSLOT = NC * H;
    constexpr int SPL = (NSLOT + 15) / 16;
    static_assert(NC >= 16, "at most one wrap of the row index per step");
    int i = li, dd = 1;  // entry p = sl * 16 + li is (row i, column (i + dd) mod NC), p = (dd - 1) NC + i
    // branch-free, fully unrolled (the entries' LDS reads and phi chains overlap): rows >= k hold
    // stale coordinates, their phi is computed and dropped
#pragma unroll
    for (int sl = 0; sl < SPL; ++sl, i += 16, dd += i >= NC ? 1 : 0, i -= i >= NC ? NC : 0) {
        if (NSLOT % 16 == 0 || sl + 1 < SPL || sl * 16 + li < NSLOT) {
            int j = i + dd;
            j -= j >= NC ? NC : 0;
            const double4 yv = ye[i], yj = ye[j];
            const double dx = yv.x - yj.x, dy = yv.y - yj.y, dz = yv.z - yj.z;
            const double ph = phi_ns_t<KERN>((dx * dx + dy * dy) + dz * dz, lt);
            const double e = i < k && j < k ? ph : 0.0;
            if constexpr (FULL) {
                ss[i * MS + j] = e;
                ss[j * MS + i] = e;
            } else {
                ss[Bd::addr(i, dd - 1)] = e;
            }
        }
    }
}

// rank[q] += #{sources j >= J: id_j < id[q]}, source j = lane j % 16 of row set j / 16 (row_newbcast)
template <int J, int NC, int R>
__device__ __forceinline__ void ns_rank(const uint32_t (&id)[R], int (&rank)[R]) {
    if constexpr (J < NC) {
        const uint32_t o = dpp_u32<0x150 + (J & 15)>(id[J >> 4]);
#pragma unroll
        for (int q = 0; q < R; ++q) rank[q] += o < id[q] ? 1 : 0;
        ns_rank<J + 1, NC, R>(id, rank);
    }
}

// one neighbour's particle record: position, velocity, index (zeros when not loaded)
// (loaded unconditionally from an in-range slot and selected where used: a load under a branch
// makes the compiler copy its result at the branch's end, which waits for every load in flight)
struct NsRec {
    double x, y, z, id, u, v, w;
};
__device__ __forceinline__ NsRec ns_rec(const double4 *__restrict__ prec, const double4 *__restrict__ pval,
                                        uint32_t sl) {
    const double4 p = prec[sl];
    const double *q = reinterpret_cast<const double *>(pval + sl);
    return NsRec{p.x, p.y, p.z, p.w, q[0], q[1], q[2]};
}

template <int NC, int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_rbf_ns(
    RbfKernelArgs a, const double4 *__restrict__ prec, const double4 *__restrict__ pval,
    const uint32_t *__restrict__ slots, const double *__restrict__ ax, const double *__restrict__ ay,
    const double *__restrict__ az, const double *__restrict__ qpx, const double *__restrict__ qpy,
    const double *__restrict__ qpz, const double *__restrict__ smooth, const int *__restrict__ pw,
    const uint8_t *__restrict__ mask, double *__restrict__ U, double *__restrict__ V, double *__restrict__ W,
    int *__restrict__ status) {
    static_assert(NC % 4 == 0 && NC >= 16 && NC <= 32, "row slots");
    (void)pw;  // the exponents are fixed by NP (kNsPow)
    static_assert(NP >= 1 && NP < 16 && NP < NC, "polynomial terms (rows 0..NP-1 in lanes 0..NP-1)");
    constexpr int R = (NC + 15) / 16;
    using Bd = NsBuild<NC>;
    constexpr int H = Bd::H;
    // build scratch per wave (doubles): up to 20 row slots the full symmetric matrix (row stride
    // NC + 1, odd: conflict-free 16-lane rows and columns; every entry read back with a constant
    // offset, no per-entry address arithmetic), above that the half-matrix scheme of NsBuild
    constexpr bool FULL = NC <= 20;
    constexpr int MS = ns_full_stride<NC>();
    constexpr int SYS = ns_sys_stride<NC, FULL>();
    constexpr int SCS = 4 * SYS;
    constexpr int SVS = 4 * NC * 8;  // sorted (values, yhat) double4 pairs per wave
    constexpr int SRS = NP * R * 64 + 4 * (2 * NP + 1);  // reflectors (per lane) + tau, beta, pivot tolerance (per system)
    constexpr int SC0 = SCS > SVS ? SCS : SVS;
    constexpr int SC = SC0 > SRS ? SC0 : SRS;
    constexpr int YES = ns_ye_stride<NC>();
    __shared__ double2 s_ye[4][4 * YES];  // per wave and system (YES double2 apart): eps-scaled coordinates + id, id order
    __shared__ double s_sc[4][SC];
    // the log's reduction table: in LDS up to 24 slots (8 KB; two blocks per CU still fit), read
    // from global memory (L1) at 32, where the two blocks' scratch takes the whole LDS
    constexpr bool LDS_LT = NC <= 24;
    __shared__ double2 s_lt[LDS_LT ? 512 : 1];
    const double2 *lt = reinterpret_cast<const double2 *>(kLogTab);
    if constexpr (LDS_LT) {
        for (int i = threadIdx.x; i < 512; i += 256) s_lt[i] = lt[i];
        __syncthreads();
        lt = s_lt;
    }
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: the quad loop is scalar

    const long long plane = (long long)a.nx * a.ny;
    const long long nvox = (long long)(a.z1 - a.z0) * plane;
    const int k = a.k;
    const double eps = a.epsilon;
    // Persistent waves, one quad (4 voxels, one per 16-lane system) at a time.  XCD-aware: block b
    // runs on XCD b mod 8 (round-robin dispatch), and XCD x owns the contiguous eighth x of the
    // quads, so the neighbourhoods one XCD gathers overlap in its own L2.  The next quad's slots
    // and particle records are loaded while this one solves (slots after step 1, records after
    // step 3): the gather latency that one quad per wave exposes (a quarter of the cycles) hides.
    const long long nquad = (nvox + 3) / 4;
    const int xcd = (int)(blockIdx.x & 7u);
    const long long qend = nquad * (xcd + 1) / 8;
    const long long qstep = (long long)(gridDim.x >> 3) * 4;
    long long qd = nquad * xcd / 8 + (long long)(blockIdx.x >> 3) * 4 + wid;
    // records in flight: 13 VGPRs per row slot; at 32 slots the solve leaves no room for them, and
    // only the slots are prefetched (the records then load at the top of the quad)
    constexpr bool PFR = NC <= 24;
    uint32_t nsl[R];
    NsRec nrec[R];
    bool nvv;  // the next quad's voxel is in range
    uint32_t nmb;  // its mask byte
    int nz;
    long long nrem;
    double nq[3];
    // the quad after this one: voxel (z plane, in-plane offset, coordinates), mask byte and slots,
    // all loaded from in-range addresses without branches; validity applies where they are used
    auto stage1 = [&](long long qn, int seg, int li) {
        const long long vn = qn * 4 + seg;
        nvv = qn < qend && vn < nvox;
        const long long vc = nvv ? vn : nvox - 1;
        // 32-bit divisions (the launch has <= 2^32 voxels, so the offsets fit; one plane of exactly
        // 2^32 voxels takes the 64-bit branch, uniform)
        uint32_t pz, pr;
        if (plane <= 0xffffffffLL) {
            const uint32_t v32 = (uint32_t)vc, p32 = (uint32_t)plane;
            pz = v32 / p32;
            pr = v32 - pz * p32;
        } else {
            pz = (uint32_t)(vc / plane);
            pr = (uint32_t)(vc - (long long)pz * plane);
        }
        nz = a.z0 + (int)pz;
        nrem = pr;
        const uint32_t iyu = pr / (uint32_t)a.nx;
        const int iy = (int)iyu, ix = (int)(pr - iyu * (uint32_t)a.nx);
        const size_t vfull = (size_t)nz * plane + nrem;
        nmb = *(mask != nullptr ? mask + vfull : &kNsMaskOn);
        const bool sep = a.separable != 0;
        nq[0] = *(sep ? ax + ix : qpx + vfull);
        nq[1] = *(sep ? ay + iy : qpy + vfull);
        nq[2] = *(sep ? az + nz : qpz + vfull);
#pragma unroll
        for (int q = 0; q < R; ++q) nsl[q] = slots[(size_t)vc * k + (li + 16 * q < k ? li + 16 * q : k - 1)];
    };
    // stage 2 (or the top of the quad, without record prefetch): the records of the slots in use
    auto stage2 = [&](int li) {
        const bool act = nvv && nmb != 0u;
#pragma unroll
        for (int q = 0; q < R; ++q) nrec[q] = ns_rec(prec, pval, act && li + 16 * q < k ? nsl[q] : 0u);
    };
    {
        const int seg = (threadIdx.x & 63) >> 4, li = threadIdx.x & 15;
        stage1(qd, seg, li);
        if constexpr (PFR) stage2(li);
    }
    // a quad's outputs are stored after the next quad's records are in use: stores count in vmcnt,
    // and stored right away they would hold up the wait for those records at the top of the loop
    bool pend = false;
    size_t pvo = 0;
    double po[3] = {0.0, 0.0, 0.0};
    auto flush = [&]() {
        if (pend) {
            U[pvo] = po[0];
            V[pvo] = po[1];
            W[pvo] = po[2];
        }
        pend = false;
    };
    for (; qd < qend; qd += qstep) {
    // the lane index re-derived opaquely each quad: nothing lane-dependent (the many LDS addresses
    // of the unrolled steps) is hoisted out of the loop to stay live across the solve
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const int seg = lane >> 4, li = lane & 15;
    double4 *ye = reinterpret_cast<double4 *>(s_ye[wid] + seg * YES);  // 16-B aligned (ds_read_b128 pairs)
    double *sc = s_sc[wid];
    double4 *sv = reinterpret_cast<double4 *>(sc) + seg * NC * 2;  // row r: sv[2r] values, sv[2r+1] yhat
    const long long v = qd * 4 + seg;  // chunk-local voxel
    const bool valid = v < nvox;
    const int iz = nz;
    const long long rem = nrem;
    const bool active = nvv && nmb != 0u;
    const double qx = nq[0], qy = nq[1], qz = nq[2];
    if constexpr (!PFR) stage2(li);
#if PTV_NS_STAMP
    unsigned long long ts[9];
#endif
    PTV_NS_MARK(0);

    // ---- 1. neighbours li + 16 q, ranked by particle index (np.sort(yindices), _rbfinterp.py:521);
    //      the polynomial coordinates' scale ----
    double4 r[R], d[R];
    uint32_t id[R];
    double ro = 0.0;  // max-norm offset of this lane's neighbours from the voxel
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int nbr = li + 16 * q;
        const bool ld = active && nbr < k;
        r[q] = ld ? make_double4(nrec[q].x, nrec[q].y, nrec[q].z, 0.0) : make_double4(0.0, 0.0, 0.0, 0.0);
        d[q] = ld ? make_double4(nrec[q].u, nrec[q].v, nrec[q].w, 0.0) : make_double4(0.0, 0.0, 0.0, 0.0);
        id[q] = 0xffffffffu;
        if (ld) {
            id[q] = (uint32_t)nrec[q].id;
            ro = fmax(ro, fmax(fabs(r[q].x - qx), fmax(fabs(r[q].y - qy), fabs(r[q].z - qz))));
        }
    }
    flush();  // the previous quad's outputs, now that this quad's records are in registers
    // The polynomial block's coordinates: yhat = (y - x) / rho, centred on the voxel x and scaled by
    // the neighbourhood's max-norm radius rho (in [-1, 1]^3).  scipy centres and scales per axis on
    // the neighbourhood's box (_build_system); the polynomials of degree <= d span the same space
    // under any affine change of coordinates, so the interpolant is the same up to rounding, and
    // the null-space basis Q of P (its span) does not depend on the column scaling at all.  One
    // reduction where the box takes six, and P(xhat) at the voxel is (1, 0, ..., 0).
    const double rho = seg_max<16>(ro);
    const double irho = rho > 0.0 ? rcp_nr(rho) : 1.0;
    const double pm = li == 0 ? 1.0 : 0.0;
    // rank = the number of smaller particle indices in the neighbourhood (the k slots hold distinct
    // particles; unused slots hold 0xffffffff and count for nobody), each source broadcast by DPP
    int rank[R];
#pragma unroll
    for (int q = 0; q < R; ++q) rank[q] = 0;
    ns_rank<0, NC, R>(id, rank);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        if (li + 16 * q < k) {
            ye[rank[q]] = make_double4(r[q].x * eps, r[q].y * eps, r[q].z * eps, (double)id[q]);
            sv[2 * rank[q]] = d[q];
            sv[2 * rank[q] + 1] = make_double4((r[q].x - qx) * irho, (r[q].y - qy) * irho, (r[q].z - qz) * irho, 0.0);
        }
    }
    rbf_wave_sync();
    double4 yi[R], hh[R];  // own rows' eps-scaled coordinates (build only: reloaded for the evaluation), yhat
    double B[R][3], dg[R];
    bool bad = false;
    const double phi0 = phi_ns(a.kernel, 0.0, lt);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int row = li + 16 * q;
        const bool kr = row < k;
        yi[q] = kr ? ye[row] : make_double4(0.0, 0.0, 0.0, 0.0);
        const double4 dv = kr ? sv[2 * row] : make_double4(0.0, 0.0, 0.0, 0.0);
        hh[q] = kr ? sv[2 * row + 1] : make_double4(0.0, 0.0, 0.0, 0.0);
        B[q][0] = dv.x;
        B[q][1] = dv.y;
        B[q][2] = dv.z;
        double si = 0.0;
        if (kr && active) si = smooth != nullptr ? smooth[(size_t)yi[q].w] : a.smoothing;
        // consumed here, before the next quad's loads issue: a later first use would wait for those too
        asm volatile("" : "+v"(si));
        // negative smoothing: not positive definite any more; smoothing far above the phi entries'
        // scale (> 2^26): the rank-2r update then cancels the O(1) entries against it, inaccurately
        // and without a telltale pivot (2e307 on every fifth diagonal left one wrong voxel in 1000)
        bad = bad || si < 0.0 || si > 0x1p26;
        dg[q] = kr ? phi0 + si : 1.0;  // padded rows: identity block
    }
    {  // prefetch, stage 1: the next quad's slots
        stage1(qd + qstep, seg, li);
    }
    // P rows: monomials of yhat, exponents fixed by NP at compile time (kNsPow; unused rows have
    // yhat = 0, so only the constant column needs the row test)
    double P[R][NP];
#pragma unroll
    for (int q = 0; q < R; ++q) ns_prow<0, NP>(P[q], hh[q], li + 16 * q < k);
    PTV_NS_MARK(1);
    // ---- 2. Householder QR of P alone (the reflectors depend on P only; dlarfg: beta = -sign(alpha)
    //      ||x||, tau = (beta - alpha)/beta, v = x / (alpha - beta), v_t = 1), applied to P's later
    //      columns (P[0][u], u > t, of lane t ends as Rt's row t) and to the right-hand sides ----
    const double rank_tol = 1e-9 * sqrt((double)k);
    double Vr[NP][R], tau[NP], beta[NP];
#pragma unroll
    for (int t = 0; t < NP; ++t) {
        const double alpha = rowbcast_n(t, P[0][t]);
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const double x = li + 16 * q > t ? P[q][t] : 0.0;
            s = fma(x, x, s);
        }
        s = seg_sum<16>(s);
        const double nrm = sqrt(alpha * alpha + s);
        const bool triv = !(s > 0.0);
        const double b = triv ? alpha : (alpha >= 0.0 ? -nrm : nrm);
        // Newton reciprocals (a column this small is flagged rank-deficient below and re-solved)
        tau[t] = triv ? 0.0 : (b - alpha) * rcp_nr(b);
        beta[t] = b;
        const double scal = triv ? 0.0 : rcp_nr(alpha - b);
        bad = bad || !(fabs(b) >= rank_tol);
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            Vr[t][q] = row > t ? P[q][t] * scal : (row == t ? 1.0 : 0.0);
        }
#pragma unroll
        for (int u = t + 1; u < NP; ++u) {
            double w = 0.0;
#pragma unroll
            for (int q = 0; q < R; ++q) w = fma(Vr[t][q], P[q][u], w);
            w = seg_sum<16>(w) * tau[t];
#pragma unroll
            for (int q = 0; q < R; ++q) P[q][u] = fma(-w, Vr[t][q], P[q][u]);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double w = 0.0;
#pragma unroll
            for (int q = 0; q < R; ++q) w = fma(Vr[t][q], B[q][c], w);
            w = seg_sum<16>(w) * tau[t];
#pragma unroll
            for (int q = 0; q < R; ++q) B[q][c] = fma(-w, Vr[t][q], B[q][c]);
        }
    }
    double Rt[NP];  // this lane's row of Rt (lanes < NP)
#pragma unroll
    for (int t = 0; t < NP; ++t) Rt[t] = P[0][t];
    rbf_wave_sync();  // the values' LDS is the build scratch next

    PTV_NS_MARK(2);
    // ---- 3. symmetric build of Phi (NsBuild), read back row by row with y_t = Phi v_t accumulated ----
    double *ss = sc + seg * SYS;
    if constexpr (FULL) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            if (16 * q + 15 < NC || row < NC) ss[row * MS + row] = dg[q];
        }
    }
    switch (a.kernel) {
        case PTV_RBF_THIN_PLATE_SPLINE: ns_build<PTV_RBF_THIN_PLATE_SPLINE, NC, FULL>(ss, ye, li, k, lt); break;
        case PTV_RBF_CUBIC: ns_build<PTV_RBF_CUBIC, NC, FULL>(ss, ye, li, k, lt); break;
        case PTV_RBF_QUINTIC: ns_build<PTV_RBF_QUINTIC, NC, FULL>(ss, ye, li, k, lt); break;
        default: ns_build<PTV_RBF_LINEAR, NC, FULL>(ss, ye, li, k, lt);
    }
    rbf_wave_sync();
    PTV_NS_MARK(3);
    double A[R][NC], Y[NP][R];
#pragma unroll
    for (int t = 0; t < NP; ++t)
#pragma unroll
        for (int q = 0; q < R; ++q) Y[t][q] = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            if constexpr (FULL) {
                // lanes past the last row slot read a real row (finite values; those rows never
                // pivot and never reach an output)
                const int rr = row < NC ? row : row - 16;
                A[q][j] = ss[rr * MS + j];
            } else {
                int dj = j - row;
                dj += dj < 0 ? NC : 0;  // (j - row) mod NC for row < NC
                const int own = Bd::addr(row < NC ? row : 0, dj >= 1 && dj <= H ? dj - 1 : 0);
                const int par = Bd::addr(j, dj > H && dj < NC ? NC - dj - 1 : 0);
                const double e = ss[dj <= H ? own : par];
                A[q][j] = row >= NC ? 0.0 : (dj == 0 ? dg[q] : e);
            }
        }
#pragma unroll
        for (int t = 0; t < NP; ++t) {
            if (j < t) continue;  // v_t is zero above row t
            double col[R];
#pragma unroll
            for (int q = 0; q < R; ++q) col[q] = A[q][j];
            fmac_bc_n<R>(j, Y[t], Vr[t][j >> 4], col);  // Y_t += A[:, j] v_t[j]
        }
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // bounded reads in flight
    }
    rbf_wave_sync();  // every lane has its rows: the scratch now keeps the reflectors for step 8
    if constexpr (PFR) stage2(li);  // prefetch, stage 2: the next quad's particle records
    double *vst = sc;                                  // V[t][q] at vst[(t * R + q) * 64 + lane]
    double *tbs = sc + NP * R * 64 + seg * (2 * NP + 1);  // tau[t], beta[t], pivot tolerance of this system
    static_assert(SRS <= SC, "reflector store fits the scratch");
#pragma unroll
    for (int t = 0; t < NP; ++t) {
#pragma unroll
        for (int q = 0; q < R; ++q) vst[(t * R + q) * 64 + lane] = Vr[t][q];
        if (li == 0) {
            tbs[t] = tau[t];
            tbs[NP + t] = beta[t];
        }
    }

    PTV_NS_MARK(4);
    // ---- 4. Q^T Phi Q = Phi - sum_t (v_t z_t^T + z_t v_t^T), the reflectors applied in turn
    //      (H_t Phi_t H_t = Phi_t - v z^T - z v^T with p = tau Phi_t v, z = p - tau (v.p)/2 v):
    //      Phi_t v_t = y_t - sum_{s<t} (v_s (z_s.v_t) + z_s (v_s.v_t)).  Only the columns >= NP are
    //      kept (B and the e right-hand side's block); columns < NP are dead ----
#pragma unroll
    for (int t = 0; t < NP; ++t) {
#pragma unroll
        for (int s2 = 0; s2 < t; ++s2) {
            double zv = 0.0, vv = 0.0;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                zv = fma(Y[s2][q], Vr[t][q], zv);  // Y[s2] holds z_s2 by now
                vv = fma(Vr[s2][q], Vr[t][q], vv);
            }
            zv = seg_sum<16>(zv);
            vv = seg_sum<16>(vv);
#pragma unroll
            for (int q = 0; q < R; ++q) Y[t][q] = fma(-Vr[s2][q], zv, fma(-Y[s2][q], vv, Y[t][q]));
        }
        double kk = 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            Y[t][q] = Y[t][q] * tau[t];
            kk = fma(Vr[t][q], Y[t][q], kk);
        }
        kk = 0.5 * tau[t] * seg_sum<16>(kk);
#pragma unroll
        for (int q = 0; q < R; ++q) Y[t][q] = fma(-kk, Vr[t][q], Y[t][q]);  // z_t
    }
    // the projected block's largest diagonal entry, B_jj = Phi_jj - 2 sum_t v_t[j] z_t[j] over this
    // lane's rows NP <= j < k: the scale of the relative pivot test in step 5
    double dgb = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int row = li + 16 * q;
        double bjj = dg[q];
#pragma unroll
        for (int t = 0; t < NP; ++t) bjj = fma(-2.0 * Vr[t][q], Y[t][q], bjj);
        dgb = row >= NP && row < k ? fmax(dgb, bjj) : dgb;
    }
    // a pivot at or below 2^-40 of it: the block is singular to working precision (coincident
    // neighbours make it exactly singular, e_i - e_j lies in the null space of P^T and of Phi, and
    // rounding leaves a last pivot of ~1e-16 relative and either sign), so the voxel goes to the
    // pivoting kernel, which meets LAPACK's verdict; a legitimate system with cond ~1e8 keeps
    // pivots near 1e-8 of it.  Kept in LDS (tested against the reciprocals after step 6: a register
    // live across the LU spills at 32 slots)
    dgb = 0x1p-40 * seg_max<16>(dgb);
    if (li == 0) tbs[2 * NP] = dgb;
    double nV[NP][R], nY[NP][R];  // negated: A += nY v[j] + nV z[j], each an fmac with the broadcast folded
#pragma unroll
    for (int t = 0; t < NP; ++t)
#pragma unroll
        for (int q = 0; q < R; ++q) {
            nV[t][q] = -Vr[t][q];
            nY[t][q] = -Y[t][q];
        }
#pragma unroll
    for (int j = NP; j < NC; ++j) {
        double col[R];
#pragma unroll
        for (int q = 0; q < R; ++q) col[q] = A[q][j];
#pragma unroll
        for (int t = 0; t < NP; ++t) {
            fmac_bc_n<R>(j, col, Vr[t][j >> 4], nY[t]);  // - z_t v_t[j]
            fmac_bc_n<R>(j, col, Y[t][j >> 4], nV[t]);   // - v_t z_t[j]
        }
#pragma unroll
        for (int q = 0; q < R; ++q) A[q][j] = col[q];
        if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bounded broadcasts in flight
    }

    PTV_NS_MARK(5);
    // ---- 5. LU without pivoting of B = rows / columns NP..NC-1 (pivot row c = lane c % 16 of row
    //      set c / 16, look-ahead by one column as k_rbf_spd16); rows < NP are never updated ----
    double rd[R];
#pragma unroll
    for (int q = 0; q < R; ++q) rd[q] = 1.0;
    double piv = rowbcast_n(NP, A[NP / 16][NP]);
    double rp = rcp_nr(piv);
#pragma unroll
    for (int c = NP; c < NC; ++c) {
        const int pq = c / 16;
        bad = bad || !(piv > 0.0);
        rd[pq] = li == (c & 15) ? rp : rd[pq];
        // negated multipliers (A += l u, the pivot row's u broadcast inside the fmac); the live row
        // sets are pq..R-1 (a set wholly above the pivot is finished)
        const double nrp = -rp;
        double l[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            if (16 * q + 15 <= c) l[q] = 0.0;
            else if (16 * q > c) l[q] = A[q][c] * nrp;
            else l[q] = row > c ? A[q][c] * nrp : 0.0;
        }
        double pivn = 1.0, rpn = 1.0;
#pragma unroll
        for (int j = c + 1; j < NC; ++j) {
            if (R == 2 && pq == 0) fmac_bc_piv_n(c, A[R - 1][j], A[0][j], l[R - 1], l[0]);
            else fmac_bc_self_n(c, A[pq][j], l[pq]);
            if (j == c + 1) {
                pivn = rowbcast_n(c + 1, A[(c + 1) / 16][c + 1]);
                rpn = rcp_nr(pivn);
            }
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (R == 2 && pq == 0) fmac_bc_piv_n(c, B[R - 1][t], B[0][t], l[R - 1], l[0]);
            else fmac_bc_self_n(c, B[pq][t], l[pq]);
        }
        piv = pivn;
        rp = rpn;
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const double ar = fabs(rd[q]);
        bad = bad || !(ar >= 0x1p-1020 && ar <= 0x1p1020);  // the Newton reciprocal's range
    }

    PTV_NS_MARK(6);
    // ---- 6. back substitution x_c = b_c / U_cc (c >= NP) from lane c % 16; every row above c is
    //      updated, so rows < NP end with (Q^T d)[:r] - (Q^T Phi Q)[:r, r:] c~2, e's right-hand side ----
#pragma unroll
    for (int c = NC - 1; c >= NP; --c) {
        const int pq = c / 16;
        double u[R];  // this lane's U entries of column c (rows above c), the rest 0
#pragma unroll
        for (int q = 0; q < R; ++q) u[q] = li + 16 * q < c ? A[q][c] : 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const double nx = -(B[pq][t] * rd[pq]);  // -x_c on lane c % 16
            if (R == 2 && pq == 1) {
                double bb[2] = {B[0][t], B[R - 1][t]};
                const double uu[2] = {u[0], u[R - 1]};
                fmac_bc_n<2>(c, bb, nx, uu);
                B[0][t] = bb[0];
                B[R - 1][t] = bb[1];
            } else {
                double bb[1] = {B[0][t]};
                const double uu[1] = {u[0]};
                fmac_bc_n<1>(c, bb, nx, uu);
                B[0][t] = bb[0];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < R; ++q)
#pragma unroll
        for (int t = 0; t < 3; ++t) B[q][t] = B[q][t] * rd[q];

    // ---- 7. Rt e = rhs (rows 0..NP-1: lanes 0..NP-1; Rt_it = P[0][t] of lane i < t, diag beta) ----
    rbf_wave_sync();  // the reflector store is read back from here on
    {
        // the relative pivot test of step 4's tolerance: piv <= tol <=> 1/piv >= 1/tol (piv > 0 by now)
        const double ptol = tbs[2 * NP];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            if (row >= NP && row < k) bad = bad || !(rd[q] * ptol < 1.0);
        }
    }
    double E[3] = {0.0, 0.0, 0.0}, rh[3] = {B[0][0], B[0][1], B[0][2]};
#pragma unroll
    for (int t = NP - 1; t >= 0; --t) {
        const double rbt = rcp_nr(tbs[NP + t]);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double et = rowbcast_n(t, rh[c] * rbt);
            E[c] = li == t ? et : E[c];
            rh[c] = li < t ? fma(-Rt[t], et, rh[c]) : rh[c];
        }
    }

    PTV_NS_MARK(7);
    // ---- 8. evaluate: out = (Q^T phi(x))[r:] . c~2 + P(xhat) . e ----
    double ph[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {  // branch-free: slots past k (stale coordinates) are dropped
        const int row = li + 16 * q;
        const double4 y = ye[16 * q + 15 < NC || row < NC ? row : row - 16];
        const double dx = qx * eps - y.x, dy = qy * eps - y.y, dz = qz * eps - y.z;
        const double f = phi_ns(a.kernel, (dx * dx + dy * dy) + dz * dz, lt);
        ph[q] = row < k ? f : 0.0;
    }
#pragma unroll
    for (int t = 0; t < NP; ++t) {
        double vt[R], w = 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            vt[q] = vst[(t * R + q) * 64 + lane];
            w = fma(vt[q], ph[q], w);
        }
        w = seg_sum<16>(w) * tbs[t];
#pragma unroll
        for (int q = 0; q < R; ++q) ph[q] = fma(-w, vt[q], ph[q]);
    }
    double o[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        o[c] = li < NP ? pm * E[c] : 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = li + 16 * q;
            if (row >= NP && row < NC) o[c] = fma(ph[q], B[q][c], o[c]);
        }
        o[c] = seg_sum<16>(o[c]);
    }
    const bool segbad = seg_max_u32<16>((bad && active) ? 1u : 0u) != 0u;
    PTV_NS_MARK(8);
#if PTV_NS_STAMP
    if (a.stamps != nullptr && lane == 0) {
        if (qd < a.stamp_cap)
            for (int i = 0; i < 8; ++i) a.stamps[qd * 8 + i] = ts[i + 1] - ts[i];
    }
#endif
    if (valid && li == 0) {
        if (active && segbad) {  // re-solved by the pivoting kernel (k_rbf_local over the list)
            const int at = atomicAdd(&status[3], 1);
            atomicAdd(&status[5], 1);
            if (at < a.ns_cap) a.ns_list[at] = (uint32_t)v;
            else atomicOr(&status[4], 1);
        } else {  // the output (zeros for a masked voxel), stored at the top of the next quad
            if (a.flags & PTV_FLAG_NAN_TO_NUM) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    o[c] = o[c] != o[c] ? 0.0
                                        : (o[c] == INFINITY ? DBL_MAX : (o[c] == -INFINITY ? -DBL_MAX : o[c]));
            }
            pend = true;
            pvo = (size_t)(iz - a.out_z0) * plane + rem;
#pragma unroll
            for (int c = 0; c < 3; ++c) po[c] = active ? o[c] : 0.0;
        }
    }
    rbf_wave_sync();  // the next quad reuses this wave's LDS
    }  // quads
    flush();
}

template <int NC, int NP>
void launch_ns_t(const RbfKernelArgs &ka, long long nvox, hipStream_t s, const double4 *prec, const double4 *pval,
                 const uint32_t *slots, const double *ax, const double *ay, const double *az, const double *qx,
                 const double *qy, const double *qz, const double *smooth, const int *pw, const uint8_t *mask,
                 double *U, double *V, double *W, int *status) {
    static int occ = 0;
    int per_cu = __atomic_load_n(&occ, __ATOMIC_RELAXED);
    if (per_cu <= 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_rbf_ns<NC, NP>, 256, 0) != hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        __atomic_store_n(&occ, per_cu, __ATOMIC_RELAXED);
    }
    hipLaunchKernelGGL((k_rbf_ns<NC, NP>), dim3(ns_grid((nvox + 3) / 4, per_cu)), dim3(256), 0, s, ka, prec, pval, slots,
                       ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status);
}

}  // namespace ptv
