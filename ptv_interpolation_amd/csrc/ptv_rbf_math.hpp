// ptv_rbf_math.hpp — device helpers shared by the local-RBF kernels (ptv_rbf.hip,
// ptv_rbf_ns*.hip): reciprocals, the kernel functions phi, monomials, and the segment
// reductions / row broadcasts in registers (DPP, v_permlane*_swap).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "../../include/ptv_api.h"

namespace ptv {

// 1/p from v_rcp_f64 and two Newton steps (within an ulp of the IEEE quotient; the
// elimination multiplier l = a * (1/p) is LAPACK dgetf2's reciprocal scaling anyway).
// Valid only where 1/p is a normal number: see elim_multiplier.
__device__ __forceinline__ double rcp_nr(double p) {
    double r = __builtin_amdgcn_rcp(p);
    double e = fma(-p, r, 1.0);
    r = fma(r, e, r);
    e = fma(-p, r, 1.0);
    return fma(r, e, r);
}

// l = a / p as LAPACK dgetf2 forms it: a * (1/p) when |p| >= sfmin (DBL_MIN), a / p below.
// The Newton reciprocal serves 2^-1020 < |p| < 2^1020; outside it (an infinite pivot gives
// rcp 0 and fma(-inf, 0, 1) = NaN; a subnormal one overflows the seed) the IEEE forms run.
__device__ __forceinline__ double elim_multiplier(double a, double p) {
    const double ap = fabs(p);
    if (ap > 0x1p-1020 && ap < 0x1p1020) return a * rcp_nr(p);
    return ap >= DBL_MIN ? a * (1.0 / p) : a / p;
}

// 1/p for the SPD kernels' multipliers l = a * (1/p) (LAPACK dgetf2's reciprocal scaling),
// branch-free: the Newton reciprocal where it is valid, IEEE division otherwise (an infinite or
// subnormal pivot; a branch here made the 16-lane kernel's unrolled elimination spill)
__device__ __forceinline__ double spd_recip(double p) {
    const double ap = fabs(p);
    const double q = 1.0 / p;
    const double r = rcp_nr(p);
    return (ap > 0x1p-1020 && ap < 0x1p1020) ? r : q;
}

__device__ __forceinline__ void rbf_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// exp(x) for x <= 0, bit-identical to the device libm (ocml) exp this kernel used before: the
// same reduction (x log2 e rounded to even, Cody-Waite ln 2 in two parts), degree-11 polynomial
// in Horner form, ldexp and underflow to 0 below -1075.  Written out so that every Horner step is
// one VOP3 v_fma_f64 with its coefficient in an SGPR pair: the compiler's form kept the
// coefficients in VGPRs and paid a v_mov_b64 per step (v_fmac overwrites its addend).
__device__ __forceinline__ double horner(double r, double p, double c) {
    double o;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(o) : "v"(r), "v"(p), "s"(c));
    return o;
}
__device__ __forceinline__ double exp_nonpos(double x) {
    const double dn = __builtin_rint(x * 0x1.71547652b82fep+0);
    double r = fma(-0x1.62e42fefa39efp-1, dn, x);
    r = fma(-0x1.abc9e3b39803fp-56, dn, r);
    double p = fma(0x1.ade156a5dcb37p-26, r, 0x1.28af3fca7ab0cp-22);
    p = horner(r, p, 0x1.71dee623fde64p-19);
    p = horner(r, p, 0x1.a01997c89e6b0p-16);
    p = horner(r, p, 0x1.a01a014761f6ep-13);
    p = horner(r, p, 0x1.6c16c1852b7b0p-10);
    p = horner(r, p, 0x1.1111111122322p-7);
    p = horner(r, p, 0x1.55555555502a1p-5);
    p = horner(r, p, 0x1.5555555555511p-3);
    p = horner(r, p, 0x1.000000000000bp-1);
    p = fma(r, p, 1.0);
    p = fma(r, p, 1.0);
    const double e = __builtin_amdgcn_ldexp(p, (int)dn);
    return -1075.0 > x ? 0.0 : e;
}

// IEEE sqrt for x >= 2^-767 (the LLVM gfx9 f64 expansion without its small-input rescale),
// branch-free; +-0 and +inf are returned as they are.  For 0 < x < 2^-767 it may differ from
// sqrt() in the last bit, which no SPD kernel can see: phi(r) of the gaussian, inverse
// multiquadric and inverse quadratic kernels only uses r * r + 1 or exp(-r * r).
__device__ __forceinline__ double sqrt_spd(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    g = fma(fma(-g, g, x), h, g);
    g = fma(fma(-g, g, x), h, g);
    return __builtin_amdgcn_class(x, 0x260) ? x : g;  // +inf, +0, -0
}

// scipy/interpolate/_rbfinterp_pythran.py kernel functions (r >= 0)
template <int KERN>
__device__ __forceinline__ double rbf_phi(double r) {
    if constexpr (KERN == PTV_RBF_LINEAR) return -r;
    if constexpr (KERN == PTV_RBF_THIN_PLATE_SPLINE) return r == 0.0 ? 0.0 : (r * r) * log(r);
    if constexpr (KERN == PTV_RBF_CUBIC) return (r * r) * r;
    if constexpr (KERN == PTV_RBF_QUINTIC) return -((((r * r) * r) * r) * r);
    if constexpr (KERN == PTV_RBF_MULTIQUADRIC) return -sqrt(r * r + 1.0);
    if constexpr (KERN == PTV_RBF_INVERSE_MULTIQUADRIC) return 1.0 / sqrt(r * r + 1.0);
    if constexpr (KERN == PTV_RBF_INVERSE_QUADRATIC) return 1.0 / (r * r + 1.0);
    if constexpr (KERN == PTV_RBF_GAUSSIAN) return exp_nonpos(-(r * r));
    return 0.0;
}

// the SPD kernels from the squared distance (r * r -> d2: no square root for the Gaussian and the
// inverse quadratic; within an ulp of scipy's r**2, far inside the solve's conditioning)
template <int KERN>
__device__ __forceinline__ double rbf_phi_d2(double d2) {
    static_assert(KERN == PTV_RBF_GAUSSIAN || KERN == PTV_RBF_INVERSE_QUADRATIC || KERN == PTV_RBF_INVERSE_MULTIQUADRIC,
                  "SPD kernels");
    if constexpr (KERN == PTV_RBF_INVERSE_MULTIQUADRIC) return 1.0 / sqrt(d2 + 1.0);
    if constexpr (KERN == PTV_RBF_INVERSE_QUADRATIC) return 1.0 / (d2 + 1.0);
    return exp_nonpos(-d2);
}

static __device__ double rbf_phi_rt(int kern, double r) {
    switch (kern) {
        case PTV_RBF_LINEAR: return rbf_phi<PTV_RBF_LINEAR>(r);
        case PTV_RBF_THIN_PLATE_SPLINE: return rbf_phi<PTV_RBF_THIN_PLATE_SPLINE>(r);
        case PTV_RBF_CUBIC: return rbf_phi<PTV_RBF_CUBIC>(r);
        case PTV_RBF_QUINTIC: return rbf_phi<PTV_RBF_QUINTIC>(r);
        case PTV_RBF_MULTIQUADRIC: return rbf_phi<PTV_RBF_MULTIQUADRIC>(r);
        case PTV_RBF_INVERSE_MULTIQUADRIC: return rbf_phi<PTV_RBF_INVERSE_MULTIQUADRIC>(r);
        case PTV_RBF_INVERSE_QUADRATIC: return rbf_phi<PTV_RBF_INVERSE_QUADRATIC>(r);
        default: return rbf_phi<PTV_RBF_GAUSSIAN>(r);
    }
}

// libm pow for the rare exponents > 3 (degree >= 4); out of line so its code exists once
static __device__ __noinline__ double ipow_slow(double x, int p) { return pow(x, (double)p); }

// x ** p for the small integer monomial exponents (np.prod(x ** powers[j]))
__device__ __forceinline__ double ipow(double x, int p) {
    if (p == 0) return 1.0;
    if (p == 1) return x;
    if (p == 2) return x * x;
    if (p == 3) return (x * x) * x;
    return ipow_slow(x, p);
}

// monomial with exponents packed as px | py << 8 | pz << 16
__device__ __forceinline__ double mono(double hx, double hy, double hz, int code) {
    return (ipow(hx, code & 255) * ipow(hy, (code >> 8) & 255)) * ipow(hz, code >> 16);
}

// ---- segment reductions in registers: DPP within 16-lane rows (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror), v_permlane16_swap / v_permlane32_swap (gfx950) across rows.
// Every lane of the segment ends with the same value (each step combines symmetric pairs). ----
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    // bound_ctrl: every source lane of these patterns is valid, so no old value is needed
    // (the compiler then drops the v_mov that would initialise it)
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = dpp_u32<CTRL>((unsigned)b), hi = dpp_u32<CTRL>((unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// (v of this lane's row partner, v of its half-wave partner): the two results of a swap of v with itself
template <int W>
__device__ __forceinline__ void swap_self(unsigned v, unsigned &a, unsigned &b) {
    if constexpr (W == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        a = r[0];
        b = r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        a = r[0];
        b = r[1];
    }
}
template <int W>
__device__ __forceinline__ void swap_self_f64(double v, double &a, double &b) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    unsigned al, bl, ah, bh;
    swap_self<W>((unsigned)x, al, bl);
    swap_self<W>((unsigned)(x >> 32), ah, bh);
    a = __longlong_as_double((long long)(((unsigned long long)ah << 32) | al));
    b = __longlong_as_double((long long)(((unsigned long long)bh << 32) | bl));
}

template <int L, typename Op>
__device__ __forceinline__ double seg_reduce(double v, Op op) {
    static_assert(L == 16 || L == 32 || L == 64, "segment width");
    v = op(v, dpp_f64<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp_f64<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp_f64<0x141>(v));  // row_half_mirror
    v = op(v, dpp_f64<0x140>(v));  // row_mirror
    if constexpr (L >= 32) {
        double a, b;
        swap_self_f64<16>(v, a, b);
        v = op(a, b);
    }
    if constexpr (L == 64) {
        double a, b;
        swap_self_f64<32>(v, a, b);
        v = op(a, b);
    }
    return v;
}
template <int L>
__device__ __forceinline__ unsigned seg_max_u32(unsigned v) {
    v = max(v, dpp_u32<0xB1>(v));
    v = max(v, dpp_u32<0x4E>(v));
    v = max(v, dpp_u32<0x141>(v));
    v = max(v, dpp_u32<0x140>(v));
    if constexpr (L >= 32) {
        unsigned a, b;
        swap_self<16>(v, a, b);
        v = max(a, b);
    }
    if constexpr (L == 64) {
        unsigned a, b;
        swap_self<32>(v, a, b);
        v = max(a, b);
    }
    return v;
}
template <int L>
__device__ __forceinline__ double seg_sum(double v) {
    return seg_reduce<L>(v, [](double x, double y) { return x + y; });
}
template <int L>
__device__ __forceinline__ double seg_min(double v) {
    return seg_reduce<L>(v, [](double x, double y) { return fmin(x, y); });
}
template <int L>
__device__ __forceinline__ double seg_max(double v) {
    return seg_reduce<L>(v, [](double x, double y) { return fmax(x, y); });
}

template <int N>
__device__ __forceinline__ double rowbcast(double v) {  // lane N of this lane's 16-lane row
    return __longlong_as_double(
        __builtin_amdgcn_update_dpp(0LL, __double_as_longlong(v), 0x150 + N, 0xF, 0xF, true));
}

// the same with a lane index that the unrolled loops fold to a constant (the DPP control must be one)
__device__ __forceinline__ double rowbcast_n(int n, double v) {
    switch (n & 15) {
        case 0: return rowbcast<0>(v);
        case 1: return rowbcast<1>(v);
        case 2: return rowbcast<2>(v);
        case 3: return rowbcast<3>(v);
        case 4: return rowbcast<4>(v);
        case 5: return rowbcast<5>(v);
        case 6: return rowbcast<6>(v);
        case 7: return rowbcast<7>(v);
        case 8: return rowbcast<8>(v);
        case 9: return rowbcast<9>(v);
        case 10: return rowbcast<10>(v);
        case 11: return rowbcast<11>(v);
        case 12: return rowbcast<12>(v);
        case 13: return rowbcast<13>(v);
        case 14: return rowbcast<14>(v);
        default: return rowbcast<15>(v);
    }
}

// ---- v_fmac_f64 with its first operand broadcast from lane N of the 16-lane row (gfx950 DPALU
// DPP: row_newbcast only): acc += src[lane N] * mul in ONE instruction where the compiler emits a
// v_mov_b64_dpp and a v_fma_f64 (it does not fold 64-bit DPP into the fmac).  Inline asm, so the
// compiler cannot see the DPP read: each block starts with the s_nop 1 (2 wait states) a DPP read
// needs after a VALU write of its source.  A block updates the accumulators of every live row set
// of the lane (RS = 1 or 2) with one broadcast source. ----
template <int N, int RS>
__device__ __forceinline__ void fmac_bc(double (&acc)[RS], double src, const double (&mul)[RS]) {
    if constexpr (RS == 1) {
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "+v"(acc[0]) : "v"(src), "v"(mul[0]), "n"(N));
    } else {
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "+v"(acc[0]), "+v"(acc[1]) : "v"(src), "v"(mul[0]), "v"(mul[1]), "n"(N));
    }
}
// the same where the source is the accumulator `piv` itself (the pivot row's set): the other set
// `oth` first, then piv (its DPP read precedes its write)
template <int N>
__device__ __forceinline__ void fmac_bc_piv(double &oth, double &piv, double m_oth, double m_piv) {
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %1, %1, %3 row_newbcast:%4 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "+v"(oth), "+v"(piv) : "v"(m_oth), "v"(m_piv), "n"(N));
}
template <int N>
__device__ __forceinline__ void fmac_bc_self(double &piv, double m_piv) {
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "+v"(piv) : "v"(m_piv), "n"(N));
}
#define PTV_NS_SW16(n, CALL)      \
    switch ((n) & 15) {           \
        case 0: CALL(0); break;   \
        case 1: CALL(1); break;   \
        case 2: CALL(2); break;   \
        case 3: CALL(3); break;   \
        case 4: CALL(4); break;   \
        case 5: CALL(5); break;   \
        case 6: CALL(6); break;   \
        case 7: CALL(7); break;   \
        case 8: CALL(8); break;   \
        case 9: CALL(9); break;   \
        case 10: CALL(10); break; \
        case 11: CALL(11); break; \
        case 12: CALL(12); break; \
        case 13: CALL(13); break; \
        case 14: CALL(14); break; \
        default: CALL(15); break; \
    }
template <int RS>
__device__ __forceinline__ void fmac_bc_n(int n, double (&acc)[RS], double src, const double (&mul)[RS]) {
#define PTV_C(N) fmac_bc<N, RS>(acc, src, mul)
    PTV_NS_SW16(n, PTV_C)
#undef PTV_C
}
__device__ __forceinline__ void fmac_bc_piv_n(int n, double &oth, double &piv, double m_oth, double m_piv) {
#define PTV_C(N) fmac_bc_piv<N>(oth, piv, m_oth, m_piv)
    PTV_NS_SW16(n, PTV_C)
#undef PTV_C
}
__device__ __forceinline__ void fmac_bc_self_n(int n, double &piv, double m_piv) {
#define PTV_C(N) fmac_bc_self<N>(piv, m_piv)
    PTV_NS_SW16(n, PTV_C)
#undef PTV_C
}


__device__ uint8_t kNsMaskOn = 1;  // the mask byte read when there is no mask (global, not flat)

// persistent grid: the blocks one wave of residency holds (occupancy x CUs), a multiple of the 8
// XCDs; a block that waited for a free CU would find its quads' share undone at the end
inline unsigned ns_grid(long long nquad, int per_cu) {
    static int cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    int c = __atomic_load_n(&cus[dev], __ATOMIC_RELAXED);
    if (c <= 0) {
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        __atomic_store_n(&cus[dev], c, __ATOMIC_RELAXED);
    }
    long long nb = (nquad + 3) / 4, cap = (long long)c * (per_cu > 0 ? per_cu : 1);
    if (nb > cap) nb = cap;
    return (unsigned)((nb + 7) / 8 * 8);
}

// the persistent grid of a kernel instantiation (its occupancy read once)
template <typename K>
inline unsigned persistent_grid(K kernel, long long nquad, int &occ) {
    int per_cu = __atomic_load_n(&occ, __ATOMIC_RELAXED);
    if (per_cu <= 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0)
            per_cu = 1;
        __atomic_store_n(&occ, per_cu, __ATOMIC_RELAXED);
    }
    return ns_grid(nquad, per_cu);
}

}  // namespace ptv
