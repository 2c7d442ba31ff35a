// ptv_wave.hpp — wave64 cross-lane primitives for gfx950 without LDS round trips.
//
// Lane exchanges use DPP (quad_perm, row_half_mirror, row_mirror, row_shr, row_bcast)
// inside 16-lane rows, ds_swizzle (bit-mode xor) for partners 4 and 8 lanes apart, and the
// gfx950 v_permlane16_swap / v_permlane32_swap for partners 16 / 32 lanes apart.  Every
// reduction combines symmetric pairs with a commutative op, so all lanes of a group end
// with the same value.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptv {

template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ int dpp_i32(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xF, false);
}
// the same where every lane is written and an invalid source lane reads 0 (bound_ctrl): no
// old value, so no v_mov to initialise one (quad_perm / mirror patterns, and row_shr into a sum)
template <int CTRL>
__device__ __forceinline__ int dpp0_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}

// a lane's reduction partner for one step: DPP control (quad_perm xor 1 / xor 2,
// row_half_mirror, row_mirror) or a bit-mode ds_swizzle xor
template <int CTRL>
__device__ __forceinline__ int partner_i32(int v) {
    if constexpr (CTRL >= 0x1000) return __builtin_amdgcn_ds_swizzle(v, CTRL - 0x1000);
    else return dpp0_i32<CTRL>(v);
}
constexpr int kSwizzleXor4 = 0x1000 + ((4 << 10) | 0x1f);
constexpr int kSwizzleXor8 = 0x1000 + ((8 << 10) | 0x1f);

template <int W>
__device__ __forceinline__ void swap_self_u32(unsigned v, unsigned &a, unsigned &b) {
    // {a, b} = this lane's value and its partner's (16 or 32 lanes away), in some order
    static_assert(W == 16 || W == 32, "swap width");
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

template <int CTRL, typename T, typename Op>
__device__ __forceinline__ T step32(T v, Op op) {
    return op(v, __builtin_bit_cast(T, partner_i32<CTRL>(__builtin_bit_cast(int, v))));
}
template <int W, typename T, typename Op>
__device__ __forceinline__ T swap32(T v, Op op) {
    unsigned a, b;
    swap_self_u32<W>(__builtin_bit_cast(unsigned, v), a, b);
    return op(__builtin_bit_cast(T, a), __builtin_bit_cast(T, b));
}
template <int CTRL, typename Op>
__device__ __forceinline__ double step64(double v, Op op) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)partner_i32<CTRL>((int)(unsigned)x);
    const unsigned hi = (unsigned)partner_i32<CTRL>((int)(unsigned)(x >> 32));
    return op(v, __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo)));
}
template <int W, typename Op>
__device__ __forceinline__ double swap64(double v, Op op) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    unsigned alo, blo, ahi, bhi;
    swap_self_u32<W>((unsigned)x, alo, blo);
    swap_self_u32<W>((unsigned)(x >> 32), ahi, bhi);
    return op(__longlong_as_double((long long)(((unsigned long long)ahi << 32) | alo)),
              __longlong_as_double((long long)(((unsigned long long)bhi << 32) | blo)));
}

template <int CTRL, typename T, typename Op>
__device__ __forceinline__ T step(T v, Op op) {
    if constexpr (sizeof(T) == 8) return step64<CTRL>(v, op);
    else return step32<CTRL>(v, op);
}
template <int W, typename T, typename Op>
__device__ __forceinline__ T swapstep(T v, Op op) {
    if constexpr (sizeof(T) == 8) return swap64<W>(v, op);
    else return swap32<W>(v, op);
}

// reduction over the lanes that differ only in the bits of MASK (a subset of 0x3f).
// Bits {0,1,2[,3]} together use the mirror patterns (all DPP); lone bits use exact xor.
template <int MASK, typename T, typename Op>
__device__ __forceinline__ T group_reduce(T v, Op op) {
    constexpr bool low3 = (MASK & 7) == 7;
    if constexpr ((MASK & 1) != 0) v = step<0xB1>(v, op);  // quad_perm [1,0,3,2]
    if constexpr ((MASK & 2) != 0) v = step<0x4E>(v, op);  // quad_perm [2,3,0,1]
    if constexpr (low3) {
        v = step<0x141>(v, op);                            // row_half_mirror: 8 lanes
        if constexpr ((MASK & 8) != 0) v = step<0x140>(v, op);  // row_mirror: 16 lanes
    } else {
        if constexpr ((MASK & 4) != 0) v = step<kSwizzleXor4>(v, op);
        if constexpr ((MASK & 8) != 0) v = step<kSwizzleXor8>(v, op);
    }
    if constexpr ((MASK & 16) != 0) v = swapstep<16>(v, op);
    if constexpr ((MASK & 32) != 0) v = swapstep<32>(v, op);
    return v;
}

// raw min / max (operands are never NaN where these are used: no canonicalisation)
struct OpMin {
    template <typename T>
    __device__ T operator()(T a, T b) const { return a < b ? a : b; }
};
struct OpMax {
    template <typename T>
    __device__ T operator()(T a, T b) const { return a > b ? a : b; }
};
struct OpAdd {
    template <typename T>
    __device__ T operator()(T a, T b) const { return a + b; }
};

// inclusive prefix sum / prefix max over the wave: row_shr 1, 2, 4, 8 inside each
// 16-lane row, then row_bcast15 (into rows 1, 3) and row_bcast31 (into rows 2, 3)
__device__ __forceinline__ int wave_incl_scan_add(int v) {
    v += dpp0_i32<0x111>(v);
    v += dpp0_i32<0x112>(v);
    v += dpp0_i32<0x114>(v);
    v += dpp0_i32<0x118>(v);
    v += dpp_i32<0x142, 0xA>(0, v);
    v += dpp_i32<0x143, 0xC>(0, v);
    return v;
}
__device__ __forceinline__ int wave_incl_scan_max(int v) {
    constexpr int lo = (int)0x80000000;
    v = max(v, dpp_i32<0x111>(lo, v));
    v = max(v, dpp_i32<0x112>(lo, v));
    v = max(v, dpp_i32<0x114>(lo, v));
    v = max(v, dpp_i32<0x118>(lo, v));
    v = max(v, dpp_i32<0x142, 0xA>(lo, v));
    v = max(v, dpp_i32<0x143, 0xC>(lo, v));
    return v;
}

}  // namespace ptv
