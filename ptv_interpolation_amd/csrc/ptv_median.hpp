// ptv_median.hpp — numpy median by rank selection over a register list (device helpers shared
// by the outlier-filter epilogue of the k-NN kernel, filtering.py:38-44).
#pragma once

#include <hip/hip_runtime.h>

namespace ptv {

// value at sorted position `pos` of s[0..n): the element whose [#less, #less-or-equal) holds pos
template <int KMAX>
__device__ __forceinline__ double select_pos(const double (&s)[KMAX], int n, int pos) {
    double out = 0.0;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if (j < n) {
            int lt = 0, le = 0;
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                if (i < n) {
                    lt += s[i] < s[j] ? 1 : 0;
                    le += s[i] <= s[j] ? 1 : 0;
                }
            }
            if (lt <= pos && pos < le) out = s[j];
        }
    }
    return out;
}

// np.median of n values (n odd: the middle one; n even: mean of the two middle ones, i.e.
// (a + b) / 2); any NaN gives NaN (numpy's _median_nancheck)
template <int KMAX>
__device__ __forceinline__ double median_of(const double (&s)[KMAX], int n) {
    bool nan = false;
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
        if (j < n) nan = nan || (s[j] != s[j]);
    if (nan) return __longlong_as_double(0x7ff8000000000000LL);
    if (n & 1) return select_pos(s, n, n >> 1);
    const double a = select_pos(s, n, (n >> 1) - 1), b = select_pos(s, n, n >> 1);
    return (a + b) / 2.0;
}

__device__ __forceinline__ double speed_of(const double4 v) {
    return sqrt((v.x * v.x + v.y * v.y) + v.z * v.z);  // u**2 + v**2 + w**2, left to right (filtering.py:16-17)
}

}  // namespace ptv
