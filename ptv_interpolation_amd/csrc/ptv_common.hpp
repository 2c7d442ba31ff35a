// ptv_common.hpp — shared device/host definitions for the MI355X PTV interpolator.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace ptv {

// ---------------------------------------------------------------------------
// Error plumbing: thread-local message + negative codes (include/ptv_api.h).
// ---------------------------------------------------------------------------
void set_error(const std::string &msg);

#define PTV_HIP(expr)                                                              \
    do {                                                                           \
        hipError_t _e = (expr);                                                    \
        if (_e != hipSuccess) {                                                    \
            ::ptv::set_error(std::string(#expr " failed: ") + hipGetErrorString(_e) + \
                             " (" __FILE__ ":" + std::to_string(__LINE__) + ")");  \
            return PTV_E_HIP;                                                      \
        }                                                                          \
    } while (0)

// ---------------------------------------------------------------------------
// Binning cell grid: a uniform grid of cells over the particle/query bounding
// box, addressed by Morton code on a padded 2^L cube so that every octree node
// (level l, code c) owns the contiguous particle range
//     [cell_start[c << 3l], cell_start[(c + 1) << 3l]).
// ---------------------------------------------------------------------------
constexpr int kMaxLevels = 9;  // <= 512 cells per axis; stack bound 7*9+1 <= 64 lanes

struct CellGrid {
    double o[3];    // origin (lower corner)
    double cs[3];   // cell size per axis
    double ic[3];   // 1 / cs
    double mg[3];   // pruning margin per axis (covers binning round-off)
    int nc[3];      // cells per axis
    int L;          // octree levels: padded side P = 1 << L
};

__host__ __device__ inline uint32_t spread3(uint32_t v) {
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__host__ __device__ inline uint32_t compact3(uint32_t v) {
    v &= 0x09249249u;
    v = (v ^ (v >> 2)) & 0x030C30C3u;
    v = (v ^ (v >> 4)) & 0x0300F00Fu;
    v = (v ^ (v >> 8)) & 0xFF0000FFu;
    v = (v ^ (v >> 16)) & 0x000003FFu;
    return v;
}

__host__ __device__ inline uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
}

// Device buffers produced by binning (owned by the context).
struct Binned {
    const double4 *prec;    // sorted (x, y, z, original index as double)
    const double4 *pval;    // sorted (u, v, w, 0)
    const uint32_t *cstart; // P^3 + 1 Morton-ordered cell starts
    int64_t n;
};

}  // namespace ptv
