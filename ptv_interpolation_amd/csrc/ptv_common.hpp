// ptv_common.hpp — shared device/host definitions for the MI355X PTV interpolator.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>

namespace ptv {

// Dev tuning knobs (environment variables) are read only by builds compiled with
// -DPTV_DEV_KNOBS=1 (the tools/ A/B and stamp builds); the shipped library never lets the
// environment change its kernels or launch shapes.
inline const char *dev_knob(const char *name) {
#if defined(PTV_DEV_KNOBS) && PTV_DEV_KNOBS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

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

#define PTV_TRY(expr)               \
    do {                            \
        int _r = (expr);            \
        if (_r != PTV_OK) return _r; \
    } while (0)

// ---------------------------------------------------------------------------
// Binning cell grid: a uniform grid of cells over the particle/query bounding
// box in linear (z, y, x) order, x fastest.  After the counting sort, every
// x-run of cells [cx0, cx1] in row (cy, cz) owns the contiguous particle range
//     [cell_start[row + cx0], cell_start[row + cx1 + 1]),  row = (cz*ncy + cy)*ncx.
// ---------------------------------------------------------------------------
struct CellGrid {
    double o[3];   // origin (lower corner)
    double cs[3];  // cell size per axis
    double ic[3];  // 1 / cs
    double mg;     // absolute margin added to every radius (binning / bound round-off)
    int nc[3];     // cells per axis
    long long ncells;
};

// Device buffers produced by binning (owned by the context).
struct Binned {
    const double4 *prec;     // sorted (x, y, z, original index as double)
    const double4 *pval;     // sorted (u, v, w, 0)
    const uint32_t *cstart;  // ncells + 1 cell starts (linear order)
    int64_t n;
};

}  // namespace ptv
