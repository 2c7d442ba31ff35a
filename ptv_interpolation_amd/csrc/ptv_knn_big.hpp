// ptv_knn_big.hpp — grow-only device buffers, and the large-k k-NN path (ptv_knn_big.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/ptv_api.h"
#include "ptv_common.hpp"

namespace ptv {

// a grow-only device buffer (contents are not kept across a growth)
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
    int ensure(size_t n) {
        if (n <= cap && p) return PTV_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1);
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            set_error("hipMalloc of " + std::to_string(want * sizeof(T)) + " bytes failed: " + hipGetErrorString(e));
            return PTV_E_NOMEM;
        }
        cap = want;
        return PTV_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// queries of the large-k path: voxels [z0 plane ...) of a grid (separable axes or point lists, an
// optional fluid mask), or (particles = 1) the particles themselves in original order (the filter)
struct BigQueries {
    int particles = 0;
    int nx = 0, ny = 0, z0 = 0;                            // grid queries: voxel i of the slab
    const double *ax = nullptr, *ay = nullptr, *az = nullptr;  // separable axes, or
    const double *px = nullptr, *py = nullptr, *pz = nullptr;  // point lists (full grid) / particle x, y, z
    const double *pu = nullptr, *pv = nullptr, *pw = nullptr;  // the filter: particle values (speeds)
    const uint8_t *mask = nullptr;                         // (full grid) 0 = solid: output 0
};

// what the large-k path computes from each query's sorted neighbours
struct BigEpilogue {
    int filter = 0;  // 0: IDW / Sibson into U, V, W; 1: the outlier filter's keep / kth
    int method = PTV_METHOD_IDW;
    double power = 2.0, eps = 1e-10;
    uint32_t flags = 0;
    double *U = nullptr, *V = nullptr, *W = nullptr;  // slab-relative voxel outputs
    const double *spd = nullptr;                      // filter: speeds in slot order
    uint8_t *keep = nullptr;
    double *kth = nullptr;
    double threshold = 3.0, mad_eps = 1e-6;
    uint32_t *slots = nullptr;  // != NULL: write each query's k neighbour slots (query-major), nothing else
};

struct BigScratch {
    DevBuf<double> R, fmed;
    DevBuf<unsigned long long> ub, incl, temp, keys, keys2, fa, fa2, fb;
    DevBuf<uint32_t> vals, vals2;
    DevBuf<int> seg_b, seg_e, fseg;
    void release() {
        R.release(); fmed.release(); ub.release(); incl.release(); temp.release(); keys.release();
        keys2.release(); fa.release(); fa2.release(); fb.release(); vals.release(); vals2.release();
        seg_b.release(); seg_e.release(); fseg.release();
    }
};

// candidate entries per sub-chunk (a (d2, slot) pair and its sorted copy: 24 B each)
constexpr long long kBigEntryBudget = 128LL << 20;

// k neighbours per query (k + 1 with ep.filter) over the binned particles b (cell grid cg)
int run_big_knn(BigScratch &sc, const BigQueries &q, const Binned &b, const CellGrid &cg, int64_t nq_total, int k,
                const BigEpilogue &ep, hipStream_t s);

}  // namespace ptv
