// ptv_kernels.hpp — host-side launchers for the device kernels.
#pragma once

#include "ptv_common.hpp"

namespace ptv {

// ---- binning (ptv_bin.hip) ----
// Per-axis min/max over the particles and the query coordinates.
// Query coordinates: separable axes (qa[a] has qn[a] entries) or point lists.
int launch_bbox(const double *const px[3], int64_t n, const double *const qa[3], const int64_t qn[3],
                double *d_partials, int max_blocks, double *d_out6, hipStream_t s,
                const uint32_t *d_n = nullptr);  // d_n: the particle count on the device (<= n)

// Sort the particles into linear-order cells (deterministic order
// inside each cell: ascending original index).  Scratch buffers must hold
// 2n (code), n (perm) and ncells (+1) entries (count, start).
// With a BinSortScratch (keys: n entries, temp: bin_sort_temp_bytes(n, ncells)) the binning is a
// stable radix sort of (cell, index) pairs instead (no per-particle atomics; same result).
struct BinSortScratch {
    uint32_t *keys = nullptr;
    void *temp = nullptr;
    size_t temp_bytes = 0;
};
size_t bin_sort_temp_bytes(int64_t n, size_t m);
int launch_bin(const CellGrid &cg, const double *const px[3], const double *const pv[3], int64_t n,
               uint32_t *d_code, uint32_t *d_perm, uint32_t *d_count, uint32_t *d_start,
               uint32_t *d_scan_partials, double4 *d_prec, double4 *d_pval, hipStream_t s,
               const BinSortScratch *ss = nullptr);

size_t scan_partials_needed(size_t m);

// slab cull (ptv_knn_params.slab_halo): win (4 doubles) = (zlo, zhi, slab z min, slab z max),
// bcount: cull_blocks(n) + 1 scratch words; the kept count is copied to the HOST word *h_total
// (pinned; valid after the stream synchronises; NULL: left on the device in bcount[cull_blocks(n)]).
// Order-preserving.
size_t cull_blocks(int64_t n);
// per-column cull map (PTV_FLAG_SLAB_CULL_AUTO): a uniform mx x my grid of (x, y) cells of size
// cw x ch from (x0, y0); a particle outside the slab's z extent is kept iff its z is <= top[cell]
// (above the slab) or >= bot[cell] (below) of its cell (clamped to the grid)
struct CullMap {
    const double *top = nullptr, *bot = nullptr;
    int mx = 0, my = 0;
    double x0 = 0.0, y0 = 0.0, cw = 1.0, ch = 1.0, icw = 1.0, ich = 1.0;
};
// map != NULL: the per-column map replaces the scalar halo; masks: cull_mask_words(n) scratch words
size_t cull_mask_words(int64_t n);
int launch_cull(const double *const src[6], int64_t n, const double *az, int z0, int z1, double halo, double *win,
                uint32_t *bcount, unsigned long long *masks, double *const dst[6], uint32_t *h_total, hipStream_t s,
                const CullMap *map = nullptr);
// the map a slab needs, from its finest lattice (axes lax / lay / laz, n[3] points, k-th distance
// bounds dk over the particles binned): top / bot per cell of m's geometry; cols: 7 (n0-1)(n1-1)
// doubles and keys: 2 mx my u64 of scratch; every cell reach U is widened by the relative `slack`.
// With `used` (the map the binned particles were culled with) *fail is set to 0 when the need fits
// inside it everywhere (the cull is proven exact), else to +inf's bits (the slab_halo gate's
// convention).
// *fail = 0 when dk[i] <= ref[i] * factor for every i < n, else +inf's bits (the cached cull map's proof)
int launch_bounds_within(const double *dk, const double *ref, long long n, double factor, unsigned long long *fail,
                         hipStream_t s, bool reset = true);
// *fail raised to +inf's bits unless key == ref (n doubles, bitwise) and *count == expect
int launch_key_check(const double *key, const double *ref, int n, const uint32_t *count, uint32_t expect,
                     unsigned long long *fail, hipStream_t s);
int launch_cull_need(const double *lax, const double *lay, const double *laz, const int n[3], const double *dk,
                     double mg, double slack, const CullMap &m, double *top, double *bot, double *cols,
                     unsigned long long *keys, const CullMap *used, unsigned long long *fail, hipStream_t s);

// 6 * kFingerprint doubles identifying a particle set (the cull map cache's key, with n and the arrays)
constexpr int kFingerprint = 16;
int launch_fingerprint(const double *const src[6], int64_t n, double *out, hipStream_t s);

// ---- k-NN interpolation (ptv_knn.hip) ----
// Exact k-th-neighbour distances on a coarser separable lattice (every `step`-th
// point of this launch's grid, plus the last): d_k(v) <= dk(c) + |v - c| for any
// lattice point c bounds every voxel's search radius (triangle inequality).
constexpr int kLatticeShift = 2;  // coarse lattice = every (1 << kLatticeShift)-th grid point (+ last)
constexpr int kLatticeStep = 1 << kLatticeShift;

struct CoarseBound {
    const double *ax = nullptr, *ay = nullptr, *az = nullptr;  // lattice axes
    const double *dk = nullptr;                                // (n[2], n[1], n[0]) k-th distances
    const float4 *recs = nullptr;   // (n[2], n[1], n[0], k) k-NN seed records {p - c (fp32), slot}, or NULL
    int n[3] = {0, 0, 0};
};

constexpr int kModeInterp = 0;  // write U, V, W
constexpr int kModeKDist = 1;   // write the exact k-th neighbour distance into U
constexpr int kModeSlots = 2;   // write each voxel's k neighbour slots (sorted-record indices)
constexpr int kModeRadius = 3;  // IDW over every particle within a fixed radius (PTV_METHOD_IDW_RADIUS)
constexpr int kModeFilter = 4;  // the outlier filter's (k+1)-NN + median/MAD epilogue (filtering.py:20-51)
constexpr int kModeKDistMerge = 5;  // launcher-internal: k_kdist_merge of a split lattice launch

// kModeFilter inputs / outputs (point-list queries = the particles, ptv_filter.hip layout)
struct FilterEpilogue {
    const uint32_t *q_orig = nullptr;  // original index of the query at each position (~0: pad)
    const uint32_t *inv = nullptr;     // binning: slot of each original index
    const double *spd = nullptr;       // speed of each binned particle (slot order)
    uint8_t *keep = nullptr;           // keep flag per original index
    double *kth = nullptr;             // distance to the (k+1)-th neighbour per original index (or NULL)
    double threshold = 3.0, mad_eps = 1e-6;
};

struct KnnLaunch {
    CellGrid cg;
    int nx, ny, nz;      // full grid
    int z0, z1;          // planes computed by this launch
    int separable;       // 1: axes, 0: point lists
    int method;          // PTV_METHOD_*
    int k;
    double power, eps;
    uint32_t flags;
    double r0;           // first gather radius (from the mean particle density)
    int mode = kModeInterp;
    CoarseBound cb;
    float4 *kd_recs = nullptr;   // kModeKDist: also write each point's k-NN seed records here
    int lz0 = -1;                // plane of lattice point 0 (-1: z0); chunked launches keep the slab's
    uint32_t *slots = nullptr;   // kModeSlots: (z1 - z0, ny, nx, k) neighbour slots out
    double radius = 0.0;         // kModeRadius: the search radius
    FilterEpilogue fe;           // kModeFilter
    const int *order = nullptr;  // dispatch order of the launch's blocks (NULL: XCD-contiguous ranges)
    // near-tie repair of the packed-key lists (k >= 13, modes interp / slots / filter): a device
    // counter + tile list (rep_cap entries), a pinned host word for the count, and a counter of
    // repaired tiles (stats, may be NULL)
    unsigned int *rep_cnt = nullptr;
    uint32_t *rep_list = nullptr;
    int rep_cap = 0;
    unsigned int *h_rep = nullptr;
    int64_t *n_repair = nullptr;
    // slab cull proof gate (see KnnKernelArgs::gate): NULL = always run
    const unsigned long long *gate = nullptr;
    double gate_halo = 0.0;
    // kModeKDist with a block order: the first split_blocks blocks of the order run as a split
    // launch, split waves per tile, merged by k_kdist_merge (ptv_knn_impl.hpp); split_out holds
    // split_blocks * 4 * split * KMAX * 64 slots (0 = off)
    int split = 0;
    int split_blocks = 0;
    uint32_t *split_out = nullptr;
};

// the split lattice launch's partial-list buffer (slots) for a KMAX list
inline size_t kdist_split_slots(int split, int split_blocks, int kmax) {
    return (size_t)split_blocks * 4 * (size_t)split * (size_t)kmax * 64;
}

// Longest-first dispatch order for a lattice-level k-NN launch over (nx, ny, nz) points: each
// block (4 x 1 x 1 tiles of 4^3 points) is keyed by the largest coarser-level bound dk over the
// coarser points around it (D / unit, 256 buckets), and `order` lists the blocks by descending
// key, so the void tiles (long searches) start first instead of forming the launch's tail.
int launch_block_order(const double *dk_coarse, const int nc[3], int nx, int ny, int nz, double unit, int *order,
                       double *keys, hipStream_t s);  // keys: nblocks + 1 doubles of scratch

// Upper bound on the k-th neighbour distance of every point of a separable grid by
// counting the particles of cells entirely inside balls around it (coarsest lattice).
int launch_count_bound(const CellGrid &g, const uint32_t *cstart, const double *ax, const double *ay,
                       const double *az, int nx, int ny, int nz, int k, double r0, double *out, hipStream_t s);

// out[j] = in[min(step*j, n-1)] for j < nout (lattice axes)
int launch_subsample(const double *in, int n, int step, double *out, int nout, hipStream_t s);
// every lattice level's axes in one launch: level l axis d has n[l][d] points, level l's point j is
// level (l - 1)'s point min(step j, n[l-1][d] - 1), level -1 = base[d] with n0[d] points
constexpr int kMaxSubsampleLevels = 8;
struct SubsampleBatch {
    const double *base[3];
    int n0[3];
    int nlev;
    int n[kMaxSubsampleLevels][3];
    double *out[kMaxSubsampleLevels][3];
};
int launch_subsample_levels(const SubsampleBatch &b, int step, hipStream_t s);
// out = a[0..na) ++ b[0..nb) ++ c[0..nc) (device arrays)
int launch_concat3(const double *a, int na, const double *b, int nb, const double *c, int nc, double *out,
                   hipStream_t s);

// Smallest z halo that makes a slab-culled k-NN exact, from the finest lattice's k-th
// distance bounds dk over (nx, ny, nz) lattice points with axes lax, lay, laz and the slab's
// z extent win[2..3]: max over lattice points c of D(c) + diag(c) + dz(c) - m(c), where
// diag(c) / dz(c) bound the adjacent lattice cells' diagonal / z extent and m(c) is c's
// distance to the nearer slab face.  out: one u64 (max of non-negative doubles' bits),
// zeroed by the launcher; mg: absolute margin.
int launch_halo_need(const double *lax, const double *lay, const double *laz, int nx, int ny, int nz,
                     const double *dk, const double *win, double mg, unsigned long long *out, hipStream_t s);

int kmax_for(int k);  // compile-time list length serving k, 0 if unsupported
extern unsigned long long *g_dbg;  // per-wave phase stamps (diagnostics), NULL = off
extern long long g_dbg_cap;

int launch_knn(const KnnLaunch &a, const Binned &b, const double *ax, const double *ay, const double *az,
               const double *qx, const double *qy, const double *qz, const uint8_t *mask, double *U, double *V,
               double *W, hipStream_t s);

// ---- consistent divergence (ptv_div.hip) ----
struct DivArgs {
    int nx, ny, nz;          // buffer shape (nz planes, C order)
    int z_begin, z_end;      // buffer planes computed (output plane 0 = z_begin)
    int edge_lo, edge_hi;    // buffer plane 0 / nz-1 is a domain z edge (else a halo plane)
    int field_f32;           // fields are float32 (else float64)
    int result_f32;          // quotients and sums in float32 (else float64)
    double dx, dy, dz;
    int ntx = 0, nty = 0, ntiles = 0;  // tile counts (set by the launcher)
    int xcd = 0;                       // XCD-contiguous tile order
};

int launch_divergence(const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
                      hipStream_t s);

// ---- linear (ptv_linear.hip): griddata(method='linear') over scipy's Delaunay triangulation ----
struct LinearKernelArgs {
    int nx, ny;          // grid plane
    int z0, z1;          // planes of this launch (chunk)
    int out_z0;          // plane of output row 0 (the slab start)
    int separable;
    long long nsimplex;
    const int *simplices;     // (nsimplex, 4) particle indices
    const int *neighbors;     // (nsimplex, 4) neighbour opposite vertex k, -1 = hull
    const double *transform;  // (nsimplex, 4, 3) barycentric transforms (NaN: degenerate)
    const int *v2s;           // (n,) a simplex incident to each particle (start of the walk)
    const double *pu, *pv, *pw;  // values, original particle order
    double lo[3], hi[3];      // Delaunay min_bound / max_bound
    double fill;              // fill_value
    uint32_t flags;           // PTV_FLAG_NAN_TO_NUM
    int max_walk;             // walk steps before the brute-force fallback
    int *flag_count;          // voxels left to the brute force (device counter)
    long long *flag_list;     // their slab-relative voxel indices
    int flag_cap;
};

// slots: (z1 - z0, ny, nx) nearest-particle slots (launch_knn kModeSlots, k = 1)
int launch_linear(const LinearKernelArgs &a, const double4 *prec, const uint32_t *slots, const double *ax,
                  const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
                  const uint8_t *mask, double *U, double *V, double *W, hipStream_t s);
// scipy's brute-force point location for the nflag voxels the walk flagged (after every chunk)
int launch_linear_brute(const LinearKernelArgs &a, int nflag, const double *ax, const double *ay, const double *az,
                        const double *qx, const double *qy, const double *qz, double *U, double *V, double *W,
                        hipStream_t s);

// ---- local RBF (ptv_rbf.hip) ----
constexpr int kRbfNsCap = 1 << 14;   // voxels per launch k_rbf_ns may hand to the pivoting kernel
constexpr int kRbfMaxSystem = 128;  // k + #monomials per voxel system in LDS (> 64: k_rbf_big; larger: k_rbf_huge, global)

struct RbfKernelArgs {
    int nx, ny;      // grid plane
    int z0, z1;      // planes of this launch (chunk)
    int out_z0;      // plane of output row 0 (the slab start)
    int separable;
    int k, m;        // neighbours, system size (k + #monomials)
    int kernel;      // PTV_RBF_*
    double epsilon;
    double smoothing;  // scalar smoothing (when no per-particle array is given)
    uint32_t flags;
    int spd_lds;       // SPD systems: the LDS-broadcast k_rbf_spd instead of k_rbf_spd16 (the
                       // rerun after k_rbf_spd16 flagged an out-of-range pivot in status[2])
    // null-space kernel (ptv_rbf_ns.hpp): chunk-local voxels it hands to the pivoting kernel
    uint32_t *ns_list; // NULL: the null-space path is off for this launch
    int ns_cap;        // entries of ns_list
    // pivoting kernel in list mode: solve only the voxels vlist[0 .. min(*vcount, ns_cap))
    const uint32_t *vlist;
    const int *vcount;
    unsigned long long *stamps;  // dev builds (PTV_NS_STAMP): per-wave phase cycles of k_rbf_ns, 8 per wave
    long long stamp_cap;
    // m > kRbfMaxSystem (k_rbf_huge): huge_blocks persistent workgroups, each with a slice of
    // rbf_huge_slice_doubles(m, k) doubles of huge_scratch
    double *huge_scratch;
    int huge_blocks;
};
size_t rbf_huge_slice_doubles(int m, int k);

// null-space local-RBF kernels k_rbf_ns<NC, NP> (ptv_rbf_ns.hpp), one translation unit per
// row-slot count NC (16, 20, 24, 32); np = number of monomials (1, 4 or 10)
#define PTV_RBF_NS_DECL(NC)                                                                                   \
    void launch_rbf_ns##NC(const RbfKernelArgs &ka, long long nvox, int np, hipStream_t s, const double4 *prec, \
                           const double4 *pval, const uint32_t *slots, const double *ax, const double *ay,       \
                           const double *az, const double *qx, const double *qy, const double *qz,               \
                           const double *smooth, const int *pw, const uint8_t *mask, double *U, double *V,      \
                           double *W, int *status)
PTV_RBF_NS_DECL(16);
PTV_RBF_NS_DECL(20);
PTV_RBF_NS_DECL(24);
PTV_RBF_NS_DECL(32);

int rbf_system_size(int m);  // padded system size served, 0 if unsupported

// slots: (z1 - z0, ny, nx, k) neighbour slots from launch_knn(kModeSlots); pw: the
// monomial exponents (m - k entries, px | py << 8 | pz << 16); status[0] counts singular
// systems, status[1] keeps the lowest singular voxel index, status[2] != 0 asks for a rerun
// with spd_lds set; the null-space path counts its flagged voxels of this launch in status[3]
// (reset by launch_rbf), sets status[4] when more than ns_cap were flagged (the host then reruns
// without it) and accumulates the flagged voxels of every launch in status[5].
int launch_rbf(const RbfKernelArgs &ka, const Binned &b, const uint32_t *slots, const double *ax, const double *ay,
               const double *az, const double *qx, const double *qy, const double *qz, const double *smooth,
               const int *pw, const uint8_t *mask, double *U, double *V, double *W, int *status, hipStream_t s);

// ---- pore-mask path (ptv_mask.hip) ----
struct MaskSampleLaunch {
    int rn[3];             // raw mask extents x, y, z
    int flip[3];           // caller axis is descending (ra[d] holds it reversed)
    const double *ra[3];   // raw mask axes, ascending (device)
    const uint8_t *raw;    // (rn[2], rn[1], rn[0]) bytes, 1 = raw value > 0.5
    int nx, ny, nz;        // grid
    int z0, z1;            // planes sampled
};
// tabs: nx + ny + nz ints of scratch (separable grids)
int launch_mask_sample(const MaskSampleLaunch &m, const double *ax, const double *ay, const double *az,
                       const double *px, const double *py, const double *pz, int *tabs, uint8_t *out,
                       hipStream_t s);

struct BoundaryLaunch {
    int nx, ny, nz;
    const uint8_t *mask;   // (nz, ny, nx); bool bytes, or bit1 = nonzero | bit0 = low bit
    int is_bool;
    int thickness;         // >= 1 dilation iterations
    int64_t step;          // sampling_step >= 1
    double lo[3], span[3], den[3];  // x, y, z: lo + (idx * span) / den
};
size_t boundary_blocks(int64_t nvox);
// dilation passes + per-block counts + their exclusive scan (counts: boundary_blocks + 1
// entries, total at [nb]); ping/pong: nvox bytes each when thickness > 1
int launch_boundary_count(const BoundaryLaunch &m, uint8_t *ping, uint8_t *pong, unsigned long long *counts,
                          const uint8_t **grown_out, hipStream_t s);
int launch_boundary_emit(const BoundaryLaunch &m, const uint8_t *grown, const unsigned long long *offsets,
                         double *ox, double *oy, double *oz, hipStream_t s);

// ---- k-NN outlier filter (ptv_filter.hip) ----
int filter_kmax(int k);
int launch_pad_queries(const double *x, const double *y, const double *z, int64_t n, int64_t npad, double *qx,
                       double *qy, double *qz, hipStream_t s);
int launch_binned_queries(const double4 *prec, int64_t n, int64_t npad, double *qx, double *qy, double *qz,
                          hipStream_t s);
size_t morton_sort_temp_bytes(int64_t n);
// perm = particle indices sorted by a 30-bit Morton code over [lo, hi] (stable)
int launch_morton_order(const double *x, const double *y, const double *z, int64_t n, const double lo[3],
                        const double hi[3], uint32_t *keys, uint32_t *keys_out, uint32_t *ids, uint32_t *perm,
                        void *temp, size_t temp_bytes, hipStream_t s);
// speed sqrt((u^2 + v^2) + w^2) of every binned particle in slot order
int launch_slot_speed(const double4 *pval, int64_t n, double *spd, hipStream_t s);
// point-list query arrays (npad) in the sub-ball lane layout of the Morton order, and the
// original index of the query at each position (q_orig, ~0 for the pads)
int launch_query_layout(const uint32_t *perm, const double *x, const double *y, const double *z, int64_t n,
                        int64_t npad, double *qx, double *qy, double *qz, uint32_t *q_orig, hipStream_t s);

}  // namespace ptv
