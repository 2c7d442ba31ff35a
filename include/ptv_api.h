/*
 * ptv_api.h — C ABI of the MI355X-native PTV scattered-to-grid interpolator.
 *
 * Drop-in boundary for the per-voxel neighbour search + weighted average of
 * the reference `interpolator.interpolate_field` (tombultreys/ptv_interpolation,
 * interpolator.py:65-203).  Plain C types only: pointers + sizes, no torch or
 * HIP types in any signature.  Every entry point returns 0 on success and a
 * negative PTV_E* code on failure; `ptv_last_error()` then holds a message
 * (thread-local).  The Python mirror of the reference interface lives in
 * ptv_interpolation_amd/interpolator.py and binds these symbols with ctypes.
 *
 * Threading: one ptv_ctx per (process, device).  A ctx is not re-entrant;
 * calls on one ctx are synchronous with respect to the host unless the
 * *_dev variant is given a stream, in which case all work is enqueued on
 * that stream and the call returns after the enqueue (the stats fields
 * are filled at the next synchronising call).
 */
#ifndef PTV_API_H
#define PTV_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTV_API_VERSION 10

/* error codes */
#define PTV_OK 0
#define PTV_E_ARG -1      /* invalid argument (Python: ValueError)          */
#define PTV_E_HIP -2      /* HIP runtime / launch failure (RuntimeError)    */
#define PTV_E_NOMEM -3    /* device allocation failed (MemoryError)         */
#define PTV_E_UNSUPPORTED -4 /* valid but not implemented on the GPU path  */
#define PTV_E_INEXACT -5  /* slab_halo too small to prove the culled set exact (see ptv_knn_params) */
#define PTV_E_SINGULAR -6 /* local RBF system singular (Python: LinAlgError) */

/* interpolation methods (interpolator.py:83, :126, :157, :197) */
#define PTV_METHOD_IDW 0
#define PTV_METHOD_SIBSON 1
#define PTV_METHOD_NEAREST 2
/* Extension (no reference counterpart; parity unpinned): IDW over every particle
 * within ptv_knn_params.radius of the voxel (scipy query_ball_point's d2 <= r*r test), weights
 * 1/(d**power + eps) as interpolator.py:142-147, out = sum w u / sum w; an empty ball gives NaN.
 * k is ignored.  BASELINE config 2 ("IDW radius-search"). */
#define PTV_METHOD_IDW_RADIUS 3

/* local RBF kernels (scipy RBFInterpolator names, _rbfinterp.py:19-28) */
#define PTV_RBF_LINEAR 0
#define PTV_RBF_THIN_PLATE_SPLINE 1
#define PTV_RBF_CUBIC 2
#define PTV_RBF_QUINTIC 3
#define PTV_RBF_MULTIQUADRIC 4
#define PTV_RBF_INVERSE_MULTIQUADRIC 5
#define PTV_RBF_INVERSE_QUADRATIC 6
#define PTV_RBF_GAUSSIAN 7

/* flags for ptv_knn_params.flags / ptv_rbf_params.flags */
#define PTV_FLAG_NAN_TO_NUM 1u  /* fused main.py:195-199 nan_to_num on the outputs */
/* k-NN methods: write U, V, W as float32 (the buffers passed as `double *` then hold float):
 * the fused `U.astype(np.float32)` of main.py:230, applied after the float64 result, the
 * nan_to_num and the mask (half the output bytes).  Arithmetic stays float64. */
#define PTV_FLAG_OUT_F32 2u
/* local RBF, diagnostics: SPD systems through the LDS-broadcast kernel (k_rbf_spd, the one the
 * register kernel's out-of-range-pivot rerun uses) instead of k_rbf_spd16 (ABI v8) */
#define PTV_FLAG_RBF_SPD_LDS 4u
/* local RBF, diagnostics: the scale-invariant kernels through the partial-pivoting solver
 * (k_rbf_local) instead of the null-space solver k_rbf_ns (ABI v9) */
#define PTV_FLAG_RBF_PIVOTING 8u
/* k-NN, diagnostics (k >= 13): near-tie repair list of one entry, so that a launch with two or more
 * tiles to repair takes the whole-launch exact rerun (the path past the 2^22-tile list) (ABI v9) */
#define PTV_FLAG_KNN_REPAIR_ALL 16u
/* k-NN interpolation on a z-slab of a separable grid (z_begin > 0 or z_end < nz): bin only the
 * particles that can be among a slab voxel's k nearest, by a per-(x, y)-column cull map (ABI v10).
 * Replaces the scalar slab_halo (ignored under this flag) for the multi-GPU z-slab split with the
 * particle set replicated (interpolator.py:173-182 fanned out over GPUs).  The
 * context derives the map from the slab's own finest lattice bounds: every voxel v of a lattice
 * cell Q has d_k(v) <= U(Q) = max over Q's corners of D(c) + Q's half diagonal, so only particles
 * within U(Q) of some cell Q are needed; per column that is a height above / depth below the slab.
 * The first call for a (particle arrays, n, 96-value fingerprint, grid, slab, k, method) key bins
 * every particle and caches the map; later calls cull with it and PROVE on the device, from the
 * lattice of the kept particles, that the map covers what the slab needs before the main kernel
 * runs (a failed proof -- the particles changed under the same arrays -- reruns the call without
 * the cull and refreshes the map).  Results are bit-identical to the unculled call.
 * ptv_stats.n_binned reports the particles kept. */
#define PTV_FLAG_SLAB_CULL_AUTO 32u

typedef struct ptv_ctx ptv_ctx;

/*
 * Particles, structure of arrays, float64 (the reference upcasts every input
 * to float64: interpolator.py:78-79 -> cKDTree / numpy arithmetic).
 * Replaces: `points = df[['x','y','z']].values; values = df[['u','v','w']].values`
 *           (interpolator.py:78-79).
 */
typedef struct {
    int64_t n;
    const double *x, *y, *z; /* positions */
    const double *u, *v, *w; /* velocity components */
} ptv_particles;

/*
 * Query grid.  Separable regular grid: the 1-D axes returned by
 * `create_grid` (interpolator.py:54-56) — voxel (iz, iy, ix) sits at
 * (ax[ix], ay[iy], az[iz]), C order (nz, ny, nx) with x fastest exactly as
 * `np.stack([X.ravel(), Y.ravel(), Z.ravel()], -1)` (interpolator.py:135).
 * Point-list mode: ax/ay/az NULL and px/py/pz hold nx*ny*nz coordinates in
 * the same C order (any grid shape the caller passes, interpolator.py:77).
 * Only planes [z_begin, z_end) are computed (multi-GPU z-slab).
 */
typedef struct {
    int64_t nx, ny, nz;
    const double *ax, *ay, *az;
    const double *px, *py, *pz;
    int64_t z_begin, z_end;
} ptv_grid;

/*
 * k-NN interpolation parameters (interpolate_field kwargs, interpolator.py:65).
 * fluid_mask: optional uint8 (nz, ny, nx) over the FULL grid, nonzero = fluid
 * (interpolator.py:37); solid voxels are written as 0 and skipped
 * (fused main.py:202-207).  NULL = compute every voxel.
 */
typedef struct {
    int method;          /* PTV_METHOD_* */
    int k;               /* idw_neighbors / sibson_neighbors, 1 <= k <= n (k >= 128: the large-k path) */
    double power;        /* idw_power (interpolator.py:143) */
    double eps;          /* 1e-10 (interpolator.py:102, :142) */
    const uint8_t *fluid_mask;
    uint32_t flags;      /* PTV_FLAG_* */
    double cell_occupancy; /* target particles per binning cell, <=0: default */
    double r0_scale;       /* first search radius / expected k-NN radius, <=0: default */
    int lattice_bounds;    /* >=0: coarse-lattice k-th distance bounds (default), <0: off */
    /* Multi-GPU z-slab with the particle set replicated: > 0 bins only the
     * particles whose z lies within slab_halo of the slab's z extent [az[z_begin], az[z_end-1]]
     * (separable grids; order-preserving on-device compaction).  Exactness is then PROVEN
     * before the main kernel: from the finest lattice's k-th distance bounds D(c) every slab
     * voxel v has d_k(v) <= D(c) + |v - c|, and a particle outside the window is farther than
     * slab_halo + (v's distance to the nearer slab face); the call computes the halo that
     * guarantees this (ptv_stats.halo_required) and returns PTV_E_INEXACT without running the
     * interpolation when slab_halo is smaller (retry with halo_required, or 0 = no cull).
     * <= 0: every particle is binned (no check needed).  k-NN interpolation entry points only. */
    double slab_halo;
    double radius;         /* PTV_METHOD_IDW_RADIUS: the search radius (> 0) */
} ptv_knn_params;

/*
 * Local RBF parameters (interpolate_field rbf kwargs, interpolator.py:162-167, and the
 * RBFInterpolator constructor they feed, _rbfinterp.py:258-345).  The caller resolves
 * scipy's defaults and validation first (ptv_interpolation_amd/rbf.py): k is
 * min(neighbors, n) (:322), epsilon is 1.0 for the scale-invariant kernels (:300-309),
 * degree defaults to max(min_degree, 0) (:311-313).
 */
typedef struct {
    int k;                /* rbf_neighbors, 1 <= k <= n */
    int kernel;           /* PTV_RBF_* */
    double epsilon;       /* shape parameter */
    int degree;           /* polynomial degree, -1 = no polynomial (systems k + C(degree+3, 3) > 128:
                           * solved in global memory, k_rbf_huge) */
    double smoothing;     /* scalar smoothing, used when smoothing_per_point is NULL */
    const double *smoothing_per_point; /* optional (n,) array, same memory space as the particles */
    const uint8_t *fluid_mask;        /* as ptv_knn_params.fluid_mask */
    uint32_t flags;       /* PTV_FLAG_* */
    int chunk_planes;     /* z planes per k-NN + solve chunk (multiple of 4), <= 0: automatic */
} ptv_rbf_params;

/* Per-call timings (ms, hipEvent based) and sizes. */
typedef struct {
    double ms_h2d, ms_bin, ms_lattice, ms_knn, ms_d2h, ms_total;
    int64_t n_particles, n_voxels, n_cells;
    int32_t cells[3];
    double cell_size[3];
    double r0;
    double ms_solve;     /* local RBF: the per-voxel solve kernels (ms_knn = their k-NN passes) */
    int64_t n_singular;  /* local RBF: voxels whose system had an exactly zero pivot */
    double ms_stencil;   /* ptv_divergence*: the stencil kernel */
    int64_t n_binned;    /* particles binned (after the slab_halo cull; = n_particles without) */
    double halo_required;/* slab_halo cull: the smallest halo this call proves exact (-1: no cull) */
    double ms_cull;      /* slab_halo cull + exactness check (inside ms_bin / before ms_knn) */
    int64_t n_repair_tiles; /* k >= 13: 4x4x4 tiles rerun with exact (d2, slot) lists because two
                             * distinct distances shared a packed key's truncation (ABI v8) */
    int64_t n_rbf_pivoted;  /* local RBF, scale-invariant kernels: voxels the null-space solver handed
                             * to the partial-pivoting solver (rank-deficient polynomial block, a
                             * non-positive pivot, ...; ABI v9) */
} ptv_stats;

/*
 * Consistent divergence (physics.compute_consistent_divergence, physics.py:6-53).
 * Fields U, V, W and the uint8 fluid mask (nonzero = fluid, required: the reference
 * np.roll()s it, physics.py:31-32) are (nz, ny, nx) C order.  Planes [z_begin, z_end)
 * are written to `out` as (z_end - z_begin, ny, nx).  Plane 0 / nz-1 of the buffer is
 * a domain z edge when edge_lo / edge_hi is set, else a one-plane halo of the
 * neighbouring z-slab that is read but not computed (z-slab multi-GPU).
 * Types follow numpy: field_dtype is the fields' dtype; result_dtype the dtype of
 * (field difference) / spacing — PTV_F32 only for float32 fields with Python-float
 * spacings, PTV_F64 when a spacing is a numpy float64 scalar (view_divergence.py:22).
 */
#define PTV_F64 0
#define PTV_F32 1
typedef struct {
    int64_t nx, ny, nz;
    int64_t z_begin, z_end;
    int edge_lo, edge_hi;
    int field_dtype;     /* PTV_F64 | PTV_F32 */
    int result_dtype;    /* PTV_F64 | PTV_F32 */
    double dx, dy, dz;
    const uint8_t *fluid_mask;
} ptv_div_params;

/*
 * Raw pore mask for sample_mask_on_grid (interpolator.py:205-238).  `raw` is
 * (nz, ny, nx) C order, one byte per voxel, nonzero where the raw value
 * `mask_raw.astype(float)` is > 0.5 (for a bool mask: the mask itself).  The axes are
 * the raw voxel coordinates `linspace(min, max-1, n)` (or `[min]` when n == 1) and are
 * always HOST arrays (n doubles each); `raw` lives in the call's memory space.
 */
typedef struct {
    int64_t nx, ny, nz;
    const uint8_t *raw;
    const double *ax, *ay, *az;
} ptv_mask_grid;

/*
 * Boundary particles (extract_boundary_particles, interpolator.py:240-284).
 * mask: (nz, ny, nx) bytes.  encoding PTV_MASK_BOOL: bytes are 0/1 (a numpy bool mask);
 * PTV_MASK_BITS: bit 1 = (value != 0), bit 0 = (value & 1) (an integer mask, for which
 * numpy's `dilated & ~mask` keeps the low bit only).  Coordinates per axis (x, y, z):
 * lo + (index * span) / den with span = max - 1 - min and den = n - 1
 * (interpolator.py:278-280; the caller handles n == 1, where the reference returns ints).
 */
#define PTV_MASK_BOOL 0
#define PTV_MASK_BITS 1
typedef struct {
    int64_t nx, ny, nz;
    const uint8_t *mask;
    int encoding;          /* PTV_MASK_BOOL | PTV_MASK_BITS */
    int thickness;         /* binary_dilation iterations, >= 1 */
    int64_t sampling_step; /* take every Nth boundary voxel (C order), >= 1 */
    double lo[3], span[3], den[3];
} ptv_boundary_params;

/*
 * k-NN median/MAD outlier filter (filtering.py:5-58 remove_outliers_knn).
 * k: neighbours excluding the point itself (the reference queries k+1, :26), 1 <= k < n
 * (k >= 127: the large-k path);
 * threshold: MAD units (:47-51); mad_eps: 1e-6 (:46).
 */
typedef struct {
    int k;
    double threshold;
    double mad_eps;
} ptv_filter_params;

/*
 * Linear interpolation over a Delaunay triangulation: method='linear', the reference's default
 * (interpolator.py:196-197 `griddata(points, values, grid_coords, method='linear',
 * fill_value=0.0)` -> scipy LinearNDInterpolator).  The caller builds
 * `tri = scipy.spatial.Delaunay(points)` on the host, exactly as LinearNDInterpolator does (Qhull),
 * and passes its arrays; the GPU locates every voxel in it (walk from a simplex incident to the
 * voxel's nearest particle, scipy's brute-force scan where the walk meets a degenerate simplex)
 * and interpolates with scipy's barycentric arithmetic.  Arrays follow numpy's C layouts
 * (int32 / float64) and live in the call's memory space.
 */
typedef struct {
    int64_t nsimplex;
    const int32_t *simplices;         /* (nsimplex, 4) particle indices: tri.simplices */
    const int32_t *neighbors;         /* (nsimplex, 4) tri.neighbors (-1 = hull face) */
    const double *transform;          /* (nsimplex, 4, 3) tri.transform (NaN rows: degenerate) */
    const int32_t *vertex_to_simplex; /* (n,) a simplex incident to each particle (walk start;
                                         tri.vertex_to_simplex with tri.coplanar points filled in) */
    double min_bound[3], max_bound[3];/* tri.min_bound, tri.max_bound */
    double fill_value;                /* griddata fill_value (0.0 in interpolator.py:197) */
    const uint8_t *fluid_mask;        /* as ptv_knn_params.fluid_mask */
    uint32_t flags;                   /* PTV_FLAG_NAN_TO_NUM only */
    int chunk_planes;                 /* z planes per nearest-particle + walk chunk (multiple of 4), <= 0: auto */
} ptv_linear_params;

/* Library / device management. */
int ptv_version(void);
/* sizeof(ptv_particles, ptv_grid, ptv_knn_params, ptv_stats, ptv_rbf_params, ptv_div_params):
 * binding self-check */
int ptv_abi_sizes(int64_t out6[6]);
/* sizeof(ptv_mask_grid, ptv_boundary_params, ptv_filter_params): the same self-check */
int ptv_abi_sizes2(int64_t out3[3]);
/* sizeof(ptv_linear_params): the same self-check */
int ptv_abi_sizes3(int64_t out1[1]);
const char *ptv_last_error(void);
int ptv_device_count(int *out);
int ptv_init(int device, ptv_ctx **out);
int ptv_free(ptv_ctx *ctx);

/*
 * k-NN IDW / Sibson interpolation, host buffers.
 * Replaces the `method == 'idw'` branch (interpolator.py:126-155) and the
 * `method == 'sibson'` branch (interpolator.py:83-124): KDTree build
 * (:90,:132), query (:97,:139), weights (:102-116,:142-147), gather-sum
 * (:119-122,:150-153), reshape (:124,:155,:199-203).
 * Outputs U, V, W: caller-owned float64 (z_end-z_begin, ny, nx) C order.
 */
int ptv_interp_knn(ptv_ctx *ctx, const ptv_particles *p, const ptv_grid *g,
                   const ptv_knn_params *prm, double *U, double *V, double *W,
                   ptv_stats *st);

/*
 * Same, every pointer (particles, axes/points, mask, outputs) is DEVICE
 * memory on the ctx's device; work is enqueued on `stream` (hipStream_t,
 * NULL = the ctx's own stream) and the call returns after the enqueue.
 */
int ptv_interp_knn_dev(ptv_ctx *ctx, const ptv_particles *p, const ptv_grid *g,
                       const ptv_knn_params *prm, double *U, double *V, double *W,
                       void *stream, ptv_stats *st);

/*
 * Local RBF interpolation, host buffers.
 * Replaces the `method == 'rbf'` branch (interpolator.py:157-195) through scipy's
 * RBFInterpolator(neighbors=k) evaluation (_rbfinterp.py:463-556): the KDTree build and
 * query (:345, :513), the sort of each neighbourhood (:521), the per-neighbourhood
 * system build (_build_system) and dgesv solve (:82-127), and the evaluation
 * (_build_evaluation_coefficients @ coeffs, :384-418).  A system with an exactly zero
 * pivot returns PTV_E_SINGULAR (scipy: LinAlgError "Singular matrix.", :115-127);
 * the outputs are then undefined.
 */
int ptv_interp_rbf_local(ptv_ctx *ctx, const ptv_particles *p, const ptv_grid *g,
                         const ptv_rbf_params *prm, double *U, double *V, double *W,
                         ptv_stats *st);

/* Same on device pointers; enqueued on `stream`, but synchronises once at the end to
 * read the singular-system count (the return code depends on it). */
int ptv_interp_rbf_local_dev(ptv_ctx *ctx, const ptv_particles *p, const ptv_grid *g,
                             const ptv_rbf_params *prm, double *U, double *V, double *W,
                             void *stream, ptv_stats *st);

/*
 * Linear (Delaunay) interpolation, host buffers.  Replaces the griddata branch for
 * method='linear' (interpolator.py:196-197): LinearNDInterpolator's point location
 * (_find_simplex: bounding-box test, directed walk, brute force) and barycentric
 * interpolation (interpnd _do_evaluate), fill_value outside the hull.  Outputs as
 * ptv_interp_knn (float64).
 */
int ptv_interp_linear(ptv_ctx *ctx, const ptv_particles *p, const ptv_grid *g,
                      const ptv_linear_params *prm, double *U, double *V, double *W,
                      ptv_stats *st);

/* Same on device pointers (particles, grid, triangulation arrays, mask, outputs); enqueued on
 * `stream`, synchronises once at the end (the brute-force count decides a second kernel). */
int ptv_interp_linear_dev(ptv_ctx *ctx, const ptv_particles *p, const ptv_grid *g,
                          const ptv_linear_params *prm, double *U, double *V, double *W,
                          void *stream, ptv_stats *st);

/*
 * Consistent divergence, host buffers: H2D of the fields and mask, one stencil kernel,
 * D2H of the slab.  Replaces compute_consistent_divergence(u, v, w, mask, dx, dy, dz)
 * (physics.py:6-53; callers view_divergence.py:39,42, physics.py:173,193-194).
 */
int ptv_divergence(ptv_ctx *ctx, const ptv_div_params *prm, const void *U, const void *V,
                   const void *W, void *out, ptv_stats *st);

/* Same on device pointers (fields, mask, out), enqueued on `stream` (NULL = ctx's). */
int ptv_divergence_dev(ptv_ctx *ctx, const ptv_div_params *prm, const void *U, const void *V,
                       const void *W, void *out, void *stream, ptv_stats *st);

/*
 * Nearest-neighbour resampling of a raw mask onto the grid, host buffers.  Replaces
 * sample_mask_on_grid (interpolator.py:205-238): RegularGridInterpolator((z, y, x),
 * mask_raw.astype(float), method='nearest', bounds_error=False, fill_value=0) at every
 * grid voxel, then `> 0.5`.  out: (z_end - z_begin, ny, nx) bytes, 1 = fluid.
 */
int ptv_sample_mask(ptv_ctx *ctx, const ptv_mask_grid *src, const ptv_grid *g, uint8_t *out);

/* Same; src->raw, the grid arrays and `out` are DEVICE memory (src axes stay host). */
int ptv_sample_mask_dev(ptv_ctx *ctx, const ptv_mask_grid *src, const ptv_grid *g, uint8_t *out,
                        void *stream);

/*
 * Boundary particles, host buffers.  Replaces extract_boundary_particles
 * (interpolator.py:240-284): binary_dilation(mask, 6-connected, iterations=thickness)
 * & ~mask, np.where in C order, [::sampling_step], physical coordinates.
 * *count receives the number of particles; x, y, z (cap entries each) are written only
 * when cap >= *count (call once with cap = 0 to size them).
 */
int ptv_boundary_particles(ptv_ctx *ctx, const ptv_boundary_params *prm, double *x, double *y,
                           double *z, int64_t cap, int64_t *count);

/* Same; prm->mask and x, y, z are DEVICE memory.  Synchronises (the count is returned). */
int ptv_boundary_particles_dev(ptv_ctx *ctx, const ptv_boundary_params *prm, double *x,
                               double *y, double *z, int64_t cap, int64_t *count, void *stream);

/*
 * k-NN outlier filter, host buffers.  Replaces remove_outliers_knn (filtering.py:5-58):
 * KDTree(points).query(points, k+1) minus the point itself (:20-30), the median and MAD
 * of the neighbours' speeds (:38-44) and the z-score test (:47-51).
 * keep: n bytes, 1 = keep (original particle order).  kth_dist: optional (NULL) n
 * doubles, the distance to the (k+1)-th neighbour counting the point itself
 * (`dist[:, -1]`, whose median the reference prints, :33-35).  Requires n > k
 * (the reference skips the filter otherwise, :12-14).
 */
int ptv_filter_outliers_knn(ptv_ctx *ctx, const ptv_particles *p, const ptv_filter_params *prm,
                            uint8_t *keep, double *kth_dist, ptv_stats *st);

/* Same on device pointers, enqueued on `stream` (NULL = the ctx's own stream). */
int ptv_filter_outliers_knn_dev(ptv_ctx *ctx, const ptv_particles *p, const ptv_filter_params *prm,
                                uint8_t *keep, double *kth_dist, void *stream, ptv_stats *st);

/*
 * Last-launch k-NN kernel duration in ms (hipEvent pair recorded around the
 * kernel on the stream it ran on) and the synchronised phase stats.
 */
int ptv_last_stats(ptv_ctx *ctx, ptv_stats *st);

/*
 * Diagnostics: mode 1 = enable + zero per-wave phase stamps of the k-NN kernel (k <= 8
 * launches switch to an s_memtime-stamped build), 0 = disable, other = leave.  If out
 * != NULL (23 doubles) it receives {waves recorded, mean[11], max[11]} over the fields
 * {setup, seeds, rows, copy, compute, epilogue cycles, gathered candidates, merge
 * iterations, rounds, passes, candidates kept by the sub-ball filter}.
 * Profiling only: stamps perturb the schedule; never time a stamped run.
 */
int ptv_debug_stamps(ptv_ctx *ctx, int mode, double *out23);

#ifdef __cplusplus
}
#endif

#endif /* PTV_API_H */
