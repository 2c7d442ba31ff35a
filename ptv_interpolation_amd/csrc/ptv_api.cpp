// ptv_api.cpp — C ABI (include/ptv_api.h): context, device buffers, host/device entry points.
//
// The Python drop-in (ptv_interpolation_amd/interpolator.py) binds these symbols with
// ctypes; nothing here depends on torch.  One context = one device + one stream +
// grow-only device buffers reused across calls (the reference rebuilds its KDTree on
// every call, interpolator.py:90/:132; here the binning runs every call too, but no
// allocation does once the buffers are warm).
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>

#include <sys/mman.h>
#include <vector>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"
#include "ptv_knn_big.hpp"

namespace ptv {

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }


}  // namespace ptv

using namespace ptv;

static constexpr int kMaxLattice = 6;

struct ptv_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_knn0 = nullptr, ev_knn1 = nullptr, ev_bin0 = nullptr, ev_bin1 = nullptr, ev_lat1 = nullptr;
    hipEvent_t ev_main0 = nullptr, ev_cull0 = nullptr, ev_cull1 = nullptr;  // main-kernel start; slab cull
    bool cull_timed = false;
    bool timed_pending = false;
    BigScratch big;  // the large-k path (ptv_knn_big.hip)
    DevBuf<double> pin[6], axes, qpts[3], out[3];
    DevBuf<double> rbf_huge;  // k_rbf_huge's per-workgroup slices (m > 128)
    DevBuf<uint8_t> mask;
    DevBuf<uint32_t> code, perm, count, start, scanp;
    DevBuf<uint32_t> bin_keys;                                   // sort-based binning: sorted cell codes
    DevBuf<uint8_t> bin_temp;                                    //   and the radix sort's scratch
    DevBuf<double4> prec, pval;
    DevBuf<double> bbox_part, bbox_out;
    DevBuf<unsigned long long> dbg;
    DevBuf<double> lat_axes[kMaxLattice], lat_dk[kMaxLattice];  // coarse-lattice bound levels
    DevBuf<float4> lat_recs[kMaxLattice];                        // their k-NN records (seeds, fp32 relative)
    DevBuf<int> lat_order[kMaxLattice];                          // longest-first block order per level
    DevBuf<double> lat_okeys;                                    // its block keys (scratch)
    DevBuf<uint32_t> lat_split;                                  // split lattice launch: partial lists
    // PTV_FLAG_SLAB_CULL_AUTO: the cached per-column cull map (top, bot), its key, the proof's
    // need map and scratch
    DevBuf<double> cmap[2], cdk, ccols, cfp;  // map (top, bot), the lattice bounds it came from, scratch
    DevBuf<unsigned long long> ckeys;
    CullMap cmap_geo{};
    int cdk_n[3] = {0, 0, 0};
    bool cmap_valid = false;
    std::vector<double> ckey, ckey_new;
    // the speculative reuse of the cached map (no host synchronisation before the gated launch): the
    // host part of the key, the data part on the device, the kept count and bounding box of the
    // last proven culled call
    std::vector<double> ckey_host;
    DevBuf<double> ckey_dev;
    bool ckept_valid = false;
    int64_t ckept = 0;
    double cbbox[6] = {0, 0, 0, 0, 0, 0};
    DevBuf<uint32_t> slots;                                      // local RBF: chunk k-NN slots
    DevBuf<int> rbf_pw, rbf_status;                              // monomial exponents, singular count
    DevBuf<uint32_t> rbf_nslist;                                 // local RBF: voxels k_rbf_ns hands over
    DevBuf<int> rbf_cflag;                                       // local RBF: per chunk flagged / overflow
    DevBuf<double> smooth;                                       // per-particle smoothing (host calls)
    DevBuf<uint8_t> fld[4];                                      // divergence host calls: U, V, W, out
    DevBuf<double> mask_axes;                                    // sample_mask: raw axes (ascending)
    DevBuf<int> mask_tabs;                                       // sample_mask: per-axis index tables
    DevBuf<uint8_t> mask_raw, mask_out;                          // sample_mask host calls
    DevBuf<uint8_t> bnd_ping, bnd_pong;                          // boundary: dilation passes
    DevBuf<unsigned long long> bnd_counts;                       // boundary: per-block counts / offsets
    DevBuf<double> bnd_xyz;                                      // boundary host calls: coordinates
    DevBuf<uint8_t> flt_keep;                                    // outlier filter host calls
    DevBuf<uint32_t> flt_code, flt_perm, flt_count, flt_start, flt_scanp;  // filter: Morton keys/ids, sort temp
    DevBuf<double> flt_kth, flt_spd;
    DevBuf<double> cull[6], cull_win;                            // slab cull: kept particles, z window
    DevBuf<uint32_t> cull_cnt;                                   // slab cull: per-block counts
    DevBuf<unsigned long long> cull_mask;                        // slab cull: keep masks (pass 1 -> pass 2)
    DevBuf<unsigned long long> halo_need;                        // slab cull: proven halo (double bits)
    DevBuf<unsigned int> rep_cnt;                                // key-list near-tie repair: count
    DevBuf<uint32_t> rep_list;                                   //   and the listed tiles
    hipEvent_t ev_div0 = nullptr, ev_div1 = nullptr;             // around the divergence stencil
    bool div_pending = false;
    std::vector<hipEvent_t> rbf_ev;                              // 3 per chunk: knn start, solve start, end
    int rbf_chunks = 0;
    DevBuf<int> lin_simp, lin_nbr, lin_v2s, lin_count;           // linear: triangulation (host calls), flags
    DevBuf<double> lin_tr;
    DevBuf<long long> lin_flags;                                 // linear: voxels left to the brute force
    double *h_bbox = nullptr;  // pinned, 6 doubles
    unsigned long long *h_misc = nullptr;  // pinned scratch words (cull count, halo bound, repair count)
    ptv_stats last{};
};

extern "C" {

int ptv_version(void) { return PTV_API_VERSION; }

int ptv_abi_sizes(int64_t out6[6]) {
    if (!out6) {
        set_error("ptv_abi_sizes: out is NULL");
        return PTV_E_ARG;
    }
    out6[0] = (int64_t)sizeof(ptv_particles);
    out6[1] = (int64_t)sizeof(ptv_grid);
    out6[2] = (int64_t)sizeof(ptv_knn_params);
    out6[3] = (int64_t)sizeof(ptv_stats);
    out6[4] = (int64_t)sizeof(ptv_rbf_params);
    out6[5] = (int64_t)sizeof(ptv_div_params);
    return PTV_OK;
}

int ptv_abi_sizes2(int64_t out3[3]) {
    if (!out3) {
        set_error("ptv_abi_sizes2: out is NULL");
        return PTV_E_ARG;
    }
    out3[0] = (int64_t)sizeof(ptv_mask_grid);
    out3[1] = (int64_t)sizeof(ptv_boundary_params);
    out3[2] = (int64_t)sizeof(ptv_filter_params);
    return PTV_OK;
}

int ptv_abi_sizes3(int64_t out1[1]) {
    if (!out1) {
        set_error("ptv_abi_sizes3: out is NULL");
        return PTV_E_ARG;
    }
    out1[0] = (int64_t)sizeof(ptv_linear_params);
    return PTV_OK;
}

const char *ptv_last_error(void) { return g_last_error.c_str(); }

int ptv_device_count(int *out) {
    if (!out) {
        set_error("ptv_device_count: out is NULL");
        return PTV_E_ARG;
    }
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return PTV_OK;
}

int ptv_init(int device, ptv_ctx **out) {
    if (!out) {
        set_error("ptv_init: out is NULL");
        return PTV_E_ARG;
    }
    *out = nullptr;
    int n = 0;
    PTV_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) {
        set_error("ptv_init: device " + std::to_string(device) + " out of range (" + std::to_string(n) + " visible)");
        return PTV_E_ARG;
    }
    PTV_HIP(hipSetDevice(device));
    ptv_ctx *c = new ptv_ctx();
    c->device = device;
    PTV_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    PTV_HIP(hipEventCreate(&c->ev_knn0));
    PTV_HIP(hipEventCreate(&c->ev_knn1));
    PTV_HIP(hipEventCreate(&c->ev_bin0));
    PTV_HIP(hipEventCreate(&c->ev_bin1));
    PTV_HIP(hipEventCreate(&c->ev_lat1));
    PTV_HIP(hipEventCreate(&c->ev_main0));
    PTV_HIP(hipEventCreate(&c->ev_cull0));
    PTV_HIP(hipEventCreate(&c->ev_cull1));
    PTV_HIP(hipEventCreate(&c->ev_div0));
    PTV_HIP(hipEventCreate(&c->ev_div1));
    PTV_HIP(hipHostMalloc(&c->h_bbox, 8 * sizeof(double)));
    PTV_HIP(hipHostMalloc(&c->h_misc, 8 * sizeof(unsigned long long)));
    *out = c;
    return PTV_OK;
}

int ptv_free(ptv_ctx *c) {
    if (!c) return PTV_OK;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    for (auto &b : c->pin) b.release();
    for (auto &b : c->qpts) b.release();
    for (auto &b : c->out) b.release();
    c->axes.release();
    c->mask.release();
    c->code.release();
    c->perm.release();
    c->count.release();
    c->bin_keys.release();
    c->bin_temp.release();
    c->start.release();
    c->scanp.release();
    c->prec.release();
    c->pval.release();
    c->bbox_part.release();
    c->bbox_out.release();
    if (ptv::g_dbg == c->dbg.p) ptv::g_dbg = nullptr;
    c->dbg.release();
    for (auto &b : c->lat_axes) b.release();
    for (auto &b : c->lat_dk) b.release();
    for (auto &b : c->lat_recs) b.release();
    for (auto &b : c->lat_order) b.release();
    c->lat_okeys.release();
    c->big.release();
    c->rbf_huge.release();
    c->lat_split.release();
    for (auto &b : c->cmap) b.release();
    c->cdk.release();
    c->ccols.release();
    c->cfp.release();
    c->ckey_dev.release();
    c->ckeys.release();
    c->slots.release();
    c->rbf_pw.release();
    c->rbf_status.release();
    c->rbf_nslist.release();
    c->rbf_cflag.release();
    c->lin_simp.release();
    c->lin_nbr.release();
    c->lin_v2s.release();
    c->lin_count.release();
    c->lin_tr.release();
    c->lin_flags.release();
    c->smooth.release();
    for (auto &b : c->fld) b.release();
    c->mask_axes.release();
    c->mask_tabs.release();
    c->mask_raw.release();
    c->mask_out.release();
    c->bnd_ping.release();
    c->bnd_pong.release();
    c->bnd_counts.release();
    c->bnd_xyz.release();
    c->flt_keep.release();
    for (auto *b : {&c->flt_code, &c->flt_perm, &c->flt_count, &c->flt_start, &c->flt_scanp}) b->release();
    c->flt_kth.release();
    c->flt_spd.release();
    for (auto &b : c->cull) b.release();
    c->cull_win.release();
    c->cull_cnt.release();
    c->cull_mask.release();
    c->halo_need.release();
    c->rep_cnt.release();
    c->rep_list.release();
    if (c->h_misc) hipHostFree(c->h_misc);
    hipEventDestroy(c->ev_main0);
    hipEventDestroy(c->ev_cull0);
    hipEventDestroy(c->ev_cull1);
    hipEventDestroy(c->ev_div0);
    hipEventDestroy(c->ev_div1);
    for (hipEvent_t e : c->rbf_ev) hipEventDestroy(e);
    if (c->h_bbox) hipHostFree(c->h_bbox);
    hipEventDestroy(c->ev_knn0);
    hipEventDestroy(c->ev_knn1);
    hipEventDestroy(c->ev_bin0);
    hipEventDestroy(c->ev_bin1);
    hipEventDestroy(c->ev_lat1);
    hipStreamDestroy(c->stream);
    delete c;
    return PTV_OK;
}

}  // extern "C"

namespace {

// particles per binning cell: the k <= 8 kernels (seeded, sub-ball filtered copy) are fastest
// with coarse cells (fewer, longer runs per row: 512^3 / 5M k=8 main launch 19.1 -> 16.5 ms
// from 1.2 to 5.5); the larger-k kernels prefer fine cells (k=50: 477 ms at 1.2, 493 at 5.5)
// measured on the 512^3 / 5M sphere pack, k = 8 (tools/void_split.py, round 2): per-cell
// occupancy 16 / 12 with cells 12x thinner along x (16 particles per x-column of 12 cells)
// gave k-NN 14.9 ms against 16.3 ms for cubic cells of 5.5, the lattice 2.31 against 2.44
constexpr double kDefaultOccupancySmallK = 16.0;  // particles per (y, z) cell column segment
constexpr double kDefaultXRefSmallK = 12.0;       // x-refinement of the k <= 8 cells
constexpr double kDefaultOccupancy = 1.2;          // k > 8 without lattice seeds (point lists)
// k > 8 with union seeds (round 3, a dev-knob sweep, now tools/gpu_envab.sh, 512^3 / 5M IDW k = 50): the seeded
// gather radius is tight, so coarser cells (fewer runs per row) win again: main launch
// 139.7 ms at 1.2 / cubic, 137.7 at 2.5, 134.8 at 5, 133.5 at 8 with x 4x thinner, 133.4 at 16 / 12
constexpr double kDefaultOccupancyLargeK = 8.0;
constexpr double kDefaultXRefLargeK = 4.0;
// the outlier filter's particle queries (5M, k = 25): 23.3 ms at 1.2, 22.6 at 2.5, 22.4 at 5,
// 24.1 at 8 / 4, 28.4 at 16 / 12
constexpr double kFilterOccupancy = 5.0;
// the filter's first gather radius, in units of the expected (k+1)-NN radius: its queries sit on
// the particles (the pack's sphere shells), so the mean-density radius overshoots.  Same-box sweep
// (5M particles, k = 25, search ms): 1.0 19.79, 0.75 19.51, 0.6 19.45, 0.45 19.42, 0.3 23.25
constexpr double kFilterR0Scale = 0.6;
constexpr double kDefaultR0Scale = 1.0;     // first gather radius / expected k-NN radius
constexpr long long kMaxCells = 1LL << 28;
constexpr long long kLatticeStopPoints = 50000; // no coarser lattice below this many points
constexpr size_t kSeedBytesMax = 40ULL << 30;    // lattice seed records per level (C5 2048^3, k = 8: 17 GB)
// split lattice launch (k_kdist_merge): the first max(kLatticeSplitMinBlocks, blocks /
// kLatticeSplitDiv) blocks of a lattice level's longest-first order, kLatticeSplit waves per tile.
// Measured (512^3 / 5M sphere pack, k = 8, a dev-knob sweep, now tools/gpu_envab.sh): the share 2/8 lattice 1.81 ->
// 0.88 ms at 64 blocks (1.07 at 32, 2.05 at 8), C2 0.81 -> 0.69; the whole 512^3 grid's lattice
// launch is throughput-bound (35.9k tiles of ~280k cycles each), 1.91 -> 1.86 ms
constexpr int kLatticeSplit = 16;
constexpr long long kLatticeSplitMinBlocks = 64;
constexpr long long kLatticeSplitDiv = 128;
// cap on the split launch's partial-list buffer (split_blocks * 4 * kLatticeSplit * KMAX * 64 slots,
// memset once per level): 64 MiB = 512 blocks at KMAX 8, 32 at 128; the measured win came from the
// first ~64 blocks, while nb / 128 at 2048^3 would be ~4300 blocks (0.56 GB at k = 8, 9 GB at 127)
constexpr size_t kLatticeSplitBytesMax = 64ULL << 20;
// binning: the radix sort above this many particles, the atomic counting sort below (crossover
// ~2.6M from the two measured points, profiles/r06_ab/bin_sort_ab.txt)
constexpr int64_t kBinSortMinParticles = 2500000;
// relative widening of the cached slab cull map over the need it was built from
constexpr double kCullMapSlack = 1e-6;

int validate(const ptv_particles *p, const ptv_grid *g, const void *prm) {
    if (!p || !g || !prm) {
        set_error("NULL particles/grid/params");
        return PTV_E_ARG;
    }
    if (p->n <= 0 || !p->x || !p->y || !p->z || !p->u || !p->v || !p->w) {
        set_error("particles: need n > 0 and six non-NULL arrays");
        return PTV_E_ARG;
    }
    if (p->n >= (int64_t)1 << 31) {
        set_error("particles: n must be < 2^31");
        return PTV_E_ARG;
    }
    if (g->nx <= 0 || g->ny <= 0 || g->nz <= 0 || g->nx > (1 << 30) || g->ny > (1 << 30)) {
        set_error("grid: dimensions must be positive");
        return PTV_E_ARG;
    }
    const bool sep = g->ax && g->ay && g->az;
    const bool pts = g->px && g->py && g->pz;
    if (!sep && !pts) {
        set_error("grid: give either the three axes or the three point arrays");
        return PTV_E_ARG;
    }
    if (g->z_begin < 0 || g->z_end > g->nz || g->z_begin > g->z_end) {
        set_error("grid: bad z slab [" + std::to_string(g->z_begin) + ", " + std::to_string(g->z_end) + ")");
        return PTV_E_ARG;
    }
    return PTV_OK;
}

int validate_knn(const ptv_particles *p, const ptv_knn_params *prm) {
    if (prm->method != PTV_METHOD_IDW && prm->method != PTV_METHOD_SIBSON && prm->method != PTV_METHOD_NEAREST &&
        prm->method != PTV_METHOD_IDW_RADIUS) {
        set_error("unknown method " + std::to_string(prm->method));
        return PTV_E_ARG;
    }
    if (prm->method == PTV_METHOD_IDW_RADIUS) {
        if (!(prm->radius > 0.0 && std::isfinite(prm->radius))) {
            set_error("PTV_METHOD_IDW_RADIUS needs a positive finite radius");
            return PTV_E_ARG;
        }
        return PTV_OK;  // k is not used
    }
    if (prm->k < 1) {
        set_error("k must be >= 1");
        return PTV_E_ARG;
    }
    if ((int64_t)prm->k > p->n) {
        set_error("k=" + std::to_string(prm->k) + " exceeds the number of particles " + std::to_string(p->n));
        return PTV_E_ARG;
    }
    // k beyond the register lists (kmax_for(k) == 0, k >= 128) takes the large-k path (run_knn_big)
    return PTV_OK;
}

// Cell grid over the union bounding box: ~`occ` particles per cell on average.
CellGrid make_cell_grid(const double lo_in[3], const double hi_in[3], int64_t n, double occ, double xref_in) {
    CellGrid cg{};
    double ext[3];
    double maxext = 0.0, maxabs = 0.0;
    for (int a = 0; a < 3; ++a) {
        ext[a] = hi_in[a] - lo_in[a];
        if (!(ext[a] > 0.0)) ext[a] = 0.0;
        maxext = std::max(maxext, ext[a]);
        maxabs = std::max(maxabs, std::max(std::fabs(lo_in[a]), std::fabs(hi_in[a])));
    }
    if (!(occ > 0.0)) occ = kDefaultOccupancy;
    if (const char *e = dev_knob("PTV_CELL_OCC")) occ = std::atof(e);  // dev override
    double vol = 1.0;
    int dims = 0;
    for (int a = 0; a < 3; ++a)
        if (ext[a] > 1e-9 * maxext) {
            vol *= ext[a];
            ++dims;
        }
    double cs = dims ? std::pow(occ * vol / (double)n, 1.0 / dims) : 1.0;
    // x-refinement: cells `xref` times thinner along x (occupancy / xref per cell).  A gather
    // run is a contiguous x-range of cells whose cost is its two cstart loads whatever its
    // length, so thin x-cells trim the runs' ends (fewer candidates outside the sub-balls)
    // without adding rows.
    double xref = std::max(1.0, xref_in);
    if (const char *e = dev_knob("PTV_CELL_XREF")) xref = std::max(1.0, std::atof(e));  // dev override
    for (int iter = 0; iter < 64; ++iter) {  // cap the cell count (memory) by growing cs
        long long tot = 1;
        for (int a = 0; a < 3; ++a) {
            int nc = 1;
            const double csa = a == 0 ? cs / xref : cs;
            if (ext[a] > 1e-9 * maxext && csa > 0.0) nc = (int)std::max(1.0, std::min(1e6, std::ceil(ext[a] / csa)));
            cg.nc[a] = nc;
            tot *= nc;
        }
        cg.ncells = tot;
        if (tot <= kMaxCells) break;
        cs *= 1.1;
    }
    for (int a = 0; a < 3; ++a) {
        cg.cs[a] = ext[a] > 0.0 ? ext[a] / cg.nc[a] : 1.0;
        cg.ic[a] = 1.0 / cg.cs[a];
        cg.o[a] = lo_in[a];
    }
    cg.mg = 1e-12 * (maxabs + maxext) + 1e-300;
    return cg;
}

// First gather radius: the radius of a ball expected to hold k particles at the mean
// density of the bounding box, times `scale` (every lane's k-th distance usually fits).
double first_radius(const double lo[3], const double hi[3], int64_t n, int k, double scale) {
    if (!(scale > 0.0)) scale = kDefaultR0Scale;
    double vol = 1.0, maxext = 0.0;
    int dims = 0;
    for (int a = 0; a < 3; ++a) maxext = std::max(maxext, hi[a] - lo[a]);
    for (int a = 0; a < 3; ++a)
        if (hi[a] - lo[a] > 1e-9 * maxext) {
            vol *= hi[a] - lo[a];
            ++dims;
        }
    if (dims == 0 || maxext <= 0.0) return 1.0;
    const double unit = dims == 3 ? 4.18879020478639 : (dims == 2 ? 3.14159265358979 : 2.0);
    return scale * std::pow((double)k * vol / ((double)n * unit), 1.0 / dims);
}

// Search settings shared by the k-NN consumers (IDW/Sibson epilogue, local RBF).
struct SearchParams {
    int method;  // PTV_METHOD_* (k-NN interpolation), ignored by the RBF path
    int k;
    double power, eps;
    uint32_t flags;
    double cell_occupancy, r0_scale;
    int lattice_bounds;
};

// Steps 1-3 of every call: bounding box, binning, coarse-lattice k-th distance bounds.
// Fills `kl` with a launch template for planes [z_begin, z_end) of the grid.
int prepare(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const SearchParams *prm, const double *ax,
            const double *ay, const double *az, const double *qx, const double *qy, const double *qz, hipStream_t s,
            KnnLaunch &kl, Binned &bout, const double *known_bbox = nullptr, bool exact_finest = false) {
    const int64_t n = p->n;
    const bool sep = ax != nullptr;
    const int64_t plane = g->nx * g->ny;
    const int64_t z0 = g->z_begin, z1 = g->z_end;
    const int64_t nvox = (z1 - z0) * plane;

    // 1. bounding box of particles + this slab's queries
    PTV_TRY(c->bbox_part.ensure(6 * 1024));
    PTV_TRY(c->bbox_out.ensure(8));
    const double *pp[3] = {p->x, p->y, p->z};
    const double *qa[3];
    int64_t qn[3];
    if (sep) {
        qa[0] = ax;
        qa[1] = ay;
        qa[2] = az + z0;
        qn[0] = g->nx;
        qn[1] = g->ny;
        qn[2] = z1 - z0;
    } else {
        qa[0] = qx + z0 * plane;
        qa[1] = qy + z0 * plane;
        qa[2] = qz + z0 * plane;
        qn[0] = qn[1] = qn[2] = nvox;
    }
    PTV_HIP(hipEventRecord(c->ev_bin0, s));
    if (known_bbox == nullptr) {  // (the slab cull reads it back together with its kept count)
        PTV_TRY(launch_bbox(pp, n, qa, qn, c->bbox_part.p, 1024, c->bbox_out.p, s));
        PTV_HIP(hipMemcpyAsync(c->h_bbox, c->bbox_out.p, 6 * sizeof(double), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipStreamSynchronize(s));
        known_bbox = c->h_bbox;
    }
    double lo[3] = {known_bbox[0], known_bbox[1], known_bbox[2]};
    double hi[3] = {known_bbox[3], known_bbox[4], known_bbox[5]};
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) {
            set_error("non-finite particle or grid coordinates");
            return PTV_E_ARG;
        }
    }

    // 2. binning
    const bool small_k = kmax_for(prm->k) <= 8;
    const bool seeded_lattice = sep && prm->lattice_bounds >= 0;  // union seeds bound the large-k search
    const bool given = prm->cell_occupancy > 0.0;
    const double occ = given ? prm->cell_occupancy
                       : (small_k ? kDefaultOccupancySmallK : (seeded_lattice ? kDefaultOccupancyLargeK : kDefaultOccupancy));
    const double xref = given ? 1.0 : (small_k ? kDefaultXRefSmallK : (seeded_lattice ? kDefaultXRefLargeK : 1.0));
    CellGrid cg = make_cell_grid(lo, hi, n, occ, xref);
    const size_t m = (size_t)cg.ncells;
    PTV_TRY(c->code.ensure(2 * (size_t)n));  // cell codes + in-cell ranks (launch_bin)
    PTV_TRY(c->perm.ensure(n));
    PTV_TRY(c->prec.ensure(n));
    PTV_TRY(c->pval.ensure(n));
    PTV_TRY(c->count.ensure(m));
    PTV_TRY(c->start.ensure(m + 1));
    PTV_TRY(c->scanp.ensure(scan_partials_needed(m) + 1));
    const double *pv[3] = {p->u, p->v, p->w};
    // sort-based binning (a stable radix sort of (cell, index) pairs) from kBinSortMinParticles:
    // 512^3 / 5M binning 0.81 -> 0.68 ms against the atomic histogram + scatter + in-cell sort,
    // the 0.73M particles of share 2/8 0.134 -> 0.22 ms (profiles/r06_ab/bin_sort_ab.txt)
    BinSortScratch ss;
    const char *bs = dev_knob("PTV_BIN_SORT");  // dev knob: 0 = the atomic counting sort, 1 = the sort
    const bool use_sort = bs ? bs[0] == '1' : n >= kBinSortMinParticles;
    const size_t tb = use_sort ? bin_sort_temp_bytes(n, m) : 0;
    if (tb > 0) {
        PTV_TRY(c->bin_keys.ensure((size_t)n));
        PTV_TRY(c->bin_temp.ensure(std::max<size_t>(tb, 1)));
        ss.keys = c->bin_keys.p;
        ss.temp = c->bin_temp.p;
        ss.temp_bytes = tb;
    }
    PTV_TRY(launch_bin(cg, pp, pv, n, c->code.p, c->perm.p, c->count.p, c->start.p, c->scanp.p, c->prec.p,
                       c->pval.p, s, &ss));
    PTV_HIP(hipEventRecord(c->ev_bin1, s));

    // Seed records for the main launch (the finest level's k-NN lists) pay for the pair lists (k <=
    // 12): headline 22.4 -> 14.1 ms with them, k = 12 33.2 -> 29.4 ms.  For the packed-key lists (k >=
    // 13) the union-seed counting costs more than its tighter bound saves, and the finest level then
    // writes no records either (1.7 GB per launch at k = 50).  Same-box A/B, 512^3 / 5M, main launch
    // + lattice without / with them: k = 16 34.8 + 2.14 / 35.9 + 2.23 ms, Sibson k = 30 54.1 + 2.71 /
    // 55.2 + 2.84, IDW k = 50 102.3 + 5.13 / 104.2 + 5.40, Sibson k = 50 137.9 + 5.09 / 138.8 +
    // 5.38, RBF slot searches k = 20 29.0 / 29.9 and C3 48.4 / 50.0.
    bool main_seeds = kmax_for(prm->k) <= 12;
    if (const char *e = dev_knob("PTV_MAIN_SEEDS")) main_seeds = e[0] == '1';  // dev knob: 1 = always, 0 = never
    // 3. coarse-lattice k-th distance bounds (separable grids): every 4th point of the
    //    grid, recursively, down to a few tens of thousands of points; each level is an
    //    exact k-NN pass (k-th distance only) bounded by the next coarser level.
    struct Lat {
        int n[3];
        double *ax, *ay, *az, *dk;
        float4 *recs;   // NULL on the coarsest (count-bound) level and past kSeedBytesMax
    };
    Lat lat[kMaxLattice];
    int nlat = 0;
    if (sep && prm->lattice_bounds >= 0) {
        int n[3] = {(int)g->nx, (int)g->ny, (int)(z1 - z0)};
        // every level's axes from the grid's in one launch (each level takes every 4th point of the
        // one above it, plus the last)
        SubsampleBatch sb{};
        for (int d = 0; d < 3; ++d) sb.n0[d] = n[d];
        sb.base[0] = ax;
        sb.base[1] = ay;
        sb.base[2] = az + z0;
        while (nlat < kMaxLattice) {
            const long long pts = (long long)n[0] * n[1] * n[2];
            long long stop = kLatticeStopPoints;
            if (const char *e = dev_knob("PTV_LAT_STOP")) stop = std::atoll(e);  // dev override
            const int nmin = std::min(n[0], std::min(n[1], n[2]));
            // exact_finest (the slab cull map): a count-bound level above the finest, which is then an
            // exact k-th distance level (its bounds do not depend on the binning cells)
            if ((pts <= stop || nmin < 9) && !(exact_finest && nlat == 1 && nmin >= 2)) break;
            Lat &L = lat[nlat];
            for (int d = 0; d < 3; ++d) L.n[d] = n[d] <= 1 ? 1 : (n[d] - 1 + kLatticeStep - 1) / kLatticeStep + 1;
            PTV_TRY(c->lat_axes[nlat].ensure((size_t)L.n[0] + L.n[1] + L.n[2]));
            PTV_TRY(c->lat_dk[nlat].ensure((size_t)L.n[0] * L.n[1] * L.n[2]));
            L.ax = c->lat_axes[nlat].p;
            L.ay = L.ax + L.n[0];
            L.az = L.ay + L.n[1];
            L.dk = c->lat_dk[nlat].p;
            L.recs = nullptr;
            double *dst[3] = {L.ax, L.ay, L.az};
            for (int d = 0; d < 3; ++d) {
                sb.n[nlat][d] = L.n[d];
                sb.out[nlat][d] = dst[d];
                n[d] = L.n[d];
            }
            ++nlat;
        }
        sb.nlev = nlat;
        if (nlat > 0) PTV_TRY(launch_subsample_levels(sb, kLatticeStep, s));
    }

    // 4. launch template (k-NN search + consumer)
    kl.cg = cg;
    kl.nx = (int)g->nx;
    kl.ny = (int)g->ny;
    kl.nz = (int)g->nz;
    kl.z0 = (int)z0;
    kl.z1 = (int)z1;
    kl.separable = sep ? 1 : 0;
    kl.method = prm->method == PTV_METHOD_NEAREST ? PTV_METHOD_IDW : prm->method;
    kl.k = prm->k;
    kl.power = prm->power;
    kl.eps = prm->eps;
    kl.flags = prm->flags;
    kl.r0 = first_radius(lo, hi, n, prm->k, prm->r0_scale);
    Binned b{c->prec.p, c->pval.p, c->start.p, n};
    bout = b;
    PTV_HIP(hipEventRecord(c->ev_knn0, s));
    for (int l = nlat - 1; l >= 0; --l) {  // coarsest first
        if (l == nlat - 1) {
            // coarsest lattice: count-only upper bounds (no candidate is read)
            PTV_TRY(launch_count_bound(cg, c->start.p, lat[l].ax, lat[l].ay, lat[l].az, lat[l].n[0], lat[l].n[1],
                                       lat[l].n[2], prm->k, kl.r0, lat[l].dk, s));
            continue;
        }
        // seed records (each lattice point's k-NN, 16 B each) for the next finer level's tiles,
        // unless they would take more than kSeedBytesMax (then the D(c) + |v - c| bound alone)
        const size_t nrec = (size_t)lat[l].n[0] * lat[l].n[1] * lat[l].n[2] * prm->k;
        if ((l > 0 || main_seeds) && nrec * sizeof(float4) <= kSeedBytesMax) {
            PTV_TRY(c->lat_recs[l].ensure(nrec));
            lat[l].recs = c->lat_recs[l].p;
        }
        KnnLaunch ll = kl;
        const char *no_order = dev_knob("PTV_NO_LAT_ORDER");  // dev knob: 1 = XCD-contiguous order
        if (!(no_order && no_order[0] == '1')) {
            const long long nb = (long long)(((lat[l].n[0] + 3) / 4 + 3) / 4) * ((lat[l].n[1] + 3) / 4) *
                                 ((lat[l].n[2] + 3) / 4);
            PTV_TRY(c->lat_order[l].ensure((size_t)nb));
            PTV_TRY(c->lat_okeys.ensure((size_t)nb + 1));
            PTV_TRY(launch_block_order(lat[l + 1].dk, lat[l + 1].n, lat[l].n[0], lat[l].n[1], lat[l].n[2], kl.r0,
                                       c->lat_order[l].p, c->lat_okeys.p, s));
            ll.order = c->lat_order[l].p;
            if (const char *e = dev_knob("PTV_DBG_ORDER")) {  // dev builds: the order and the coarser bounds
                if (l == 0) {
                    const size_t nc = (size_t)lat[1].n[0] * lat[1].n[1] * lat[1].n[2];
                    std::vector<int> ho((size_t)nb);
                    std::vector<double> hd(nc);
                    PTV_HIP(hipMemcpyAsync(ho.data(), ll.order, nb * sizeof(int), hipMemcpyDeviceToHost, s));
                    PTV_HIP(hipMemcpyAsync(hd.data(), lat[1].dk, nc * sizeof(double), hipMemcpyDeviceToHost, s));
                    PTV_HIP(hipStreamSynchronize(s));
                    if (FILE *f = std::fopen(e, "wb")) {
                        std::fwrite(lat[1].n, sizeof(int), 3, f);
                        std::fwrite(hd.data(), sizeof(double), nc, f);
                        std::fwrite(ho.data(), sizeof(int), ho.size(), f);
                        std::fclose(f);
                    }
                }
            }
            // the first blocks of the order (the void tiles) as a split launch (k_kdist_merge)
            int split = kLatticeSplit;
            long long sblk = std::min<long long>(nb, std::max<long long>(kLatticeSplitMinBlocks, nb / kLatticeSplitDiv));
            if (const char *e = dev_knob("PTV_LAT_SPLIT")) split = std::atoi(e);          // dev: 0 = off
            if (const char *e = dev_knob("PTV_LAT_SPLIT_BLOCKS")) sblk = std::min<long long>(nb, std::atoll(e));
            if (split > 1)
                sblk = std::min<long long>(sblk, (long long)(kLatticeSplitBytesMax / sizeof(uint32_t) /
                                                             kdist_split_slots(split, 1, kmax_for(prm->k))));
            if (split > 1 && sblk > 0) {
                PTV_TRY(c->lat_split.ensure(kdist_split_slots(split, (int)sblk, kmax_for(prm->k))));
                ll.split = split;
                ll.split_blocks = (int)sblk;
                ll.split_out = c->lat_split.p;
            }
        }
        ll.kd_recs = lat[l].recs;
        ll.nx = lat[l].n[0];
        ll.ny = lat[l].n[1];
        ll.nz = lat[l].n[2];
        ll.z0 = 0;
        ll.z1 = lat[l].n[2];
        ll.mode = kModeKDist;
        ll.flags = 0;
        ll.cb.ax = lat[l + 1].ax;
        ll.cb.ay = lat[l + 1].ay;
        ll.cb.az = lat[l + 1].az;
        ll.cb.dk = lat[l + 1].dk;
        ll.cb.recs = lat[l + 1].recs;
        if (const char *e = dev_knob("PTV_LAT_SEEDS"))  // dev knob: 0 = lattice levels unseeded
            if (e[0] == '0') ll.cb.recs = nullptr;
        for (int d = 0; d < 3; ++d) ll.cb.n[d] = lat[l + 1].n[d];
        PTV_TRY(launch_knn(ll, b, lat[l].ax, lat[l].ay, lat[l].az, nullptr, nullptr, nullptr, nullptr, lat[l].dk,
                           lat[l].dk, lat[l].dk, s));
    }
    if (nlat > 0) {
        kl.cb.ax = lat[0].ax;
        kl.cb.ay = lat[0].ay;
        kl.cb.az = lat[0].az;
        kl.cb.dk = lat[0].dk;
        kl.cb.recs = lat[0].recs;  // NULL unless main_seeds
        for (int d = 0; d < 3; ++d) kl.cb.n[d] = lat[0].n[d];
    }
    PTV_HIP(hipEventRecord(c->ev_lat1, s));
    PTV_HIP(hipEventRecord(c->ev_main0, s));  // moved to the main launch when a check runs in between
    if (const char *e = dev_knob("PTV_DBG_LATDK")) {  // dev builds: the finest lattice bounds to a file
        if (nlat > 0) {
            const size_t np = (size_t)lat[0].n[0] * lat[0].n[1] * lat[0].n[2];
            std::vector<double> h(np);
            PTV_HIP(hipMemcpyAsync(h.data(), lat[0].dk, np * sizeof(double), hipMemcpyDeviceToHost, s));
            PTV_HIP(hipStreamSynchronize(s));
            if (FILE *f = std::fopen(e, "wb")) {
                std::fwrite(lat[0].n, sizeof(int), 3, f);
                std::fwrite(h.data(), sizeof(double), np, f);
                std::fclose(f);
            }
        }
    }

    ptv_stats &ls = c->last;
    ls = ptv_stats{};
    ls.n_particles = n;
    ls.n_voxels = nvox;
    ls.n_cells = (int64_t)cg.nc[0] * cg.nc[1] * cg.nc[2];
    for (int a = 0; a < 3; ++a) {
        ls.cells[a] = cg.nc[a];
        ls.cell_size[a] = cg.cs[a];
    }
    ls.r0 = kl.r0;
    ls.n_binned = n;
    ls.halo_required = -1.0;
    if (kmax_for(prm->k) >= 16) {
        // packed-key lists: the near-tie repair list (tiles whose order the keys did not prove;
        // a handful per launch: past the cap the whole launch reruns exact)
        const long long tiles = (long long)((g->nx + 3) / 4) * ((g->ny + 3) / 4) * ((z1 - z0 + 3) / 4);
        // (PTV_FLAG_KNN_REPAIR_ALL: a one-entry list, so any second listed tile reruns the whole launch)
        const int cap = (prm->flags & PTV_FLAG_KNN_REPAIR_ALL)
                            ? 1
                            : (int)std::max<long long>(1, std::min<long long>(tiles, 1LL << 22));
        PTV_TRY(c->rep_cnt.ensure(1));
        PTV_TRY(c->rep_list.ensure((size_t)cap));
        kl.rep_cnt = c->rep_cnt.p;
        kl.rep_list = c->rep_list.p;
        kl.rep_cap = cap;
        kl.h_rep = reinterpret_cast<unsigned int *>(c->h_misc + 2);
        kl.n_repair = &ls.n_repair_tiles;
    }
    return PTV_OK;
}

// Whether prepare() will build the coarse lattice for planes [z0, z1) of a separable grid
// (the same test as its loop's first iteration).
bool lattice_built(const ptv_grid *g, int lattice_bounds) {
    if (lattice_bounds < 0) return false;
    const long long n[3] = {g->nx, g->ny, g->z_end - g->z_begin};
    long long stop = kLatticeStopPoints;
    if (const char *e = dev_knob("PTV_LAT_STOP")) stop = std::atoll(e);
    return n[0] * n[1] * n[2] > stop && std::min(n[0], std::min(n[1], n[2])) >= 9;
}

SearchParams knn_search(const ptv_knn_params *prm) {
    return SearchParams{prm->method, prm->k, prm->power, prm->eps, prm->flags, prm->cell_occupancy, prm->r0_scale,
                        prm->lattice_bounds};
}

// PTV_FLAG_SLAB_CULL_AUTO (see ptv_api.h): the per-column cull map, cached per context.  A call
// whose key matches the cached map culls with it and proves the cull on the device (the need map
// of the kept particles' lattice inside the used map everywhere) before the gated main launch; a
// call without a cached map (or whose proof fails) bins every particle and builds the map from its
// own lattice.  Key: the particle arrays, n, a 96-value fingerprint, the axis values, the grid, the
// slab, k, method.
int run_knn_auto(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_knn_params *prm,
                 const double *ax, const double *ay, const double *az, const uint8_t *mask, double *U, double *V,
                 double *W, hipStream_t s, ptv_stats *st) {
    const SearchParams sp = knn_search(prm);
    const int64_t n = p->n;
    const double *src[6] = {p->x, p->y, p->z, p->u, p->v, p->w};
    // the fingerprint, then the grid's axis values: the map and the cached lattice bounds belong to
    // lattice positions, and a reused axis buffer (the host path's c->axes, a recycled torch
    // allocation) can hold other coordinates under the same pointer.  Gathered on the device and
    // read back in one copy (one copy per array cost ~20 us each)
    const size_t nfp = 6 * kFingerprint, nkey = nfp + (size_t)(g->nx + g->ny + g->nz);
    PTV_TRY(c->cfp.ensure(nkey));
    PTV_TRY(launch_fingerprint(src, n, c->cfp.p, s));
    PTV_TRY(launch_concat3(ax, (int)g->nx, ay, (int)g->ny, az, (int)g->nz, c->cfp.p + nfp, s));
    // the host part of the key: the arrays, n, the grid, the slab, k, method
    std::vector<double> hkey;
    for (const void *q : {(const void *)p->x, (const void *)p->y, (const void *)p->z, (const void *)p->u,
                          (const void *)p->v, (const void *)p->w, (const void *)ax, (const void *)ay,
                          (const void *)az}) {
        uint64_t bits = (uint64_t)(uintptr_t)q;
        double d;
        std::memcpy(&d, &bits, sizeof(d));
        hkey.push_back(d);
    }
    for (int64_t v : {n, g->nx, g->ny, g->nz, g->z_begin, g->z_end, (int64_t)prm->k, (int64_t)prm->method,
                      (int64_t)prm->lattice_bounds})
        hkey.push_back((double)v);
    const bool host_match = c->cmap_valid && c->ckey_host.size() == hkey.size() &&
                            std::memcmp(c->ckey_host.data(), hkey.data(), hkey.size() * sizeof(double)) == 0 &&
                            c->ckey.size() == nkey + hkey.size();
    // speculative: a proven culled call already ran with this host key, so cull with the map at once and
    // let the device compare the data part (fingerprint + axis values) and the kept count, folded into
    // the gate of the main launch; the host reads the gate once, after it (no synchronisation before)
    bool spec = host_match && c->ckept_valid;
    std::vector<double> &key = c->ckey_new;
    auto read_key = [&]() -> int {
        key.assign(nkey, 0.0);
        PTV_HIP(hipMemcpyAsync(key.data(), c->cfp.p, nkey * sizeof(double), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipStreamSynchronize(s));
        key.insert(key.end(), hkey.begin(), hkey.end());
        return PTV_OK;
    };
    bool use_map = spec;
    if (!spec) {
        PTV_TRY(read_key());
        // bitwise comparison (a NaN fingerprint value never matches itself otherwise)
        use_map = c->cmap_valid && c->ckey.size() == key.size() &&
                  std::memcmp(c->ckey.data(), key.data(), key.size() * sizeof(double)) == 0;
    }
    if (dev_knob("PTV_DBG_CULL"))
        std::fprintf(stderr, "[cull] slab [%lld, %lld) n %lld: cached map %d, key match %d, speculative %d\n",
                     (long long)g->z_begin, (long long)g->z_end, (long long)n, (int)c->cmap_valid, (int)use_map,
                     (int)spec);
    for (int attempt = 0; attempt < 2; ++attempt) {
        KnnLaunch kl;
        Binned b{};
        ptv_particles pe = *p;
        bool culled = false;
        c->cull_timed = false;
        if (use_map) {
            const size_t nb = cull_blocks(n);
            for (auto &d : c->cull) PTV_TRY(d.ensure(n));
            PTV_TRY(c->cull_win.ensure(4));
            PTV_TRY(c->cull_cnt.ensure(nb + 1));
            PTV_TRY(c->cull_mask.ensure(cull_mask_words(n)));
            double *dst[6];
            for (int a = 0; a < 6; ++a) dst[a] = c->cull[a].p;
            CullMap used = c->cmap_geo;
            used.top = c->cmap[0].p;
            used.bot = c->cmap[1].p;
            uint32_t *h_total = reinterpret_cast<uint32_t *>(c->h_misc);
            PTV_HIP(hipEventRecord(c->ev_cull0, s));
            PTV_TRY(launch_cull(src, n, az, (int)g->z_begin, (int)g->z_end, 0.0, c->cull_win.p, c->cull_cnt.p,
                                c->cull_mask.p, dst, nullptr, s, &used));
            if (spec) {
                // the cached kept count and bounding box (the same particles give the same), checked on
                // the device: a mismatch fails the gate and the call reruns with every particle binned
                PTV_TRY(c->halo_need.ensure(1));
                PTV_HIP(hipMemsetAsync(c->halo_need.p, 0, sizeof(unsigned long long), s));
                PTV_TRY(launch_key_check(c->cfp.p, c->ckey_dev.p, (int)nkey, c->cull_cnt.p + nb, (uint32_t)c->ckept,
                                         c->halo_need.p, s));
                PTV_HIP(hipEventRecord(c->ev_cull1, s));
                std::memcpy(c->h_bbox, c->cbbox, sizeof(c->cbbox));
                pe = ptv_particles{c->ckept, dst[0], dst[1], dst[2], dst[3], dst[4], dst[5]};
                culled = true;
                c->cull_timed = true;
            }
        }
        if (use_map && !spec) {
            const size_t nb = cull_blocks(n);
            double *dst[6];
            for (int a = 0; a < 6; ++a) dst[a] = c->cull[a].p;
            uint32_t *h_total = reinterpret_cast<uint32_t *>(c->h_misc);
            PTV_TRY(c->bbox_part.ensure(6 * 1024));
            PTV_TRY(c->bbox_out.ensure(8));
            const double *kp[3] = {dst[0], dst[1], dst[2]};
            const double *qa[3] = {ax, ay, az + g->z_begin};
            const int64_t qn[3] = {g->nx, g->ny, g->z_end - g->z_begin};
            PTV_TRY(launch_bbox(kp, n, qa, qn, c->bbox_part.p, 1024, c->bbox_out.p, s, c->cull_cnt.p + nb));
            PTV_HIP(hipMemcpyAsync(c->h_bbox, c->bbox_out.p, 6 * sizeof(double), hipMemcpyDeviceToHost, s));
            PTV_HIP(hipMemcpyAsync(h_total, c->cull_cnt.p + nb, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            PTV_HIP(hipEventRecord(c->ev_cull1, s));
            PTV_HIP(hipStreamSynchronize(s));
            const int64_t kept = (int64_t)*h_total;
            if (kept >= prm->k) {
                pe = ptv_particles{kept, dst[0], dst[1], dst[2], dst[3], dst[4], dst[5]};
                culled = true;
                c->cull_timed = true;
            }
        }
        PTV_TRY(prepare(c, &pe, g, &sp, ax, ay, az, nullptr, nullptr, nullptr, s, kl, b, culled ? c->h_bbox : nullptr,
                        true));
        if (kl.cb.dk == nullptr) {
            // no lattice bounds (nothing to prove the cull or to build a map from): every particle
            if (culled) {
                culled = false;
                c->cull_timed = false;
                PTV_TRY(prepare(c, p, g, &sp, ax, ay, az, nullptr, nullptr, nullptr, s, kl, b, nullptr, true));
            }
            PTV_TRY(launch_knn(kl, b, ax, ay, az, nullptr, nullptr, nullptr, mask, U, V, W, s));
            PTV_HIP(hipEventRecord(c->ev_knn1, s));
            c->timed_pending = true;
            if (st) *st = c->last;
            return PTV_OK;
        }
        // the map geometry: cells of two finest-lattice cells per axis over the grid's (x, y) extent
        // (edge cells reach to infinity, so any extent is valid; it only sets the resolution)
        CullMap geo = c->cmap_geo;
        if (!culled) {
            double e[4];
            PTV_HIP(hipMemcpyAsync(&e[0], ax, sizeof(double), hipMemcpyDefault, s));
            PTV_HIP(hipMemcpyAsync(&e[1], ax + (g->nx - 1), sizeof(double), hipMemcpyDefault, s));
            PTV_HIP(hipMemcpyAsync(&e[2], ay, sizeof(double), hipMemcpyDefault, s));
            PTV_HIP(hipMemcpyAsync(&e[3], ay + (g->ny - 1), sizeof(double), hipMemcpyDefault, s));
            PTV_HIP(hipStreamSynchronize(s));
            geo = CullMap{};
            geo.mx = std::max(1, std::min(256, (kl.cb.n[0] - 1) / 2));
            geo.my = std::max(1, std::min(256, (kl.cb.n[1] - 1) / 2));
            geo.x0 = std::min(e[0], e[1]);
            geo.y0 = std::min(e[2], e[3]);
            const double wx = std::fabs(e[1] - e[0]), wy = std::fabs(e[3] - e[2]);
            geo.cw = wx > 0.0 && std::isfinite(wx) ? wx / geo.mx : 1.0;
            geo.ch = wy > 0.0 && std::isfinite(wy) ? wy / geo.my : 1.0;
            if (!std::isfinite(geo.x0)) geo.x0 = 0.0;
            if (!std::isfinite(geo.y0)) geo.y0 = 0.0;
            geo.icw = 1.0 / geo.cw;
            geo.ich = 1.0 / geo.ch;
        }
        const size_t nm = (size_t)geo.mx * geo.my;
        const size_t ncol = (size_t)std::max(kl.cb.n[0] - 1, 1) * std::max(kl.cb.n[1] - 1, 1);
        PTV_TRY(c->ccols.ensure(7 * ncol));
        PTV_TRY(c->ckeys.ensure(2 * nm));
        PTV_TRY(c->halo_need.ensure(1));
        const long long nlp = (long long)kl.cb.n[0] * kl.cb.n[1] * kl.cb.n[2];
        if (culled && !(kl.cb.n[0] == c->cdk_n[0] && kl.cb.n[1] == c->cdk_n[1] && kl.cb.n[2] == c->cdk_n[2])) {
            // (cannot happen for one key: the lattice follows the grid and the slab) a different
            // lattice proves nothing against the cached bounds: a failing gate, rerun below
            PTV_HIP(hipMemsetAsync(c->halo_need.p, 0xff, sizeof(unsigned long long), s));
            kl.gate = c->halo_need.p;
            kl.gate_halo = 0.0;
        } else if (culled) {
            // the proof, gating the main launch: the need map grows with the lattice bounds, and the
            // cached map was built from the bounds of the call that binned every particle (widened by
            // kCullMapSlack), so bounds of the kept particles within half that of the cached ones
            // prove that the map holds every particle a slab voxel can need
            PTV_TRY(launch_bounds_within(kl.cb.dk, c->cdk.p, nlp, 1.0 + 0.5 * kCullMapSlack, c->halo_need.p, s,
                                         !spec));
            kl.gate = c->halo_need.p;
            kl.gate_halo = 0.0;
            PTV_HIP(hipEventRecord(c->ev_main0, s));
        }
        PTV_TRY(launch_knn(kl, b, ax, ay, az, nullptr, nullptr, nullptr, mask, U, V, W, s));
        PTV_HIP(hipEventRecord(c->ev_knn1, s));
        c->timed_pending = true;
        c->last.n_particles = n;
        c->last.n_binned = pe.n;
        if (!culled) {
            // every particle binned: this call's lattice gives the map later calls cull with
            for (auto &d : c->cmap) PTV_TRY(d.ensure(nm));
            // (widened by kCullMapSlack: the packed-key lattice bounds of a culled call carry other slots in
            // their low bits, a few 1e-9 relative from this call's)
            PTV_TRY(launch_cull_need(kl.cb.ax, kl.cb.ay, kl.cb.az, kl.cb.n, kl.cb.dk, kl.cg.mg, kCullMapSlack, geo,
                                     c->cmap[0].p, c->cmap[1].p, c->ccols.p, c->ckeys.p, nullptr, nullptr, s));
            PTV_TRY(c->cdk.ensure((size_t)nlp));
            PTV_HIP(hipMemcpyAsync(c->cdk.p, kl.cb.dk, (size_t)nlp * sizeof(double), hipMemcpyDeviceToDevice, s));
            for (int d = 0; d < 3; ++d) c->cdk_n[d] = kl.cb.n[d];
            c->cmap_geo = geo;
            c->cmap_valid = true;
            c->ckey = key;
            c->ckey_host = hkey;
            PTV_TRY(c->ckey_dev.ensure(nkey));
            PTV_HIP(hipMemcpyAsync(c->ckey_dev.p, c->cfp.p, nkey * sizeof(double), hipMemcpyDeviceToDevice, s));
            c->ckept_valid = false;
            if (st) *st = c->last;
            return PTV_OK;
        }
        PTV_HIP(hipMemcpyAsync(c->h_misc + 1, c->halo_need.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipStreamSynchronize(s));
        if (dev_knob("PTV_DBG_CULL"))  // dev builds: the cull and its proof
            std::fprintf(stderr, "[cull] slab [%lld, %lld) kept %lld of %lld, map %dx%d, proof %llx\n",
                         (long long)g->z_begin, (long long)g->z_end, (long long)pe.n, (long long)n, geo.mx, geo.my,
                         (unsigned long long)c->h_misc[1]);
        if (c->h_misc[1] == 0ull) {  // proven: the gated launch wrote every output
            c->last.halo_required = 0.0;
            if (!spec) {  // later calls with this key may run speculatively
                c->ckept = pe.n;
                std::memcpy(c->cbbox, c->h_bbox, sizeof(c->cbbox));
                c->ckept_valid = true;
            }
            if (st) *st = c->last;
            return PTV_OK;
        }
        // not proven (the particles changed under the same arrays and fingerprint, or under a
        // speculative reuse the data key or kept count differed): no outputs were written; again with
        // every particle binned, which refreshes the map
        c->cmap_valid = false;
        c->ckept_valid = false;
        if (spec) {
            spec = false;
            PTV_TRY(read_key());  // the map built next is keyed by this call's data
        }
        use_map = false;
    }
    set_error("slab cull map: unreachable retry state");
    return PTV_E_HIP;
}

// k >= 128 (beyond the register lists): bin every particle (no lattice), then the large-k path --
// per-query ball bound, candidate gather, segmented sort, the reference's epilogue (ptv_knn_big.hip)
int run_knn_big(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_knn_params *prm, const double *ax,
                const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
                const uint8_t *mask, double *U, double *V, double *W, hipStream_t s, ptv_stats *st) {
    SearchParams sp = knn_search(prm);
    sp.lattice_bounds = -1;
    if (!(sp.cell_occupancy > 0.0)) sp.cell_occupancy = std::max(1.0, prm->k / 256.0);
    KnnLaunch kl;
    Binned b{};
    c->cull_timed = false;
    c->rbf_chunks = 0;
    PTV_TRY(prepare(c, p, g, &sp, ax, ay, az, qx, qy, qz, s, kl, b));
    BigQueries q;
    q.nx = (int)g->nx;
    q.ny = (int)g->ny;
    q.z0 = (int)g->z_begin;
    q.ax = ax;
    q.ay = ay;
    q.az = az;
    q.px = qx;
    q.py = qy;
    q.pz = qz;
    q.mask = mask;
    BigEpilogue ep;
    ep.method = prm->method;
    ep.power = prm->power;
    ep.eps = prm->eps;
    ep.flags = prm->flags;
    ep.U = U;
    ep.V = V;
    ep.W = W;
    const int64_t nvox = (g->z_end - g->z_begin) * g->nx * g->ny;
    PTV_TRY(run_big_knn(c->big, q, b, kl.cg, nvox, prm->k, ep, s));
    PTV_HIP(hipEventRecord(c->ev_knn1, s));
    c->timed_pending = true;
    c->last.n_particles = p->n;
    c->last.n_binned = p->n;
    if (st) *st = c->last;
    return PTV_OK;
}

int run_knn(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_knn_params *prm, const double *ax,
            const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
            const uint8_t *mask, double *U, double *V, double *W, hipStream_t s, ptv_stats *st) {
    if (prm->method != PTV_METHOD_IDW_RADIUS && kmax_for(prm->k) == 0)
        return run_knn_big(c, p, g, prm, ax, ay, az, qx, qy, qz, mask, U, V, W, s, st);
    if ((prm->flags & PTV_FLAG_SLAB_CULL_AUTO) && prm->method != PTV_METHOD_IDW_RADIUS && ax != nullptr &&
        (g->z_begin > 0 || g->z_end < g->nz) && lattice_built(g, prm->lattice_bounds))
        return run_knn_auto(c, p, g, prm, ax, ay, az, mask, U, V, W, s, st);
    SearchParams sp = knn_search(prm);
    const bool radius = prm->method == PTV_METHOD_IDW_RADIUS;
    if (radius) {
        // fixed-radius IDW: one pass over the radius ball, no k-th distance bounds or seeds
        sp.k = 1;
        sp.lattice_bounds = -1;
    }
    KnnLaunch kl;
    Binned b{};
    // slab cull (ptv_knn_params.slab_halo): bin only the particles near this z-slab
    ptv_particles pe = *p;
    bool culled = false;
    c->cull_timed = false;
    if (!radius && prm->slab_halo > 0.0 && ax != nullptr && lattice_built(g, prm->lattice_bounds)) {
        const int64_t n = p->n;
        const size_t nb = cull_blocks(n);
        for (auto &d : c->cull) PTV_TRY(d.ensure(n));
        PTV_TRY(c->cull_win.ensure(4));
        PTV_TRY(c->cull_cnt.ensure(nb + 1));
        PTV_TRY(c->cull_mask.ensure(cull_mask_words(n)));
        const double *src[6] = {p->x, p->y, p->z, p->u, p->v, p->w};
        double *dst[6];
        for (int a = 0; a < 6; ++a) dst[a] = c->cull[a].p;
        uint32_t *h_total = reinterpret_cast<uint32_t *>(c->h_misc);
        PTV_HIP(hipEventRecord(c->ev_cull0, s));
        PTV_TRY(launch_cull(src, n, az, (int)g->z_begin, (int)g->z_end, prm->slab_halo, c->cull_win.p,
                            c->cull_cnt.p, c->cull_mask.p, dst, nullptr, s));
        // the kept particles' bounding box (with the slab's query planes) from the count on the device,
        // read back with the count: one host synchronisation for the cull and the cell grid
        PTV_TRY(c->bbox_part.ensure(6 * 1024));
        PTV_TRY(c->bbox_out.ensure(8));
        const double *kp[3] = {dst[0], dst[1], dst[2]};
        const double *qa[3] = {ax, ay, az + g->z_begin};
        const int64_t qn[3] = {g->nx, g->ny, g->z_end - g->z_begin};
        PTV_TRY(launch_bbox(kp, n, qa, qn, c->bbox_part.p, 1024, c->bbox_out.p, s, c->cull_cnt.p + nb));
        PTV_HIP(hipMemcpyAsync(c->h_bbox, c->bbox_out.p, 6 * sizeof(double), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipMemcpyAsync(h_total, c->cull_cnt.p + nb, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipEventRecord(c->ev_cull1, s));
        PTV_HIP(hipStreamSynchronize(s));
        const int64_t kept = (int64_t)*h_total;
        if (kept >= prm->k) {  // fewer than k could never be proven exact: bin everything
            pe = ptv_particles{kept, dst[0], dst[1], dst[2], dst[3], dst[4], dst[5]};
            culled = true;
            c->cull_timed = true;
        }
    }
    PTV_TRY(prepare(c, &pe, g, &sp, ax, ay, az, qx, qy, qz, s, kl, b, culled ? c->h_bbox : nullptr));
    if (culled && kl.cb.dk == nullptr) {
        // no lattice bounds were built, so nothing proves the cull exact: bin every particle
        // instead (same result as slab_halo = 0), never refuse the call for it
        culled = false;
        c->cull_timed = false;
        PTV_TRY(prepare(c, p, g, &sp, ax, ay, az, qx, qy, qz, s, kl, b));
    }
    if (culled) {
        // the exactness proof runs on the device and gates the main launch (it writes nothing
        // unless the halo is proven); the host reads the proof back after it, so no
        // synchronisation stalls the stream between the lattice and the main launch
        PTV_TRY(c->halo_need.ensure(1));
        PTV_TRY(launch_halo_need(kl.cb.ax, kl.cb.ay, kl.cb.az, kl.cb.n[0], kl.cb.n[1], kl.cb.n[2], kl.cb.dk,
                                 c->cull_win.p, kl.cg.mg, c->halo_need.p, s));
        kl.gate = c->halo_need.p;
        kl.gate_halo = prm->slab_halo;
        PTV_HIP(hipEventRecord(c->ev_main0, s));
    }
    c->rbf_chunks = 0;
    if (radius) {
        kl.mode = kModeRadius;
        kl.radius = prm->radius;
    }
    PTV_TRY(launch_knn(kl, b, ax, ay, az, qx, qy, qz, mask, U, V, W, s));
    PTV_HIP(hipEventRecord(c->ev_knn1, s));
    c->timed_pending = true;
    if (culled) {
        PTV_HIP(hipMemcpyAsync(c->h_misc + 1, c->halo_need.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipStreamSynchronize(s));
        double need;
        std::memcpy(&need, &c->h_misc[1], sizeof(need));
        c->last.n_particles = p->n;
        c->last.n_binned = pe.n;
        c->last.halo_required = need;
        if (!(need <= prm->slab_halo)) {
            if (st) *st = c->last;  // halo_required for the caller's retry
            set_error("slab cull not proven exact: slab_halo " + std::to_string(prm->slab_halo) +
                      " < required " + std::to_string(need) + " (retry with >= halo_required, or 0)");
            return PTV_E_INEXACT;
        }
    }
    if (st) *st = c->last;
    return PTV_OK;
}

// monomial exponents of _monomial_powers(3, degree) (_rbfinterp.py:48-79), packed
std::vector<int> monomial_powers(int degree) {
    std::vector<int> out;
    for (int d = 0; d <= degree; ++d) {
        // combinations_with_replacement(range(3), d) in lexicographic order
        std::vector<int> idx(d, 0);
        while (true) {
            int pw[3] = {0, 0, 0};
            for (int v : idx) ++pw[v];
            out.push_back(pw[0] | (pw[1] << 8) | (pw[2] << 16));
            int i = d - 1;
            while (i >= 0 && idx[i] == 2) --i;
            if (i < 0) break;
            ++idx[i];
            for (int j = i + 1; j < d; ++j) idx[j] = idx[i];
        }
    }
    return out;
}

int validate_rbf(const ptv_particles *p, const ptv_rbf_params *prm, int *m_out) {
    if (prm->flags & PTV_FLAG_OUT_F32) {
        set_error("local RBF: PTV_FLAG_OUT_F32 is supported by the k-NN methods only");
        return PTV_E_UNSUPPORTED;
    }
    if (prm->kernel < PTV_RBF_LINEAR || prm->kernel > PTV_RBF_GAUSSIAN) {
        set_error("unknown RBF kernel " + std::to_string(prm->kernel));
        return PTV_E_ARG;
    }
    if (prm->k < 1 || (int64_t)prm->k > p->n) {
        set_error("k must be in [1, n]");
        return PTV_E_ARG;
    }
    if (prm->degree < -1 || prm->degree > 8) {
        set_error("degree must be in [-1, 8]");
        return PTV_E_ARG;
    }
    if (!std::isfinite(prm->epsilon)) {
        set_error("epsilon must be finite");
        return PTV_E_ARG;
    }
    const int nm = (int)monomial_powers(prm->degree).size();
    if (nm > prm->k) {
        set_error("At least " + std::to_string(nm) + " data points are required when `degree` is " +
                  std::to_string(prm->degree) + " and the number of dimensions is 3.");
        return PTV_E_ARG;
    }
    const int m = prm->k + nm;
    if (rbf_system_size(m) == 0) {
        set_error("local RBF system of size " + std::to_string(m) + " (k=" + std::to_string(prm->k) +
                  ") exceeds the GPU limit (" + std::to_string(kRbfMaxSystem) + ")");
        return PTV_E_UNSUPPORTED;
    }
    *m_out = m;
    return PTV_OK;
}

// Local RBF: per z chunk, a k-NN pass in slot mode, then the per-voxel solve.
int run_rbf(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_rbf_params *prm, int m,
            const double *ax, const double *ay, const double *az, const double *qx, const double *qy,
            const double *qz, const double *smooth, const uint8_t *mask, double *U, double *V, double *W,
            hipStream_t s, int64_t *n_singular) {
    // k >= 128: the large-k slot search (ptv_knn_big.hip; no lattice, its own cell occupancy)
    const bool big = kmax_for(prm->k) == 0;
    const SearchParams sp{PTV_METHOD_IDW, prm->k, 2.0, 1e-10, 0u, big ? std::max(1.0, prm->k / 256.0) : 0.0, 0.0,
                          big ? -1 : 0};
    KnnLaunch kl;
    Binned b{};
    PTV_TRY(prepare(c, p, g, &sp, ax, ay, az, qx, qy, qz, s, kl, b));
    const std::vector<int> pw = monomial_powers(prm->degree);
    PTV_TRY(c->rbf_pw.ensure(pw.size() + 1));
    PTV_TRY(c->rbf_status.ensure(6));
    PTV_TRY(c->rbf_nslist.ensure(kRbfNsCap));
    if (!pw.empty())
        PTV_HIP(hipMemcpyAsync(c->rbf_pw.p, pw.data(), pw.size() * sizeof(int), hipMemcpyHostToDevice, s));
    const int st_init[6] = {0, 0x7fffffff, 0, 0, 0, 0};

    const int64_t plane = g->nx * g->ny;
    const int64_t z0 = g->z_begin, z1 = g->z_end;
    int cp = prm->chunk_planes;
    if (cp <= 0) {
        // about 512 MB of slots per chunk
        const int64_t per_plane = plane * (int64_t)prm->k * 4;
        cp = (int)std::max<int64_t>(4, std::min<int64_t>(z1 - z0, ((int64_t)512 << 20) / std::max<int64_t>(per_plane, 1)));
    }
    cp = std::max(4, (cp + 3) & ~3);
    PTV_TRY(c->slots.ensure((size_t)std::min<int64_t>(cp, z1 - z0) * plane * prm->k));
    const int nchunks = (int)((z1 - z0 + cp - 1) / cp);
    while ((int)c->rbf_ev.size() < 3 * nchunks) {
        hipEvent_t e;
        PTV_HIP(hipEventCreate(&e));
        c->rbf_ev.push_back(e);
    }
    RbfKernelArgs ra{};
    ra.nx = (int)g->nx;
    ra.ny = (int)g->ny;
    ra.out_z0 = (int)z0;
    ra.separable = ax != nullptr ? 1 : 0;
    ra.k = prm->k;
    ra.m = m;
    ra.kernel = prm->kernel;
    ra.epsilon = prm->epsilon;
    ra.smoothing = prm->smoothing;
    ra.flags = prm->flags;
    if (m > kRbfMaxSystem) {
        // k_rbf_huge: persistent workgroups with a global-memory slice each (about 2 GB in total)
        const size_t slice = rbf_huge_slice_doubles(m, prm->k);
        const long long nb = std::max<long long>(64, std::min<long long>(4096, (2LL << 30) / (long long)(slice * 8)));
        PTV_TRY(c->rbf_huge.ensure((size_t)nb * slice));
        ra.huge_scratch = c->rbf_huge.p;
        ra.huge_blocks = (int)nb;
    }
    int st_out[6] = {0, 0, 0, 0, 0, 0};
    // per chunk: the voxels k_rbf_ns flagged (status[3] of its launch), whether they overflowed the
    // list (status[4]) and the running singular count (status[0]), copied on the device after each chunk
    PTV_TRY(c->rbf_cflag.ensure(3 * (size_t)nchunks));
    std::vector<int> cflag(3 * (size_t)nchunks, 0);
    std::vector<char> rerun((size_t)nchunks, 1);
    int64_t pivoted = 0;
    int64_t singular_redone = 0;  // pass 0's singular counts of the chunks an overflow rerun solves again
    for (int pass = 0; pass < 2; ++pass) {
    // pass 1 (rare): k_rbf_spd16 met a pivot its reciprocal does not serve (every chunk again with the
    // LDS-broadcast SPD kernel: the same arithmetic plus the IEEE division for such pivots), or
    // k_rbf_ns flagged more voxels in a chunk than its list holds (that chunk again, pivoting)
    ra.spd_lds = pass;
    ra.ns_list = pass == 0 ? c->rbf_nslist.p : nullptr;
    ra.ns_cap = kRbfNsCap;
    // (a full SPD rerun starts its counts afresh; an overflow rerun adds to pass 0's)
    if (pass == 0 || st_out[2] != 0)
        PTV_HIP(hipMemcpyAsync(c->rbf_status.p, st_init, sizeof(st_init), hipMemcpyHostToDevice, s));
    for (int ch = 0; ch < nchunks; ++ch) {
        if (!rerun[ch]) continue;
        const int za = (int)(z0 + (int64_t)ch * cp), zb = (int)std::min<int64_t>(z1, za + cp);
        KnnLaunch cl = kl;
        cl.z0 = za;
        cl.z1 = zb;
        cl.lz0 = (int)z0;
        cl.mode = kModeSlots;
        cl.slots = c->slots.p;
        PTV_HIP(hipEventRecord(c->rbf_ev[3 * ch], s));
        if (big) {
            BigQueries q;
            q.nx = (int)g->nx;
            q.ny = (int)g->ny;
            q.z0 = za;
            q.ax = ax;
            q.ay = ay;
            q.az = az;
            q.px = qx;
            q.py = qy;
            q.pz = qz;
            q.mask = mask;
            BigEpilogue ep;
            ep.slots = c->slots.p;
            PTV_TRY(run_big_knn(c->big, q, b, kl.cg, (int64_t)(zb - za) * plane, prm->k, ep, s));
        } else {
            PTV_TRY(launch_knn(cl, b, ax, ay, az, qx, qy, qz, mask, nullptr, nullptr, nullptr, s));
        }
        PTV_HIP(hipEventRecord(c->rbf_ev[3 * ch + 1], s));
        ra.z0 = za;
        ra.z1 = zb;
        PTV_TRY(launch_rbf(ra, b, c->slots.p, ax, ay, az, qx, qy, qz, smooth, c->rbf_pw.p, mask, U, V, W,
                           c->rbf_status.p, s));
        if (pass == 0) {
            PTV_HIP(hipMemcpyAsync(c->rbf_cflag.p + 3 * ch, c->rbf_status.p + 3, 2 * sizeof(int),
                                   hipMemcpyDeviceToDevice, s));
            PTV_HIP(hipMemcpyAsync(c->rbf_cflag.p + 3 * ch + 2, c->rbf_status.p, sizeof(int),
                                   hipMemcpyDeviceToDevice, s));
            PTV_HIP(hipMemsetAsync(c->rbf_status.p + 4, 0, sizeof(int), s));
        }
        PTV_HIP(hipEventRecord(c->rbf_ev[3 * ch + 2], s));
    }
    PTV_HIP(hipMemcpyAsync(st_out, c->rbf_status.p, sizeof(st_out), hipMemcpyDeviceToHost, s));
    if (pass == 0)
        PTV_HIP(hipMemcpyAsync(cflag.data(), c->rbf_cflag.p, cflag.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    PTV_HIP(hipStreamSynchronize(s));
    if (pass == 1) {
        st_out[0] -= (int)singular_redone;  // each rerun chunk's singular voxels, counted once
        break;
    }
    bool again = false;
    for (int ch = 0; ch < nchunks; ++ch) {
        const int za = (int)(z0 + (int64_t)ch * cp), zb = (int)std::min<int64_t>(z1, za + cp);
        const bool over = cflag[3 * ch + 1] != 0;
        // voxels the pivoting kernel solved: the flagged ones, or every voxel of an overflowed chunk
        pivoted += over ? (int64_t)(zb - za) * plane : cflag[3 * ch];
        rerun[ch] = (st_out[2] != 0 || over) ? 1 : 0;
        again = again || rerun[ch];
        if (over && st_out[2] == 0) singular_redone += cflag[3 * ch + 2] - (ch > 0 ? cflag[3 * ch - 1] : 0);
    }
    if (st_out[2] != 0) pivoted = 0;  // the SPD rerun: no null-space kernel ran
    if (!again) break;
    }
    c->rbf_chunks = nchunks;
    *n_singular = st_out[0];
    c->last.n_singular = st_out[0];
    c->last.n_rbf_pivoted = pivoted;
    if (st_out[0] > 0) {
        set_error("Singular matrix. (" + std::to_string(st_out[0]) + " voxel system(s), first at linear voxel " +
                  std::to_string(st_out[1]) + ")");
        return PTV_E_SINGULAR;
    }
    return PTV_OK;
}

// method='linear' on device pointers: binning + k = 1 slot search per z-chunk (the walk starts),
// the walk / interpolation kernel, then scipy's brute-force location for the flagged voxels.
constexpr int kLinearMaxWalk = 4096;
constexpr int kLinearFlagCap = 1 << 20;

int run_linear(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_linear_params *prm,
               const int32_t *simp, const int32_t *nbr, const double *tr, const int32_t *v2s, const double *ax,
               const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
               const uint8_t *mask, double *U, double *V, double *W, hipStream_t s) {
    const SearchParams sp{PTV_METHOD_NEAREST, 1, 2.0, 1e-10, 0u, 0.0, 0.0, 0};
    KnnLaunch kl;
    Binned b{};
    PTV_TRY(prepare(c, p, g, &sp, ax, ay, az, qx, qy, qz, s, kl, b));
    const int64_t plane = g->nx * g->ny;
    const int64_t z0 = g->z_begin, z1 = g->z_end;
    int cp = prm->chunk_planes;
    if (cp <= 0) cp = (int)std::max<int64_t>(4, std::min<int64_t>(z1 - z0, ((int64_t)512 << 20) / std::max<int64_t>(plane * 4, 1)));
    cp = std::max(4, (cp + 3) & ~3);
    PTV_TRY(c->slots.ensure((size_t)std::min<int64_t>(cp, z1 - z0) * plane));
    PTV_TRY(c->lin_count.ensure(1));
    PTV_TRY(c->lin_flags.ensure(kLinearFlagCap));
    PTV_HIP(hipMemsetAsync(c->lin_count.p, 0, sizeof(int), s));
    const int nchunks = (int)((z1 - z0 + cp - 1) / cp);
    while ((int)c->rbf_ev.size() < 3 * nchunks) {
        hipEvent_t e;
        PTV_HIP(hipEventCreate(&e));
        c->rbf_ev.push_back(e);
    }
    LinearKernelArgs la{};
    la.nx = (int)g->nx;
    la.ny = (int)g->ny;
    la.out_z0 = (int)z0;
    la.separable = ax != nullptr ? 1 : 0;
    la.nsimplex = prm->nsimplex;
    la.simplices = simp;
    la.neighbors = nbr;
    la.transform = tr;
    la.v2s = v2s;
    la.pu = p->u;
    la.pv = p->v;
    la.pw = p->w;
    for (int d = 0; d < 3; ++d) {
        la.lo[d] = prm->min_bound[d];
        la.hi[d] = prm->max_bound[d];
    }
    la.fill = prm->fill_value;
    la.flags = prm->flags;
    la.max_walk = kLinearMaxWalk;
    la.flag_count = c->lin_count.p;
    la.flag_list = c->lin_flags.p;
    la.flag_cap = kLinearFlagCap;
    for (int ch = 0; ch < nchunks; ++ch) {
        const int za = (int)(z0 + (int64_t)ch * cp), zb = (int)std::min<int64_t>(z1, za + cp);
        KnnLaunch cl = kl;
        cl.z0 = za;
        cl.z1 = zb;
        cl.lz0 = (int)z0;
        cl.mode = kModeSlots;
        cl.slots = c->slots.p;
        PTV_HIP(hipEventRecord(c->rbf_ev[3 * ch], s));
        PTV_TRY(launch_knn(cl, b, ax, ay, az, qx, qy, qz, mask, nullptr, nullptr, nullptr, s));
        PTV_HIP(hipEventRecord(c->rbf_ev[3 * ch + 1], s));
        la.z0 = za;
        la.z1 = zb;
        PTV_TRY(launch_linear(la, b.prec, c->slots.p, ax, ay, az, qx, qy, qz, mask, U, V, W, s));
        PTV_HIP(hipEventRecord(c->rbf_ev[3 * ch + 2], s));
    }
    c->rbf_chunks = nchunks;
    int nflag = 0;
    PTV_HIP(hipMemcpyAsync(&nflag, c->lin_count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    PTV_HIP(hipStreamSynchronize(s));
    if (nflag > kLinearFlagCap) {
        set_error("linear: " + std::to_string(nflag) + " voxels need the brute-force point location (limit " +
                  std::to_string(kLinearFlagCap) + "): degenerate triangulation");
        return PTV_E_UNSUPPORTED;
    }
    c->last.n_singular = nflag;  // reported: voxels located by the brute-force scan
    if (nflag > 0) {
        la.z0 = (int)z0;
        la.z1 = (int)z1;
        PTV_TRY(launch_linear_brute(la, nflag, ax, ay, az, qx, qy, qz, U, V, W, s));
    }
    return PTV_OK;
}

int finish_timing(ptv_ctx *c) {
    float ms = 0.f;
    if (c->div_pending) {
        PTV_HIP(hipEventSynchronize(c->ev_div1));
        PTV_HIP(hipEventElapsedTime(&ms, c->ev_div0, c->ev_div1));
        c->last.ms_stencil = ms;
        c->div_pending = false;
    }
    if (!c->timed_pending) return PTV_OK;
    if (c->rbf_chunks > 0) {
        PTV_HIP(hipEventSynchronize(c->rbf_ev[3 * c->rbf_chunks - 1]));
        double knn = 0.0, solve = 0.0;
        for (int ch = 0; ch < c->rbf_chunks; ++ch) {
            PTV_HIP(hipEventElapsedTime(&ms, c->rbf_ev[3 * ch], c->rbf_ev[3 * ch + 1]));
            knn += ms;
            PTV_HIP(hipEventElapsedTime(&ms, c->rbf_ev[3 * ch + 1], c->rbf_ev[3 * ch + 2]));
            solve += ms;
        }
        c->last.ms_knn = knn;
        c->last.ms_solve = solve;
    } else {
        PTV_HIP(hipEventSynchronize(c->ev_knn1));
        PTV_HIP(hipEventElapsedTime(&ms, c->ev_main0, c->ev_knn1));
        c->last.ms_knn = ms;
    }
    if (c->cull_timed) {
        float a = 0.f, b = 0.f;
        PTV_HIP(hipEventElapsedTime(&a, c->ev_cull0, c->ev_cull1));
        PTV_HIP(hipEventElapsedTime(&b, c->ev_lat1, c->ev_main0));
        c->last.ms_cull = (double)a + (double)b;
    }
    PTV_HIP(hipEventElapsedTime(&ms, c->ev_knn0, c->ev_lat1));
    c->last.ms_lattice = ms;
    PTV_HIP(hipEventElapsedTime(&ms, c->ev_bin0, c->ev_bin1));
    c->last.ms_bin = ms;
    c->timed_pending = false;
    return PTV_OK;
}

struct EventSet {
    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
    ~EventSet() {
        for (hipEvent_t x : e)
            if (x) hipEventDestroy(x);
    }
};

// First-touch of the caller's output pages on host threads while the device works.  A fresh
// (never written) host buffer pays a page fault per 4 KiB page inside the D2H copy: measured
// on the MI355X box, 1 GiB into fresh pageable memory 65-72 ms against 19 ms (52 GiB/s) into
// touched memory, and pinning (hipHostMalloc / hipHostRegister) costs the same ~45 ms/GiB.  The
// faults are taken in parallel here (a write per page; the D2H then overwrites every byte), so
// only the copy remains on the critical path.  Joined before the D2H is enqueued, and on every
// early return.
constexpr int kMadvPopulateWrite = 23;  // MADV_POPULATE_WRITE (Linux 5.14), absent from older headers

struct PageToucher {
    std::vector<std::thread> th;
    void start(void *const *bufs, int nbuf, size_t bytes) {
        constexpr size_t kPage = 4096, kMin = (size_t)32 << 20;
        if (bytes < kMin) return;
        const unsigned hw = std::thread::hardware_concurrency();
        const int nt = (int)std::max(1u, std::min(16u, hw ? hw : 1u));
        const size_t pages = (bytes + kPage - 1) / kPage;
        for (int t = 0; t < nt; ++t) {
            const size_t p0 = pages * t / nt, p1 = pages * (t + 1) / nt;
            std::vector<char *> b(nbuf);
            for (int i = 0; i < nbuf; ++i) b[i] = static_cast<char *>(bufs[i]);
            th.emplace_back([b, p0, p1, bytes]() {
                // fault the pages in writable WITHOUT changing them (a failed call must leave the
                // caller's arrays as they were): MADV_POPULATE_WRITE where the kernel has it, else a
                // volatile read-modify-write of one byte per page
                for (char *base : b) {
                    const uintptr_t lo = (reinterpret_cast<uintptr_t>(base) + p0 * kPage) & ~(uintptr_t)(kPage - 1);
                    const uintptr_t hi = reinterpret_cast<uintptr_t>(base) + std::min(p1 * kPage, bytes);
                    if (hi > lo && madvise(reinterpret_cast<void *>(lo), hi - lo, kMadvPopulateWrite) == 0) continue;
                    for (size_t pg = p0; pg < p1; ++pg) {
                        volatile char *q = base + std::min(pg * kPage, bytes - 1);
                        *q = *q;
                    }
                }
            });
        }
    }
    void join() {
        for (auto &t : th) t.join();
        th.clear();
    }
    ~PageToucher() { join(); }
};

// Host-buffer call: H2D into the context's buffers, `compute` on device pointers, D2H of
// the slab's three output planes, timings.  compute(dp, dg, dmask, dsmooth, U, V, W, s).
template <typename F>
int host_call(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const uint8_t *mask_h, const double *smooth_h,
              double *U, double *V, double *W, F &&compute, size_t out_elem = sizeof(double)) {
    hipStream_t s = c->stream;
    EventSet ev;
    for (hipEvent_t &e : ev.e) PTV_HIP(hipEventCreate(&e));
    const int64_t n = p->n;
    const int64_t plane = g->nx * g->ny;
    const int64_t nvox = (g->z_end - g->z_begin) * plane;
    const int64_t nfull = g->nz * plane;
    PageToucher touch;
    {
        void *outs[3] = {U, V, W};
        touch.start(outs, 3, (size_t)nvox * out_elem);
    }
    PTV_HIP(hipEventRecord(ev.e[0], s));
    const double *src[6] = {p->x, p->y, p->z, p->u, p->v, p->w};
    for (int i = 0; i < 6; ++i) {
        PTV_TRY(c->pin[i].ensure(n));
        PTV_HIP(hipMemcpyAsync(c->pin[i].p, src[i], n * sizeof(double), hipMemcpyHostToDevice, s));
    }
    ptv_particles dp{n, c->pin[0].p, c->pin[1].p, c->pin[2].p, c->pin[3].p, c->pin[4].p, c->pin[5].p};
    ptv_grid dg = *g;
    const bool sep = g->ax && g->ay && g->az;
    if (sep) {
        PTV_TRY(c->axes.ensure(g->nx + g->ny + g->nz));
        PTV_HIP(hipMemcpyAsync(c->axes.p, g->ax, g->nx * sizeof(double), hipMemcpyHostToDevice, s));
        PTV_HIP(hipMemcpyAsync(c->axes.p + g->nx, g->ay, g->ny * sizeof(double), hipMemcpyHostToDevice, s));
        PTV_HIP(hipMemcpyAsync(c->axes.p + g->nx + g->ny, g->az, g->nz * sizeof(double), hipMemcpyHostToDevice, s));
        dg.ax = c->axes.p;
        dg.ay = c->axes.p + g->nx;
        dg.az = c->axes.p + g->nx + g->ny;
        dg.px = dg.py = dg.pz = nullptr;
    } else {
        const double *q[3] = {g->px, g->py, g->pz};
        for (int i = 0; i < 3; ++i) {
            PTV_TRY(c->qpts[i].ensure(nfull));
            PTV_HIP(hipMemcpyAsync(c->qpts[i].p, q[i], nfull * sizeof(double), hipMemcpyHostToDevice, s));
        }
        dg.ax = dg.ay = dg.az = nullptr;
        dg.px = c->qpts[0].p;
        dg.py = c->qpts[1].p;
        dg.pz = c->qpts[2].p;
    }
    const uint8_t *dmask = nullptr;
    if (mask_h) {
        PTV_TRY(c->mask.ensure(nfull));
        PTV_HIP(hipMemcpyAsync(c->mask.p, mask_h, nfull, hipMemcpyHostToDevice, s));
        dmask = c->mask.p;
    }
    const double *dsmooth = nullptr;
    if (smooth_h) {
        PTV_TRY(c->smooth.ensure(n));
        PTV_HIP(hipMemcpyAsync(c->smooth.p, smooth_h, n * sizeof(double), hipMemcpyHostToDevice, s));
        dsmooth = c->smooth.p;
    }
    for (int i = 0; i < 3; ++i) PTV_TRY(c->out[i].ensure(nvox));
    PTV_HIP(hipEventRecord(ev.e[1], s));
    PTV_TRY(compute(&dp, &dg, dmask, dsmooth, c->out[0].p, c->out[1].p, c->out[2].p, s));
    PTV_HIP(hipEventRecord(ev.e[2], s));
    touch.join();
    double *dst[3] = {U, V, W};
    for (int i = 0; i < 3; ++i)
        PTV_HIP(hipMemcpyAsync(dst[i], c->out[i].p, nvox * out_elem, hipMemcpyDeviceToHost, s));
    PTV_HIP(hipEventRecord(ev.e[3], s));
    PTV_HIP(hipStreamSynchronize(s));
    PTV_TRY(finish_timing(c));
    float h2d = 0.f, d2h = 0.f, tot = 0.f;
    PTV_HIP(hipEventElapsedTime(&h2d, ev.e[0], ev.e[1]));
    PTV_HIP(hipEventElapsedTime(&d2h, ev.e[2], ev.e[3]));
    PTV_HIP(hipEventElapsedTime(&tot, ev.e[0], ev.e[3]));
    c->last.ms_h2d = h2d;
    c->last.ms_d2h = d2h;
    c->last.ms_total = tot;
    return PTV_OK;
}

int check_call(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const void *prm, double *U, double *V,
               double *W) {
    if (!c) {
        set_error("NULL context");
        return PTV_E_ARG;
    }
    PTV_TRY(validate(p, g, prm));
    if (!U || !V || !W) {
        set_error("NULL output");
        return PTV_E_ARG;
    }
    PTV_HIP(hipSetDevice(c->device));
    return PTV_OK;
}

// ptv_div_params -> DivArgs, with the same checks for the host and device calls.
int div_args(ptv_ctx *c, const ptv_div_params *prm, const void *U, const void *V, const void *W, const void *out,
             DivArgs &a) {
    if (!c || !prm) {
        set_error("NULL context/params");
        return PTV_E_ARG;
    }
    if (!U || !V || !W || !out || !prm->fluid_mask) {
        set_error("divergence: NULL field, output or fluid mask");
        return PTV_E_ARG;
    }
    if (prm->nx <= 0 || prm->ny <= 0 || prm->nz <= 0 || prm->nx > (1 << 30) || prm->ny > (1 << 30) ||
        prm->nz > (1 << 30)) {
        set_error("divergence: dimensions must be positive");
        return PTV_E_ARG;
    }
    const int64_t lo = prm->edge_lo ? 0 : 1, hi = prm->nz - (prm->edge_hi ? 0 : 1);
    if (prm->z_begin < lo || prm->z_end > hi || prm->z_begin > prm->z_end) {
        set_error("divergence: planes [" + std::to_string(prm->z_begin) + ", " + std::to_string(prm->z_end) +
                  ") must lie in [" + std::to_string(lo) + ", " + std::to_string(hi) +
                  ") (a non-edge buffer end is a halo plane)");
        return PTV_E_ARG;
    }
    if ((prm->field_dtype != PTV_F64 && prm->field_dtype != PTV_F32) ||
        (prm->result_dtype != PTV_F64 && prm->result_dtype != PTV_F32)) {
        set_error("divergence: dtype must be PTV_F64 or PTV_F32");
        return PTV_E_ARG;
    }
    a.nx = (int)prm->nx;
    a.ny = (int)prm->ny;
    a.nz = (int)prm->nz;
    a.z_begin = (int)prm->z_begin;
    a.z_end = (int)prm->z_end;
    a.edge_lo = prm->edge_lo ? 1 : 0;
    a.edge_hi = prm->edge_hi ? 1 : 0;
    a.field_f32 = prm->field_dtype == PTV_F32;
    a.result_f32 = prm->result_dtype == PTV_F32;
    a.dx = prm->dx;
    a.dy = prm->dy;
    a.dz = prm->dz;
    if (!a.field_f32 && a.result_f32) {
        set_error("divergence: float64 fields cannot give float32 results (numpy promotion)");
        return PTV_E_ARG;
    }
    PTV_HIP(hipSetDevice(c->device));
    return PTV_OK;
}

int run_div(ptv_ctx *c, const DivArgs &a, const void *U, const void *V, const void *W, const uint8_t *M, void *out,
            hipStream_t s) {
    PTV_HIP(hipEventRecord(c->ev_div0, s));
    PTV_TRY(launch_divergence(a, U, V, W, M, out, s));
    PTV_HIP(hipEventRecord(c->ev_div1, s));
    c->div_pending = true;
    return PTV_OK;
}

}  // namespace

extern "C" {

int ptv_interp_knn_dev(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_knn_params *prm, double *U,
                       double *V, double *W, void *stream, ptv_stats *st) {
    PTV_TRY(check_call(c, p, g, prm, U, V, W));
    PTV_TRY(validate_knn(p, prm));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const bool sep = g->ax && g->ay && g->az;
    return run_knn(c, p, g, prm, sep ? g->ax : nullptr, sep ? g->ay : nullptr, sep ? g->az : nullptr,
                   sep ? nullptr : g->px, sep ? nullptr : g->py, sep ? nullptr : g->pz, prm->fluid_mask, U, V, W, s,
                   st);
}

int ptv_interp_knn(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_knn_params *prm, double *U,
                   double *V, double *W, ptv_stats *st) {
    PTV_TRY(check_call(c, p, g, prm, U, V, W));
    PTV_TRY(validate_knn(p, prm));
    PTV_TRY(host_call(c, p, g, prm->fluid_mask, nullptr, U, V, W,
                      [&](const ptv_particles *dp, const ptv_grid *dg, const uint8_t *dmask, const double *,
                          double *dU, double *dV, double *dW, hipStream_t s) {
                          // st: on PTV_E_INEXACT the caller gets halo_required (host_call returns early)
                          return run_knn(c, dp, dg, prm, dg->ax, dg->ay, dg->az, dg->px, dg->py, dg->pz, dmask, dU,
                                         dV, dW, s, st);
                      },
                      (prm->flags & PTV_FLAG_OUT_F32) ? sizeof(float) : sizeof(double)));
    if (st) *st = c->last;
    return PTV_OK;
}

int ptv_interp_rbf_local_dev(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_rbf_params *prm,
                             double *U, double *V, double *W, void *stream, ptv_stats *st) {
    PTV_TRY(check_call(c, p, g, prm, U, V, W));
    int m = 0;
    PTV_TRY(validate_rbf(p, prm, &m));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const bool sep = g->ax && g->ay && g->az;
    int64_t nsing = 0;
    const int rc = run_rbf(c, p, g, prm, m, sep ? g->ax : nullptr, sep ? g->ay : nullptr, sep ? g->az : nullptr,
                           sep ? nullptr : g->px, sep ? nullptr : g->py, sep ? nullptr : g->pz,
                           prm->smoothing_per_point, prm->fluid_mask, U, V, W, s, &nsing);
    c->timed_pending = true;
    if (st) *st = c->last;
    return rc;
}

int ptv_interp_rbf_local(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_rbf_params *prm,
                         double *U, double *V, double *W, ptv_stats *st) {
    PTV_TRY(check_call(c, p, g, prm, U, V, W));
    int m = 0;
    PTV_TRY(validate_rbf(p, prm, &m));
    PTV_TRY(host_call(c, p, g, prm->fluid_mask, prm->smoothing_per_point, U, V, W,
                      [&](const ptv_particles *dp, const ptv_grid *dg, const uint8_t *dmask, const double *dsmooth,
                          double *dU, double *dV, double *dW, hipStream_t s) {
                          int64_t nsing = 0;
                          const int rc = run_rbf(c, dp, dg, prm, m, dg->ax, dg->ay, dg->az, dg->px, dg->py, dg->pz,
                                                 dsmooth, dmask, dU, dV, dW, s, &nsing);
                          c->timed_pending = true;
                          return rc;
                      }));
    if (st) *st = c->last;
    return PTV_OK;
}

static int validate_linear(const ptv_particles *p, const ptv_linear_params *prm) {
    if (!prm || !prm->simplices || !prm->neighbors || !prm->transform || !prm->vertex_to_simplex) {
        set_error("linear: NULL parameters or triangulation array");
        return PTV_E_ARG;
    }
    if (prm->nsimplex < 1 || prm->nsimplex > 0x7fffffffLL) {
        set_error("linear: nsimplex must be in [1, 2^31)");
        return PTV_E_ARG;
    }
    if (p->n > 0x7fffffffLL) {
        set_error("linear: more than 2^31 particles");
        return PTV_E_ARG;
    }
    if (prm->flags & ~PTV_FLAG_NAN_TO_NUM) {
        set_error("linear: only PTV_FLAG_NAN_TO_NUM is supported");
        return PTV_E_UNSUPPORTED;
    }
    return PTV_OK;
}

int ptv_interp_linear_dev(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_linear_params *prm,
                          double *U, double *V, double *W, void *stream, ptv_stats *st) {
    PTV_TRY(check_call(c, p, g, prm, U, V, W));
    PTV_TRY(validate_linear(p, prm));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const bool sep = g->ax && g->ay && g->az;
    const int rc = run_linear(c, p, g, prm, prm->simplices, prm->neighbors, prm->transform, prm->vertex_to_simplex,
                              sep ? g->ax : nullptr, sep ? g->ay : nullptr, sep ? g->az : nullptr,
                              sep ? nullptr : g->px, sep ? nullptr : g->py, sep ? nullptr : g->pz, prm->fluid_mask, U,
                              V, W, s);
    c->timed_pending = true;
    if (st) *st = c->last;
    return rc;
}

int ptv_interp_linear(ptv_ctx *c, const ptv_particles *p, const ptv_grid *g, const ptv_linear_params *prm,
                      double *U, double *V, double *W, ptv_stats *st) {
    PTV_TRY(check_call(c, p, g, prm, U, V, W));
    PTV_TRY(validate_linear(p, prm));
    PTV_TRY(host_call(c, p, g, prm->fluid_mask, nullptr, U, V, W,
                      [&](const ptv_particles *dp, const ptv_grid *dg, const uint8_t *dmask, const double *,
                          double *dU, double *dV, double *dW, hipStream_t s) {
                          const size_t ns = (size_t)prm->nsimplex, n = (size_t)p->n;
                          PTV_TRY(c->lin_simp.ensure(4 * ns));
                          PTV_TRY(c->lin_nbr.ensure(4 * ns));
                          PTV_TRY(c->lin_tr.ensure(12 * ns));
                          PTV_TRY(c->lin_v2s.ensure(n));
                          PTV_HIP(hipMemcpyAsync(c->lin_simp.p, prm->simplices, 4 * ns * sizeof(int), hipMemcpyHostToDevice, s));
                          PTV_HIP(hipMemcpyAsync(c->lin_nbr.p, prm->neighbors, 4 * ns * sizeof(int), hipMemcpyHostToDevice, s));
                          PTV_HIP(hipMemcpyAsync(c->lin_tr.p, prm->transform, 12 * ns * sizeof(double), hipMemcpyHostToDevice, s));
                          PTV_HIP(hipMemcpyAsync(c->lin_v2s.p, prm->vertex_to_simplex, n * sizeof(int), hipMemcpyHostToDevice, s));
                          const int rc = run_linear(c, dp, dg, prm, c->lin_simp.p, c->lin_nbr.p, c->lin_tr.p, c->lin_v2s.p,
                                                    dg->ax, dg->ay, dg->az, dg->px, dg->py, dg->pz, dmask, dU, dV, dW, s);
                          c->timed_pending = true;
                          return rc;
                      }));
    if (st) *st = c->last;
    return PTV_OK;
}

int ptv_debug_stamps(ptv_ctx *c, int mode, double *out) {
    if (!c) {
        set_error("NULL context");
        return PTV_E_ARG;
    }
    PTV_HIP(hipSetDevice(c->device));
    constexpr long long cap = 1LL << 21;  // waves recorded (modulo-free: later waves dropped)
    constexpr int nf = 8;
    if (mode == 1) {  // enable + zero
        PTV_TRY(c->dbg.ensure((size_t)cap * nf));
        PTV_HIP(hipMemsetAsync(c->dbg.p, 0, (size_t)cap * nf * sizeof(unsigned long long), c->stream));
        PTV_HIP(hipStreamSynchronize(c->stream));
        ptv::g_dbg = c->dbg.p;
        ptv::g_dbg_cap = cap;
    } else if (mode == 0) {
        ptv::g_dbg = nullptr;
        ptv::g_dbg_cap = 0;
    }
    if (out && c->dbg.p) {
        PTV_HIP(hipDeviceSynchronize());
        std::vector<unsigned long long> h((size_t)cap * nf);
        PTV_HIP(hipMemcpy(h.data(), c->dbg.p, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (const char *dump = dev_knob("PTV_STAMPS_DUMP")) {  // raw per-wave records (dev tool)
            if (FILE *f = std::fopen(dump, "wb")) {
                std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
                std::fclose(f);
            }
        }
        // out: [records, mean of 11 fields, max of 11 fields]: 6 phase cycle counts, then
        // gathered candidates, merge iterations, rounds, passes, candidates kept by the
        // sub-ball filter (packed two or three to a u64 in fields 6 and 7)
        constexpr int nv = 11;
        double sum[nv] = {0}, mx[nv] = {0};
        long long nrec = 0;
        for (long long w = 0; w < cap; ++w) {
            const unsigned long long *r = &h[(size_t)w * nf];
            if (r[0] == 0 && r[2] == 0 && r[5] == 0) continue;
            ++nrec;
            double v[nv];
            for (int f = 0; f < 6; ++f) v[f] = (double)r[f];
            v[6] = (double)(r[6] & 0xffffffffULL);
            v[7] = (double)(r[6] >> 32);
            v[8] = (double)(r[7] & 0xffffULL);
            v[9] = (double)((r[7] >> 16) & 0xffffULL);
            v[10] = (double)(r[7] >> 32);
            for (int f = 0; f < nv; ++f) {
                sum[f] += v[f];
                mx[f] = std::max(mx[f], v[f]);
            }
        }
        out[0] = (double)nrec;
        for (int f = 0; f < nv; ++f) {
            out[1 + f] = nrec ? sum[f] / (double)nrec : 0.0;
            out[1 + nv + f] = mx[f];
        }
    }
    return PTV_OK;
}

int ptv_divergence_dev(ptv_ctx *c, const ptv_div_params *prm, const void *U, const void *V, const void *W,
                       void *out, void *stream, ptv_stats *st) {
    DivArgs a{};
    PTV_TRY(div_args(c, prm, U, V, W, out, a));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    PTV_TRY(run_div(c, a, U, V, W, prm->fluid_mask, out, s));
    c->last.n_voxels = (prm->z_end - prm->z_begin) * prm->nx * prm->ny;
    if (st) *st = c->last;
    return PTV_OK;
}

int ptv_divergence(ptv_ctx *c, const ptv_div_params *prm, const void *U, const void *V, const void *W, void *out,
                   ptv_stats *st) {
    DivArgs a{};
    PTV_TRY(div_args(c, prm, U, V, W, out, a));
    hipStream_t s = c->stream;
    EventSet ev;
    for (hipEvent_t &e : ev.e) PTV_HIP(hipEventCreate(&e));
    const size_t ts = a.field_f32 ? 4 : 8, rs = a.result_f32 ? 4 : 8;
    const int64_t nfull = prm->nz * prm->nx * prm->ny;
    const int64_t nout = (prm->z_end - prm->z_begin) * prm->nx * prm->ny;
    PTV_HIP(hipEventRecord(ev.e[0], s));
    const void *src[3] = {U, V, W};
    for (int i = 0; i < 3; ++i) {
        PTV_TRY(c->fld[i].ensure(nfull * ts));
        PTV_HIP(hipMemcpyAsync(c->fld[i].p, src[i], nfull * ts, hipMemcpyHostToDevice, s));
    }
    PTV_TRY(c->mask.ensure(nfull));
    PTV_HIP(hipMemcpyAsync(c->mask.p, prm->fluid_mask, nfull, hipMemcpyHostToDevice, s));
    PTV_TRY(c->fld[3].ensure(nout * rs));
    PTV_HIP(hipEventRecord(ev.e[1], s));
    PTV_TRY(run_div(c, a, c->fld[0].p, c->fld[1].p, c->fld[2].p, c->mask.p, c->fld[3].p, s));
    PTV_HIP(hipEventRecord(ev.e[2], s));
    PTV_HIP(hipMemcpyAsync(out, c->fld[3].p, nout * rs, hipMemcpyDeviceToHost, s));
    PTV_HIP(hipEventRecord(ev.e[3], s));
    PTV_HIP(hipStreamSynchronize(s));
    PTV_TRY(finish_timing(c));
    float h2d = 0.f, d2h = 0.f, tot = 0.f;
    PTV_HIP(hipEventElapsedTime(&h2d, ev.e[0], ev.e[1]));
    PTV_HIP(hipEventElapsedTime(&d2h, ev.e[2], ev.e[3]));
    PTV_HIP(hipEventElapsedTime(&tot, ev.e[0], ev.e[3]));
    c->last.ms_h2d = h2d;
    c->last.ms_d2h = d2h;
    c->last.ms_total = tot;
    c->last.n_voxels = nout;
    if (st) *st = c->last;
    return PTV_OK;
}

int ptv_last_stats(ptv_ctx *c, ptv_stats *st) {
    if (!c || !st) {
        set_error("NULL argument");
        return PTV_E_ARG;
    }
    PTV_HIP(hipSetDevice(c->device));
    PTV_TRY(finish_timing(c));
    *st = c->last;
    return PTV_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// pore-mask path and outlier filter
// ---------------------------------------------------------------------------
namespace {

// raw axes -> device (ascending; a descending axis is reversed and flagged, as scipy's
// RegularGridInterpolator flips descending grids, _rgi.py _check_dimensionality/flip)
int mask_source(ptv_ctx *c, const ptv_mask_grid *src, MaskSampleLaunch &m, hipStream_t s) {
    if (!src || !src->raw || !src->ax || !src->ay || !src->az) {
        set_error("sample_mask: NULL raw mask or axis");
        return PTV_E_ARG;
    }
    const int64_t rn[3] = {src->nx, src->ny, src->nz};
    for (int d = 0; d < 3; ++d)
        if (rn[d] <= 0 || rn[d] > (1 << 30)) {
            set_error("sample_mask: raw mask extents must be positive");
            return PTV_E_ARG;
        }
    std::vector<double> h;
    h.reserve(rn[0] + rn[1] + rn[2]);
    const double *ax[3] = {src->ax, src->ay, src->az};
    size_t off[3];
    for (int d = 0; d < 3; ++d) {
        const double *a = ax[d];
        const int64_t n = rn[d];
        const bool desc = n > 1 && a[0] > a[n - 1];
        off[d] = h.size();
        for (int64_t i = 0; i < n; ++i) h.push_back(desc ? a[n - 1 - i] : a[i]);
        for (int64_t i = 1; i < n; ++i)
            if (!(h[off[d] + i] > h[off[d] + i - 1])) {
                set_error("The points in dimension " + std::to_string(2 - d) +
                          " must be strictly ascending or descending");
                return PTV_E_ARG;
            }
        m.rn[d] = (int)n;
        m.flip[d] = desc ? 1 : 0;
    }
    PTV_TRY(c->mask_axes.ensure(h.size()));
    PTV_HIP(hipMemcpyAsync(c->mask_axes.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s));
    for (int d = 0; d < 3; ++d) m.ra[d] = c->mask_axes.p + off[d];
    // the host vector must outlive the async copy
    PTV_HIP(hipStreamSynchronize(s));
    return PTV_OK;
}

int mask_grid_check(const ptv_grid *g, uint8_t *out) {
    if (!g || !out) {
        set_error("sample_mask: NULL grid or output");
        return PTV_E_ARG;
    }
    if (g->nx <= 0 || g->ny <= 0 || g->nz <= 0 || g->nx > (1 << 30) || g->ny > (1 << 30) || g->nz > (1 << 30)) {
        set_error("grid: dimensions must be positive");
        return PTV_E_ARG;
    }
    const bool sep = g->ax && g->ay && g->az, pts = g->px && g->py && g->pz;
    if (!sep && !pts) {
        set_error("grid: give either the three axes or the three point arrays");
        return PTV_E_ARG;
    }
    if (g->z_begin < 0 || g->z_end > g->nz || g->z_begin > g->z_end) {
        set_error("grid: bad z slab");
        return PTV_E_ARG;
    }
    return PTV_OK;
}

int run_mask_sample(ptv_ctx *c, MaskSampleLaunch &m, const ptv_grid *g, const uint8_t *raw, uint8_t *out,
                    hipStream_t s) {
    const bool sep = g->ax && g->ay && g->az;
    m.raw = raw;
    m.nx = (int)g->nx;
    m.ny = (int)g->ny;
    m.nz = (int)g->nz;
    m.z0 = (int)g->z_begin;
    m.z1 = (int)g->z_end;
    PTV_TRY(c->mask_tabs.ensure(g->nx + g->ny + g->nz));
    return launch_mask_sample(m, sep ? g->ax : nullptr, sep ? g->ay : nullptr, sep ? g->az : nullptr,
                              sep ? nullptr : g->px, sep ? nullptr : g->py, sep ? nullptr : g->pz, c->mask_tabs.p,
                              out, s);
}

int boundary_check(ptv_ctx *c, const ptv_boundary_params *prm, int64_t *count, BoundaryLaunch &m) {
    if (!c || !prm || !prm->mask || !count) {
        set_error("boundary: NULL context, params, mask or count");
        return PTV_E_ARG;
    }
    if (prm->nx <= 0 || prm->ny <= 0 || prm->nz <= 0 || prm->nx > (1 << 30) || prm->ny > (1 << 30) ||
        prm->nz > (1 << 30)) {
        set_error("boundary: dimensions must be positive");
        return PTV_E_ARG;
    }
    if (prm->thickness < 1 || prm->sampling_step < 1 ||
        (prm->encoding != PTV_MASK_BOOL && prm->encoding != PTV_MASK_BITS)) {
        set_error("boundary: need thickness >= 1, sampling_step >= 1 and a known encoding");
        return PTV_E_ARG;
    }
    m.nx = (int)prm->nx;
    m.ny = (int)prm->ny;
    m.nz = (int)prm->nz;
    m.mask = prm->mask;
    m.is_bool = prm->encoding == PTV_MASK_BOOL;
    m.thickness = prm->thickness;
    m.step = prm->sampling_step;
    for (int d = 0; d < 3; ++d) {
        m.lo[d] = prm->lo[d];
        m.span[d] = prm->span[d];
        m.den[d] = prm->den[d];
    }
    PTV_HIP(hipSetDevice(c->device));
    return PTV_OK;
}

// count pass (dilations + block counts + scan), then the emit pass into x, y, z if they fit
int run_boundary(ptv_ctx *c, const BoundaryLaunch &m, double *x, double *y, double *z, int64_t cap, int64_t *count,
                 hipStream_t s) {
    const int64_t nvox = (int64_t)m.nx * m.ny * m.nz;
    const size_t nb = boundary_blocks(nvox);
    PTV_TRY(c->bnd_counts.ensure(nb + 1));
    if (m.thickness > 1) {
        PTV_TRY(c->bnd_ping.ensure(nvox));
        if (m.thickness > 2) PTV_TRY(c->bnd_pong.ensure(nvox));
    }
    const uint8_t *grown = nullptr;
    PTV_HIP(hipEventRecord(c->ev_div0, s));
    PTV_TRY(launch_boundary_count(m, c->bnd_ping.p, c->bnd_pong.p, c->bnd_counts.p, &grown, s));
    unsigned long long total = 0;
    PTV_HIP(hipMemcpyAsync(&total, c->bnd_counts.p + nb, sizeof(total), hipMemcpyDeviceToHost, s));
    PTV_HIP(hipStreamSynchronize(s));
    const int64_t nsel = (int64_t)((total + (unsigned long long)m.step - 1) / (unsigned long long)m.step);
    *count = nsel;
    if (x && y && z && cap >= nsel && nsel > 0)
        PTV_TRY(launch_boundary_emit(m, grown, c->bnd_counts.p, x, y, z, s));
    PTV_HIP(hipEventRecord(c->ev_div1, s));
    c->div_pending = true;
    return PTV_OK;
}

int filter_check(ptv_ctx *c, const ptv_particles *p, const ptv_filter_params *prm, uint8_t *keep) {
    if (!c || !p || !prm || !keep) {
        set_error("filter: NULL context, particles, params or keep");
        return PTV_E_ARG;
    }
    if (p->n <= 0 || !p->x || !p->y || !p->z || !p->u || !p->v || !p->w) {
        set_error("particles: need n > 0 and six non-NULL arrays");
        return PTV_E_ARG;
    }
    if (p->n >= (int64_t)1 << 31) {
        set_error("particles: n must be < 2^31");
        return PTV_E_ARG;
    }
    if (prm->k < 1) {
        set_error("filter: k must be >= 1");
        return PTV_E_ARG;
    }
    if (p->n <= prm->k) {
        set_error("filter: need more particles than k (the reference skips the filter)");
        return PTV_E_ARG;
    }
    PTV_HIP(hipSetDevice(c->device));
    return PTV_OK;
}

// (k+1)-NN of every particle among the particles (slot mode, binned query order), then
// the per-particle median / MAD statistics
int run_filter(ptv_ctx *c, const ptv_particles *p, const ptv_filter_params *prm, uint8_t *keep, double *kth,
               hipStream_t s) {
    const int64_t n = p->n;
    const int64_t npad = (n + 255) & ~(int64_t)255;  // 64 queries per wave tile, 4 tiles per block
    for (int i = 0; i < 3; ++i) PTV_TRY(c->qpts[i].ensure(npad));
    PTV_TRY(launch_pad_queries(p->x, p->y, p->z, n, npad, c->qpts[0].p, c->qpts[1].p, c->qpts[2].p, s));
    ptv_grid g{};
    g.nx = 16;  // 4 wave tiles along x per block (ptv_filter.hip pos_of)
    g.ny = 4;
    g.nz = npad / 64;
    g.px = c->qpts[0].p;
    g.py = c->qpts[1].p;
    g.pz = c->qpts[2].p;
    g.z_begin = 0;
    g.z_end = g.nz;
    double r0s = kFilterR0Scale, occ = kFilterOccupancy;
    if (const char *e = dev_knob("PTV_FILTER_R0")) r0s = std::atof(e);       // dev knobs
    if (const char *e = dev_knob("PTV_FILTER_OCC")) occ = std::atof(e);
    if (filter_kmax(prm->k) == 0) {
        // k >= 127: the large-k path on the particles in original order (ptv_knn_big.hip)
        const SearchParams sb{PTV_METHOD_IDW, prm->k + 1, 2.0, 1e-10, 0u, std::max(1.0, (prm->k + 1) / 256.0), 1.0, -1};
        KnnLaunch kl;
        Binned b{};
        c->rbf_chunks = 0;
        c->cull_timed = false;
        PTV_TRY(prepare(c, p, &g, &sb, nullptr, nullptr, nullptr, g.px, g.py, g.pz, s, kl, b));
        PTV_TRY(c->flt_spd.ensure((size_t)n));
        PTV_TRY(launch_slot_speed(b.pval, n, c->flt_spd.p, s));
        BigQueries q;
        q.particles = 1;
        q.px = p->x;
        q.py = p->y;
        q.pz = p->z;
        q.pu = p->u;
        q.pv = p->v;
        q.pw = p->w;
        BigEpilogue ep;
        ep.filter = 1;
        ep.spd = c->flt_spd.p;
        ep.keep = keep;
        ep.kth = kth;
        ep.threshold = prm->threshold;
        ep.mad_eps = prm->mad_eps;
        PTV_TRY(run_big_knn(c->big, q, b, kl.cg, n, prm->k + 1, ep, s));
        PTV_HIP(hipEventRecord(c->ev_knn1, s));
        c->timed_pending = true;
        c->last.n_voxels = n;
        return PTV_OK;
    }
    const SearchParams sp{PTV_METHOD_IDW, prm->k + 1, 2.0, 1e-10, 0u, occ, r0s, -1};
    KnnLaunch kl;
    Binned b{};
    PTV_TRY(prepare(c, p, &g, &sp, nullptr, nullptr, nullptr, g.px, g.py, g.pz, s, kl, b));
    // query order: Morton order of the particles over the bounding box prepare() measured,
    // laid out in the k-NN kernel's sub-ball lane pattern (ptv_filter.hip)
    const double lo[3] = {c->h_bbox[0], c->h_bbox[1], c->h_bbox[2]};
    const double hi[3] = {c->h_bbox[3], c->h_bbox[4], c->h_bbox[5]};
    const size_t tb = morton_sort_temp_bytes(n);
    PTV_TRY(c->flt_code.ensure((size_t)npad));  // Morton keys, then the queries' original indices
    PTV_TRY(c->flt_count.ensure(n));
    PTV_TRY(c->flt_start.ensure(n));
    PTV_TRY(c->flt_perm.ensure(n));
    PTV_TRY(c->flt_scanp.ensure(tb / 4 + 1));
    PTV_TRY(launch_morton_order(p->x, p->y, p->z, n, lo, hi, c->flt_code.p, c->flt_count.p, c->flt_start.p,
                                c->flt_perm.p, c->flt_scanp.p, tb, s));
    // q_orig: the original index at each query position (reuses the Morton key buffer, dead
    // after the sort); the speeds of the binned particles in slot order
    uint32_t *q_orig = c->flt_code.p;
    PTV_TRY(launch_query_layout(c->flt_perm.p, p->x, p->y, p->z, n, npad, c->qpts[0].p, c->qpts[1].p, c->qpts[2].p,
                                q_orig, s));
    PTV_TRY(c->flt_spd.ensure((size_t)n));
    PTV_TRY(launch_slot_speed(b.pval, n, c->flt_spd.p, s));
    // the (k+1)-NN search with the statistics fused into its epilogue (no slot list in HBM)
    kl.mode = kModeFilter;
    kl.fe.q_orig = q_orig;
    kl.fe.inv = c->code.p;  // the binning's inverse permutation (launch_bin: code = inv after the scatter)
    kl.fe.spd = c->flt_spd.p;
    kl.fe.keep = keep;
    kl.fe.kth = kth;
    kl.fe.threshold = prm->threshold;
    kl.fe.mad_eps = prm->mad_eps;
    c->rbf_chunks = 0;
    PTV_TRY(launch_knn(kl, b, nullptr, nullptr, nullptr, c->qpts[0].p, c->qpts[1].p, c->qpts[2].p, nullptr, nullptr,
                       nullptr, nullptr, s));
    PTV_HIP(hipEventRecord(c->ev_knn1, s));
    c->timed_pending = true;
    c->last.n_voxels = n;
    return PTV_OK;
}

}  // namespace

extern "C" {

int ptv_sample_mask_dev(ptv_ctx *c, const ptv_mask_grid *src, const ptv_grid *g, uint8_t *out, void *stream) {
    if (!c) {
        set_error("NULL context");
        return PTV_E_ARG;
    }
    PTV_TRY(mask_grid_check(g, out));
    PTV_HIP(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    MaskSampleLaunch m{};
    PTV_TRY(mask_source(c, src, m, s));
    return run_mask_sample(c, m, g, src->raw, out, s);
}

int ptv_sample_mask(ptv_ctx *c, const ptv_mask_grid *src, const ptv_grid *g, uint8_t *out) {
    if (!c) {
        set_error("NULL context");
        return PTV_E_ARG;
    }
    PTV_TRY(mask_grid_check(g, out));
    PTV_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    MaskSampleLaunch m{};
    PTV_TRY(mask_source(c, src, m, s));
    const int64_t nraw = src->nx * src->ny * src->nz;
    PTV_TRY(c->mask_raw.ensure(nraw));
    PTV_HIP(hipMemcpyAsync(c->mask_raw.p, src->raw, nraw, hipMemcpyHostToDevice, s));
    ptv_grid dg = *g;
    const int64_t plane = g->nx * g->ny, nfull = g->nz * plane, nout = (g->z_end - g->z_begin) * plane;
    if (g->ax && g->ay && g->az) {
        PTV_TRY(c->axes.ensure(g->nx + g->ny + g->nz));
        PTV_HIP(hipMemcpyAsync(c->axes.p, g->ax, g->nx * sizeof(double), hipMemcpyHostToDevice, s));
        PTV_HIP(hipMemcpyAsync(c->axes.p + g->nx, g->ay, g->ny * sizeof(double), hipMemcpyHostToDevice, s));
        PTV_HIP(hipMemcpyAsync(c->axes.p + g->nx + g->ny, g->az, g->nz * sizeof(double), hipMemcpyHostToDevice, s));
        dg.ax = c->axes.p;
        dg.ay = c->axes.p + g->nx;
        dg.az = c->axes.p + g->nx + g->ny;
        dg.px = dg.py = dg.pz = nullptr;
    } else {
        const double *q[3] = {g->px, g->py, g->pz};
        for (int i = 0; i < 3; ++i) {
            PTV_TRY(c->qpts[i].ensure(nfull));
            PTV_HIP(hipMemcpyAsync(c->qpts[i].p, q[i], nfull * sizeof(double), hipMemcpyHostToDevice, s));
        }
        dg.ax = dg.ay = dg.az = nullptr;
        dg.px = c->qpts[0].p;
        dg.py = c->qpts[1].p;
        dg.pz = c->qpts[2].p;
    }
    PTV_TRY(c->mask_out.ensure(nout));
    PTV_TRY(run_mask_sample(c, m, &dg, c->mask_raw.p, c->mask_out.p, s));
    PTV_HIP(hipMemcpyAsync(out, c->mask_out.p, nout, hipMemcpyDeviceToHost, s));
    PTV_HIP(hipStreamSynchronize(s));
    return PTV_OK;
}

int ptv_boundary_particles_dev(ptv_ctx *c, const ptv_boundary_params *prm, double *x, double *y, double *z,
                               int64_t cap, int64_t *count, void *stream) {
    BoundaryLaunch m{};
    PTV_TRY(boundary_check(c, prm, count, m));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    PTV_TRY(run_boundary(c, m, x, y, z, cap, count, s));
    PTV_HIP(hipStreamSynchronize(s));
    return PTV_OK;
}

int ptv_boundary_particles(ptv_ctx *c, const ptv_boundary_params *prm, double *x, double *y, double *z, int64_t cap,
                           int64_t *count) {
    BoundaryLaunch m{};
    PTV_TRY(boundary_check(c, prm, count, m));
    hipStream_t s = c->stream;
    const int64_t nvox = prm->nx * prm->ny * prm->nz;
    PTV_TRY(c->mask_raw.ensure(nvox));
    PTV_HIP(hipMemcpyAsync(c->mask_raw.p, prm->mask, nvox, hipMemcpyHostToDevice, s));
    m.mask = c->mask_raw.p;
    // size the device output from the count pass when the caller's buffers are large enough
    int64_t nsel = 0;
    PTV_TRY(run_boundary(c, m, nullptr, nullptr, nullptr, 0, &nsel, s));
    *count = nsel;
    if (x && y && z && cap >= nsel && nsel > 0) {
        PTV_TRY(c->bnd_xyz.ensure((size_t)3 * nsel));
        double *d = c->bnd_xyz.p;
        PTV_TRY(run_boundary(c, m, d, d + nsel, d + 2 * nsel, nsel, &nsel, s));
        PTV_HIP(hipMemcpyAsync(x, d, nsel * sizeof(double), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipMemcpyAsync(y, d + nsel, nsel * sizeof(double), hipMemcpyDeviceToHost, s));
        PTV_HIP(hipMemcpyAsync(z, d + 2 * nsel, nsel * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    PTV_HIP(hipStreamSynchronize(s));
    return PTV_OK;
}

int ptv_filter_outliers_knn_dev(ptv_ctx *c, const ptv_particles *p, const ptv_filter_params *prm, uint8_t *keep,
                                double *kth_dist, void *stream, ptv_stats *st) {
    PTV_TRY(filter_check(c, p, prm, keep));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    PTV_TRY(run_filter(c, p, prm, keep, kth_dist, s));
    if (st) *st = c->last;
    return PTV_OK;
}

int ptv_filter_outliers_knn(ptv_ctx *c, const ptv_particles *p, const ptv_filter_params *prm, uint8_t *keep,
                            double *kth_dist, ptv_stats *st) {
    PTV_TRY(filter_check(c, p, prm, keep));
    hipStream_t s = c->stream;
    const int64_t n = p->n;
    const double *src[6] = {p->x, p->y, p->z, p->u, p->v, p->w};
    for (int i = 0; i < 6; ++i) {
        PTV_TRY(c->pin[i].ensure(n));
        PTV_HIP(hipMemcpyAsync(c->pin[i].p, src[i], n * sizeof(double), hipMemcpyHostToDevice, s));
    }
    ptv_particles dp{n, c->pin[0].p, c->pin[1].p, c->pin[2].p, c->pin[3].p, c->pin[4].p, c->pin[5].p};
    PTV_TRY(c->flt_keep.ensure(n));
    PTV_TRY(c->flt_kth.ensure(n));
    PTV_TRY(run_filter(c, &dp, prm, c->flt_keep.p, c->flt_kth.p, s));
    PTV_HIP(hipMemcpyAsync(keep, c->flt_keep.p, n, hipMemcpyDeviceToHost, s));
    if (kth_dist) PTV_HIP(hipMemcpyAsync(kth_dist, c->flt_kth.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
    PTV_HIP(hipStreamSynchronize(s));
    PTV_TRY(finish_timing(c));
    if (st) *st = c->last;
    return PTV_OK;
}

}  // extern "C"
