// ptv_knn_impl.hpp — exact k-nearest-neighbour IDW / Sibson interpolation onto a voxel grid (gfx950).
//
// Replaces, per voxel, the reference hot loop
//   distances, indices = tree.query(flat_coords, k)                 interpolator.py:139 (:97)
//   weights = 1/(d**p + 1e-10); weights /= weights.sum(axis=1)       interpolator.py:142-147
//   (Sibson: inv-distance * exp(-d/std(d)), renormalised            interpolator.py:102-116)
//   out[:, c] = (weights * values[indices, c]).sum(axis=1)          interpolator.py:150-153 (:119-122)
//
// Work decomposition: one wave64 = one 4x4x4 voxel tile (lane = voxel); a 256-thread
// workgroup = 4 independent tiles along x (16x4x4 voxels, 128-B output rows).
//
// Exact search by radius shells around the tile's bounding box B:
//   pass 1 gathers every particle whose cell lies within R0 of B (R0 from the mean
//   particle density); pass j gathers the shell R_{j-1} < dist <= R_j.  A lane whose
//   current k-th distance is <= R_j is exact (every particle it has not seen is
//   farther than R_j from B, hence from its voxel).  If all lists are full the next
//   radius is the largest lane k-th distance (one more pass finishes every lane);
//   otherwise R doubles.  Sphere interiors (empty voids) just take more passes.
// Gather: the candidate cells of a pass are, per cell row (cy, cz), one or two x-runs
// of consecutive cells = contiguous particle ranges of the linear-order counting sort.
// Lane i takes row i: it loads its run bounds from cell_start (64 rows per round,
// all loads in flight together), a wave prefix sum places the runs, and the lanes
// copy the particle records into a per-wave LDS buffer.  The compute loop then reads
// each candidate with a wave-uniform LDS address (broadcast) and updates every lane's
// sorted register list of the KMAX best (d2, slot) with a branch-free insertion
// network, skipped wave-wide when no lane improves.
//
// Bit-level contract with the reference (compiled with -ffp-contract=off):
//   d2 = (dx*dx + dy*dy) + dz*dz, d = sqrt(d2)      (cKDTree p=2 accumulation, then sqrt)
//   d**p: p=2 -> d*d, 1 -> d, 0.5 -> sqrt, -1 -> 1/d, else pow (numpy scalar fast paths)
//   row sums: numpy pairwise order from identity 0.0 (8 accumulators, n%8 tail)
// Ties at equal d2 keep the earlier candidate in the (deterministic) gather order
// (cKDTree's tie order is traversal dependent too).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <utility>

#include "../../include/ptv_api.h"
#include "ptv_kernels.hpp"
#include "ptv_median.hpp"
#include "ptv_wave.hpp"

namespace ptv {

#ifndef PTV_SUBBALL_RUNS
#define PTV_SUBBALL_RUNS 1  // clip the gather runs to the sub-balls' chords (0: the tile ball's)
#endif
#ifndef PTV_KNN_WAVES
#define PTV_KNN_WAVES 4  // waves per SIMD the k <= 8 kernels are register-capped for
#endif
#ifndef PTV_KNN_WAVES_BIG
#define PTV_KNN_WAVES_BIG 2  // KMAX > 32: capped for 2 waves per SIMD (spills, yet k = 50 -30 %: one wave could not hide its latency)
#endif
#ifndef PTV_KNN_WAVES_SMALL
#define PTV_KNN_WAVES_SMALL 5  // KMAX = 4 (nearest, radius, k <= 4): 5 waves per SIMD (nearest -2 %)
#endif
#ifndef PTV_KNN_WAVES_MID
#define PTV_KNN_WAVES_MID 3  // 8 < KMAX <= 32: capped for 3 waves per SIMD (Sibson k=30 and the RBF k=32 slot search -7 %)
#endif

#ifndef PTV_KNN_KEYI_2W
#define PTV_KNN_KEYI_2W 40  // key-list interpolation kernels of at least this many slots: 2 waves per SIMD
#endif

#ifndef PTV_KNN_UNROLL_MAX
// key-list interpolation epilogues up to this many slots unroll their blocks at compile time;
// longer lists run the rolled passes.  Round 5: 32 -> 56 (with KEEP below; the key list's 2 x KMAX
// VGPRs are dead by the epilogue, so the kept distances fit the 2-wave budget: 8 VGPRs spilled at
// 56 slots).  Same-box A/B, 512^3 / 5M main launch: Sibson k = 45 119.6 -> 87.9 ms, Sibson k = 50
// 137.2 -> 100.0, IDW k = 36 77.7 -> 75.4, IDW k = 50 101.8 -> 100.8.  At 64 slots Sibson k = 60
// gains (160.9 -> 126.5) but IDW k = 60 loses (122.1 -> 130.2, 49 VGPRs spilled): 64 stays rolled.
#define PTV_KNN_UNROLL_MAX 56
#endif
#ifndef PTV_VALUE_HALF_BLOCKS
#define PTV_VALUE_HALF_BLOCKS 1  // dev builds: 0 = the value pass in whole blocks of 8
#endif
#ifndef PTV_KNN_KEEP_MAX
// key lists up to this many slots keep the epilogue's distances (then weights) in registers
// between passes; longer ones re-gather the records every pass (Sibson: four passes)
#define PTV_KNN_KEEP_MAX 56
#endif
// unroll factors (same-box A/B, 512^3 / 5M, profiles/r06_ab/unroll_ab.txt): the k <= 8 seed
// network's loop over pairs of seeds by 2 (headline main launch 14.09 -> 13.98 ms; the filter's
// seed loop slower unrolled), the fp32 prefilter's loop over 4 candidates by 2 in the filter only
#ifndef PTV_SEED_UNROLL
#define PTV_SEED_UNROLL 2
#endif
#ifndef PTV_K1_BROADCAST_SEEDS
#define PTV_K1_BROADCAST_SEEDS 1  // one-slot list: corner seeds by lane broadcast (no LDS hash)
#endif
#ifndef PTV_SEED_UNROLL_FILTER
#define PTV_SEED_UNROLL_FILTER 1
#endif
#ifndef PTV_MASK_UNROLL
#define PTV_MASK_UNROLL 1
#endif
#ifndef PTV_MASK_UNROLL_FILTER
#define PTV_MASK_UNROLL_FILTER 2
#endif
#define PTV_PRAGMA_(x) _Pragma(#x)
#define PTV_UNROLL(n) PTV_PRAGMA_(unroll n)
#ifndef PTV_FILTER_SEEDED
#define PTV_FILTER_SEEDED 0  // dev builds: 1 = the filter's first gather pass at its wave's largest seed bound
#endif
#ifndef PTV_STAMP_SEEDSPLIT
#define PTV_STAMP_SEEDSPLIT 0  // dev stamp builds: union-seed counting passes stamped as 'setup'
#endif
#ifndef PTV_STAMP_ALL
#define PTV_STAMP_ALL 0  // dev builds: 1 = the STAMP instantiation for every KMAX (not only 8)
#endif

constexpr int kStampFields = 8;
#ifndef PTV_TIGHTEN_MIN
#define PTV_TIGHTEN_MIN 32
#endif
// lattice levels: insertions per group that pay for the fp32 k-th network (same-box A/B, 512^3 / 5M:
// lattice 1.86 ms without it, 1.80 at 16, 1.72 at 32; C2 and the 2/8 share unchanged)
constexpr int kTightenMin = PTV_TIGHTEN_MIN;
#ifndef PTV_TIGHTEN_KEYS
// dev builds: key-list modes that tighten a group's threshold first (1 = filter, 2 = interp).  Off:
// same-box A/B at 512^3 / 5M, filter k = 25 19.80 -> 20.52 ms, Sibson k = 30 55.2 -> 60.3, IDW k = 50
// 104.0 -> 121.8 (the key lists' thresholds are already tight after the first group)
#define PTV_TIGHTEN_KEYS 0
#endif
template <int MODE>
constexpr bool tighten_keys() {
    return (MODE == kModeFilter && (PTV_TIGHTEN_KEYS & 1)) || (MODE == kModeInterp && (PTV_TIGHTEN_KEYS & 2));
}
constexpr int kCap = 128;        // LDS candidate slots per wave (16 B fp32 + 32 B fp64 each)
// dev builds: candidate slots and waves per SIMD of the one-slot (k = 1) kernel.  Same-box A/B,
// 512^3 / 5M nearest: 128 slots at 5 waves 8.42 ms; 96 at 6 (80 VGPRs, 24 spilled) 9.12; 96 at 7
// 10.06; 80 at 6 9.23 -- the spills cost more than the occupancy gives
#ifndef PTV_KCAP1
#define PTV_KCAP1 128
#endif
#ifndef PTV_KNN_WAVES_K1
#define PTV_KNN_WAVES_K1 PTV_KNN_WAVES_SMALL  // dev builds: waves per SIMD of the one-slot kernel
#endif
template <int KMAX>
constexpr int cand_cap() { return KMAX == 1 ? PTV_KCAP1 : kCap; }
constexpr int kRowsPerLane = 1;  // cell rows examined per lane per gather round
constexpr int kRunEntries = 64 * 2 * kRowsPerLane;  // x-runs per gather round (power of two)

// Diagnostics (ptv_debug_stamps): when set, KMAX=8 launches use the STAMP instantiation,
// which writes one record of kStampFields u64 per wave (s_memtime phase cycles + counts).

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct KnnKernelArgs {
    CellGrid cg;
    int nx, ny, nz, z0, z1;
    int ntx, nty, ntz, ntxb;
    int separable, method, k, kpad;
    double power, eps;
    uint32_t flags;
    double r0;    // first gather radius
    double rall;  // radius that covers the whole cell grid from any query
    int mode;     // kModeInterp / kModeKDist
    CoarseBound cb;
    float4 *kd_recs;   // kModeKDist: k-NN seed records out (NULL = none): {p - c (fp32), slot}
    int lz0;           // plane of coarse-lattice point 0
    uint32_t *slots;   // kModeSlots: neighbour slots out
    int seed_n;        // seed records used per lattice corner (<= k)
    int nblocks;       // workgroups of the launch (the grid may be 2-D, see launch_knn)
    double radius;     // kModeRadius: every particle with d2 <= radius^2 (query_ball_point's test)
    FilterEpilogue fe;  // kModeFilter
    const int *order;  // block dispatch order (NULL: XCD-contiguous ranges)
    // packed-key lists (KMAX >= 16, see insert_key): slot bits of a key, and the factor that
    // turns a key into an upper bound on its exact d2 (1 + 2^(B - 51), B = slot bits)
    uint32_t smask;
    double kscale;
    // near-tie repair: key-list waves whose order is not proven exact list their tile here
    // (b * 4 + wave) and skip their outputs; the exact instantiation reruns them
    unsigned int *rep_cnt;
    uint32_t *rep_list;
    int rep_cap;
    const uint32_t *tiles;  // repair launch: the listed tiles (wave e of the launch takes tiles[e])
    int ntiles;
    // slab cull: the proven halo (a double's bits, launch_halo_need) and the halo binned; the
    // launch does nothing unless gate_halo >= proven (the host reads the proof after it)
    const unsigned long long *gate;
    double gate_halo;
    // lattice void tiles (kModeKDist, see k_kdist_merge): a split launch runs `split` waves per
    // tile over the first split_tiles tiles of the block order (tile t = block order[t / 4], x-tile
    // t % 4), wave part p taking every split-th cell row of one pass at the lattice bound,
    // and leaves its partial list in split_out[((t * split + p) * KMAX + j) * 64 + lane] (slots,
    // ~0 = none); 0 = an ordinary launch
    int split;
    int split_tiles;
    uint32_t *split_out;
    // a fused lattice launch: its first split_lb blocks are the split waves, the others ordinary
    // blocks of the order from entry lb + order_skip (0 and 0: every block one kind)
    int split_lb;
    int order_skip;
};

// Packed keys (the KMAX >= 16 lists).  A key is the candidate's exact f64 d2 with the low B
// mantissa bits replaced by its slot (B = bits of the largest slot): a non-negative double
// whose order is (truncated d2, slot), so a sorted insertion is one v_min_f64 + one v_max_f64
// per slot (5 VALU per slot and a third register per entry with a separate slot array).
// Truncation keeps the order of keys whose truncated d2 differ; ties of the exact d2 keep slot
// order (equal d2 -> equal truncation).  Only distinct d2 values sharing one truncation can be
// misordered: the epilogue recomputes the exact d2 of the list, checks that it ascends and that
// the (k+1)-th key's truncation differs from the k-th's (nothing outside the list can then beat
// the k-th), and otherwise lists the tile for the exact rerun.
__device__ __forceinline__ double make_key(bool has, double e2, uint32_t slot, uint32_t smask) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(e2);
    uint32_t lo = ((uint32_t)bits & ~smask) | slot;  // v_bfi_b32
    uint32_t hi = (uint32_t)(bits >> 32);
    lo = has ? lo : 0u;  // no candidate: +inf, a no-op for the network
    hi = has ? hi : 0x7ff00000u;
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ uint32_t key_slot(double key, uint32_t smask) {
    return (uint32_t)__double_as_longlong(key) & smask;
}

// keys a and b (both finite, >= 0) hold the same truncated d2
__device__ __forceinline__ bool same_trunc(double a, double b, uint32_t smask) {
    const unsigned long long x = (unsigned long long)(__double_as_longlong(a) ^ __double_as_longlong(b));
    return (x & ~(unsigned long long)smask) == 0ull;
}

template <int KMAX>
__device__ __forceinline__ void insert_key(double (&bd)[KMAX], double key) {
    // ascending min/max carry sweep, every slot updated in place (see insert())
    double cd = key;
#pragma unroll
    for (int j = 0; j < KMAX - 1; ++j) {
        double nc;
        asm("v_max_f64 %[nc], %[bd], %[cd]\n\t"
            "v_min_f64 %[bd], %[bd], %[cd]"
            : [bd] "+v"(bd[j]), [nc] "=&v"(nc)
            : [cd] "v"(cd));
        cd = nc;
    }
    asm("v_min_f64 %[bd], %[bd], %[cd]" : [bd] "+v"(bd[KMAX - 1]) : [cd] "v"(cd));
}

// Batched insertion into a key list: 8 keys sorted by a network, then Batcher's odd-even merge
// of the sorted list (registers 0 .. KMAX-1) with them (KMAX .. KMAX+7), keeping the KMAX
// smallest.  The merge leaves the kept outputs in registers 0 .. KMAX-1 in order, and every
// comparator that only feeds the dropped 8 outputs is removed (one op for those that keep
// only their min or max): 310 ops for 8 keys at KMAX = 56 against 896 for 8 insert_key sweeps.
// Keys are distinct (the slot is part of the key), so the list equals the sequential one.
struct KeyNet {
    int n;
    short a[1536], b[1536];    // up to the 1471 comparators of a full 128-entry sort (SortNetOf)
    unsigned char kind[1536];  // 1: a = min only, 2: b = max only, 3: both
};
struct RegList {
    int n;
    short r[160];
};
constexpr RegList reg_sub(const RegList &x, int start) {
    RegList o{};
    o.n = 0;
    for (int i = start; i < x.n; i += 2) o.r[o.n++] = x.r[i];
    return o;
}
// merge sorted register lists A and B in place (comparators appended to net); out = the sorted
// register order
constexpr void net_merge(const RegList &A, const RegList &B, KeyNet &net, RegList &out) {
    out.n = 0;
    if (A.n == 0 || B.n == 0) {
        const RegList &s = A.n == 0 ? B : A;
        for (int i = 0; i < s.n; ++i) out.r[out.n++] = s.r[i];
        return;
    }
    if (A.n == 1 && B.n == 1) {
        net.a[net.n] = A.r[0];
        net.b[net.n] = B.r[0];
        net.kind[net.n++] = 3;
        out.r[out.n++] = A.r[0];
        out.r[out.n++] = B.r[0];
        return;
    }
    RegList v{}, w{};
    net_merge(reg_sub(A, 0), reg_sub(B, 0), net, v);
    net_merge(reg_sub(A, 1), reg_sub(B, 1), net, w);
    out.r[out.n++] = v.r[0];
    for (int i = 0;; ++i) {
        const bool hw = i < w.n, hv = i + 1 < v.n;
        if (hw && hv) {
            net.a[net.n] = w.r[i];
            net.b[net.n] = v.r[i + 1];
            net.kind[net.n++] = 3;
            out.r[out.n++] = w.r[i];
            out.r[out.n++] = v.r[i + 1];
        } else if (hw) {
            out.r[out.n++] = w.r[i];
        } else if (hv) {
            out.r[out.n++] = v.r[i + 1];
        } else {
            break;
        }
    }
}
constexpr void net_sort(const RegList &x, KeyNet &net, RegList &out) {
    if (x.n <= 1) {
        out = x;
        return;
    }
    RegList lo{}, hi{}, slo{}, shi{};
    const int h = x.n / 2;
    for (int i = 0; i < x.n; ++i) (i < h ? lo.r[lo.n++] : hi.r[hi.n++]) = x.r[i];
    net_sort(lo, net, slo);
    net_sort(hi, net, shi);
    net_merge(slo, shi, net, out);
}
template <int KMAX, int NB>
constexpr KeyNet make_key_net() {
    KeyNet net{};
    RegList L{}, Bk{}, sb{}, out{};
    for (int i = 0; i < KMAX; ++i) L.r[L.n++] = (short)i;
    for (int i = 0; i < NB; ++i) Bk.r[Bk.n++] = (short)(KMAX + i);
    net_sort(Bk, net, sb);
    const int nsort = net.n;
    net_merge(L, sb, net, out);
    // the kept outputs sit in registers 0 .. KMAX-1 in order (checked here); remove dead ops
    bool live[KMAX + NB] = {};
    for (int i = 0; i < KMAX; ++i) {
        if (out.r[i] != i) net.n = -1;  // not in place: refuse (the static_assert below fires)
        live[i] = true;
    }
    if (net.n < 0) return net;
    KeyNet res{};
    int keep[1536] = {};
    for (int c = net.n - 1; c >= 0; --c) {
        const bool la = live[net.a[c]], lb = live[net.b[c]];
        keep[c] = c < nsort ? 3 : (la ? 1 : 0) | (lb ? 2 : 0);
        if (keep[c]) live[net.a[c]] = live[net.b[c]] = true;
    }
    for (int c = 0; c < net.n; ++c)
        if (keep[c]) {
            res.a[res.n] = net.a[c];
            res.b[res.n] = net.b[c];
            res.kind[res.n++] = (unsigned char)keep[c];
        }
    return res;
}
template <int KMAX, int NB>
struct KeyNetOf {
    static constexpr KeyNet net = make_key_net<KMAX, NB>();
    static_assert(net.n > 0, "merge network outputs not in place");
};
template <int KMAX, int NB, int C>
__device__ __forceinline__ void key_net_op(double (&v)[KMAX + NB]) {
    constexpr int a = KeyNetOf<KMAX, NB>::net.a[C], b = KeyNetOf<KMAX, NB>::net.b[C], kd = KeyNetOf<KMAX, NB>::net.kind[C];
    const double x = v[a], y = v[b];
    if constexpr (kd & 1) {
        double r;
        asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
        v[a] = r;
    }
    if constexpr (kd & 2) {
        double r;
        asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
        v[b] = r;
    }
}
template <int KMAX, int NB, int... C>
__device__ __forceinline__ void key_net_run(double (&v)[KMAX + NB], std::integer_sequence<int, C...>) {
    (key_net_op<KMAX, NB, C>(v), ...);
}
#ifndef PTV_KEY_BATCH
#define PTV_KEY_BATCH 8  // dev builds: keys per merge network
#endif
template <int KMAX>
constexpr int key_batch() { return PTV_KEY_BATCH; }
// the NB keys nk (any order, +inf = none) into the sorted list bd
template <int KMAX, int NB>
__device__ __forceinline__ void insert_keys(double (&bd)[KMAX], const double (&nk)[NB]) {
    double v[KMAX + NB];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) v[j] = bd[j];
#pragma unroll
    for (int j = 0; j < NB; ++j) v[KMAX + j] = nk[j];
    key_net_run<KMAX, NB>(v, std::make_integer_sequence<int, KeyNetOf<KMAX, NB>::net.n>{});
#pragma unroll
    for (int j = 0; j < KMAX; ++j) bd[j] = v[j];
}

// Full sort of KMAX registers (net_sort: Batcher's odd-even merge sort, every comparator
// ascending) and the register that holds each sorted position.
template <int KMAX>
struct SortNetOf {
    static constexpr KeyNet make() {
        KeyNet net{};
        RegList x{}, out{};
        for (int i = 0; i < KMAX; ++i) x.r[x.n++] = (short)i;
        net_sort(x, net, out);
        return net;
    }
    static constexpr RegList order() {
        KeyNet net{};
        RegList x{}, out{};
        for (int i = 0; i < KMAX; ++i) x.r[x.n++] = (short)i;
        net_sort(x, net, out);
        return out;
    }
    static constexpr KeyNet net = make();
    static constexpr RegList ord = order();
};
template <int KMAX, int C>
__device__ __forceinline__ void sort_net_op(double (&v)[KMAX]) {
    constexpr int a = SortNetOf<KMAX>::net.a[C], b = SortNetOf<KMAX>::net.b[C];
    const double x = v[a], y = v[b];
    double lo, hi;
    asm("v_min_f64 %0, %1, %2" : "=v"(lo) : "v"(x), "v"(y));
    asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(x), "v"(y));
    v[a] = lo;
    v[b] = hi;
}
template <int KMAX, int... C>
__device__ __forceinline__ void sort_net_run(double (&v)[KMAX], std::integer_sequence<int, C...>) {
    (sort_net_op<KMAX, C>(v), ...);
}
#ifndef PTV_MEDIAN_NET
#define PTV_MEDIAN_NET 1  // dev builds: 0 = the O(KMAX^2) rank selection (ptv_median.hpp)
#endif
// np.median of s[0..n) for values >= +0 or NaN (the filter's speeds and absolute deviations:
// no signed zeros, so any order of equal values gives the same bits): entries past n become
// +inf, one sorting network, the middle one (n odd) or the mean of the two middle ones; any NaN
// gives NaN (numpy's _median_nancheck).  191 comparators at KMAX = 32 against the rank
// selection's 2 x 1024 compares per call.
template <int KMAX>
__device__ __forceinline__ double median_sorted(const double (&s)[KMAX], int n) {
    bool nan = false;
    double v[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if (j < n) nan = nan || (s[j] != s[j]);
        v[j] = j < n ? s[j] : INFINITY;
    }
    sort_net_run<KMAX>(v, std::make_integer_sequence<int, SortNetOf<KMAX>::net.n>{});
    const int h = n >> 1;
    double lo = 0.0, hi = 0.0;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        const double x = v[SortNetOf<KMAX>::ord.r[i]];
        if (i == h - 1) lo = x;
        if (i == h) hi = x;
    }
    const double m = (n & 1) ? hi : (lo + hi) / 2.0;
    return nan ? __longlong_as_double(0x7ff8000000000000LL) : m;
}
template <int KMAX>
__device__ __forceinline__ double filter_median(const double (&s)[KMAX], int n) {
    if constexpr (PTV_MEDIAN_NET) return median_sorted<KMAX>(s, n);
    else return median_of<KMAX>(s, n);
}

// numpy's pairwise sum (see pairwise()) fed in index order in blocks of 8 values: block m
// holds a[m .. m + 7] (entries at or past n ignored).
struct PairwiseStream {
    double r[8];
    double res = 0.0;
    __device__ __forceinline__ void add(int m, int n, const double (&a)[8]) {
        if (n < 8) {  // m == 0: sequential from identity 0.0
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (i < n) s += a[i];
            res = s;
            return;
        }
        const int stop = n - (n & 7);
        if (m == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = a[i];
        } else if (m < stop) {
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] += a[i];
        } else {  // the tail block (n % 8 entries), after the tree of the accumulators
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (m + i < n) res += a[i];
        }
    }
    // the same as add(m, n, a) over the block's half h (entries m + 4h .. m + 4h + 3), both halves in
    // order: each entry meets the same accumulator or running sum in the same order
    __device__ __forceinline__ void add4(int m, int h, int n, const double (&a)[4]) {
        if (n < 8) {
            double s = h == 0 ? 0.0 : res;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * h + i < n) s += a[i];
            res = s;
            return;
        }
        const int stop = n - (n & 7);
        if (m == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) r[4 * h + i] = a[i];
        } else if (m < stop) {
#pragma unroll
            for (int i = 0; i < 4; ++i) r[4 * h + i] += a[i];
        } else {
            if (h == 0) res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (m + 4 * h + i < n) res += a[i];
        }
    }
    __device__ __forceinline__ double finish(int n) {
        if (n >= 8 && (n & 7) == 0) res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        return res;
    }
};

// numpy pairwise sum of a[0..n) (n <= KMAX <= 128), from identity 0.0.
template <int KMAX>
__device__ __forceinline__ double pairwise(const double (&a)[KMAX], int n) {
    if (KMAX < 8 || n < 8) {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (j < n) r += a[j];
        return r;
    }
    if constexpr (KMAX >= 8) {
        double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
        const int stop = n - (n & 7);
#pragma unroll
        for (int i = 8; i + 8 <= KMAX; i += 8) {
            if (i < stop) {
                r0 += a[i + 0];
                r1 += a[i + 1];
                r2 += a[i + 2];
                r3 += a[i + 3];
                r4 += a[i + 4];
                r5 += a[i + 5];
                r6 += a[i + 6];
                r7 += a[i + 7];
            }
        }
        double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
#pragma unroll
        for (int j = 8; j < KMAX; ++j)
            if (j >= stop && j < n) res += a[j];
        return res;
    }
    return 0.0;
}

// numpy pairwise sum of t[j] = w[j] * values[bp[j], c] over j < n (n >= 1), streaming the
// value loads in blocks of 8 (one block in flight at a time) instead of holding KMAX of them.
// Same order as pairwise(): 8 accumulators seeded with t[0..7], blocks of 8, then the tail.
template <int KMAX>
__device__ __forceinline__ double gather_pairwise(const double (&w)[KMAX], const int (&bp)[KMAX],
                                                  const double *__restrict__ vb, int c, int n) {
    auto val = [&](int j) { return vb[(size_t)max(bp[j], 0) * 4 + c]; };
    double v8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v8[i] = val(i);
    if (n < 8) {
        double r = 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i < n) r += w[i] * v8[i];
        return r;
    }
    double r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = w[i] * v8[i];
    const int stop = n - (n & 7);
#pragma unroll
    for (int m = 8; m + 8 <= KMAX; m += 8) {
        if (m < stop) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v8[i] = val(m + i);
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] += w[m + i] * v8[i];
        }
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int j = 8; j < KMAX; ++j)
        if (j >= stop && j < n) res += w[j] * val(j);
    return res;
}

// d ** p with numpy's scalar fast paths (p uniform).
__device__ __forceinline__ double np_pow(double d, double p) {
    if (p == 2.0) return d * d;
    if (p == 1.0) return d;
    if (p == 0.5) return sqrt(d);
    if (p == -1.0) return 1.0 / d;
    return pow(d, p);
}

// a / b correctly rounded from r = RN(1/b): q = RN(a r), then q + RN(a - b q) r (Markstein; exact
// for normal operands, checked against IEEE division on 3.6e8 random pairs).  One division
// serves every numerator that shares the denominator.
__device__ __forceinline__ double div_by(double a, double b, double r) {
    const double q = a * r;
    return fma(fma(-q, b, a), r, q);
}

// whether div_by(a, b, RN(1/b)) is the IEEE quotient for every a in {0} u [amin, amax] (amin the
// smallest nonzero numerator): b in [2^-1000, 2^1000] (1/b finite and normal), the nonzero
// numerators normal with margin (the residual a - b q exact) and every quotient normal
__device__ __forceinline__ bool div_by_ok(double amin, double amax, double b) {
    return b >= 0x1p-1000 && b <= 0x1p1000 && amin >= 0x1p-960 && amin >= b * 0x1p-1000 && amax <= b * 0x1p1000;
}

// IEEE sqrt for x >= 2^-767: the LLVM gfx9 f64 expansion (rsq seed, two Goldschmidt
// corrections) without its small-input rescale; tiny, zero and infinite x take sqrt()
__device__ __forceinline__ double sqrt_cr(double x) {
    if (!(x >= 0x1p-767 && x < INFINITY)) return sqrt(x);
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    g = fma(fma(-g, g, x), h, g);
    return fma(fma(-g, g, x), h, g);
}

// one voxel's outputs: float64, or float32 (RNE, numpy astype) under PTV_FLAG_OUT_F32
__device__ __forceinline__ void store_out(uint32_t flags, double *U, double *V, double *W, size_t vo, double u,
                                          double v, double w) {
    if (flags & PTV_FLAG_OUT_F32) {
        reinterpret_cast<float *>(U)[vo] = (float)u;
        reinterpret_cast<float *>(V)[vo] = (float)v;
        reinterpret_cast<float *>(W)[vo] = (float)w;
    } else {
        U[vo] = u;
        V[vo] = v;
        W[vo] = w;
    }
}

__device__ __forceinline__ double nan_to_num(double v) {
    if (v != v) return 0.0;
    if (v == INFINITY) return DBL_MAX;
    if (v == -INFINITY) return -DBL_MAX;
    return v;
}

// a wave-uniform double held in SGPRs
__device__ __forceinline__ double uniform(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_min(double v) { return group_reduce<0x3f>(v, OpMin{}); }
__device__ __forceinline__ double wave_max(double v) { return group_reduce<0x3f>(v, OpMax{}); }
__device__ __forceinline__ int wave_max_i(int v) { return group_reduce<0x3f>(v, OpMax{}); }
__device__ __forceinline__ int wave_incl_max_scan_i(int v) { return wave_incl_scan_max(v); }
__device__ __forceinline__ int wave_incl_scan_i(int v) { return wave_incl_scan_add(v); }

// order this wave's LDS writes before its later reads (and vice versa)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v_min_f64 / v_max_f64 without the input canonicalisation fmin/fmax get in IEEE mode (the
// list never holds NaN or signalling values)
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmax_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int KMAX>
__device__ __forceinline__ void insert(double (&bd)[KMAX], int (&bp)[KMAX], double d2, int p) {
    // Ascending carry sweep: m_j = d2 < bd[j] is monotone in j over the sorted list; from the
    // first j where it holds, slot j takes the carry (the candidate, then each displaced
    // entry) and hands its old entry on.  Ties keep the earlier entry first.  Every slot is
    // updated in place (selects on v_cmp masks, no exec-mask branches).
    // On a sorted list the carry is never below bd[j] once it differs from d2, so the distance
    // slot is min(bd[j], carry) and the new carry the max (one op each).  One asm block per slot
    // updates bd[j] and bp[j] IN PLACE (the carries go to fresh registers): written with
    // separate selects, the compiler renamed the list every step and paid 14 moves per insert
    // at the loop back-edge to put it back.
    double cd = d2;
    int cp = p;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if (j == KMAX - 1) {  // the last slot: no carry leaves the list
            asm("v_cmp_lt_f64 vcc, %[d2], %[bd]\n\t"
                "v_min_f64 %[bd], %[bd], %[cd]\n\t"
                "v_cndmask_b32 %[bp], %[bp], %[cp], vcc"
                : [bd] "+v"(bd[j]), [bp] "+v"(bp[j])
                : [d2] "v"(d2), [cd] "v"(cd), [cp] "v"(cp)
                : "vcc");
            break;
        }
        double ncd;
        int ncp;
        asm("v_cmp_lt_f64 vcc, %[d2], %[bd]\n\t"
            "v_max_f64 %[nc], %[bd], %[cd]\n\t"
            "v_min_f64 %[bd], %[bd], %[cd]\n\t"
            "v_cndmask_b32 %[np], %[cp], %[bp], vcc\n\t"
            "v_cndmask_b32 %[bp], %[bp], %[cp], vcc"
            : [bd] "+v"(bd[j]), [bp] "+v"(bp[j]), [nc] "=&v"(ncd), [np] "=&v"(ncp)
            : [d2] "v"(d2), [cd] "v"(cd), [cp] "v"(cp)
            : "vcc");
        cd = ncd;
        cp = ncp;
    }
}

// min(a, b) for non-NaN operands without fmin's canonicalising v_max
__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }

// fp32 prefilter threshold: every candidate whose exact d2 is < thr has fp32 d2 <= this
// (thr < 0: inactive lane, never; thr = inf: everything).
__device__ __forceinline__ float f32_bound(double thr, double cpass) {
    if (thr < 0.0) return -1.0f;
    return (float)((thr * (1.0 + 9.5367431640625e-07) + cpass) * (1.0 + 2.384185791015625e-07));
}

__device__ __forceinline__ int clampi(double f, int n) {
    return f < 0.0 ? 0 : (f >= (double)(n - 1) ? n - 1 : (int)f);
}

// an upper bound on sqrt(x), x >= 0, from the fp32 square root (any over-estimate of a
// gather half-width only adds cells; the same inputs always give the same bound)
__device__ __forceinline__ float sqrtf_up(float x) {  // x >= 0 already rounded up
    // v_sqrt_f32 (1 ulp) with 8 ulps of slack; inputs below 1e-30 are raised to it
    return __builtin_amdgcn_sqrtf(fmaxf(x, 1e-30f)) * 1.0000005f;
}
__device__ __forceinline__ double sqrt_up(double x) {
    return (double)sqrtf_up((float)(x * (1.0 + 2.384185791015625e-07)));
}

// bijection of [0, nb): block b (dispatched to XCD b % 8) -> a contiguous range per XCD
__device__ __forceinline__ int xcd_block(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, i = b >> 3;
    return (x < r) ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// distance between the extent [lo, hi] of a query box and cell c of an axis
__device__ __forceinline__ double axis_gap(int c, double o, double cs, double lo, double hi) {
    const double c0 = o + (double)c * cs;
    const double c1 = o + (double)(c + 1) * cs;
    return fmax(fmax(c0 - hi, lo - c1), 0.0);
}

// kModeKDist outputs of a lattice point's final list: an upper bound on its k-th neighbour distance
// in U[vo] and, with kd_recs, its k nearest records {particle - point (fp32), slot}, which seed the
// next finer level's tiles (any k distinct particles do: list order need not be exact there).
// Key lists (KEYS) hold k + 1 entries after the kpad sentinels, pair lists k.
template <int KMAX, bool KEYS>
__device__ __forceinline__ void kdist_out(const KnnKernelArgs &a, const double4 *__restrict__ prec,
                                          const double (&bd)[KMAX], const int (&bp)[KEYS ? 1 : KMAX], double qx,
                                          double qy, double qz, size_t vo, double *__restrict__ U) {
    if constexpr (KEYS) {
        U[vo] = sqrt(bd[KMAX - 2] * a.kscale) * (1.0 + 0x1p-50);
        if (a.kd_recs != nullptr) {
            float4 *o = a.kd_recs + vo * (size_t)a.k;
#pragma unroll
            for (int j0 = 0; j0 < KMAX; j0 += 8) {  // blocks of 8 gathers in flight
                double4 rec[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int j = min(j0 + i, KMAX - 1);
                    const bool ok = bd[j] >= 0.0 && bd[j] < INFINITY;
                    rec[i] = prec[ok ? key_slot(bd[j], a.smask) : 0u];
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int j = j0 + i;
                    if (j < KMAX - 1 && j >= a.kpad) {
                        const bool ok = bd[j] >= 0.0 && bd[j] < INFINITY;
                        o[j - a.kpad] = make_float4(ok ? (float)(rec[i].x - qx) : 0.f, ok ? (float)(rec[i].y - qy) : 0.f,
                                                    ok ? (float)(rec[i].z - qz) : 0.f,
                                                    __uint_as_float(ok ? key_slot(bd[j], a.smask) : 0xffffffffu));
                    }
                }
            }
        }
    } else {
        U[vo] = sqrt(bd[KMAX - 1]);
        if (a.kd_recs != nullptr) {
            float4 *o = a.kd_recs + vo * (size_t)a.k;
            double4 rec[KMAX];
#pragma unroll
            for (int j = 0; j < KMAX; ++j) rec[j] = prec[max(bp[j], 0)];  // every load in flight at once
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if (j >= a.kpad) {
                    const bool ok = bp[j] >= 0;
                    o[j - a.kpad] = make_float4(ok ? (float)(rec[j].x - qx) : 0.f, ok ? (float)(rec[j].y - qy) : 0.f,
                                                ok ? (float)(rec[j].z - qz) : 0.f,
                                                __uint_as_float(ok ? (uint32_t)bp[j] : 0xffffffffu));
                }
            }
        }
    }
}

// MODE (kModeInterp / kModeKDist / kModeSlots) is a template parameter so that the search-only
// modes carry no interpolation epilogue: one kernel for every mode put the KMAX = 32 lists at
// 284 registers (one wave per SIMD); split, every KMAX <= 32 kernel runs two waves per SIMD.
// KMAX >= 16 lists are packed keys (insert_key) unless EXACT: the (d2, slot) pair network, which
// the near-tie repair launches use.
template <int KMAX, bool EXACT>
constexpr bool kKeyList = KMAX >= 16 && !EXACT;

template <int KMAX, int MODE, bool EXACT>
constexpr int knn_waves() {
    if (KMAX == 1) return PTV_KNN_WAVES_K1;
    if (KMAX <= 4) return PTV_KNN_WAVES_SMALL;
    if (KMAX <= 8) return PTV_KNN_WAVES;
    // key lists: the search fits 3 waves per SIMD up to 32 slots, the streamed interpolation
    // epilogue (slots + two blocks of records + three pairwise accumulators) needs 2 from 24
    if (kKeyList<KMAX, EXACT> && MODE == kModeInterp && KMAX >= PTV_KNN_KEYI_2W) return KMAX <= 64 ? 2 : 1;
    return KMAX <= 32 ? PTV_KNN_WAVES_MID : (KMAX <= 64 ? PTV_KNN_WAVES_BIG : 1);
}

template <int KMAX, bool STAMP, int MODE, bool EXACT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(knn_waves<KMAX, MODE, EXACT>()))) void k_knn_interp(KnnKernelArgs a, const double4 *__restrict__ prec,
                                                    const double4 *__restrict__ pval,
                                                    const uint32_t *__restrict__ cstart,
                                                    const double *__restrict__ ax, const double *__restrict__ ay,
                                                    const double *__restrict__ az, const double *__restrict__ qpx,
                                                    const double *__restrict__ qpy, const double *__restrict__ qpz,
                                                    const uint8_t *__restrict__ mask, double *__restrict__ U,
                                                    double *__restrict__ V, double *__restrict__ W,
                                                    unsigned long long *__restrict__ dbg, long long dbg_cap) {
    unsigned long long t_mark = 0, t_setup = 0, t_seed = 0, t_rows = 0, t_copy = 0, t_comp = 0, t_epi = 0;
    auto stamp = [&](unsigned long long &acc) {
        if constexpr (STAMP) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc += t - t_mark;
            t_mark = t;
        }
    };
    if constexpr (STAMP) t_mark = __builtin_amdgcn_s_memtime();
    constexpr int kCap = cand_cap<KMAX>();
    __shared__ double4 lds_cand[4][kCap];
    __shared__ __attribute__((aligned(16))) float lds_cfx[4][kCap], lds_cfy[4][kCap], lds_cfz[4][kCap];
    __shared__ uint2 lds_runs[4][kRunEntries];
    __shared__ int lds_owner[4][64];
    // kModeRadius: the value records of the buffered candidates (the weights are summed in the flush)
    __shared__ double4 lds_val[4][MODE == kModeRadius ? kCap : 1];
    // key-list interpolation (k >= 13): the final slot lists in LDS, lane-major ([entry][lane] u32),
    // in this wave's candidate buffer (free once the search is done) and, past its kCap * 8 words,
    // lds_kx: the epilogue's passes read their blocks of 8 slots from here instead of holding KMAX
    // slot registers (and rotating them per block)
    constexpr bool KSLI = kKeyList<KMAX, EXACT> && MODE == kModeInterp;
    constexpr int KSLN = KSLI ? KMAX * 64 : 0;
    constexpr int KCW = kCap * 8;
    __shared__ uint32_t lds_kx[4][KSLN > KCW ? KSLN - KCW : 1];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    double4 *buf = lds_cand[wid];
    float *fbx = lds_cfx[wid], *fby = lds_cfy[wid], *fbz = lds_cfz[wid];
    uint2 *runs = lds_runs[wid];
    int *owner = lds_owner[wid];
    // XCD-aware block order: the dispatcher deals workgroups round-robin over the 8 XCDs,
    // so give XCD x a contiguous range of tiles (neighbouring tiles share cell rows and
    // particle records; each XCD has its own L2)
    constexpr bool KEYS = kKeyList<KMAX, EXACT>;
    const int lb = (int)(blockIdx.y * gridDim.x + blockIdx.x);  // linear dispatch order
    if (lb >= a.nblocks) return;                                  // 2-D grid padding (block-uniform)
    if (a.gate != nullptr && !(__longlong_as_double((long long)*a.gate) <= a.gate_halo))
        return;  // slab cull not proven exact: no outputs (the call returns PTV_E_INEXACT)
    int b, tw;  // block of the tile grid, wave (x-tile) within it
    // split lattice launch: this wave's part of its tile's cell rows (wave-uniform)
    int part = 0, nparts = 1;
    bool split_epi = false;
    if (MODE == kModeKDist && a.split > 0 && lb < a.split_lb) {
        const int e = lb * 4 + wid;
        const int t = e / a.split;
        if (t >= a.split_tiles) return;
        part = __builtin_amdgcn_readfirstlane(e - t * a.split);
        nparts = a.split;
        split_epi = true;
        b = a.order[t >> 2];
        tw = t & 3;
    } else if (a.tiles != nullptr) {
        // repair launch: wave e takes the e-th listed tile (wave-uniform exit)
        const int e = lb * 4 + wid;
        if (e >= a.ntiles) return;
        const uint32_t t = a.tiles[e];
        b = (int)(t >> 2);
        tw = (int)(t & 3u);
    } else {
        b = a.order != nullptr ? a.order[lb + a.order_skip] : xcd_block(lb, a.nblocks);
        tw = wid;
    }
    b = __builtin_amdgcn_readfirstlane(b);  // wave-uniform (the tile list is read per wave)
    const int bx = b % a.ntxb;
    const int rr = b / a.ntxb;
    const int ty = rr % a.nty;
    const int tz = rr / a.nty;
    const int tx = __builtin_amdgcn_readfirstlane(bx * 4 + tw);  // wave-uniform: scalar tile-box loads
    if (tx >= a.ntx) return;  // wave-uniform
    const int ix = tx * 4 + (lane & 3);
    const int iy = ty * 4 + ((lane >> 2) & 3);
    const int iz = a.z0 + tz * 4 + (lane >> 4);
    const bool valid = ix < a.nx && iy < a.ny && iz < a.z1;
    const int cx = min(ix, a.nx - 1), cy = min(iy, a.ny - 1), cz = min(iz, a.z1 - 1);
    const size_t vfull = ((size_t)cz * a.ny + cy) * a.nx + cx;
    double qx, qy, qz;
    if (a.separable) {
        qx = ax[cx];
        qy = ay[cy];
        qz = az[cz];
    } else {
        qx = qpx[vfull];
        qy = qpy[vfull];
        qz = qpz[vfull];
    }
    const bool active = valid && (mask == nullptr || mask[vfull] != 0);
    // seed records (k-NN lists of the tile's 8 lattice corners: lane = corner * 8 + entry, each
    // {particle - corner in fp32, slot}, 16 B), issued first so that their latency overlaps the
    // lattice-bound loads below
    float4 seed = make_float4(0.f, 0.f, 0.f, __uint_as_float(0xffffffffu));
    double scx = 0.0, scy = 0.0, scz = 0.0;  // the lane's corner
    if constexpr (KMAX <= 8) {
        if (a.cb.recs != nullptr) {
            const int jx0 = __builtin_amdgcn_readfirstlane(cx >> kLatticeShift);
            const int jy0 = __builtin_amdgcn_readfirstlane(cy >> kLatticeShift);
            const int jz0 = __builtin_amdgcn_readfirstlane((cz - a.lz0) >> kLatticeShift);
            const int cc = lane >> 3, j = lane & 7;
            const int jx = min(jx0 + (cc & 1), a.cb.n[0] - 1);
            const int jy = min(jy0 + ((cc >> 1) & 1), a.cb.n[1] - 1);
            const int jz = min(jz0 + (cc >> 2), a.cb.n[2] - 1);
            if (j < a.seed_n) seed = a.cb.recs[(((size_t)jz * a.cb.n[1] + jy) * a.cb.n[0] + jx) * a.k + j];
            scx = a.cb.ax[jx];
            scy = a.cb.ay[jy];
            scz = a.cb.az[jz];
        }
    }

    // upper bound on this voxel's k-th distance from the coarse lattice (triangle inequality)
    auto lattice_ub = [&]() -> double {
        double u = INFINITY;
        if (a.cb.dk == nullptr || !active) return u;
        // |v - c| in fp32 from lattice-relative offsets, rounded up: any upper bound is valid
        // the tile is one lattice cell: its corners are wave-uniform (scalar loads)
        const int j0[3] = {__builtin_amdgcn_readfirstlane(cx >> kLatticeShift),
                           __builtin_amdgcn_readfirstlane(cy >> kLatticeShift),
                           __builtin_amdgcn_readfirstlane((cz - a.lz0) >> kLatticeShift)};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int jx = min(j0[0] + (c & 1), a.cb.n[0] - 1);
            const int jy = min(j0[1] + ((c >> 1) & 1), a.cb.n[1] - 1);
            const int jz = min(j0[2] + (c >> 2), a.cb.n[2] - 1);
            const float ex = (float)(qx - a.cb.ax[jx]), ey = (float)(qy - a.cb.ay[jy]), ez = (float)(qz - a.cb.az[jz]);
            const float e2 = __fmaf_rn(ez, ez, __fmaf_rn(ey, ey, ex * ex));
            const double D = a.cb.dk[((size_t)jz * a.cb.n[1] + jy) * a.cb.n[0] + jx];
            u = fmin(u, D + (double)(sqrtf_up(e2) * 1.000002f));
        }
        return u * (1.0 + 1e-9) + a.cg.mg;
    };
    // With seed records the seeds' bound is the tighter one for (nearly) every lane: the
    // D(c) + |v - c| bound is then formed only when some active lane got no seed bound.
    const bool seeds_defer = a.cb.recs != nullptr;
    double ub = seeds_defer ? INFINITY : lattice_ub();
    // candidates at or beyond the bound can never be among the k nearest
    double ub2 = !active ? -1.0 : (ub < INFINITY ? ub * ub : INFINITY);
    // radius mode: every candidate with d2 <= R^2 counts (the list stays unused)
    const double rad2 = a.radius * a.radius;
    double rs = 0.0, rsu = 0.0, rsv = 0.0, rsw = 0.0;  // sum w, sum w*u, sum w*v, sum w*w
    if constexpr (MODE == kModeRadius) ub2 = !active ? -1.0 : rad2 * (1.0 + 2.220446049250313e-16) + 1e-300;

    // sorted list: KMAX-k front sentinels (-1) so bd[KMAX-1] is the k-th best.
    // Inactive lanes (padding / solid voxels) hold -1 everywhere: they never accept a
    // candidate and never ask for a larger radius.
    // Key lists (KEYS) hold k + 1 entries after the sentinels: the k-th at KMAX - 2, the
    // (k+1)-th at KMAX - 1 (the near-tie check); bp is unused.
    double bd[KMAX];
    int bp[KEYS ? 1 : KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) bd[j] = (!active || j < a.kpad) ? -1.0 : INFINITY;
#pragma unroll
    for (int j = 0; j < (KEYS ? 1 : KMAX); ++j) bp[j] = -1;
    // upper bound on the exact d2 of the list's k-th entry (the key may sit below it)
    auto kth2 = [&]() -> double {
        if constexpr (KEYS) return bd[KMAX - 2] * a.kscale;
        else return bd[KMAX - 1];
    };
    double thr = dmin(kth2(), ub2);

    uint32_t n_pass = 0, n_round = 0, n_rows = 0, n_cand = 0, n_acc = 0, n_surv = 0;

    stamp(t_setup);
    if (__builtin_amdgcn_ballot_w64(active) != 0) {
        // tile box (the gather geometry): on separable grids the extents of the tile's <= 4
        // axis values (wave-uniform loads; padded and masked voxels only enlarge it), otherwise
        // wave reductions over the active voxels
        double bx0, bx1, by0, by1, bz0, bz1;
        if (a.separable) {
            auto ext = [](const double *axv, int i0, int imax, double &lo, double &hi) {
                const double v0 = axv[i0], v1 = axv[min(i0 + 1, imax)], v2 = axv[min(i0 + 2, imax)],
                             v3 = axv[min(i0 + 3, imax)];
                lo = uniform(fmin(fmin(v0, v1), fmin(v2, v3)));
                hi = uniform(fmax(fmax(v0, v1), fmax(v2, v3)));
            };
            ext(ax, tx * 4, a.nx - 1, bx0, bx1);
            ext(ay, ty * 4, a.ny - 1, by0, by1);
            ext(az, a.z0 + tz * 4, a.z1 - 1, bz0, bz1);
        } else {
            bx0 = uniform(wave_min(active ? qx : INFINITY));
            bx1 = uniform(wave_max(active ? qx : -INFINITY));
            by0 = uniform(wave_min(active ? qy : INFINITY));
            by1 = uniform(wave_max(active ? qy : -INFINITY));
            bz0 = uniform(wave_min(active ? qz : INFINITY));
            bz1 = uniform(wave_max(active ? qz : -INFINITY));
        }
        const CellGrid &g = a.cg;
        // tile centre: candidates and voxels get fp32 coordinates relative to it
        const double tcx = uniform(0.5 * (bx0 + bx1)), tcy = uniform(0.5 * (by0 + by1)), tcz = uniform(0.5 * (bz0 + bz1));
        const float qfx = (float)(qx - tcx), qfy = (float)(qy - tcy), qfz = (float)(qz - tcz);
        const f32x2 qf2x = {qfx, qfx}, qf2y = {qfy, qfy}, qf2z = {qfz, qfz};
        const double bhalf = 0.5 * sqrt_up(((bx1 - bx0) * (bx1 - bx0) + (by1 - by0) * (by1 - by0)) + (bz1 - bz0) * (bz1 - bz0));
        bool seeded = false;
#if PTV_K1_BROADCAST_SEEDS
        if constexpr (KMAX == 1) {
            if (a.cb.recs != nullptr) {
                // ---- seeds (one-slot list): the 8 corners' nearest particles (lanes 0, 8, ..., 56)
                //      broadcast to every lane; a lane's smallest distance to them bounds its nearest
                //      neighbour.  Duplicates are harmless for a minimum: no LDS hash, no barriers ----
                const uint32_t sl = __float_as_uint(seed.w);
                const bool has = sl != 0xffffffffu;
                // particle - tile centre = (particle - corner) + (corner - centre), as below
                const float ex = seed.x + (float)(scx - tcx), ey = seed.y + (float)(scy - tcy),
                            ez = seed.z + (float)(scz - tcz);
                const float pm = has ? (fabsf(ex) + fabsf(ey)) + fabsf(ez) : -1.0f;
                float best = INFINITY, pmax = -1.0f;
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const float sx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ex), c * 8));
                    const float sy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ey), c * 8));
                    const float sz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ez), c * 8));
                    const float sp = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pm), c * 8));
                    const float dx = qfx - sx, dy = qfy - sy, dz = qfz - sz;
                    const float d2 = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, dx * dx));
                    best = sp >= 0.0f ? fminf(best, d2) : best;
                    pmax = fmaxf(pmax, sp);
                }
                // seed-voxel distances are <= Ms; fp32 coordinate + distance error <= Ms * 2^-19
                const double Ms = (double)pmax * (1.0 + 1e-6) + bhalf;
                if (active && best < INFINITY) {
                    const double dl = Ms * 1.9073486328125e-06;
                    const double st2 = ((double)best * (1.0 + 9.5367431640625e-07) + (2.0 * Ms * dl + dl * dl)) * (1.0 + 1e-12);
                    if (st2 < ub2) {
                        ub2 = st2;
                        ub = sqrt_up(st2);
                    }
                }
                if (__builtin_amdgcn_ballot_w64(active && !(best < INFINITY)) != 0) {
                    const double u = lattice_ub();  // no corner had a record: the lattice bound
                    if (u < ub) {
                        ub = u;
                        ub2 = u * u;
                    }
                }
                seeded = true;
                thr = dmin(kth2(), ub2);
                stamp(t_seed);
            }
        } else
#endif
        if constexpr (KMAX <= 8) {
            if (a.cb.recs != nullptr) {
                // ---- seeds: the k-NN lists of the tile's 8 coarse-lattice corners.  Every lane's
                //      k-th smallest distance to their (deduplicated) union bounds its k-th
                //      neighbour distance from above, usually to within a few ulps, so the gather
                //      radius is tight and one pass is exact. ----
                // deduplicate through an LDS hash table (the candidate buffer, unused yet): every
                // lane writes its id at its slot's hash and keeps the slot if its own id is read
                // back.  Equal slots -> one survivor; distinct slots that collide -> one survivor
                // too, which only drops a seed: any subset of k distinct particles still bounds.
                uint32_t *tab = reinterpret_cast<uint32_t *>(buf);
                const uint32_t sl = __float_as_uint(seed.w);
                const bool has = sl != 0xffffffffu;
                // 1024 entries = the 4 KB buffer (512 in a smaller one-slot buffer)
                const uint32_t hsh = (sl * 2654435761u) >> (kCap >= 128 ? 22 : 23);
                if (has) tab[hsh] = (uint32_t)lane;
                wave_lds_sync();
                const bool uniq = has && tab[hsh] == (uint32_t)lane;
                const unsigned long long um = __builtin_amdgcn_ballot_w64(uniq);
                const int nu = __builtin_popcountll(um);
                const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(um >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)um, 0u));
                double pm = 0.0;
                if (uniq) {
                    // particle - tile centre = (particle - corner) + (corner - centre): three fp32
                    // roundings of magnitude <= Ms (covered by dl below)
                    const float ex = seed.x + (float)(scx - tcx), ey = seed.y + (float)(scy - tcy),
                                ez = seed.z + (float)(scz - tcz);
                    fbx[pos] = ex;
                    fby[pos] = ey;
                    fbz[pos] = ez;
                    // >= the Euclidean distance to the centre (fp32 sum rounded up)
                    pm = ((double)fabsf(ex) + (double)fabsf(ey) + (double)fabsf(ez)) * (1.0 + 1e-6);
                }
                // seed-voxel distances are <= Ms; fp32 coordinate + distance error <= Ms * 2^-19
                const double Ms = uniform(wave_max(pm)) + bhalf;
                wave_lds_sync();
                float sd[KMAX];
#pragma unroll
                for (int q = 0; q < KMAX; ++q) sd[q] = INFINITY;
                PTV_UNROLL(PTV_SEED_UNROLL)
                for (int i = 0; i < nu; i += 2) {
                    const float2 X = *reinterpret_cast<const float2 *>(fbx + i);
                    const float2 Y = *reinterpret_cast<const float2 *>(fby + i);
                    const float2 Z = *reinterpret_cast<const float2 *>(fbz + i);
                    const f32x2 ex = qf2x - f32x2{X.x, X.y}, ey = qf2y - f32x2{Y.x, Y.y}, ez = qf2z - f32x2{Z.x, Z.y};
                    f32x2 s2 = ex * ex;
                    s2 = __builtin_elementwise_fma(ey, ey, s2);
                    s2 = __builtin_elementwise_fma(ez, ez, s2);
                    const float xs[2] = {s2.x, i + 1 < nu ? s2.y : INFINITY};
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
#pragma unroll
                        for (int q = KMAX - 1; q > 0; --q) sd[q] = __builtin_amdgcn_fmed3f(sd[q - 1], sd[q], xs[u]);
                        sd[0] = fminf(sd[0], xs[u]);
                    }
                }
                float kth = sd[0];
#pragma unroll
                for (int q = 1; q < KMAX; ++q)
                    if (q == a.k - 1) kth = sd[q];
                if (active && kth < INFINITY) {
                    const double dl = Ms * 1.9073486328125e-06;
                    const double st2 = ((double)kth * (1.0 + 9.5367431640625e-07) + (2.0 * Ms * dl + dl * dl)) * (1.0 + 1e-12);
                    if (st2 < ub2) {
                        ub2 = st2;
                        ub = sqrt_up(st2);
                    }
                }
                if (__builtin_amdgcn_ballot_w64(active && !(kth < INFINITY)) != 0) {
                    // rare (fewer than k distinct seeds survived the hash): the lattice bound
                    const double u = lattice_ub();
                    if (u < ub) {
                        ub = u;
                        ub2 = u * u;
                    }
                }
                seeded = true;
                thr = dmin(kth2(), ub2);
                wave_lds_sync();  // the gather reuses the candidate buffers
                stamp(t_seed);
            }
        }
        // (the launcher gives the key-list interpolation and slot launches no seed records: the
        // union-seed code is not compiled into them, which frees its registers)
        if constexpr (KMAX > 8 && !(KEYS && (MODE == kModeInterp || MODE == kModeSlots))) {
            if (a.cb.recs != nullptr) {
                // ---- seeds (k > 8): the union of the 8 corners' k-NN lists bounds every voxel's
                //      k-th distance (measured: within 0.03 % of it in volume, the D(c) + |v - c|
                //      bound 2.2x).  8 rounds of up to 64 records (one corner per round),
                //      deduplicated through two LDS hash tables in the candidate buffer: T keeps the
                //      slot that claimed each entry, T2 the round's winning lane.  A record is kept
                //      only if its entry was free and it won the round: duplicates and collisions are
                //      dropped (any subset of distinct particles bounds).  Instead of each lane's
                //      k-th smallest seed distance (a KMAX-slot fp32 network per seed: 40 % of the
                //      k = 50 kernel), every lane counts the seeds within 8 radii spread over
                //      [max_c D(c) - |v - c|, min_c D(c) + |v - c|] and takes the smallest radius
                //      that holds k of them (2 VALU per seed and radius). ----
                uint32_t *T = reinterpret_cast<uint32_t *>(buf);
                uint32_t *T2 = T + 512;
#pragma unroll
                for (int i = 0; i < 8; ++i) T[i * 64 + lane] = 0xffffffffu;
                const int jx0 = __builtin_amdgcn_readfirstlane(cx >> kLatticeShift);
                const int jy0 = __builtin_amdgcn_readfirstlane(cy >> kLatticeShift);
                const int jz0 = __builtin_amdgcn_readfirstlane((cz - a.lz0) >> kLatticeShift);
                // the lane's bracket [lo, hi] of its k-th distance, and Ms >= |seed - tile centre|
                // for every seed (the corner lists lie within D(c) of their corner)
                double lo = 0.0, hi = INFINITY, msc = 0.0;
                // corner - tile centre in fp32 per axis (the corners take 2 values on each axis;
                // rounding covered by dl)
                float ox0 = 0.f, ox1 = 0.f, oy0 = 0.f, oy1 = 0.f, oz0 = 0.f, oz1 = 0.f;  // named: an
                // array indexed by a select comes back as a scratch array
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int jx = min(jx0 + (c & 1), a.cb.n[0] - 1);
                    const int jy = min(jy0 + ((c >> 1) & 1), a.cb.n[1] - 1);
                    const int jz = min(jz0 + (c >> 2), a.cb.n[2] - 1);
                    const double D = a.cb.dk[((size_t)jz * a.cb.n[1] + jy) * a.cb.n[0] + jx];
                    const double ex = qx - a.cb.ax[jx], ey = qy - a.cb.ay[jy], ez = qz - a.cb.az[jz];
                    const double e = sqrt((ex * ex + ey * ey) + ez * ez);
                    lo = fmax(lo, D - e);
                    hi = fmin(hi, D + e);
                    const double fx = a.cb.ax[jx] - tcx, fy = a.cb.ay[jy] - tcy, fz = a.cb.az[jz] - tcz;
                    msc = fmax(msc, D + fabs(fx) + fabs(fy) + fabs(fz));
                    if (c == 0) {
                        ox0 = (float)fx;
                        oy0 = (float)fy;
                        oz0 = (float)fz;
                    }
                    if (c == 1) ox1 = (float)fx;
                    if (c == 2) oy1 = (float)fy;
                    if (c == 4) oz1 = (float)fz;
                }
                const double Ms = uniform(msc) * (1.0 + 1e-6) + bhalf;
                // fp32 seed-voxel distance error: coordinates within Ms of the centre (see the k <= 8 path)
                const double dl = Ms * 1.9073486328125e-06;
                const double err = (2.0 * Ms * dl + dl * dl) * (1.0 + 1e-12);
                const bool bracket = active && hi < INFINITY && lo < hi;
                double rt[8];   // the radii
                float tf[8];    // a seed counts at radius i when its fp32 d2 <= tf[i] (it is then within rt[i])
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    rt[i] = bracket ? lo + (hi - lo) * (double)(i + 1) * 0.125 : 0.0;
                    const double t2 = (rt[i] * rt[i]) * (1.0 - 1e-12) - err;
                    // (1 - 2^-19) covers the fp32 distance's relative error (2^-20, as below) and the
                    // rounding of this conversion
                    tf[i] = bracket && t2 > 0.0 ? (float)(t2 * (1.0 - 1.9073486328125e-06)) : -1.0f;
                }
                int cnt[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) cnt[i] = 0;
                int nb = 0;
                auto count = [&]() __attribute__((always_inline)) {
#if PTV_STAMP_SEEDSPLIT
                    stamp(t_seed);  // dev stamp builds: the counting passes go to 'setup'
#endif
                    wave_lds_sync();
                    for (int i = 0; i < nb; i += 2) {
                        const float2 X = *reinterpret_cast<const float2 *>(fbx + i);
                        const float2 Y = *reinterpret_cast<const float2 *>(fby + i);
                        const float2 Z = *reinterpret_cast<const float2 *>(fbz + i);
                        const f32x2 ex = qf2x - f32x2{X.x, X.y}, ey = qf2y - f32x2{Y.x, Y.y}, ez = qf2z - f32x2{Z.x, Z.y};
                        f32x2 s2 = ex * ex;
                        s2 = __builtin_elementwise_fma(ey, ey, s2);
                        s2 = __builtin_elementwise_fma(ez, ez, s2);
                        const float xs[2] = {s2.x, i + 1 < nb ? s2.y : INFINITY};
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) cnt[r] += xs[u] <= tf[r] ? 1 : 0;
                        }
                    }
                    nb = 0;
                    wave_lds_sync();
#if PTV_STAMP_SEEDSPLIT
                    stamp(t_setup);
#endif
                };
                const int ks = a.seed_n;
                // rounds t = 0 .. 8 * rpc - 1 of up to 64 records (corner t / rpc, entries from
                // (t % rpc) * 64); each round's records are loaded one round ahead
                const int rpc = (ks + 63) >> 6;
                const int nrounds = 8 * rpc;
                const float4 none = make_float4(0.f, 0.f, 0.f, __uint_as_float(0xffffffffu));
                auto load_round = [&](int t) -> float4 {
                    const int c = t / rpc, e = (t - c * rpc) * 64 + lane;
                    const int jx = min(jx0 + (c & 1), a.cb.n[0] - 1);
                    const int jy = min(jy0 + ((c >> 1) & 1), a.cb.n[1] - 1);
                    const int jz = min(jz0 + (c >> 2), a.cb.n[2] - 1);
                    const size_t base = (((size_t)jz * a.cb.n[1] + jy) * a.cb.n[0] + jx) * a.k;
                    return e < ks ? a.cb.recs[base + e] : none;
                };
                float4 recn = load_round(0);  // nrounds >= 8
                for (int t = 0; t < nrounds; ++t) {
                    const float4 rec = recn;
                    recn = load_round(min(t + 1, nrounds - 1));  // the last round reloads its own
                    const int c = t / rpc;
                    const float ocx = (c & 1) ? ox1 : ox0, ocy = (c & 2) ? oy1 : oy0, ocz = (c & 4) ? oz1 : oz0;
                    {
                        const uint32_t sl = __float_as_uint(rec.w);
                        const uint32_t h = (sl * 2654435761u) >> 23;  // 512 entries
                        wave_lds_sync();                               // the previous round's claims
                        const bool freeh = sl != 0xffffffffu && T[h] == 0xffffffffu;
                        const uint32_t tag = (uint32_t)((t << 6) + lane);
                        if (freeh) T2[h] = tag;
                        wave_lds_sync();
                        const bool win = freeh && T2[h] == tag;
                        if (win) T[h] = sl;
                        const unsigned long long wm = __builtin_amdgcn_ballot_w64(win);
                        if (win) {
                            const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(wm >> 32),
                                                                                __builtin_amdgcn_mbcnt_lo((unsigned)wm, 0u));
                            fbx[pos] = rec.x + ocx;
                            fby[pos] = rec.y + ocy;
                            fbz[pos] = rec.z + ocz;
                        }
                        nb += __builtin_popcountll(wm);
                        if (nb > kCap - 64) count();
                    }
                }
                if (nb > 0) count();
                // the smallest radius holding k distinct seeds
                double rsel = INFINITY;
#pragma unroll
                for (int i = 7; i >= 0; --i)
                    if (cnt[i] >= a.k) rsel = rt[i];
                if (active && rsel < INFINITY) {
                    const double st2 = rsel * rsel * (1.0 + 1e-12);
                    if (st2 < ub2) {
                        ub2 = st2;
                        ub = sqrt_up(st2);
                    }
                }
                if (__builtin_amdgcn_ballot_w64(active && !(rsel < INFINITY)) != 0) {
                    const double u = lattice_ub();  // no radius held k seeds: the lattice bound
                    if (u < ub) {
                        ub = u;
                        ub2 = u * u;
                    }
                }
                seeded = true;
                thr = dmin(kth2(), ub2);
                wave_lds_sync();  // the gather reuses the candidate buffers
                stamp(t_seed);
            }
        }
        if constexpr (MODE == kModeFilter) {
            // ---- seeds (outlier filter, filtering.py:26): the tile's queries are the 64 distinct
            //      particles of one Morton blob; with the blobs before and after it (the tiles g - 1
            //      and g + 1 of the query layout, ptv_filter.hip pos_of) every lane's k-th (= k + 1
            //      of the filter) smallest distance to those <= 192 particles bounds its own k-th
            //      neighbour distance.  A blob's edge lanes see few of their neighbours in the blob
            //      alone: measured offline on the sphere pack (1M particles, k + 1 = 26) the bound is
            //      1.66x the true distance on average with the blob, 1.22x with its two neighbours,
            //      and the worst lane of a wave (which sets the wave's insertion rounds) 6x (volume)
            //      instead of 237x.  The padding queries (q_orig ~0) are left out. ----
            const long long ntile = ((long long)a.nx * a.ny * a.nz) >> 6;
            const long long g = (long long)tz * a.ntx + tx;  // this tile = Morton blob g
            auto qpos = [&](long long gt) -> size_t {
                const long long gz = gt / a.ntx, gx = gt - gz * a.ntx;
                return ((size_t)(gz * 4 + (lane >> 4)) * a.ny + ((lane >> 2) & 3)) * a.nx + gx * 4 + (lane & 3);
            };
            float nx_[2], ny_[2], nz_[2];
            bool nreal[2];
            double pmn = 0.0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const long long gn = g + (h ? 1 : -1);
                nreal[h] = false;
                nx_[h] = ny_[h] = nz_[h] = 0.f;
                if (gn >= 0 && gn < ntile) {
                    const size_t pn = qpos(gn);
                    if (a.fe.q_orig[pn] != 0xffffffffu) {
                        nreal[h] = true;
                        nx_[h] = (float)(qpx[pn] - tcx);
                        ny_[h] = (float)(qpy[pn] - tcy);
                        nz_[h] = (float)(qpz[pn] - tcz);
                        pmn = fmax(pmn, ((double)fabsf(nx_[h]) + (double)fabsf(ny_[h]) + (double)fabsf(nz_[h])) * (1.0 + 1e-6));
                    }
                }
            }
            const bool realq = active && a.fe.q_orig[vfull] != 0xffffffffu;
            // |fp32 coordinate - exact| <= |p - centre| 2^-24 per axis: the seed-voxel distances are
            // within Ms (the farthest seed plus the farthest voxel from the centre), their fp32
            // error within Ms * 2^-19 overall
            const double pmq = realq ? ((double)fabsf(qfx) + (double)fabsf(qfy) + (double)fabsf(qfz)) * (1.0 + 1e-6) : 0.0;
            const double Ms = uniform(wave_max(fmax(pmq, pmn))) + uniform(wave_max(pmq)) + bhalf;
            float sd[KMAX];
#pragma unroll
            for (int q = 0; q < KMAX; ++q) sd[q] = INFINITY;
            // two rounds through the candidate buffer (kCap = 128 entries): this blob and the one
            // before it, then the one after it
#pragma unroll
            for (int round = 0; round < 2; ++round) {
                int nu = 0;
                auto put = [&](bool has, float x, float y, float z) {
                    const unsigned long long m = __builtin_amdgcn_ballot_w64(has);
                    if (has) {
                        const int pos = nu + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                            __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                        fbx[pos] = x;
                        fby[pos] = y;
                        fbz[pos] = z;
                    }
                    nu += __builtin_popcountll(m);
                };
                if (round == 0) {
                    put(realq, qfx, qfy, qfz);
                    put(nreal[0], nx_[0], ny_[0], nz_[0]);
                } else {
                    put(nreal[1], nx_[1], ny_[1], nz_[1]);
                }
                wave_lds_sync();
                PTV_UNROLL(PTV_SEED_UNROLL_FILTER)
                for (int i = 0; i < nu; i += 2) {
                    const float2 X = *reinterpret_cast<const float2 *>(fbx + i);
                    const float2 Y = *reinterpret_cast<const float2 *>(fby + i);
                    const float2 Z = *reinterpret_cast<const float2 *>(fbz + i);
                    const f32x2 ex = qf2x - f32x2{X.x, X.y}, ey = qf2y - f32x2{Y.x, Y.y}, ez = qf2z - f32x2{Z.x, Z.y};
                    f32x2 s2 = ex * ex;
                    s2 = __builtin_elementwise_fma(ey, ey, s2);
                    s2 = __builtin_elementwise_fma(ez, ez, s2);
                    const float xs[2] = {s2.x, i + 1 < nu ? s2.y : INFINITY};
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
#pragma unroll
                        for (int q = KMAX - 1; q > 0; --q) sd[q] = __builtin_amdgcn_fmed3f(sd[q - 1], sd[q], xs[u]);
                        sd[0] = fminf(sd[0], xs[u]);
                    }
                }
                wave_lds_sync();  // the buffer is refilled next
            }
            float kth = sd[0];
#pragma unroll
            for (int q = 1; q < KMAX; ++q)
                if (q == a.k - 1) kth = sd[q];
            if (active && kth < INFINITY) {
                const double dl = Ms * 1.9073486328125e-06;
                const double st2 = ((double)kth * (1.0 + 9.5367431640625e-07) + (2.0 * Ms * dl + dl * dl)) * (1.0 + 1e-12);
                if (st2 < ub2) {
                    ub2 = st2;
                    ub = sqrt_up(st2);
                }
            }
            // the per-lane bounds prune candidates; the gather radius starts at the density radius
            // (PTV_FILTER_SEEDED = 1: one pass at the wave's largest bound)
            seeded = PTV_FILTER_SEEDED != 0;
            thr = dmin(kth2(), ub2);
            stamp(t_seed);
        }
        double cpass = 0.0;
        float thrf = 0.f;
        double Rp = -1.0;  // radius already gathered (none yet)
        // R_ub covers every lane's k-th neighbour: small (fluid) -> try r0 first and then
        // the exact max k-th distance; large (void) -> one pass at R_ub.
        const double R_ub = uniform(wave_max(active ? ub : -INFINITY));
        double R = a.r0;
        // a tight lattice bound (fine level) is used directly in one pass; a loose one
        // (coarse level) is preceded by a pass at the density radius r0.
        if (R_ub < INFINITY) R = (seeded || R_ub <= 2.0 * a.r0) ? R_ub : a.r0;
        if constexpr (MODE == kModeRadius) R = a.radius;  // one pass
        if (nparts > 1) {
            // split lattice tile: one pass at the bound, which covers every lane's k nearest, so the
            // merged lists are exact; without a bound the first part searches alone
            if (R_ub < INFINITY) {
                R = R_ub;
            } else {
                if (part != 0) return;  // its list stays empty (the launcher cleared split_out)
                nparts = 1;
            }
        }
        // ---- sub-balls: the tile's 8 sub-boxes of 2x2x2 voxels (lanes differing in bits 0, 2, 4),
        //      each with centre c_s and radius max_v sqrt(thr_v) + |v - c_s|: a candidate outside
        //      every sub-ball can never enter any list (thresholds only shrink), so the copy drops it.
        //      fp32 on tile-relative coordinates, inflated for round-off (any over-estimate is safe).
        float sbx[2], sby[2], sbz[2], sbr2[8];  // sub-box s spans x-half s&1, y-half s>>1&1, z-half s>>2
        float sb_hd;                              // this lane's sub-box half-diagonal (rounded up)
        {
            // extent of this lane's x-half (lanes agreeing in bit 1), y-half (bit 3), z-half (bit 5)
            const float mnx = group_reduce<0x3d>(qfx, OpMin{}), mxx = group_reduce<0x3d>(qfx, OpMax{});
            const float mny = group_reduce<0x37>(qfy, OpMin{}), mxy = group_reduce<0x37>(qfy, OpMax{});
            const float mnz = group_reduce<0x1f>(qfz, OpMin{}), mxz = group_reduce<0x1f>(qfz, OpMax{});
            const float ux = mxx - mnx, uy = mxy - mny, uz = mxz - mnz;
            sb_hd = 0.5f * sqrtf_up(__fmaf_rn(uz, uz, __fmaf_rn(uy, uy, ux * ux)) * 1.000001f) * 1.00001f;
            const float cxs = 0.5f * (mnx + mxx), cys = 0.5f * (mny + mxy), czs = 0.5f * (mnz + mxz);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                sbx[h] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cxs), h << 1));
                sby[h] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cys), h << 3));
                sbz[h] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(czs), h << 5));
            }
        }
        double Mpass = 0.0;  // bound on |coordinate - tile centre| of this pass's candidates
        auto subballs = [&]() {
            // radius of sub-ball s: max over its 8 lanes of sqrt(thr) + the half-diagonal
            float rv = thr < 0.0 ? -1.0f : sqrtf_up((float)(thr * (1.0 + 2.384185791015625e-07)));
            rv = group_reduce<0x15>(rv, OpMax{});
            const float Rs = (rv + sb_hd) * 1.00001f + (float)(Mpass * 1e-6);
            const float R2s = rv < 0.0f ? -1.0f : Rs * Rs;
#pragma unroll
            for (int sb = 0; sb < 8; ++sb) {
                const int L = ((sb & 1) << 1) | ((sb & 2) << 2) | ((sb & 4) << 3);
                sbr2[sb] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R2s), L));
            }
        };
        int nbuf = 0;  // compacted candidates waiting in this wave's LDS buffer (uniform)
        // ---- every buffered candidate against all 64 voxels, in groups of 32 candidates:
        //      (1) a branch-free fp32 stream on tile-relative coordinates leaves each lane a bit
        //          mask of the candidates that may beat its threshold;
        //      (2) each lane then walks its own bits in candidate order: exact fp64 d2 and the
        //          insertion network.  The wave runs (2) max-over-lanes-popcount times instead of
        //          once per candidate any lane accepts. ----
        auto flush = [&]() {
            if (nbuf == 0) return;
            wave_lds_sync();
            for (int g0 = 0; g0 < nbuf; g0 += 64) {
                const int ng = min(64, nbuf - g0);
                // candidate g0 + j ends at bit nb - 1 - j (shift-in order keeps the loop rolled)
                const int nb = (ng + 3) & ~3;
                auto mask4 = [&](int i0) -> uint32_t {
                    // 4 candidates as two packed-fp32 pairs (v_pk_add / v_pk_mul / v_pk_fma);
                    // slots past nbuf hold stale values, their bits are cleared below
                    const float4 X = *reinterpret_cast<const float4 *>(fbx + g0 + i0);
                    const float4 Y = *reinterpret_cast<const float4 *>(fby + g0 + i0);
                    const float4 Z = *reinterpret_cast<const float4 *>(fbz + g0 + i0);
                    const f32x2 e0x = qf2x - f32x2{X.x, X.y}, e1x = qf2x - f32x2{X.z, X.w};
                    const f32x2 e0y = qf2y - f32x2{Y.x, Y.y}, e1y = qf2y - f32x2{Y.z, Y.w};
                    const f32x2 e0z = qf2z - f32x2{Z.x, Z.y}, e1z = qf2z - f32x2{Z.z, Z.w};
                    f32x2 s0 = e0x * e0x, s1 = e1x * e1x;
                    s0 = __builtin_elementwise_fma(e0y, e0y, s0);
                    s1 = __builtin_elementwise_fma(e1y, e1y, s1);
                    s0 = __builtin_elementwise_fma(e0z, e0z, s0);
                    s1 = __builtin_elementwise_fma(e1z, e1z, s1);
                    return ((s0.x <= thrf) ? 8u : 0u) | ((s0.y <= thrf) ? 4u : 0u) |
                           ((s1.x <= thrf) ? 2u : 0u) | ((s1.y <= thrf) ? 1u : 0u);
                };
                auto group_mask = [&]() -> unsigned long long {
                    unsigned long long m = 0ull;
                    if constexpr (MODE == kModeFilter) {
                        // unrolled by 2 for the filter's long candidate streams (search 19.35 ->
                        // 19.14 ms); rolled elsewhere (the headline +0.7 % unrolled)
                        PTV_UNROLL(PTV_MASK_UNROLL_FILTER)
                        for (int i0 = 0; i0 < ng; i0 += 4) m = (m << 4) | mask4(i0);
                    } else {
                        PTV_UNROLL(PTV_MASK_UNROLL)
                        for (int i0 = 0; i0 < ng; i0 += 4) m = (m << 4) | mask4(i0);
                    }
                    return m & ~((1ull << (nb - ng)) - 1ull);  // stale slots past nbuf
                };
                unsigned long long m = group_mask();
                const double4 *gbuf = buf + g0 + nb - 64;  // bit position p <-> gbuf[63 - p]
                int nit = __builtin_amdgcn_readfirstlane(wave_max_i(__builtin_popcountll(m)));
                if constexpr ((MODE == kModeKDist && !KEYS) || (KEYS && tighten_keys<MODE>())) {
                    // lattice levels start from the coarse bound (no seeds): a lane whose list is not
                    // full yet takes every candidate under it.  When some lane would insert more than
                    // kTightenMin of this group, first each lane's k-th smallest fp32 d2 over its list
                    // and the group (fmed3 network; list entries rounded up, the group's within cpass):
                    // an upper bound on the k-th of the two, so the insertions keep to the candidates
                    // that can stay in the list (the lists come out the same).  Key lists (the outlier
                    // filter, whose seeds are only its Morton blob): an entry's key times kscale bounds
                    // its exact d2, the k-th sits at KMAX - 2, and the bound is widened by kscale so
                    // that every candidate sharing the final k-th key's truncation still reaches the
                    // (k+1)-th slot (the near-tie check); a candidate past it cannot be the (k+1)-th
                    // key's near tie either.
                    if (nit > kTightenMin) {
                        constexpr int KT = KEYS ? KMAX - 2 : KMAX - 1;  // the k-th entry
                        const double ks = KEYS ? a.kscale : 1.0;
                        float sd[KMAX];
#pragma unroll
                        for (int j = 0; j < KMAX; ++j)
                            sd[j] = bd[j] < 0.0 ? -1.0f
                                                : (bd[j] < INFINITY ? (float)(bd[j] * ks * (1.0 + 2.384185791015625e-07)) : INFINITY);
                        for (int i = 0; i < ng; i += 2) {
                            const float2 X = *reinterpret_cast<const float2 *>(fbx + g0 + i);
                            const float2 Y = *reinterpret_cast<const float2 *>(fby + g0 + i);
                            const float2 Z = *reinterpret_cast<const float2 *>(fbz + g0 + i);
                            const f32x2 ex = qf2x - f32x2{X.x, X.y}, ey = qf2y - f32x2{Y.x, Y.y}, ez = qf2z - f32x2{Z.x, Z.y};
                            f32x2 s2 = ex * ex;
                            s2 = __builtin_elementwise_fma(ey, ey, s2);
                            s2 = __builtin_elementwise_fma(ez, ez, s2);
                            const float xs[2] = {s2.x, i + 1 < ng ? s2.y : INFINITY};
#pragma unroll
                            for (int u = 0; u < 2; ++u) {
#pragma unroll
                                for (int q = KMAX - 1; q > 0; --q) sd[q] = __builtin_amdgcn_fmed3f(sd[q - 1], sd[q], xs[u]);
                                sd[0] = fminf(sd[0], xs[u]);
                            }
                        }
                        if (active && sd[KT] >= 0.0f && sd[KT] < INFINITY) {
                            const double t = ((double)sd[KT] * (1.0 + 9.5367431640625e-07) + cpass) * ks * (1.0 + 1e-12);
                            if (t < thr) {
                                thr = t;
                                thrf = f32_bound(thr, cpass);
                            }
                        }
                        m = group_mask();
                        nit = __builtin_amdgcn_readfirstlane(wave_max_i(__builtin_popcountll(m)));
                    }
                }
                if constexpr (KEYS && MODE != kModeRadius) {
                    // key lists: NB candidates per lane at a time into one merge network
                    // (insert_keys); iterations past nit find m = 0 everywhere (+inf keys).
                    // No exact threshold test: a key past the list's end drops out, and every
                    // candidate sharing the k-th key's truncation reaches the (k+1)-th slot
                    // (the near-tie check)
                    constexpr int NB = key_batch<KMAX>();
                    for (int it = 0; it < nit; it += NB) {
                        n_acc += (uint32_t)min(NB, nit - it);
                        double nk[NB];
#pragma unroll
                        for (int j = 0; j < NB; ++j) {
                            const bool has = m != 0ull;
                            const int lz = __builtin_clzll(m | 1ull);
                            m &= ~(0x8000000000000000ull >> lz);
                            const double4 c = gbuf[lz];
                            const double dx = qx - c.x, dy = qy - c.y, dz = qz - c.z;
                            const double e2 = (dx * dx + dy * dy) + dz * dz;
                            nk[j] = make_key(has, e2, (uint32_t)__double_as_longlong(c.w), a.smask);
                        }
                        insert_keys<KMAX, NB>(bd, nk);
                    }
                } else for (int it = 0; it < nit; ++it) {
                    // branch-free body (lanes without bits read a valid stale slot and insert inf)
                    ++n_acc;
                    const bool has = m != 0ull;
                    const int lz = __builtin_clzll(m | 1ull);
                    m &= ~(0x8000000000000000ull >> lz);
                    const double4 c = gbuf[lz];
                    const double dx = qx - c.x, dy = qy - c.y, dz = qz - c.z;
                    const double e2 = (dx * dx + dy * dy) + dz * dz;
                    if constexpr (MODE == kModeRadius) {
                        // IDW term of a particle inside the ball (cKDTree's d2 <= r*r test)
                        if (has && active && e2 <= rad2) {
                            const double4 val = lds_val[wid][gbuf - buf + lz];
                            const double w = 1.0 / (np_pow(sqrt_cr(e2), a.power) + a.eps);
                            rs += w;
                            rsu += w * val.x;
                            rsv += w * val.y;
                            rsw += w * val.z;
                        }
                    } else if constexpr (!KEYS) {
                        const double d2 = (has && e2 < thr) ? e2 : INFINITY;
                        insert<KMAX>(bd, bp, d2, (int)__double_as_longlong(c.w));  // no-op where d2 = inf
                        thr = dmin(bd[KMAX - 1], ub2);
                    }
                }
                if constexpr (KEYS) thr = dmin(thr, kth2());  // thresholds only shrink (a tightened one stays)
                thrf = f32_bound(thr, cpass);
            }
            n_surv += (uint32_t)nbuf;
            nbuf = 0;
            wave_lds_sync();  // the buffer is refilled next
            subballs();
            stamp(t_comp);
        };
        int py0 = 1, py1 = 0, pz0 = 1, pz1 = 0;  // row box of the previous pass (empty)
        while (true) {
            ++n_pass;
            const double Rg = R + g.mg, Rg2 = Rg * Rg;
            {
                // |fp32 - exact| distance error <= delta = M * 2^-21 for coordinates within M of the
                // tile centre; (s + delta)^2 <= s^2 + 2 M delta + delta^2 bounds the test.
                const double M = Rg + 2.0 * bhalf + 2.0 * fmax(g.cs[0], fmax(g.cs[1], g.cs[2]));
                const double delta = M * 4.76837158203125e-07;
                cpass = 2.0 * M * delta + delta * delta;
                thrf = f32_bound(thr, cpass);
                Mpass = M;
                subballs();
            }
            const double Rpg2 = Rp < 0.0 ? -1.0 : (Rp + g.mg) * (Rp + g.mg);
            const int ry0 = clampi(floor((by0 - Rg - g.o[1]) * g.ic[1]), g.nc[1]);
            const int ry1 = clampi(floor((by1 + Rg - g.o[1]) * g.ic[1]), g.nc[1]);
            const int rz0 = clampi(floor((bz0 - Rg - g.o[2]) * g.ic[2]), g.nc[2]);
            const int rz1 = clampi(floor((bz1 + Rg - g.o[2]) * g.ic[2]), g.nc[2]);
            // rows are visited centre-out (zigzag in y within zigzag in z around the tile's
            // cell) so that near candidates come first and the k-th distances tighten early
            const int cyc = clampi(floor((tcy - g.o[1]) * g.ic[1]), g.nc[1]);
            const int czc = clampi(floor((tcz - g.o[2]) * g.ic[2]), g.nc[2]);
            const int hy = max(cyc - ry0, ry1 - cyc), hz = max(czc - rz0, rz1 - czc);
            const int nyr = 2 * hy + 1;
            const int nrows = nyr * (2 * hz + 1);
            const float inv_nyr = 1.0f / (float)nyr;
            // this wave's rows: every one, or (split lattice launch) every nparts-th from its part, still
            // centre-out.  Each part clips its runs to its own sub-balls: a candidate outside them is
            // farther from every lane than the part's k-th, which bounds the merged k-th from above
            const int nrp = (nrows - part + nparts - 1) / nparts;
            for (int rb = 0; rb < nrp; rb += 64 * kRowsPerLane) {
                ++n_round;
                // ---- lane = kRowsPerLane cell rows: x-runs of this shell -> particle ranges ----
                uint32_t rs[2 * kRowsPerLane];
                int rc[2 * kRowsPerLane];
#pragma unroll
                for (int q = 0; q < kRowsPerLane; ++q) {
                    const int row = part + nparts * (rb + q * 64 + lane);
                    rs[2 * q] = rs[2 * q + 1] = 0;
                    rc[2 * q] = rc[2 * q + 1] = 0;
                    if (row < nrows) {
                        int rq = (int)((float)row * inv_nyr);  // row / nyr without an integer divide
                        rq -= (rq * nyr > row) ? 1 : 0;
                        rq += ((rq + 1) * nyr <= row) ? 1 : 0;
                        const int ty = row - rq * nyr;
                        const int ccy = cyc + ((ty & 1) ? ((ty + 1) >> 1) : -(ty >> 1));
                        const int ccz = czc + ((rq & 1) ? ((rq + 1) >> 1) : -(rq >> 1));
                        const double gy = axis_gap(ccy, g.o[1], g.cs[1], by0, by1);
                        const double gz = axis_gap(ccz, g.o[2], g.cs[2], bz0, bz1);
                        const double h2 = gy * gy + gz * gz;
                        if (h2 <= Rg2 && ccy >= ry0 && ccy <= ry1 && ccz >= rz0 && ccz <= rz1) {
                            const double rx = sqrt_up(Rg2 - h2);
                            const int a1 = clampi(floor((bx0 - rx - g.o[0]) * g.ic[0]), g.nc[0]);
                            const int b1 = clampi(floor((bx1 + rx - g.o[0]) * g.ic[0]), g.nc[0]);
                            int lo1 = a1, hi1 = b1, lo2 = 1, hi2 = 0;  // [lo, hi] inclusive runs
                            if (h2 <= Rpg2 && ccy >= py0 && ccy <= py1 && ccz >= pz0 && ccz <= pz1) {
                                // row was gathered by the previous pass: only the x extensions are new
                                const double rxo = sqrt_up(Rpg2 - h2);
                                const int a0 = clampi(floor((bx0 - rxo - g.o[0]) * g.ic[0]), g.nc[0]);
                                const int b0 = clampi(floor((bx1 + rxo - g.o[0]) * g.ic[0]), g.nc[0]);
                                hi1 = a0 - 1;
                                lo2 = b0 + 1;
                                hi2 = b1;
                            }
                            // both runs' bounds in flight together (an empty run reads cell 0 twice)
#if PTV_SUBBALL_RUNS
                            {
                                // clip the runs to the union of the 8 sub-balls' chords of this row: a
                                // particle that can enter any list lies in some sub-ball (the copy filter
                                // below), so cells outside every chord are never needed.  fp32 on
                                // tile-relative coordinates, every rounding widened (em).
                                const float em = (float)(Mpass * 1e-6) + 1e-6f;
                                const float ylo = (float)(g.o[1] + (double)ccy * g.cs[1] - tcy) - em;
                                const float yhi = (float)(g.o[1] + (double)(ccy + 1) * g.cs[1] - tcy) + em;
                                const float zlo = (float)(g.o[2] + (double)ccz * g.cs[2] - tcz) - em;
                                const float zhi = (float)(g.o[2] + (double)(ccz + 1) * g.cs[2] - tcz) + em;
                                float xl = INFINITY, xh = -INFINITY;
#pragma unroll
                                for (int sb = 0; sb < 8; ++sb) {
                                    const float cyv = sby[(sb >> 1) & 1], czv = sbz[sb >> 2];
                                    const float gy = fmaxf(fmaxf(ylo - cyv, cyv - yhi), 0.f);
                                    const float gz = fmaxf(fmaxf(zlo - czv, czv - zhi), 0.f);
                                    const float h2s = __fmaf_rn(gz, gz, gy * gy);
                                    if (h2s <= sbr2[sb]) {
                                        const float hw = sqrtf_up(fmaxf(sbr2[sb] - h2s, 0.f) + sbr2[sb] * 1e-6f);
                                        xl = fminf(xl, sbx[sb & 1] - hw);
                                        xh = fmaxf(xh, sbx[sb & 1] + hw);
                                    }
                                }
                                if (xl <= xh) {
                                    const int s0 = clampi(floor((tcx + (double)(xl - em) - g.o[0]) * g.ic[0]), g.nc[0]);
                                    const int s1 = clampi(floor((tcx + (double)(xh + em) - g.o[0]) * g.ic[0]), g.nc[0]);
                                    lo1 = max(lo1, s0);
                                    hi1 = min(hi1, s1);
                                    lo2 = max(lo2, s0);
                                    hi2 = min(hi2, s1);
                                } else {
                                    hi1 = lo1 - 1;
                                    hi2 = lo2 - 1;
                                }
                            }
#endif
                            const uint32_t *rp = cstart + ((long long)ccz * g.nc[1] + ccy) * g.nc[0];
                            const bool e1 = lo1 <= hi1, e2 = lo2 <= hi2;
                            const uint32_t s1 = rp[e1 ? lo1 : 0], t1 = rp[e1 ? hi1 + 1 : 0];
                            const uint32_t s2 = rp[e2 ? lo2 : 0], t2 = rp[e2 ? hi2 + 1 : 0];
                            rs[2 * q] = s1;
                            rc[2 * q] = (int)(t1 - s1);
                            rs[2 * q + 1] = s2;
                            rc[2 * q + 1] = (int)(t2 - s2);
                            ++n_rows;
                        }
                    }
                }
                int cnt = 0;
#pragma unroll
                for (int r = 0; r < 2 * kRowsPerLane; ++r) cnt += rc[r];
                const int incl = wave_incl_scan_i(cnt);
                const int off = incl - cnt;
                const int total = __builtin_amdgcn_readlane(incl, 63);
                // run table in LDS: entry lane*R+r = (first candidate index, first particle slot)
#pragma unroll
                for (int r = 0, pre = off; r < 2 * kRowsPerLane; ++r) {
                    runs[lane * 2 * kRowsPerLane + r] = make_uint2((uint32_t)pre, rs[r]);
                    pre += rc[r];
                }
                wave_lds_sync();
                stamp(t_rows);
                // ---- copy windows [src, src + 64) of this round's candidates.  Each run marks its
                //      first window position with its id (ids grow with candidate order), a prefix
                //      max gives every lane its run; lane i takes candidate src + i and keeps it
                //      only if it lies in some sub-ball (compacted into the LDS buffer).  Software
                //      pipelined: the next window's records are in flight while this one is filtered.
                auto window_slot = [&](int src) -> uint32_t {
                    owner[lane] = -1;
                    wave_lds_sync();
#pragma unroll
                    for (int r = 0, pre = off; r < 2 * kRowsPerLane; ++r) {
                        if (rc[r] > 0 && pre < src + 64 && pre + rc[r] > src)
                            owner[max(pre, src) - src] = lane * 2 * kRowsPerLane + r;
                        pre += rc[r];
                    }
                    wave_lds_sync();
                    const int o = wave_incl_max_scan_i(owner[lane]);
                    uint32_t sl = 0;  // lanes past the end read record 0 and drop it
                    if (src + lane < total) {
                        const uint2 rn = runs[o];
                        sl = rn.y + (uint32_t)(src + lane - (int)rn.x);
                    }
                    return sl;
                };
                uint32_t next_slot = total > 0 ? window_slot(0) : 0u;
                double4 next_rec = prec[next_slot];
                // the pass's last round runs at least one (possibly empty) window, so that the
                // final flush below is the loop's own (one inlined copy of the insert network)
                const bool last_round = rb + 64 * kRowsPerLane >= nrp;
                const int tot_it = (total == 0 && last_round) ? 1 : total;
                for (int src = 0; src < tot_it; src += 64) {
                    const uint32_t slot = next_slot;
                    const double4 p4 = next_rec;
                    if (src + 64 < total) {
                        next_slot = window_slot(src + 64);
                        next_rec = prec[next_slot];
                    }
                    const int i = src + lane;
                    bool keep = false;
                    float ex = 0.f, ey = 0.f, ez = 0.f;
                    if (i < total) {
                        ex = (float)(p4.x - tcx);
                        ey = (float)(p4.y - tcy);
                        ez = (float)(p4.z - tcz);
                        float qx2[2], qy2[2], qz2[2];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const float dx = ex - sbx[h], dy = ey - sby[h], dz = ez - sbz[h];
                            qx2[h] = dx * dx;
                            qy2[h] = dy * dy;
                            qz2[h] = dz * dz;
                        }
#pragma unroll
                        for (int sb = 0; sb < 8; ++sb)
                            keep = keep || (qx2[sb & 1] + qy2[(sb >> 1) & 1]) + qz2[sb >> 2] <= sbr2[sb];
                    }
                    const unsigned long long km = __builtin_amdgcn_ballot_w64(keep);
                    if (keep) {
                        const int pos = nbuf + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km >> 32),
                                                                              __builtin_amdgcn_mbcnt_lo((unsigned)km, 0u));
                        buf[pos] = make_double4(p4.x, p4.y, p4.z, __longlong_as_double((long long)slot));
                        if constexpr (MODE == kModeRadius) lds_val[wid][pos] = pval[slot];
                        fbx[pos] = ex;
                        fby[pos] = ey;
                        fbz[pos] = ez;
                    }
                    nbuf += __builtin_popcountll(km);
                    n_cand += (uint32_t)min(64, total - src);
                    stamp(t_copy);
                    if (nbuf > kCap - 64 || (last_round && src + 64 >= tot_it)) flush();
                }
            }
            // ---- exactness: lanes with k-th distance <= R are final ----
            // (key lists: the key bound covers every candidate sharing the k-th key's truncation,
            // so the (k+1)-th slot sees them all too)
            const double worst = uniform(wave_max(kth2()));  // inactive lanes hold -1
            if (MODE == kModeRadius || worst <= R * R || R >= a.rall || nparts > 1) break;
            Rp = R;
            py0 = ry0;
            py1 = ry1;
            pz0 = rz0;
            pz1 = rz1;
            if (worst < INFINITY) {
                R = sqrt(worst) * (1.0 + 1e-12);  // every list full: one exact pass left
            } else if (R_ub < INFINITY && R < R_ub) {
                R = R_ub;  // the coarse-lattice bound covers every lane
            } else {
                // some list not full.  Void tiles: grow geometrically while nothing has been
                // found (rows only, no candidates), then in small steps so that the last
                // shell does not overshoot the lens of particles the voxels actually need.
                bool seen = false;
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if constexpr (KEYS) seen = seen || (bd[j] >= 0.0 && bd[j] < INFINITY);
                    else seen = seen || bp[j] >= 0;
                }
                const bool any_seen = __builtin_amdgcn_ballot_w64(seen) != 0;
                R = any_seen ? R + fmax(a.r0, 0.125 * R) : 1.5 * R;
            }
            R = fmin(R, a.rall);
        }
    }
    stamp(t_setup);  // exactness checks / radius updates count as setup

    // per-wave stamp record (ptv_debug_stamps), written by the first valid lane
    auto write_stamps = [&]() {
        if constexpr (STAMP) {
            stamp(t_epi);
            const long long gw = (long long)lb * 4 + wid;
            if (dbg != nullptr && gw < dbg_cap && (threadIdx.x & 63) == (int)__builtin_ffsll((long long)__builtin_amdgcn_ballot_w64(true)) - 1) {
                unsigned long long *r = dbg + gw * kStampFields;
                r[0] = t_setup;
                r[1] = t_seed;
                r[2] = t_rows;
                r[3] = t_copy;
                r[4] = t_comp;
                r[5] = t_epi;
                r[6] = n_cand + ((unsigned long long)n_acc << 32);
                r[7] = (n_round & 0xffffu) + ((unsigned long long)(n_pass & 0xffffu) << 16) + ((unsigned long long)n_surv << 32);
            }
        }
    };
    if (!valid) return;
    const size_t vo = ((size_t)(iz - a.z0) * a.ny + iy) * a.nx + ix;
    // near-tie repair (key lists): this wave's tile goes to the exact rerun, its outputs unwritten
    auto list_tile = [&]() {
        const unsigned long long m = __builtin_amdgcn_ballot_w64(true);
        if (lane == (int)__builtin_ffsll((long long)m) - 1) {
            const unsigned int i = atomicAdd(a.rep_cnt, 1u);
            if ((int)i < a.rep_cap) a.rep_list[i] = (uint32_t)b * 4u + (uint32_t)tw;
        }
    };
    // exact d2 of slot s from this lane's query, bit-identical to the search's e2
    auto exact_d2 = [&](const double4 &c) {
        const double dx = qx - c.x, dy = qy - c.y, dz = qz - c.z;
        return (dx * dx + dy * dy) + dz * dz;
    };
    if constexpr (MODE == kModeKDist) {
        if (split_epi) {
            // split lattice tile: this part's list (slots, ~0 = none) for k_kdist_merge
            uint32_t *o = a.split_out + (size_t)(lb * 4 + wid) * KMAX * 64 + lane;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if constexpr (KEYS) o[j * 64] = (bd[j] >= 0.0 && bd[j] < INFINITY) ? key_slot(bd[j], a.smask) : 0xffffffffu;
                else o[j * 64] = bp[j] >= 0 ? (uint32_t)bp[j] : 0xffffffffu;
            }
        } else {
            kdist_out<KMAX, KEYS>(a, prec, bd, bp, qx, qy, qz, vo, U);
        }
        write_stamps();
        return;
    }
    // key lists: the k + 1 entries' slots, shifted to 0..k (kpad uniform), and the (k+1)-th
    // key's near-tie with the k-th (before the shift: compile-time slots)
    constexpr bool KSL = KEYS && MODE != kModeKDist;
    constexpr bool KSLR = KSL && !KSLI;  // slot list in registers (filter, slots modes)
    int ksl[KSLR ? KMAX : 1];
    auto ksl_word = [&](int j) -> uint32_t * {
        return j * 64 < KCW ? reinterpret_cast<uint32_t *>(lds_cand[wid]) + j * 64 + lane : &lds_kx[wid][j * 64 - KCW + lane];
    };
    bool amb = false;
    if constexpr (KSL) {
        amb = active && bd[KMAX - 1] < INFINITY && same_trunc(bd[KMAX - 2], bd[KMAX - 1], a.smask);
        if constexpr (KSLI) {
            wave_lds_sync();  // every lane is done with the candidate buffer
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                const int pos = j - a.kpad;  // shifted so that the k + 1 entries are 0 .. k
                if (pos >= 0) *ksl_word(pos) = key_slot(bd[j], a.smask);
            }
            wave_lds_sync();
        } else {
#pragma unroll
            for (int j = 0; j < KMAX; ++j) ksl[j] = (int)key_slot(bd[j], a.smask);
            if constexpr (MODE != kModeSlots) {
#pragma unroll
                for (int sh = 1; sh < KMAX; sh <<= 1) {
                    if (a.kpad & sh) {
#pragma unroll
                        for (int j = 0; j + sh < KMAX; ++j) ksl[j] = ksl[j + sh];
                    }
                }
            }
        }
    }
    // slot of list entry j (after the shift)
    auto slot_at = [&](int j) -> int {
        if constexpr (KSLI) return (int)*ksl_word(j);
        else if constexpr (KSL) return ksl[j];
        else return bp[j];
    };
    // exact d2 of the first n listed entries in ascending order (key lists), in blocks of 8
    // gathers; false where two distinct d2 sharing a truncation came out of order
    auto keys_ascend = [&](int n, double &last) -> bool {
        bool ok = true;
        double prev = -1.0;
#pragma unroll
        for (int m = 0; m < KMAX; m += 8) {
            if (m < n) {
                double4 rc[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) rc[i] = prec[m + i < KMAX && m + i < n ? slot_at(min(m + i, KMAX - 1)) : slot_at(0)];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (m + i < n) {
                        const double d2 = exact_d2(rc[i]);
                        ok = ok && !(d2 < prev);
                        prev = d2;
                    }
                }
            }
        }
        last = prev;
        return ok;
    };
    if constexpr (MODE == kModeFilter) {
        // remove_outliers_knn (filtering.py:20-51) for the query particle of this lane: its k+1
        // nearest (the list, slots kpad..KMAX-1, ascending), minus "the point itself" (column 0
        // of the reference's query: the query's own record when it is in the list, the nearest
        // otherwise), the neighbours' speeds, median and MAD, the keep test, and the (k+1)-th
        // distance (printed median, :33-35)
        const uint32_t orig = a.fe.q_orig[vfull];
        if (!active || orig == 0xffffffffu) return;
        const uint32_t qslot = a.fe.inv[orig];
        const int k1 = a.k, kk = a.k - 1;  // k1 = k + 1 listed, kk = k neighbours without the point
        double dk1;  // the (k+1)-th distance
        if constexpr (KSL) {
            double last = 0.0;
            amb = amb || !keys_ascend(k1, last);
            if (__builtin_amdgcn_ballot_w64(amb) != 0) {
                list_tile();
                return;
            }
            dk1 = sqrt(last);
        } else {
            dk1 = sqrt(bd[KMAX - 1]);
            // left-shift the list by kpad (uniform) so the k+1 entries occupy slots 0..k
#pragma unroll
            for (int sh = 1; sh < KMAX; sh <<= 1) {
                if (a.kpad & sh) {
#pragma unroll
                    for (int j = 0; j + sh < KMAX; ++j) bp[j] = bp[j + sh];
                }
            }
        }
        int drop = 0;
        double v[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (j < k1 && (uint32_t)slot_at(j) == qslot) drop = j;
            v[j] = j < k1 ? a.fe.spd[max(slot_at(j), 0)] : 0.0;  // every gather in flight together
        }
        double sp[KMAX];
#pragma unroll
        for (int t = 0; t < KMAX; ++t) sp[t] = t + 1 < KMAX ? (t < drop ? v[t] : v[t + 1]) : 0.0;
        const double med = filter_median(sp, kk);
        double dev[KMAX];
#pragma unroll
        for (int t = 0; t < KMAX; ++t) dev[t] = fabs(sp[t] - med);
        const double mad = filter_median(dev, kk);
        const double zsc = fabs(a.fe.spd[qslot] - med) / (mad + a.fe.mad_eps);
        a.fe.keep[orig] = zsc <= a.fe.threshold ? 1 : 0;
        if (a.fe.kth != nullptr) a.fe.kth[orig] = dk1;
        write_stamps();
        return;
    }
    if constexpr (MODE == kModeSlots) {
        // the k neighbour slots (list order) for the local-RBF solve (ptv_rbf.hip)
        // (order inside the k does not matter there, np.sort(yindices): only the set)
        if constexpr (KSL) {
            if (__builtin_amdgcn_ballot_w64(amb) != 0) {
                list_tile();
                return;
            }
        }
        if (!active) return;
        uint32_t *o = a.slots + vo * (size_t)a.k;
#pragma unroll
        for (int j = 0; j < KMAX - (KSL ? 1 : 0); ++j)
            if (j >= a.kpad) o[j - a.kpad] = (uint32_t)slot_at(j);
        return;
    }
    if (!active) {
        store_out(a.flags, U, V, W, vo, 0.0, 0.0, 0.0);
        return;
    }
    if constexpr (MODE == kModeRadius) {
        // sum_j w_j u_j / sum_j w_j (an empty ball gives 0 / 0 = NaN, "no data")
        double o[3] = {rsu / rs, rsv / rs, rsw / rs};
        if (a.flags & PTV_FLAG_NAN_TO_NUM) {
#pragma unroll
            for (int c = 0; c < 3; ++c) o[c] = nan_to_num(o[c]);
        }
        store_out(a.flags, U, V, W, vo, o[0], o[1], o[2]);
        return;
    }
    if constexpr (KSL && MODE == kModeInterp && KMAX <= PTV_KNN_UNROLL_MAX) {
        // up to PTV_KNN_UNROLL_MAX (56) slots: blocks unrolled at compile time (the loads of different
        // blocks overlap, measured faster than the rolled loop below: Sibson k = 30 79 vs 92 ms at 3
        // waves per SIMD, Sibson k = 50 100 vs 137 ms at 2)
        // Key lists (k >= 13): the weights are streamed in blocks of 8 neighbours from the exact
        // d2, recomputed from the records (the keys hold truncated d2), in the reference's order:
        // interpolator.py:142-153 (IDW), :102-122 (Sibson).  Register-kept distances where the
        // list is short enough, record re-gathers otherwise.
        const int k = a.k;
        constexpr bool KEEP = KMAX <= PTV_KNN_KEEP_MAX;
        double dk[KEEP ? KMAX : 1];  // Sibson: d_j, IDW: d2_j
        auto d2_block = [&](int m, double (&d2)[8]) {
            double4 rc[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) rc[i] = prec[m + i < k ? slot_at(min(m + i, KMAX - 1)) : slot_at(0)];
#pragma unroll
            for (int i = 0; i < 8; ++i) d2[i] = exact_d2(rc[i]);
        };
        // u, v, w of 8 value records straight into the product arrays (24 of the 32 bytes: 48
        // registers in flight, not 64 plus the products)
        auto val_block = [&](int m, double (&tu)[8], double (&tv)[8], double (&tw)[8]) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double *r = reinterpret_cast<const double *>(
                    pval + (m + i < k ? slot_at(min(m + i, KMAX - 1)) : slot_at(0)));
                const double2 uv = *reinterpret_cast<const double2 *>(r);
                tu[i] = uv.x;
                tv[i] = uv.y;
                tw[i] = r[2];
            }
        };
#if PTV_VALUE_HALF_BLOCKS
        // the 3-wave lists (KMAX <= 32): blocks in halves (spilled VGPRs at 24 / 32 slots: 30 / 98 ->
        // 0 / 22; IDW k = 24 46.0 -> 45.0 ms, Sibson k = 30 unchanged); the 2-wave lists keep whole
        // blocks (IDW / Sibson k = 50 +1.3 / +2.6 % in halves; profiles/r06_ab/value_half_blocks_ab.txt)
        constexpr bool HALF = KEEP && KMAX <= 32;
#endif
        double out[3];
        bool ok = true;
        double prev = -1.0;
        if (a.method == PTV_METHOD_SIBSON) {
            // pass 1: d, 1/(d + eps) -> sum (pairwise), sum d -> mean; the order check
            PairwiseStream ps_inv, ps_d;
            double ivmin = INFINITY, dmax = 0.0, dmin_nz = INFINITY;  // operand ranges for div_by below
#if PTV_VALUE_HALF_BLOCKS
            if constexpr (HALF) {
#pragma unroll
                for (int m = 0; m < KMAX; m += 8) {
                    if (m < k) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            double d2[4], dv[4], iv[4];
                            {
                                double4 rc[4];
#pragma unroll
                                for (int i = 0; i < 4; ++i) {
                                    const int j = m + 4 * h + i;
                                    rc[i] = prec[j < k ? slot_at(min(j, KMAX - 1)) : slot_at(0)];
                                }
#pragma unroll
                                for (int i = 0; i < 4; ++i) d2[i] = exact_d2(rc[i]);
                            }
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int j = m + 4 * h + i;
                                dv[i] = sqrt_cr(d2[i]);
                                iv[i] = 1.0 / (dv[i] + a.eps);
                                if (j < k) {
                                    ok = ok && !(d2[i] < prev);
                                    prev = d2[i];
                                    ivmin = fmin(ivmin, iv[i]);
                                    dmax = fmax(dmax, dv[i]);
                                    if (dv[i] > 0.0) dmin_nz = fmin(dmin_nz, dv[i]);
                                }
                                if (j < KMAX) dk[min(j, KMAX - 1)] = dv[i];
                            }
                            ps_inv.add4(m, h, k, iv);
                            ps_d.add4(m, h, k, dv);
                        }
                    }
                }
            } else
#endif
#pragma unroll
            for (int m = 0; m < KMAX; m += 8) {
                if (m < k) {
                    double d2[8], dv[8], iv[8];
                    d2_block(m, d2);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        dv[i] = sqrt_cr(d2[i]);
                        iv[i] = 1.0 / (dv[i] + a.eps);
                        if (m + i < k) {
                            ok = ok && !(d2[i] < prev);
                            prev = d2[i];
                            ivmin = fmin(ivmin, iv[i]);
                            dmax = fmax(dmax, dv[i]);
                            if (dv[i] > 0.0) dmin_nz = fmin(dmin_nz, dv[i]);
                        }
                        if constexpr (KEEP) {
                            if (m + i < KMAX) dk[min(m + i, KMAX - 1)] = dv[i];
                        }
                    }
                    ps_inv.add(m, k, iv);
                    ps_d.add(m, k, dv);
                }
            }
            if (__builtin_amdgcn_ballot_w64(amb || !ok) != 0) {
                list_tile();
                return;
            }
            const double s_inv = ps_inv.finish(k);
            const double mean = ps_d.finish(k) / (double)k;
            auto d_block = [&](int m, double (&dv)[8]) {
                if constexpr (KEEP) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) dv[i] = dk[min(m + i, KMAX - 1)];
                } else {
                    double d2[8];
                    d2_block(m, d2);
#pragma unroll
                    for (int i = 0; i < 8; ++i) dv[i] = sqrt_cr(d2[i]);
                }
            };
            // pass 2: std (ddof 0)
            PairwiseStream ps_var;
#if PTV_VALUE_HALF_BLOCKS
            if constexpr (HALF) {
#pragma unroll
                for (int m = 0; m < KMAX; m += 8) {
                    if (m < k) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            double t[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const double c = dk[min(m + 4 * h + i, KMAX - 1)] - mean;
                                t[i] = c * c;
                            }
                            ps_var.add4(m, h, k, t);
                        }
                    }
                }
            } else
#endif
#pragma unroll
            for (int m = 0; m < KMAX; m += 8) {
                if (m < k) {
                    double dv[8], t[8];
                    d_block(m, dv);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const double c = dv[i] - mean;
                        t[i] = c * c;
                    }
                    ps_var.add(m, k, t);
                }
            }
            const double den = sqrt(ps_var.finish(k) / (double)k) + a.eps;
            // the quotients iv / s_inv and -d / den through one reciprocal each (div_by: correctly
            // rounded for normal operands and quotients; d = 0 gives 0 exactly) when every lane's
            // operands are in range, IEEE division otherwise
            const bool fdiv = __builtin_amdgcn_ballot_w64(!(div_by_ok(ivmin, s_inv, s_inv) && div_by_ok(dmin_nz, dmax, den))) == 0;
            const double rsi = 1.0 / s_inv, rden = 1.0 / den;
            auto w_block = [&](int m, double (&w)[8]) {
                double dv[8];
                d_block(m, dv);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const double iv = 1.0 / (dv[i] + a.eps);
                    w[i] = fdiv ? div_by(iv, s_inv, rsi) * exp(div_by(-dv[i], den, rden))
                                : iv / s_inv * exp(-dv[i] / den);
                }
            };
            // pass 3: the exponential weights (kept in place of the distances when the list is
            // register-held: pass 4 reads them back) and their sum
            PairwiseStream ps_w;
            double wmin = INFINITY;
#if PTV_VALUE_HALF_BLOCKS
            if constexpr (HALF) {
#pragma unroll
                for (int m = 0; m < KMAX; m += 8) {
                    if (m < k) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            double w[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int j = m + 4 * h + i;
                                const double dv = dk[min(j, KMAX - 1)];
                                const double iv = 1.0 / (dv + a.eps);
                                w[i] = fdiv ? div_by(iv, s_inv, rsi) * exp(div_by(-dv, den, rden))
                                            : iv / s_inv * exp(-dv / den);
                                if (j < k && w[i] > 0.0) wmin = fmin(wmin, w[i]);  // exp underflow: 0 / s2 exact
                                if (j < KMAX) dk[min(j, KMAX - 1)] = w[i];
                            }
                            ps_w.add4(m, h, k, w);
                        }
                    }
                }
            } else
#endif
#pragma unroll
            for (int m = 0; m < KMAX; m += 8) {
                if (m < k) {
                    double w[8];
                    w_block(m, w);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        if (m + i < k && w[i] > 0.0) wmin = fmin(wmin, w[i]);  // exp underflow: 0 / s2 exact
                        if constexpr (KEEP) {
                            if (m + i < KMAX) dk[min(m + i, KMAX - 1)] = w[i];
                        }
                    }
                    ps_w.add(m, k, w);
                }
            }
            const double s2 = ps_w.finish(k);
            // w / s2 through one reciprocal when s2, the nonzero w and every quotient are normal
            const bool fast = __builtin_amdgcn_ballot_w64(!div_by_ok(wmin, s2, s2)) == 0;
            const double rs2 = 1.0 / s2;
            // pass 4: normalised weights times the values
            PairwiseStream pu, pv, pw;
#if PTV_VALUE_HALF_BLOCKS
            if constexpr (HALF) {
#pragma unroll
                for (int m = 0; m < KMAX; m += 8) {
                    if (m < k) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            double tu[4], tv[4], tw4[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int j = m + 4 * h + i;
                                const double *r = reinterpret_cast<const double *>(
                                    pval + (j < k ? slot_at(min(j, KMAX - 1)) : slot_at(0)));
                                const double2 uv = *reinterpret_cast<const double2 *>(r);
                                tu[i] = uv.x;
                                tv[i] = uv.y;
                                tw4[i] = r[2];
                            }
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const double w = dk[min(m + 4 * h + i, KMAX - 1)];
                                const double wn = fast ? div_by(w, s2, rs2) : w / s2;
                                tu[i] = wn * tu[i];
                                tv[i] = wn * tv[i];
                                tw4[i] = wn * tw4[i];
                            }
                            pu.add4(m, h, k, tu);
                            pv.add4(m, h, k, tv);
                            pw.add4(m, h, k, tw4);
                        }
                    }
                }
            } else
#endif
#pragma unroll
            for (int m = 0; m < KMAX; m += 8) {
                if (m < k) {
                    double w[8], tu[8], tv[8], tw8[8];
                    val_block(m, tu, tv, tw8);
                    if constexpr (KEEP) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) w[i] = dk[min(m + i, KMAX - 1)];
                    } else {
                        w_block(m, w);
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const double wn = fast ? div_by(w[i], s2, rs2) : w[i] / s2;
                        tu[i] = wn * tu[i];
                        tv[i] = wn * tv[i];
                        tw8[i] = wn * tw8[i];
                    }
                    pu.add(m, k, tu);
                    pv.add(m, k, tv);
                    pw.add(m, k, tw8);
                }
            }
            out[0] = pu.finish(k);
            out[1] = pv.finish(k);
            out[2] = pw.finish(k);
        } else {
            // pass 1: w = 1/(d**p + eps) -> sum (pairwise); the order check
            PairwiseStream ps;
            double wmin = INFINITY;
#if PTV_VALUE_HALF_BLOCKS
            if constexpr (HALF) {
#pragma unroll
                for (int m = 0; m < KMAX; m += 8) {
                    if (m < k) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            double d2[4], w[4];
                            {
                                double4 rc[4];
#pragma unroll
                                for (int i = 0; i < 4; ++i) {
                                    const int j = m + 4 * h + i;
                                    rc[i] = prec[j < k ? slot_at(min(j, KMAX - 1)) : slot_at(0)];
                                }
#pragma unroll
                                for (int i = 0; i < 4; ++i) d2[i] = exact_d2(rc[i]);
                            }
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int j = m + 4 * h + i;
                                if (j < k) {
                                    ok = ok && !(d2[i] < prev);
                                    prev = d2[i];
                                }
                                if (j < KMAX) dk[min(j, KMAX - 1)] = d2[i];
                                w[i] = 1.0 / (np_pow(sqrt_cr(d2[i]), a.power) + a.eps);
                                if (j < k) wmin = fmin(wmin, w[i]);
                            }
                            ps.add4(m, h, k, w);
                        }
                    }
                }
            } else
#endif
#pragma unroll
            for (int m = 0; m < KMAX; m += 8) {
                if (m < k) {
                    double d2[8], w[8];
                    d2_block(m, d2);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        if (m + i < k) {
                            ok = ok && !(d2[i] < prev);
                            prev = d2[i];
                        }
                        if constexpr (KEEP) {
                            if (m + i < KMAX) dk[min(m + i, KMAX - 1)] = d2[i];
                        }
                        w[i] = 1.0 / (np_pow(sqrt_cr(d2[i]), a.power) + a.eps);
                        if (m + i < k) wmin = fmin(wmin, w[i]);
                    }
                    ps.add(m, k, w);
                }
            }
            if (__builtin_amdgcn_ballot_w64(amb || !ok) != 0) {
                list_tile();
                return;
            }
            const double s = ps.finish(k);
            // w_j / s through one reciprocal when every quotient is normal (see the k <= 12 path)
            const bool fast = __builtin_amdgcn_ballot_w64(!div_by_ok(wmin, s, s)) == 0;
            const double rs = 1.0 / s;
            // pass 2: normalised weights times the values
            PairwiseStream pu, pv, pw;
#if PTV_VALUE_HALF_BLOCKS
            if constexpr (HALF) {
#pragma unroll
                for (int m = 0; m < KMAX; m += 8) {
                    if (m < k) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            double tu[4], tv[4], tw4[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int j = m + 4 * h + i;
                                const double *r = reinterpret_cast<const double *>(
                                    pval + (j < k ? slot_at(min(j, KMAX - 1)) : slot_at(0)));
                                const double2 uv = *reinterpret_cast<const double2 *>(r);
                                tu[i] = uv.x;
                                tv[i] = uv.y;
                                tw4[i] = r[2];
                            }
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const double d2 = dk[min(m + 4 * h + i, KMAX - 1)];
                                const double w = 1.0 / (np_pow(sqrt_cr(d2), a.power) + a.eps);
                                const double wn = fast ? div_by(w, s, rs) : w / s;
                                tu[i] = wn * tu[i];
                                tv[i] = wn * tv[i];
                                tw4[i] = wn * tw4[i];
                            }
                            pu.add4(m, h, k, tu);
                            pv.add4(m, h, k, tv);
                            pw.add4(m, h, k, tw4);
                        }
                    }
                }
            } else
#endif
#pragma unroll
            for (int m = 0; m < KMAX; m += 8) {
                if (m < k) {
                    double d2[8], tu[8], tv[8], tw8[8];
                    val_block(m, tu, tv, tw8);
                    if constexpr (KEEP) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) d2[i] = dk[min(m + i, KMAX - 1)];
                    } else {
                        d2_block(m, d2);
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const double w = 1.0 / (np_pow(sqrt_cr(d2[i]), a.power) + a.eps);
                        const double wn = fast ? div_by(w, s, rs) : w / s;
                        tu[i] = wn * tu[i];
                        tv[i] = wn * tv[i];
                        tw8[i] = wn * tw8[i];
                    }
                    pu.add(m, k, tu);
                    pv.add(m, k, tv);
                    pw.add(m, k, tw8);
                }
            }
            out[0] = pu.finish(k);
            out[1] = pv.finish(k);
            out[2] = pw.finish(k);
        }
        if (a.flags & PTV_FLAG_NAN_TO_NUM) {
#pragma unroll
            for (int c = 0; c < 3; ++c) out[c] = nan_to_num(out[c]);
        }
        store_out(a.flags, U, V, W, vo, out[0], out[1], out[2]);
        write_stamps();
        return;
    } else if constexpr (KSL && MODE == kModeInterp) {
        // Key lists (k >= 13): the weights are streamed in blocks of 8 neighbours from the exact
        // d2, recomputed from the records (the keys hold truncated d2), in the reference's order:
        // interpolator.py:142-153 (IDW), :102-122 (Sibson).  Every pass is a rolled loop over the
        // blocks (a fully unrolled epilogue was tens of KB of straight-line code per wave): block
        // b takes slots 0..7 of a copy of the slot list that is rotated down by 8 per block.
        const int k = a.k;
        // the slots of block m from the LDS slot list (entries past k: entry 0's, a valid slot)
        auto rewind = [&]() {};
        auto next_slots = [&](int m, int (&s8)[8]) {
            const int s0 = slot_at(0);
#pragma unroll
            for (int i = 0; i < 8; ++i) s8[i] = m + i < k ? slot_at(m + i) : s0;
        };
        // x, y, z of 8 records (24 of each 32-byte record: 48 VGPRs in flight, not 64)
        auto xyz_block = [&](const double4 *__restrict__ src, const int (&s8)[8], double (&x)[8], double (&y)[8],
                             double (&z)[8]) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double *r = reinterpret_cast<const double *>(src + s8[i]);
                const double2 xy = *reinterpret_cast<const double2 *>(r);
                x[i] = xy.x;
                y[i] = xy.y;
                z[i] = r[2];
            }
        };
        auto d2_block = [&](const int (&s8)[8], double (&d2)[8]) {
            double x[8], y[8], z[8];
            xyz_block(prec, s8, x, y, z);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double dx = qx - x[i], dy = qy - y[i], dz = qz - z[i];
                d2[i] = (dx * dx + dy * dy) + dz * dz;
            }
        };
        double out[3];
        bool ok = true;
        double prev = -1.0;
        if (a.method == PTV_METHOD_SIBSON) {
            // pass 1: d, 1/(d + eps) -> sum (pairwise), sum d -> mean; the order check
            PairwiseStream ps_inv, ps_d;
            double ivmin = INFINITY, dmax = 0.0, dmin_nz = INFINITY;  // operand ranges for div_by below
            rewind();
#pragma unroll 1
            for (int m = 0; m < k; m += 8) {
                int s8[8];
                next_slots(m, s8);
                double d2[8], dv[8], iv[8];
                d2_block(s8, d2);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    dv[i] = sqrt_cr(d2[i]);
                    iv[i] = 1.0 / (dv[i] + a.eps);
                    if (m + i < k) {
                        ok = ok && !(d2[i] < prev);
                        prev = d2[i];
                        ivmin = fmin(ivmin, iv[i]);
                        dmax = fmax(dmax, dv[i]);
                        if (dv[i] > 0.0) dmin_nz = fmin(dmin_nz, dv[i]);
                    }
                }
                ps_inv.add(m, k, iv);
                ps_d.add(m, k, dv);
            }
            stamp(t_epi);  // stamp builds: pass 1 of the key-list epilogue
            if (__builtin_amdgcn_ballot_w64(amb || !ok) != 0) {
                list_tile();
                return;
            }
            const double s_inv = ps_inv.finish(k);
            const double mean = ps_d.finish(k) / (double)k;
            // pass 2: std (ddof 0)
            PairwiseStream ps_var;
            rewind();
#pragma unroll 1
            for (int m = 0; m < k; m += 8) {
                int s8[8];
                next_slots(m, s8);
                double d2[8], t[8];
                d2_block(s8, d2);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const double c = sqrt_cr(d2[i]) - mean;
                    t[i] = c * c;
                }
                ps_var.add(m, k, t);
            }
            const double den = sqrt(ps_var.finish(k) / (double)k) + a.eps;
            // iv / s_inv and -d / den through one reciprocal each where div_by_ok (the k <= 32 path)
            const bool fdiv = __builtin_amdgcn_ballot_w64(!(div_by_ok(ivmin, s_inv, s_inv) && div_by_ok(dmin_nz, dmax, den))) == 0;
            const double rsi = 1.0 / s_inv, rden = 1.0 / den;
            auto w_of = [&](double d2) {
                const double d = sqrt_cr(d2);
                const double iv = 1.0 / (d + a.eps);
                return fdiv ? div_by(iv, s_inv, rsi) * exp(div_by(-d, den, rden)) : iv / s_inv * exp(-d / den);
            };
            // pass 3: the exponential weights' sum
            PairwiseStream ps_w;
            double wmin = INFINITY;
            rewind();
#pragma unroll 1
            for (int m = 0; m < k; m += 8) {
                int s8[8];
                next_slots(m, s8);
                double d2[8], w[8];
                d2_block(s8, d2);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    w[i] = w_of(d2[i]);
                    if (m + i < k && w[i] > 0.0) wmin = fmin(wmin, w[i]);
                }
                ps_w.add(m, k, w);
            }
            const double s2 = ps_w.finish(k);
            const bool fast = __builtin_amdgcn_ballot_w64(!div_by_ok(wmin, s2, s2)) == 0;
            const double rs2 = 1.0 / s2;
            // pass 4: normalised weights times the values
            PairwiseStream pu, pv, pw;
            rewind();
#pragma unroll 1
            for (int m = 0; m < k; m += 8) {
                int s8[8];
                next_slots(m, s8);
                double d2[8], wn[8];
                d2_block(s8, d2);
#pragma unroll
                for (int i = 0; i < 8; ++i) wn[i] = fast ? div_by(w_of(d2[i]), s2, rs2) : w_of(d2[i]) / s2;
                double tu[8], tv[8], tw8[8];
                xyz_block(pval, s8, tu, tv, tw8);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    tu[i] = wn[i] * tu[i];
                    tv[i] = wn[i] * tv[i];
                    tw8[i] = wn[i] * tw8[i];
                }
                pu.add(m, k, tu);
                pv.add(m, k, tv);
                pw.add(m, k, tw8);
            }
            out[0] = pu.finish(k);
            out[1] = pv.finish(k);
            out[2] = pw.finish(k);
        } else {
            // pass 1: w = 1/(d**p + eps) -> sum (pairwise); the order check
            auto w_of = [&](double d2) { return 1.0 / (np_pow(sqrt_cr(d2), a.power) + a.eps); };
            PairwiseStream ps;
            double wmin = INFINITY;
            rewind();
#pragma unroll 1
            for (int m = 0; m < k; m += 8) {
                int s8[8];
                next_slots(m, s8);
                double d2[8], w[8];
                d2_block(s8, d2);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (m + i < k) {
                        ok = ok && !(d2[i] < prev);
                        prev = d2[i];
                    }
                    w[i] = w_of(d2[i]);
                    if (m + i < k) wmin = fmin(wmin, w[i]);
                }
                ps.add(m, k, w);
            }
            stamp(t_epi);  // stamp builds: pass 1 of the key-list epilogue
            if (__builtin_amdgcn_ballot_w64(amb || !ok) != 0) {
                list_tile();
                return;
            }
            const double s = ps.finish(k);
            // w_j / s through one reciprocal when every quotient is normal (see the k <= 12 path)
            const bool fast = __builtin_amdgcn_ballot_w64(!div_by_ok(wmin, s, s)) == 0;
            const double rs = 1.0 / s;
            // pass 2: normalised weights times the values
            PairwiseStream pu, pv, pw;
            rewind();
#pragma unroll 1
            for (int m = 0; m < k; m += 8) {
                int s8[8];
                next_slots(m, s8);
                double d2[8], wn[8];
                d2_block(s8, d2);
                if (fast) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) wn[i] = div_by(w_of(d2[i]), s, rs);
                } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i) wn[i] = w_of(d2[i]) / s;
                }
                double tu[8], tv[8], tw8[8];
                xyz_block(pval, s8, tu, tv, tw8);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    tu[i] = wn[i] * tu[i];
                    tv[i] = wn[i] * tv[i];
                    tw8[i] = wn[i] * tw8[i];
                }
                pu.add(m, k, tu);
                pv.add(m, k, tv);
                pw.add(m, k, tw8);
            }
            out[0] = pu.finish(k);
            out[1] = pv.finish(k);
            out[2] = pw.finish(k);
        }
        if (a.flags & PTV_FLAG_NAN_TO_NUM) {
#pragma unroll
            for (int c = 0; c < 3; ++c) out[c] = nan_to_num(out[c]);
        }
        store_out(a.flags, U, V, W, vo, out[0], out[1], out[2]);
        write_stamps();
        return;
    } else if constexpr (!KEYS) {

    // left-shift the list by kpad so real entries occupy slots 0..k-1 (kpad uniform)
#pragma unroll
    for (int sh = 1; sh < KMAX; sh <<= 1) {
        if (a.kpad & sh) {
#pragma unroll
            for (int j = 0; j + sh < KMAX; ++j) {
                bd[j] = bd[j + sh];
                bp[j] = bp[j + sh];
            }
        }
    }
    const int k = a.k;
    if (a.method == PTV_METHOD_NEAREST) {
        // griddata(method='nearest') (interpolator.py:196-197): NearestNDInterpolator returns
        // values[i] of the single nearest particle (k = 1 query), no arithmetic
        const double4 r = pval[max(bp[0], 0)];
        const bool fix = (a.flags & PTV_FLAG_NAN_TO_NUM) != 0;
        store_out(a.flags, U, V, W, vo, fix ? nan_to_num(r.x) : r.x, fix ? nan_to_num(r.y) : r.y,
                  fix ? nan_to_num(r.z) : r.z);
        return;
    }
    // k <= 8: the neighbours' value records are all loaded here, before the weight
    // arithmetic below, so their latency overlaps it (slots past k are clamped to a valid
    // record).  Larger lists stream them per component after the weights (register budget).
    constexpr int KV = KMAX <= 8 ? KMAX : 1;
    double pvu[KV], pvv[KV], pvw[KV];
#pragma unroll
    for (int j = 0; j < KV; ++j) {
        const double4 r = pval[max(bp[j], 0)];
        pvu[j] = r.x;
        pvv[j] = r.y;
        pvw[j] = r.z;
    }
    double w[KMAX];
    if (a.method == PTV_METHOD_SIBSON) {
        // interpolator.py:106-116
        double d[KMAX], t[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            d[j] = (j < k) ? sqrt_cr(bd[j]) : 0.0;
            t[j] = (j < k) ? 1.0 / (d[j] + a.eps) : 0.0;
        }
        const double s_inv = pairwise<KMAX>(t, k);
        const double mean = pairwise<KMAX>(d, k) / (double)k;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            w[j] = t[j] / s_inv;
            const double c = d[j] - mean;
            t[j] = c * c;
        }
        const double sd = sqrt(pairwise<KMAX>(t, k) / (double)k);
        const double den = sd + a.eps;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) w[j] = (j < k) ? w[j] * exp(-d[j] / den) : 0.0;
        const double s2 = pairwise<KMAX>(w, k);
#pragma unroll
        for (int j = 0; j < KMAX; ++j) w[j] = w[j] / s2;
    } else {
        // interpolator.py:143-147
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            const double d = sqrt_cr(bd[j]);
            w[j] = (j < k) ? 1.0 / (np_pow(d, a.power) + a.eps) : 0.0;
        }
        const double s = pairwise<KMAX>(w, k);
        // w_j / s through one reciprocal when s and every quotient are normal (w_j > 0 here:
        // div_by_ok); IEEE division on any lane otherwise
        double wmin = w[0];
#pragma unroll
        for (int j = 1; j < KMAX; ++j)
            if (j < k) wmin = fmin(wmin, w[j]);
        const bool fast = div_by_ok(wmin, s, s);
        if (__builtin_amdgcn_ballot_w64(!fast) == 0) {
            const double rs = 1.0 / s;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) w[j] = div_by(w[j], s, rs);
        } else {
#pragma unroll
            for (int j = 0; j < KMAX; ++j) w[j] = w[j] / s;
        }
    }

    // interpolator.py:150-153: per component, sum_k w * values[idx, c]
    double out[3];
    if constexpr (KMAX <= 8) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double t[KMAX];
#pragma unroll
            for (int j = 0; j < KMAX; ++j) t[j] = (j < k) ? w[j] * (c == 0 ? pvu[j] : (c == 1 ? pvv[j] : pvw[j])) : 0.0;
            out[c] = pairwise<KMAX>(t, k);
        }
    } else {
        const double *vb = reinterpret_cast<const double *>(pval);
#pragma unroll 1
        for (int c = 0; c < 3; ++c) out[c] = gather_pairwise<KMAX>(w, bp, vb, c, k);
    }
    if (a.flags & PTV_FLAG_NAN_TO_NUM) {
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = nan_to_num(out[c]);
    }
    store_out(a.flags, U, V, W, vo, out[0], out[1], out[2]);
    write_stamps();
    }  // exact-pair lists
}

// Lattice void tiles.  A 4x4x4-point lattice tile inside a large solid sphere of the pack gathers
// the particle shell around it (~59k candidates at 512^3 / 5M) in one wave: 1.7 of the 1.8 ms
// lattice level, on the critical path of every launch and z-slab that holds it.  The launcher runs
// the first tiles of the longest-first block order as a split launch (KnnKernelArgs::split: S
// waves per tile, each taking every S-th cell row of one pass at the lattice bound, which
// covers every lane's k nearest) and merges the S partial lists here: one wave per tile, lane =
// lattice point, each listed slot's exact d2 recomputed (bit-identical to the search's) and
// inserted into a fresh list.  The k smallest of the union are the k smallest of the parts' k
// smallest, so the k-th distance (the bound every finer level uses) is the unsplit launch's.
template <int KMAX>
__global__ __launch_bounds__(256) void k_kdist_merge(KnnKernelArgs a, const double4 *__restrict__ prec,
                                                     const double *__restrict__ ax, const double *__restrict__ ay,
                                                     const double *__restrict__ az, double *__restrict__ U) {
    constexpr bool KEYS = kKeyList<KMAX, false>;
    const int lane = threadIdx.x & 63;
    const int t = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (t >= a.split_tiles) return;  // wave-uniform
    const int b = a.order[t >> 2], tw = t & 3;
    const int bx = b % a.ntxb, rr = b / a.ntxb;
    const int ty = rr % a.nty, tz = rr / a.nty;
    const int tx = bx * 4 + tw;
    if (tx >= a.ntx) return;
    const int ix = tx * 4 + (lane & 3), iy = ty * 4 + ((lane >> 2) & 3), iz = a.z0 + tz * 4 + (lane >> 4);
    if (!(ix < a.nx && iy < a.ny && iz < a.z1)) return;
    const size_t vo = ((size_t)(iz - a.z0) * a.ny + iy) * a.nx + ix;
    const double qx = ax[ix], qy = ay[iy], qz = az[iz];
    double bd[KMAX];
    int bp[KEYS ? 1 : KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) bd[j] = j < a.kpad ? -1.0 : INFINITY;
#pragma unroll
    for (int j = 0; j < (KEYS ? 1 : KMAX); ++j) bp[j] = -1;
    const uint32_t *in = a.split_out + (size_t)t * a.split * KMAX * 64 + lane;
#pragma unroll 2
    for (int p = 0; p < a.split; ++p) {
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            const uint32_t sl = in[((size_t)p * KMAX + j) * 64];
            const bool has = sl != 0xffffffffu;
            const double4 c = prec[has ? sl : 0u];
            const double dx = qx - c.x, dy = qy - c.y, dz = qz - c.z;
            const double e2 = (dx * dx + dy * dy) + dz * dz;
            if constexpr (KEYS) insert_key<KMAX>(bd, make_key(has, e2, has ? sl : 0u, a.smask));
            else insert<KMAX>(bd, bp, has ? e2 : INFINITY, (int)sl);  // +inf: a no-op
        }
    }
    kdist_out<KMAX, KEYS>(a, prec, bd, bp, qx, qy, qz, vo, U);
}

template <int KMAX, int MODE, bool EXACT>
void launch_m(dim3 grid, hipStream_t s, const KnnKernelArgs &ka, const Binned &b, const double *ax,
                     const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
                     const uint8_t *mask, double *U, double *V, double *W) {
    if constexpr ((KMAX == 8 || PTV_STAMP_ALL) && MODE != kModeSlots && !EXACT) {
        // stamps record the main launch, or the lattice-level launches under PTV_STAMP_LATTICE=1,
        // or the outlier filter's search under PTV_STAMP_LATTICE=4
        const char *sl = dev_knob("PTV_STAMP_LATTICE");
        const int stamp_mode = (sl && sl[0] == '1') ? kModeKDist : ((sl && sl[0] == '4') ? kModeFilter : kModeInterp);
        if (g_dbg != nullptr && MODE == stamp_mode) {
            hipLaunchKernelGGL((k_knn_interp<KMAX, true, MODE, false>), grid, dim3(256), 0, s, ka, b.prec, b.pval,
                               b.cstart, ax, ay, az, qx, qy, qz, mask, U, V, W, g_dbg, g_dbg_cap);
            return;
        }
    }
    hipLaunchKernelGGL((k_knn_interp<KMAX, false, MODE, EXACT>), grid, dim3(256), 0, s, ka, b.prec, b.pval, b.cstart,
                       ax, ay, az, qx, qy, qz, mask, U, V, W, (unsigned long long *)nullptr, 0LL);
}

// EXACT: the (d2, slot) pair network (the near-tie repair of a key-list launch; only modes
// whose output depends on the exact order or set)
template <int KMAX, bool EXACT>
void launch_t(dim3 grid, hipStream_t s, const KnnKernelArgs &ka, const Binned &b, const double *ax,
                     const double *ay, const double *az, const double *qx, const double *qy, const double *qz,
                     const uint8_t *mask, double *U, double *V, double *W) {
    switch (ka.mode) {
        case kModeKDist:
            if constexpr (!EXACT) launch_m<KMAX, kModeKDist, false>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
            break;
        case kModeKDistMerge:
            if constexpr (!EXACT)
                hipLaunchKernelGGL((k_kdist_merge<KMAX>), grid, dim3(256), 0, s, ka, b.prec, ax, ay, az, U);
            break;
        case kModeSlots: launch_m<KMAX, kModeSlots, EXACT>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W); break;
        case kModeRadius:
            if constexpr (KMAX == 4 && !EXACT)
                launch_m<KMAX, kModeRadius, false>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
            break;
        case kModeFilter:
            if constexpr (KMAX >= 4) launch_m<KMAX, kModeFilter, EXACT>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
            break;
        default: launch_m<KMAX, kModeInterp, EXACT>(grid, s, ka, b, ax, ay, az, qx, qy, qz, mask, U, V, W);
    }
}

}  // namespace ptv
