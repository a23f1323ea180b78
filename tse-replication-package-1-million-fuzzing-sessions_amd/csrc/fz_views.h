// Sorted views and stream compaction (templated on the row predicate, so the RQ translation
// units instantiate their own filters).
//
// A view is the replacement for one "WHERE project = X AND <filter> ORDER BY time" query issued
// per project by the reference (e.g. queries1.py:267-278, rq4a_bug.py:124-137): all projects at
// once, rows in (project, time) order, with per-project [offs[p], offs[p+1]) segments.
#pragma once

#include "fz_device.h"
#include "fz_internal.h"
#include "fz_lookback.h"

#include <type_traits>

namespace fz {

// A view whose buffers live in the arena (valid for one public call).
struct TmpView {
    int64_t cap = 0;          // upper bound of n (host-known)
    int64_t *d_n = nullptr;   // device count
    int32_t *row = nullptr;   // original row ids
    int64_t *time = nullptr;  // sort time
    uint32_t *proj = nullptr;
    int64_t *offs = nullptr;  // [P + 1]
};

// Offsets [P + 1] of a project-sorted array of device length *d_n <= n_cap (row-parallel; d_n null:
// the length is n_cap).
void segment_offsets_dn(fz_ctx *c, const uint32_t *sorted_proj, const int64_t *d_n, int64_t n_cap, int64_t P,
                        int64_t *offsets);

// Single-pass order-preserving compaction of a view: each 4096-row tile evaluates pred, ranks its
// kept rows in LDS, gets its output base by decoupled look-back over the preceding tiles, and
// writes (row, time, proj) of the kept rows; the last tile writes the count.  One launch instead of
// flag -> device-wide scan -> compact.  The output's segment offsets [P + 1] come from the same
// pass: the view is project-ordered, so project q's output segment starts at the kept count before
// q's first input row - written by the item holding that row (the projects between its
// predecessor's and its own: empty ones too), the ones past the last live row by the last tile.
#ifndef FZ_FC_ITEMS
#define FZ_FC_ITEMS 16
#endif
#ifndef FZ_FC_BLOCK
#define FZ_FC_BLOCK 256
#endif
constexpr int kFcItems = FZ_FC_ITEMS;
constexpr int kFcBlock = FZ_FC_BLOCK;  // threads of a filter workgroup (tile = kFcBlock x kFcItems rows)
constexpr int kFcTile = kFcBlock * kFcItems;

// lower_bound of v in a[lo, hi)
__device__ inline int64_t lower_bound_i64(const int64_t *a, int64_t lo, int64_t hi, int64_t v) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The projects a filter can keep (k_filter_compact's tile skip): flags[p] & mask != 0; count
// (optional, device) 0 = none at all.
struct Selection {
    const uint8_t *flags = nullptr;
    uint8_t mask = 0xff;
    const int64_t *count = nullptr;
    // view_offs (optional, the view's [P + 1] segment offsets): filter the selected projects' rows
    // only - a virtual index over their segments back to back (voff, built by filter_view), so the
    // launch's live tiles cover just those rows (no look-back chain through the skipped ones)
    const int64_t *view_offs = nullptr;
    const int64_t *voff = nullptr;  // [P + 1] exclusive prefix of the selected segments' lengths
    int64_t P = 0;
    // time bound (with view_offs): a selected segment's virtual rows are only those with view time
    // < lim - a prefix of the segment, since the view is time-ordered inside each project (NULL
    // times, INT64_MAX, sort last and fail every `<`).  The reference's per-project queries
    // "WHERE project = X AND date < LIMIT ORDER BY date" (queries1.py:120-129, rq4b_coverage.py:
    // 315-326, rq2_coverage_and_added.py:30-47, rq3:263) are index range scans over (project,
    // date): the rows past the bound are never read.  (lim_time: the view's time column, set by
    // filter_view.)
    bool has_lim = false;
    int64_t lim = 0;
    const int64_t *lim_time = nullptr;
    static Selection segments(const uint8_t *flags, uint8_t mask, const int64_t *count, const int64_t *view_offs,
                              int64_t time_lim) {
        Selection s;
        s.flags = flags;
        s.mask = mask;
        s.count = count;
        s.view_offs = view_offs;
        s.has_lim = true;
        s.lim = time_lim;
        return s;
    }
    // the view row of virtual row v, walking forward from project p (v only grows per thread)
    __device__ int64_t phys(int64_t v, int64_t &p) const {
        if (voff[p + 1] <= v) {  // past p's segment: the next selected segment holding v
            int64_t lo = p + 1, hi = P;  // voff[lo] <= v < voff[hi + 1] ... find last lo with voff[lo] <= v
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) >> 1;
                if (voff[mid] <= v) lo = mid;
                else hi = mid - 1;
            }
            p = lo;
            while (p < P && voff[p + 1] <= v) ++p;  // (skip empty segments ending at v)
        }
        return view_offs[p] + (v - voff[p]);
    }
    // none of the projects [p0, p1] selected (checked one by one for a few; a tile spanning more
    // projects is read)
    __device__ bool none(uint32_t p0, uint32_t p1) const {
        if (p1 - p0 > 64u) return false;
        for (uint32_t p = p0; p <= p1; ++p)
            if (flags[p] & mask) return false;
        return true;
    }
};

// A second predicate counted per project while filtering (off by default): out[p] += the rows of
// project p it holds (one atomic per wave and item where the wave's rows share a project).
struct NoCount {
    static constexpr bool on = false;
    int64_t *out = nullptr;
    __device__ bool operator()(int32_t) const { return false; }
};

// VIRT: the rows are the virtual rows of a Selection with view_offs (the selected projects'
// segments back to back): item i's view row comes from Selection::phys.
struct FcShared {
    int32_t pos[kFcTile];
    uint32_t pj[kFcTile];  // the items' projects (their predecessors' for the offsets)
    int64_t pprev, plast;  // project of the row before the tile / of the last live row
    int32_t tmp[kFcBlock / kWave];
    int64_t prefix;
    unsigned int tile;
    int skip;
    int64_t p0, p1;  // (VIRT) the selected segments holding the tile's first and last virtual rows
};
// (VIRT) a tile whose rows span at most this many segments (empty ones included) stages their
// virtual offsets in LDS (in sh.pos, before it holds the keep flags): an item crossing into a
// later segment searches LDS instead of the [P + 1] offsets in global memory - a tile of the Zipf
// tail's small projects crossed on nearly every item, 14 dependent global loads a crossing
#ifndef FZ_FC_VOFF_LDS
#define FZ_FC_VOFF_LDS 1
#endif
constexpr int kFcVoffLds = FZ_FC_VOFF_LDS ? kFcTile / 2 - 1 : 0;
// What a filter writes for kept row q (its rank among the kept rows): by default the view row's
// store row id, time and project (a TmpView); an analysis may pass its own emitter to write what
// it reads next straight from the row (e.g. RQ2 count's trend value), instead of a (row, time,
// project) copy and a second pass that gathers through it.  kTime = false: the time column is
// not loaded.
struct RowTimeProj {
    static constexpr bool kTime = true;
    int32_t *orow;
    int64_t *otime;
    uint32_t *oproj;
    __device__ void operator()(int64_t q, int32_t r, int64_t tm, uint32_t pj) const {
        orow[q] = r;
        otime[q] = tm;
        oproj[q] = pj;
    }
};

// One filter launch's arguments (the view, the predicate, the outputs).
template <typename Pred, typename Count = NoCount, bool VIRT = false, typename Emit = RowTimeProj>
struct FcJob {
    int64_t row0;
    const int64_t *times;
    const uint32_t *proj;
    int64_t n;
    const int64_t *d_live;
    Pred pred;
    Lookback lb;
    int64_t ntiles;
    Emit out;
    int64_t *d_n;
    int64_t *oofs;
    int64_t P;
    Selection sel;
    Count cnt;
};
// tile `bid` of a filter launch (the workgroup's LDS in sh)
template <typename Pred, typename Count, bool VIRT, typename Emit>
__device__ inline void filter_tile(const FcJob<Pred, Count, VIRT, Emit> &J, int64_t bid, FcShared &sh) {
    const int64_t row0 = J.row0;
    const int64_t *__restrict__ times = J.times;
    const uint32_t *__restrict__ proj = J.proj;
    const int64_t n = J.n;
    const int64_t *__restrict__ d_live = J.d_live;
    const Pred &pred = J.pred;
    const Lookback &lb = J.lb;
    int64_t ntiles = J.ntiles;
    int64_t *__restrict__ d_n = J.d_n;
    int64_t *__restrict__ oofs = J.oofs;
    const int64_t P = J.P;
    const Selection &sel = J.sel;
    const Count &cnt = J.cnt;
    const int tid = threadIdx.x;
    const int64_t live = d_live ? *d_live : n;
    int64_t lim = live < n ? live : n;
    // tiles over the live rows only: workgroups past them leave before drawing a ticket; nothing
    // selected at all (*sel.count == 0: configs 3 / 5 have no issue) - every workgroup leaves and
    // the first writes the empty count
    ntiles = lim > 0 ? (lim + kFcTile - 1) / kFcTile : 1;
    if (sel.count && *sel.count == 0) {
        if (bid == 0) {
            if (tid == 0) *d_n = 0;
            for (int64_t q = tid; q <= P; q += kFcBlock) oofs[q] = 0;
        }
        return;
    }
    if (int64_t(bid) >= ntiles) return;
    if (tid == 0) {
        sh.tile = lb_take_tile(lb.ticket, unsigned(ntiles));
        const int64_t b0 = int64_t(sh.tile) * kFcTile, b1 = b0 + kFcTile < lim ? b0 + kFcTile : lim;
        const bool last_tile = int64_t(sh.tile) == ntiles - 1;
        if (VIRT) {  // the selected segment holding the tile's first virtual row
            int64_t p = 0;
            sh.p0 = (b0 < b1) ? (sel.phys(b0, p), p) : 0;
            sh.p1 = (b0 < b1) ? (sel.phys(b1 - 1, p), p) : 0;  // (p: from the first row's segment on)
            sh.skip = 0;
            int64_t q = 0;
            sh.pprev = (b0 > 0 && b0 < b1) ? (sel.phys(b0 - 1, q), q) : -1;
            q = 0;
            sh.plast = (last_tile && lim > 0) ? (sel.phys(lim - 1, q), q) : -1;
        } else {
            sh.pprev = (b0 > 0 && b0 < b1) ? int64_t(proj[b0 - 1]) : -1;
            sh.plast = (last_tile && lim > 0) ? int64_t(proj[lim - 1]) : -1;
            // (a tile of the project-ordered view whose few projects are all unselected keeps
            // nothing: none of its columns is read)
            sh.skip = sel.flags && (b0 >= b1 || sel.none(proj[b0], proj[b1 - 1]));
        }
    }
    __syncthreads();
    const int64_t tile = sh.tile;
    const int64_t base = tile * kFcTile;
    const int64_t lim_rows = lim;  // (the live rows, skipped tile or not)
    if (sh.skip) lim = 0;
    // view row of item i (VIRT: through the selected segments; tables hold < 2^31 rows)
    int32_t pidx[VIRT ? kFcItems : 1];
    if constexpr (VIRT) {
        // the current segment's end and view shift kept in registers: a load only when an item
        // crosses into a later segment (not three dependent loads per item)
        const int64_t p0 = sh.p0, nseg = sh.p1 - p0 + 1;
        int64_t *const s_voff = reinterpret_cast<int64_t *>(sh.pos);  // voff[p0 .. p1 + 1]
        const bool staged = base < lim && nseg > 1 && nseg + 1 <= kFcVoffLds;  // (block-uniform)
        if (staged) {
            for (int64_t q = tid; q <= nseg; q += kFcBlock) s_voff[q] = sel.voff[p0 + q];
            __syncthreads();
        }
        int64_t p = p0;
        int64_t vend = 0, shift = 0;
        if (base < lim) {
            vend = sel.voff[p + 1];
            shift = sel.view_offs[p] - sel.voff[p];
        }
#pragma unroll
        for (int i = 0; i < kFcItems; ++i) {
            const int64_t v = base + i * kFcBlock + tid;
            pidx[i] = 0;
            if (v < lim) {
                if (v >= vend) {
                    if (staged) {  // last q in (p - p0, nseg) with voff[p0 + q] <= v, in LDS
                        int64_t lo = p - p0 + 1, hi = nseg - 1;
                        while (lo < hi) {
                            const int64_t mid = (lo + hi + 1) >> 1;
                            if (s_voff[mid] <= v) lo = mid;
                            else hi = mid - 1;
                        }
                        p = p0 + lo;
                        vend = s_voff[lo + 1];
                        shift = sel.view_offs[p] - s_voff[lo];
                    } else {
                        sel.phys(v, p);
                        vend = sel.voff[p + 1];
                        shift = sel.view_offs[p] - sel.voff[p];
                    }
                }
                pidx[i] = int32_t(v + shift);
            }
        }
        if (staged) __syncthreads();  // (sh.pos is the keep flags' next)
    }
    auto row_at = [&](int i) -> int64_t {
        if constexpr (VIRT) return pidx[i];
        else return base + i * kFcBlock + tid;
    };
    // the store row of every item (implicit: row0 + view position), then all predicate loads:
    // independent loads in flight together, no row-id load before them
    int32_t r[kFcItems];
    bool keep[kFcItems];
#pragma unroll
    for (int i = 0; i < kFcItems; ++i) {
        const int64_t idx = base + i * kFcBlock + tid;
        r[i] = int32_t(row0 + (idx < lim ? row_at(i) : 0));
    }
    // the output columns of every live item, loaded with the predicate's (almost every row is kept
    // on the big tables): their latency overlaps the predicate loads instead of following the
    // look-back as a second dependent round
    int64_t tm[kFcItems];
    uint32_t pj[kFcItems];
#pragma unroll
    for (int i = 0; i < kFcItems; ++i) {
        const bool live = base + i * kFcBlock + tid < lim;
        tm[i] = Emit::kTime && live ? times[row_at(i)] : 0;
        pj[i] = live ? proj[row_at(i)] : 0u;
    }
    // every item's predicate evaluated without a branch (the predicates are branch-free too: `&`,
    // not `&&`), so the compiler issues all items' column loads before the first wait - a short-
    // circuit chain per item was one dependent memory round trip per column and item; items past
    // the live rows read row r = row0 (in bounds) and are masked
    if (base < lim) {
#pragma unroll
        for (int i = 0; i < kFcItems; ++i) keep[i] = pred(r[i]);
#pragma unroll
        for (int i = 0; i < kFcItems; ++i) keep[i] = keep[i] & (base + i * kFcBlock + tid < lim);
    } else {
#pragma unroll
        for (int i = 0; i < kFcItems; ++i) keep[i] = false;
    }
    if constexpr (Count::on) {
        const int lane = lane_id();
#pragma unroll
        for (int i = 0; i < kFcItems; ++i) {
            const int64_t idx = base + i * kFcBlock + tid;
            const bool valid = idx < lim;
            const uint64_t act = __ballot(valid);
            if (!act) continue;  // (wave-uniform)
            const bool c2 = valid && cnt(r[i]);
            const uint64_t m = __ballot(c2);
            if (!m) continue;  // (wave-uniform: nothing to count in this item - the common case)
            const uint32_t p = valid ? pj[i] : 0u;
            const int first = __ffsll((long long)act) - 1;
            const uint32_t pf = __shfl(p, first, kWave);
            if (__ballot(valid && p == pf) == act) {  // the wave's rows all in one project
                if (lane == first && m)
                    atomicAdd(reinterpret_cast<unsigned long long *>(&cnt.out[pf]), (unsigned long long)__popcll(m));
            } else if (c2) {
                atomicAdd(reinterpret_cast<unsigned long long *>(&cnt.out[p]), 1ull);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < kFcItems; ++i) {
        sh.pos[i * kFcBlock + tid] = keep[i] ? 1 : 0;
        sh.pj[i * kFcBlock + tid] = pj[i];
    }
    __syncthreads();
    int32_t loc[kFcItems];
    int32_t run = 0;
    for (int i = 0; i < kFcItems; ++i) {
        loc[i] = run;
        run += sh.pos[tid * kFcItems + i];
    }
    int32_t agg;
    const int32_t off = block_excl_scan<int32_t, kFcBlock / kWave>(run, sh.tmp, &agg);
    if (tid < kWave) {
        const int64_t prefix = lb_exclusive_prefix(lb, tile, agg);
        if (tid == 0) {
            sh.prefix = prefix;
            if (tile == ntiles - 1) *d_n = prefix + agg;
        }
    }
    __syncthreads();
    // keep flag in bit 31 of the exclusive in-tile position
    for (int i = 0; i < kFcItems; ++i) {
        const int k = tid * kFcItems + i;
        sh.pos[k] = (loc[i] + off) | (sh.pos[k] ? int32_t(0x80000000u) : 0);
    }
    __syncthreads();
    const int64_t pre = sh.prefix;
#pragma unroll
    for (int i = 0; i < kFcItems; ++i) {
        if (!keep[i]) continue;
        const int k = i * kFcBlock + tid;
        const int64_t q = pre + (sh.pos[k] & 0x7fffffff);
        J.out(q, r[i], tm[i], pj[i]);
    }
    // segment offsets: the projects starting in this tile, then (last tile) the ones after its rows
    if (sh.skip) {  // (nothing kept: every project starting here starts at pre)
        const int64_t b1 = base + kFcTile < lim_rows ? base + kFcTile : lim_rows;
        const int64_t p1 = b1 > base ? int64_t(proj[b1 - 1]) : sh.pprev;
        for (int64_t q = sh.pprev + 1 + tid; q <= p1; q += kFcBlock) oofs[q] = pre;
    } else {
        for (int i = 0; i < kFcItems; ++i) {
            const int k = i * kFcBlock + tid;
            int64_t a = 1, e = 0, o = 0;
            if (base + k < lim) {
                const int64_t pp = k > 0 ? int64_t(sh.pj[k - 1]) : sh.pprev;
                const int64_t pc = int64_t(pj[i]);
                if (pc > pp) {
                    a = pp + 1;
                    e = pc;
                    o = pre + (sh.pos[k] & 0x7fffffff);
                }
            }
            wave_fill_ranges(oofs, a, e, o);
        }
    }
    if (tile == ntiles - 1) {
        const int64_t tot = pre + agg;
        for (int64_t q = sh.plast + 1 + tid; q <= P; q += kFcBlock) oofs[q] = tot;
    }
}


template <typename Pred, typename Count = NoCount, bool VIRT = false, typename Emit = RowTimeProj>
__global__ __launch_bounds__(kFcBlock) void k_filter_compact(const FcJob<Pred, Count, VIRT, Emit> J) {
    __shared__ FcShared sh;
    filter_tile(J, int64_t(blockIdx.x), sh);
}

// Three filters in one launch (blocks [0, g0) the first one's tiles, then the second's, then the
// third's): independent views filtered back to back by one kernel instead of three.
template <typename P0, typename P1, typename P2>
__global__ __launch_bounds__(kFcBlock) void k_filter_compact3(const FcJob<P0> J0, const FcJob<P1> J1,
                                                            const FcJob<P2> J2, unsigned g0, unsigned g1) {
    __shared__ FcShared sh;
    const unsigned b = blockIdx.x;
    if (b < g0) filter_tile(J0, int64_t(b), sh);
    else if (b < g0 + g1) filter_tile(J1, int64_t(b - g0), sh);
    else filter_tile(J2, int64_t(b - g0 - g1), sh);
}

// The selected projects' segment lengths (0 for the others; entry P = 0) for the virtual rows.
template <typename S>
__global__ __launch_bounds__(kBlock) void k_sel_lengths(const S sel, int64_t P, int64_t *__restrict__ len);
template <typename S>
__global__ __launch_bounds__(kBlock) void k_sel_lengths(const S sel, int64_t P, int64_t *__restrict__ len) {
    for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p <= P; p += int64_t(gridDim.x) * kBlock) {
        int64_t l = 0;
        if (p < P && (sel.flags[p] & sel.mask)) {
            const int64_t a = sel.view_offs[p], b = sel.view_offs[p + 1];
            l = (sel.has_lim ? lower_bound_i64(sel.lim_time, a, b, sel.lim) : b) - a;
        }
        len[p] = l;
    }
}

// The same lengths and their exclusive prefix (voff, [P + 1]) in ONE workgroup when the project axis
// is small (one launch instead of a lengths map + a device-wide scan: config 2's filters are launch-
// latency bound): each thread its run of consecutive projects, one block scan.
constexpr int kSvBlock = 1024;
constexpr int64_t kSvOneWg = int64_t(kSvBlock) * 64;
template <typename S>
__global__ __launch_bounds__(kSvBlock) void k_sel_voff(const S sel, int64_t P, int64_t *__restrict__ voff) {
    __shared__ int64_t s_tmp[kSvBlock / kWave];
    const int64_t per = (P + 1 + kSvBlock - 1) / kSvBlock;
    const int64_t p0 = int64_t(threadIdx.x) * per, p1 = p0 + per < P + 1 ? p0 + per : P + 1;
    int64_t sum = 0;
    for (int64_t p = p0; p < p1; ++p) {
        int64_t l = 0;
        if (p < P && (sel.flags[p] & sel.mask)) {
            const int64_t a = sel.view_offs[p], b = sel.view_offs[p + 1];
            l = (sel.has_lim ? lower_bound_i64(sel.lim_time, a, b, sel.lim) : b) - a;
        }
        voff[p] = l;  // (this thread's own entries: read back below by the same thread)
        sum += l;
    }
    int64_t run = block_excl_scan<int64_t, kSvBlock / kWave>(sum, s_tmp, (int64_t *)nullptr);
    for (int64_t p = p0; p < p1; ++p) {
        const int64_t l = voff[p];
        voff[p] = run;
        run += l;
    }
}

// Views of fewer rows than this take time-bounded selections as plain filters (no range scan).
#ifndef FZ_RANGE_SCAN_MIN
#define FZ_RANGE_SCAN_MIN (int64_t(1) << 22)
#endif
constexpr int64_t kRangeScanMin = FZ_RANGE_SCAN_MIN;

// Algorithmic bytes the predicate reads per row (Pred::kBytes when it declares them).
template <class P, class = void>
struct PredBytes {
    static constexpr double value = 0.0;
};
template <class P>
struct PredBytes<P, std::void_t<decltype(P::kBytes)>> {
    static constexpr double value = double(P::kBytes);
};

// Rows of src (n rows, in view order; only the first *src_live when given) satisfying pred(row)
// -> dst (same order).
// sel (optional): the projects pred can keep - tiles of the (project-ordered) view covering none of
// them are skipped without reading their columns.
// emit (optional): what to write per kept row instead of dst.row / time / proj (which are then
// not allocated; dst.d_n and dst.offs are written as always); bytes_out = its bytes per kept row
// (the probe's booking)
template <typename Pred, typename Count = NoCount, typename Emit = RowTimeProj>
void filter_view(fz_ctx *c, const View &v, int64_t n, int64_t P, Pred pred, TmpView &dst,
                 const int64_t *src_live = nullptr, Selection sel = Selection{}, Count cnt = Count{},
                 const Emit *emit = nullptr, double bytes_out = 0.0) {
    const int64_t *times = v.time;
    const uint32_t *proj = v.proj;
    const int64_t row0 = v.row0;
    dst.cap = n;
    dst.d_n = c->arena.get<int64_t>(1);
    if (!emit) {
        dst.row = c->arena.get<int32_t>(n);
        dst.time = c->arena.get<int64_t>(n);
        dst.proj = c->arena.get<uint32_t>(n);
    }
    dst.offs = c->arena.get<int64_t>(P + 1);
    Emit out{};
    if (emit) out = *emit;
    else if constexpr (std::is_same<Emit, RowTimeProj>::value) out = RowTimeProj{dst.row, dst.time, dst.proj};
    // (probe name: the filters of a few projects - a count given, or a project selection without a
    // time bound - are "filter_select" (scripts/pmc_traffic.py scopes them by predicate), the rest
    // "filter_compact", whether or not the range scan applies at this size)
    const bool selective = sel.count || (sel.flags && !sel.has_lim);
    if (sel.has_lim && n < kRangeScanMin) {
        // a small view: the plain filter (the predicate tests the bound itself) - the virtual-row
        // setup is one more launch on the analyses' latency-bound chains (config 2)
        sel.has_lim = false;
        sel.view_offs = nullptr;
        if (!sel.count) sel.flags = nullptr;
    }
    if (sel.has_lim) sel.lim_time = times;
    if (n > 0 && sel.flags && sel.view_offs) {  // the selected segments back to back (virtual rows)
        int64_t *voff = c->arena.get<int64_t>(P + 1);
        // (one workgroup when the segments' lengths are offset differences; the time-bounded
        // lengths are binary searches - one thread per project across the chip, then the scan)
        if (P + 1 <= kSvOneWg && !sel.has_lim) {
            k_sel_voff<Selection><<<1, kSvBlock, 0, c->stream>>>(sel, P, voff);
            FZ_LAUNCH_CHECK();
        } else {
            int64_t *vl = c->arena.get<int64_t>(P + 1);
            k_sel_lengths<Selection><<<grid_for(P + 1), kBlock, 0, c->stream>>>(sel, P, vl);
            FZ_LAUNCH_CHECK();
            scan_exclusive_i64(c, vl, voff, P + 1, nullptr);
        }
        sel.voff = voff;
        sel.P = P;
        src_live = voff + P;  // (a view filter: no other live bound)
    }
    if (n > 0) {
        const int64_t ntiles = (n + kFcTile - 1) / kFcTile;
        const Lookback lb = lookback_begin(c, ntiles);
        // per input row: the predicate's columns; per kept row: time 8 + project 4 read, (row, time,
        // project) 16 written
        // (a selective filter reads only the tiles of its projects: probed apart, kept rows' bytes)
        // (a time-bounded view is a range scan: its virtual rows' predicate bytes are booked from
        // their device count - the rows past the bound are not read)
        const bool ranged = sel.voff && sel.has_lim;
        ProbeScope ps(c, selective ? "filter_select" : "filter_compact",
                      sel.flags ? 0.0 : double(n) * PredBytes<Pred>::value, dst.d_n, emit ? bytes_out : 28.0);
        if (ranged) ps.add_count(sel.voff + P, PredBytes<Pred>::value);
        if (sel.voff)
            k_filter_compact<Pred, Count, true, Emit><<<unsigned(ntiles), kFcBlock, 0, c->stream>>>(
                FcJob<Pred, Count, true, Emit>{row0, times, proj, n, src_live, pred, lb, ntiles, out, dst.d_n, dst.offs, P,
                                               sel, cnt});
        else
            k_filter_compact<Pred, Count, false, Emit><<<unsigned(ntiles), kFcBlock, 0, c->stream>>>(
                FcJob<Pred, Count, false, Emit>{row0, times, proj, n, src_live, pred, lb, ntiles, out, dst.d_n, dst.offs,
                                                P, sel, cnt});
        FZ_LAUNCH_CHECK();
        lookback_end(c, ntiles);
    } else {
        const int64_t zero = 0;
        set_i64(c, dst.d_n, &zero, 1);
        if (!dst.proj) dst.proj = c->arena.get<uint32_t>(1);
        segment_offsets_dn(c, dst.proj, dst.d_n, n, P, dst.offs);
    }
}

// Ordered stream compaction of the indices i < *d_n (d_n null: n_cap) kept by pred(i): emit(i, q)
// for each, q = its rank among the kept ones; *d_total (optional) = their number.  One launch -
// decoupled look-back over 4096-index tiles - instead of a flag map, a device-wide scan and an emit
// map.  pred may have side effects (write what emit reads back for the same i).  ITEMS indices per
// thread: 16 for light predicates; a heavy one (binary searches) takes 1 - 4, so that the tiles
// spread over the whole chip.
template <int ITEMS, typename Pred, typename Emit>
__global__ __launch_bounds__(kBlock) void k_compact_emit(int64_t n_cap, const int64_t *__restrict__ d_n, Pred pred,
                                                         Emit emit, Lookback lb, int64_t *__restrict__ d_total) {
    constexpr int kCeItems = ITEMS, kCeTile = kBlock * ITEMS;
    __shared__ int32_t s_pos[kCeTile];
    __shared__ int32_t s_tmp[4];
    __shared__ int64_t s_prefix;
    __shared__ unsigned int s_tile;
    const int tid = threadIdx.x;
    const int64_t n = d_n ? (*d_n < n_cap ? *d_n : n_cap) : n_cap;
    const int64_t ntiles = n > 0 ? (n + kCeTile - 1) / kCeTile : 1;
    if (int64_t(blockIdx.x) >= ntiles) return;
    if (tid == 0) s_tile = lb_take_tile(lb.ticket, unsigned(ntiles));
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t base = tile * kCeTile;
    bool keep[kCeItems];
#pragma unroll
    for (int i = 0; i < kCeItems; ++i) {
        const int64_t idx = base + i * kBlock + tid;
        keep[i] = idx < n && pred(idx);
        s_pos[i * kBlock + tid] = keep[i] ? 1 : 0;
    }
    __syncthreads();
    int32_t loc[kCeItems];
    int32_t run = 0;
    for (int i = 0; i < kCeItems; ++i) {
        loc[i] = run;
        run += s_pos[tid * kCeItems + i];
    }
    int32_t agg;
    const int32_t off = block_excl_scan(run, s_tmp, &agg);
    if (tid < kWave) {
        const int64_t prefix = lb_exclusive_prefix(lb, tile, agg);
        if (tid == 0) {
            s_prefix = prefix;
            if (tile == ntiles - 1 && d_total) *d_total = prefix + agg;
        }
    }
    __syncthreads();
    for (int i = 0; i < kCeItems; ++i) s_pos[tid * kCeItems + i] = loc[i] + off;
    __syncthreads();
    const int64_t pre = s_prefix;
#pragma unroll
    for (int i = 0; i < kCeItems; ++i)
        if (keep[i]) emit(base + i * kBlock + tid, pre + s_pos[i * kBlock + tid]);
}
template <int ITEMS = 16, typename Pred, typename Emit>
void compact_emit(fz_ctx *c, int64_t n_cap, const int64_t *d_n, Pred pred, Emit emit, int64_t *d_total) {
    constexpr int64_t kCeTile = int64_t(kBlock) * ITEMS;
    if (n_cap <= 0) {
        if (d_total) {
            const int64_t zero = 0;
            set_i64(c, d_total, &zero, 1);
        }
        return;
    }
    const int64_t ntiles = (n_cap + kCeTile - 1) / kCeTile;
    const Lookback lb = lookback_begin(c, ntiles);
    k_compact_emit<ITEMS, Pred, Emit><<<unsigned(ntiles), kBlock, 0, c->stream>>>(n_cap, d_n, pred, emit, lb, d_total);
    FZ_LAUNCH_CHECK();
    lookback_end(c, ntiles);
}

// Two independent filters in one launch (as filter_views3)
template <typename P0, typename P1>
__global__ __launch_bounds__(kFcBlock) void k_filter_compact2(const FcJob<P0> J0, const FcJob<P1> J1, unsigned g0) {
    __shared__ FcShared sh;
    const unsigned b = blockIdx.x;
    if (b < g0) filter_tile(J0, int64_t(b), sh);
    else filter_tile(J1, int64_t(b - g0), sh);
}
template <typename P0, typename P1>
void filter_views2(fz_ctx *c, int64_t P, const View &v0, int64_t n0, P0 p0, TmpView &d0, const View &v1, int64_t n1,
                   P1 p1, TmpView &d1) {
    TmpView *dst[2] = {&d0, &d1};
    const int64_t ns[2] = {n0, n1};
    for (int k = 0; k < 2; ++k) {
        TmpView &d = *dst[k];
        const int64_t n = ns[k];
        d.cap = n;
        d.d_n = c->arena.get<int64_t>(1);
        d.row = c->arena.get<int32_t>(n > 0 ? n : 1);
        d.time = c->arena.get<int64_t>(n > 0 ? n : 1);
        d.proj = c->arena.get<uint32_t>(n > 0 ? n : 1);
        d.offs = c->arena.get<int64_t>(P + 1);
    }
    const int64_t tiles[2] = {(n0 + kFcTile - 1) / kFcTile > 0 ? (n0 + kFcTile - 1) / kFcTile : 1,
                              (n1 + kFcTile - 1) / kFcTile > 0 ? (n1 + kFcTile - 1) / kFcTile : 1};
    Lookback lb[2];
    lookback_begin_n(c, tiles, 2, lb);
    ProbeScope ps(c, "filter_compact", double(n0) * PredBytes<P0>::value + double(n1) * PredBytes<P1>::value);
    const FcJob<P0> j0{v0.row0, v0.time, v0.proj, n0, nullptr, p0, lb[0], tiles[0],
                       RowTimeProj{d0.row, d0.time, d0.proj}, d0.d_n,
                       d0.offs, P, Selection{}, NoCount{}};
    const FcJob<P1> j1{v1.row0, v1.time, v1.proj, n1, nullptr, p1, lb[1], tiles[1],
                       RowTimeProj{d1.row, d1.time, d1.proj}, d1.d_n,
                       d1.offs, P, Selection{}, NoCount{}};
    k_filter_compact2<P0, P1><<<unsigned(tiles[0] + tiles[1]), kFcBlock, 0, c->stream>>>(j0, j1, unsigned(tiles[0]));
    FZ_LAUNCH_CHECK();
}

// Three independent filters (views v0 / v1 / v2 with n0 / n1 / n2 rows, predicates p0 / p1 / p2,
// no selection, no second count) in one launch -> d0 / d1 / d2, as three filter_view calls.
template <typename P0, typename P1, typename P2>
void filter_views3(fz_ctx *c, int64_t P, const View &v0, int64_t n0, P0 p0, TmpView &d0, const View &v1, int64_t n1,
                   P1 p1, TmpView &d1, const View &v2, int64_t n2, P2 p2, TmpView &d2) {
    TmpView *dst[3] = {&d0, &d1, &d2};
    const int64_t ns[3] = {n0, n1, n2};
    for (int k = 0; k < 3; ++k) {
        TmpView &d = *dst[k];
        const int64_t n = ns[k];
        d.cap = n;
        d.d_n = c->arena.get<int64_t>(1);
        d.row = c->arena.get<int32_t>(n > 0 ? n : 1);
        d.time = c->arena.get<int64_t>(n > 0 ? n : 1);
        d.proj = c->arena.get<uint32_t>(n > 0 ? n : 1);
        d.offs = c->arena.get<int64_t>(P + 1);
    }
    // (an empty view still gets one workgroup: it writes the zero count and the offsets)
    const int64_t tiles[3] = {(n0 + kFcTile - 1) / kFcTile > 0 ? (n0 + kFcTile - 1) / kFcTile : 1,
                              (n1 + kFcTile - 1) / kFcTile > 0 ? (n1 + kFcTile - 1) / kFcTile : 1,
                              (n2 + kFcTile - 1) / kFcTile > 0 ? (n2 + kFcTile - 1) / kFcTile : 1};
    Lookback lb[3];
    lookback_begin_n(c, tiles, 3, lb);
    ProbeScope ps(c, "filter_compact",
                  double(n0) * PredBytes<P0>::value + double(n1) * PredBytes<P1>::value +
                      double(n2) * PredBytes<P2>::value);
    const FcJob<P0> j0{v0.row0, v0.time, v0.proj, n0, nullptr, p0, lb[0], tiles[0],
                       RowTimeProj{d0.row, d0.time, d0.proj}, d0.d_n,
                       d0.offs, P, Selection{}, NoCount{}};
    const FcJob<P1> j1{v1.row0, v1.time, v1.proj, n1, nullptr, p1, lb[1], tiles[1],
                       RowTimeProj{d1.row, d1.time, d1.proj}, d1.d_n,
                       d1.offs, P, Selection{}, NoCount{}};
    const FcJob<P2> j2{v2.row0, v2.time, v2.proj, n2, nullptr, p2, lb[2], tiles[2],
                       RowTimeProj{d2.row, d2.time, d2.proj}, d2.d_n,
                       d2.offs, P, Selection{}, NoCount{}};
    k_filter_compact3<P0, P1, P2><<<unsigned(tiles[0] + tiles[1] + tiles[2]), kFcBlock, 0, c->stream>>>(
        j0, j1, j2, unsigned(tiles[0]), unsigned(tiles[1]));
    FZ_LAUNCH_CHECK();
}

__device__ inline int64_t upper_bound_i64(const int64_t *a, int64_t lo, int64_t hi, int64_t v) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ inline void atomic_add_i64(int64_t *p, int64_t v) {
    atomicAdd(reinterpret_cast<unsigned long long *>(p), static_cast<unsigned long long>(v));
}

// Count nonzero bytes of flags[0..P) into *out (adds).
void count_flags(fz_ctx *c, const uint8_t *flags, int64_t P, int64_t *out);
// the same for k <= 4 flag arrays of P bytes each in one launch (outs[j] += count of flags[j])
void count_flags_n(fz_ctx *c, const uint8_t *const *flags, int64_t *const *outs, int k, int64_t P);
// describe of x[0..*d_n) with nmax a host upper bound (fz_prims.hip).
void describe_f64_dn(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n, fz_describe *dev_out);
// up to kDescBatch independent describes; all small ones (nmax <= 4096) share one launch (one
// workgroup each), larger ones take the multi-launch path.
constexpr int kDescBatch = 4;
struct DescJob {
    const double *x;
    int64_t nmax;
    const int64_t *d_n;
    fz_describe *out;
};
void describe_f64_dn_batch(fz_ctx *c, const DescJob *jobs, int njobs);
struct SortedDescJob {
    const uint64_t *k;  // ascending f64_key of x[0..*d_n)
    const double *x;
    int64_t nmax;
    const int64_t *d_n;
    fz_describe *out;
};
struct SortedDescArgs {
    const uint64_t *k[kDescBatch];
    const double *x[kDescBatch];
    const int64_t *d_n[kDescBatch];
    fz_describe *out[kDescBatch];
};
void describe_sorted_dn_batch(fz_ctx *c, const SortedDescJob *jobs, int njobs);
// The same with each job's mean and standard deviation given (ms[2j], ms[2j + 1] = sqrt(sum of
// squared deviations / n)): only the finishing launch.
void describe_sorted_dn_finish(fz_ctx *c, const SortedDescJob *jobs, int njobs, const double *ms);
// ascending order-preserving keys (f64_key) of x[0..*d_n); entries past *d_n are ~0.
uint64_t *sorted_keys_dn(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n);
// the same for nmax <= 4096 in one workgroup (LDS bitonic network, fz_series.hip)
uint64_t *sort_small_keys(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n);
void describe_sorted_dn(fz_ctx *c, const uint64_t *sorted_keys, const double *x, int64_t nmax, const int64_t *d_n,
                        fz_describe *dev_out);

}  // namespace fz
