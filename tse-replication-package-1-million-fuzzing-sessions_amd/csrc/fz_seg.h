// Segmented series toolkit: many independent series (one per project, per session index, or a
// single series) laid out contiguously with offsets[S + 1].
//
// Load balance (Zipf projects, 1e6-point series - SURVEY.md 8(d) configs 4/5): reductions never
// map one segment to one workgroup.  Segments are cut into chunks of at most kChunk elements
// (ChunkMap); one workgroup reduces one chunk into double-double partials, then one wave per
// segment adds its chunks in order.  Results are deterministic (fixed order, no float atomics).
#pragma once

#include "fz_device.h"
#include "fz_internal.h"
#include "fz_stats.h"
#include "fz_views.h"

namespace fz {

constexpr int kChunk = 2048;
constexpr int kRedItems = kChunk / kBlock;  // elements per thread of one chunk
// (k_chunk_reduce takes the items in even / odd pairs: x[u], x[u + 1])
static_assert(kRedItems % 2 == 0, "k_chunk_reduce reads items in pairs");
static_assert(kChunk % kBlock == 0, "chunk shape");

struct Segs {
    int64_t S = 0;                 // number of segments
    const int64_t *offs = nullptr; // [S + 1] device
    int64_t n_cap = 0;             // host upper bound of offs[S]
    int64_t max_len = 0;           // host upper bound of one segment's length (0: n_cap)
    int64_t len_bound() const { return max_len > 0 && max_len < n_cap ? max_len : n_cap; }
};

// Segments no longer than this are sorted inside one workgroup (LDS bitonic network); longer
// ones take the device-wide LSD radix path.
constexpr int64_t kLdsSortMax = 4096;

// Layouts with very many segments (one session per index of the
// longest project - up to ~2e7 sessions, almost all holding a handful of values) are handled by
// size class: every kernel visits only its own class's segments (device-built lists), a tiny
// segment is sorted by one wave (register bitonic network) and reduced by one thread, instead of
// one workgroup walking every segment.  Used when S > kManySegs.
constexpr int kMicroSeg = 8;   // sorted by one thread (register sorting network), no list
constexpr int kTinySeg = 64;   // reduced by one thread; sorted by one wave (9..64 values)
constexpr int64_t kManySegs = 16384;
enum { kClassTiny = 0, kClassMid, kClassWide, kClassBig, kClassNonTiny, kNumClasses };
struct SegLists {
    bool on = false;
    int64_t *d_n = nullptr;  // [kNumClasses] device counts
    int32_t *ids[kNumClasses] = {};
    int64_t cap[kNumClasses] = {};
};
// Lists of segment ids: tiny (kMicroSeg < len <= kTinySeg), mid (<= 1024), wide (<= kLdsSortMax),
// big (longer) and non-tiny (mid + wide + big).  Order inside a list is unspecified.
SegLists seg_lists(fz_ctx *c, const Segs &sg);

struct ChunkMap {
    int64_t cap = 0;
    int64_t *d_n = nullptr;
    int32_t *seg = nullptr;
    int64_t *begin = nullptr;
    int64_t *end = nullptr;
};

ChunkMap make_chunks(fz_ctx *c, const Segs &sg);
// seg id of every element (binary search over offsets); elements past offs[S] get S.
int32_t *segment_ids(fz_ctx *c, const Segs &sg);
// Segment-major merge of R runs, each grouped by segment: sizes [R * S] (run r's count of segment s
// at r * S + s), values = the runs one after another -> out (segment s: run 0's values, run 1's,
// ...) and out_offs [S + 1]
void runs_merge(fz_ctx *c, const double *values, const int64_t *sizes, int64_t R, int64_t S, double *out,
                int64_t *out_offs);

// Chunk k of a segmented reduction.  Explicit maps (cm.d_n != null) list the chunks; implicit
// ones (cps chunks per segment, chosen on the host when every segment is short) derive chunk k
// from the offsets - segment k / cps, piece k % cps - so no map kernels run.  With out != null
// (cps == 1) the chunk sum is the segment result and is written straight to out.
// Chunks [blockIdx.x, nk) step gridDim.x (nk = *cm.d_n for explicit maps, else nk_host).
// With tickets (implicit maps, part and out both set) the chunk that completes its segment folds
// the segment's partials itself - in k_seg_sum's order, so the same bits - instead of a k_seg_sum
// launch: partials stored write-through and drained, then one agent-scope ticket add per chunk;
// the last arriver's acquire, fold and ticket reset (MI355X hand-off: sc1 payload + counter).
// (true in wave 0 of the workgroup that folded)
template <int NV>
__device__ inline bool chunk_arrive(unsigned *tickets, const double *part, double *out, int32_t seg, int64_t cps) {
    if (threadIdx.x >= kWave) return false;  // wave 0 stored the partials
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned old = 0;
    if (threadIdx.x == 0)
        old = __hip_atomic_fetch_add(&tickets[seg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old != unsigned(cps - 1)) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int64_t c0 = int64_t(seg) * cps, c1 = c0 + cps;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        DD acc{0.0, 0.0};
        for (int64_t k = c0 + lane_id(); k < c1; k += 64)
            acc = dd_add(acc, DD{part[(k * NV + v) * 2], part[(k * NV + v) * 2 + 1]});
        acc = wave_dd_sum(acc);
        if (lane_id() == 0) out[int64_t(seg) * NV + v] = acc.hi + acc.lo;
    }
    if (threadIdx.x == 0) __hip_atomic_store(&tickets[seg], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

#ifndef FZ_CR_WPE
#define FZ_CR_WPE 4  // k_chunk_reduce's minimum waves per SIMD: the Shapiro-Wilk / rank-test reductions at
                     // 3 waves (135-175 registers) get 4 (a few spilled): config 2 1.077 -> 1.065 ms, 3L
                     // unchanged (profiles/r06_occupancy_ab.txt)
#endif
template <int NV, typename F>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FZ_CR_WPE))) void k_chunk_reduce(ChunkMap cm, const int64_t *__restrict__ offs, int64_t cps,
                                                         int64_t nk_host, F f, double *__restrict__ part,
                                                         double *__restrict__ out, unsigned *tickets = nullptr) {
    __shared__ double s_hi[4][NV], s_lo[4][NV];
    const int64_t nk = cm.d_n ? *cm.d_n : nk_host;
    const bool fold = tickets != nullptr;
    for (int64_t k = blockIdx.x; k < nk; k += gridDim.x) {
        int32_t seg;
        int64_t b, e;
        if (cm.d_n) {
            seg = cm.seg[k];
            b = cm.begin[k];
            e = cm.end[k];
        } else {
            seg = int32_t(k / cps);
            b = offs[seg] + (k % cps) * kChunk;
            e = b + kChunk < offs[seg + 1] ? b + kChunk : offs[seg + 1];
        }
        if (b >= e && (!out || fold)) {  // an empty chunk (past its segment's live end): zero partials, no barriers
            if (threadIdx.x < NV) {
                if (fold) {
                    store_wt(&part[(k * NV + threadIdx.x) * 2], 0.0);
                    store_wt(&part[(k * NV + threadIdx.x) * 2 + 1], 0.0);
                } else {
                    part[(k * NV + threadIdx.x) * 2] = 0.0;
                    part[(k * NV + threadIdx.x) * 2 + 1] = 0.0;
                }
            }
            if (fold) chunk_arrive<NV>(tickets, part, out, seg, cps);
            continue;
        }
        // two independent double-double accumulators per value (even / odd items), added at the
        // end: the dependent add chain per thread is half as long (the kernel waits on these
        // chains, not on memory: SQ_WAIT_INST_ANY).  This changed the per-thread
        // summation order of round 4 (one accumulator): the order is still fixed, so results are
        // deterministic run to run, and the double-double sums agree with the single-chain ones to
        // well within the 1e-9 parity tolerance, but not bit for bit
        DD acc[NV], acc2[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] = acc2[v] = DD{0.0, 0.0};
        // a chunk is at most kRedItems elements per thread: every element's loads are issued
        // before the first add (one memory round trip per chunk, not kRedItems dependent ones)
        for (int64_t i0 = b + threadIdx.x; i0 < e; i0 += int64_t(kBlock) * kRedItems) {
            double x[kRedItems][NV];
#pragma unroll
            for (int u = 0; u < kRedItems; ++u) {
                const int64_t i = i0 + int64_t(u) * kBlock;
                if (i < e) {
                    f(i, seg, x[u]);
                } else {
#pragma unroll
                    for (int v = 0; v < NV; ++v) x[u][v] = 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < kRedItems; u += 2)
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    if (i0 + int64_t(u) * kBlock < e) acc[v] = dd_add_d(acc[v], x[u][v]);
                    if (i0 + int64_t(u + 1) * kBlock < e) acc2[v] = dd_add_d(acc2[v], x[u + 1][v]);
                }
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            DD r = wave_dd_sum(dd_add(acc[v], acc2[v]));
            if (lane_id() == 0) {
                s_hi[wave_id()][v] = r.hi;
                s_lo[wave_id()][v] = r.lo;
            }
        }
        __syncthreads();
        if (threadIdx.x < NV) {
            const int v = threadIdx.x;
            DD t{s_hi[0][v], s_lo[0][v]};
            for (int w = 1; w < 4; ++w) t = dd_add(t, DD{s_hi[w][v], s_lo[w][v]});
            if (fold) {
                store_wt(&part[(k * NV + v) * 2], t.hi);
                store_wt(&part[(k * NV + v) * 2 + 1], t.lo);
            } else if (out) {
                out[int64_t(seg) * NV + v] = t.hi + t.lo;
            } else {
                part[(k * NV + v) * 2] = t.hi;
                part[(k * NV + v) * 2 + 1] = t.lo;
            }
        }
        if (fold) chunk_arrive<NV>(tickets, part, out, seg, cps);
        __syncthreads();
    }
}

// out[s * NV + v] = sum over segment s's chunks (one wave per segment, chunks in order; implicit
// maps: chunk_off == null, segment s owns chunks [s * cps, (s + 1) * cps)).  With a list, the
// waves walk the listed segments only (*d_ln of them).
template <int NV>
__global__ __launch_bounds__(kBlock) void k_seg_sum(int64_t S, const int64_t *__restrict__ chunk_off, int64_t cps,
                                                    const double *__restrict__ part, double *__restrict__ out,
                                                    const int32_t *__restrict__ list, const int64_t *__restrict__ d_ln) {
    const int64_t ns = list ? *d_ln : S;
    for (int64_t w = int64_t(blockIdx.x) * 4 + wave_id(); w < ns; w += int64_t(gridDim.x) * 4) {
        const int64_t s = list ? list[w] : w;
        const int64_t c0 = chunk_off ? chunk_off[s] : s * cps, c1 = chunk_off ? chunk_off[s + 1] : (s + 1) * cps;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            DD acc{0.0, 0.0};
            for (int64_t k = c0 + lane_id(); k < c1; k += 64)
                acc = dd_add(acc, DD{part[(k * NV + v) * 2], part[(k * NV + v) * 2 + 1]});
            acc = wave_dd_sum(acc);
            if (lane_id() == 0) out[s * NV + v] = acc.hi + acc.lo;
        }
    }
}

// Segments with very many chunks (a single 1e8-value sample has ~5e4): one wave per segment would
// add them one lane-stride at a time (~1 ms).  Instead G workgroups per segment each fold a slice
// of its chunks into one double-double partial (part2[s][g][v]), and k_seg_sum folds the G
// partials per segment (implicit map, cps = G).
template <int NV>
__global__ __launch_bounds__(kBlock) void k_seg_fold(int64_t S, const int64_t *__restrict__ chunk_off, int64_t cps,
                                                     int G, const double *__restrict__ part,
                                                     double *__restrict__ part2, const int32_t *__restrict__ list,
                                                     const int64_t *__restrict__ d_ln) {
    __shared__ double s_hi[4][NV], s_lo[4][NV];
    const int64_t ns = list ? *d_ln : S;
    const int64_t w = blockIdx.x / G;
    const int g = int(blockIdx.x % G);
    if (w >= ns) return;
    const int64_t s = list ? list[w] : w;
    const int64_t c0 = chunk_off ? chunk_off[s] : s * cps, c1 = chunk_off ? chunk_off[s + 1] : (s + 1) * cps;
    const int64_t span = (c1 - c0 + G - 1) / G;
    const int64_t k0 = c0 + g * span, k1 = k0 + span < c1 ? k0 + span : c1;
    DD acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = DD{0.0, 0.0};
    for (int64_t k = k0 + threadIdx.x; k < k1; k += kBlock)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] = dd_add(acc[v], DD{part[(k * NV + v) * 2], part[(k * NV + v) * 2 + 1]});
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const DD r = wave_dd_sum(acc[v]);
        if (lane_id() == 0) {
            s_hi[wave_id()][v] = r.hi;
            s_lo[wave_id()][v] = r.lo;
        }
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        const int v = threadIdx.x;
        DD t{s_hi[0][v], s_lo[0][v]};
        for (int q = 1; q < 4; ++q) t = dd_add(t, DD{s_hi[q][v], s_lo[q][v]});
        part2[((s * G + g) * NV + v) * 2] = t.hi;
        part2[((s * G + g) * NV + v) * 2 + 1] = t.lo;
    }
}

// Segments of <= kTinySeg values, one thread each (sequential double-double sum).
template <int NV, typename F>
__global__ __launch_bounds__(kBlock) void k_tiny_reduce(const int64_t *__restrict__ offs, int64_t S, F f,
                                                        double *__restrict__ out) {
    for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < S; s += int64_t(gridDim.x) * kBlock) {
        const int64_t b = offs[s], e = offs[s + 1];
        if (e - b > kTinySeg) continue;
        DD acc[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] = DD{0.0, 0.0};
        for (int64_t i = b; i < e; ++i) {
            double x[NV];
            f(i, int32_t(s), x);
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[v] = dd_add_d(acc[v], x[v]);
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) out[s * NV + v] = acc[v].hi + acc[v].lo;
    }
}

// Chunk offsets per segment (kept beside the map so k_seg_sum can find a segment's chunks).
// Implicit when cps > 0 (then cm is empty and chunk_off null).
struct ChunkedSegs {
    Segs sg;
    ChunkMap cm;
    int64_t *chunk_off = nullptr;  // [S + 1]
    int64_t cps = 0;               // implicit: chunks per segment
    SegLists lists;                // on: the map covers only the non-tiny segments (see kManySegs)
};
ChunkedSegs chunked(fz_ctx *c, const Segs &sg);

template <int NV>
void seg_fold_parts(fz_ctx *c, const ChunkedSegs &cs, const double *part, double *out);

// Chunks per segment up to which a chunked reduction's last chunk folds its segment (one wave,
// a few dependent double-double adds per lane); longer ones take k_seg_fold + k_seg_sum.
constexpr int64_t kFoldChunks = 512;

// Segmented sum of NV per-element values f(i, seg, x[NV]) -> out[S][NV] (device).
template <int NV, typename F>
void seg_reduce(fz_ctx *c, const ChunkedSegs &cs, F f, double *out, double in_bytes = -1.0) {
    const int64_t S = cs.sg.S;
    if (S <= 0) return;
    // algorithmic bytes: what f reads per live element (offs[S]; in_bytes, default NV doubles - a
    // functor that computes its terms, e.g. Shapiro-Wilk's normal scores, states fewer), NV
    // doubles per segment out
    ProbeScope ps(c, "seg_reduce", 8.0 * NV * double(S), cs.sg.offs + S, in_bytes >= 0.0 ? in_bytes : 8.0 * NV);
    if (cs.cps == 1) {
        k_chunk_reduce<NV, F><<<unsigned(S), kBlock, 0, c->stream>>>(cs.cm, cs.sg.offs, 1, S, f, nullptr, out);
        FZ_LAUNCH_CHECK();
        return;
    }
    const SegLists &L = cs.lists;
    if (L.on) {  // tiny segments one thread each; chunks of the others over a persistent grid
        k_tiny_reduce<NV, F><<<grid_for(S, kBlock, 4096), kBlock, 0, c->stream>>>(cs.sg.offs, S, f, out);
        FZ_LAUNCH_CHECK();
    }
    const int64_t blocks = cs.cps > 0 ? S * cs.cps : cs.cm.cap;
    double *part = c->arena.get<double>(blocks * NV * 2);
    // a persistent grid over the chunks (a capacity-sized implicit map of a short live segment -
    // RQ3's union at config 3 - is mostly empty chunks, each a few loads)
    const unsigned g = unsigned(blocks < 8192 ? blocks : 8192);
    // implicit maps of a few hundred chunks per segment: the last chunk folds (one launch fewer)
    unsigned *tickets = fused_fold_on() && cs.cps > 1 && cs.cps <= kFoldChunks && !L.on ? seg_tickets(c, S) : nullptr;
    k_chunk_reduce<NV, F><<<g, kBlock, 0, c->stream>>>(cs.cm, cs.sg.offs, cs.cps, blocks, f, part,
                                                       tickets ? out : nullptr, tickets);
    FZ_LAUNCH_CHECK();
    if (!tickets) seg_fold_parts<NV>(c, cs, part, out);
}

// The fold of a chunked reduction: per-chunk double-double partials part[(k * NV + v) * 2 + {0, 1}]
// (chunk k of cs's map) -> out[s * NV + v], chunks in order.
template <int NV>
void seg_fold_parts(fz_ctx *c, const ChunkedSegs &cs, const double *part, double *out) {
    const int64_t S = cs.sg.S;
    const SegLists &L = cs.lists;
    const int64_t nsum = L.on ? L.cap[kClassNonTiny] : S;
    const int32_t *lst = L.on ? L.ids[kClassNonTiny] : nullptr;
    const int64_t *dln = L.on ? L.d_n + kClassNonTiny : nullptr;
    // chunks of the longest segment (host bound): a slice of >= kSliceChunks per fold workgroup
    constexpr int64_t kSliceChunks = 512;
    const int64_t maxc = cs.cps > 0 ? cs.cps : (cs.sg.len_bound() + kChunk - 1) / kChunk;
    const int64_t G = maxc > kSliceChunks ? ((maxc + kSliceChunks - 1) / kSliceChunks < 256
                                                 ? (maxc + kSliceChunks - 1) / kSliceChunks : 256) : 1;
    // (only while the sliced fold stays a few thousand workgroups: with very many segments - config
    // 5's ten thousand projects beside one giant - G workgroups for EVERY segment are mostly idle,
    // and one wave per segment folds even the giant's few thousand chunks faster)
    if (G > 1 && nsum * G <= 8192) {
        double *part2 = c->arena.get<double>(S * G * NV * 2);
        k_seg_fold<NV><<<unsigned(nsum * G), kBlock, 0, c->stream>>>(S, cs.chunk_off, cs.cps, int(G), part, part2,
                                                                     lst, dln);
        FZ_LAUNCH_CHECK();
        const unsigned gs = unsigned((nsum + 3) / 4 < 4096 ? (nsum + 3) / 4 : 4096);
        k_seg_sum<NV><<<gs > 0 ? gs : 1, kBlock, 0, c->stream>>>(S, nullptr, G, part2, out, lst, dln);
        FZ_LAUNCH_CHECK();
        return;
    }
    const unsigned gs = unsigned(L.on ? ((nsum + 3) / 4 < 4096 ? (nsum + 3) / 4 : 4096) : (S + 3) / 4);
    k_seg_sum<NV><<<gs > 0 ? gs : 1, kBlock, 0, c->stream>>>(S, cs.chunk_off, cs.cps, part, out, lst, dln);
    FZ_LAUNCH_CHECK();
}

// Per-segment finishing: f(s) for s in [0, S).
template <typename F>
__global__ __launch_bounds__(kBlock) void k_per_seg(int64_t S, F f) {
    for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < S; s += int64_t(gridDim.x) * kBlock) f(s);
}
template <typename F>
void per_seg(fz_ctx *c, int64_t S, F f) {
    if (S <= 0) return;
    k_per_seg<F><<<grid_for(S, kBlock, 4096), kBlock, 0, c->stream>>>(S, f);
    FZ_LAUNCH_CHECK();
}
// Per-element map over [0, n_cap) with the device count d_n (elements >= *d_n skipped).
template <typename F>
__global__ __launch_bounds__(kBlock) void k_map(int64_t n_cap, const int64_t *__restrict__ d_n, F f) {
    const int64_t n = d_n ? *d_n : n_cap;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) f(i);
}
template <typename F>
void map_n(fz_ctx *c, int64_t n_cap, const int64_t *d_n, F f) {
    if (n_cap <= 0) return;
    k_map<F><<<grid_for(n_cap, kBlock, 8192), kBlock, 0, c->stream>>>(n_cap, d_n, f);
    FZ_LAUNCH_CHECK();
}

// ---- series operations (fz_series.hip) ----------------------------------------------------
// Values of each segment sorted ascending (stable: ties keep source order).  pos[i] = source
// index of sorted element i.  Elements past offs[S] are left at the end (undefined after the radix
// path of one long segment, which sorts up to offs[1] only).
struct SortedSegs {
    double *val = nullptr;
    int32_t *pos = nullptr;
};
SortedSegs seg_sort_f64(fz_ctx *c, const double *src, const Segs &sg, const int32_t *segid);

// Average (tie-aware) 1-based rank of every sorted element within its segment, and the number of
// distinct values per segment (ngroups[S], as double).
struct TieRanks {
    double *rank = nullptr;
    double *ngroups = nullptr;
    int64_t *flag = nullptr;    // 1 at the first element of each tie group
    int64_t *gid = nullptr;     // exclusive scan of flag (group of element i = gid[i] - 1 + flag[i])
    int64_t *gstart = nullptr;  // [groups + 1] first element of each group, sentinel offs[S]
};
TieRanks seg_tie_ranks(fz_ctx *c, const ChunkedSegs &cs, const int32_t *segid, const double *sorted);

// scipy.stats.spearmanr(range(n), series) per segment -> rho[S], p[S] (NaN: n < 2 or constant).
void seg_spearman_index(fz_ctx *c, const ChunkedSegs &cs, const SortedSegs &ss, const TieRanks &tr, double *rho,
                        double *pval);
// scipy.stats.shapiro per segment (src in original order, ss its sorted image) -> W[S], p[S]
// (NaN where n < 3).
void seg_shapiro(fz_ctx *c, const ChunkedSegs &cs, const double *src, const SortedSegs &ss, double *w, double *p);
// spearmanr(range(n), x) (rho, pv) and shapiro(x) (w, wp) of x[0, *d_n), n_cap <= 4096
// (series_small_ok), in one launch; every output pointer non-null
bool series_small_ok(int64_t n_cap);
void series_small(fz_ctx *c, const double *x, const int64_t *d_n, double *rho, double *pv, double *w, double *wp);
// spearman_index_sorted (rho, pval; rho null: none) and seg_shapiro of the same sorted segments -
// one launch, one workgroup per segment, when no segment is longer than kSpearmanSmall values
void spearman_shapiro_sorted(fz_ctx *c, const ChunkedSegs &cs, const int32_t *segid, const SortedSegs &ss,
                             const double *src, double *rho, double *pval, double *w, double *p);
// numpy.percentile(seg, q[j]) for sorted segments -> out[s * nq + j] (NaN for empty segments).
// (median != null: statistics.median of every segment too, as seg_median, in the same launch;
// out2 != null: segments in (even, odd) pairs written to two tables, segment s to
// (s odd ? out2 : out)[(s / 2) * nq + j] - RQ4b's G2 / G1 quartile columns, no copy afterwards)
void seg_percentiles(fz_ctx *c, const Segs &sg, const double *sorted, const double *q_host, int nq, double *out,
                     double *median = nullptr, double *out2 = nullptr);
// sum / n per segment in double-double (statistics.mean / np.mean within 1 ulp) -> out[S].
void seg_mean(fz_ctx *c, const ChunkedSegs &cs, const double *vals, double *out);
// statistics.median / np.median of sorted segments: middle value or (a + b) / 2 -> out[S].
void seg_median(fz_ctx *c, const Segs &sg, const double *sorted, double *out);

// statistics.mean (double-double sum / n), statistics.median and numpy.percentile(q[j]) of every
// segment by selection (no sorted copy): mean[S], median[S], pcts[S * nq]; segments of >= 100
// values added to *d_ge100.  Segments of at most kQsMax values (seg_qstats_ok).
constexpr int64_t kQsMax = 16384;
bool seg_qstats_ok(const Segs &sg);
// (mean2 optional: a second copy of the means)
void seg_qstats(fz_ctx *c, const double *vals, const Segs &sg, const double *q_host, int nq, double *mean,
                double *median, double *pcts, int64_t *d_ge100, double *mean2 = nullptr);

// Two-sample rank tests per segment (x = grp 0, y = grp 1): Brunner-Munzel and Mann-Whitney U
// (asymptotic).  Any output pointer may be null.  All outputs are [S] doubles.
__device__ inline int64_t lower_bound_d(const double *a, int64_t lo, int64_t hi, double v) {
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}
__device__ inline int64_t upper_bound_d(const double *a, int64_t lo, int64_t hi, double v) {
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (a[m] <= v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// The special functions called once per segment by one thread, kept out of line: inlined, their
// code set the register count of every per-segment kernel that finishes a test (the Spearman /
// Shapiro-Wilk kernel: 175 VGPRs, two workgroups per CU)
__device__ __noinline__ inline double t_sf_once(double t, double df) { return stats::t_sf(t, df); }
__device__ __noinline__ inline double sw_pvalue_once(int64_t n, double w, double w1) {
    return stats::sw_pvalue(n, w, w1);
}

// scipy.stats.spearmanr(range(n), x) of one sorted segment sv[b, b + n) (pos[j]: the source
// position of sorted value j; ties in any order) by a workgroup of BS threads, each over a
// contiguous run: a tie group's bounds from one binary search where it starts, the rank products
// summed directly (exact half-integer sums).  Thread 0 writes *rho and *pval (when non-null);
// with defer_p the p-value is left to the caller (spearman_p of the returned t statistic, every
// thread holds it): a kernel that also runs Shapiro-Wilk computes the two p-values on different
// waves after both passes instead of one after the other.  s_tmp: BS / 64 doubles.
struct SpearmanT {
    double t = 0.0, dof = -1.0;  // dof < 0: no p-value (NaN)
};
__device__ inline double spearman_p(const SpearmanT &st) {
    return st.dof < 0.0 ? NAN : 2.0 * t_sf_once(fabs(st.t), st.dof);
}
template <int BS>
__device__ inline SpearmanT spearman_block(const double *sv, const int32_t *pos, int64_t b, int64_t n, double *s_tmp,
                                           double *rho, double *pval, bool defer_p = false) {
    constexpr int NW = BS / kWave;
    const double m = double(n + 1) / 2.0;
    double sxy = 0.0, sxx = 0.0, syy = 0.0, ng = 0.0;
    const int64_t per = (n + BS - 1) / BS;
    const int64_t k0 = b + int64_t(threadIdx.x) * per, k1 = k0 + per < b + n ? k0 + per : b + n;
    if (k0 < k1) {
        double v = sv[k0];
        int64_t gs = lower_bound_d(sv, b, k0 + 1, v), ge = upper_bound_d(sv, k0, b + n, v);
        ng += gs == k0 ? 1.0 : 0.0;
        for (int64_t j = k0; j < k1; ++j) {
            if (j > k0 && sv[j] != v) {
                v = sv[j];
                gs = j;
                // (a group of one - the common case - needs no search)
                ge = (j + 1 < b + n && sv[j + 1] == v) ? upper_bound_d(sv, j + 1, b + n, v) : j + 1;
                ng += 1.0;
            }
            const double rx = double(pos[j] - b + 1) - m;
            const double ry = double((gs - b) + (ge - b) + 1) / 2.0 - m;
            sxy += rx * ry;
            sxx += rx * rx;
            syy += ry * ry;
        }
    }
    auto bsum = [&](double x) {
        x = wave_sum(x);
        if (lane_id() == 0) s_tmp[wave_id()] = x;
        __syncthreads();
        double t = s_tmp[0];
        for (int w = 1; w < NW; ++w) t += s_tmp[w];
        __syncthreads();
        return t;
    };
    sxy = bsum(sxy);
    sxx = bsum(sxx);
    syy = bsum(syy);
    ng = bsum(ng);
    double r = NAN;
    SpearmanT st;
    if (n >= 2 && ng > 1.0) {  // as seg_spearman_index
        const double f = 1.0 / double(n - 1);  // (np.cov: times the reciprocal of n - 1)
        r = (sxy * f) / sqrt(sxx * f) / sqrt(syy * f);
        if (r > 1.0) r = 1.0;
        if (r < -1.0) r = -1.0;
        st.dof = double(n - 2);
        double q = st.dof / ((r + 1.0) * (1.0 - r));
        if (q < 0.0) q = 0.0;
        st.t = r * sqrt(q);
    }
    if (threadIdx.x == 0) {
        *rho = r;
        if (pval && !defer_p) *pval = spearman_p(st);
    }
    return st;
}

struct RankTestOut {
    double *bm_stat = nullptr, *bm_p = nullptr;
    double *u1 = nullptr, *mwu_p_two = nullptr, *mwu_p_greater = nullptr, *ties = nullptr;
    double *nx = nullptr, *ny = nullptr;
    // scipy's method='auto' picks the EXACT null distribution when min(nx, ny) <= 8 and there are
    // no ties; that path needs a polynomial of (8 * n_cap + 1) doubles per segment (single-segment
    // calls only).  Null: always asymptotic.
    double *exact_scratch = nullptr;
};
void seg_rank_tests(fz_ctx *c, const double *vals, const uint8_t *grp, const Segs &sg, const int32_t *segid,
                    const RankTestOut &o);
// the same on already sorted segments (grp indexed by source position ss.pos)
void seg_rank_tests_sorted(fz_ctx *c, const SortedSegs &ss, const uint8_t *grp, const ChunkedSegs &cs,
                           const int32_t *segid, const RankTestOut &o);

// Brunner-Munzel p of M sessions whose samples are sorted halves: x = sorted[offs2[2i], offs2[2i+1]),
// y = sorted[offs2[2i+1], offs2[2i+2]); NaN unless both hold >= min_n values.
void bm_sorted_halves(fz_ctx *c, const double *sorted, const int64_t *offs2, int64_t M, int64_t min_n, double *pbm);
constexpr int64_t kBmHalvesMax = 2048;  // bm_sorted_halves is for halves of at most this many values
// the same for sessions of up to kBmLdsMax values (both halves together), staged in LDS
// (soffs[M + 1]: session offsets, soffs[k] = offs2[2k]; n_cap: values of all sessions)
void bm_halves(fz_ctx *c, const double *sorted, const int64_t *offs2, const int64_t *soffs, int64_t M, int64_t n_cap,
               int64_t min_n, double *pbm);
constexpr int kBmLdsMax = 12288;

// brunnermunzel(x, y) from the sorted union of the two samples (one segment, Segs one): x = the
// values whose source position pos[i] < *d_nx; before[i] = x values before union position i,
// before[live] their total (an exclusive scan) -> *bm_stat, *bm_p (either may be null)
void bm_union_sorted(fz_ctx *c, const Segs &one, const double *sorted, const int32_t *pos, const int64_t *before,
                     const int64_t *d_nx, double *bm_stat, double *bm_p);

// spearmanr(range(n), x) per segment from the sorted segments: one workgroup per segment when they
// are short (no tie-rank passes), else seg_tie_ranks + seg_spearman_index.
void spearman_index_sorted(fz_ctx *c, const ChunkedSegs &cs, const int32_t *segid, const SortedSegs &ss, double *rho,
                           double *pval);

// scipy.stats.levene([x, y]) (center='median') from the samples and their medians (device
// scalars) -> out[0] = W, out[1] = p (F(1, N-2) survival, cephes fdtrc rounding).
// mannwhitneyu (two-sided p), brunnermunzel, Cliff's delta (2 U1 / (nx ny) - 1) and levene
// (center='median': W, p) of x[0, *d_nx) vs y[0, *d_ny) in one workgroup - samples whose host
// capacities pass two_sample_small_ok (<= 4096 values each)
bool two_sample_small_ok(int64_t nx_cap, int64_t ny_cap);
void two_sample_small(fz_ctx *c, const double *x, const int64_t *d_nx, const double *y, const int64_t *d_ny,
                      double *mwu_p_two, double *bm_stat, double *bm_p, double *cliff, double *levene);
void levene_two_med(fz_ctx *c, const double *medx, const double *x, int64_t nxm, const int64_t *d_nx,
                    const double *medy, const double *y, int64_t nym, const int64_t *d_ny, double *out);

// A device offsets array [0, *d_n] for one segment whose length is known only on the device.
const int64_t *single_segment(fz_ctx *c, const int64_t *d_n);

}  // namespace fz
