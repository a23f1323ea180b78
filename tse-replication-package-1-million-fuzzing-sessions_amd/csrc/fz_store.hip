// The columnar store: replaces the PostgreSQL tables + (project, time) indexes every RQ query
// scans through dbFile.DB.executeQuery (program/__module/dbFile.py:16-24).
//
// fz_store_build sorts each table once: stable LSD radix passes (fz_prims.hip) on the prefix
// ([build_type |] project) group the rows by segment in row order - moving the time column and
// the other columns with the keys - then every segment is sorted by time in registers (one wave
// for <= 1024 rows, one workgroup for <= 16384: fz_regsort.h), through the segmented merge sort
// (fz_segsort.h) when longer, with NULL timestamps last (PostgreSQL's ASC NULLS LAST) and equal
// times in row order.  The bucket sorts write each sorted row's columns themselves (the segment's
// rows are contiguous after the prefix passes); one pass then gathers the merge-sorted rows.
#include <vector>

#include "fz_device.h"
#include "fz_internal.h"
#include "fz_segsort.h"
#include "fz_views.h"

namespace fz {

struct Prefix {
    const uint32_t *proj;
    const uint8_t *type;  // null: prefix = project only
    int pbits;
    __device__ uint64_t operator()(int64_t r) const {
        uint64_t p = proj[r];
        if (type) {
            uint64_t t = type[r] > 1 ? 2u : type[r];  // Fuzzing, Coverage, any other type last
            p |= t << pbits;
        }
        return p;
    }
};

// The store prologue: the issues' number min / max (NULL skipped) as per-workgroup partials
// part[4 * block + {2, 3}] that the host reduces after the build's single read-back - no atomics, no
// initialisation launch.  (The build-type counts come off the prefix offsets: k_store_views.)
constexpr int kProBlocks = 192;
#ifndef FZ_SPIN_READBACK
#define FZ_SPIN_READBACK 0  // (same-box A/B at config 2: 1.240 / 1.241 ms spinning, 1.240 / 1.243 blocking)
#endif
__global__ __launch_bounds__(kBlock) void k_store_prologue(const int64_t *__restrict__ num, int64_t ni,
                                                           int64_t *__restrict__ part) {
    __shared__ int64_t s_lo[4], s_hi[4];
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < ni; i += int64_t(gridDim.x) * kBlock) {
        const int64_t v = num[i];
        if (v == FZ_TS_NULL) continue;
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (lane_id() == 0) {
        s_lo[wave_id()] = lo;
        s_hi[wave_id()] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            lo = s_lo[w] < lo ? s_lo[w] : lo;
            hi = s_hi[w] > hi ? s_hi[w] : hi;
        }
        part[4 * blockIdx.x + 2] = lo;
        part[4 * blockIdx.x + 3] = hi;
    }
}


// One workgroup: the four views' per-project offsets (fuzz / coverage builds / coverage / issues)
// read off the prefix offsets - a view is a contiguous range of one table's prefixes, and the time
// sorts (merge sort included) keep every row in its prefix's range - their longest segments
// (out[0..3]), a copy of the 9 store counters (out[4..12]: merge-sort rows and longest segment
// per table, rows the long bucket class gathered per table), the views' row counts (out[13..16])
// and the issue-number range off the prologue's partials (out[17..18]), written straight to the
// pinned read-back area: one launch, no copy.  A view starts at its first prefix's offset (the
// builds' Coverage view after all Fuzzing rows), read here rather than counted beforehand.
struct ViewSrc {
    const int64_t *lim_max = nullptr;  // the eligibility pass's most rows of a project before the limit
    const int64_t *src[4] = {};  // prefix offsets of the view's table (null: empty table)
    int64_t first[4] = {};       // prefix of the view's project 0
    int64_t *dst[4] = {};        // [P + 1]
    const unsigned long long *big = nullptr;  // [9] merge-sort rows / longest segment / fused rows
};
__global__ __launch_bounds__(kSortBlock) void k_store_views(const ViewSrc v, int64_t P, const int64_t *__restrict__ part,
                                                           int pblk, int64_t *__restrict__ out) {
    __shared__ int64_t s_m[kSortBlock / kWave];
    __shared__ int64_t s_n[2][kSortBlock / kWave];
    {  // the prologue's issue-number partials: min (out[17]) and max (out[18])
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int b = threadIdx.x; b < pblk; b += kSortBlock) {
            const int64_t l = part[4 * b + 2], h = part[4 * b + 3];
            lo = l < lo ? l : lo;
            hi = h > hi ? h : hi;
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane_id() == 0) s_n[0][wave_id()] = lo, s_n[1][wave_id()] = hi;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < kSortBlock / kWave; ++w) {
                lo = s_n[0][w] < lo ? s_n[0][w] : lo;
                hi = s_n[1][w] > hi ? s_n[1][w] : hi;
            }
            out[17] = lo;
            out[18] = hi;
        }
    }
    for (int i = 0; i < 4; ++i) {
        const int64_t *src = v.src[i];
        const int64_t base = src ? src[v.first[i]] : 0;  // rows of the table before the view
        if (threadIdx.x == 0) out[13 + i] = src ? src[v.first[i] + P] - base : 0;
        int64_t m = 0;
        for (int64_t p = threadIdx.x; p <= P; p += kSortBlock) {
            const int64_t o = src ? src[v.first[i] + p] - base : 0;
            v.dst[i][p] = o;
            if (src && p < P) {
                const int64_t l = src[v.first[i] + p + 1] - src[v.first[i] + p];
                m = l > m ? l : m;
            }
        }
        m = wave_max(m);
        if (lane_id() == 0) s_m[wave_id()] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t r = 0;
            for (int w = 0; w < kSortBlock / kWave; ++w) r = s_m[w] > r ? s_m[w] : r;
            out[i] = r;
        }
        __syncthreads();
    }
    if (threadIdx.x < 9) out[4 + threadIdx.x] = int64_t(v.big[threadIdx.x]);
    if (threadIdx.x == 0) out[19] = v.lim_max ? *v.lim_max : 0;
}

// ---- fork / join onto the store-build helpers (fz_store_set_helpers) -------------------------
// Used only while no probe window is open (the probes bracket launches on the context's own
// stream).  fork: every helper's stream waits for the work enqueued on c so far; join: c waits
// for everything enqueued on the helpers.
// The fork onto the helpers only for large tables: same-box A/B at config 2 (scripts/store_ab.sh,
// profiles/r05_c2_store_fork_ab.txt) - the store alone 0.473 / 0.476 ms with the fork, 0.476 /
// 0.475 without; the whole step 1.202 / 1.206 with, 1.173 / 1.176 without (the helpers are the
// analysis groups' streams: the store's cross-stream waits delay their graphs); configs 3 / 5
// (1e8 rows: the eligibility pass, ~0.4 ms, beside the prefix sort, the time-sort classes side by
// side) 13.1 / 17.8 ms with it, 14.0 / 19.6 without.  FZ_STORE_FORK=1 / 0 forces it on / off.
constexpr int64_t kForkMinRows = int64_t(1) << 22;
static int store_fork_mode() {  // -1: by size, 0: off, 1: on
    static const int m = [] {
        const char *e = std::getenv("FZ_STORE_FORK");
        return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
    }();
    return m;
}
static int store_helpers(fz_ctx *c) {
    if (c->probe.active()) return 0;
    const int m = store_fork_mode();
    const fz_tables &t = store_of(c).t;
    const bool big = t.n_builds + t.n_cov + t.n_issues >= kForkMinRows;
    return (m == 1 || (m < 0 && big)) ? int(c->helpers.size()) : 0;
}
static void store_fork(fz_ctx *c) {
    if (!c->ev_fork) FZ_HIP(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    FZ_HIP(hipEventRecord(c->ev_fork, c->stream));
    for (fz_ctx *h : c->helpers) FZ_HIP(hipStreamWaitEvent(h->stream, c->ev_fork, 0));
}
static void store_join(fz_ctx *c) {
    for (size_t i = 0; i < c->helpers.size(); ++i) {
        hipEvent_t &e = c->ev_join[i];
        if (!e) FZ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        FZ_HIP(hipEventRecord(e, c->helpers[i]->stream));
        FZ_HIP(hipStreamWaitEvent(c->stream, e, 0));
    }
}

// ---- prefix LSD passes (moving the columns) + per-segment register sort by (time, row) -------
// Up to three tables' (prefix, row) keys in one launch: table k's rows are [base[k], base[k + 1])
// of the combined index.
struct PrefixKeys {
    Prefix pre[3];
    uint32_t *keys[3] = {};  // ([type |] project: at most 32 bits)
    uint32_t *vals[3] = {};
    int64_t base[4] = {0, 0, 0, 0};
};
__global__ __launch_bounds__(kBlock) void k_keys_prefix_rows(const PrefixKeys K) {
    for (int64_t gi = int64_t(blockIdx.x) * kBlock + threadIdx.x; gi < K.base[3]; gi += int64_t(gridDim.x) * kBlock) {
        const int k = gi >= K.base[2] ? 2 : (gi >= K.base[1] ? 1 : 0);
        const int64_t i = gi - K.base[k];
        K.keys[k][i] = uint32_t(K.pre[k](i));
        K.vals[k][i] = uint32_t(i);
    }
}

// offs[s] = first position of prefix s in the prefix-sorted keys (s in [0, S]): row i starts the
// prefixes (keys[i-1], keys[i]]; one coalesced read of the keys instead of a binary search per s.
// Up to three tables in one launch: table k covers [base[k], base[k + 1]) = max(n, S + 1) items.
// (A table of many rows per prefix - configs 3 / 5: 1e8 rows, 2^14 prefixes - takes one binary
// search per prefix instead, k_prefix_offsets_bs: S + 1 threads, not a pass over every key.)
struct PrefixOffs {
    const uint32_t *keys[3] = {};
    int64_t n[3] = {0, 0, 0};
    int64_t S[3] = {0, 0, 0};
    int64_t *offs[3] = {};
    int64_t base[4] = {0, 0, 0, 0};
};
__global__ __launch_bounds__(kBlock) void k_prefix_offsets(const PrefixOffs O) {
    // (wave-uniform trip count: the gaps between consecutive keys are filled by whole waves; a wave
    // straddling two tables fills each lane's range in its own table's offsets, one table a round)
    for (int64_t g0 = int64_t(blockIdx.x) * kBlock + (threadIdx.x & ~(kWave - 1)); g0 < O.base[3];
         g0 += int64_t(gridDim.x) * kBlock) {
        const int64_t gi = g0 + lane_id();
        const bool in = gi < O.base[3];
        const int k = gi >= O.base[2] ? 2 : (gi >= O.base[1] ? 1 : 0);
        int64_t a = 1, e = 0, i = 0;
        if (in) {
            i = gi - O.base[k];
            const uint32_t *keys = O.keys[k];
            const int64_t n = O.n[k], S = O.S[k];
            int64_t *offs = O.offs[k];
            const int64_t first = int64_t(keys[0]), last = int64_t(keys[n - 1]);  // n >= 1, keys < S
            if (i <= S) {
                if (i <= first) offs[i] = 0;
                else if (i > last) offs[i] = n;
            }
            if (i > 0 && i < n) {
                const int64_t pp = int64_t(keys[i - 1]), pc = int64_t(keys[i]);
                a = pp + 1;
                e = pc < S ? pc : S;
            }
        }
        for (int t = 0; t < 3; ++t) {  // (uniform: every lane takes part in each table's round)
            const bool mine = in && k == t;
            wave_fill_ranges(O.offs[t], mine ? a : 1, mine ? e : 0, i);
        }
    }
}

// offs[s] = lower_bound(keys, s) for s in [0, S] (the keys ascending, every key < S), one thread
// per prefix; up to three tables in one launch, table k's threads [base[k], base[k + 1]) = S + 1.
__global__ __launch_bounds__(kBlock) void k_prefix_offsets_bs(const PrefixOffs O) {
    for (int64_t gi = int64_t(blockIdx.x) * kBlock + threadIdx.x; gi < O.base[3]; gi += int64_t(gridDim.x) * kBlock) {
        const int k = gi >= O.base[2] ? 2 : (gi >= O.base[1] ? 1 : 0);
        const int64_t sidx = gi - O.base[k];
        const uint32_t *keys = O.keys[k];
        int64_t lo = 0, hi = O.n[k];
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (int64_t(keys[mid]) < sidx) lo = mid + 1;
            else hi = mid;
        }
        O.offs[k][sidx] = lo;
    }
}

// Columns the store materialises in sorted order (k_store_gather, after the sorts): perm[q] =
// the caller's row id of sorted row q, dst[j][q] = src[j][spos[q]] with src the prefix-sorted
// columns.  (Store row id = sorted position: the views' row ids are implicit, View::row0.)
constexpr int kMaxGather = 4;
struct GatherCols {
    int n = 0;
    const void *src[kMaxGather] = {};
    void *dst[kMaxGather] = {};
    int size[kMaxGather] = {};  // bytes: 1, 4 or 8
    int32_t *perm = nullptr;
    double bytes() const {
        double b = 0.0;
        for (int j = 0; j < n; ++j) b += size[j];
        return b;
    }
};

// What every time sort writes for sorted row q: its time (NULL restored), its project, and the
// prefix-sorted position it came from (spos: the gather's index), or kGathered when the sort
// gathered the row's columns itself (the bucket sorts; the merge sort leaves them to the gather).
constexpr uint32_t kGathered = ~0u;
struct TimeSortOut {
    int64_t *otime;
    uint32_t *oproj;
    uint32_t *spos;
    __device__ void put(int64_t q, int64_t t, uint32_t p, int64_t sp) const {
        otime[q] = t;
        oproj[q] = p;
        spos[q] = uint32_t(sp);
    }
};

// One table's gather (below) and the three tables' gathers in one launch: table k owns blocks
// [blk[k], blk[k + 1]), each range a multiple of 8.
struct GatherTab {
    const uint32_t *spos = nullptr;
    const uint32_t *rows = nullptr;
    int64_t n = 0;
    GatherCols gc;
};
struct GatherTabs {
    GatherTab tab[3];
    unsigned blk[4] = {0, 0, 0, 0};
};

// XCD-aware: blocks b and b + 8 share an XCD (round-robin dispatch), so a table's 8 block groups
// each stream through one contiguous eighth of its rows - an XCD's rows in flight then come from a
// few segments whose source ranges stay in its 4 MiB L2 (with the plain grid stride every XCD
// touched every segment in flight and the reads went to HBM).
__global__ __launch_bounds__(kBlock) void k_store_gather(const GatherTabs G) {
    const unsigned bid = blockIdx.x;
    const int k = bid >= G.blk[2] ? 2 : (bid >= G.blk[1] ? 1 : 0);
    const GatherTab &tb = G.tab[k];
    const GatherCols &gc = tb.gc;
    const int64_t n = tb.n;
    const int64_t lb = bid - G.blk[k], nblk = G.blk[k + 1] - G.blk[k];
    const int64_t part = (n + 7) / 8;
    const int64_t g = lb % 8, slot = lb / 8, slots = nblk / 8;
    const int64_t lo = g * part, hi = lo + part < n ? lo + part : n;
    for (int64_t q = lo + slot * kBlock + threadIdx.x; q < hi; q += slots * kBlock) {
        const uint32_t s32 = tb.spos[q];
        if (s32 == kGathered) continue;  // a bucket sort wrote this row's columns
        const int64_t sp = s32;
        gc.perm[q] = int32_t(tb.rows[sp]);
        for (int j = 0; j < gc.n; ++j) {
            if (gc.size[j] == 8)
                static_cast<uint64_t *>(gc.dst[j])[q] = static_cast<const uint64_t *>(gc.src[j])[sp];
            else if (gc.size[j] == 4)
                static_cast<uint32_t *>(gc.dst[j])[q] = static_cast<const uint32_t *>(gc.src[j])[sp];
            else
                static_cast<uint8_t *>(gc.dst[j])[q] = static_cast<const uint8_t *>(gc.src[j])[sp];
        }
    }
}

// A segment the bucket sort cannot take (longer than its largest class, clustered times, or a time
// span that does not fit its key) goes to the merge sort: counted in *big, flagged in bigflag.
__device__ inline void flag_big(unsigned long long *big, uint8_t *bigflag, int64_t s, int64_t len) {
    atomicAdd(big, (unsigned long long)len);
    atomicMax(big + 3, (unsigned long long)len);
    bigflag[s] = 1;
}

constexpr int kBlkPosBits = 14;  // key = time above the segment minimum << 14 | position
constexpr uint64_t kBlkTop = (uint64_t(1) << (64 - kBlkPosBits)) - 1;  // time field of NULL rows

// Bucket (distribution) sort of one segment per workgroup, for segments of min_len < rows <= MAXN:
// n rows go to n + 1 buckets by time - the bucket of t is floor((t - min) * n / (span + 1)),
// monotone in t, NULL times in the last bucket - counted with LDS atomics (the returned count is
// the row's slot in its bucket), bucket starts by one block scan, and a row's final position is
// its bucket start plus the number of rows of its bucket with a smaller key (time above the
// minimum << 14 | position: unique, so equal times keep row order - stable).  O(n) work for
// times spread over the segment's span (sessions: about one build per day); a segment whose
// largest bucket holds more than kBucketSkew rows (clustered or NULL-heavy times), or whose span
// does not fit the key, is flagged for the merge sort instead.  MAXN <= 4096 keeps the keys in LDS;
// larger classes re-read them from the (prefix-sorted, cache-resident) time column.
constexpr int kBucketSkew = 32;
#ifndef FZ_TS_DIRECT
// 1: the short classes write every column themselves, no gather pass - measured slower (same box,
// config 2: store 0.470 vs 0.410 ms, profiles/r06_c2_ts_direct_ab.txt): the scattered partial-line
// writes cost more than the gather's coalesced ones
#define FZ_TS_DIRECT 0
#endif
constexpr bool kTsDirect = FZ_TS_DIRECT;
#ifndef FZ_LONG_FUSE
#define FZ_LONG_FUSE 1  // the 16384-row class gathers its columns itself (0: k_store_gather does)
#endif
#ifndef FZ_TS_PF
#define FZ_TS_PF 8  // long classes of at most this many rows per thread prefetch the next column
#endif
// The sub-bucket pass of long segments (tie != null: equal times ordered by prefix position, any
// span) ranks inside a bucket by re-reading the bucket's rows from global memory - quadratic in the
// bucket size - so its cap is looser but still bounded: a sub-bucket whose largest bucket holds more
// than kTieSkew rows (one timestamp or NULL repeated that often) sends the table's long segments
// to the merge sort (big_segments_bucketed returns false).
constexpr int kTieSkew = 256;
//
// The three tables share each length class's launch: a workgroup takes combined segment gs and
// finds its table from the bases (T.tab[k] is read in place from the kernel arguments).
struct TimeSortTab {
    const int64_t *time = nullptr;   // prefix-sorted times
    const int64_t *offs = nullptr;   // [S + 1] segment offsets
    uint32_t pmask = 0;
    TimeSortOut out{};
    unsigned long long *big = nullptr;  // the table's merge-sort counters
    uint8_t *bigflag = nullptr;
    const uint32_t *rows = nullptr;  // caller row ids in prefix order
    GatherCols gc;
    // sub-bucket pass of long segments (big_segments_bucketed): segment s's rows are written at
    // output positions + oshift[s], its project is sproj[s], and equal times are ordered by tie[]
    // (their prefix-order positions) instead of their position in the segment
    const int64_t *oshift = nullptr;
    const uint32_t *sproj = nullptr;
    const uint32_t *tie = nullptr;
    // (tie_pos: equal times ordered by their position in the segment, with the sub-bucket pass's
    // any-span comparison - its rows arrive in prefix order from the stable radix distribution)
    bool tie_pos = false;
    // rows whose columns the long class gathered itself (the probe's algorithmic bytes), or null
    unsigned long long *fused = nullptr;
    // spos already holds kGathered for every row (time_sort_tables fills it before the class
    // launches): flagged segments and the long class's fused rows need not write it
    bool prefilled = false;
};
struct TimeSortTabs {
    TimeSortTab tab[3];
    int64_t base[4] = {0, 0, 0, 0};  // combined index of table k's first segment; base[3] = total
};
template <int BS, int MAXN>
__device__ __forceinline__ void seg_time_bucket(const TimeSortTabs &T, int64_t min_len, bool flag_longer) {
    constexpr int IPT = MAXN / BS;               // rows per thread
    constexpr int EPT = (MAXN + 1 + BS - 1) / BS;  // buckets per thread in the scan
    constexpr int NW = BS / kWave;
    constexpr bool KEYS_LDS = MAXN <= 4096;
    constexpr bool FUSE = MAXN > 4096 && FZ_LONG_FUSE;  // this class gathers its segments' columns itself
    static_assert(MAXN <= (1 << kBlkPosBits) && MAXN % BS == 0, "bucket sort shape");
    // 16-bit bucket counts, then bucket starts (+ sentinel; every count and start is <= MAXN <=
    // 16384), the rows in bucket order; after the ranking the same bytes are the u64 staging of the
    // fused gather.  (16-bit counters: 32 KiB of counters and positions for the 16384-row class.)
    constexpr int CNT_BYTES = ((EPT * BS + 1) * 2 + 15) / 16 * 16;
    // (the long class stages a whole segment's column at once in the same bytes: one round per
    // column instead of two; 128 KiB - one workgroup per CU, as its registers allow anyway)
    constexpr int MEM_BYTES =
        KEYS_LDS || !FUSE || CNT_BYTES + MAXN * 2 >= MAXN * 8 ? CNT_BYTES + MAXN * 2 : MAXN * 8;
    __shared__ alignas(16) uint8_t s_mem[MEM_BYTES];
    uint16_t *const s_cnt = reinterpret_cast<uint16_t *>(s_mem);
    uint32_t *const s_cnt32 = reinterpret_cast<uint32_t *>(s_mem);  // word q / 2 holds counters q, q ^ 1
    uint16_t *const s_pos = reinterpret_cast<uint16_t *>(s_mem + CNT_BYTES);  // rows in bucket order
    __shared__ uint64_t s_key[KEYS_LDS ? MAXN : 1];
    __shared__ int64_t s_lo[NW], s_hi[NW];
    __shared__ uint32_t s_tmp[NW], s_max[NW];
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    for (int64_t gs = blockIdx.x; gs < T.base[3]; gs += gridDim.x) {
        const int k = gs >= T.base[2] ? 2 : (gs >= T.base[1] ? 1 : 0);
        const TimeSortTab &tb = T.tab[k];
        const int64_t s = gs - T.base[k];
        const int64_t *__restrict__ time = tb.time;
        const TimeSortOut &out = tb.out;
        const GatherCols &gc = tb.gc;
        unsigned long long *big = tb.big;
        uint8_t *bigflag = tb.bigflag;
        const int64_t b = tb.offs[s];
        const int64_t len = tb.offs[s + 1] - b;
        const uint32_t *tie = KEYS_LDS ? nullptr : tb.tie;  // (the sub-bucket pass runs the long class)
        const bool tiemode = !KEYS_LDS && (tb.tie || tb.tie_pos);
        auto tie_of = [&](int idx) { return tie ? tie[b + idx] : uint32_t(idx); };
        const int64_t ob = b + (tb.oshift ? tb.oshift[s] : 0);  // where the sorted rows go
        if (len <= min_len) continue;
        // a segment left to the long-segment pass / merge sort: its rows are marked kGathered so
        // the gather launched before the host has read the counters skips them (the later pass
        // writes them, or writes their source positions and the gather runs again)
        auto flag_segment = [&]() {
            if (tid == 0) flag_big(big, bigflag, s, len);
            if (!tb.prefilled)
                for (int64_t q = tid; q < len; q += BS) out.spos[ob + q] = kGathered;
        };
        if (len > MAXN) {
            if (flag_longer) flag_segment();
            continue;
        }
        const int n = int(len);
        // (LEAN - the unfused long class: the times are not kept in registers but re-read from the
        // segment's cache-resident column where needed, so two workgroups fit a CU)
        constexpr bool LEAN = !KEYS_LDS && !FUSE;
        int64_t t[LEAN ? 1 : IPT];
        auto tm_at = [&](int m) -> int64_t {
            if constexpr (LEAN) {
                const int i = tid + m * BS;
                return i < n ? time[b + i] : FZ_TS_NULL;
            } else {
                return t[m];
            }
        };
        int64_t lo = INT64_MAX, hi = INT64_MIN;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            const int64_t tv = i < n ? time[b + i] : FZ_TS_NULL;
            if constexpr (!LEAN) t[m] = tv;
            if (tv != FZ_TS_NULL) {
                lo = tv < lo ? tv : lo;
                hi = tv > hi ? tv : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane == 0) {
            s_lo[w] = lo;
            s_hi[w] = hi;
        }
        for (int j = tid; j < CNT_BYTES / 4; j += BS) s_cnt32[j] = 0u;
        __syncthreads();
        lo = INT64_MAX;
        hi = INT64_MIN;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            lo = s_lo[q] < lo ? s_lo[q] : lo;
            hi = s_hi[q] > hi ? s_hi[q] : hi;
        }
        if (!tiemode && hi >= lo && uint64_t(hi) - uint64_t(lo) >= kBlkTop) {  // span too wide for the key
            flag_segment();
            __syncthreads();
            continue;
        }
        const double scale = hi >= lo ? double(n) / (double(uint64_t(hi) - uint64_t(lo)) + 1.0) : 0.0;
        // the row's key: time above the minimum (NULL: top) << 14 | position
        auto row_key = [&](int64_t tv, int i) -> uint64_t {
            return ((tv == FZ_TS_NULL ? kBlkTop : uint64_t(tv - lo)) << kBlkPosBits) | uint64_t(i);
        };
        uint32_t bs[IPT];  // bucket << 16 | slot in the bucket
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            const int64_t tv = tm_at(m);
            const bool null = tv == FZ_TS_NULL;
            uint32_t q = null ? uint32_t(n) : uint32_t(double(uint64_t(tv - lo)) * scale);
            q = q < uint32_t(n) || null ? q : uint32_t(n - 1);
            bs[m] = q << 16;
            if (i < n) {
                const uint32_t sh = (q & 1u) * 16u;
                bs[m] |= (atomicAdd(&s_cnt32[q >> 1], 1u << sh) >> sh) & 0xffffu;
                if (KEYS_LDS) s_key[i] = row_key(tv, i);
            }
        }
        __syncthreads();
        // bucket starts: each thread scans EPT consecutive buckets; the largest bucket decides skew
        uint32_t sum = 0, mx = 0;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const uint32_t ce = s_cnt[tid * EPT + e];
            sum += ce;
            mx = ce > mx ? ce : mx;
        }
        mx = wave_max(mx);
        if (lane == 0) s_max[w] = mx;
        uint32_t run = block_excl_scan<uint32_t, NW>(sum, s_tmp, (uint32_t *)nullptr);
#pragma unroll
        for (int e = 0; e < EPT; ++e) {  // (block_excl_scan's barriers ordered every read above)
            const uint32_t ce = s_cnt[tid * EPT + e];
            s_cnt[tid * EPT + e] = uint16_t(run);
            run += ce;
        }
        if (tid == 0) s_cnt[EPT * BS] = uint16_t(n);
        __syncthreads();
        uint32_t gmax = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) gmax = s_max[q] > gmax ? s_max[q] : gmax;
        if (gmax > uint32_t(tiemode ? kTieSkew : kBucketSkew)) {  // clustered times: the merge sort takes it
            flag_segment();
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            if (i < n) s_pos[s_cnt[bs[m] >> 16] + (bs[m] & 0xffffu)] = uint16_t(i);
        }
        __syncthreads();
        const uint32_t p = tb.sproj ? tb.sproj[s] : uint32_t(s) & tb.pmask;
        int32_t dq[IPT];  // sorted position of row i inside the segment
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            dq[m] = -1;
            if (i >= n) continue;
            const uint32_t st = s_cnt[bs[m] >> 16], en = s_cnt[(bs[m] >> 16) + 1];
            if (en - st <= 1) {  // alone in its bucket - the common case for evenly spread times
                dq[m] = int32_t(st);
                continue;
            }
            // (the long class re-reads its own time: t[] need not stay live past the bucketing)
            const int64_t tm = KEYS_LDS ? tm_at(m) : time[b + i];
            const uint64_t key = row_key(tm, i);
            const uint32_t my_tie = tiemode ? tie_of(i) : 0u;
            uint32_t rank = 0;
            for (uint32_t x = st; x < en; ++x) {
                const int ox = s_pos[x];
                if (ox == i) continue;
                if (tiemode) {  // (time, prefix position): no packed key, any span
                    const int64_t tx = time[b + ox];
                    rank += tx < tm || (tx == tm && tie_of(ox) < my_tie);
                    continue;
                }
                uint64_t kx;
                if (KEYS_LDS) {
                    kx = s_key[ox];
                } else {
                    kx = row_key(time[b + ox], ox);
                }
                rank += kx < key;
            }
            dq[m] = int32_t(st + rank);
        }
        if constexpr (!FUSE) {
            if constexpr (KEYS_LDS && kTsDirect) {
                // short segments (<= 4096 rows): every column written straight to the row's sorted
                // slot - the segment's source rows are contiguous (prefix order) and its output range
                // a few KiB that the partial-line writes fill in L2 - so no gather pass follows
                // (spos keeps the prefilled kGathered marker)
                if (tid == 0 && tb.fused) atomicAdd(tb.fused, (unsigned long long)n);
#pragma unroll
                for (int m = 0; m < IPT; ++m) {
                    if (dq[m] < 0) continue;
                    const int64_t q = ob + dq[m], r = b + tid + m * BS;
                    out.otime[q] = tm_at(m);
                    out.oproj[q] = p;
                    if (!tb.prefilled) out.spos[q] = kGathered;
                    gc.perm[q] = int32_t(tb.rows[r]);
                    for (int j = 0; j < gc.n; ++j) {
                        if (gc.size[j] == 8)
                            static_cast<uint64_t *>(gc.dst[j])[q] = static_cast<const uint64_t *>(gc.src[j])[r];
                        else if (gc.size[j] == 4)
                            static_cast<uint32_t *>(gc.dst[j])[q] = static_cast<const uint32_t *>(gc.src[j])[r];
                        else
                            static_cast<uint8_t *>(gc.dst[j])[q] = static_cast<const uint8_t *>(gc.src[j])[r];
                    }
                }
            } else {
                // short segments: time, project and source position written to the sorted slot (the
                // segment's few KiB stay in L2); k_store_gather moves the other columns afterwards
                // (the classes without their keys in LDS re-read the segment's cache-resident times
                // here: t[] is not live past the bucketing - fewer registers, more workgroups per CU)
#pragma unroll
                for (int m = 0; m < IPT; ++m)
                    if (dq[m] >= 0)
                        out.put(ob + dq[m], KEYS_LDS ? tm_at(m) : time[b + tid + m * BS], p, b + tid + m * BS);
            }
            __syncthreads();  // LDS is reused by the next segment
            continue;
        }
        __syncthreads();  // the rank loops' reads of s_cnt / s_pos / s_key are done: LDS is staging now
        // Long segments (config 3: 10k rows) - the gather fused, with coalesced writes: every column
        // of the segment goes through LDS in sorted order (row i's value to slot dq[m]), then out in
        // sorted order - the sorted rows' time, caller row id and gathered columns; project, row id and
        // the kGathered marker (which tells k_store_gather to skip the row) are written directly.
        // Staging: the key array (8-byte slots for the whole segment) or, in the long class, the
        // counter bytes sized for a whole segment's column (one round per column).  (A separate gather would re-read the 250 KB segment at random from
        // HBM; the short classes' segments stay in L2 and gather faster than they stage.)
        uint64_t *stg = KEYS_LDS ? s_key : reinterpret_cast<uint64_t *>(s_mem);
        constexpr int CAP = MAXN;
        static_assert(!FUSE || KEYS_LDS || MEM_BYTES / 8 >= CAP, "gather staging");
        // stage one column (x[m]: row i's value) through LDS in sorted order, write it coalesced
        auto emit = [&](const uint64_t *x, auto store) {
            for (int h = 0; h < n; h += CAP) {
#pragma unroll
                for (int m = 0; m < IPT; ++m)
                    if (dq[m] >= h && dq[m] < h + CAP) stg[dq[m] - h] = x[m];
                __syncthreads();
                const int e = n - h < CAP ? n - h : CAP;
                for (int q = tid; q < e; q += BS) store(ob + h + q, stg[q]);
                __syncthreads();
            }
        };
        // the columns: the time (re-read from the segment's cache-resident prefix-sorted times - the
        // registers holding t[] are free again), the prefix-sorted caller row ids (-> perm), then the
        // gathered ones; column j + 1's loads are issued before column j is staged (their latency
        // hides behind it)
        const int nc = 2 + gc.n;
        auto src_of = [&](int j) {
            return j == 0 ? static_cast<const void *>(time) : (j == 1 ? static_cast<const void *>(tb.rows) : gc.src[j - 2]);
        };
        auto size_of = [&](int j) { return j == 0 ? 8 : (j == 1 ? 4 : gc.size[j - 2]); };
        auto load = [&](int j, uint64_t *x) {
            const void *src = src_of(j);
            const int sz = size_of(j);
#pragma unroll
            for (int m = 0; m < IPT; ++m) {
                const int64_t r = b + tid + m * BS;
                x[m] = dq[m] < 0 ? 0ull
                                 : (sz == 8 ? static_cast<const uint64_t *>(src)[r]
                                            : (sz == 4 ? static_cast<const uint32_t *>(src)[r]
                                                       : static_cast<const uint8_t *>(src)[r]));
            }
        };
        // (the 16-rows-per-thread class has no registers for a second column in flight)
        constexpr bool kPrefetch = IPT <= FZ_TS_PF;
        uint64_t xa[IPT], xb[kPrefetch ? IPT : 1];
        load(0, xa);
        if (tid == 0 && tb.fused) atomicAdd(tb.fused, (unsigned long long)n);
        for (int q = tid; q < n; q += BS) {
            out.oproj[ob + q] = p;
            if (!tb.prefilled) out.spos[ob + q] = kGathered;
        }
        for (int j = 0; j < nc; ++j) {
            if constexpr (kPrefetch) {
                if (j + 1 < nc) load(j + 1, xb);
            } else if (j > 0) {
                load(j, xa);
            }
            void *dst = j == 0 ? static_cast<void *>(out.otime) : (j == 1 ? static_cast<void *>(gc.perm) : gc.dst[j - 2]);
            const int sz = size_of(j);
            emit(xa, [&](int64_t q, uint64_t v) {
                if (sz == 8) static_cast<uint64_t *>(dst)[q] = v;
                else if (sz == 4) static_cast<uint32_t *>(dst)[q] = uint32_t(v);
                else static_cast<uint8_t *>(dst)[q] = uint8_t(v);
            });
            if constexpr (kPrefetch) {
#pragma unroll
                for (int m = 0; m < IPT; ++m) xa[m] = xb[m];
            }
        }
        __syncthreads();  // LDS is reused by the next segment
    }
}

template <int BS, int MAXN>
__global__ __launch_bounds__(BS) void k_seg_time_bucket(const TimeSortTabs T, int64_t min_len, bool flag_longer) {
    seg_time_bucket<BS, MAXN>(T, min_len, flag_longer);
}
#if !FZ_LONG_FUSE
// (the unfused long class at two workgroups per CU: its LDS (68 KB) allows it, its registers must
// fit 64 per lane)
#ifndef FZ_LONG_WPE
#define FZ_LONG_WPE 8
#endif
template <int BS, int MAXN>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(FZ_LONG_WPE, FZ_LONG_WPE))) void k_seg_time_bucket2(
    const TimeSortTabs T, int64_t min_len, bool flag_longer) {
    seg_time_bucket<BS, MAXN>(T, min_len, flag_longer);
}
#endif

// Prefix-sorts the tables by ([type |] project, row) - the columns riding along; the keys of all
// three and their segment offsets in one launch each - and sets up their time sort
// (time_sort_tables, all tables at once): segments too long for the bucket sorts
// are counted in the (zeroed) device counter *big (big[3] = the longest such segment, bigflag[s] =
// 1) for the segmented merge sort; every table's columns are then gathered (gather_tables).
struct PrefixSorted {
    int64_t n = 0;
    int64_t S = 0;
    const int64_t *offs = nullptr;   // [S + 1] segment offsets of the prefix-sorted rows
    const uint32_t *rows = nullptr;  // row ids in (prefix, row) order
    uint8_t *bigflag = nullptr;      // [S] 1: the segment is left to the merge sort
    const int64_t *time = nullptr;   // times in (prefix, row) order
    GatherCols gc;                   // the gathered columns' sources in (prefix, row) order
    TimeSortOut out{};
    uint32_t pmask = 0;
    unsigned long long *big = nullptr;
};
struct TableIn {
    int64_t n;
    Prefix pre;
    int prefix_bits;
    const int64_t *time;
    int64_t *otime;
    uint32_t *oproj;
    GatherCols gc;
    unsigned long long *big;
};
static void prefix_sort_tables(fz_ctx *c, const TableIn *in, PrefixSorted *pss, unsigned long long *hist0,
                               uint32_t *const *spos, const RadixSideMinMax *side) {
    PrefixKeys K;
    // every table is sorted straight from its project column with implicit row ids (key_src): no
    // key / row-id copy pass (0.42 ms at config 3) - the builds' (type | project) key made from the
    // two columns in the histogram and the first pass (type_src); k_keys_prefix_rows only for a
    // table of one row (no pass: its key and row id are the result)
    bool direct[3];
    int64_t total = 0;
    for (int k = 0; k < 3; ++k) {
        const int64_t n = in[k].n > 0 ? in[k].n : 0;
        direct[k] = n > 1 && in[k].prefix_bits > 0;
        K.base[k + 1] = K.base[k] + (direct[k] ? 0 : n);
        K.pre[k] = in[k].pre;
        K.keys[k] = n ? c->arena.get<uint32_t>(n) : nullptr;
        K.vals[k] = n ? c->arena.get<uint32_t>(n) : nullptr;
        pss[k] = PrefixSorted{};
        pss[k].n = n;
        total += n;
    }
    if (total == 0) return;
    if (K.base[3] > 0) {
        k_keys_prefix_rows<<<grid_for(K.base[3], kBlock, 4096), kBlock, 0, c->stream>>>(K);
        FZ_LAUNCH_CHECK();
    }
    // the three tables' radix sorts share their launches (one histogram launch, one launch per
    // digit pass): config 2's nine launches - each a few-tile look-back tail plus a launch gap -
    // become three.  The prefix passes move the time column and the gathered columns with the keys
    // (each pass's writes land in per-digit runs): the time sort and the gather then read every
    // segment's rows from one contiguous range instead of gathering them from the heap-ordered table
    RadixTab rt[3];
    for (int k = 0; k < 3; ++k) {
        const TableIn &t = in[k];
        RadixTab &r = rt[k];
        r.n = pss[k].n;
        r.bits = r.n > 1 ? t.prefix_bits : 0;
        r.key_src = direct[k] ? t.pre.proj : nullptr;
        r.type_src = direct[k] ? t.pre.type : nullptr;
        r.type_shift = t.pre.pbits;
        r.keys = K.keys[k];
        r.vals = K.vals[k];
        r.pl.no_digit_probe = true;
        r.pl.n = 1 + t.gc.n;
        r.pl.in[0] = t.time;
        r.pl.size[0] = 8;
        for (int j = 0; j < t.gc.n; ++j) {
            r.pl.in[1 + j] = t.gc.src[j];
            r.pl.size[1 + j] = t.gc.size[j];
        }
    }
    radix_sort_tables_payload32(c, rt, 3, hist0, side);
    PrefixOffs O;
    for (int k = 0; k < 3; ++k) {
        const TableIn &t = in[k];
        PrefixSorted &ps = pss[k];
        const int64_t n = ps.n;
        O.base[k + 1] = O.base[k];
        if (n == 0) continue;
        K.keys[k] = rt[k].keys;
        K.vals[k] = rt[k].vals;
        ps.time = static_cast<const int64_t *>(rt[k].pl.out[0]);
        ps.gc = t.gc;
        for (int j = 0; j < t.gc.n; ++j) ps.gc.src[j] = rt[k].pl.out[1 + j];
        const int64_t S = int64_t(1) << t.prefix_bits;
        ps.S = S;
        ps.offs = c->arena.get<int64_t>(S + 1);
        ps.rows = K.vals[k];
        ps.out = TimeSortOut{t.otime, t.oproj, spos[k]};
        ps.pmask = t.pre.pbits >= 32 ? 0xffffffffu : uint32_t((1ull << t.pre.pbits) - 1ull);
        ps.big = t.big;
        O.keys[k] = K.keys[k];
        O.n[k] = n;
        O.S[k] = S;
        O.offs[k] = const_cast<int64_t *>(ps.offs);
        O.base[k + 1] = O.base[k] + (n > S + 1 ? n : S + 1);
    }
    // per prefix binary searches when the tables hold many rows per prefix (O(S log n) instead of a
    // pass over every key: 0.37 ms at config 3)
    int64_t nall = 0, sall = 0;
    for (int k = 0; k < 3; ++k)
        if (O.n[k] > 0) nall += O.n[k], sall += O.S[k] + 1;
    if (nall >= 64 * sall) {
        PrefixOffs B = O;
        for (int k = 0; k < 3; ++k) B.base[k + 1] = B.base[k] + (O.n[k] > 0 ? O.S[k] + 1 : 0);
        k_prefix_offsets_bs<<<grid_for(B.base[3], kBlock, 4096), kBlock, 0, c->stream>>>(B);
    } else {
        k_prefix_offsets<<<grid_for(O.base[3], kBlock, 4096), kBlock, 0, c->stream>>>(O);
    }
    FZ_LAUNCH_CHECK();
}

// Every segment of the three prefix-sorted tables sorted by time: one launch per length class for
// all tables, the bigflag arrays cleared by one fill.
#ifndef FZ_TS_MID
#define FZ_TS_MID 1
#endif
constexpr bool kTsMid = FZ_TS_MID;  // the 12,288-row time-sort class
#ifndef FZ_TS_CLASSES
#define FZ_TS_CLASSES 0
#endif
#ifndef FZ_SPOS_PREFILL
#define FZ_SPOS_PREFILL 1
#endif
static void time_sort_tables(fz_ctx *c, PrefixSorted *pss, uint8_t *flags) {
    TimeSortTabs T;
    int64_t ntot = 0;
    for (int k = 0; k < 3; ++k) {
        const PrefixSorted &ps = pss[k];
        T.base[k + 1] = T.base[k] + ps.S;
        ntot += ps.n;
    }
    const int64_t S = T.base[3];
    if (S == 0) return;
    for (int k = 0; k < 3; ++k) {
        PrefixSorted &ps = pss[k];
        if (ps.S == 0) continue;
        ps.bigflag = flags + T.base[k];
        TimeSortTab &tb = T.tab[k];
        tb.time = ps.time;
        tb.offs = ps.offs;
        tb.pmask = ps.pmask;
        tb.out = ps.out;
        tb.big = ps.big;
        tb.bigflag = ps.bigflag;
        tb.rows = ps.rows;
        tb.gc = ps.gc;
        tb.fused = ps.big + 6;  // big3[6 + k]
        tb.prefilled = FZ_SPOS_PREFILL;
    }
    // every row's source position starts as kGathered and the bigflag arrays as 0 (store_build's
    // one fill): the bucket sorts overwrite the rows they sort; a segment they leave to the
    // long-segment pass or the merge sort keeps the marker without a write of its own (a workgroup
    // marking config 5's 20.8 M-row giant alone took ~1 ms, the long class's whole launch waiting
    // on it)
    // algorithmic bytes: time 8 read; time 8 + project 4 + source position 4 written; the long
    // class also moves row id 4 + columns in, perm 4 + row 4 + columns out for its rows (added by
    // store_build once their count is read back: fused_gather_bytes)
    ProbeScope probe(c, "seg_time_sort", 24.0 * double(ntot));
    // bucket sorts by length class (each launch skips the others' segments): <= 1024 rows one
    // 256-thread workgroup each (15 KiB of LDS: many per CU), <= 2048 512 threads, <= 4096 1024
    // threads, <= 16384 1024 threads with the keys re-read from memory (LDS: one per CU, a
    // persistent grid); longer or clustered segments are flagged for the merge sort
    // (with helpers the four class launches run side by side on their streams: disjoint segments,
    // disjoint output rows, atomic counters)
    const int nh = store_helpers(c);
    if (nh > 0) store_fork(c);
    auto st = [&](int i) { return i > 0 && i <= nh ? c->helpers[i - 1]->stream : c->stream; };
    // (FZ_TS_CLASSES, experiment builds: 1 - the 512-thread class takes every segment of <= 2048
    // rows, 2 - the 1024-thread class every segment of <= 4096: fewer launches, fewer rows per
    // thread idle... or not)
    if (FZ_TS_CLASSES == 0) {
        k_seg_time_bucket<256, 1024><<<unsigned(S < 16384 ? S : 16384), 256, 0, st(0)>>>(T, 0, false);
        FZ_LAUNCH_CHECK();
    }
    if (FZ_TS_CLASSES <= 1) {
        k_seg_time_bucket<512, 2048><<<unsigned(S < 4096 ? S : 4096), 512, 0, st(1)>>>(T, FZ_TS_CLASSES ? 0 : 1024,
                                                                                        false);
        FZ_LAUNCH_CHECK();
    }
    k_seg_time_bucket<1024, 4096><<<unsigned(S < 2048 ? S : 2048), 1024, 0, st(2)>>>(
        T, FZ_TS_CLASSES == 2 ? 0 : 2048, false);
    FZ_LAUNCH_CHECK();
    // (a workgroup per CU at most; fewer when the tables are too small to hold many long segments)
    const int64_t g16 = ntot / 16384 < 8 ? 8 : (ntot / 16384 > 256 ? 256 : ntot / 16384);
#if FZ_LONG_FUSE
    if (kTsMid) {
        // 4,097-12,288 rows at 12 rows per thread: the 16-row class needs 128 VGPRs and spilled 29
        // of them to scratch; longer segments take the 16-row class after it (same stream)
        k_seg_time_bucket<1024, 12288><<<unsigned(S < g16 ? S : g16), 1024, 0, st(3)>>>(T, 4096, false);
        FZ_LAUNCH_CHECK();
    }
    k_seg_time_bucket<1024, 16384><<<unsigned(S < g16 ? S : g16), 1024, 0, st(3)>>>(T, kTsMid ? 12288 : 4096, true);
#else
    k_seg_time_bucket2<1024, 16384><<<unsigned(S < 2 * g16 ? S : 2 * g16), 1024, 0, st(3)>>>(T, 4096, true);
#endif
    FZ_LAUNCH_CHECK();
    if (nh > 0) store_join(c);
}

// Gather of every sorted row's columns (after all sorts, merge sort included), all tables in one
// launch, each table's blocks in proportion to its rows.
// (the probe's algorithmic bytes are added by the caller once the gathered row counts are known:
// gather_bytes)
static void gather_tables(fz_ctx *c, const PrefixSorted *pss) {
    GatherTabs G;
    for (int k = 0; k < 3; ++k) {
        const PrefixSorted &ps = pss[k];
        const unsigned g = ps.n > 0 ? (grid_for(ps.n, kBlock, 8192) + 7u) & ~7u : 0u;
        G.blk[k + 1] = G.blk[k] + g;
        if (ps.n <= 0) continue;
        G.tab[k] = GatherTab{ps.out.spos, ps.rows, ps.n, ps.gc};
    }
    if (G.blk[3] == 0) return;
    ProbeScope probe(c, "store_gather", 0.0);
    k_store_gather<<<G.blk[3], kBlock, 0, c->stream>>>(G);
    FZ_LAUNCH_CHECK();
}
// algorithmic bytes of one gather pass: spos 4 read per row; for the rows it gathers (gathered[k])
// row id 4 + columns read, perm 4 + columns written
static double gather_bytes(const PrefixSorted *pss, const int64_t *gathered) {
    double bytes = 0.0;
    for (int k = 0; k < 3; ++k)
        if (pss[k].n > 0) bytes += 4.0 * double(pss[k].n) + (8.0 + 2.0 * pss[k].gc.bytes()) * double(gathered[k]);
    return bytes;
}

// ---- long segments (> 16384 rows, config 5's Zipf head): a distribution by time sub-bucket ----
// A segment the bucket sorts flagged is cut by time into B = ceil(len / 8192) sub-buckets (the
// bucket of t is floor((t - min) * B / (span + 1)), NULL last).  The flagged segments' rows are
// copied back to back with their global sub-bucket id as a 32-bit key (k_big_compact: coalesced
// both ways), a stable LSD radix sort on that key moves them (time, row id, columns as payload)
// into sub-bucket order - prefix order kept inside each sub-bucket - and a per-tile LDS histogram
// gives the sub-bucket offsets.  The long bucket class then sorts every sub-bucket as a segment
// (equal times by position in the sub-bucket = prefix position) and writes time, project, row id
// and columns to the segment's output range, coalesced.  This replaces the segmented merge sort
// and the random gather of those rows (config 5: ~8x their algorithmic bytes in HBM traffic), and
// since round 3 also the single-pass scatter into the sub-buckets (whole-segment partial-line
// appends: 8.7 ms per config-5 store).  Declined (the merge sort runs) for a segment of more than
// 8192 x 8192 rows; a sub-bucket that comes out longer than 16384 rows (clustered times) sends the
// table back to the merge sort as well.
#ifndef FZ_BIG_TILE
#define FZ_BIG_TILE 65536
#endif
#ifndef FZ_BIG_BLOCK
#define FZ_BIG_BLOCK 1024
#endif
constexpr int kBigTile = FZ_BIG_TILE;    // rows per histogram / scatter workgroup
constexpr int kBigBlock = FZ_BIG_BLOCK;  // threads of a histogram / scatter workgroup
constexpr int kBigSub = 8192;       // target rows per sub-bucket
constexpr int kBigMaxSub = 8192;    // sub-buckets per segment (LDS bins)
struct BigPlan {
    const int64_t *t_begin, *t_end;  // [tiles] prefix-order row range of the tile
    const int32_t *t_seg;            // [tiles] big-segment index j of the tile
    const int64_t *sbase;            // [nb] first sub-bucket of big segment j
    const int32_t *nsub;             // [nb] sub-buckets of big segment j
    const int64_t *cstart;           // [nb] compact start of big segment j
    long long *lo, *hi;              // [nb] time range (non-NULL)
    int64_t ntiles;
};
__device__ inline int big_sub(int64_t t, long long lo, long long hi, int B) {
    if (t == FZ_TS_NULL || hi < lo) return B - 1;
    const double q = double(uint64_t(t - lo)) * (double(B) / (double(uint64_t(hi) - uint64_t(lo)) + 1.0));
    const int k = int(q);
    return k < B ? k : B - 1;
}
// (the min / max and compaction passes split every tile over kBigSplit workgroups, each with
// several rows' loads in flight per thread: one workgroup per 64 K-row tile left most CUs idle and
// waited on one load at a time - k_big_compact at 15 % of HBM on config 5's giant shard)
constexpr int kBigSplit = 8;
__device__ inline void big_slice(const BigPlan &pl, int64_t tl, int part, int64_t &r0, int64_t &r1) {
    const int64_t b = pl.t_begin[tl], e = pl.t_end[tl], span = (e - b + kBigSplit - 1) / kBigSplit;
    r0 = b + part * span;
    r1 = r0 + span < e ? r0 + span : e;
}
__global__ __launch_bounds__(kBlock) void k_big_minmax(const int64_t *__restrict__ time, BigPlan pl) {
    __shared__ int64_t s_lo[4], s_hi[4];
    for (int64_t g = blockIdx.x; g < pl.ntiles * kBigSplit; g += gridDim.x) {
        const int64_t tl = g / kBigSplit;
        int64_t r0, r1;
        big_slice(pl, tl, int(g % kBigSplit), r0, r1);
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += 4 * kBlock) {
            int64_t t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) t[u] = r + u * kBlock < r1 ? time[r + u * kBlock] : FZ_TS_NULL;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (t[u] == FZ_TS_NULL) continue;
                lo = t[u] < lo ? t[u] : lo;
                hi = t[u] > hi ? t[u] : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane_id() == 0) {
            s_lo[wave_id()] = lo;
            s_hi[wave_id()] = hi;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < 4; ++w) {
                lo = s_lo[w] < lo ? s_lo[w] : lo;
                hi = s_hi[w] > hi ? s_hi[w] : hi;
            }
            const int j = pl.t_seg[tl];
            atomicMin(&pl.lo[j], (long long)lo);
            atomicMax(&pl.hi[j], (long long)hi);
        }
        __syncthreads();
    }
}
__global__ __launch_bounds__(kBigBlock) void k_big_hist(const int64_t *__restrict__ time, BigPlan pl,
                                                     int64_t *__restrict__ cnt) {
    __shared__ uint32_t h[kBigMaxSub];
    for (int64_t tl = blockIdx.x; tl < pl.ntiles; tl += gridDim.x) {
        const int j = pl.t_seg[tl];
        const int B = pl.nsub[j];
        const long long lo = pl.lo[j], hi = pl.hi[j];
        for (int k = threadIdx.x; k < B; k += kBigBlock) h[k] = 0u;
        __syncthreads();
        for (int64_t r = pl.t_begin[tl] + threadIdx.x; r < pl.t_end[tl]; r += kBigBlock)
            atomicAdd(&h[big_sub(time[r], lo, hi, B)], 1u);
        __syncthreads();
        for (int k = threadIdx.x; k < B; k += kBigBlock)
            if (h[k]) atomicAdd(reinterpret_cast<unsigned long long *>(&cnt[pl.sbase[j] + k]), (unsigned long long)h[k]);
        __syncthreads();
    }
}
// The flagged segments' rows copied back to back (compact space, segment order; coalesced both
// ways), each with its sub-bucket id as a 32-bit radix key: a stable radix sort of the compact rows
// then groups them by sub-bucket, rows in prefix order inside each (k_big_compact + radix passes
// instead of a scatter whose per-tile appends of ~30 rows to each of thousands of sub-buckets
// wrote partial lines across the whole segment - 8.7 ms per store at config 5).
struct BigCompact {
    uint32_t *key;
    int64_t *time;
    uint32_t *rows;
    void *col[kMaxGather];
};
__global__ __launch_bounds__(kBlock) void k_big_compact(const int64_t *__restrict__ time,
                                                        const uint32_t *__restrict__ rows, GatherCols gc, BigPlan pl,
                                                        const int64_t *__restrict__ sstart, BigCompact out) {
    constexpr int U = 4;  // rows per thread in flight
    for (int64_t g = blockIdx.x; g < pl.ntiles * kBigSplit; g += gridDim.x) {
        const int64_t tl = g / kBigSplit;
        int64_t r0, r1;
        big_slice(pl, tl, int(g % kBigSplit), r0, r1);
        const int j = pl.t_seg[tl];
        const int B = pl.nsub[j];
        const long long lo = pl.lo[j], hi = pl.hi[j];
        const int64_t shift = pl.cstart[j] - sstart[j];
        const uint32_t kb = uint32_t(pl.sbase[j]);
        for (int64_t r = r0 + threadIdx.x; r < r1; r += U * kBlock) {
            int64_t t[U];
            uint32_t rw[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t ru = r + u * kBlock;
                t[u] = ru < r1 ? time[ru] : 0;
                rw[u] = ru < r1 ? rows[ru] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t ru = r + u * kBlock;
                if (ru >= r1) continue;
                const int64_t d = ru + shift;
                out.key[d] = kb + uint32_t(big_sub(t[u], lo, hi, B));
                out.time[d] = t[u];
                out.rows[d] = rw[u];
            }
        }
        for (int c = 0; c < gc.n; ++c) {  // column by column: one type per loop
            const int sz = gc.size[c];
            for (int64_t r = r0 + threadIdx.x; r < r1; r += U * kBlock) {
                uint64_t x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t ru = r + u * kBlock;
                    x[u] = ru >= r1 ? 0ull
                                    : (sz == 8 ? static_cast<const uint64_t *>(gc.src[c])[ru]
                                               : (sz == 4 ? static_cast<const uint32_t *>(gc.src[c])[ru]
                                                          : static_cast<const uint8_t *>(gc.src[c])[ru]));
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t ru = r + u * kBlock;
                    if (ru >= r1) continue;
                    const int64_t d = ru + shift;
                    if (sz == 8) static_cast<uint64_t *>(out.col[c])[d] = x[u];
                    else if (sz == 4) static_cast<uint32_t *>(out.col[c])[d] = uint32_t(x[u]);
                    else static_cast<uint8_t *>(out.col[c])[d] = uint8_t(x[u]);
                }
            }
        }
    }
}

// The distribution pass for the flagged segments of one prefix-sorted table (bigrows of its rows);
// false: declined or a sub-bucket overflowed - the caller runs the merge sort (which rewrites every
// row of the flagged segments, so nothing written here survives).
static bool big_segments_bucketed(fz_ctx *c, const PrefixSorted &ps, int64_t bigrows) {
    const int64_t S = ps.S;
    std::vector<int64_t> offs(S + 1);
    std::vector<uint8_t> flag(S);
    FZ_HIP(hipMemcpyAsync(offs.data(), ps.offs, size_t(S + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    FZ_HIP(hipMemcpyAsync(flag.data(), ps.bigflag, size_t(S), hipMemcpyDeviceToHost, c->stream));
    sync(c);
    std::vector<int64_t> t_begin, t_end, sbase, cstart, oshift_seg;
    std::vector<int32_t> t_seg, nsub, segid;
    int64_t nsubs = 0, ncomp = 0;
    for (int64_t s = 0; s < S; ++s) {
        const int64_t len = offs[s + 1] - offs[s];
        if (!flag[s] || len <= 0) continue;
        const int64_t B = (len + kBigSub - 1) / kBigSub;
        if (B > kBigMaxSub) return false;
        const int32_t j = int32_t(segid.size());
        segid.push_back(int32_t(s));
        nsub.push_back(int32_t(B));
        sbase.push_back(nsubs);
        cstart.push_back(ncomp);
        for (int64_t r = offs[s]; r < offs[s + 1]; r += kBigTile) {
            t_begin.push_back(r);
            t_end.push_back(r + kBigTile < offs[s + 1] ? r + kBigTile : offs[s + 1]);
            t_seg.push_back(j);
        }
        nsubs += B;
        ncomp += len;
    }
    if (segid.empty() || ncomp != bigrows) return false;
    const int64_t nb = int64_t(segid.size()), nt = int64_t(t_seg.size());
    // per sub-bucket: big segment, output shift (segment start - compact start), project
    std::vector<int64_t> sub_shift(nsubs);
    std::vector<uint32_t> sub_proj(nsubs);
    for (int64_t j = 0; j < nb; ++j)
        for (int64_t k = 0; k < nsub[j]; ++k) {
            sub_shift[sbase[j] + k] = offs[segid[j]] - cstart[j];
            sub_proj[sbase[j] + k] = uint32_t(segid[j]) & ps.pmask;
        }
    auto up = [&](const void *h, size_t bytes) {
        void *d = c->arena.alloc(bytes);
        FZ_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
        return d;
    };
    BigPlan pl;
    pl.t_begin = static_cast<const int64_t *>(up(t_begin.data(), size_t(nt) * 8));
    pl.t_end = static_cast<const int64_t *>(up(t_end.data(), size_t(nt) * 8));
    pl.t_seg = static_cast<const int32_t *>(up(t_seg.data(), size_t(nt) * 4));
    pl.sbase = static_cast<const int64_t *>(up(sbase.data(), size_t(nb) * 8));
    pl.nsub = static_cast<const int32_t *>(up(nsub.data(), size_t(nb) * 4));
    pl.cstart = static_cast<const int64_t *>(up(cstart.data(), size_t(nb) * 8));
    const int64_t *d_shift = static_cast<const int64_t *>(up(sub_shift.data(), size_t(nsubs) * 8));
    const uint32_t *d_sproj = static_cast<const uint32_t *>(up(sub_proj.data(), size_t(nsubs) * 4));
    std::vector<long long> lohi(2 * nb);
    for (int64_t j = 0; j < nb; ++j) {
        lohi[j] = INT64_MAX;
        lohi[nb + j] = INT64_MIN;
    }
    long long *d_lohi = static_cast<long long *>(up(lohi.data(), size_t(2 * nb) * 8));
    pl.lo = d_lohi;
    pl.hi = d_lohi + nb;
    pl.ntiles = nt;
    sync(c);  // the host vectors above die with this function
    const unsigned grid = unsigned(nt < 4096 ? nt : 4096);
    const unsigned gsplit = unsigned(nt * kBigSplit < 8192 ? nt * kBigSplit : 8192);
    k_big_minmax<<<gsplit, kBlock, 0, c->stream>>>(ps.time, pl);
    FZ_LAUNCH_CHECK();
    int64_t *cnt = c->arena.get<int64_t>(nsubs + 1);
    dev_fill(c, cnt, 0, (nsubs + 1) * 8);
    k_big_hist<<<grid, kBigBlock, 0, c->stream>>>(ps.time, pl, cnt);
    FZ_LAUNCH_CHECK();
    // sub-bucket offsets in the compact space (big segments back to back, in segment order)
    int64_t *soffs = c->arena.get<int64_t>(nsubs + 1);
    scan_exclusive_i64(c, cnt, soffs, nsubs + 1, nullptr);
    // the flagged segments' rows back to back with their sub-bucket ids, then the stable radix
    // sort on the id (rows inside a sub-bucket stay in prefix order: equal times are ordered by
    // position in the sub-bucket pass - tie_pos)
    std::vector<int64_t> sst(nb);
    for (int64_t j = 0; j < nb; ++j) sst[j] = offs[segid[j]];
    const int64_t *d_sst = static_cast<const int64_t *>(up(sst.data(), size_t(nb) * 8));
    BigCompact cp;
    cp.key = c->arena.get<uint32_t>(ncomp);
    cp.time = c->arena.get<int64_t>(ncomp);
    cp.rows = c->arena.get<uint32_t>(ncomp);
    for (int k = 0; k < ps.gc.n; ++k) cp.col[k] = c->arena.alloc(size_t(ncomp) * size_t(ps.gc.size[k]));
    {
        // read time 8 + row id 4 + columns; write key 4 + time 8 + row id 4 + columns
        ProbeScope probe(c, "big_compact", (28.0 + 2.0 * ps.gc.bytes()) * double(ncomp));
        k_big_compact<<<gsplit, kBlock, 0, c->stream>>>(ps.time, ps.rows, ps.gc, pl, d_sst, cp);
        FZ_LAUNCH_CHECK();
    }
    RadixPayload rpl;
    rpl.n = 2 + ps.gc.n;
    rpl.in[0] = cp.time;
    rpl.size[0] = 8;
    rpl.in[1] = cp.rows;
    rpl.size[1] = 4;
    for (int k = 0; k < ps.gc.n; ++k) {
        rpl.in[2 + k] = cp.col[k];
        rpl.size[2 + k] = ps.gc.size[k];
    }
    uint32_t *no_vals = nullptr;
    uint32_t *key = cp.key;
    radix_sort_pairs_payload32(c, key, no_vals, ncomp, bits_for(uint64_t(nsubs - 1)), rpl);
    sync(c);  // (the plan's host vectors - sst - die with this function)
    GatherCols cg = ps.gc;  // the sub-bucket sort reads the sorted compact columns, writes the table's
    for (int k = 0; k < ps.gc.n; ++k) cg.src[k] = rpl.out[2 + k];
    // every sub-bucket a segment of the long bucket class; overflow (> 16384 rows) counted in big
    unsigned long long *big = c->arena.get<unsigned long long>(6);
    dev_fill(c, big, 0, 6 * 8);
    uint8_t *flags = c->arena.get<uint8_t>(nsubs);
    dev_fill(c, flags, 0, nsubs);
    TimeSortTabs T;
    TimeSortTab &tb = T.tab[0];
    tb.time = static_cast<const int64_t *>(rpl.out[0]);
    tb.offs = soffs;
    tb.pmask = ps.pmask;
    tb.out = ps.out;
    tb.big = big;
    tb.bigflag = flags;
    tb.rows = static_cast<const uint32_t *>(rpl.out[1]);
    tb.gc = cg;
    tb.oshift = d_shift;
    tb.sproj = d_sproj;
    tb.tie_pos = true;
    T.base[1] = T.base[2] = T.base[3] = nsubs;
    {
        // time 8 read; time 8 + project 4 + marker 4 written; row id 4 + columns read, perm 4 +
        // columns written (the gather is fused)
        ProbeScope probe(c, "big_sub_sort", (32.0 + 2.0 * ps.gc.bytes()) * double(ncomp));
        const unsigned g16 = unsigned(nsubs < 256 ? nsubs : 256);
        if (kTsMid) {  // (sub-buckets of <= 12,288 rows in the class without spills, then the rest)
            k_seg_time_bucket<1024, 12288><<<g16, 1024, 0, c->stream>>>(T, 0, false);
            FZ_LAUNCH_CHECK();
        }
        k_seg_time_bucket<1024, 16384><<<g16, 1024, 0, c->stream>>>(T, kTsMid ? 12288 : 0, true);
        FZ_LAUNCH_CHECK();
    }
    FZ_HIP(hipMemcpyAsync(c->h_pinned + 16, big, 8, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    return c->h_pinned[16] == 0;
}

// The merge-sort path of the store: key = signed time as an order-preserving u64 (NULL =
// INT64_MAX -> ~0: last), stable by row; the sink writes what the register sorts write.
struct StoreTimeKey {
    const int64_t *time;  // prefix-sorted times
    __device__ uint64_t operator()(int64_t i) const { return uint64_t(time[i]) ^ (uint64_t(1) << 63); }
};
struct StoreSink {
    uint32_t pmask;
    TimeSortOut out;
    __device__ void operator()(int32_t s, int64_t q, uint64_t k, uint32_t v) const {
        out.put(q, int64_t(k ^ (uint64_t(1) << 63)), uint32_t(s) & pmask, v);
    }
};

void store_eligibility(fz_ctx *c, bool zeroed);  // fz_rq1.hip

// Point s.t at the sorted copies of every column (row ids become positions; perm keeps the
// caller's ids).
static void materialize_sorted(fz_ctx *c) {
    Store &s = c->store;
    const int64_t nb = s.t.n_builds, nc = s.t.n_cov, ni = s.t.n_issues;
    fz_tables &t = s.t;
    s.bperm = s.b_perm.ensure<int32_t>(nb);
    s.cperm = s.c_perm.ensure<int32_t>(nc);
    s.iperm = s.i_perm.ensure<int32_t>(ni);
    t.b_project = s.b_proj.ensure<uint32_t>(nb);
    t.b_type = s.sb_type.ensure<uint8_t>(nb);
    t.b_result = s.sb_result.ensure<uint8_t>(nb);
    t.b_time = s.b_time.ensure<int64_t>(nb);
    t.b_group = s.sb_group.ensure<int32_t>(nb);
    t.b_rev_canon = s.sb_canon.ensure<int32_t>(nb);
    t.c_project = s.c_proj.ensure<uint32_t>(nc);
    t.c_date = s.c_time.ensure<int64_t>(nc);
    t.c_coverage = s.sc_coverage.ensure<double>(nc);
    t.c_covered = s.sc_covered.ensure<int64_t>(nc);
    t.c_total = s.sc_total.ensure<int64_t>(nc);
    t.c_valid = s.sc_valid.ensure<uint8_t>(nc);
    t.i_number = s.si_number.ensure<int64_t>(ni);
    t.i_project = s.i_proj.ensure<uint32_t>(ni);
    t.i_rts = s.i_time.ensure<int64_t>(ni);
    t.i_status = s.si_status.ensure<uint8_t>(ni);
}

void store_build(fz_ctx *c, const fz_tables *t, fz_store_stats *stats) {
    FZ_CHECK(t != nullptr, "fz_store_build: tables is null");
    FZ_CHECK(c->parent == nullptr, "fz_store_build: a child context reads its parent's store");
    for (fz_ctx *h : c->helpers)  // the build resets the helpers' arenas and runs sorts on them
        FZ_STATE(h->in_call.load() == 0, "fz_store_build: a store-build helper is inside a libfz call of its own "
                                         "(join the helper threads before building the store)");
    FZ_CHECK(t->n_projects >= 0 && t->n_builds >= 0 && t->n_cov >= 0 && t->n_issues >= 0, "negative table size");
    FZ_CHECK(t->n_builds < (int64_t(1) << 31) && t->n_cov < (int64_t(1) << 31) && t->n_issues < (int64_t(1) << 31),
             "tables are limited to 2^31 rows per shard");
    Store &s = c->store;
    s.built = false;
    s.t = *t;
    s.P = t->n_projects;
    c->sort_passes = 0;
    const int64_t P = s.P;
    const int pbits = bits_for(uint64_t(P > 0 ? P - 1 : 0));

    // ONE fill for the whole build: the eligibility counters, the merge-sort counters and the prefix
    // sorts' digit totals (big3), the time sort's bigflag arrays (0) and source positions
    // (kGathered) - sized from the host-known table shapes
    const int tpbits[3] = {pbits + 2, pbits, pbits};
    const int64_t tn[3] = {t->n_builds, t->n_cov, t->n_issues};
    int64_t S_all = 0;
    for (int k = 0; k < 3; ++k) S_all += tn[k] > 0 ? (int64_t(1) << tpbits[k]) : 0;
    // big3[k]: rows of table k in segments left to the merge sort, big3[3 + k]: the longest such
    // segment, big3[6 + k]: rows whose columns the long bucket class gathered (one zeroing for all)
    unsigned long long *big3 = c->arena.get<unsigned long long>(9 + kRadixTabHistWords);
    unsigned long long *hist0 = big3 + 9;  // the prefix sorts' digit totals
    uint8_t *tflags = c->arena.get<uint8_t>(S_all > 0 ? S_all : 1);
    uint32_t *spos[3];
    for (int k = 0; k < 3; ++k) spos[k] = tn[k] > 0 ? c->arena.get<uint32_t>(tn[k]) : nullptr;
    {
        s.n_elig.ensure<int64_t>(2);
        const int64_t pf = FZ_SPOS_PREFILL ? 4 : 0;
        fill_batch(c, {{s.n_elig.ptr, 16, 0},
                       {big3, (9 + kRadixTabHistWords) * 8, 0},
                       {tflags, S_all, 0},
                       {spos[0], tn[0] * pf, 0xff},
                       {spos[1], tn[1] * pf, 0xff},
                       {spos[2], tn[2] * pf, 0xff}});
    }
    // the eligibility histogram reads only the input coverage table: on the third store-build
    // helper beside the prefix sorts (joined with the helpers after them, and again before the
    // build returns)
    bool elig_aside = store_helpers(c) >= 3;
    if (elig_aside) {
        store_fork(c);
        store_eligibility(c->helpers[2], true);
    } else {
        store_eligibility(c, true);
    }
    // the issue-number range (RQ1's ROW_NUMBER dedup key) as per-workgroup partials, read back with
    // the views' counters below (the build's one host round trip) - computed by extra workgroups of
    // the prefix sorts' histogram launch
    const int pblk = int(grid_for(t->n_issues, kBlock * 16, kProBlocks));
    int64_t *ppart = c->arena.get<int64_t>(4 * pblk);
    RadixSideMinMax side;
    side.src = t->i_number;
    side.n = t->n_issues;
    side.part = ppart;
    side.blocks = unsigned(pblk);

    // the three tables: (prefix = [type|]project) LSD passes, then each segment sorted by time in LDS
    struct Tab {
        int64_t n;
        Prefix pre;
        int pbits_total;
        const int64_t *time;
        DevBuf *tm, *pr;
    };
    Tab tabs[3] = {
        {t->n_builds, Prefix{t->b_project, t->b_type, pbits}, pbits + 2, t->b_time, &s.b_time, &s.b_proj},
        {t->n_cov, Prefix{t->c_project, nullptr, pbits}, pbits, t->c_date, &s.c_time, &s.c_proj},
        {t->n_issues, Prefix{t->i_project, nullptr, pbits}, pbits, t->i_rts, &s.i_time, &s.i_proj},
    };
    GatherCols gcs[3];
    {
        const int64_t nb = t->n_builds, nc = t->n_cov, ni = t->n_issues;
        GatherCols &gb = gcs[0];
        gb.n = 4;
        gb.perm = s.b_perm.ensure<int32_t>(nb);
        gb.src[0] = t->b_type, gb.dst[0] = s.sb_type.ensure<uint8_t>(nb), gb.size[0] = 1;
        gb.src[1] = t->b_result, gb.dst[1] = s.sb_result.ensure<uint8_t>(nb), gb.size[1] = 1;
        gb.src[2] = t->b_group, gb.dst[2] = s.sb_group.ensure<int32_t>(nb), gb.size[2] = 4;
        gb.src[3] = t->b_rev_canon, gb.dst[3] = s.sb_canon.ensure<int32_t>(nb), gb.size[3] = 4;
        GatherCols &gv = gcs[1];
        gv.n = 4;
        gv.perm = s.c_perm.ensure<int32_t>(nc);
        gv.src[0] = t->c_coverage, gv.dst[0] = s.sc_coverage.ensure<double>(nc), gv.size[0] = 8;
        gv.src[1] = t->c_covered, gv.dst[1] = s.sc_covered.ensure<int64_t>(nc), gv.size[1] = 8;
        gv.src[2] = t->c_total, gv.dst[2] = s.sc_total.ensure<int64_t>(nc), gv.size[2] = 8;
        gv.src[3] = t->c_valid, gv.dst[3] = s.sc_valid.ensure<uint8_t>(nc), gv.size[3] = 1;
        GatherCols &gi = gcs[2];
        gi.n = 2;
        gi.perm = s.i_perm.ensure<int32_t>(ni);
        gi.src[0] = t->i_number, gi.dst[0] = s.si_number.ensure<int64_t>(ni), gi.size[0] = 8;
        gi.src[1] = t->i_status, gi.dst[1] = s.si_status.ensure<uint8_t>(ni), gi.size[1] = 1;
    }
    PrefixSorted pss[3];
    TableIn tin[3];
    for (int k = 0; k < 3; ++k) {
        Tab &b = tabs[k];
        tin[k] = TableIn{b.n, b.pre, b.pbits_total, b.time, b.tm->ensure<int64_t>(b.n), b.pr->ensure<uint32_t>(b.n),
                         gcs[k], big3 + k};
    }
    prefix_sort_tables(c, tin, pss, hist0, spos, &side);
    time_sort_tables(c, pss, tflags);
    // the views (per-project ranges of the sorted tables): their offsets, longest segments and row
    // counts off the prefix offsets - builds' prefix is type << pbits | project (Fuzzing 0, Coverage 1)
    ViewSrc vs;
    DevBuf *voff[4] = {&s.off_fuzz, &s.off_covb, &s.off_cov, &s.off_iss};
    const int tab_of[4] = {0, 0, 1, 2};
    for (int i = 0; i < 4; ++i) {
        vs.src[i] = pss[tab_of[i]].offs;
        vs.first[i] = i == 1 ? (int64_t(1) << pbits) : 0;
        vs.dst[i] = voff[i]->ensure<int64_t>(P + 1);
    }
    vs.big = big3;
    vs.lim_max = s.n_elig.as<int64_t>() + 1;
    // (the eligibility pass on its helper is long done - the prefix and time sorts outlast it - and
    // its bound travels with this read-back)
    if (elig_aside) {
        store_join(c);
        elig_aside = false;
    }
    // (written straight into the pinned read-back area through its device address: two blit copies
    // fewer in front of the gather and the host's wake-up)
    k_store_views<<<1, kSortBlock, 0, c->stream>>>(vs, P, ppart, pblk, c->d_pinned);
    FZ_LAUNCH_CHECK();
    if (!c->ev_readback) FZ_HIP(hipEventCreateWithFlags(&c->ev_readback, hipEventDisableTiming));
    FZ_HIP(hipEventRecord(c->ev_readback, c->stream));
    // the gather of the short classes' rows, launched before the host reads the counters (rows of
    // segments left to the long-segment pass / merge sort are marked kGathered: skipped here); the
    // host's round trip overlaps it.  (With the direct short classes every bucket-sorted row's
    // columns are written already: no gather unless the merge sort runs, below.)
    if (!(kTsDirect && FZ_SPOS_PREFILL)) gather_tables(c, pss);
#if FZ_SPIN_READBACK
    // spin on the event rather than a blocking wait: the analyses' launches follow this read-back,
    // and a blocking wait's wake-up latency idles the GPU after the gather
    for (;;) {
        const hipError_t q = hipEventQuery(c->ev_readback);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) FZ_HIP(q);
    }
#else
    FZ_HIP(hipEventSynchronize(c->ev_readback));
#endif
    // (no non-NULL number: the empty range min = INT64_MAX > max = INT64_MIN, as the old read-back gave)
    s.num_min = c->h_pinned[17];
    s.num_max = c->h_pinned[18];
    const int64_t maxseg[4] = {c->h_pinned[0], c->h_pinned[1], c->h_pinned[2], c->h_pinned[3]};
    const int64_t bigrows[3] = {c->h_pinned[4], c->h_pinned[5], c->h_pinned[6]};
    const int64_t bigmax[3] = {c->h_pinned[7], c->h_pinned[8], c->h_pinned[9]};
    const int64_t fused[3] = {c->h_pinned[10], c->h_pinned[11], c->h_pinned[12]};
    const int64_t n_fuzz = c->h_pinned[13], n_covb = c->h_pinned[14];
    // (read now: the long-segment pass below reuses the pinned area - its radix sort's digit
    // read-back overwrote word 19, and config 5's shards got the longest segment as their session
    // bound, 39 K instead of 2,960 rows)
    const int64_t lim_rows = c->h_pinned[19];
    {
        auto view = [&](View &v, DevBuf &tmb, DevBuf &prb, int64_t at, int64_t n, DevBuf &offb) {
            v.n = n;
            v.row0 = at;
            v.time = tmb.as<int64_t>() + at;
            v.proj = prb.as<uint32_t>() + at;
            v.offs = offb.as<int64_t>();
        };
        view(s.fuzz, s.b_time, s.b_proj, 0, n_fuzz, s.off_fuzz);
        view(s.covb, s.b_time, s.b_proj, n_fuzz, n_covb, s.off_covb);
        view(s.cov, s.c_time, s.c_proj, 0, t->n_cov, s.off_cov);
        view(s.issues, s.i_time, s.i_proj, 0, t->n_issues, s.off_iss);
    }
    // the probes' algorithmic bytes of the gathers: the long bucket class's fused gather, then the
    // rows the gather above moved (short classes; not the flagged segments' rows)
    int64_t gathered[3];
    for (int k = 0; k < 3; ++k) {
        const double per = 8.0 + 2.0 * pss[k].gc.bytes();  // row 4 + columns in; perm 4 + columns out
        ProbeScope::add_bytes(c, "seg_time_sort", per * double(fused[k]));
        // (the flagged segments' rows are not sorted by these launches - long ones are not read at
        // all: the booking of time_sort_tables counted every row)
        ProbeScope::add_bytes(c, "seg_time_sort", -24.0 * double(bigrows[k]));
        gathered[k] = pss[k].n - fused[k] - bigrows[k];
    }
    ProbeScope::add_bytes(c, "store_gather", gather_bytes(pss, gathered));
    // segments the bucket sorts left (longer than 16384 rows, clustered, or a time span too wide
    // for their packed key): the long-segment distribution pass (which gathers their columns
    // itself), else the segmented merge sort of those rows only, writing the same outputs; merged
    // rows are then gathered by a second gather pass (which redoes the short classes' rows too)
    bool regather = false, bucketed[3] = {false, false, false};
    for (int k = 0; k < 3; ++k) {
        if (bigrows[k] == 0) continue;
        const PrefixSorted &ps = pss[k];
        bucketed[k] = big_segments_bucketed(c, ps, bigrows[k]);
        if (bucketed[k]) continue;
        ProbeScope probe(c, "seg_merge_sort", 36.0 * double(bigrows[k]));
        sort_big_segments(c, ps.offs, ps.S, ps.n, bigmax[k], ps.bigflag, StoreTimeKey{ps.time},
                          StoreSink{ps.pmask, ps.out});
        regather = true;
    }
    if (regather) {
        for (int k = 0; k < 3; ++k) gathered[k] = pss[k].n - fused[k] - (bucketed[k] ? bigrows[k] : 0);
        gather_tables(c, pss);
        ProbeScope::add_bytes(c, "store_gather", gather_bytes(pss, gathered));
    }
    materialize_sorted(c);
    if (elig_aside) store_join(c);
    s.fuzz.max_seg = maxseg[0];
    s.covb.max_seg = maxseg[1];
    s.cov.max_seg = maxseg[2];
    // (at least 1 when the table has rows: the analyses keep one - empty - session, rq2_count:285)
    s.cov.lim_seg = lim_rows < maxseg[2] ? (lim_rows > 0 ? lim_rows : 1) : maxseg[2];
    s.issues.max_seg = maxseg[3];
    s.built = true;
    if (stats) {
        stats->n_projects = P;
        stats->n_fuzz = n_fuzz;
        stats->n_coverage_builds = n_covb;
        stats->max_fuzz_per_project = s.fuzz.max_seg;
        stats->max_cov_per_project = s.cov.max_seg;
        stats->sort_passes = c->sort_passes;
    }
}

}  // namespace fz
