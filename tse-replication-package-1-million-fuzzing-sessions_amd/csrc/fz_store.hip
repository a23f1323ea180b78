// The columnar store: replaces the PostgreSQL tables + (project, time) indexes every RQ query
// scans through dbFile.DB.executeQuery (program/__module/dbFile.py:16-24).
//
// fz_store_build sorts each table once: stable LSD radix passes (fz_prims.hip) on the prefix
// ([build_type |] project) group the rows by segment in row order, then every segment is sorted by
// time - in one workgroup (LDS) when it has <= 4096 rows, through the segmented merge sort
// (fz_segsort.h) otherwise - with NULL timestamps last (PostgreSQL's ASC NULLS LAST) and equal
// times in row order.  The same kernels gather the tables' columns into the sorted order.
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

__global__ __launch_bounds__(kBlock) void k_count_types(const uint8_t *__restrict__ type, int64_t n,
                                                        unsigned long long *__restrict__ cnt) {
    __shared__ int64_t s_tmp[4];
    int64_t a = 0, b = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        a += type[i] == 0;
        b += type[i] == 1;
    }
    a = block_sum(a, s_tmp);
    b = block_sum(b, s_tmp);
    if (threadIdx.x == 0) {
        atomicAdd(&cnt[0], (unsigned long long)a);
        atomicAdd(&cnt[1], (unsigned long long)b);
    }
}


// One workgroup: the longest segment of each of 4 views (out[0..3]) and a copy of the 6
// merge-sort counters (out[4..9]) - one launch and one D2H copy for the host's store stats.
struct Offs4 {
    const int64_t *offs[4];
    const unsigned long long *big;  // [6] merge-sort rows / longest segment per table
};
__global__ __launch_bounds__(kSortBlock) void k_store_stats(Offs4 v, int64_t P, int64_t *__restrict__ out) {
    __shared__ int64_t s_m[kSortBlock / kWave];
    for (int i = 0; i < 4; ++i) {
        int64_t m = 0;
        for (int64_t p = threadIdx.x; p < P; p += kSortBlock) {
            const int64_t l = v.offs[i][p + 1] - v.offs[i][p];
            m = l > m ? l : m;
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
    if (threadIdx.x < 6) out[4 + threadIdx.x] = int64_t(v.big[threadIdx.x]);
}

// ---- fast path: prefix LSD (2 passes) + per-segment LDS sort by (time, row) -----------------
constexpr int kSegSortMax = 4096;
#ifndef FZ_TS_BLOCK
#define FZ_TS_BLOCK 1024
#endif
constexpr int kTimeSortBlock = FZ_TS_BLOCK;  // threads of the per-segment time sort

__global__ __launch_bounds__(kBlock) void k_keys_prefix_rows(Prefix pre, int64_t n, uint64_t *__restrict__ keys,
                                                             uint32_t *__restrict__ vals) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        keys[i] = pre(i);
        vals[i] = uint32_t(i);
    }
}

// offs[s] = first position of prefix s in the prefix-sorted keys (s in [0, S]): row i starts the
// prefixes (keys[i-1], keys[i]]; one coalesced read of the keys instead of a binary search per s.
__global__ __launch_bounds__(kBlock) void k_prefix_offsets(const uint64_t *__restrict__ keys, int64_t n, int64_t S,
                                                           int64_t *__restrict__ offs) {
    const int64_t first = int64_t(keys[0]), last = int64_t(keys[n - 1]);  // n >= 1, keys < S
    const int64_t span = n > S + 1 ? n : S + 1;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < span; i += int64_t(gridDim.x) * kBlock) {
        if (i <= S) {
            if (i <= first) offs[i] = 0;
            else if (i > last) offs[i] = n;
        }
        if (i > 0 && i < n) {
            const int64_t pp = int64_t(keys[i - 1]), pc = int64_t(keys[i]);
            for (int64_t q = pp + 1; q <= pc && q <= S; ++q) offs[q] = i;
        }
    }
}

// One workgroup per prefix segment, already in row order: bitonic sort in LDS of one packed u64 per
// row, (time - segment min) << 12 | position (NULL times and the power-of-two pads get the top time
// field): the position tie-break keeps equal times in row order (stable), and each compare-exchange
// moves one word instead of a (time, position) pair.  Segments longer than MAXN rows, or whose
// times span 2^52 us or more, are counted into *big (the host re-sorts that table on the full-key
// path).  (Size-class variants - 256 / 512 / 1024 threads for <= 1024 / 2048 / 4096 rows - measured
// slower in total: each class launch still walks every segment.)
// Columns the time sort gathers into sorted order as it writes each segment (the materialisation
// of the sorted store, fused: the random reads overlap other workgroups' sorting).  With perm set,
// the kernel writes orow[k] = k (row id = sorted position) and perm[k] = the source row.
constexpr int kMaxGather = 4;
struct GatherCols {
    int n = 0;
    const void *src[kMaxGather] = {};
    void *dst[kMaxGather] = {};
    int size[kMaxGather] = {};  // bytes: 1, 4 or 8
    int32_t *perm = nullptr;
};

constexpr int kTsPosBits = 12;  // positions < 4096 = kSegSortMax
constexpr uint64_t kTsTop = (uint64_t(1) << (64 - kTsPosBits)) - 1;  // time field of NULL / pad
template <int BS, int MAXN>
__global__ __launch_bounds__(BS) void k_seg_time_sort(const uint32_t *__restrict__ rows, const int64_t *__restrict__ time,
                                                      const int64_t *__restrict__ offs, int64_t S, uint32_t pmask,
                                                      int32_t *__restrict__ orow, int64_t *__restrict__ otime,
                                                      uint32_t *__restrict__ oproj, unsigned long long *__restrict__ big,
                                                      uint8_t *__restrict__ bigflag, GatherCols gc) {
    static_assert(MAXN <= (1 << kTsPosBits), "positions must fit the key");
    __shared__ uint64_t sk[MAXN];
    __shared__ int64_t s_lo[BS / kWave], s_hi[BS / kWave];
    const int tid = threadIdx.x;

    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t b = offs[s];
        const int64_t len = offs[s + 1] - b;
        if (len <= 0) continue;
        if (len > MAXN) {
            if (tid == 0) {
                atomicAdd(big, (unsigned long long)len);
                atomicMax(big + 3, (unsigned long long)len);
                bigflag[s] = 1;
            }
            continue;
        }
        const int n = int(len);
        int np2 = 1;
        while (np2 < n) np2 <<= 1;
        // gather the times (raw bits parked in sk) and their min / max over non-NULL rows
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int i = tid; i < n; i += BS) {
            const int64_t t = time[rows[b + i]];
            sk[i] = uint64_t(t);
            if (t != FZ_TS_NULL) {
                lo = t < lo ? t : lo;
                hi = t > hi ? t : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane_id() == 0) {
            s_lo[wave_id()] = lo;
            s_hi[wave_id()] = hi;
        }
        __syncthreads();
        lo = INT64_MAX;
        hi = INT64_MIN;
        for (int w = 0; w < BS / kWave; ++w) {
            lo = s_lo[w] < lo ? s_lo[w] : lo;
            hi = s_hi[w] > hi ? s_hi[w] : hi;
        }
        if (hi >= lo && uint64_t(hi) - uint64_t(lo) >= kTsTop) {  // span too wide for the key
            if (tid == 0) {
                atomicAdd(big, (unsigned long long)len);
                atomicMax(big + 3, (unsigned long long)len);
                bigflag[s] = 1;
            }
            __syncthreads();
            continue;
        }
        for (int i = tid; i < np2; i += BS) {
            const int64_t t = i < n ? int64_t(sk[i]) : FZ_TS_NULL;
            const uint64_t f = t == FZ_TS_NULL ? kTsTop : uint64_t(t - lo);
            sk[i] = (f << kTsPosBits) | uint64_t(i);
        }
        __syncthreads();
        for (int k = 2; k <= np2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = tid; t < (np2 >> 1); t += BS) {  // every thread owns pairs
                    const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ixj = i + j;  // j = 2^m
                    const uint64_t ka = sk[i], kb = sk[ixj];
                    if ((ka > kb) == ((i & k) == 0)) {
                        sk[i] = kb;
                        sk[ixj] = ka;
                    }
                }
                bitonic_stage_sync(k, j, np2);
            }
        }
        const uint32_t p = uint32_t(s) & pmask;
        for (int i = tid; i < n; i += BS) {
            const uint64_t key = sk[i];
            const uint64_t f = key >> kTsPosBits;
            const int64_t q = b + i;
            const int32_t r = int32_t(rows[b + int64_t(key & ((1u << kTsPosBits) - 1))]);
            otime[q] = f == kTsTop ? FZ_TS_NULL : lo + int64_t(f);
            oproj[q] = p;
            if (gc.perm) {
                gc.perm[q] = r;
                orow[q] = int32_t(q);
                for (int j = 0; j < gc.n; ++j) {
                    if (gc.size[j] == 8)
                        static_cast<uint64_t *>(gc.dst[j])[q] = static_cast<const uint64_t *>(gc.src[j])[r];
                    else if (gc.size[j] == 4)
                        static_cast<uint32_t *>(gc.dst[j])[q] = static_cast<const uint32_t *>(gc.src[j])[r];
                    else
                        static_cast<uint8_t *>(gc.dst[j])[q] = static_cast<const uint8_t *>(gc.src[j])[r];
                }
            } else {
                orow[q] = r;
            }
        }
        __syncthreads();
    }
}

// Sorts by (prefix, time, row); adds to the (zeroed) device counter *big the rows in segments too
// long for LDS (and big[3] = the longest such segment, bigflag[s] = 1): the caller sorts those
// through the segmented merge sort.
// nonempty_bound: host upper bound on the number of non-empty segments (picks the workgroup size).
constexpr int kTimeSortSmallBlock = 256;
constexpr int kTimeSortSmallMean = 256;  // mean rows per segment at or below which it is used
struct PrefixSorted {
    int64_t S = 0;
    const int64_t *offs = nullptr;   // [S + 1] segment offsets of the prefix-sorted rows
    const uint32_t *rows = nullptr;  // row ids in (prefix, row) order
    uint8_t *bigflag = nullptr;      // [S] 1: the segment is left to the merge sort
};
static PrefixSorted sort_table_fast(fz_ctx *c, int64_t n, Prefix pre, int prefix_bits, const int64_t *time,
                                    int32_t *orow, int64_t *otime, uint32_t *oproj, const GatherCols &gc,
                                    unsigned long long *big, int64_t nonempty_bound) {
    PrefixSorted ps;
    if (n <= 0) return ps;
    uint64_t *keys = c->arena.get<uint64_t>(n);
    uint32_t *vals = c->arena.get<uint32_t>(n);
    const unsigned g = grid_for(n, kBlock, 4096);
    k_keys_prefix_rows<<<g, kBlock, 0, c->stream>>>(pre, n, keys, vals);
    FZ_LAUNCH_CHECK();
    radix_sort_pairs_swap(c, keys, vals, n, prefix_bits);
    const int64_t S = int64_t(1) << prefix_bits;
    int64_t *offs = c->arena.get<int64_t>(S + 1);
    k_prefix_offsets<<<grid_for(n > S + 1 ? n : S + 1, kBlock, 4096), kBlock, 0, c->stream>>>(keys, n, S, offs);
    FZ_LAUNCH_CHECK();
    uint8_t *bigflag = c->arena.get<uint8_t>(S);
    FZ_HIP(hipMemsetAsync(bigflag, 0, size_t(S), c->stream));
    ps.S = S;
    ps.offs = offs;
    ps.rows = vals;
    ps.bigflag = bigflag;
    const uint32_t pmask = pre.pbits >= 32 ? 0xffffffffu : uint32_t((1ull << pre.pbits) - 1ull);
    {
        ProbeScope ps(c, "seg_time_sort", 28.0 * double(n));  // row 4 + gathered time 8 + out 16 B
        const unsigned g = unsigned(S < 16384 ? S : 16384);
        if (n <= int64_t(kTimeSortSmallMean) * nonempty_bound) {
            // short segments on average (issues: ~65 rows per project): 256-thread workgroups, five
            // per CU by LDS instead of two, so the whole table sorts in one round of the grid
            k_seg_time_sort<kTimeSortSmallBlock, kSegSortMax><<<g, kTimeSortSmallBlock, 0, c->stream>>>(
                vals, time, offs, S, pmask, orow, otime, oproj, big, bigflag, gc);
        } else {
            k_seg_time_sort<kTimeSortBlock, kSegSortMax><<<g, kTimeSortBlock, 0, c->stream>>>(
                vals, time, offs, S, pmask, orow, otime, oproj, big, bigflag, gc);
        }
        FZ_LAUNCH_CHECK();
    }
    return ps;
}

// The merge-sort path of the store: key = signed time as an order-preserving u64 (NULL =
// INT64_MAX -> ~0: last), stable by row; the sink writes what k_seg_time_sort writes for a short
// segment (time, project, row = position, perm = source row, gathered columns).
struct StoreTimeKey {
    const int64_t *time;
    const uint32_t *rows;
    __device__ uint64_t operator()(int64_t i) const { return uint64_t(time[rows[i]]) ^ (uint64_t(1) << 63); }
};
struct StoreSink {
    const uint32_t *rows;
    uint32_t pmask;
    int32_t *orow;
    int64_t *otime;
    uint32_t *oproj;
    GatherCols gc;
    __device__ void operator()(int32_t s, int64_t q, uint64_t k, uint32_t v) const {
        const int32_t r = int32_t(rows[v]);
        otime[q] = int64_t(k ^ (uint64_t(1) << 63));
        oproj[q] = uint32_t(s) & pmask;
        gc.perm[q] = r;
        orow[q] = int32_t(q);
        for (int j = 0; j < gc.n; ++j) {
            if (gc.size[j] == 8)
                static_cast<uint64_t *>(gc.dst[j])[q] = static_cast<const uint64_t *>(gc.src[j])[r];
            else if (gc.size[j] == 4)
                static_cast<uint32_t *>(gc.dst[j])[q] = static_cast<const uint32_t *>(gc.src[j])[r];
            else
                static_cast<uint8_t *>(gc.dst[j])[q] = static_cast<const uint8_t *>(gc.src[j])[r];
        }
    }
};

static View make_view(fz_ctx *c, const int32_t *row, const int64_t *time, const uint32_t *proj, int64_t n, int64_t P,
                      DevBuf &offbuf) {
    View v;
    v.n = n;
    v.row = row;
    v.time = time;
    v.proj = proj;
    int64_t *offs = offbuf.ensure<int64_t>(P + 1);
    segment_offsets(c, proj, n, P, offs);
    v.offs = offs;
    return v;
}

void store_eligibility(fz_ctx *c);  // fz_rq1.hip

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
    FZ_CHECK(t->n_projects >= 0 && t->n_builds >= 0 && t->n_cov >= 0 && t->n_issues >= 0, "negative table size");
    FZ_CHECK(t->n_builds < (int64_t(1) << 31) && t->n_cov < (int64_t(1) << 31) && t->n_issues < (int64_t(1) << 31),
             "tables are limited to 2^31 rows per shard");
    Store &s = c->store;
    s.built = false;
    s.t = *t;
    s.P = t->n_projects;
    s.passes = 0;
    const int64_t P = s.P;
    const int pbits = bits_for(uint64_t(P > 0 ? P - 1 : 0));

    // one host round trip: the issue-number range (RQ1's ROW_NUMBER dedup key) + build-type counts
    int64_t mm[2];
    const int64_t *cols[1] = {t->i_number};
    const int64_t ns[1] = {t->n_issues};
    store_eligibility(c);
    unsigned long long *tcnt = c->arena.get<unsigned long long>(2);
    FZ_HIP(hipMemsetAsync(tcnt, 0, 16, c->stream));
    if (t->n_builds > 0) {
        k_count_types<<<grid_for(t->n_builds, kBlock * 8, 512), kBlock, 0, c->stream>>>(t->b_type, t->n_builds, tcnt);
        FZ_LAUNCH_CHECK();
    }
    minmax_i64_to_host(c, cols, ns, 1, mm);  // syncs the stream
    s.num_min = mm[0];
    s.num_max = mm[1];
    unsigned long long hcnt[2];
    FZ_HIP(hipMemcpy(hcnt, tcnt, 16, hipMemcpyDeviceToHost));
    const int64_t n_fuzz = int64_t(hcnt[0]), n_covb = int64_t(hcnt[1]);

    // the three tables: (prefix = [type|]project) LSD passes, then each segment sorted by time in LDS
    struct Tab {
        int64_t n;
        Prefix pre;
        int pbits_total;
        const int64_t *time;
        DevBuf *row, *tm, *pr;
    };
    Tab tabs[3] = {
        {t->n_builds, Prefix{t->b_project, t->b_type, pbits}, pbits + 2, t->b_time, &s.b_row, &s.b_time,
         &s.b_proj},
        {t->n_cov, Prefix{t->c_project, nullptr, pbits}, pbits, t->c_date, &s.c_row, &s.c_time, &s.c_proj},
        {t->n_issues, Prefix{t->i_project, nullptr, pbits}, pbits, t->i_rts, &s.i_row, &s.i_time,
         &s.i_proj},
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
    // big3[k]: rows of table k in segments left to the merge sort, big3[3 + k]: the longest such
    // segment (one zeroing for all six counters)
    unsigned long long *big3 = c->arena.get<unsigned long long>(6);
    FZ_HIP(hipMemsetAsync(big3, 0, 6 * 8, c->stream));
    PrefixSorted pss[3];
    for (int k = 0; k < 3; ++k) {
        Tab &b = tabs[k];
        // non-empty segments: at most one per project (and build type: 2 prefix bits for builds)
        const int64_t segs = int64_t(P > 0 ? P : 1) * (k == 0 ? 4 : 1);
        pss[k] = sort_table_fast(c, b.n, b.pre, b.pbits_total, b.time, b.row->ensure<int32_t>(b.n),
                                 b.tm->ensure<int64_t>(b.n), b.pr->ensure<uint32_t>(b.n), gcs[k], big3 + k, segs);
    }
    auto make_views = [&]() {
        int32_t *row = s.b_row.as<int32_t>();
        int64_t *tm = s.b_time.as<int64_t>();
        uint32_t *pr = s.b_proj.as<uint32_t>();
        s.fuzz = make_view(c, row, tm, pr, n_fuzz, P, s.off_fuzz);
        s.covb = make_view(c, row + n_fuzz, tm + n_fuzz, pr + n_fuzz, n_covb, P, s.off_covb);
        s.cov = make_view(c, s.c_row.as<int32_t>(), s.c_time.as<int64_t>(), s.c_proj.as<uint32_t>(), t->n_cov, P,
                          s.off_cov);
        s.issues = make_view(c, s.i_row.as<int32_t>(), s.i_time.as<int64_t>(), s.i_proj.as<uint32_t>(), t->n_issues,
                             P, s.off_iss);
    };
    // longest segments (sizes the per-iteration outputs) + the merge-sort counters
    int64_t *mx = c->arena.get<int64_t>(10);
    auto read_stats = [&]() {
        Offs4 v{{s.fuzz.offs, s.covb.offs, s.cov.offs, s.issues.offs}, big3};
        k_store_stats<<<1, kSortBlock, 0, c->stream>>>(v, P, mx);
        FZ_LAUNCH_CHECK();
        FZ_HIP(hipMemcpyAsync(c->h_pinned, mx, 10 * 8, hipMemcpyDeviceToHost, c->stream));
        sync(c);
    };
    // segments the LDS time sort left (longer than 4096 rows, or a time span too wide for its
    // packed key): segmented merge sort of those rows only, writing the same outputs
    make_views();
    read_stats();
    const int64_t bigrows[3] = {c->h_pinned[4], c->h_pinned[5], c->h_pinned[6]};
    const int64_t bigmax[3] = {c->h_pinned[7], c->h_pinned[8], c->h_pinned[9]};
    bool redo = false;
    for (int k = 0; k < 3; ++k) {
        if (bigrows[k] == 0) continue;
        Tab &b = tabs[k];
        const PrefixSorted &ps = pss[k];
        const uint32_t pmask = b.pre.pbits >= 32 ? 0xffffffffu : uint32_t((1ull << b.pre.pbits) - 1ull);
        ProbeScope probe(c, "seg_merge_sort", 36.0 * double(bigrows[k]));
        sort_big_segments(c, ps.offs, ps.S, b.n, bigmax[k], ps.bigflag, StoreTimeKey{b.time, ps.rows},
                          StoreSink{ps.rows, pmask, b.row->as<int32_t>(), b.tm->as<int64_t>(), b.pr->as<uint32_t>(),
                                    gcs[k]});
        redo = true;
    }
    if (redo) {  // the merged segments' projects are written now
        make_views();
        read_stats();
    }
    materialize_sorted(c);
    s.fuzz.max_seg = c->h_pinned[0];
    s.covb.max_seg = c->h_pinned[1];
    s.cov.max_seg = c->h_pinned[2];
    s.issues.max_seg = c->h_pinned[3];
    s.built = true;
    if (stats) {
        stats->n_projects = P;
        stats->n_fuzz = n_fuzz;
        stats->n_coverage_builds = n_covb;
        stats->max_fuzz_per_project = s.fuzz.max_seg;
        stats->max_cov_per_project = s.cov.max_seg;
        stats->sort_passes = s.passes;
    }
}

}  // namespace fz
