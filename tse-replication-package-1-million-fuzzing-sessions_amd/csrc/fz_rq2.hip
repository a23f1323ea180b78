// RQ2 - coverage trends per project and per session index (rq2_coverage_count.py:244-483).
//
//   878 x GET_TOTAL_COVERAGE_EACH_PROJECT (queries1.py:120-129) -> one filtered view of the
//        (project, date)-sorted coverage store
//   trend = covered/total*100 (:300-303)                         -> elementwise fp64
//   shapiro / spearmanr per project (:305-322)                   -> segmented sort + tie ranks +
//        chunked segmented reductions (fz_series.hip)
//   coverage_by_session_index transpose (:330-333)               -> ragged transpose (fz_transpose.h)
//   per-session mean/median/percentiles (:139-152, :439-440)     -> order-statistic selection per session
//   spearman/shapiro of the median trend (:443-458)              -> the same kernels, one segment
#include "fz_seg.h"
#include "fz_stats.h"
#include "fz_transpose.h"

namespace fz {

constexpr int64_t kLimitUs2 = 1736294400000000LL;  // '2025-01-08'

void eligible_projects(fz_ctx *c, uint8_t *elig, int64_t *d_count, std::initializer_list<Fill> fills = {});

struct CovTrendRows {  // coverage IS NOT NULL AND coverage != 0 AND DATE(date) < LIMIT, eligible only
    static constexpr int kBytes = 21;  // column bytes read per row (filter_compact probe)
    const uint32_t *proj;
    const double *cov;
    const uint8_t *valid;
    const int64_t *date;
    const uint8_t *elig;
    __device__ bool operator()(int32_t r) const {
        return bool(valid[r] & FZ_VALID_COVERAGE) & (cov[r] != 0.0) & (date[r] < kLimitUs2) & bool(elig[proj[r]]);
    }
};
struct NonZeroTotal {  // `if x[1] != 0` (:300-303); a NULL total (stored 0) passes: None != 0
    static constexpr int kBytes = 9;  // column bytes read per row (filter_compact probe)
    const int64_t *total;
    const uint8_t *valid;
    __device__ bool operator()(int32_t r) const { return (total[r] != 0) | !(valid[r] & FZ_VALID_TOTAL); }
};
// the trend rows (CovTrendRows, then NonZeroTotal) in one filter pass
struct TrendRows {
    static constexpr int kBytes = 30;  // column bytes read per row (filter_compact probe)
    CovTrendRows v;
    NonZeroTotal nz;
    __device__ bool operator()(int32_t r) const { return bool(int(v(r)) & int(nz(r))); }
};
// raw_n[p] (the project's CovTrendRows rows, the fetched rows of :291-298) = its trend rows + the
// fetched rows the zero-total test drops: only those (rare) are counted in the filter pass - a count
// of every fetched row would put one atomic per wave on the same project's counter
struct CountZeroTotal {
    static constexpr bool on = true;
    int64_t *out;
    CovTrendRows v;
    NonZeroTotal nz;
    __device__ bool operator()(int32_t r) const { return bool(int(v(r)) & int(!nz(r))); }
};

// What the trend filter writes per kept row: the trend value covered / total * 100 (:300-303) and
// the project (the per-project sort's segment id) - read from the row while it is filtered, instead
// of a (row, time, project) copy and a map that gathers the two line counts through it.  A NULL line
// count makes the reference's float(None) raise (:301): counted, NaN stored.
struct TrendEmit {
    static constexpr bool kTime = false;
    double *tv;
    uint32_t *oproj;
    const int64_t *covered, *total;
    const uint8_t *valid;
    int64_t *null_lines;
    __device__ void operator()(int64_t q, int32_t r, int64_t, uint32_t pj) const {
        oproj[q] = pj;
        if ((valid[r] & (FZ_VALID_COVERED | FZ_VALID_TOTAL)) != (FZ_VALID_COVERED | FZ_VALID_TOTAL)) {
            atomicAdd(reinterpret_cast<unsigned long long *>(null_lines), 1ull);
            tv[q] = NAN;
            return;
        }
        tv[q] = double(covered[r]) / double(total[r]) * 100.0;
    }
};

// statistics.mean / median + np.percentile(5, 25, 50, 75, 95) of every session segment; sessions
// with >= 100 values counted into *d_ge100 (which must be zero on entry)
// (*d_ge100 zero on entry)
// (average2 optional: a second copy of the averages)
void session_stats(fz_ctx *c, const double *sv, const Segs &ses, double *average, double *median, double *pcts,
                   int64_t *d_ge100, double *average2 = nullptr) {
    const double q5[5] = {5.0, 25.0, 50.0, 75.0, 95.0};
    if (seg_qstats_ok(ses)) {  // order statistics by selection: no sorted copy of the sessions
        seg_qstats(c, sv, ses, q5, 5, average, median, pcts, d_ge100, average2);
        return;
    }
    ChunkedSegs cs2 = chunked(c, ses);
    SortedSegs ss2 = seg_sort_f64(c, sv, ses, nullptr);
    const int64_t *soffs = ses.offs;
    per_seg(c, ses.S, [=] __device__(int64_t i) {
        if (soffs[i + 1] - soffs[i] >= 100) atomic_add_i64(d_ge100, 1);
    });
    seg_mean(c, cs2, sv, average);
    seg_percentiles(c, ses, ss2.val, q5, 5, pcts, median);
    if (average2) dev_copy(c, average2, average, (ses.S > 0 ? ses.S : 1) * 8);
}

// spearmanr(range(n), x) and shapiro(x) of x[0, *d_n) (n_cap >= *d_n) -> out = rho, p, W, p
void series_tests(fz_ctx *c, const double *x, int64_t n_cap, const int64_t *d_n, double *out) {
    if (series_small_ok(n_cap)) {  // one workgroup: sort, Spearman and Shapiro-Wilk in LDS
        series_small(c, x, d_n, out, out + 1, out + 2, out + 3);
        return;
    }
    Segs one{1, single_segment(c, d_n), n_cap};
    ChunkedSegs cs3 = chunked(c, one);
    int32_t *sg3 = segment_ids(c, one);
    SortedSegs ss3 = seg_sort_f64(c, x, one, sg3);
    spearman_shapiro_sorted(c, cs3, sg3, ss3, x, out, out + 1, out + 2, out + 3);
}

void spearman_index_seg(fz_ctx *c, const double *x, int64_t n, const int64_t *offs, int64_t S, int64_t max_len,
                        double *rho, double *p) {
    Segs sg{S, offs, n > 0 ? n : 1, max_len};
    ChunkedSegs cs = chunked(c, sg);
    int32_t *id = segment_ids(c, sg);
    SortedSegs ss = seg_sort_f64(c, x, sg, id);
    spearman_index_sorted(c, cs, id, ss, rho, p);
}

__global__ void k_session_keys(const int64_t *__restrict__ sid, int64_t n, uint32_t *__restrict__ keys) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
        keys[i] = uint32_t(sid[i]);
}

void rq2_session_stats(fz_ctx *c, const double *values, const int64_t *session_ids, int64_t n, int64_t S,
                       int64_t max_len, double *average, double *median, double *pcts, int64_t *n_ge100) {
    hipStream_t st = c->stream;
    dev_fill(c, n_ge100, 0, 8);
    FZ_CHECK(S < (int64_t(1) << 32), "fz_rq2_session_stats: too many sessions");
    uint32_t *key = c->arena.get<uint32_t>(n);
    const double *svals = values;  // the values ride along as the sort's payload (no gather after)
    if (n > 0) {
        k_session_keys<<<grid_for(n), kBlock, 0, st>>>(session_ids, n, key);
        FZ_LAUNCH_CHECK();
        RadixPayload pl;
        pl.n = 1;
        pl.in[0] = values;
        pl.size[0] = 8;
        uint32_t *no_vals = nullptr;
        // stable: input order kept per session (32-bit keys: session index < 2^32)
        radix_sort_pairs_payload32(c, key, no_vals, n, bits_for(uint64_t(S)), pl);
        svals = static_cast<const double *>(pl.out[0]);
    }
    double *sv = c->arena.get<double>(n);
    uint32_t *sid = c->arena.get<uint32_t>(n);
    int64_t *d_n = c->arena.get<int64_t>(1);
    int64_t *offs = c->arena.get<int64_t>(S + 1);
    map_n(c, n > 0 ? n : 1, nullptr, [=] __device__(int64_t k) {
        if (k == 0) *d_n = n;
        if (k < n) {
            sv[k] = svals[k];
            sid[k] = uint32_t(key[k]);
        }
    });
    segment_offsets_dn(c, sid, d_n, n > 0 ? n : 1, S, offs);
    Segs ses{S, offs, n, max_len};
    session_stats(c, sv, ses, average, median, pcts, n_ge100);
}

// The same from values already grouped by session (offs [S + 1], offs[0] = 0) - a shard's
// fz_rq2_count_ex output or what fz_runs_merge made of the exchanged runs: no key pass, no sort
void rq2_session_stats_grouped(fz_ctx *c, const double *values, const int64_t *offs, int64_t n, int64_t S,
                               int64_t max_len, double *average, double *median, double *pcts, int64_t *n_ge100) {
    dev_fill(c, n_ge100, 0, 8);
    FZ_CHECK(S < (int64_t(1) << 31), "fz_rq2_session_stats_grouped: too many sessions");
    Segs ses{S, offs, n, max_len};
    session_stats(c, values, ses, average, median, pcts, n_ge100);
}

void rq2_count(fz_ctx *c, uint32_t flags, const fz_rq2_count_out *o) {
    Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_rq2_count: call fz_store_build first");
    FZ_CHECK(o && o->counts && o->scalars && o->eligible && o->raw_n && o->n_trend && o->sw_w && o->sw_p && o->corr &&
                 o->session_offsets && o->session_values && o->average_trend && o->median_trend &&
                 o->dist_percentiles && o->dist_mean,
             "fz_rq2_count: null output buffer");
    const fz_tables &t = s.t;
    const int64_t P = s.P;
    const int64_t M = s.cov.lim_seg;  // longest possible trend (rows before the date limit)
    const int64_t NC = s.cov.n;
    // (the counters and raw_n zeroed in the eligibility copy's launch)
    eligible_projects(c, o->eligible, o->counts + FZ_RQ2C_ELIGIBLE,
                      {{o->counts, FZ_RQ2C_NCOUNTS * 8, 0}, {o->raw_n, (P > 0 ? P : 1) * 8, 0}});
    // the trend rows in one pass over the coverage view; the fetched rows per project (raw_n)
    // counted on the way instead of a first filter whose rows a second one would re-read
    int64_t *counts = o->counts;
    int64_t *raw_n = o->raw_n, *n_trend = o->n_trend;
    TmpView T;
    const CovTrendRows vrows{t.c_project, t.c_coverage, t.c_valid, t.c_date, o->eligible};
    const NonZeroTotal nzt{t.c_total, t.c_valid};
    // trend values in (project, date) order, written by the filter itself (project-major output:
    // straight into the caller's session_values - the runs of the sharded session exchange)
    const bool pmajor = (flags & FZ_RQ2C_PROJECT_MAJOR) && (flags & FZ_RQ2C_SKIP_SESSION_STATS);
    double *tv = pmajor ? o->session_values : c->arena.get<double>(NC);
    T.proj = c->arena.get<uint32_t>(NC);
    const TrendEmit te{tv, T.proj, t.c_covered, t.c_total, t.c_valid, counts + FZ_RQ2C_NULL_LINES};
    // (an index range scan: the eligible projects' rows before the date limit only; per kept row:
    // covered 8 + total 8 + valid 1 read, value 8 + project 4 written)
    filter_view(c, s.cov, NC, P, TrendRows{vrows, nzt}, T, nullptr,
                Selection::segments(o->eligible, 1, nullptr, s.cov.offs, kLimitUs2),
                CountZeroTotal{raw_n, vrows, nzt}, &te, 29.0);
    const int64_t *toffs = T.offs;
    int64_t *d_nt = T.d_n;
    per_seg(c, P, [=] __device__(int64_t p) {
        const int64_t nt = toffs[p + 1] - toffs[p];
        raw_n[p] += nt;
        n_trend[p] = nt;
        // (sessions start as [[]] (:285): at least one - the max taken with 1)
        atomicMax(reinterpret_cast<unsigned long long *>(&counts[FZ_RQ2C_SESSIONS]),
                  (unsigned long long)(nt > 1 ? nt : 1));
        if (p == 0) counts[FZ_RQ2C_VALUES] = *d_nt;
    });
    if (P <= 0)
        map_n(c, 1, nullptr, [=] __device__(int64_t) {
            counts[FZ_RQ2C_VALUES] = *d_nt;
            counts[FZ_RQ2C_SESSIONS] = 1;
        });

    // per-project Spearman (vs index) and Shapiro-Wilk
    Segs sp{P, T.offs, NC, M};
    ChunkedSegs cs = chunked(c, sp);
    const int32_t *segid = reinterpret_cast<const int32_t *>(T.proj);
    SortedSegs ss = seg_sort_f64(c, tv, sp, segid);
    spearman_shapiro_sorted(c, cs, segid, ss, tv, o->corr, nullptr, o->sw_w, o->sw_p);
    if (pmajor) return;

    // coverage_by_session_index (:329-333): session i = value i of every project longer than i, in
    // project order - the ragged transpose (fz_transpose.h) moves each value straight to its slot
    double *sv = o->session_values;
    if (ragged_transpose_ok(P, M, 1)) {
        const double *tvc = tv;
        ragged_transpose<1>(c, T.offs, P, M, NC, [=] __device__(int64_t j) { return tvc[j]; }, RtOneGroup{}, sv,
                            o->session_offsets);
    } else {
        // (tables past the transpose's bounds) order by (index within project, project): the values
        // are in project order, so a stable radix sort on the index alone keeps projects in order
        const int ibits = bits_for(uint64_t(M));
        uint32_t *key = c->arena.get<uint32_t>(NC);  // (an index within a project: < 2^31 rows)
        const uint32_t *tproj = T.proj;
        map_n(c, NC, nullptr, [=] __device__(int64_t j) {
            const int64_t live = *d_nt;
            key[j] = j < live ? uint32_t(j - toffs[tproj[j]]) : uint32_t(M);  // M: past every real index
        });
        RadixPayload pl;
        pl.n = 1;
        pl.in[0] = tv;
        pl.size[0] = 8;
        uint32_t *no_vals = nullptr;
        radix_sort_pairs_payload32(c, key, no_vals, NC, ibits, pl);
        const double *stv = static_cast<const double *>(pl.out[0]);
        uint32_t *sid = c->arena.get<uint32_t>(NC);
        map_n(c, NC, nullptr, [=] __device__(int64_t k) {
            const int64_t live = *d_nt;
            sid[k] = uint32_t(key[k]);
            if (k < live) sv[k] = stv[k];
        });
        segment_offsets_dn(c, sid, d_nt, NC, M, o->session_offsets);
    }
    if (flags & FZ_RQ2C_SKIP_SESSION_STATS) return;

    // per-session statistics (sessions are non-increasing in size: >= 100 is a prefix)
    Segs ses{M, o->session_offsets, NC, P};  // a session holds at most one value per project
    session_stats(c, sv, ses, o->average_trend, o->median_trend, o->dist_percentiles, counts + FZ_RQ2C_GE100,
                  o->dist_mean);

    // tests on the median trend (one segment of K values)
    double *sc = o->scalars;
    {
        double *t4 = c->arena.get<double>(4);
        if (series_small_ok(M)) {  // (straight into the scalars)
            series_small(c, o->median_trend, counts + FZ_RQ2C_GE100, sc + FZ_RQ2C_SP_RHO, sc + FZ_RQ2C_SP_P, t4 + 2,
                         sc + FZ_RQ2C_SW_MEDIAN_P);
        } else {
            series_tests(c, o->median_trend, M, counts + FZ_RQ2C_GE100, t4);
            map_n(c, 1, nullptr, [=] __device__(int64_t) {
                sc[FZ_RQ2C_SP_RHO] = t4[0];
                sc[FZ_RQ2C_SP_P] = t4[1];
                sc[FZ_RQ2C_SW_MEDIAN_P] = t4[3];
            });
        }
    }
    // mean / median of the valid (non-NaN) per-project correlations
    {
        int64_t *d_nv = c->arena.get<int64_t>(1);
        const double *corr = o->corr;
        double *vals = c->arena.get<double>(P > 0 ? P : 1);
        compact_emit(c, P, nullptr, [=] __device__(int64_t p) { return raw_n[p] > 0 && !isnan(corr[p]); },
                     [=] __device__(int64_t p, int64_t q) { vals[q] = corr[p]; }, d_nv);
        fz_describe *d = c->arena.get<fz_describe>(1);
        describe_f64_dn(c, vals, P, d_nv, d);
        map_n(c, 1, nullptr, [=] __device__(int64_t) {
            sc[FZ_RQ2C_CORR_MEAN] = d->mean;
            sc[FZ_RQ2C_CORR_MEDIAN] = d->median;
        });
    }
}

// The sharded step's RQ2-count tail, after the session exchange and the gather of the per-session
// rows (rq2_coverage_count.py:335-372): the tests on the first k entries of the median trend and
// the mean / median of the valid per-project correlations (eligible, raw_n > 0, not NaN) -
// out[0..3] as fz_series_tests, out[4..5] mean and median; one library call instead of the
// driver's slicing, host-side mask and upload.
void rq2_count_tail(fz_ctx *c, const double *median_trend, int64_t k, const double *corr, const int64_t *raw_n,
                    const int64_t *eligible, int64_t P, double *out) {
    int64_t *d_k = c->arena.get<int64_t>(1);
    set_i64(c, d_k, &k, 1);
    if (series_small_ok(k > 0 ? k : 1))
        series_small(c, median_trend, d_k, out, out + 1, out + 2, out + 3);
    else
        series_tests(c, median_trend, k > 0 ? k : 1, d_k, out);
    int64_t *d_nv = c->arena.get<int64_t>(1);
    double *vals = c->arena.get<double>(P > 0 ? P : 1);
    compact_emit(c, P, nullptr,
                 [=] __device__(int64_t p) { return eligible[p] != 0 && raw_n[p] > 0 && !isnan(corr[p]); },
                 [=] __device__(int64_t p, int64_t q) { vals[q] = corr[p]; }, d_nv);
    fz_describe *d = c->arena.get<fz_describe>(1);
    describe_f64_dn(c, vals, P, d_nv, d);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        out[4] = d->mean;
        out[5] = d->median;
    });
}

// ------------------------------------------------------------------------------ RQ2 (add)
// rq2_coverage_and_added.py:73-238: change points of (modules, revisions) over Coverage builds.
constexpr int64_t kDayUs = 86400000000LL;

struct CovBuildRows {  // result IN ('HalfWay', 'Finish') AND timecreated < LIMIT (:50-69), eligible
    static constexpr int kBytes = 13;  // column bytes read per row (filter_compact probe)
    const uint32_t *proj;
    const uint8_t *result;
    const int64_t *time;
    const uint8_t *elig;
    __device__ bool operator()(int32_t r) const {
        const uint8_t x = result[r];
        return ((x == 2) | (x == 0)) & (time[r] < kLimitUs2) & bool(elig[proj[r]]);
    }
};
struct CovRowsBeforeLimit {  // GET_COVERAGE_DATA: date < LIMIT, no NULL filter (:30-47), eligible
    static constexpr int kBytes = 12;  // column bytes read per row (filter_compact probe)
    const uint32_t *proj;
    const int64_t *date;
    const uint8_t *elig;  // (RQ2 add: the projects with a selected Coverage build - the only ones read)
    __device__ bool operator()(int32_t r) const { return (date[r] < kLimitUs2) & bool(elig[proj[r]]); }
};

__device__ inline int64_t floor_div(int64_t a, int64_t b) {
    const int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

// first coverage row of [lo, hi) whose calendar day equals `day` (the reference's first match), or -1
__device__ inline int64_t first_row_on_day(const int64_t *ctime, const int32_t *crow, int64_t lo, int64_t hi,
                                           int64_t day) {
    const int64_t k = lower_bound_i64(ctime, lo, hi, day * kDayUs);
    if (k < hi && floor_div(ctime[k], kDayUs) == day) return crow[k];
    return -1;
}

void rq2_add(fz_ctx *c, const fz_rq2_add_out *o) {
    Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_rq2_add: call fz_store_build first");
    FZ_CHECK(o && o->counts && o->eligible && o->row_project && o->row_first_build && o->row_end_build &&
                 o->row_start_build && o->row_cov_i && o->row_cov_i1 && o->diff_total && o->diff_coverage &&
                 o->covered_is_float && o->total_is_float,
             "fz_rq2_add: null output buffer");
    const fz_tables &t = s.t;
    const int64_t P = s.P;
    uint8_t *anyc = c->arena.get<uint8_t>(P), *anyt = c->arena.get<uint8_t>(P);
    eligible_projects(c, o->eligible, o->counts + FZ_RQ2A_ELIGIBLE,
                      {{o->counts, FZ_RQ2A_NCOUNTS * 8, 0},
                       {o->covered_is_float, P > 0 ? P : 1, 0},
                       {o->total_is_float, P > 0 ? P : 1, 0},
                       {anyc, P > 0 ? P : 1, 0},
                       {anyt, P > 0 ? P : 1, 0}});

    TmpView B, CV;
    filter_view(c, s.covb, s.covb.n, P,
                CovBuildRows{t.b_project, t.b_result, t.b_time, o->eligible}, B);
    // the coverage rows are read for projects with a selected Coverage build only (their change
    // points' date joins and pandas upcast flags): the view's other tiles are skipped, all of them
    // on a table without builds (configs 3 / 5)
    uint8_t *withb = c->arena.get<uint8_t>(P);
    {
        const uint8_t *el = o->eligible;
        const int64_t *bo = B.offs;
        map_n(c, P, nullptr, [=] __device__(int64_t p) { withb[p] = el[p] && bo[p + 1] > bo[p] ? 1 : 0; });
    }
    filter_view(c, s.cov, s.cov.n, P, CovRowsBeforeLimit{t.c_project, t.c_date, withb},
                CV, nullptr, Selection::segments(withb, 1, B.d_n, s.cov.offs, kLimitUs2));
    const int64_t NB = s.covb.n;
    const int64_t *boffs = B.offs, *coffs = CV.offs;
    // pandas upcast flags: a NULL covered/total among the project's fetched coverage rows
    {
        const int32_t *crow = CV.row;
        const uint32_t *cproj = CV.proj;
        const uint8_t *valid = t.c_valid;
        map_n(c, s.cov.n, CV.d_n, [=] __device__(int64_t j) {
            const uint8_t v = valid[crow[j]];
            if (!(v & FZ_VALID_COVERED)) anyc[cproj[j]] = 1;
            if (!(v & FZ_VALID_TOTAL)) anyt[cproj[j]] = 1;
        });
        uint8_t *cf = o->covered_is_float, *tf = o->total_is_float;
        per_seg(c, P, [=] __device__(int64_t p) {
            const bool used = boffs[p + 1] > boffs[p] && coffs[p + 1] > coffs[p];
            cf[p] = used && anyc[p];
            tf[p] = used && anyt[p];
        });
    }
    // run starts: group = cumsum(key != key.shift()) within the project (:129-131) - the start
    // positions compacted in one pass
    int64_t *runpos = c->arena.get<int64_t>(NB + 1);
    int64_t *d_runs = o->counts + FZ_RQ2A_RUNS;
    const int32_t *brow = B.row;
    const uint32_t *bproj = B.proj;
    const int32_t *grp = t.b_group;
    const int64_t *d_nb = B.d_n;
    compact_emit<4>(c, NB, d_nb,
                 [=] __device__(int64_t j) {
                     const uint32_t p = bproj[j];
                     return (coffs[p + 1] > coffs[p]) && (j == boffs[p] || grp[brow[j]] != grp[brow[j - 1]]);
                 },
                 [=] __device__(int64_t j, int64_t q) { runpos[q] = j; }, d_runs);
    const int64_t *btime = t.b_time;
    const int64_t *ctime = CV.time;
    const int32_t *crow = CV.row;
    const int64_t *cov_c = t.c_covered, *cov_t = t.c_total;
    const uint8_t *valid = t.c_valid;
    const fz_rq2_add_out out = *o;
    const int32_t *bperm = s.bperm, *cperm = s.cperm;  // sorted positions -> the caller's row ids
    // a row for run r when run r + 1 belongs to the same project, rows compacted in the same pass
    compact_emit<1>(c, NB, d_runs,
                 [=] __device__(int64_t r) {
                     return r + 1 < *d_runs && bproj[runpos[r]] == bproj[runpos[r + 1]];
                 },
                 [=] __device__(int64_t r, int64_t q) {
        const int64_t j0 = runpos[r], j1 = runpos[r + 1];
        const uint32_t p = bproj[j0];
        const int32_t f = brow[j0], e = brow[j1 - 1], sb = brow[j1];
        const int64_t c0 = first_row_on_day(ctime, crow, coffs[p], coffs[p + 1], floor_div(btime[e], kDayUs));
        const int64_t c1 = first_row_on_day(ctime, crow, coffs[p], coffs[p + 1], floor_div(btime[sb], kDayUs));
        auto cell = [&](int64_t cr, double &cv, double &tv) {
            cv = tv = NAN;
            if (cr < 0) return;
            const uint8_t v = valid[cr];
            if (v & FZ_VALID_COVERED) cv = double(cov_c[cr]);
            if (v & FZ_VALID_TOTAL) tv = double(cov_t[cr]);
        };
        double cv0, tv0, cv1, tv1;
        cell(c0, cv0, tv0);
        cell(c1, cv1, tv1);
        double dt = NAN, dc = NAN;
        if (!isnan(tv0) && tv0 != 0.0 && !isnan(tv1) && tv1 != 0.0) {
            dt = tv1 - tv0;
            dc = (cv1 / tv1) * 100.0 - (cv0 / tv0) * 100.0;
        }
        out.row_project[q] = p;
        out.row_first_build[q] = bperm[f];
        out.row_end_build[q] = bperm[e];
        out.row_start_build[q] = bperm[sb];
        out.row_cov_i[q] = c0 >= 0 ? cperm[c0] : -1;
        out.row_cov_i1[q] = c1 >= 0 ? cperm[c1] : -1;
        out.diff_total[q] = dt;
        out.diff_coverage[q] = dc;
    }, o->counts + FZ_RQ2A_ROWS);
}

}  // namespace fz
