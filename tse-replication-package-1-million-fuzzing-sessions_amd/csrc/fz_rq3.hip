// RQ3 - coverage change on the day after a bug is fixed vs ordinary day-to-day changes
// (rq3_diff_coverage_at_detection.py:202-360).
//
//   per-issue loop with 3 queries per project (:241-302)  -> one thread per issue over three
//        filtered views: last Fuzzing build before rts (lower_bound), first Coverage build after
//        rts (upper_bound), coverage pair on day rts+1 (lower_bound on the day)
//   non-detected flush on project change (:245-257)      -> one thread per coverage row of the
//        flushed projects, excluded days found by binary search in that project's detections
//   summary / anderson / levene / brunnermunzel (:25-66, :321-352) -> sorted keys + chunked
//        double-double reductions + the segmented rank tests (fz_series.hip)
#include "fz_seg.h"
#include "fz_stats.h"

namespace fz {

constexpr int64_t kLim3 = 1736294400000000LL;    // '2025-01-08'
constexpr int64_t kLim3b = 1736380800000000LL;   // '2025-01-09' (rq3:262-263)
constexpr int64_t kDay3 = 86400000000LL;
constexpr int64_t kGapUs = 24LL * 3600LL * 1000000LL;
#ifndef FZ_RQ3_A2_MAP
#define FZ_RQ3_A2_MAP 1  // the Anderson-Darling terms by a full-width map (0: inside the reduction)
#endif
#ifndef FZ_RQ3_NON_ITEMS
#define FZ_RQ3_NON_ITEMS 4  // coverage rows per thread of the non-detected pass
#endif

void eligible_projects(fz_ctx *c, uint8_t *elig, int64_t *d_count, std::initializer_list<Fill> fills = {});

__device__ inline int64_t fdiv_day(int64_t a) {
    const int64_t q = a / kDay3;
    return (a % kDay3 != 0 && a < 0) ? q - 1 : q;
}

// Three independent binary searches over non-empty ranges [lo, hi) in lock step: each round issues
// the three probes' loads together, so one issue's searches cost one chain of ~log2(range) dependent
// loads instead of three (the detected pass runs one thread per issue - about one wave per SIMD -
// and is bound by that load latency).  upper: first index with a[i] > v, else first with a[i] >= v.
struct Probe3 {
    const int64_t *a;
    int64_t lo, hi, v;
    bool upper;
};
__device__ inline void search3(Probe3 &x, Probe3 &y, Probe3 &z) {
    const int64_t xl = x.hi - 1, yl = y.hi - 1, zl = z.hi - 1;  // clamps for a finished search's probe
    while (x.lo < x.hi || y.lo < y.hi || z.lo < z.hi) {
        const int64_t mx = x.lo < x.hi ? (x.lo + x.hi) >> 1 : (x.lo < xl ? x.lo : xl);
        const int64_t my = y.lo < y.hi ? (y.lo + y.hi) >> 1 : (y.lo < yl ? y.lo : yl);
        const int64_t mz = z.lo < z.hi ? (z.lo + z.hi) >> 1 : (z.lo < zl ? z.lo : zl);
        const int64_t ax = x.a[mx], ay = y.a[my], az = z.a[mz];
        if (x.lo < x.hi) {
            if (x.upper ? ax <= x.v : ax < x.v) x.lo = mx + 1;
            else x.hi = mx;
        }
        if (y.lo < y.hi) {
            if (y.upper ? ay <= y.v : ay < y.v) y.lo = my + 1;
            else y.hi = my;
        }
        if (z.lo < z.hi) {
            if (z.upper ? az <= z.v : az < z.v) z.lo = mz + 1;
            else z.hi = mz;
        }
    }
}

struct FixedIssuesRq3 {  // status fixed, eligible project, rts < LIMIT (:219-232)
    static constexpr int kBytes = 13;  // column bytes read per row (filter_compact probe)
    const uint32_t *proj;
    const uint8_t *status;
    const int64_t *rts;
    const uint8_t *elig;
    __device__ bool operator()(int32_t r) const { return (status[r] <= 1) & (rts[r] < kLim3) & bool(elig[proj[r]]); }
};
struct FuzzRq3 {  // Fuzzing, result IN ('HalfWay', 'Finish'), DATE(timecreated) < '2025-01-08' (:260-261)
    static constexpr int kBytes = 9;  // column bytes read per row (filter_compact probe)
    const uint8_t *result;
    const int64_t *time;
    __device__ bool operator()(int32_t r) const { return ((result[r] == 2) | (result[r] == 0)) & (time[r] < kLim3); }
};
struct CovBuildRq3 {  // Coverage, any result, DATE(timecreated) < '2025-01-09' (:262)
    static constexpr int kBytes = 8;  // column bytes read per row (filter_compact probe)
    const int64_t *time;
    __device__ bool operator()(int32_t r) const { return time[r] < kLim3b; }
};
struct CovRowsRq3 {  // covered_line IS NOT NULL AND DATE(date) < '2025-01-09' (:263), projects with
                     // a fixed issue only (the only ones whose rows the per-issue loop reads, :241)
    static constexpr int kBytes = 13;  // column bytes read per row (filter_compact probe)
    const uint8_t *valid;
    const int64_t *date;
    const uint32_t *proj;
    const uint8_t *sel;  // [P] 1: the project has a fixed issue
    __device__ bool operator()(int32_t r) const {
        return bool(sel[proj[r]]) & bool(valid[r] & FZ_VALID_COVERED) & (date[r] < kLim3b);
    }
};

void rq3_stats(fz_ctx *c, const double *det_pct, const int64_t *det_tot, int64_t NI, const int64_t *d_nd,
               const double *non_pct, int64_t NC, const int64_t *d_nn, fz_describe *describe, double *tests);

void rq3(fz_ctx *c, uint32_t flags, const fz_rq3_out *o) {
    Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_rq3: call fz_store_build first");
    FZ_CHECK(o && o->counts && o->eligible && o->det_pct && o->det_cov && o->det_tot && o->det_project &&
                 o->det_issue && o->non_pct && o->non_cov && o->non_tot && o->describe && o->tests,
             "fz_rq3: null output buffer");
    const fz_tables &t = s.t;
    const int64_t P = s.P, NI = s.issues.n, NC = s.cov.n;
    int64_t *counts = o->counts;
    eligible_projects(c, o->eligible, counts + FZ_RQ3_ELIGIBLE, {{counts, FZ_RQ3_NCOUNTS * 8, 0}});

    TmpView I, F, CB, TC;
    filter_views3(c, P, s.issues, NI, FixedIssuesRq3{t.i_project, t.i_status, t.i_rts, o->eligible}, I, s.fuzz,
                  s.fuzz.n, FuzzRq3{t.b_result, t.b_time}, F, s.covb, s.covb.n, CovBuildRq3{t.b_time}, CB);
    // the coverage rows of the projects with a fixed issue only: the view's tiles of other projects
    // are skipped unread (config 3 / 5, coverage-only tables: all of them)
    uint8_t *self = c->arena.get<uint8_t>(P);
    {
        const int64_t *ioff = I.offs;
        map_n(c, P, nullptr, [=] __device__(int64_t p) { self[p] = ioff[p + 1] > ioff[p] ? 1 : 0; });
    }
    filter_view(c, s.cov, NC, P, CovRowsRq3{t.c_valid, t.c_date, t.c_project, self}, TC,
                nullptr, Selection::segments(self, 1, I.d_n, s.cov.offs, kLim3b));

    // ---- detected: one thread per issue (:241-302), the detected ones compacted in the same pass
    int64_t *pa = c->arena.get<int64_t>(NI);  // coverage pair (row a, row b)
    int64_t *pb = c->arena.get<int64_t>(NI);
    const int32_t *irow = I.row;
    const uint32_t *iproj = I.proj;
    const int64_t *irts = I.time;
    const int64_t *d_ni = I.d_n;
    const TmpView Fv = F, CBv = CB, TCv = TC;
    const uint8_t *result = t.b_result;
    const int64_t *btime = t.b_time;
    const int32_t *canon = t.b_rev_canon;
    const int64_t *cvd = t.c_covered, *ctot = t.c_total;
    const uint8_t *cval = t.c_valid;
    // `prev_cov[2] > 0 and curr_cov[2] > 0` (rq3:253,297) in Python: a NULL total_line (None) on
    // the left, or on the right after a positive left, raises TypeError (the query filters only
    // covered_line IS NOT NULL, :263); NULL totals are stored as 0 with the valid bit clear
    auto null_cmp = [=] __device__(int32_t ra, int32_t rb) {
        return !(cval[ra] & FZ_VALID_TOTAL) || (ctot[ra] > 0 && !(cval[rb] & FZ_VALID_TOTAL));
    };
    uint32_t *dproj = c->arena.get<uint32_t>(NI);
    int64_t *dday = c->arena.get<int64_t>(NI);
    const fz_rq3_out out = *o;
    const int32_t *iperm = s.iperm;  // sorted positions -> the caller's issue row ids
    auto detected = [=] __device__(int64_t j) -> bool {
        if (j == 0) counts[FZ_RQ3_ISSUES] = *d_ni;  // (no issues: the zero fill stands)
        const uint32_t p = iproj[j];
        const int64_t rts = irts[j];
        const int64_t f0 = Fv.offs[p], f1 = Fv.offs[p + 1];
        const int64_t b0 = CBv.offs[p], b1 = CBv.offs[p + 1];
        const int64_t c0 = TCv.offs[p], c1 = TCv.offs[p + 1];
        if (f0 == f1 || b0 == b1 || c0 == c1) return false;
        // the last fuzz build before rts, the first coverage build after rts, the first coverage
        // row on day rts + 1: three searches at once (the conditions below are side-effect free,
        // so testing them after all three lookups keeps the reference's outcome)
        const int64_t target = fdiv_day(rts) + 1;
        Probe3 sf{Fv.time, f0, f1, rts, false}, sb{CBv.time, b0, b1, rts, true}, sc{TCv.time, c0, c1, target * kDay3, false};
        search3(sf, sb, sc);
        const int64_t k = sf.lo - 1, k2 = sb.lo;
        int64_t kk = sc.lo;
        if (k < f0 || k2 >= b1) return false;
        if (kk < c0 + 1) kk = c0 + 1;  // the reference scans rows i >= 1
        if (kk >= c1) return false;
        const int32_t lf = Fv.row[k], fc = CBv.row[k2];
        const int64_t tkk = TCv.time[kk];
        const int32_t ra = TCv.row[kk - 1], rb = TCv.row[kk];
        if (!(result[fc] == 2 || result[fc] == 0)) return false;
        if (btime[fc] - btime[lf] > kGapUs) return false;  // total_seconds()/3600 > 24 (:277)
        if (canon[lf] < 0 || canon[lf] != canon[fc]) return false;
        if (fdiv_day(tkk) != target) return false;
        if (cvd[rb] == 0) return false;      // break without a pair (:291)
        if (null_cmp(ra, rb)) {
            atomic_add_i64(&counts[FZ_RQ3_NULL_TOTAL], 1);
            return false;
        }
        if (!(ctot[ra] > 0 && ctot[rb] > 0)) return false;
        pa[j] = ra;
        pb[j] = rb;
        return true;
    };
    compact_emit<1>(c, NI, d_ni, detected, [=] __device__(int64_t j, int64_t q) {
        const int64_t ra = pa[j], rb = pb[j];
        out.det_pct[q] = (double(cvd[rb]) / double(ctot[rb]) - double(cvd[ra]) / double(ctot[ra])) * 100.0;
        out.det_cov[q] = cvd[rb] - cvd[ra];
        out.det_tot[q] = ctot[rb] - ctot[ra];
        out.det_project[q] = iproj[j];
        out.det_issue[q] = iperm[irow[j]];
        dproj[q] = iproj[j];
        dday[q] = fdiv_day(irts[j]);
    }, counts + FZ_RQ3_DETECTED);
    int64_t *doffs = c->arena.get<int64_t>(P + 1);
    segment_offsets_dn(c, dproj, counts + FZ_RQ3_DETECTED, NI, P, doffs);

    // ---- non-detected: projects with issues, except the last one (never flushed, :245-257) -
    // unless this is a shard that is not the last one (FZ_RQ3_FLUSH_LAST; the caller decides)
    const int64_t *ioffs = I.offs;
    const bool flush_last = flags & FZ_RQ3_FLUSH_LAST;
    // (over the live rows of TC only: *TCv.d_n of capacity NC; the kept pairs compacted in the pass)
    // (several rows per thread: their loads overlap, and fewer tiles to look back over)
    compact_emit<FZ_RQ3_NON_ITEMS>(c, NC, TCv.d_n, [=] __device__(int64_t k) -> bool {
        // every load that depends on the row alone first - the project's bounds, the row pair's
        // validity and totals (in range for any k < n) - so the loads of a thread's items overlap
        // instead of one dependent round trip after each test; then the tests in the reference's
        // order, the NULL counts (side effects) only where the reference reaches them
        const uint32_t p = TCv.proj[k];
        const int32_t rb = TCv.row[k], ra = TCv.row[k > 0 ? k - 1 : k];
        const int64_t tk = TCv.time[k];
        const int64_t ni = *d_ni;
        const int64_t i0 = ioffs[p], i1 = ioffs[p + 1], o0 = TCv.offs[p], lo = doffs[p], hi = doffs[p + 1];
        const uint32_t plast = ni > 0 ? iproj[ni - 1] : 0xffffffffu;
        const uint8_t va = cval[ra], vb = cval[rb];
        const int64_t ta = ctot[ra], tb = ctot[rb];
        const bool hasiss = (i1 > i0) & (flush_last | (ni <= 0) | (p != plast));
        if (!hasiss | (k == o0)) return false;
        const int64_t day = fdiv_day(tk);
        const int64_t q = lower_bound_i64(dday, lo, hi, day);
        if (q < hi && dday[q] == day) return false;  // a detection day of this project
        const bool last = p == plast;  // (ni > 0 here: a project with issues)
        if (!(va & FZ_VALID_TOTAL) | ((ta > 0) & !(vb & FZ_VALID_TOTAL))) {  // null_cmp(ra, rb)
            atomic_add_i64(&counts[FZ_RQ3_NULL_TOTAL], 1);
            if (last) atomic_add_i64(&counts[FZ_RQ3_NULL_LAST], 1);
            return false;
        }
        if (!((ta > 0) & (tb > 0))) return false;
        if (last) atomic_add_i64(&counts[FZ_RQ3_NON_LAST], 1);
        return true;
    }, [=] __device__(int64_t k, int64_t q) {
        const int32_t ra = TCv.row[k - 1], rb = TCv.row[k];
        out.non_pct[q] = (double(cvd[rb]) / double(ctot[rb]) - double(cvd[ra]) / double(ctot[ra])) * 100.0;
        out.non_cov[q] = cvd[rb] - cvd[ra];
        out.non_tot[q] = ctot[rb] - ctot[ra];
    }, counts + FZ_RQ3_NON_DETECTED);

    // (no issue at all - configs 3 / 5, coverage-only: both samples are empty whatever the coverage
    // table holds, so the statistics run over a zero capacity instead of the 1e8-row one - the
    // capacity-sized reduction maps walked ~1e5 empty chunks per launch)
    if (!(flags & FZ_RQ3_SKIP_STATS))
        rq3_stats(c, o->det_pct, o->det_tot, NI, counts + FZ_RQ3_DETECTED, o->non_pct, NI > 0 ? NC : 0,
                  counts + FZ_RQ3_NON_DETECTED, o->describe, o->tests);
}

// anderson(det), anderson(non) (:329, :335) and levene(det, non) (:344) in one set of reductions:
// the two samples are segments {0, nd, nd + nn} (oseg) of the union v (their sums do not depend on
// order) and of cat (the union partitioned by sample, each part ascending: medians, A2 terms).
// Written only when both samples are non-empty.
// (ms: the two samples' describe moments from the same sums - mean = sum x / n, sqrt(sum of squared
// deviations / n) - so the describes need no double-double passes of their own)
static void sample_tests(fz_ctx *c, const double *v, const double *cat, int64_t cap, const int64_t *oseg,
                         double *tests, double *ms) {
    const Segs two{2, oseg, cap};
    const ChunkedSegs cs = chunked(c, two);
    // sample s's median from its sorted part of cat (computed where it is used: no launch of its own)
    auto med = [=] __device__(int32_t s) {
        const int64_t b = oseg[s], n = oseg[s + 1] - b;
        return n <= 0 ? NAN : ((n & 1) ? cat[b + n / 2] : (cat[b + n / 2 - 1] + cat[b + n / 2]) / 2.0);
    };
    double *r1 = c->arena.get<double>(4);  // [s]: sum x, sum |x - median|
    seg_reduce<2>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        x[0] = v[i];
        x[1] = fabs(v[i] - med(s));
    }, r1, 8.0);
    double *r2 = c->arena.get<double>(4);  // [s]: sum (x - mean)^2, sum (|x - median| - its mean)^2
    seg_reduce<2>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const double n = double(oseg[s + 1] - oseg[s]);
        const double d = v[i] - r1[2 * s] / n;
        const double e = fabs(v[i] - med(s)) - r1[2 * s + 1] / n;
        x[0] = d * d;
        x[1] = e * e;
    }, r2, 8.0);
    double *r3 = c->arena.get<double>(2);  // [s]: sum of the A2 terms (ascending order)
    // the terms (two log_ndtr each) by a map over every element - a thread each, the whole chip -
    // then summed in the reduction's usual order; inside the chunked reduction's 8-per-thread loop
    // the dependent fp64 chains of one wave per SIMD were latency-bound (config 2: 37 us -> ~10)
#if FZ_RQ3_A2_MAP
    double *a2 = c->arena.get<double>(cap > 0 ? cap : 1);
    map_n(c, cap > 0 ? cap : 1, oseg + 2, [=] __device__(int64_t i) {
        const int s = i < oseg[1] ? 0 : 1;
        const int64_t b = oseg[s], n = oseg[s + 1] - b, k = i - b;
        const double N = double(n), xbar = r1[2 * s] / N;
        const double sd = sqrt(r2[2 * s] / (N - 1.0));  // np.std(ddof=1)
        const double wi = (cat[i] - xbar) / sd, wj = (cat[b + n - 1 - k] - xbar) / sd;
        a2[i] = (2.0 * double(k + 1) - 1.0) / N * (stats::log_ndtr(wi) + stats::log_ndtr(-wj));
    });
    seg_reduce<1>(c, cs, [=] __device__(int64_t i, int32_t, double *x) { x[0] = a2[i]; }, r3, 24.0);
    // (algorithmic bytes: the value and its mirror read, the term written and read back)
#else  // (A/B build: the terms inside the chunked reduction)
    seg_reduce<1>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const int64_t b = oseg[s], n = oseg[s + 1] - b, k = i - b;
        const double N = double(n), xbar = r1[2 * s] / N;
        const double sd = sqrt(r2[2 * s] / (N - 1.0));
        const double wi = (cat[i] - xbar) / sd, wj = (cat[b + n - 1 - k] - xbar) / sd;
        x[0] = (2.0 * double(k + 1) - 1.0) / N * (stats::log_ndtr(wi) + stats::log_ndtr(-wj));
    }, r3, 16.0);
#endif
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        const double nx = double(oseg[1] - oseg[0]), ny = double(oseg[2] - oseg[1]);
        for (int s = 0; s < 2; ++s) {
            const double ns = s ? ny : nx;
            ms[2 * s] = ns > 0.0 ? r1[2 * s] / ns : NAN;
            ms[2 * s + 1] = ns > 0.0 ? sqrt(r2[2 * s] / ns) : NAN;
        }
        if (!(nx > 0.0 && ny > 0.0)) return;
        const double av[5] = {0.576, 0.656, 0.787, 0.918, 1.092};
        for (int s = 0; s < 2; ++s) {
            const double N = s ? ny : nx;
            double *out = tests + (s ? FZ_RQ3_AD_NON : FZ_RQ3_AD_DET);
            out[0] = -N - r3[s];
            for (int k = 0; k < 5; ++k) out[1 + k] = rint(av[k] / (1.0 + 4.0 / N - 25.0 / N / N) * 1000.0) / 1000.0;
        }
        // levene([x, y], center='median') (scipy _morestats.py levene)
        const double zb0 = r1[1] / nx, zb1 = r1[3] / ny, N = nx + ny;
        double zbar = 0.0;
        zbar += zb0 * nx;
        zbar += zb1 * ny;
        zbar /= N;
        const double numer = (N - 2.0) * (nx * (zb0 - zbar) * (zb0 - zbar) + ny * (zb1 - zbar) * (zb1 - zbar));
        double dvar = 0.0;
        dvar += r2[1];
        dvar += r2[3];
        const double W = numer / (1.0 * dvar);
        tests[FZ_RQ3_LEVENE_W] = W;
        tests[FZ_RQ3_LEVENE_P] = stats::f1_sf(W, N - 2.0);
    });
}

// ---- statistics (:321-352) over samples of device lengths *d_nd <= NI and *d_nn <= NC
void rq3_stats(fz_ctx *c, const double *det_pct, const int64_t *det_tot, int64_t NI, const int64_t *d_nd,
               const double *non_pct, int64_t NC, const int64_t *d_nn, fz_describe *describe, double *tests) {
    double *dtot_f = c->arena.get<double>(NI);
    const int64_t *dt = det_tot;
    // One sort of det u non serves everything: Brunner-Munzel ranks the union, and a stable
    // partition of the sorted union by sample gives each sample's sorted values (describe,
    // anderson, levene) - instead of three separate device-wide sorts.
    const int64_t cap = NI + NC;
    int64_t *oseg = c->arena.get<int64_t>(3);  // {0, nd, nd + nn}: the samples in the union
    uint64_t *skd = c->arena.get<uint64_t>(cap);
    uint64_t *skn = c->arena.get<uint64_t>(cap);
    double *v = c->arena.get<double>(cap);
    double *cat = c->arena.get<double>(cap);
    {
        const double *dp = det_pct, *np_ = non_pct;
        int64_t *oall = c->arena.get<int64_t>(2);  // {0, *d_nd + *d_nn}: the union's one segment
        const int64_t *d_all = oall + 1;
        // the union's values and segment bounds and det_tot as doubles in one pass, over the live
        // elements only (config 3's union is empty, config 2's ~80 % of the capacity NI + NC)
        int32_t *sid = c->arena.get<int32_t>(cap);
        const int64_t *d_det0 = d_nd;
        map_n(c, cap > 0 ? cap : 1, nullptr, [=] __device__(int64_t i) {
            const int64_t nd = *d_det0, nn = *d_nn;
            if (i == 0) {
                oall[0] = 0;
                oall[1] = nd + nn;
                oseg[0] = 0;
                oseg[1] = nd;
                oseg[2] = nd + nn;
            }
            if (i < nd) dtot_f[i] = double(dt[i]);
            if (i >= nd + nn) return;
            v[i] = i < nd ? dp[i] : np_[i - nd];
            sid[i] = 0;
        });
        Segs one{1, oall, cap};
        SortedSegs ss = seg_sort_f64(c, v, one, sid);
        // stable partition of the sorted union into the two samples: before[i] = det values before
        // union position i (det: source position < nd), before[live] = their total
        int64_t *isdet = c->arena.get<int64_t>(cap), *before = c->arena.get<int64_t>(cap + 1);
        const int32_t *pos = ss.pos;
        const double *sv = ss.val;
        map_n(c, cap, d_all, [=] __device__(int64_t i) { isdet[i] = pos[i] < *d_nd ? 1 : 0; });
        scan_exclusive_i64_dn(c, isdet, before, cap, d_all, before + cap);
        // brunnermunzel(det, non) (:349): union and within-sample ranks off the sorted union and the
        // det counts, chunk by chunk
        bm_union_sorted(c, one, sv, pos, before, d_nd, tests + FZ_RQ3_BM_STAT, tests + FZ_RQ3_BM_P);
        const int64_t *d_det = d_nd;
        map_n(c, cap, d_all, [=] __device__(int64_t i) {
            const uint64_t k = f64_key(sv[i]);
            if (isdet[i]) {
                skd[before[i]] = k;
                cat[before[i]] = sv[i];
            } else {
                skn[i - before[i]] = k;
                cat[*d_det + i - before[i]] = sv[i];
            }
        });
    }
    const DescJob tot{dtot_f, NI, d_nd, describe + 2};  // (by selection: no sort of its own)
    describe_f64_dn_batch(c, &tot, 1);
    // the samples' describes: their order statistics off the sorted keys, mean / std from the
    // Levene / Anderson-Darling sums (sample_tests) - one finishing launch
    double *ms = c->arena.get<double>(4);
    sample_tests(c, v, cat, cap, oseg, tests, ms);
    const SortedDescJob jobs[2] = {{skd, det_pct, NI, d_nd, describe}, {skn, non_pct, NC, d_nn, describe + 1}};
    describe_sorted_dn_finish(c, jobs, 2, ms);
}

}  // namespace fz
