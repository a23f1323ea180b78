// RQ4 - seed-corpus groups (rq4a_bug.py: bug detection; rq4b_coverage.py: coverage).
//
// Groups come from project_corpus_analysis.csv, parsed on the host into per-project columns
// (fz_rq4_groups, see fz.h); everything per build / issue / coverage row runs here:
//   rq4a  G1/G2 per-iteration tables (:302-346)        -> histogram + reverse scan; distinct
//         (iteration, project) by adjacency in (project, rts) order
//         G4 pre/post windows + introduction (:246-412) -> one thread per G4 project, issue counts
//         in [t_k, t_k+1) by two lower_bounds
//   rq4b  per-session quartiles + Brunner-Munzel (:910-1015) -> radix transpose to
//         (session, group, project) order, segmented sorts, segmented rank tests
//         coverage deltas around the corpus date (:725-797), initial-coverage MWU / Cliff /
//         BM / Levene (:221-313)                        -> per-project binary searches + rank tests
#include "fz_seg.h"
#include "fz_stats.h"
#include "fz_transpose.h"

namespace fz {

constexpr int64_t kLim4 = 1736294400000000LL;  // '2025-01-08'
constexpr int64_t kDay4 = 86400000000LL;
void rq2_session_stats_grouped(fz_ctx *c, const double *values, const int64_t *offs, int64_t n, int64_t S,
                               int64_t max_len, double *average, double *median, double *pcts, int64_t *n_ge100);
constexpr int kWin = 7;                         // ANALYSIS_ITERATIONS / DAYS_THRESHOLD (rq4a:43-46)

void eligible_projects(fz_ctx *c, uint8_t *elig, int64_t *d_count, std::initializer_list<Fill> fills = {});

__device__ inline int64_t fdiv4(int64_t a, int64_t b) {
    const int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

struct BuildsBeforeLimit {  // get_project_fuzzing_builds: Fuzzing, any result, timecreated < LIMIT (rq4a:124-137)
    const int64_t *time;
    __device__ bool operator()(int32_t r) const { return time[r] < kLim4; }
};
struct FixedBeforeLimit {  // get_project_fixed_issues: Fixed*, rts < LIMIT (rq4a:140-153)
    const uint8_t *status;
    const int64_t *rts;
    __device__ bool operator()(int32_t r) const { return (status[r] <= 1) & (rts[r] < kLim4); }
};

// eligible group membership; rq4a (missing_to_g1) also puts CSV-missing eligible projects in G1
static void group_members(fz_ctx *c, const fz_rq4_groups *g, const uint8_t *elig, uint8_t *member,
                          int64_t *counts4, bool missing_to_g1) {
    const uint8_t *m = g->member;
    const int64_t P = store_of(c).P;
    per_seg(c, P, [=] __device__(int64_t p) {
        uint8_t b = 0;
        if (elig[p]) {
            b = m[p] & 0xF;
            if (missing_to_g1 && (m[p] & 0x10)) b |= 1;
        }
        member[p] = b;
        for (int k = 0; k < 4; ++k)
            if (b & (1 << k)) atomic_add_i64(&counts4[k], 1);
    });
}

// ------------------------------------------------------------------------------------ RQ4a
void rq4a_finish(fz_ctx *c, int64_t M, int64_t P, const int64_t *g1t, const int64_t *g1d, const int64_t *g2t,
                 const int64_t *g2d, const int64_t *intro, const int64_t *steps, int64_t *counts, double *sc);

// ---- one-workgroup versions of RQ4a's table passes (iteration tables and project counts of at most
// kFinSmall entries - config 2's 1,000 projects and ~4,000 iterations): one launch each instead of
// a chain of single-purpose maps and scans
constexpr int64_t kFinSmall = 65536;
constexpr int kFinBlock = 1024;
constexpr int kFinWaves = kFinBlock / kWave;

// tot_k[i] = number of projects of group k with more than i builds = sum_{j > i} hist_k[j], i < M
// (hist_k = hist + k (M + 1), k = 0, 1): a suffix scan, each thread a contiguous run from the top
__global__ __launch_bounds__(kFinBlock) void k_rq4a_totals(const int64_t *__restrict__ hist, int64_t M,
                                                          int64_t *__restrict__ t1, int64_t *__restrict__ t2) {
    __shared__ int64_t s_tmp[kFinWaves];
    const int tid = threadIdx.x;
    const int64_t per = (M + kFinBlock - 1) / kFinBlock;
    // thread tid owns j in [a, b) of 1..M, threads in descending order of j (tid 0 the top run)
    const int64_t b = M + 1 - int64_t(tid) * per, a = b - per > 1 ? b - per : 1;
    for (int k = 0; k < 2; ++k) {
        const int64_t *h = hist + k * (M + 1);
        int64_t *tot = k == 0 ? t1 : t2;
        int64_t sum = 0;
        for (int64_t j = a; j < b; ++j) sum += h[j];
        int64_t run = block_excl_scan<int64_t, kFinWaves>(b > a ? sum : 0, s_tmp, (int64_t *)nullptr);
        for (int64_t j = b - 1; j >= a; --j) {
            run += h[j];
            tot[j - 1] = run;
        }
    }
}

// rq4a_finish's table part: the kept rows (both totals >= 100: a prefix), their rates and first
// rate < 5, the after-slices, the positive introduction iterations in project order
__global__ __launch_bounds__(kFinBlock) void k_rq4a_finish_small(int64_t M, int64_t P, const int64_t *__restrict__ g1t,
                                                                const int64_t *__restrict__ g1d,
                                                                const int64_t *__restrict__ g2t,
                                                                const int64_t *__restrict__ g2d,
                                                                const int64_t *__restrict__ intro, int64_t *counts,
                                                                double *__restrict__ rates, double *__restrict__ after,
                                                                double *__restrict__ iv, int64_t *__restrict__ d_np) {
    chain_prio();
    __shared__ int64_t s_tmp[kFinWaves];
    __shared__ unsigned long long s_rows, s_first[2];
    const int tid = threadIdx.x;
    const int64_t MM = M > 0 ? M : 1;
    if (tid == 0) {
        s_rows = 0ull;
        s_first[0] = s_first[1] = ~0ull;
    }
    __syncthreads();
    unsigned long long rows = 0, f0 = ~0ull, f1 = ~0ull;
    for (int64_t i = tid; i < M; i += kFinBlock) {
        const int64_t a = g1t[i], b = g2t[i];
        if (a < 100 || b < 100) continue;
        ++rows;
        const double r1 = a > 0 ? double(g1d[i]) / double(a) * 100.0 : 0.0;
        const double r2 = b > 0 ? double(g2d[i]) / double(b) * 100.0 : 0.0;
        rates[i] = r1;
        rates[MM + i] = r2;
        if (r1 < 5.0 && (unsigned long long)i < f0) f0 = (unsigned long long)i;
        if (r2 < 5.0 && (unsigned long long)i < f1) f1 = (unsigned long long)i;
    }
    rows = wave_sum(rows);
    f0 = wave_min(f0);
    f1 = wave_min(f1);
    if (lane_id() == 0) {
        atomicAdd(&s_rows, rows);
        atomicMin(&s_first[0], f0);
        atomicMin(&s_first[1], f1);
    }
    __syncthreads();  // (also orders this block's rates writes before the after-slice reads)
    const int64_t K = int64_t(s_rows);
    int64_t fk[2], na[2];
    for (int k = 0; k < 2; ++k) {
        fk[k] = s_first[k] == ~0ull ? K : int64_t(s_first[k]);
        na[k] = K - fk[k];
    }
    if (tid == 0) {
        counts[FZ_RQ4A_ROWS] = K;
        counts[FZ_RQ4A_AFTER_G1] = na[0];
        counts[FZ_RQ4A_AFTER_G2] = na[1];
    }
    for (int k = 0; k < 2; ++k)
        for (int64_t j = tid; j < na[k]; j += kFinBlock) after[k * MM + j] = rates[k * MM + fk[k] + j];
    // positive introduction iterations, in project order
    const int64_t per = (P + kFinBlock - 1) / kFinBlock;
    const int64_t p0 = int64_t(tid) * per < P ? int64_t(tid) * per : P, p1 = p0 + per < P ? p0 + per : P;
    int64_t cnt = 0;
    for (int64_t p = p0; p < p1; ++p) cnt += intro[p] > 0;
    int64_t tot;
    int64_t q = block_excl_scan<int64_t, kFinWaves>(cnt, s_tmp, &tot);
    for (int64_t p = p0; p < p1; ++p)
        if (intro[p] > 0) iv[q++] = double(intro[p]);
    if (tid == 0) *d_np = tot;
}

void rq4a(fz_ctx *c, const fz_rq4_groups *g, const fz_rq4a_out *o) {
    Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_rq4a: call fz_store_build first");
    FZ_CHECK(g && g->member && g->corpus_us, "fz_rq4a: null groups");
    FZ_CHECK(o && o->counts && o->scalars && o->eligible && o->member && o->g1_total && o->g1_det && o->g2_total &&
                 o->g2_det && o->intro && o->g4_steps && o->g4_transition,
             "fz_rq4a: null output buffer");
    const fz_tables &t = s.t;
    const int64_t P = s.P, M = s.fuzz.max_seg, NI = s.issues.n;
    const int64_t MM = M > 0 ? M : 1;
    int64_t *counts = o->counts;
    double *sc = o->scalars;
    int64_t *hist = c->arena.get<int64_t>(2 * (M + 1));
    int64_t *scratch = c->arena.get<int64_t>(4);
    eligible_projects(c, o->eligible, scratch,
                      {{counts, FZ_RQ4A_NCOUNTS * 8, 0},
                       {o->g1_total, MM * 8, 0},
                       {o->g1_det, MM * 8, 0},
                       {o->g2_total, MM * 8, 0},
                       {o->g2_det, MM * 8, 0},
                       {o->intro, (P > 0 ? P : 1) * 8, 0xff},
                       {o->g4_steps, 30 * 8, 0},
                       {o->g4_transition, 4 * 8, 0},
                       {hist, 2 * (M + 1) * 8, 0}});
    group_members(c, g, o->eligible, o->member, counts + FZ_RQ4A_G1, true);
    const uint8_t *member = o->member;

    TmpView FB, FI;
    filter_views2(c, P, s.fuzz, s.fuzz.n, BuildsBeforeLimit{t.b_time}, FB, s.issues, NI,
                  FixedBeforeLimit{t.i_status, t.i_rts}, FI);
    const int64_t *fboffs = FB.offs, *fbtime = FB.time, *fioffs = FI.offs, *fitime = FI.time;

    // totals[i] += 1 for i = 1..#builds, per group (:339-340)
    // (whole waves: the range is rounded up to 64 so every lane of a wave runs the wave reduction)
    map_n(c, (P + kWave - 1) / kWave * kWave, nullptr, [=] __device__(int64_t p) {
        const int64_t nb = p < P ? fboffs[p + 1] - fboffs[p] : 0;
        const uint8_t b = p < P ? member[p] : 0;
        for (int k = 0; k < 2; ++k)
            if (nb > 0 && (b & (1 << k))) atomic_add_i64(&hist[k * (M + 1) + nb], 1);
        // the longest G1 / G2 series: one atomic per wave, not one per project on one word
        const unsigned long long mx = wave_max((unsigned long long)((nb > 0 && (b & 3)) ? nb : 0));
        if (lane_id() == 0 && mx) atomicMax(reinterpret_cast<unsigned long long *>(&counts[FZ_RQ4A_MAX_ITER]), mx);
    });
    if (M > 0 && M <= kFinSmall) {  // one workgroup: both suffix sums
        k_rq4a_totals<<<1, kFinBlock, 0, c->stream>>>(hist, M, o->g1_total, o->g2_total);
        FZ_LAUNCH_CHECK();
    } else {
        int64_t *rev = c->arena.get<int64_t>(MM), *rex = c->arena.get<int64_t>(MM);
        for (int k = 0; k < 2; ++k) {
            const int64_t *h = hist + k * (M + 1);
            int64_t *tot = k == 0 ? o->g1_total : o->g2_total;
            if (M <= 0) break;
            map_n(c, M, nullptr, [=] __device__(int64_t j) { rev[j] = h[M - j]; });
            scan_exclusive_i64(c, rev, rex, M, nullptr);
            map_n(c, M, nullptr, [=] __device__(int64_t i0) { tot[i0] = rex[M - (i0 + 1)] + rev[M - (i0 + 1)]; });
        }
    }
    // detected[k] |= {p}: k = #builds < issue time (:341-346), distinct per (k, p)
    int64_t *kk = c->arena.get<int64_t>(NI);
    const uint32_t *fiproj = FI.proj;
    const int64_t *d_nfi = FI.d_n;
    map_n(c, NI, d_nfi, [=] __device__(int64_t j) {
        const uint32_t p = fiproj[j];
        const int64_t lo = fboffs[p], hi = fboffs[p + 1];
        kk[j] = (member[p] & 3) ? lower_bound_i64(fbtime, lo, hi, fitime[j]) - lo : 0;
    });
    int64_t *g1d = o->g1_det, *g2d = o->g2_det;
    map_n(c, NI, d_nfi, [=] __device__(int64_t j) {
        const int64_t k = kk[j];
        if (k <= 0) return;
        const uint32_t p = fiproj[j];
        if (j > 0 && fiproj[j - 1] == p && kk[j - 1] == k) return;
        if (member[p] & 1) atomic_add_i64(&g1d[k - 1], 1);
        if (member[p] & 2) atomic_add_i64(&g2d[k - 1], 1);
    });

    // G4: introduction iteration and pre/post windows (:246-299, :350-412) - one wave per project,
    // its 2 x kWin window tests on separate lanes (each two dependent binary searches: one thread
    // walking all fourteen in turn was a 45 us latency chain at config 2)
    const int64_t *cus = g->corpus_us;
    int64_t *intro = o->intro, *steps = o->g4_steps, *trans = o->g4_transition;
    static_assert(2 * kWin <= kWave, "one lane per window");
    map_n(c, P * kWave, nullptr, [=] __device__(int64_t gi) {
        const int64_t p = gi / kWave;
        const int lane = int(gi % kWave);
        if (!(member[p] & 8) || cus[p] == FZ_TS_NULL) return;  // (wave-uniform)
        const int64_t ct = cus[p];
        const int64_t lo = fboffs[p], hi = fboffs[p + 1], nb = hi - lo;
        const int64_t npre = lower_bound_i64(fbtime, lo, hi, ct) - lo;
        if (lane == 0) {
            intro[p] = npre;
            if (npre > 0) atomic_add_i64(&counts[FZ_RQ4A_INTRO_POS], 1);
        }
        if (npre == 0) return;
        const int64_t idx = npre - 1;
        if (idx - (kWin - 1) < 0 || idx + kWin >= nb - 1) return;
        if (lane == 0) counts[FZ_RQ4A_HAS_WINDOW] = 1;
        const int64_t i0 = fioffs[p], i1 = fioffs[p + 1];
        // lane k - 1 (k = 1..kWin): Pre-k = [t[idx-k+1], t[idx-k+2]); lane kWin + k - 1: Post-k
        bool det = false;
        int slot = -1;
        if (lane < 2 * kWin) {
            const bool is_pre = lane < kWin;
            const int k = is_pre ? lane + 1 : lane - kWin + 1;
            const int64_t a = is_pre ? fbtime[lo + idx - (k - 1)] : fbtime[lo + idx + k];
            const int64_t b = is_pre ? fbtime[lo + idx - (k - 1) + 1] : fbtime[lo + idx + k + 1];
            det = lower_bound_i64(fitime, i0, i1, b) > lower_bound_i64(fitime, i0, i1, a);  // an issue in [a, b)
            slot = is_pre ? kWin - k : kWin + k;
            atomic_add_i64(&steps[2 * slot], 1);
            if (det) atomic_add_i64(&steps[2 * slot + 1], 1);
        }
        const uint64_t m = __ballot(det);
        if (lane == 0) {
            const bool pre = (m & ((1ull << kWin) - 1ull)) != 0ull;
            const bool post = ((m >> kWin) & ((1ull << kWin) - 1ull)) != 0ull;
            atomic_add_i64(&trans[(pre && post) ? 0 : pre ? 1 : post ? 2 : 3], 1);
        }
    });
    rq4a_finish(c, M, P, o->g1_total, o->g1_det, o->g2_total, o->g2_det, o->intro, o->g4_steps, counts, sc);
}

static void rq4a_finish_tables(fz_ctx *c, int64_t M, int64_t P, const int64_t *g1t, const int64_t *g1d,
                               const int64_t *g2t, const int64_t *g2d, const int64_t *intro, int64_t *counts,
                               double *rates, double *after, double *iv, int64_t *d_np);

// Finishing of RQ4a from the per-iteration tables, the per-project introduction iterations and the
// G4 step counts (all shard-additive): kept rows, rates, first rate < 5 and the
// after-slices (:156-207, :698-747), introduction stats (:246-299) and pre/post rates (:412-510).
void rq4a_finish(fz_ctx *c, int64_t M, int64_t P, const int64_t *g1t, const int64_t *g1d, const int64_t *g2t,
                 const int64_t *g2d, const int64_t *intro, const int64_t *steps, int64_t *counts, double *sc) {
    const int64_t MM = M > 0 ? M : 1;
    double *rates = c->arena.get<double>(2 * MM);
    double *after = c->arena.get<double>(2 * MM);
    int64_t *nafter = counts + FZ_RQ4A_AFTER_G1;
    fz_describe *dsc = c->arena.get<fz_describe>(3);
    double *iv = c->arena.get<double>(P > 0 ? P : 1);
    int64_t *d_np = c->arena.get<int64_t>(1);
    if (M <= kFinSmall && P <= kFinSmall) {  // the table part in one workgroup
        k_rq4a_finish_small<<<1, kFinBlock, 0, c->stream>>>(M, P, g1t, g1d, g2t, g2d, intro, counts, rates, after, iv,
                                                           d_np);
        FZ_LAUNCH_CHECK();
    } else {
        rq4a_finish_tables(c, M, P, g1t, g1d, g2t, g2d, intro, counts, rates, after, iv, d_np);
    }
    const DescJob jobs[3] = {{after, MM, nafter, dsc}, {after + MM, MM, nafter + 1, dsc + 1}, {iv, P, d_np, dsc + 2}};
    describe_f64_dn_batch(c, jobs, 3);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        sc[FZ_RQ4A_AFTER_G1_MEDIAN] = dsc[0].median;
        sc[FZ_RQ4A_AFTER_G1_IQR] = dsc[0].q3 - dsc[0].q1;
        sc[FZ_RQ4A_AFTER_G2_MEDIAN] = dsc[1].median;
        sc[FZ_RQ4A_AFTER_G2_IQR] = dsc[1].q3 - dsc[1].q1;
        sc[FZ_RQ4A_INTRO_MEAN] = dsc[2].mean;
        sc[FZ_RQ4A_INTRO_MEDIAN] = dsc[2].median;
        sc[FZ_RQ4A_INTRO_MIN] = dsc[2].min;
        sc[FZ_RQ4A_INTRO_MAX] = dsc[2].max;
        int64_t pn = 0, pd = 0, qn = 0, qd = 0;
        for (int k = 1; k <= kWin; ++k) {
            pn += steps[2 * (kWin - k)];
            pd += steps[2 * (kWin - k) + 1];
            qn += steps[2 * (kWin + k)];
            qd += steps[2 * (kWin + k) + 1];
        }
        sc[FZ_RQ4A_PRE_RATE] = pn ? double(pd) / double(pn) * 100.0 : 0.0;
        sc[FZ_RQ4A_POST_RATE] = qn ? double(qd) / double(qn) * 100.0 : 0.0;
    });
}

// rq4a_finish's table part for large tables (device-wide maps and scans)
static void rq4a_finish_tables(fz_ctx *c, int64_t M, int64_t P, const int64_t *g1t, const int64_t *g1d,
                               const int64_t *g2t, const int64_t *g2d, const int64_t *intro, int64_t *counts,
                               double *rates, double *after, double *iv, int64_t *d_np) {
    const int64_t MM = M > 0 ? M : 1;
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        counts[FZ_RQ4A_ROWS] = 0;
        counts[FZ_RQ4A_AFTER_G1] = 0;
        counts[FZ_RQ4A_AFTER_G2] = 0;
    });
    // rows with both totals >= 100 (a prefix), rates, first rate < 5, after-slices (:156-207, :698-747)
    int64_t *first = c->arena.get<int64_t>(2);
    map_n(c, 1, nullptr, [=] __device__(int64_t) { first[0] = first[1] = INT64_MAX; });
    map_n(c, M, nullptr, [=] __device__(int64_t i) {
        const int64_t a = g1t[i], b = g2t[i];
        if (a < 100 || b < 100) return;
        atomic_add_i64(&counts[FZ_RQ4A_ROWS], 1);
        const double r1 = a > 0 ? double(g1d[i]) / double(a) * 100.0 : 0.0;
        const double r2 = b > 0 ? double(g2d[i]) / double(b) * 100.0 : 0.0;
        rates[i] = r1;
        rates[MM + i] = r2;
        if (r1 < 5.0) atomicMin(reinterpret_cast<unsigned long long *>(&first[0]), (unsigned long long)i);
        if (r2 < 5.0) atomicMin(reinterpret_cast<unsigned long long *>(&first[1]), (unsigned long long)i);
    });
    int64_t *nafter = counts + FZ_RQ4A_AFTER_G1;
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        const int64_t K = counts[FZ_RQ4A_ROWS];
        for (int k = 0; k < 2; ++k) {
            const int64_t f = first[k] == INT64_MAX ? K : first[k];
            nafter[k] = K - f;
            first[k] = f;
        }
    });
    map_n(c, 2 * MM, nullptr, [=] __device__(int64_t i) {
        const int k = i >= MM;
        const int64_t j = i - k * MM;
        if (j < nafter[k]) after[k * MM + j] = rates[k * MM + first[k] + j];
    });

    // introduction-iteration stats over the positive ones (pandas Series mean/median/min/max)
    int64_t *pf = c->arena.get<int64_t>(P), *pp = c->arena.get<int64_t>(P);
    map_n(c, P, nullptr, [=] __device__(int64_t p) { pf[p] = intro[p] > 0 ? 1 : 0; });
    scan_exclusive_i64(c, pf, pp, P, d_np);
    map_n(c, P, nullptr, [=] __device__(int64_t p) {
        if (pf[p]) iv[pp[p]] = double(intro[p]);
    });
}

// ------------------------------------------------------------------------------------ RQ4b
struct FullTrendRows {  // get_full_coverage_trend: coverage > 0, date < LIMIT (rq4b:315-326), G1/G2 only
    static constexpr int kBytes = 21;  // column bytes read per row (filter_compact probe)
    const uint32_t *proj;
    const double *cov;
    const uint8_t *valid;
    const int64_t *date;
    const uint8_t *member;
    __device__ bool operator()(int32_t r) const {
        return bool(valid[r] & FZ_VALID_COVERAGE) & (cov[r] > 0.0) & (date[r] < kLim4) & bool(member[proj[r]] & 3);
    }
};
// A filter emitter: the kept row's coverage value and its project (rq4b's full series).
struct ValueProjEmit {
    static constexpr bool kTime = false;
    double *val;
    uint32_t *oproj;
    const double *cov;
    __device__ void operator()(int64_t q, int32_t r, int64_t, uint32_t pj) const {
        val[q] = cov[r];
        oproj[q] = pj;
    }
};
struct PositiveCoverage34 {  // get_coverage_deltas: coverage > 0, any date (rq4b:745-772), G3/G4 only
    static constexpr int kBytes = 13;  // column bytes read per row (filter_compact probe)
    const uint32_t *proj;
    const double *cov;
    const uint8_t *valid;
    const uint8_t *member;
    __device__ bool operator()(int32_t r) const {
        return bool(valid[r] & FZ_VALID_COVERAGE) & (cov[r] > 0.0) & bool(member[proj[r]] & 12);
    }
};

// mannwhitneyu (two-sided p; U1 of 'greater' -> Cliff's delta), brunnermunzel and levene of the
// initial-coverage samples a[0, *n2) (G2) and b[0, *n1) (G1) (rq4b_coverage.py:248-313)
void two_sample_tests(fz_ctx *c, const double *a, int64_t na_cap, const int64_t *n2, const double *b,
                      int64_t nb_cap, const int64_t *n1, double *ts) {
    if (two_sample_small_ok(na_cap, nb_cap)) {  // small samples (config 2: one per project): one launch
        two_sample_small(c, a, n2, b, n1, ts + FZ_RQ4B_MWU_P, ts + FZ_RQ4B_BM_STAT, ts + FZ_RQ4B_BM_P,
                         ts + FZ_RQ4B_CLIFF, ts + FZ_RQ4B_LEVENE_W);
        return;
    }
    const int64_t cap = (na_cap > 0 ? na_cap : 1) + (nb_cap > 0 ? nb_cap : 1);
    double *v = c->arena.get<double>(cap);
    uint8_t *gr = c->arena.get<uint8_t>(cap);
    int64_t *oall = c->arena.get<int64_t>(2);  // {0, *n2 + *n1}: offsets of the union's one segment
    map_n(c, cap, nullptr, [=] __device__(int64_t i) {
        const int64_t na = *n2, nb = *n1;
        if (i == 0) {
            oall[0] = 0;
            oall[1] = na + nb;
        }
        if (i < na) {
            v[i] = a[i];
            gr[i] = 0;
        } else if (i < na + nb) {
            v[i] = b[i - na];
            gr[i] = 1;
        }
    });
    Segs one{1, oall, cap};
    int32_t *sid = segment_ids(c, one);
    double *u1 = c->arena.get<double>(1);
    RankTestOut rt;
    rt.mwu_p_two = ts + FZ_RQ4B_MWU_P;
    rt.u1 = u1;
    rt.bm_stat = ts + FZ_RQ4B_BM_STAT;
    rt.bm_p = ts + FZ_RQ4B_BM_P;
    rt.exact_scratch = c->arena.get<double>(8 * cap + 1);
    seg_rank_tests(c, v, gr, one, sid, rt);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        ts[FZ_RQ4B_CLIFF] = (2.0 * u1[0]) / (double(*n2) * double(*n1)) - 1.0;
    });
    // levene's medians by selection (one launch for both samples, no sorted copies)
    fz_describe *dd = c->arena.get<fz_describe>(2);
    const DescJob jobs[2] = {{a, na_cap, n2, dd}, {b, nb_cap, n1, dd + 1}};
    describe_f64_dn_batch(c, jobs, 2);
    levene_two_med(c, &dd[0].median, a, na_cap, n2, &dd[1].median, b, nb_cap, n1, ts + FZ_RQ4B_LEVENE_W);
}

// Per-session quartiles / counts / Brunner-Munzel of G2 vs G1 (:910-1015) from values v2 ordered
// by segment id sid2 = 2 * session + group (group 0 = G2), *d_n live of n_cap
// half_len / sess_len: host bounds of one (session, group) half and of one whole session
// (offs2_in: the segment offsets when the caller has them - values grouped by a session exchange)
void rq4b_sessions(fz_ctx *c, const double *v2, const uint32_t *sid2, int64_t n_cap, const int64_t *d_n, int64_t MM,
                   int64_t half_len, int64_t sess_len, int64_t *c2, int64_t *c1, double *g2q, double *g1q,
                   double *pbm, const int64_t *offs2_in = nullptr) {
    const int64_t S2 = 2 * MM, NC = n_cap, P = half_len;
    const int64_t *d_nf = d_n;
    const int64_t *offs2 = offs2_in;  // segment 2i: session i's G2 values, 2i + 1: G1
    if (!offs2) {
        int64_t *o2 = c->arena.get<int64_t>(S2 + 1);
        segment_offsets_dn(c, sid2, d_nf, NC, S2, o2);
        offs2 = o2;
    }
    // Brunner-Munzel from the sorted halves: per-thread merge walks for short halves, both halves in
    // LDS for sessions of up to kBmLdsMax values, else the device-wide rank passes
    const bool lds = P > kBmHalvesMax && sess_len <= kBmLdsMax;
    const bool small = P <= kBmHalvesMax || lds;
    if (!small && !sid2)  // (segment ids only for the device-wide rank passes; null from the transpose)
        sid2 = reinterpret_cast<const uint32_t *>(segment_ids(c, Segs{S2, offs2, NC}));
    int32_t *sess = small ? nullptr : c->arena.get<int32_t>(NC);
    uint8_t *grp2 = small ? nullptr : c->arena.get<uint8_t>(NC);
    int64_t *soffs = small && !lds ? nullptr : c->arena.get<int64_t>(MM + 1);
    map_n(c, small ? MM + 1 : (NC > MM + 1 ? NC : MM + 1), nullptr, [=] __device__(int64_t k) {
        if (k < MM) {
            c2[k] = offs2[2 * k + 1] - offs2[2 * k];
            c1[k] = offs2[2 * k + 2] - offs2[2 * k + 1];
        }
        if (soffs && k <= MM) soffs[k] = offs2[2 * k];
        if (small) return;
        if (k < NC) {
            sess[k] = int32_t(sid2[k] >> 1);
            grp2[k] = uint8_t(sid2[k] & 1u);
        }
    });
    Segs sg2{S2, offs2, NC, P};
    SortedSegs ss2 = seg_sort_f64(c, v2, sg2, nullptr);
    const double q3[3] = {25.0, 50.0, 75.0};
    seg_percentiles(c, sg2, ss2.val, q3, 3, g2q, nullptr, g1q);  // (segment 2i -> G2 row i, 2i + 1 -> G1)
    // per-session Brunner-Munzel (:978-985; NaN unless both sides >= 5)
    if (lds) {
        bm_halves(c, ss2.val, offs2, soffs, MM, NC, 5, pbm);
        return;
    }
    if (small) {
        bm_sorted_halves(c, ss2.val, offs2, MM, 5, pbm);
        return;
    }
    RankTestOut rt;
    rt.bm_p = pbm;
    seg_rank_tests(c, v2, grp2, Segs{MM, soffs, NC, sess_len}, sess, rt);
    map_n(c, MM, nullptr, [=] __device__(int64_t i) {
        if (!(c2[i] >= 5 && c1[i] >= 5)) pbm[i] = NAN;
    });
}

__global__ void k_rq4b_keys(const int64_t *__restrict__ sid, const uint8_t *__restrict__ grp, int64_t n,
                            uint32_t *__restrict__ keys) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
        keys[i] = uint32_t(sid[i]) * 2u + (grp[i] ? 1u : 0u);
}

void rq4b_session_stats(fz_ctx *c, const double *values, const int64_t *sid, const uint8_t *grp, int64_t n, int64_t S,
                        int64_t max_len, int64_t *c2, int64_t *c1, double *g2q, double *g1q, double *pbm) {
    hipStream_t st = c->stream;
    const int64_t MM = S > 0 ? S : 1;
    FZ_CHECK(2 * MM < (int64_t(1) << 32), "fz_rq4b_session_stats: too many sessions");
    uint32_t *key = c->arena.get<uint32_t>(n);
    const double *svals = values;  // the values ride along as the sort's payload (no gather after)
    if (n > 0) {
        k_rq4b_keys<<<grid_for(n), kBlock, 0, st>>>(sid, grp, n, key);
        FZ_LAUNCH_CHECK();
        RadixPayload pl;
        pl.n = 1;
        pl.in[0] = values;
        pl.size[0] = 8;
        uint32_t *no_vals = nullptr;
        radix_sort_pairs_payload32(c, key, no_vals, n, bits_for(uint64_t(2 * MM)), pl);
        svals = static_cast<const double *>(pl.out[0]);
    }
    double *v2 = c->arena.get<double>(n);
    uint32_t *sid2 = c->arena.get<uint32_t>(n);
    int64_t *d_n = c->arena.get<int64_t>(1);
    set_i64(c, d_n, &n, 1);
    map_n(c, n, nullptr, [=] __device__(int64_t k) {
        v2[k] = svals[k];
        sid2[k] = uint32_t(key[k]);
    });
    // max_len bounds one group of a session: a whole session holds up to twice that
    const int64_t half = max_len > 0 && max_len < n ? max_len : n;
    rq4b_sessions(c, v2, sid2, n, d_n, MM, half, 2 * half < n ? 2 * half : n, c2, c1, g2q, g1q, pbm);
}

// The same from values already grouped by (session, group) segment - the layout a shard's
// fz_rq4b_ex output and fz_runs_merge leave: no key pass and no sort
void rq4b_session_stats_grouped(fz_ctx *c, const double *values, const int64_t *offs2, int64_t n, int64_t S,
                                int64_t max_len, int64_t *c2, int64_t *c1, double *g2q, double *g1q, double *pbm) {
    const int64_t MM = S > 0 ? S : 1;
    FZ_CHECK(2 * MM < (int64_t(1) << 32), "fz_rq4b_session_stats_grouped: too many sessions");
    int64_t *d_n = c->arena.get<int64_t>(1);
    set_i64(c, d_n, &n, 1);
    // max_len bounds a whole session (both groups: at most one value per project), so each half too
    // (segment ids only when the device-wide rank passes need them: rq4b_sessions makes them then)
    const int64_t sess = max_len > 0 && max_len < n ? max_len : n;
    rq4b_sessions(c, values, nullptr, n, d_n, MM, sess, sess, c2, c1, g2q, g1q, pbm, offs2);
}

// The last session index with both groups >= 100 (:849-860) -> *last (-1 if none), and Spearman
// (rho, p) vs index of G1 Q1 / Med / Q3, then G2 Q1 / Med / Q3 over sessions 0..last (:879-899) ->
// sp[12], from the per-session counts and quartiles of MM sessions (device; no host read)
// One workgroup per quartile sequence (sessions of at most kTrendSmall): the last index from the
// counts (every workgroup), the sequence sorted in LDS by (key, index), Spearman vs index off it.
constexpr int64_t kTrendSmall = 4096;
constexpr int kTrendBlock = 512;
__global__ __launch_bounds__(kTrendBlock) void k_rq4b_trends_small(const int64_t *__restrict__ c2,
                                                                  const int64_t *__restrict__ c1,
                                                                  const double *__restrict__ g2q,
                                                                  const double *__restrict__ g1q, int64_t MM,
                                                                  int64_t *__restrict__ last, double *__restrict__ sp) {
    chain_prio();
    __shared__ uint64_t sk[kTrendSmall];
    __shared__ int32_t spos[kTrendSmall];
    __shared__ double s_tmp[kTrendBlock / kWave];
    __shared__ unsigned long long s_last;
    const int tid = threadIdx.x, sgi = blockIdx.x;  // G1 Q1, Med, Q3, then G2 Q1, Med, Q3
    if (tid == 0) s_last = 0ull;
    __syncthreads();
    unsigned long long lp = 0;
    for (int64_t i = tid; i < MM; i += kTrendBlock)
        if (c2[i] >= 100 && c1[i] >= 100) lp = (unsigned long long)(i + 1);
    lp = wave_max(lp);
    if (lane_id() == 0) atomicMax(&s_last, lp);
    __syncthreads();
    const int n = int(s_last);
    if (sgi == 0 && tid == 0) *last = int64_t(n) - 1;
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = tid; i < np2; i += kTrendBlock) {
        sk[i] = i < n ? f64_key(sgi < 3 ? g1q[i * 3 + sgi] : g2q[i * 3 + sgi - 3]) : ~0ull;
        spos[i] = i;
    }
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < (np2 >> 1); t += kTrendBlock) {
                const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ixj = i + j;
                const uint64_t a = sk[i], d = sk[ixj];
                if ((a > d) == ((i & k) == 0)) {
                    sk[i] = d;
                    sk[ixj] = a;
                    const int32_t q = spos[i];
                    spos[i] = spos[ixj];
                    spos[ixj] = q;
                }
            }
            __syncthreads();
        }
    }
    double *sv = reinterpret_cast<double *>(sk);
    for (int i = tid; i < n; i += kTrendBlock) sv[i] = f64_from_key(sk[i]);
    __syncthreads();
    spearman_block<kTrendBlock>(sv, spos, 0, n, s_tmp, sp + 2 * sgi, sp + 2 * sgi + 1);
}

void rq4b_trends(fz_ctx *c, const int64_t *c2, const int64_t *c1, const double *g2q, const double *g1q, int64_t MM,
                 int64_t *last, double *sp) {
    if (MM <= kTrendSmall) {  // (config 2: one launch instead of about a dozen)
        k_rq4b_trends_small<<<6, kTrendBlock, 0, c->stream>>>(c2, c1, g2q, g1q, MM, last, sp);
        FZ_LAUNCH_CHECK();
        return;
    }
    int64_t *lastp1 = c->arena.get<int64_t>(1);
    map_n(c, 1, nullptr, [=] __device__(int64_t) { *lastp1 = 0; });
    map_n(c, MM, nullptr, [=] __device__(int64_t i) {
        if (c2[i] >= 100 && c1[i] >= 100)
            atomicMax(reinterpret_cast<unsigned long long *>(lastp1), (unsigned long long)(i + 1));
    });
    map_n(c, 1, nullptr, [=] __device__(int64_t) { *last = *lastp1 - 1; });
    double *seq = c->arena.get<double>(6 * MM);
    int64_t *offs6 = c->arena.get<int64_t>(7);
    map_n(c, 7, nullptr, [=] __device__(int64_t k) { offs6[k] = k * (*lastp1); });
    map_n(c, 6 * MM, nullptr, [=] __device__(int64_t k) {
        const int64_t n = *lastp1;
        if (n <= 0 || k >= 6 * n) return;
        const int64_t sgi = k / n, i = k % n;  // G1 Q1, Med, Q3, then G2 Q1, Med, Q3
        seq[k] = sgi < 3 ? g1q[i * 3 + sgi] : g2q[i * 3 + sgi - 3];
    });
    Segs s6{6, offs6, 6 * MM, MM};
    ChunkedSegs cs6 = chunked(c, s6);
    int32_t *id6 = segment_ids(c, s6);
    SortedSegs ss6 = seg_sort_f64(c, seq, s6, id6);
    double *rho = c->arena.get<double>(6), *pv = c->arena.get<double>(6);
    spearman_index_sorted(c, cs6, id6, ss6, rho, pv);
    map_n(c, 6, nullptr, [=] __device__(int64_t k) {
        sp[2 * k] = rho[k];
        sp[2 * k + 1] = pv[k];
    });
}

// The sharded step's RQ4b tail, after the session exchange and the gathers: the trends over the
// per-session columns of all M sessions (:849-899), the delta columns put in corpus CSV order
// (:725-797; their keys delta_order[nd] are distinct CSV rows < n_order: scattered by key, then
// compacted in key order - stable, no sort) with the medians of their 14 rows (:797), and the
// initial-coverage tests (:221-313; NaN unless both samples are non-empty) - one call instead of
// the driver's stack / argsort / gather / median / test launches.
void rq4b_tail(fz_ctx *c, const int64_t *c2, const int64_t *c1, const double *g2q, const double *g1q, int64_t M,
               const int64_t *order, const double *pre, const double *post, int64_t nd, int64_t n_order,
               const double *x, int64_t nx, const double *y, int64_t ny, int64_t *last, double *sp, double *pre_out,
               double *post_out, double *med14, double *tests) {
    if (M > 0) {
        rq4b_trends(c, c2, c1, g2q, g1q, M, last, sp);
    } else {
        const int64_t m1 = -1;
        set_i64(c, last, &m1, 1);
    }
    // the columns in key order: slot[k] = 1 + the column holding key k (0: none)
    const int64_t NO = n_order > 0 ? n_order : 1;
    int64_t *slot = c->arena.get<int64_t>(NO);
    int64_t *perm = c->arena.get<int64_t>(nd > 0 ? nd : 1);
    int64_t *offs = c->arena.get<int64_t>(2 * kWin + 1);
    fill_batch(c, {{slot, NO * 8, 0}});
    if (nd > 0) {
        map_n(c, nd, nullptr, [=] __device__(int64_t i) { slot[order[i]] = i + 1; });
        compact_emit<1>(c, NO, nullptr, [=] __device__(int64_t k) { return slot[k] != 0; },
                        [=] __device__(int64_t k, int64_t q) { perm[q] = slot[k] - 1; }, nullptr);
    }
    // pre rows then post rows, [14, nd] row-major, and the 15 row offsets
    double *rows = c->arena.get<double>(2 * kWin * (nd > 0 ? nd : 1));
    map_n(c, 2 * kWin * nd > 2 * kWin + 1 ? 2 * kWin * nd : 2 * kWin + 1, nullptr, [=] __device__(int64_t k) {
        if (k <= 2 * kWin) offs[k] = k * nd;
        if (k >= 2 * kWin * nd) return;
        const int64_t r = k / nd, j = k % nd;
        const int64_t src = (r % kWin) * nd + perm[j];
        const double v = r < kWin ? pre[src] : post[src];
        rows[k] = v;
        (r < kWin ? pre_out : post_out)[k - (r < kWin ? 0 : kWin * nd)] = v;
    });
    double *avg = c->arena.get<double>(2 * kWin), *pct = c->arena.get<double>(10 * kWin);
    int64_t *ge = c->arena.get<int64_t>(1);
    rq2_session_stats_grouped(c, rows, offs, 2 * kWin * nd, 2 * kWin, nd, avg, med14, pct, ge);
    if (nx > 0 && ny > 0) {
        int64_t *d_n = c->arena.get<int64_t>(2);
        const int64_t h[2] = {nx, ny};
        set_i64(c, d_n, h, 2);
        two_sample_tests(c, x, nx, d_n, y, ny, d_n + 1, tests);
    } else {
        map_n(c, FZ_RQ4B_NTESTS, nullptr, [=] __device__(int64_t k) { tests[k] = NAN; });
    }
}

void rq4b(fz_ctx *c, const fz_rq4_groups *g, uint32_t flags, const fz_rq4b_out *o) {
    Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_rq4b: call fz_store_build first");
    FZ_CHECK(g && g->member && g->corpus_us && (g->order || g->n_order == 0), "fz_rq4b: null groups");
    FZ_CHECK(o && o->counts && o->eligible && o->member && o->c2 && o->c1 && o->g2_q && o->g1_q && o->p_bm &&
                 o->spearman6 && o->pre_cov && o->post_cov && o->pre_median && o->post_median && o->init_g2 &&
                 o->init_g1 && o->tests,
             "fz_rq4b: null output buffer");
    const fz_tables &t = s.t;
    // (session axis: at most the rows of one project before the date limit)
    const int64_t P = s.P, M = s.cov.lim_seg, NC = s.cov.n;
    const int64_t MM = M > 0 ? M : 1;
    int64_t *counts = o->counts;
    int64_t *scratch = c->arena.get<int64_t>(4);
    eligible_projects(c, o->eligible, scratch, {{counts, FZ_RQ4B_NCOUNTS * 8, 0}});
    group_members(c, g, o->eligible, o->member, counts + FZ_RQ4B_G1, false);
    const uint8_t *member = o->member;
    const double *cov = t.c_coverage;

    // ---- per-session quartiles and Brunner-Munzel, G2 (x) vs G1 (y) (:910-1015)
    // the filter writes each kept row's coverage value and project itself (no (row, time, project)
    // copy gathered through afterwards); G1 / G2 projects' rows before the limit only (range scan)
    TmpView F;
    // (project-major output: the filter writes the series into the caller's trend_values, the
    // per-project offsets follow into trend_offsets - the runs of the sharded session exchange)
    const bool pmajor = (flags & FZ_RQ4B_PROJECT_MAJOR) && (flags & FZ_RQ4B_SKIP_SESSION_STATS) && o->trend_values &&
                        o->trend_offsets;
    double *fval = pmajor ? o->trend_values : c->arena.get<double>(NC);
    F.proj = c->arena.get<uint32_t>(NC);
    const ValueProjEmit fe{fval, F.proj, cov};
    filter_view(c, s.cov, NC, P,
                FullTrendRows{t.c_project, t.c_coverage, t.c_valid, t.c_date, member}, F, nullptr,
                Selection::segments(member, 3, nullptr, s.cov.offs, kLim4), NoCount{}, &fe, 20.0);
    const int64_t *foffs = F.offs;
    const double *fv0 = fval;
    const uint32_t *fproj = F.proj;
    const int64_t *d_nf = F.d_n;
    per_seg(c, P > 0 ? P : 1, [=] __device__(int64_t p) {
        if (p < P)
            atomicMax(reinterpret_cast<unsigned long long *>(&counts[FZ_RQ4B_SESSIONS]),
                      (unsigned long long)(foffs[p + 1] - foffs[p]));
        if (p == 0) counts[FZ_RQ4B_VALUES] = *d_nf;
    });
    const bool sharded = flags & FZ_RQ4B_SKIP_SESSION_STATS;
    // a shard's contribution to the session exchange: its values grouped by (session, group)
    // segment, as the unsharded path groups them before the statistics
    const bool contribute = o->trend_values && o->trend_offsets && !pmajor;
    if (pmajor) dev_copy(c, o->trend_offsets, foffs, (P + 1) * int64_t(sizeof(int64_t)));
    int64_t *c2 = o->c2, *c1 = o->c1;
    double *g2q = o->g2_q, *g1q = o->g1_q;
    if (!sharded || (contribute && !pmajor)) {
        const int64_t S2 = 2 * MM;
        if (ragged_transpose_ok(P, MM, 2)) {
            // the ragged transpose (fz_transpose.h): value i of project p straight to segment
            // (i, group) in project order, read through the view's rows - no sort, no gather pass
            double *v2 = contribute ? o->trend_values : c->arena.get<double>(NC);
            int64_t *o2 = contribute ? o->trend_offsets : c->arena.get<int64_t>(S2 + 1);
            ragged_transpose<2>(c, foffs, P, MM, NC, [=] __device__(int64_t j) { return fv0[j]; },
                                [=] __device__(int64_t p) { return (member[p] & 2) ? 0 : 1; }, v2, o2);
            if (!sharded) rq4b_sessions(c, v2, nullptr, NC, d_nf, MM, P, P, c2, c1, g2q, g1q, o->p_bm, o2);
        } else {
            // (session, group) key per value: G2 -> group 0 (x), G1 -> group 1 (y); the values are in
            // project order, so the stable sort on (session, group) alone keeps projects in order
            // the values (read in view order: rising rows) ride along as the sort's payload - no random
            // double gather through the permutation afterwards
            const int sbits = bits_for(uint64_t(S2 + 1));
            uint32_t *key = c->arena.get<uint32_t>(NC);  // (2 * index + group < 2^32: < 2^31 rows)
            double *fv = c->arena.get<double>(NC);
            map_n(c, NC, nullptr, [=] __device__(int64_t j) {
                if (j < *d_nf) {
                    const uint32_t p = fproj[j];
                    const uint32_t grp = (member[p] & 2) ? 0u : 1u;
                    key[j] = uint32_t(j - foffs[p]) * 2u + grp;
                    fv[j] = fv0[j];
                } else {
                    key[j] = uint32_t(S2);
                }
            });
            RadixPayload pl;
            pl.n = 1;
            pl.in[0] = fv;
            pl.size[0] = 8;
            uint32_t *no_vals = nullptr;
            radix_sort_pairs_payload32(c, key, no_vals, NC, sbits, pl);
            const double *sfv = static_cast<const double *>(pl.out[0]);
            double *v2 = contribute ? o->trend_values : c->arena.get<double>(NC);
            uint32_t *sid2 = c->arena.get<uint32_t>(NC);
            map_n(c, NC, nullptr, [=] __device__(int64_t k) {
                sid2[k] = uint32_t(key[k]);
                if (k < *d_nf) v2[k] = sfv[k];
            });
            if (contribute) segment_offsets_dn(c, sid2, d_nf, NC, S2, o->trend_offsets);
            if (!sharded)
                rq4b_sessions(c, v2, sid2, NC, d_nf, MM, P, P, c2, c1, g2q, g1q, o->p_bm,
                              contribute ? o->trend_offsets : nullptr);  // <= 1 value per project
        }
    }
    // last session with both groups >= 100 (:849-860); Spearman of the quartile sequences (:879-899)
    if (!sharded) rq4b_trends(c, c2, c1, g2q, g1q, MM, counts + FZ_RQ4B_LAST, o->spearman6);

    // ---- coverage deltas around the corpus date for G3 u G4, CSV order (:725-797)
    {
        TmpView PC;
        filter_view(c, s.cov, NC, P,
                    PositiveCoverage34{t.c_project, t.c_coverage, t.c_valid, member}, PC, nullptr,
                    Selection{member, 12, nullptr, s.cov.offs});  // (G3 / G4: their rows only, virtual rows)
        const int64_t NO = g->n_order;
        const int64_t NOC = NO > 0 ? NO : 1;
        int64_t *df = c->arena.get<int64_t>(NOC), *dp = c->arena.get<int64_t>(NOC), *dj = c->arena.get<int64_t>(NOC);
        const int32_t *order = g->order;
        const int64_t *cus = g->corpus_us;
        const int64_t *pcoffs = PC.offs, *pctime = PC.time;
        const int32_t *pcrow = PC.row;
        map_n(c, NOC, nullptr, [=] __device__(int64_t k) {
            df[k] = 0;
            if (k >= NO) return;
            const int32_t p = order[k];
            if (!(member[p] & 12) || cus[p] == FZ_TS_NULL) return;
            const int64_t cd = fdiv4(cus[p], kDay4) * kDay4;  // corpus_time.date() (UTC)
            const int64_t lo = pcoffs[p], hi = pcoffs[p + 1];
            const int64_t j = lower_bound_i64(pctime, lo, hi, cd);
            if (j - lo >= kWin && hi - j >= kWin) {
                df[k] = 1;
                dj[k] = j;
            }
        });
        int64_t *d_nd = counts + FZ_RQ4B_DELTA_PROJECTS;
        scan_exclusive_i64(c, df, dp, NOC, d_nd);
        double *pre = o->pre_cov, *post = o->post_cov;
        int64_t *dord = o->delta_order;
        map_n(c, NOC, nullptr, [=] __device__(int64_t k) {
            if (!df[k]) return;
            const int64_t n = *d_nd, q = dp[k], j = dj[k];
            if (dord) dord[q] = k;
            for (int i = 0; i < kWin; ++i) {
                pre[i * n + q] = cov[pcrow[j - 1 - i]];  // DESC LIMIT 7 before the date
                post[i * n + q] = cov[pcrow[j + i]];     // first 7 from the date
            }
        });
        if (!sharded) {
        int64_t *offs7 = c->arena.get<int64_t>(kWin + 1);
        map_n(c, kWin + 1, nullptr, [=] __device__(int64_t i) { offs7[i] = i * (*d_nd); });
        Segs s7{kWin, offs7, int64_t(kWin) * (P > 0 ? P : 1), P};
        int32_t *id7 = segment_ids(c, s7);
        SortedSegs sp = seg_sort_f64(c, pre, s7, id7);
        seg_median(c, s7, sp.val, o->pre_median);
        SortedSegs so = seg_sort_f64(c, post, s7, id7);
        seg_median(c, s7, so.val, o->post_median);
        }
    }

    // ---- initial coverage of G2 vs G1 (:221-313)
    {
        int64_t *f2 = c->arena.get<int64_t>(P), *f1 = c->arena.get<int64_t>(P);
        int64_t *q2 = c->arena.get<int64_t>(P), *q1 = c->arena.get<int64_t>(P);
        map_n(c, P, nullptr, [=] __device__(int64_t p) {
            const bool has = foffs[p + 1] > foffs[p];
            f2[p] = has && (member[p] & 2);
            f1[p] = has && (member[p] & 1);
        });
        int64_t *n2 = counts + FZ_RQ4B_INIT_G2, *n1 = counts + FZ_RQ4B_INIT_G1;
        scan_exclusive_i64(c, f2, q2, P, n2);
        scan_exclusive_i64(c, f1, q1, P, n1);
        double *a = o->init_g2, *b = o->init_g1;
        map_n(c, P, nullptr, [=] __device__(int64_t p) {
            if (f2[p]) a[q2[p]] = fv0[foffs[p]];
            if (f1[p]) b[q1[p]] = fv0[foffs[p]];
        });
        if (!sharded) two_sample_tests(c, a, P, n2, b, P, n1, o->tests);
    }
}

}  // namespace fz
