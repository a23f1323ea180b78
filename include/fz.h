/*
 * fz.h - C ABI of libfz, the MI355X (gfx950) analytics engine for the RQ1-RQ4 computations of
 * the "1 million fuzzing sessions" replication package.
 *
 * What this boundary replaces (reference paths relative to /root/reference):
 *   program/__module/dbFile.py:5-38        DB(...).connect() / executeQuery("select", sql) -> rows.
 *                                          Every RQ script fetches session rows through it; the
 *                                          columnar store (fz_store_build) is its replacement.
 *   program/__module/queries1.py:15-314    the SQL the scripts send (GROUP BY/HAVING eligibility,
 *                                          as-of joins with ROW_NUMBER, per-project ordered scans).
 *   program/research_questions/rq*.py      the Python loops + numpy/scipy statistics over those rows
 *                                          (one fz_rq* entry point per script, see each declaration).
 *
 * Conventions
 *   - Every pointer in fz_tables and in the *_out structs is a DEVICE pointer (HBM), owned by the
 *     caller; the library never frees or retains them past the call (fz_tables must stay alive
 *     until the fz_rq* calls that use the store built from it have returned).
 *   - The library allocates only scratch and the sorted store, owned by the opaque fz_ctx.
 *   - Every call returns 0 on success or a negative FZ_E* code; fz_last_error() returns a
 *     thread-local message for the last failure.  No C++ exception crosses this boundary.
 *   - Calls on one fz_ctx are serialised by the caller; contexts on different GPUs may be used
 *     concurrently (one host thread / process per GPU).  All work is enqueued on the stream
 *     given to fz_ctx_create; a call returns after its device results are complete.
 *   - Timestamps are int64 microseconds since 1970-01-01 of the naive DB value; FZ_TS_NULL marks
 *     SQL NULL.  Codes: build_type 0 Fuzzing / 1 Coverage; result 0 'Finish', 1 'Halfway',
 *     2 'HalfWay', 3 'Error', 255 NULL; status 0 'Fixed', 1 'Fixed (Verified)', others not fixed.
 */
#ifndef FZ_H
#define FZ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FZ_ABI_VERSION 1
#define FZ_TS_NULL INT64_MAX

#define FZ_OK 0
#define FZ_E_INVALID (-1)   /* bad argument / shape */
#define FZ_E_DEVICE (-2)    /* HIP runtime error */
#define FZ_E_STATE (-3)     /* call order (e.g. fz_rq* before fz_store_build) */
#define FZ_E_NOMEM (-4)

/* validity bits of fz_tables.c_valid */
#define FZ_VALID_COVERAGE 1u
#define FZ_VALID_COVERED 2u
#define FZ_VALID_TOTAL 4u

typedef struct fz_ctx fz_ctx;

/* The four session tables in columnar form (schema: SURVEY.md 8(c)).  Row order is arbitrary
 * (heap order); the store sorts.  All arrays are device pointers. */
typedef struct fz_tables {
    int64_t n_projects;          /* project ids are 0..n_projects-1, id order == byte order of names */
    /* buildlog_data (queries1.py:18-55) */
    int64_t n_builds;
    const uint32_t *b_project;
    const uint8_t *b_type;
    const uint8_t *b_result;
    const int64_t *b_time;       /* timecreated */
    const int32_t *b_group;      /* id of str(modules)+'_'+str(revisions)  (rq2_coverage_and_added.py:129) */
    const int32_t *b_rev_canon;  /* id of sorted(revisions[1:-2].split(',')), -1 NULL (rq3:280) */
    /* total_coverage (3_get_coverage_data.py:132) */
    int64_t n_cov;
    const uint32_t *c_project;
    const int64_t *c_date;
    const double *c_coverage;
    const int64_t *c_covered;
    const int64_t *c_total;
    const uint8_t *c_valid;      /* FZ_VALID_* bits */
    /* issues (queries1.py:20-43) */
    int64_t n_issues;
    const int64_t *i_number;
    const uint32_t *i_project;
    const int64_t *i_rts;
    const uint8_t *i_status;
    /* project_info: number of rows per project id (queries1.py:292-295 inner join) */
    const int32_t *pi_count;
} fz_tables;

/* Returned by fz_store_build: sizes the caller needs to allocate fz_rq* outputs. */
typedef struct fz_store_stats {
    int64_t n_projects;
    int64_t n_fuzz;                 /* Fuzzing builds (any result, any time) */
    int64_t n_coverage_builds;
    int64_t max_fuzz_per_project;   /* RQ1 iteration axis length upper bound */
    int64_t max_cov_per_project;    /* coverage rows of one project */
    int64_t sort_passes;            /* radix passes run (builds + coverage + issues) */
} fz_store_stats;

/* Numbers of rq3's print_summary_statistics (rq3_diff_coverage_at_detection.py:25-66) and the RQ1
 * late-stage block (rq1_detection_rate.py:256-268): numpy mean (pairwise), median, std(ddof=0),
 * percentile(linear) 25/75, min, max, counts. */
typedef struct fz_describe {
    int64_t count, n_pos, n_zero, n_neg;
    double mean, median, std, min, max, q1, q3;
    double min_nonzero;             /* NaN if none */
    int64_t has_nonzero;
} fz_describe;

/* ---- context ---------------------------------------------------------------------------- */
int fz_abi_version(void);
const char *fz_last_error(void);
/* stream: a hipStream_t (NULL = the device's null stream). */
int fz_ctx_create(int device, void *stream, fz_ctx **out);
/* A context that runs analyses on its own stream over `parent`'s store (built by the parent; read
 * only): the six analyses of one store can run concurrently, one child per stream (and host
 * thread - calls on one context are serialised by the caller).  The parent must outlive it and
 * must not rebuild its store while a child's work is in flight (order the streams). */
int fz_ctx_create_child(fz_ctx *parent, void *stream, fz_ctx **out);
int fz_ctx_destroy(fz_ctx *ctx);
/* Re-target the context to another stream (e.g. torch's current stream). */
int fz_ctx_set_stream(fz_ctx *ctx, void *stream);

/* ---- store: replaces the PostgreSQL tables + indexes behind dbFile.DB ------------------ */
/* Sorts buildlog_data by (build_type, project, timecreated), total_coverage by (project, date),
 * issues by (project, rts) (stable: ties keep row order), builds per-project segment offsets. */
int fz_store_build(fz_ctx *ctx, const fz_tables *t, fz_store_stats *stats);
/* Up to 4 children of ctx (fz_ctx_create_child) that fz_store_build may use while it runs - the
 * three tables' prefix sorts and the time-sort length classes are independent, and are forked onto
 * the helpers' streams / contexts (joined before the build returns).  The helpers must be idle
 * during the build (the caller orders their streams after it, as for any child); n = 0 turns it
 * off.  No reference counterpart: the PostgreSQL restore builds the indexes one after another. */
int fz_store_set_helpers(fz_ctx *ctx, fz_ctx *const *helpers, int n);

/* ---- RQ1: rq1_detection_rate.py:101-269 ------------------------------------------------- */
enum {
    FZ_RQ1_ISSUES_LIM = 0,        /* issues with rts < LIMIT                         :121-127 */
    FZ_RQ1_ISSUES_LIM_PROJECTS,
    FZ_RQ1_FIXED_LIM,             /* fixed issues with rts < LIMIT                   :129-136 */
    FZ_RQ1_FIXED_LIM_PROJECTS,
    FZ_RQ1_ELIGIBLE,              /* projects with >= 365 coverage rows              :144-152 */
    FZ_RQ1_WITHOUT_MATCHING,      /* queries1.py:280-314                                      */
    FZ_RQ1_TARGET,                /* :172-185                                                 */
    FZ_RQ1_TARGET_PROJECTS,
    FZ_RQ1_TOTAL_FUZZ,            /* sum of Fuzzing builds of eligible projects       :189-203 */
    FZ_RQ1_MATCHED,               /* SAME_DATE_BUILD_ISSUE rows after ROW_NUMBER dedup        */
    FZ_RQ1_MATCHED_PROJECTS,
    FZ_RQ1_MAX_ITER,              /* length of iter_total / iter_detected                     */
    FZ_RQ1_KEPT_ITERS,            /* iterations with total >= threshold                :233-239 */
    FZ_RQ1_FIRST_DOWN,            /* first kept iteration key with rate < 5, -1 if none :247-253 */
    FZ_RQ1_LATE,                  /* late-stage rates described in late (0 = none)            */
    FZ_RQ1_NCOUNTS = 16
};

typedef struct fz_rq1_out {
    int64_t *counts;              /* [FZ_RQ1_NCOUNTS] */
    uint8_t *eligible;            /* [n_projects] 1 = eligible */
    int64_t *iter_total;          /* [max_fuzz_per_project] projects with >= i Fuzzing builds */
    int64_t *iter_detected;       /* [max_fuzz_per_project] distinct projects detecting at i */
    int64_t *matched_issue;       /* [n_issues] issue rows, ORDER BY project, rts */
    int64_t *matched_build;       /* [n_issues] joined build row */
    fz_describe *late;            /* [1] late-stage detection-rate summary */
} fz_rq1_out;

int fz_rq1(fz_ctx *ctx, int64_t min_project_threshold, const fz_rq1_out *out);

/* Project-sharded RQ1.  SAME_DATE_BUILD_ISSUE dedups with ROW_NUMBER() OVER
 * (PARTITION BY i.number ORDER BY timecreated DESC) (queries1.py:29-32) - across projects, so across
 * shards.  fz_rq1_ex runs fz_rq1 with the other shards' matches as extra competitors: a local
 * match survives only if it beats every competitor with its number (later build time; on a tie the
 * earlier row in ORDER BY project, rts - i.e. a competitor with before = 1 wins ties).  Device
 * arrays of n entries; n = 0 is fz_rq1. */
typedef struct fz_rq1_ext {
    int64_t n;
    const int64_t *number;        /* issue number */
    const int64_t *build_time;    /* matched build timecreated */
    const uint8_t *before;        /* 1: the competitor's shard precedes this one in project order */
} fz_rq1_ext;

int fz_rq1_ex(fz_ctx *ctx, int64_t min_project_threshold, const fz_rq1_ext *ext, const fz_rq1_out *out);

/* Finishing of RQ1 (rq1_detection_rate.py:233-268) on shard-summed iteration tables: recomputes
 * counts[FZ_RQ1_KEPT_ITERS], counts[FZ_RQ1_FIRST_DOWN], counts[FZ_RQ1_LATE] and *late from
 * iter_total / iter_detected[max_iter] (device).  Other counts are left untouched. */
int fz_rq1_finish(fz_ctx *ctx, int64_t min_project_threshold, const int64_t *iter_total,
                  const int64_t *iter_detected, int64_t max_iter, int64_t *counts, fz_describe *late);

/* ---- RQ2 (count): rq2_coverage_count.py:244-483 ------------------------------------------ */
enum {
    FZ_RQ2C_ELIGIBLE = 0,   /* eligible projects                                     :272-280 */
    FZ_RQ2C_SESSIONS,       /* len(coverage_by_session_index) = max(1, longest trend)  :285,330 */
    FZ_RQ2C_GE100,          /* sessions with >= 100 values (a prefix)                  :390 */
    FZ_RQ2C_VALUES,         /* trend values over all projects                          :300-303 */
    FZ_RQ2C_NULL_LINES,     /* fetched rows whose float(covered) / float(total) meets a NULL line
                               count (`x[1] != 0` keeps a None total): the reference raises
                               TypeError there (:300-303), so the caller must when non-zero */
    FZ_RQ2C_NCOUNTS = 8
};
enum {
    FZ_RQ2C_CORR_MEAN = 0,  /* np.mean / np.median of the valid per-project Spearman rho :356-361 */
    FZ_RQ2C_CORR_MEDIAN,
    FZ_RQ2C_SP_RHO,         /* spearmanr(range(K), median_trend)                       :443-445 */
    FZ_RQ2C_SP_P,
    FZ_RQ2C_SW_MEDIAN_P,    /* shapiro(median_trend).pvalue                            :449-458 */
    FZ_RQ2C_NSCALARS = 8
};
typedef struct fz_rq2_count_out {
    int64_t *counts;            /* [FZ_RQ2C_NCOUNTS] */
    double *scalars;            /* [FZ_RQ2C_NSCALARS] */
    uint8_t *eligible;          /* [n_projects] */
    int64_t *raw_n;             /* [n_projects] rows fetched per project (queries1.py:120-129) */
    int64_t *n_trend;           /* [n_projects] values after `total_line != 0` */
    double *sw_w, *sw_p;        /* [n_projects] Shapiro-Wilk (NaN when n < 3)              :305-314 */
    double *corr;               /* [n_projects] Spearman vs index (NaN when undefined)     :316-322 */
    int64_t *session_offsets;   /* [max_cov_per_project + 2] CSR of coverage_by_session_index */
    double *session_values;     /* [n_cov] */
    double *average_trend;      /* [max_cov_per_project] statistics.mean per session       :439 */
    double *median_trend;       /* [max_cov_per_project] statistics.median per session     :440 */
    double *dist_percentiles;   /* [max_cov_per_project * 5] np.percentile 5/25/50/75/95   :139-152 */
    double *dist_mean;          /* [max_cov_per_project] np.mean per session */
} fz_rq2_count_out;

int fz_rq2_count(fz_ctx *ctx, const fz_rq2_count_out *out);

/* Project-sharded RQ2 count.  A session index i holds the i-th trend value of
 * every project (project order, rq2_coverage_count.py:330-333), so per-session statistics need the
 * values of all shards: each shard runs fz_rq2_count_ex with FZ_RQ2C_SKIP_SESSION_STATS (per-project
 * outputs + its session-major values), the values are exchanged by session index (all-to-all), and
 * the owner of a session range runs fz_rq2_session_stats on what it received. */
#define FZ_RQ2C_SKIP_SESSION_STATS 1u  /* no per-session / median-trend / correlation summaries */
/* (with SKIP_SESSION_STATS) the trend values project-major instead of session-major: session_values
 * = every eligible project's values in (project, date) order, project p's n_trend[p] of them after the
 * earlier projects' (session_offsets not written) - the runs fz_pack_runs sends to the session owners */
#define FZ_RQ2C_PROJECT_MAJOR 2u
int fz_rq2_count_ex(fz_ctx *ctx, uint32_t flags, const fz_rq2_count_out *out);

/* Per-session statistics (:139-152, :390, :439-440) of n_values (session id, value) pairs, ids in
 * [0, n_sessions); pairs of one session keep their input order (stable).  average / median:
 * statistics.mean / statistics.median, percentiles[s * 5 + j]: np.percentile at 5/25/50/75/95,
 * n_ge100[0] = sessions with >= 100 values.  Empty sessions get NaN.  max_session_len: a host upper
 * bound of one session's size (e.g. the number of projects), 0 if unknown. */
int fz_rq2_session_stats(fz_ctx *ctx, const double *values, const int64_t *session_ids, int64_t n_values,
                         int64_t n_sessions, int64_t max_session_len, double *average, double *median,
                         double *percentiles, int64_t *n_ge100);

/* fz_rq2_session_stats over values already grouped by session: session s holds
 * values[session_offsets[s], session_offsets[s + 1]) (session_offsets [n_sessions + 1], device,
 * offsets[0] = 0, in the order the reference pools them - project order).  A shard's
 * fz_rq2_count_ex output (session_values / session_offsets) and fz_runs_merge's output have this
 * layout, so the sharded path's owner needs no per-value session ids and no sort. */
int fz_rq2_session_stats_grouped(fz_ctx *ctx, const double *values, const int64_t *session_offsets, int64_t n_values,
                                 int64_t n_sessions, int64_t max_session_len, double *average, double *median,
                                 double *percentiles, int64_t *n_ge100);

/* The session exchange's receive side: n_runs runs (one per source shard, one after another in
 * `values`), each grouped by segment over n_segments segments, are merged segment by segment:
 * out = for each segment s, run 0's values of s, then run 1's, ... (sources in rank order = global
 * project order); out_offsets [n_segments + 1].  run_sizes: device [n_runs * n_segments], run r's
 * count of segment s at r * n_segments + s.  (No reference counterpart: the reference is one
 * process; this is what keeps the sharded per-session pools in its project order.) */
int fz_runs_merge(fz_ctx *ctx, const double *values, const int64_t *run_sizes, int64_t n_runs, int64_t n_segments,
                  double *out, int64_t *out_offsets);

/* scipy.stats.spearmanr(range(n), x) and scipy.stats.shapiro(x) of one device series:
 * out[0..3] = rho, p, W, p (NaN where scipy returns NaN: n < 2 / constant, n < 3). */
int fz_series_tests(fz_ctx *ctx, const double *x, int64_t n, double *out);

/* Read-back of many small device arrays at once (the sharded drivers' per-step host reads): piece i
 * copies n elements of elem_bytes (1, 2, 4 or 8) bytes, `stride` elements apart, from device src to
 * host_out + dst_offset (8-byte elements at 8-byte aligned offsets), on the current device.  One
 * launch on `stream` writing the process's pinned staging area through its device address, one
 * synchronisation of `stream`,
 * then one host copy into host_out [total_bytes] - instead of a gather kernel per strided slice, a
 * concatenation and a blit copy.  (No reference counterpart: the reference is one process.) */
typedef struct fz_host_piece {
    const void *src;
    int64_t n;
    int64_t stride;
    int64_t dst_offset;
    int32_t elem_bytes;
    int32_t pad_;
} fz_host_piece;
int fz_gather_to_host(void *stream, const fz_host_piece *pieces, int n_pieces, void *host_out, int64_t total_bytes);

/* The sharded RQ2-count tail in one call (rq2_coverage_count.py:335-372): fz_series_tests of the
 * first k entries of the gathered median trend (the sessions with >= 100 values) -> out[0..3], and
 * the mean / median of the per-project correlations of eligible projects with raw_n > 0 and a
 * non-NaN correlation (n_projects entries each, device) -> out[4], out[5] (NaN when none).  Device
 * in, device out, no host read. */
int fz_rq2_count_tail(fz_ctx *ctx, const double *median_trend, int64_t k, const double *corr, const int64_t *raw_n,
                      const int64_t *eligible, int64_t n_projects, double *out);

/* scipy.stats.spearmanr(range(n_s), x_s) of S device series at once (segment s = x[offs[s],
 * offs[s+1]), n = offs[S] values, max_len a host bound of one segment, 0 if unknown): rho[s], p[s]
 * (NaN where scipy returns NaN).  Replaces the per-sequence calls of rq4b_coverage.py:879-899 on the
 * sharded path (the six quartile sequences in one call). */
int fz_spearman_index_seg(fz_ctx *ctx, const double *x, int64_t n, const int64_t *offs, int64_t S, int64_t max_len,
                          double *rho, double *p);

/* ---- RQ2/RQ3 support (add): rq2_coverage_and_added.py:73-238 ------------------------------- */
enum { FZ_RQ2A_ELIGIBLE = 0, FZ_RQ2A_ROWS, FZ_RQ2A_RUNS, FZ_RQ2A_NCOUNTS = 4 };
typedef struct fz_rq2_add_out {
    int64_t *counts;            /* [FZ_RQ2A_NCOUNTS] */
    uint8_t *eligible;          /* [n_projects] */
    /* one row per pair of consecutive (modules, revisions) runs, ORDER BY project, time; capacity
     * n_coverage_builds */
    int64_t *row_project;
    int64_t *row_first_build;   /* first build of run i (modules_i / revisions_i)            :135-149 */
    int64_t *row_end_build;     /* last build of run i (timecreated_i)                               */
    int64_t *row_start_build;   /* first build of run i+1                                            */
    int64_t *row_cov_i;         /* coverage row on date(end of run i), -1 none               :170-184 */
    int64_t *row_cov_i1;        /* coverage row on date(start of run i+1)                            */
    double *diff_total;         /* t1 - t0 (NaN unless both totals valid and != 0)           :189-200 */
    double *diff_coverage;      /* c1/t1*100 - c0/t0*100                                             */
    uint8_t *covered_is_float;  /* [n_projects] pandas upcast: a NULL covered_line in the project    */
    uint8_t *total_is_float;    /* [n_projects]                                                      */
} fz_rq2_add_out;

int fz_rq2_add(fz_ctx *ctx, const fz_rq2_add_out *out);

/* ---- RQ3: rq3_diff_coverage_at_detection.py:202-360 -------------------------------------- */
enum {
    FZ_RQ3_ISSUES = 0,
    FZ_RQ3_DETECTED,
    FZ_RQ3_NON_DETECTED,
    FZ_RQ3_ELIGIBLE,
    FZ_RQ3_NON_LAST,              /* non-detected rows of the last issue-bearing project (0 unless
                                     FZ_RQ3_FLUSH_LAST; they are the tail of non_*) */
    FZ_RQ3_NULL_TOTAL,            /* coverage pairs whose `prev[2] > 0 and curr[2] > 0` test meets a NULL
                                     total_line (rq3:253,297): the reference raises TypeError there, so
                                     the caller must too when this is non-zero */
    FZ_RQ3_NULL_LAST,             /* those of them in the flush of the last issue-bearing project
                                     (0 unless FZ_RQ3_FLUSH_LAST; dropped with FZ_RQ3_NON_LAST) */
    FZ_RQ3_NCOUNTS = 8
};
enum {
    FZ_RQ3_AD_DET = 0,            /* anderson(detected).statistic, then 5 critical values   :329 */
    FZ_RQ3_AD_NON = 6,            /* anderson(non-detected)                                 :335 */
    FZ_RQ3_LEVENE_W = 12,         /* levene(det, non) (center='median')                     :344 */
    FZ_RQ3_LEVENE_P,
    FZ_RQ3_BM_STAT,               /* brunnermunzel(det, non)                                :349 */
    FZ_RQ3_BM_P,
    FZ_RQ3_NTESTS = 16
};
typedef struct fz_rq3_out {
    int64_t *counts;              /* [FZ_RQ3_NCOUNTS] */
    uint8_t *eligible;            /* [n_projects] */
    double *det_pct;              /* [n_issues] detected: (c1/t1 - c0/t0) * 100            :296-302 */
    int64_t *det_cov, *det_tot;   /* covered / total line deltas                                   */
    int64_t *det_project, *det_issue;
    double *non_pct;              /* [n_cov] non-detected day-to-day changes               :245-257 */
    int64_t *non_cov, *non_tot;
    fz_describe *describe;        /* [3] detected pct, non-detected pct, detected total    :25-66 */
    double *tests;                /* [FZ_RQ3_NTESTS] */
} fz_rq3_out;

int fz_rq3(fz_ctx *ctx, const fz_rq3_out *out);

/* Project-sharded RQ3.  The reference flushes a project's non-detected changes when the issue loop
 * moves to the next project, so the globally last issue-bearing project is never flushed
 * (rq3:245-257).  With FZ_RQ3_FLUSH_LAST a shard flushes its last project too and reports that
 * project's row count in counts[FZ_RQ3_NON_LAST]; the caller drops those rows on the last shard
 * that has issues and runs the statistics once over the gathered samples (fz_rq3_stats). */
#define FZ_RQ3_FLUSH_LAST 1u
#define FZ_RQ3_SKIP_STATS 2u    /* leave describe / tests untouched (a shard: fz_rq3_stats runs once) */
int fz_rq3_ex(fz_ctx *ctx, uint32_t flags, const fz_rq3_out *out);

/* RQ3 statistics (rq3:321-352) over two device samples: describe[3] (detected pct, non-detected
 * pct, detected total-line delta) and tests[FZ_RQ3_NTESTS] (Anderson x2, Levene, Brunner-Munzel;
 * left unset unless both samples are non-empty). */
int fz_rq3_stats(fz_ctx *ctx, const double *det_pct, const int64_t *det_tot, int64_t n_det, const double *non_pct,
                 int64_t n_non, fz_describe *describe, double *tests);
/* The same with the sample lengths on the device (e.g. &counts[FZ_RQ3_DETECTED] and
 * &counts[FZ_RQ3_NON_DETECTED] of an fz_rq3_ex(FZ_RQ3_SKIP_STATS) call) and host capacities
 * det_cap >= *d_det, non_cap >= *d_non: no host round trip, so the statistics can run on another
 * stream (or graph) after the sample extraction. */
int fz_rq3_stats_dn(fz_ctx *ctx, const double *det_pct, const int64_t *det_tot, int64_t det_cap, const int64_t *d_det,
                    const double *non_pct, int64_t non_cap, const int64_t *d_non, fz_describe *describe,
                    double *tests);

/* ---- RQ4 inputs: data/processed_data/csv/project_corpus_analysis.csv (user_corpus.py:225-233) ---
 * Parsed on the host (it is a ~1k-row CSV) into per-project columns, independent of eligibility:
 *   member[p]   bit g (g = 0..3) set when some CSV row puts p in G(g+1) (rq4a_bug.py:94-108:
 *               time_elapsed_seconds NaN -> G1, == 0 -> G2, (0, 7 d) -> G3, >= 7 d -> G4);
 *               bit 4 when p has no CSV row at all (rq4a adds eligible ones to G1, :110-113)
 *   corpus_us[p]  corpus_commit_time as UTC microseconds (pd.to_datetime(utc=True)), FZ_TS_NULL if none
 *   order[k]    project of the k-th CSV row with a non-NaN time_elapsed_seconds (rq4b :216, :744) */
typedef struct fz_rq4_groups {
    const uint8_t *member;
    const int64_t *corpus_us;
    const int32_t *order;
    int64_t n_order;
} fz_rq4_groups;

/* ---- RQ4a: rq4a_bug.py:653-884 ----------------------------------------------------------- */
enum {
    FZ_RQ4A_MAX_ITER = 0,        /* length of the G1/G2 iteration tables                          */
    FZ_RQ4A_ROWS,                /* iterations where both totals >= 100 (a prefix)         :164-193 */
    FZ_RQ4A_G1, FZ_RQ4A_G2, FZ_RQ4A_G3, FZ_RQ4A_G4,   /* group sizes (eligible)                    */
    FZ_RQ4A_HAS_WINDOW,          /* some G4 project had a full pre/post window             :374-401 */
    FZ_RQ4A_AFTER_G1, FZ_RQ4A_AFTER_G2, /* rates after the first < 5 %                     :698-747 */
    FZ_RQ4A_INTRO_POS,           /* G4 projects with introduction iteration > 0             :277-285 */
    FZ_RQ4A_NCOUNTS = 12
};
enum {
    FZ_RQ4A_AFTER_G1_MEDIAN = 0, FZ_RQ4A_AFTER_G1_IQR, FZ_RQ4A_AFTER_G2_MEDIAN, FZ_RQ4A_AFTER_G2_IQR,
    FZ_RQ4A_INTRO_MEAN, FZ_RQ4A_INTRO_MEDIAN, FZ_RQ4A_INTRO_MIN, FZ_RQ4A_INTRO_MAX,
    FZ_RQ4A_PRE_RATE, FZ_RQ4A_POST_RATE, FZ_RQ4A_NSCALARS = 12
};
typedef struct fz_rq4a_out {
    int64_t *counts;             /* [FZ_RQ4A_NCOUNTS] */
    double *scalars;             /* [FZ_RQ4A_NSCALARS] */
    uint8_t *eligible;           /* [n_projects] */
    uint8_t *member;             /* [n_projects] bit g: project in G(g+1) (eligible, rq4a rules) */
    int64_t *g1_total, *g1_det, *g2_total, *g2_det;  /* [max_fuzz_per_project]       :302-346 */
    int64_t *intro;              /* [n_projects] G4 introduction iteration, -1 n/a       :246-299 */
    int64_t *g4_steps;           /* [15 * 2] (projects, detected) at step s = -7..7 -> (s + 7) */
    int64_t *g4_transition;      /* [4] pre&post, pre only, post only, neither            :806-841 */
} fz_rq4a_out;

int fz_rq4a(fz_ctx *ctx, const fz_rq4_groups *groups, const fz_rq4a_out *out);

/* Finishing of RQ4a on shard-combined inputs: the per-iteration tables summed over
 * shards ([max_iter] each), intro[n_projects] (every shard's own projects) and g4_steps[30] summed.
 * Recomputes counts[FZ_RQ4A_ROWS / AFTER_G1 / AFTER_G2] and every scalars[] entry; other counts
 * (group sizes, INTRO_POS, HAS_WINDOW, MAX_ITER) are the caller's sums / maxima. */
int fz_rq4a_finish(fz_ctx *ctx, const int64_t *g1_total, const int64_t *g1_det, const int64_t *g2_total,
                   const int64_t *g2_det, int64_t max_iter, const int64_t *intro, int64_t n_projects,
                   const int64_t *g4_steps, int64_t *counts, double *scalars);

/* ---- RQ4b: rq4b_coverage.py:1209-1261 ---------------------------------------------------- */
enum {
    FZ_RQ4B_SESSIONS = 0,        /* longest G1/G2 coverage series                          :917-936 */
    FZ_RQ4B_LAST,                /* last session with both groups >= 100 values, -1 none   :849-860 */
    FZ_RQ4B_DELTA_PROJECTS,      /* G3/G4 projects with 7 + 7 coverage points              :725-797 */
    FZ_RQ4B_INIT_G2, FZ_RQ4B_INIT_G1,  /* initial-coverage sample sizes                    :221-246 */
    FZ_RQ4B_G1, FZ_RQ4B_G2, FZ_RQ4B_G3, FZ_RQ4B_G4,
    FZ_RQ4B_VALUES,              /* G1/G2 series values (= trend_offsets[2 * sessions])            */
    FZ_RQ4B_NCOUNTS = 12
};
enum { FZ_RQ4B_MWU_P = 0, FZ_RQ4B_CLIFF, FZ_RQ4B_BM_STAT, FZ_RQ4B_BM_P, FZ_RQ4B_LEVENE_W, FZ_RQ4B_LEVENE_P,
       FZ_RQ4B_NTESTS = 8 };
typedef struct fz_rq4b_out {
    int64_t *counts;             /* [FZ_RQ4B_NCOUNTS] */
    uint8_t *eligible;           /* [n_projects] */
    uint8_t *member;             /* [n_projects] bit g: project in G(g+1) (eligible, rq4b rules) */
    int64_t *c2, *c1;            /* [max_cov_per_project] values per session index, G2 / G1 (the
                                    per-session arrays are written up to counts[FZ_RQ4B_SESSIONS]:
                                    at most the rows of one project before the date limit)      */
    double *g2_q, *g1_q;         /* [max_cov_per_project * 3] np.percentile 25/50/75        :966-972 */
    double *p_bm;                /* [max_cov_per_project] brunnermunzel p, NaN if a side < 5 :978-985 */
    double *spearman6;           /* [12] (rho, p): G1 Q1, Med, Q3, G2 Q1, Med, Q3            :879-899 */
    double *pre_cov, *post_cov;  /* [7 * n_projects] step-major: step i occupies [i*n, i*n+n)  */
    double *pre_median, *post_median; /* [7]                                              :1061-1085 */
    double *init_g2, *init_g1;   /* [n_projects] first coverage per project (sorted ids)   :221-246 */
    double *tests;               /* [FZ_RQ4B_NTESTS] MWU p, Cliff delta, BM, Levene        :248-313 */
    /* optional (may be NULL): what a shard contributes to the cross-shard recombination */
    double *trend_values;        /* [n_cov] G1/G2 full coverage values grouped by (session index,
                                    group): segment 2i = the i-th value of every G2 project, 2i + 1
                                    = of every G1 project, projects in order inside a segment      */
    int64_t *trend_offsets;      /* [2 * max_cov_per_project + 1] segment offsets into trend_values;
                                    entries past 2 * counts[FZ_RQ4B_SESSIONS] unspecified          */
    int64_t *delta_order;        /* [n_projects] CSV row (index into groups->order) of each column  */
} fz_rq4b_out;

int fz_rq4b(fz_ctx *ctx, const fz_rq4_groups *groups, const fz_rq4b_out *out);

/* Project-sharded RQ4b.  A shard runs fz_rq4b_ex with FZ_RQ4B_SKIP_SESSION_STATS
 * (per-project outputs, trend series, delta columns, initial values; no per-session, delta-median or
 * initial-coverage statistics); the G1/G2 values are exchanged by session index and the owner of a
 * session range runs fz_rq4b_session_stats; the initial-coverage samples are gathered for
 * fz_two_sample_tests. */
#define FZ_RQ4B_SKIP_SESSION_STATS 1u
/* (with SKIP_SESSION_STATS) the G1/G2 series project-major: trend_values = their values in
 * (project, date) order, trend_offsets[0 .. n_projects] = per-project offsets into them (capacity
 * n_projects + 1) - the runs of the project-major session exchange */
#define FZ_RQ4B_PROJECT_MAJOR 2u
int fz_rq4b_ex(fz_ctx *ctx, const fz_rq4_groups *groups, uint32_t flags, const fz_rq4b_out *out);

/* Per-session G2 (group 0) vs G1 (group 1) statistics (:910-1015) of n_values (session id, group,
 * value) triples, ids in [0, n_sessions): c2 / c1 counts, g2_q / g1_q [s * 3 + j] np.percentile
 * 25/50/75 (NaN if empty), p_bm brunnermunzel p (NaN unless both sides >= 5).  max_session_len: host
 * bound of one session's size per group (e.g. the number of projects), 0 if unknown. */
int fz_rq4b_session_stats(fz_ctx *ctx, const double *values, const int64_t *session_ids, const uint8_t *groups,
                          int64_t n_values, int64_t n_sessions, int64_t max_session_len, int64_t *c2, int64_t *c1,
                          double *g2_q, double *g1_q, double *p_bm);

/* fz_rq4b_session_stats over values already grouped by (session, group) segment: segment 2s holds
 * session s's G2 values, 2s + 1 its G1 values, values[segment_offsets[k], segment_offsets[k + 1])
 * (segment_offsets [2 * n_sessions + 1], device, offsets[0] = 0) - the layout of a shard's
 * fz_rq4b_ex trend output and of fz_runs_merge over 2 * n_sessions segments.  max_session_len: host
 * bound of one WHOLE session (both groups; the number of projects - one value per project), 0 if
 * unknown. */
int fz_rq4b_session_stats_grouped(fz_ctx *ctx, const double *values, const int64_t *segment_offsets,
                                  int64_t n_values, int64_t n_sessions, int64_t max_session_len, int64_t *c2,
                                  int64_t *c1, double *g2_q, double *g1_q, double *p_bm);

/* RQ4b's trend tests from the per-session tables (device, n_sessions entries; quartiles [s * 3 + j]):
 * *last = the last session index with both groups >= 100 (:849-860; -1 if none) and spearman6 =
 * (rho, p) vs index of G1 Q1 / Med / Q3, then G2 Q1 / Med / Q3 over sessions 0..last (:879-899) -
 * what fz_rq4b computes after its session statistics, for the sharded path's gathered tables. */
int fz_rq4b_trends(fz_ctx *ctx, const int64_t *c2, const int64_t *c1, const double *g2_q, const double *g1_q,
                   int64_t n_sessions, int64_t *last, double *spearman6);

/* Two-sample tests of rq4b's initial coverage (:248-313) on device samples x (G2) and y (G1):
 * out[FZ_RQ4B_MWU_P .. FZ_RQ4B_LEVENE_P] = mannwhitneyu two-sided p, Cliff's delta from
 * mannwhitneyu(greater) U1, brunnermunzel statistic / p, levene W / p. */
int fz_two_sample_tests(fz_ctx *ctx, const double *x, int64_t nx, const double *y, int64_t ny, double *out);

/* The sharded RQ4b tail in one call, after the session exchange and the gathers (the statistics
 * fz_rq4b computes after its session tables, rq4b_coverage.py:725-797, :849-899, :221-313):
 * fz_rq4b_trends over n_sessions per-session rows -> *last, spearman6; the n_delta delta columns
 * (pre_cov / post_cov [7 * n_delta], row-major: window i of column q at i * n_delta + q) put in CSV
 * order by their keys delta_order[n_delta] (distinct, < n_order) -> pre_out / post_out (same
 * layout), with statistics.median of each of the 14 rows -> medians14 (pre rows, then post; NaN when
 * n_delta == 0); fz_two_sample_tests(init_g2, init_g1) -> tests (NaN unless both are non-empty).
 * Device in, device out, no host read. */
int fz_rq4b_tail(fz_ctx *ctx, const int64_t *c2, const int64_t *c1, const double *g2_q, const double *g1_q,
                 int64_t n_sessions, const int64_t *delta_order, const double *pre_cov, const double *post_cov,
                 int64_t n_delta, int64_t n_order, const double *init_g2, int64_t n2, const double *init_g1, int64_t n1,
                 int64_t *last, double *spearman6, double *pre_out, double *post_out, double *medians14,
                 double *tests);

/* ---- a project cut across ranks (config 5's Zipf giant) --------
 * A coverage-only project larger than one rank's share is cut into date ranges on consecutive ranks
 * (tse_amd/parallel.py live_plan).  The reference reads it as one series (queries1.py:120-129,
 * rq2_coverage_count.py:292-333); these calls keep its eligibility, its sessions and its
 * per-project tests exact across the cut.  (No reference counterpart: the reference is one process.) */

/* out[i] = the store's count of qualifying coverage rows (coverage valid, > 0, date < 2025-01-08:
 * rq1:144-152) of project proj[i] on this rank (device in, device out). */
int fz_store_elig_counts(fz_ctx *ctx, const int32_t *proj, int64_t n, int64_t *out);
/* Overrides the store's eligibility of the distinct projects proj[i] by flag[i] (device) until the
 * next fz_store_build - the flags of the whole project's summed counts, set on its first piece's
 * rank, cleared on the others; every analysis after it reads the overridden set.  ctx: the context
 * that built the store. */
int fz_store_set_eligible(fz_ctx *ctx, const int32_t *proj, const uint8_t *flag, int64_t n);

/* One project's filtered coverage values on this rank, date order (out: capacity the project's rows
 * here).  FZ_PIECE_RQ2: RQ2-count's trend values (coverage NOT NULL AND != 0 AND date < LIMIT, then
 * total != 0; covered / total * 100, NaN for a NULL line count) with counts[0..2] = values, fetched
 * rows, NULL-line rows; FZ_PIECE_RQ4B: rq4b's full series (coverage > 0, date < LIMIT,
 * rq4b_coverage.py:315-326) with counts[0..2] = values, values, 0.  counts: device [3]. */
enum { FZ_PIECE_RQ2 = 0, FZ_PIECE_RQ4B = 1 };
int fz_piece_values(fz_ctx *ctx, int64_t project, int kind, double *out, int64_t *counts);

/* The project-major session exchange's send side: run r = desc[r].len values at (src 0: a, 1: b) +
 * src_off covering sessions [base, base + len); the slice of run r for destination d (sessions
 * [cuts[d], cuts[d + 1]), d < n_dest) is written at out + table[d * (n_runs + 1) + r].  in_off[r]:
 * exclusive prefix of the runs' lengths; n_values their total.  Every pointer device. */
typedef struct fz_run_desc {
    int64_t src_off;
    int64_t len;
    int64_t base;
    int32_t src;
    int32_t pad_;
} fz_run_desc;
int fz_pack_runs(fz_ctx *ctx, const double *a, const double *b, const fz_run_desc *desc, const int64_t *in_off,
                 int64_t n_runs, const int64_t *cuts, int n_dest, const int64_t *table, int64_t n_values, double *out);

/* The receive side: n_runs runs (run k = values[run_offs[k], run_offs[k + 1]) in project order, all
 * starting at the owner's first session; group run_group[k] (0 = G2, 1 = G1) when n_groups == 2,
 * else null) -> out = value i of every run longer than i, runs in order, grouped by segment (session
 * i, group) with out_offs [n_sessions * n_groups + 1] - coverage_by_session_index (:329-333) and
 * rq4b_coverage.py:917-931 over the owner's session range.  n_values = run_offs[n_runs]. */
int fz_transpose_runs(fz_ctx *ctx, const double *values, const int64_t *run_offs, const uint8_t *run_group,
                      int64_t n_runs, int n_groups, int64_t n_sessions, int64_t n_values, double *out,
                      int64_t *out_offs);

/* spearmanr(range(n), x) and shapiro(x) (rq2_coverage_count.py:305-322) of one n-value series whose
 * values are sorted in buckets over ranks (ties never cross a bucket): this rank's bucket holds m
 * values sorted ascending at global sorted positions [g0, g0 + m), gidx[j] the series index of value
 * j.  Three passes; after each, every rank combines the buckets' partials in bucket order:
 *   fz_series_dist_partials(pass, ...) -> part [FZ_DIST_PART_WIDTH(pass)] (device)
 *   fz_series_dist_combine(pass, parts [k * width], k, n, params, result)
 * params: device [FZ_DIST_PARAMS] state between passes; result: device [4] = rho, p (after pass 0),
 * W, p (after pass 2) - scipy's values as fz_series_tests gives them.  x0_src: device pointer to
 * series value n / 2 (scipy's y -= x[N // 2]) on the rank that holds it, else null. */
#define FZ_DIST_PARAMS 10
#define FZ_DIST_PART_WIDTH(pass) ((pass) == 0 ? 14 : ((pass) == 1 ? 4 : 6))
int fz_series_dist_partials(fz_ctx *ctx, int pass, const double *sorted, const int64_t *gidx, int64_t m, int64_t g0,
                            int64_t n, const double *params, const double *x0_src, double *part);
int fz_series_dist_combine(fz_ctx *ctx, int pass, const double *parts, int64_t k, int64_t n, double *params,
                           double *result);

/* ---- build-log analysis ------------------------------------------
 * Replaces buildlog_analysis(row) of program/preparation/4_get_buildlog_analysis.py:14-246 for a
 * batch of logs already downloaded: text = the UTF-8 bytes of every log back to back (device),
 * log_offs[n_logs + 1] its byte offsets (host AND device copies: the host one cuts the work list).
 * Lines are str.splitlines() lines.  Per log: build_type / result (FZ_BT_* / FZ_BR_*), the project
 * name as a byte span of text, log_line0 (index of its first line) and a status: 0 analysed,
 * 1 empty text (the reference returns its defaults, :54-55), 2 one line (the reference raises
 * IndexError at lines[-2], :230).  The lines the srcmap extraction needs (:162-214) - flags
 * FZ_BL_SKIP / JQ / OPEN / CLOSE - are listed in ev_* (unordered; *n_events may exceed event_cap:
 * then call again with room for that many). */
enum { FZ_BT_NONE = 0, FZ_BT_coverage = 1, FZ_BT_introspector = 2, FZ_BT_FUZZING = 3, FZ_BT_UNKNOWN = 4,
       FZ_BT_INTROSPECTOR = 5, FZ_BT_COVERAGE = 6 };
enum { FZ_BR_NONE = 0, FZ_BR_ERROR = 1, FZ_BR_SUCCESS = 2, FZ_BR_UNKNOWN = 3 };
enum { FZ_BL_SKIP = 1 << 2, FZ_BL_JQ = 1 << 8, FZ_BL_OPEN = 1 << 9, FZ_BL_CLOSE = 1 << 10 };
typedef struct fz_buildlog_out {
    int32_t *log_type;      /* [n_logs] device */
    int32_t *log_result;    /* [n_logs] */
    int32_t *log_status;    /* [n_logs] */
    int64_t *log_proj_off;  /* [n_logs] byte offset in text of the project name (-1: none) */
    int32_t *log_proj_len;  /* [n_logs] */
    int64_t *log_line0;     /* [n_logs] first line index of the log */
    int64_t *n_lines;       /* [1] total lines */
    int64_t *ev_line;       /* [event_cap] line index */
    int64_t *ev_start;      /* [event_cap] byte offset of the line */
    int32_t *ev_len;        /* [event_cap] bytes of the line (without its break) */
    uint32_t *ev_flags;     /* [event_cap] FZ_BL_* */
    int64_t event_cap;
    int64_t *n_events;      /* [1] */
} fz_buildlog_out;
int fz_buildlog(fz_ctx *ctx, const uint8_t *text, int64_t n_bytes, const int64_t *log_offs_host,
                const int64_t *log_offs, int64_t n_logs, const fz_buildlog_out *out);

/* ---- per-kernel probe (bench.py roofline) ------------------------------------------------ */
/* Start timing every launch of the named kernels (one name, or several separated by commas, e.g.
 * "radix_scatter,elig_hist") with HIP events on the context stream; fz_probe_end synchronises the
 * stream and returns the FIRST name's number of launches, summed device milliseconds and summed
 * algorithmic bytes; fz_probe_get returns the same for any probed name until the next begin. */
int fz_probe_begin(fz_ctx *ctx, const char *kernel_names);
int fz_probe_end(fz_ctx *ctx, int64_t *launches, double *total_ms, double *algo_bytes);
int fz_probe_get(fz_ctx *ctx, const char *kernel_name, int64_t *launches, double *total_ms, double *algo_bytes);

/* ---- HIP graphs: record a context's analyses once, replay them per store build ------------- */
/* A repeated analysis over a store rebuilt in place (same table sizes: same buffers) is a fixed
 * sequence of launches; recording it as a HIP graph removes the per-launch host work and most of
 * the inter-kernel gaps (config 2 is launch-latency bound: ~380 launches per step).  Between
 * fz_capture_begin and fz_capture_end every call on ctx is recorded, not run (no host sync may
 * occur: not fz_store_build, not fz_probe_*).  The context must be warm - the same calls made once
 * before, so that no scratch buffer grows while recording.  The graph starts by resetting the
 * context's look-back / radix state, so every replay is self-contained; fz_graph_launch enqueues
 * one replay on ctx's current stream (a context on the null stream records on a private stream).
 * Results are identical to the direct calls'. */
typedef struct fz_graph fz_graph;
int fz_capture_begin(fz_ctx *ctx);
int fz_capture_end(fz_ctx *ctx, fz_graph **out);
int fz_graph_launch(fz_ctx *ctx, fz_graph *graph);
int fz_graph_destroy(fz_graph *graph);

/* ---- primitives (exported for kernel-level tests and the roofline bench) ----------------- */
/* Stable LSD radix sort of (key, value) pairs over key bits [0, bits).  keys/vals in place. */
int fz_radix_sort_u64(fz_ctx *ctx, uint64_t *keys, uint32_t *vals, int64_t n, int bits);
/* numpy-compatible describe of a device fp64 vector (sorts a scratch copy). */
int fz_describe_f64(fz_ctx *ctx, const double *x, int64_t n, fz_describe *host_out);
/* The same into a device fz_describe (no host read: the sharded drivers copy it with their other
 * results). */
int fz_describe_f64_dev(fz_ctx *ctx, const double *x, int64_t n, fz_describe *dev_out);
/* Stable sort of a device fp64 vector by (value, position): val = the values ascending (NaN
 * last), pos = their positions - the single-segment sort RQ3's statistics run over the detected u
 * non-detected union (rq3:321-352; scipy / numpy sort the samples themselves).  val / pos device
 * arrays of n. */
int fz_sort_f64(fz_ctx *ctx, const double *x, int64_t n, double *val, int32_t *pos);
/* Per-project count of total_coverage rows with coverage valid, > 0 and date < limit
 * (the GROUP BY/HAVING of rq1_detection_rate.py:144-152), on the unsorted table. */
int fz_eligibility_count(fz_ctx *ctx, const fz_tables *t, int64_t date_limit, int32_t *counts);

#ifdef __cplusplus
}
#endif
#endif /* FZ_H */
