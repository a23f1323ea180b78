// Public C ABI (include/fz.h): error capture, context lifetime, and thin wrappers that reset the
// scratch arena and forward to the implementation.
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "fz_internal.h"
#include "fz_lookback.h"
#include "fz_seg.h"
#include "fz_views.h"

namespace fz {
void store_build(fz_ctx *c, const fz_tables *t, fz_store_stats *stats);
void rq1(fz_ctx *c, int64_t threshold, const fz_rq1_ext *ext, const fz_rq1_out *o);
void rq1_finish(fz_ctx *c, int64_t threshold, const int64_t *iter_total, const int64_t *iter_det, int64_t M,
                int64_t *counts, fz_describe *late);
void eligibility_counts(fz_ctx *c, const fz_tables *t, int64_t limit, int32_t *counts);
void rq2_count(fz_ctx *c, uint32_t flags, const fz_rq2_count_out *o);
void rq2_session_stats(fz_ctx *c, const double *values, const int64_t *session_ids, int64_t n, int64_t S,
                       int64_t max_len, double *average, double *median, double *pcts, int64_t *n_ge100);
void rq2_session_stats_grouped(fz_ctx *c, const double *values, const int64_t *offs, int64_t n, int64_t S,
                               int64_t max_len, double *average, double *median, double *pcts, int64_t *n_ge100);
void series_tests(fz_ctx *c, const double *x, int64_t n_cap, const int64_t *d_n, double *out);
void runs_merge(fz_ctx *c, const double *values, const int64_t *sizes, int64_t R, int64_t S, double *out,
                int64_t *out_offs);
void spearman_index_seg(fz_ctx *c, const double *x, int64_t n, const int64_t *offs, int64_t S, int64_t max_len,
                        double *rho, double *p);
void rq2_add(fz_ctx *c, const fz_rq2_add_out *o);
void rq3(fz_ctx *c, uint32_t flags, const fz_rq3_out *o);
void rq3_stats(fz_ctx *c, const double *det_pct, const int64_t *det_tot, int64_t NI, const int64_t *d_nd,
               const double *non_pct, int64_t NC, const int64_t *d_nn, fz_describe *describe, double *tests);
void rq4a(fz_ctx *c, const fz_rq4_groups *g, const fz_rq4a_out *o);
void rq4a_finish(fz_ctx *c, int64_t M, int64_t P, const int64_t *g1t, const int64_t *g1d, const int64_t *g2t,
                 const int64_t *g2d, const int64_t *intro, const int64_t *steps, int64_t *counts, double *sc);
void rq4b(fz_ctx *c, const fz_rq4_groups *g, uint32_t flags, const fz_rq4b_out *o);
void rq4b_session_stats(fz_ctx *c, const double *values, const int64_t *sid, const uint8_t *grp, int64_t n, int64_t S,
                        int64_t max_len, int64_t *c2, int64_t *c1, double *g2q, double *g1q, double *pbm);
void rq4b_session_stats_grouped(fz_ctx *c, const double *values, const int64_t *offs2, int64_t n, int64_t S,
                                int64_t max_len, int64_t *c2, int64_t *c1, double *g2q, double *g1q, double *pbm);
void rq4b_trends(fz_ctx *c, const int64_t *c2, const int64_t *c1, const double *g2q, const double *g1q, int64_t MM,
                 int64_t *last, double *sp);
void two_sample_tests(fz_ctx *c, const double *a, int64_t na_cap, const int64_t *n2, const double *b,
                      int64_t nb_cap, const int64_t *n1, double *ts);
void rq2_count_tail(fz_ctx *c, const double *median_trend, int64_t k, const double *corr, const int64_t *raw_n,
                    const int64_t *eligible, int64_t P, double *out);
void rq4b_tail(fz_ctx *c, const int64_t *c2, const int64_t *c1, const double *g2q, const double *g1q, int64_t M,
               const int64_t *order, const double *pre, const double *post, int64_t nd, int64_t n_order,
               const double *x, int64_t nx, const double *y, int64_t ny, int64_t *last, double *sp, double *pre_out,
               double *post_out, double *med14, double *tests);
void store_elig_counts(fz_ctx *c, const int32_t *proj, int64_t n, int64_t *out);
void store_set_eligible(fz_ctx *c, const int32_t *proj, const uint8_t *flag, int64_t n);
void piece_values(fz_ctx *c, int64_t project, int kind, double *out, int64_t *counts);
void pack_runs(fz_ctx *c, const double *a, const double *b, const fz_run_desc *runs, const int64_t *in_off, int64_t R,
               const int64_t *cuts, int W, const int64_t *table, int64_t n, double *out);
void transpose_runs(fz_ctx *c, const double *vals, const int64_t *offs, const uint8_t *grp, int64_t R, int G,
                    int64_t M, int64_t n, double *out, int64_t *out_offs);
void series_dist_partials(fz_ctx *c, int pass, const double *sorted, const int64_t *gidx, int64_t m, int64_t g0,
                          int64_t n, const double *params, const double *x0_src, double *part);
void series_dist_combine(fz_ctx *c, int pass, const double *part, int64_t k, int64_t n, double *params,
                         double *result);
void buildlog(fz_ctx *c, const uint8_t *text, int64_t n_bytes, const int64_t *log_offs_host, const int64_t *log_offs,
              int64_t n_logs, const fz_buildlog_out *o);
}  // namespace fz

struct fz_graph {
    hipGraph_t graph;
    hipGraphExec_t exec;
    // the context's host-side look-back / radix state after one replay
    unsigned int epoch_end;
    int hist_end;
    uint64_t sig;  // ctx_signature() at the end of the recording
};

namespace {
// The device state a recording bakes in: the store it reads (the parent's, for a child) and the
// context's own look-back / radix buffers.  fz_graph_launch refuses a replay after any of them was
// reallocated or the store was rebuilt over other tables (the graph would use freed memory or
// stale sizes).
uint64_t ctx_signature(fz_ctx *c) {
    uint64_t h = fz::store_of(c).signature();
    for (const fz::DevBuf *d : {&c->os_status, &c->os_ticket, &c->os_hist, &c->seg_tickets})
        h = (h ^ (reinterpret_cast<uintptr_t>(d->ptr) + 0x9e3779b97f4a7c15ull * d->gen)) * 1099511628211ull;
    return h;
}
}  // namespace

namespace {
thread_local std::string g_err;

template <typename F>
int guarded(fz_ctx *c, F &&f) {
    struct InCall {  // the context's in-call flag for the duration of the call
        fz_ctx *c;
        explicit InCall(fz_ctx *x) : c(x) { if (c) c->in_call.fetch_add(1); }
        ~InCall() { if (c) c->in_call.fetch_sub(1); }
    };
    try {
        if (!c) throw fz::Error(FZ_E_INVALID, "null fz_ctx");
        InCall ic(c);
        FZ_HIP(hipSetDevice(c->device));
        c->arena.reset();
        f();
        return FZ_OK;
    } catch (const fz::Error &e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        g_err = "host allocation failed";
        return FZ_E_NOMEM;
    } catch (const std::exception &e) {
        g_err = e.what();
        return FZ_E_INVALID;
    }
}
}  // namespace

extern "C" {

int fz_abi_version(void) { return FZ_ABI_VERSION; }

const char *fz_last_error(void) { return g_err.c_str(); }

int fz_ctx_create(int device, void *stream, fz_ctx **out) {
    try {
        if (!out) throw fz::Error(FZ_E_INVALID, "fz_ctx_create: out is null");
        *out = nullptr;
        int n = 0;
        FZ_HIP(hipGetDeviceCount(&n));
        if (device < 0 || device >= n) throw fz::Error(FZ_E_INVALID, "fz_ctx_create: no such device");
        FZ_HIP(hipSetDevice(device));
        fz_ctx *c = new fz_ctx();
        c->device = device;
        c->stream = static_cast<hipStream_t>(stream);
        void *h = nullptr;
        if (hipHostMalloc(&h, 32768, hipHostMallocDefault) != hipSuccess) {
            delete c;
            throw fz::Error(FZ_E_DEVICE, "fz_ctx_create: hipHostMalloc failed");
        }
        c->h_pinned = static_cast<int64_t *>(h);
        void *dh = nullptr;
        FZ_HIP(hipHostGetDevicePointer(&dh, h, 0));
        c->d_pinned = static_cast<int64_t *>(dh);
        *out = c;
        return FZ_OK;
    } catch (const fz::Error &e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception &e) {
        g_err = e.what();
        return FZ_E_INVALID;
    }
}

int fz_ctx_create_child(fz_ctx *parent, void *stream, fz_ctx **out) {
    try {
        if (!out || !parent) throw fz::Error(FZ_E_INVALID, "fz_ctx_create_child: null argument");
        *out = nullptr;
        FZ_HIP(hipSetDevice(parent->device));
        fz_ctx *c = new fz_ctx();
        c->device = parent->device;
        c->stream = static_cast<hipStream_t>(stream);
        c->parent = parent->parent ? parent->parent : parent;
        void *h = nullptr;
        if (hipHostMalloc(&h, 32768, hipHostMallocDefault) != hipSuccess) {
            delete c;
            throw fz::Error(FZ_E_DEVICE, "fz_ctx_create_child: hipHostMalloc failed");
        }
        c->h_pinned = static_cast<int64_t *>(h);
        void *dh = nullptr;
        FZ_HIP(hipHostGetDevicePointer(&dh, h, 0));
        c->d_pinned = static_cast<int64_t *>(dh);
        *out = c;
        return FZ_OK;
    } catch (const fz::Error &e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception &e) {
        g_err = e.what();
        return FZ_E_INVALID;
    }
}

int fz_ctx_destroy(fz_ctx *ctx) {
    if (!ctx) return FZ_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->parent) {  // a destroyed child is no longer a store-build helper of its parent
        auto &h = ctx->parent->helpers;
        for (size_t i = 0; i < h.size();)
            if (h[i] == ctx) h.erase(h.begin() + long(i));
            else ++i;
    }
    if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
    if (ctx->capture_stream) (void)hipStreamDestroy(ctx->capture_stream);
    if (ctx->ev_readback) (void)hipEventDestroy(ctx->ev_readback);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    for (hipEvent_t e : ctx->ev_join)
        if (e) (void)hipEventDestroy(e);
    delete ctx;
    return FZ_OK;
}

int fz_ctx_set_stream(fz_ctx *ctx, void *stream) {
    return guarded(ctx, [&] { ctx->stream = static_cast<hipStream_t>(stream); });
}

int fz_store_set_helpers(fz_ctx *ctx, fz_ctx *const *helpers, int n) {
    return guarded(ctx, [&] {
        FZ_CHECK(n >= 0 && n <= 4 && (n == 0 || helpers != nullptr), "fz_store_set_helpers: 0..4 helpers");
        FZ_CHECK(ctx->parent == nullptr, "fz_store_set_helpers: the store's own context only");
        std::vector<fz_ctx *> h;
        for (int i = 0; i < n; ++i) {
            FZ_CHECK(helpers[i] != nullptr && helpers[i]->parent == ctx && helpers[i] != ctx,
                     "fz_store_set_helpers: helpers must be children of this context");
            h.push_back(helpers[i]);
        }
        ctx->helpers = h;
    });
}

int fz_store_build(fz_ctx *ctx, const fz_tables *t, fz_store_stats *stats) {
    return guarded(ctx, [&] { fz::store_build(ctx, t, stats); });
}

int fz_rq1(fz_ctx *ctx, int64_t min_project_threshold, const fz_rq1_out *out) {
    return guarded(ctx, [&] { fz::rq1(ctx, min_project_threshold, nullptr, out); });
}

int fz_rq1_ex(fz_ctx *ctx, int64_t min_project_threshold, const fz_rq1_ext *ext, const fz_rq1_out *out) {
    return guarded(ctx, [&] { fz::rq1(ctx, min_project_threshold, ext, out); });
}

int fz_rq1_finish(fz_ctx *ctx, int64_t min_project_threshold, const int64_t *iter_total,
                  const int64_t *iter_detected, int64_t max_iter, int64_t *counts, fz_describe *late) {
    return guarded(ctx, [&] {
        FZ_CHECK(counts && late && max_iter >= 0 && (max_iter == 0 || (iter_total && iter_detected)),
                 "fz_rq1_finish: bad arguments");
        fz::rq1_finish(ctx, min_project_threshold, iter_total, iter_detected, max_iter, counts, late);
    });
}

int fz_rq2_count(fz_ctx *ctx, const fz_rq2_count_out *out) {
    return guarded(ctx, [&] { fz::rq2_count(ctx, 0u, out); });
}

int fz_rq2_count_ex(fz_ctx *ctx, uint32_t flags, const fz_rq2_count_out *out) {
    return guarded(ctx, [&] { fz::rq2_count(ctx, flags, out); });
}

int fz_rq2_session_stats(fz_ctx *ctx, const double *values, const int64_t *session_ids, int64_t n_values,
                         int64_t n_sessions, int64_t max_session_len, double *average, double *median,
                         double *percentiles, int64_t *n_ge100) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_values >= 0 && n_sessions >= 0 && (n_values == 0 || (values && session_ids)) && n_ge100 &&
                     (n_sessions == 0 || (average && median && percentiles)) && n_sessions < (int64_t(1) << 31),
                 "fz_rq2_session_stats: bad arguments");
        fz::rq2_session_stats(ctx, values, session_ids, n_values, n_sessions, max_session_len, average, median,
                              percentiles, n_ge100);
    });
}

int fz_rq2_session_stats_grouped(fz_ctx *ctx, const double *values, const int64_t *session_offsets, int64_t n_values,
                                 int64_t n_sessions, int64_t max_session_len, double *average, double *median,
                                 double *percentiles, int64_t *n_ge100) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_values >= 0 && n_sessions >= 0 && (n_values == 0 || values) && n_ge100 && session_offsets &&
                     (n_sessions == 0 || (average && median && percentiles)) && n_sessions < (int64_t(1) << 31),
                 "fz_rq2_session_stats_grouped: bad arguments");
        fz::rq2_session_stats_grouped(ctx, values, session_offsets, n_values, n_sessions, max_session_len, average,
                                      median, percentiles, n_ge100);
    });
}

int fz_runs_merge(fz_ctx *ctx, const double *values, const int64_t *run_sizes, int64_t n_runs, int64_t n_segments,
                  double *out, int64_t *out_offsets) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_runs >= 0 && n_segments >= 0 && out_offsets && (n_runs * n_segments == 0 || (run_sizes && values && out)),
                 "fz_runs_merge: bad arguments");
        fz::runs_merge(ctx, values, run_sizes, n_runs, n_segments, out, out_offsets);
    });
}

int fz_series_tests(fz_ctx *ctx, const double *x, int64_t n, double *out) {
    return guarded(ctx, [&] {
        FZ_CHECK(out && n >= 0 && (n == 0 || x), "fz_series_tests: bad arguments");
        int64_t *d_n = ctx->arena.get<int64_t>(1);
        fz::set_i64(ctx, d_n, &n, 1);
        fz::series_tests(ctx, x, n > 0 ? n : 1, d_n, out);
    });
}

int fz_spearman_index_seg(fz_ctx *ctx, const double *x, int64_t n, const int64_t *offs, int64_t S, int64_t max_len,
                          double *rho, double *p) {
    return guarded(ctx, [&] {
        FZ_CHECK(S >= 0 && n >= 0 && (S == 0 || (offs && rho && p)) && (n == 0 || x),
                 "fz_spearman_index_seg: bad arguments");
        if (S > 0) fz::spearman_index_seg(ctx, x, n, offs, S, max_len, rho, p);
    });
}

int fz_rq2_add(fz_ctx *ctx, const fz_rq2_add_out *out) {
    return guarded(ctx, [&] { fz::rq2_add(ctx, out); });
}

int fz_rq3(fz_ctx *ctx, const fz_rq3_out *out) {
    return guarded(ctx, [&] { fz::rq3(ctx, 0u, out); });
}

int fz_rq3_ex(fz_ctx *ctx, uint32_t flags, const fz_rq3_out *out) {
    return guarded(ctx, [&] { fz::rq3(ctx, flags, out); });
}

int fz_rq3_stats(fz_ctx *ctx, const double *det_pct, const int64_t *det_tot, int64_t n_det, const double *non_pct,
                 int64_t n_non, fz_describe *describe, double *tests) {
    return guarded(ctx, [&] {
        FZ_CHECK(describe && tests && n_det >= 0 && n_non >= 0 && (n_det == 0 || (det_pct && det_tot)) &&
                     (n_non == 0 || non_pct),
                 "fz_rq3_stats: bad arguments");
        int64_t *d_n = ctx->arena.get<int64_t>(2);
        const int64_t h[2] = {n_det, n_non};
        fz::set_i64(ctx, d_n, h, 2);
        fz::rq3_stats(ctx, det_pct, det_tot, n_det, d_n, non_pct, n_non, d_n + 1, describe, tests);
    });
}

int fz_rq3_stats_dn(fz_ctx *ctx, const double *det_pct, const int64_t *det_tot, int64_t det_cap, const int64_t *d_det,
                    const double *non_pct, int64_t non_cap, const int64_t *d_non, fz_describe *describe,
                    double *tests) {
    return guarded(ctx, [&] {
        FZ_CHECK(describe && tests && d_det && d_non && det_cap >= 0 && non_cap >= 0 &&
                     (det_cap == 0 || (det_pct && det_tot)) && (non_cap == 0 || non_pct),
                 "fz_rq3_stats_dn: bad arguments");
        fz::rq3_stats(ctx, det_pct, det_tot, det_cap, d_det, non_pct, non_cap, d_non, describe, tests);
    });
}

int fz_rq4a(fz_ctx *ctx, const fz_rq4_groups *groups, const fz_rq4a_out *out) {
    return guarded(ctx, [&] { fz::rq4a(ctx, groups, out); });
}

int fz_rq4a_finish(fz_ctx *ctx, const int64_t *g1_total, const int64_t *g1_det, const int64_t *g2_total,
                   const int64_t *g2_det, int64_t max_iter, const int64_t *intro, int64_t n_projects,
                   const int64_t *g4_steps, int64_t *counts, double *scalars) {
    return guarded(ctx, [&] {
        FZ_CHECK(max_iter >= 0 && n_projects >= 0 && counts && scalars && g4_steps &&
                     (max_iter == 0 || (g1_total && g1_det && g2_total && g2_det)) && (n_projects == 0 || intro),
                 "fz_rq4a_finish: bad arguments");
        fz::rq4a_finish(ctx, max_iter, n_projects, g1_total, g1_det, g2_total, g2_det, intro, g4_steps, counts,
                        scalars);
    });
}

int fz_rq4b(fz_ctx *ctx, const fz_rq4_groups *groups, const fz_rq4b_out *out) {
    return guarded(ctx, [&] { fz::rq4b(ctx, groups, 0u, out); });
}

int fz_rq4b_ex(fz_ctx *ctx, const fz_rq4_groups *groups, uint32_t flags, const fz_rq4b_out *out) {
    return guarded(ctx, [&] { fz::rq4b(ctx, groups, flags, out); });
}

int fz_rq4b_session_stats(fz_ctx *ctx, const double *values, const int64_t *session_ids, const uint8_t *groups,
                          int64_t n_values, int64_t n_sessions, int64_t max_session_len, int64_t *c2, int64_t *c1,
                          double *g2_q, double *g1_q, double *p_bm) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_values >= 0 && n_sessions >= 0 && n_sessions < (int64_t(1) << 30) &&
                     (n_values == 0 || (values && session_ids && groups)) &&
                     (n_sessions == 0 || (c2 && c1 && g2_q && g1_q && p_bm)),
                 "fz_rq4b_session_stats: bad arguments");
        if (n_sessions == 0) return;
        fz::rq4b_session_stats(ctx, values, session_ids, groups, n_values, n_sessions, max_session_len, c2, c1, g2_q,
                               g1_q, p_bm);
    });
}

int fz_rq4b_session_stats_grouped(fz_ctx *ctx, const double *values, const int64_t *segment_offsets,
                                  int64_t n_values, int64_t n_sessions, int64_t max_session_len, int64_t *c2,
                                  int64_t *c1, double *g2_q, double *g1_q, double *p_bm) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_values >= 0 && n_sessions >= 0 && n_sessions < (int64_t(1) << 30) && (n_values == 0 || values) &&
                     (n_sessions == 0 || (segment_offsets && c2 && c1 && g2_q && g1_q && p_bm)),
                 "fz_rq4b_session_stats_grouped: bad arguments");
        if (n_sessions == 0) return;
        fz::rq4b_session_stats_grouped(ctx, values, segment_offsets, n_values, n_sessions, max_session_len, c2, c1,
                                       g2_q, g1_q, p_bm);
    });
}

int fz_two_sample_tests(fz_ctx *ctx, const double *x, int64_t nx, const double *y, int64_t ny, double *out) {
    return guarded(ctx, [&] {
        FZ_CHECK(out && nx >= 0 && ny >= 0 && (nx == 0 || x) && (ny == 0 || y), "fz_two_sample_tests: bad arguments");
        int64_t *d_n = ctx->arena.get<int64_t>(2);
        const int64_t h[2] = {nx, ny};
        fz::set_i64(ctx, d_n, h, 2);
        fz::two_sample_tests(ctx, x, nx, d_n, y, ny, d_n + 1, out);
    });
}

int fz_buildlog(fz_ctx *ctx, const uint8_t *text, int64_t n_bytes, const int64_t *log_offs_host,
                const int64_t *log_offs, int64_t n_logs, const fz_buildlog_out *out) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_logs == 0 || (log_offs_host && log_offs && (n_bytes == 0 || text)), "fz_buildlog: bad arguments");
        fz::buildlog(ctx, text, n_bytes, log_offs_host, log_offs, n_logs, out);
    });
}

int fz_probe_begin(fz_ctx *ctx, const char *kernel_names) {
    return guarded(ctx, [&] {
        FZ_CHECK(kernel_names != nullptr, "fz_probe_begin: null name");
        fz::Probe &p = ctx->probe;
        p.names.clear();
        std::string all(kernel_names), cur;
        for (size_t i = 0; i <= all.size(); ++i) {
            if (i == all.size() || all[i] == ',') {
                if (!cur.empty() && p.index(cur.c_str()) < 0) p.names.push_back(cur);
                cur.clear();
            } else {
                cur += all[i];
            }
        }
        FZ_CHECK(!p.names.empty(), "fz_probe_begin: no kernel name");
        p.used = 0;
        p.owner.clear();
        p.deferred.clear();
        p.counts.ensure<int64_t>(fz::Probe::kMaxCounts);
        p.launches.assign(p.names.size(), 0);
        p.bytes.assign(p.names.size(), 0.0);
        p.ms.assign(p.names.size(), 0.0);
    });
}

int fz_probe_end(fz_ctx *ctx, int64_t *launches, double *total_ms, double *algo_bytes) {
    return guarded(ctx, [&] {
        fz::Probe &p = ctx->probe;
        fz::sync(ctx);
        for (size_t i = 0; i + 1 < p.used; i += 2) {
            float e = 0.f;
            FZ_HIP(hipEventElapsedTime(&e, p.pool[i], p.pool[i + 1]));
            p.ms[size_t(p.owner[i / 2])] += e;
        }
        if (!p.deferred.empty()) {
            std::vector<int64_t> cnt(p.deferred.size());
            FZ_HIP(hipMemcpy(cnt.data(), p.counts.as<int64_t>(), cnt.size() * 8, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < cnt.size(); ++i)
                p.bytes[size_t(p.deferred[i].owner)] += double(cnt[i]) * p.deferred[i].per_count;
            p.deferred.clear();
        }
        if (launches) *launches = p.launches.empty() ? 0 : p.launches[0];
        if (total_ms) *total_ms = p.ms.empty() ? 0.0 : p.ms[0];
        if (algo_bytes) *algo_bytes = p.bytes.empty() ? 0.0 : p.bytes[0];
        p.results = p.names;  // fz_probe_get reads them until the next fz_probe_begin
        p.names.clear();
        p.used = 0;
        p.owner.clear();
    });
}

int fz_probe_get(fz_ctx *ctx, const char *kernel_name, int64_t *launches, double *total_ms, double *algo_bytes) {
    return guarded(ctx, [&] {
        fz::Probe &p = ctx->probe;
        FZ_CHECK(kernel_name != nullptr && !p.active(), "fz_probe_get: call after fz_probe_end");
        int k = -1;
        for (size_t i = 0; i < p.results.size(); ++i)
            if (p.results[i] == kernel_name) k = int(i);
        FZ_CHECK(k >= 0, std::string("fz_probe_get: kernel not probed: ") + kernel_name);
        if (launches) *launches = p.launches[size_t(k)];
        if (total_ms) *total_ms = p.ms[size_t(k)];
        if (algo_bytes) *algo_bytes = p.bytes[size_t(k)];
    });
}

int fz_capture_begin(fz_ctx *ctx) {
    return guarded(ctx, [&] {
        FZ_CHECK(!ctx->probe.active(), "fz_capture_begin: a probe window is open");
        FZ_CHECK(!ctx->capturing, "fz_capture_begin: already recording");
        // the null stream cannot be recorded: record on a private stream instead (the graph is not
        // tied to the stream it was recorded on; fz_graph_launch replays it on ctx's own stream)
        ctx->capture_saved = ctx->stream;
        if (ctx->stream == nullptr) {
            if (!ctx->capture_stream) FZ_HIP(hipStreamCreateWithFlags(&ctx->capture_stream, hipStreamNonBlocking));
            ctx->stream = ctx->capture_stream;
        }
        const hipError_t e = hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal);
        if (e != hipSuccess) ctx->stream = ctx->capture_saved;
        FZ_HIP(e);
        ctx->capturing = true;
        // every replay starts from the same device state: a zero tile ticket (the recorded launches
        // carry ticket bases from 0), status words with no epoch of this graph, and radix digit
        // totals zeroed by the first recorded sort
        fz::lookback_reset(ctx);
        ctx->os_hist_cur = -1;
    });
}

int fz_capture_end(fz_ctx *ctx, fz_graph **out) {
    return guarded(ctx, [&] {
        FZ_CHECK(out != nullptr, "fz_capture_end: out is null");
        *out = nullptr;
        FZ_CHECK(ctx->capturing, "fz_capture_end: not recording");
        hipGraph_t g = nullptr;
        const hipError_t ec = hipStreamEndCapture(ctx->stream, &g);
        ctx->stream = ctx->capture_saved;
        ctx->capturing = false;
        FZ_HIP(ec);
        hipGraphExec_t x = nullptr;
        const hipError_t e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
        if (e != hipSuccess) {
            (void)hipGraphDestroy(g);
            FZ_HIP(e);
        }
        // the host-side look-back / radix state a replay leaves behind (fz_graph_launch restores it,
        // so direct calls can follow a replay); nothing ran while recording: reset the live state
        *out = new fz_graph{g, x, ctx->os_epoch, ctx->os_hist_cur, ctx_signature(ctx)};
        fz::lookback_reset(ctx);
        ctx->os_hist_cur = -1;
    });
}

int fz_graph_launch(fz_ctx *ctx, fz_graph *graph) {
    return guarded(ctx, [&] {
        FZ_CHECK(graph != nullptr, "fz_graph_launch: null graph");
        FZ_STATE(graph->sig == ctx_signature(ctx),
                 "fz_graph_launch: the store or a context buffer the recording uses was rebuilt over other "
                 "tables or reallocated since fz_capture_end; record the graph again");
        FZ_HIP(hipGraphLaunch(graph->exec, ctx->stream));
        ctx->os_epoch = graph->epoch_end;
        ctx->os_hist_cur = graph->hist_end;
    });
}

int fz_graph_destroy(fz_graph *graph) {
    if (!graph) return FZ_OK;
    (void)hipGraphExecDestroy(graph->exec);
    (void)hipGraphDestroy(graph->graph);
    delete graph;
    return FZ_OK;
}

int fz_radix_sort_u64(fz_ctx *ctx, uint64_t *keys, uint32_t *vals, int64_t n, int bits) {
    return guarded(ctx, [&] {
        FZ_CHECK((keys != nullptr || n == 0) && n >= 0 && bits >= 0 && bits <= 64, "fz_radix_sort_u64: bad arguments");
        fz::radix_sort_pairs(ctx, keys, vals, n, bits);
    });
}

int fz_sort_f64(fz_ctx *ctx, const double *x, int64_t n, double *val, int32_t *pos) {
    return guarded(ctx, [&] {
        FZ_CHECK(n >= 0 && n < (int64_t(1) << 31) && (n == 0 || (x && val && pos)), "fz_sort_f64: bad arguments");
        if (n == 0) return;
        int64_t *offs = ctx->arena.get<int64_t>(2);
        const int64_t h[2] = {0, n};
        fz::set_i64(ctx, offs, h, 2);
        fz::Segs one;
        one.S = 1;
        one.offs = offs;
        one.n_cap = n;
        const fz::SortedSegs s = fz::seg_sort_f64(ctx, x, one, nullptr);
        fz::dev_copy(ctx, val, s.val, n * int64_t(sizeof(double)));
        fz::dev_copy(ctx, pos, s.pos, n * int64_t(sizeof(int32_t)));
    });
}

int fz_describe_f64_dev(fz_ctx *ctx, const double *x, int64_t n, fz_describe *dev_out) {
    return guarded(ctx, [&] {
        FZ_CHECK(dev_out != nullptr && n >= 0 && (x != nullptr || n == 0), "fz_describe_f64_dev: bad arguments");
        fz::describe_f64(ctx, x, n, dev_out);
    });
}

int fz_rq4b_trends(fz_ctx *ctx, const int64_t *c2, const int64_t *c1, const double *g2_q, const double *g1_q,
                   int64_t n_sessions, int64_t *last, double *spearman6) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_sessions >= 0 && last && spearman6 && (n_sessions == 0 || (c2 && c1 && g2_q && g1_q)),
                 "fz_rq4b_trends: bad arguments");
        if (n_sessions == 0) {
            const int64_t m1 = -1;
            fz::set_i64(ctx, last, &m1, 1);
            return;
        }
        fz::rq4b_trends(ctx, c2, c1, g2_q, g1_q, n_sessions, last, spearman6);
    });
}

int fz_rq2_count_tail(fz_ctx *ctx, const double *median_trend, int64_t k, const double *corr, const int64_t *raw_n,
                      const int64_t *eligible, int64_t n_projects, double *out) {
    return guarded(ctx, [&] {
        FZ_CHECK(out && k >= 0 && n_projects >= 0 && (k == 0 || median_trend) &&
                     (n_projects == 0 || (corr && raw_n && eligible)),
                 "fz_rq2_count_tail: bad arguments");
        fz::rq2_count_tail(ctx, median_trend, k, corr, raw_n, eligible, n_projects, out);
    });
}

int fz_rq4b_tail(fz_ctx *ctx, const int64_t *c2, const int64_t *c1, const double *g2_q, const double *g1_q,
                 int64_t n_sessions, const int64_t *delta_order, const double *pre_cov, const double *post_cov,
                 int64_t n_delta, int64_t n_order, const double *init_g2, int64_t n2, const double *init_g1, int64_t n1,
                 int64_t *last, double *spearman6, double *pre_out, double *post_out, double *medians14,
                 double *tests) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_sessions >= 0 && n_delta >= 0 && n_order >= 0 && n2 >= 0 && n1 >= 0 && last && spearman6 &&
                     medians14 && tests && (n_sessions == 0 || (c2 && c1 && g2_q && g1_q)) &&
                     (n_delta == 0 || (delta_order && pre_cov && post_cov && pre_out && post_out)) &&
                     n_delta <= n_order && (n2 == 0 || init_g2) && (n1 == 0 || init_g1),
                 "fz_rq4b_tail: bad arguments");
        fz::rq4b_tail(ctx, c2, c1, g2_q, g1_q, n_sessions, delta_order, pre_cov, post_cov, n_delta, n_order, init_g2,
                      n2, init_g1, n1, last, spearman6, pre_out, post_out, medians14, tests);
    });
}

int fz_store_elig_counts(fz_ctx *ctx, const int32_t *proj, int64_t n, int64_t *out) {
    return guarded(ctx, [&] {
        FZ_CHECK(n >= 0 && (n == 0 || (proj && out)), "fz_store_elig_counts: bad arguments");
        fz::store_elig_counts(ctx, proj, n, out);
    });
}

int fz_store_set_eligible(fz_ctx *ctx, const int32_t *proj, const uint8_t *flag, int64_t n) {
    return guarded(ctx, [&] {
        FZ_CHECK(n >= 0 && (n == 0 || (proj && flag)), "fz_store_set_eligible: bad arguments");
        fz::store_set_eligible(ctx, proj, flag, n);
    });
}

int fz_piece_values(fz_ctx *ctx, int64_t project, int kind, double *out, int64_t *counts) {
    return guarded(ctx, [&] {
        FZ_CHECK(out && counts, "fz_piece_values: bad arguments");
        fz::piece_values(ctx, project, kind, out, counts);
    });
}

int fz_pack_runs(fz_ctx *ctx, const double *a, const double *b, const fz_run_desc *desc, const int64_t *in_off,
                 int64_t n_runs, const int64_t *cuts, int n_dest, const int64_t *table, int64_t n_values, double *out) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_runs >= 0 && n_dest >= 1 && n_values >= 0 &&
                     (n_values == 0 || (desc && in_off && cuts && table && out && (a || b))),
                 "fz_pack_runs: bad arguments");
        fz::pack_runs(ctx, a, b, desc, in_off, n_runs, cuts, n_dest, table, n_values, out);
    });
}

int fz_transpose_runs(fz_ctx *ctx, const double *values, const int64_t *run_offs, const uint8_t *run_group,
                      int64_t n_runs, int n_groups, int64_t n_sessions, int64_t n_values, double *out,
                      int64_t *out_offs) {
    return guarded(ctx, [&] {
        FZ_CHECK(n_runs >= 0 && n_sessions >= 0 && n_values >= 0 && out_offs && (n_groups == 1 || n_groups == 2) &&
                     (n_runs == 0 || (run_offs && (n_values == 0 || (values && out)) && (n_groups == 1 || run_group))),
                 "fz_transpose_runs: bad arguments");
        fz::transpose_runs(ctx, values, run_offs, run_group, n_runs, n_groups, n_sessions, n_values, out, out_offs);
    });
}

int fz_series_dist_partials(fz_ctx *ctx, int pass, const double *sorted, const int64_t *gidx, int64_t m, int64_t g0,
                            int64_t n, const double *params, const double *x0_src, double *part) {
    return guarded(ctx, [&] {
        FZ_CHECK(part && (m == 0 || (sorted && gidx)) && (pass == 0 || params), "fz_series_dist_partials: bad arguments");
        fz::series_dist_partials(ctx, pass, sorted, gidx, m, g0, n, params, x0_src, part);
    });
}

int fz_series_dist_combine(fz_ctx *ctx, int pass, const double *parts, int64_t k, int64_t n, double *params,
                           double *result) {
    return guarded(ctx, [&] {
        FZ_CHECK(parts != nullptr, "fz_series_dist_combine: bad arguments");
        fz::series_dist_combine(ctx, pass, parts, k, n, params, result);
    });
}

// ---- fz_gather_to_host: many small device arrays -> one host buffer, one launch, one sync
namespace {
constexpr int kGatherPieces = 48;
struct GatherList {
    const unsigned char *src[kGatherPieces];
    int64_t n[kGatherPieces];       // elements
    int64_t stride[kGatherPieces];  // elements
    int64_t dst[kGatherPieces];     // byte offset
    int32_t elem[kGatherPieces];    // bytes: 1, 2, 4 or 8
    int count;
};
// one row of workgroups per piece; 8-byte elements move as words, the others byte by byte
__global__ __launch_bounds__(256) void k_gather_to_host(const GatherList g, unsigned char *__restrict__ out) {
    const int k = blockIdx.y;
    if (k >= g.count) return;
    const unsigned char *src = g.src[k];
    const int64_t n = g.n[k], st = g.stride[k];
    const int e = g.elem[k];
    unsigned char *dst = out + g.dst[k];
    const int64_t step = int64_t(gridDim.x) * blockDim.x;
    if (e == 8) {
        for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += step)
            reinterpret_cast<uint64_t *>(dst)[i] = reinterpret_cast<const uint64_t *>(src)[i * st];
    } else {
        for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n * e; i += step)
            dst[i] = src[(i / e) * st * e + i % e];
    }
}
}  // namespace

int fz_gather_to_host(void *stream, const fz_host_piece *pieces, int n_pieces, void *host_out, int64_t total_bytes) {
    // one pinned staging area per device (mapped: kernels write it through its device address),
    // allocated at parallel.host_many's 4 MiB cap and grown only for a larger caller; the lock makes
    // concurrent callers take turns.  Every use ends with a sync of its own stream and the copy out
    // before the lock is released, so the area is idle whenever a caller holds the lock: growing it
    // needs no device-wide synchronisation (other threads' streams keep running)
    struct Area {
        void *h = nullptr, *d = nullptr;
        size_t cap = 0;
    };
    static std::mutex mu;
    static std::map<int, Area> areas;
    constexpr size_t kAreaMin = size_t(4) << 20;
    try {
        FZ_CHECK(n_pieces >= 0 && total_bytes >= 0 && (n_pieces == 0 || pieces) && (total_bytes == 0 || host_out),
                 "fz_gather_to_host: bad arguments");
        for (int i = 0; i < n_pieces; ++i) {
            const fz_host_piece &p = pieces[i];
            const int e = p.elem_bytes;
            FZ_CHECK((e == 1 || e == 2 || e == 4 || e == 8) && p.n >= 0 && p.stride >= 1 && p.dst_offset >= 0 &&
                         p.dst_offset + p.n * e <= total_bytes && (p.n == 0 || p.src) &&
                         (e != 8 || p.dst_offset % 8 == 0),
                     "fz_gather_to_host: bad piece");
        }
        if (total_bytes == 0) return FZ_OK;
        hipStream_t st = static_cast<hipStream_t>(stream);
        int dev = 0;
        FZ_HIP(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu);
        Area &a = areas[dev];
        if (size_t(total_bytes) > a.cap) {
            if (a.h) {  // (idle: its last user synchronised its stream before releasing the lock)
                FZ_HIP(hipHostFree(a.h));
                a = Area{};
            }
            const size_t want = size_t(total_bytes) <= kAreaMin ? kAreaMin : size_t(total_bytes) * 2;
            FZ_HIP(hipHostMalloc(&a.h, want, hipHostMallocMapped | hipHostMallocPortable));
            FZ_HIP(hipHostGetDevicePointer(&a.d, a.h, 0));
            a.cap = want;
        }
        void *h_area = a.h, *d_area = a.d;
        // a launch that fails part way (FZ_LAUNCH_CHECK throws) may leave earlier gathers writing
        // the area: drain the stream before the lock is released on that path too, so the next
        // caller never frees or reuses an area a kernel still writes
        struct DrainOnThrow {
            hipStream_t st;
            bool armed = true;
            ~DrainOnThrow() {
                if (armed) (void)hipStreamSynchronize(st);
            }
        } drain{st};
        for (int b = 0; b < n_pieces; b += kGatherPieces) {
            GatherList g{};
            int64_t most = 0;
            for (int i = b; i < n_pieces && i < b + kGatherPieces; ++i) {
                const fz_host_piece &p = pieces[i];
                const int k = g.count++;
                g.src[k] = static_cast<const unsigned char *>(p.src);
                g.n[k] = p.n;
                g.stride[k] = p.stride;
                g.dst[k] = p.dst_offset;
                g.elem[k] = p.elem_bytes;
                const int64_t w = p.elem_bytes == 8 ? p.n : p.n * p.elem_bytes;
                most = w > most ? w : most;
            }
            if (most == 0) continue;
            const int64_t gx64 = (most + 255) / 256;
            const dim3 grid(unsigned(gx64 < 64 ? gx64 : 64), unsigned(g.count));
            k_gather_to_host<<<grid, 256, 0, st>>>(g, static_cast<unsigned char *>(d_area));
            FZ_LAUNCH_CHECK();
        }
        drain.armed = false;
        FZ_HIP(hipStreamSynchronize(st));
        std::memcpy(host_out, h_area, size_t(total_bytes));
        return FZ_OK;
    } catch (const fz::Error &e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception &e) {
        g_err = e.what();
        return FZ_E_INVALID;
    }
}

int fz_describe_f64(fz_ctx *ctx, const double *x, int64_t n, fz_describe *host_out) {
    return guarded(ctx, [&] {
        FZ_CHECK(host_out != nullptr && n >= 0 && (x != nullptr || n == 0), "fz_describe_f64: bad arguments");
        fz_describe *d = ctx->arena.get<fz_describe>(1);
        fz::describe_f64(ctx, x, n, d);
        FZ_HIP(hipMemcpyAsync(host_out, d, sizeof(fz_describe), hipMemcpyDeviceToHost, ctx->stream));
        fz::sync(ctx);
    });
}

int fz_eligibility_count(fz_ctx *ctx, const fz_tables *t, int64_t date_limit, int32_t *counts) {
    return guarded(ctx, [&] {
        FZ_CHECK(t != nullptr && counts != nullptr, "fz_eligibility_count: bad arguments");
        fz::eligibility_counts(ctx, t, date_limit, counts);
    });
}

}  // extern "C"
