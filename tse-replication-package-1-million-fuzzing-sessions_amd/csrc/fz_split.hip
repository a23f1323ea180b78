// Project-sharded sessions with a project cut across ranks.
//
// A coverage-only project larger than one rank's share of rows (config 5's Zipf giant: 20.8 M of
// 100 M rows, every one of them read by RQ2-count in the live-row variant) is cut into date ranges
// on consecutive ranks.  The reference reads such a project as ONE series: its trend values
// (queries1.py:120-129, rq2_coverage_count.py:292-303) are value i of session i
// (coverage_by_session_index, :329-333) and go through one shapiro / spearmanr (:305-322).  The
// primitives here keep both exact across the cut:
//
//   * the store's eligibility counts of given projects, and an override of their flags - the
//     GROUP BY ... HAVING COUNT(*) >= 365 of rq1:144-152 counted over every piece;
//   * the filtered values of ONE project's rows on this rank (a piece past the first), as the
//     analyses' own filters produce them;
//   * the project-major session exchange: a rank's runs (a project's values in date order, each
//     starting at its session base) packed into per-owner slices, and the owner's ragged transpose
//     of the runs it receives (fz_transpose.h) - the per-session work sized by the owner's session
//     range, never by the longest project;
//   * Spearman vs index and Shapiro-Wilk of one series whose sorted values are spread over ranks
//     in value buckets (ties never cross a bucket): per-bucket double-double partial sums at their
//     global sorted positions, combined in bucket order - the passes of seg_shapiro and the sums of
//     k_spearman_chunks (fz_series.hip) with the same formulas.
#include "fz_seg.h"
#include "fz_stats.h"
#include "fz_transpose.h"
#include "fz_views.h"

namespace fz {

constexpr int64_t kLimitSplit = 1736294400000000LL;  // '2025-01-08' (queries1.py:3)

// ---- eligibility across pieces ------------------------------------------------------------------
void store_elig_counts(fz_ctx *c, const int32_t *proj, int64_t n, int64_t *out) {
    const Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_store_elig_counts: call fz_store_build first");
    const int64_t P = s.P;
    const int32_t *cnt = s.elig_cnt.as<int32_t>();
    map_n(c, n, nullptr, [=] __device__(int64_t i) {
        const int32_t p = proj[i];
        out[i] = (p >= 0 && p < P && cnt) ? int64_t(cnt[p]) : 0;
    });
}

void store_set_eligible(fz_ctx *c, const int32_t *proj, const uint8_t *flag, int64_t n) {
    FZ_CHECK(c->parent == nullptr, "fz_store_set_eligible: call it on the context that built the store");
    Store &s = c->store;
    FZ_CHECK(s.built, "fz_store_set_eligible: call fz_store_build first");
    const int64_t P = s.P;
    uint8_t *el = s.elig.as<uint8_t>();
    int64_t *ne = s.n_elig.as<int64_t>();
    map_n(c, n, nullptr, [=] __device__(int64_t i) {
        const int32_t p = proj[i];
        if (p < 0 || p >= P) return;
        const uint8_t nw = flag[i] ? 1 : 0;
        if (el[p] != nw) {
            el[p] = nw;
            atomicAdd(reinterpret_cast<unsigned long long *>(ne), nw ? 1ull : ~0ull);  // (+1 / -1)
        }
    });
}

// ---- one project's filtered values -----------------------------------------------------------------
// RQ2 piece counts of rows [offs[p], offs[p + 1]): fetched rows (the query's rows) and NULL-line rows
// among the kept ones, added to counts[1] / counts[2] once per workgroup (per-row atomics on two
// words serialise: 2.6 ms for config 5's 13 M-row piece)
__global__ __launch_bounds__(kBlock) void k_piece_counts(const int64_t *__restrict__ offs, int64_t p,
                                                         const uint8_t *__restrict__ valid,
                                                         const double *__restrict__ cov,
                                                         const int64_t *__restrict__ date,
                                                         const int64_t *__restrict__ total,
                                                         int64_t *__restrict__ counts) {
    __shared__ int64_t s_tmp[4];
    const int64_t a = offs[p], e = offs[p + 1];
    int64_t fetched = 0, nulls = 0;
    for (int64_t r = a + int64_t(blockIdx.x) * kBlock + threadIdx.x; r < e; r += int64_t(gridDim.x) * kBlock) {
        const uint8_t v = valid[r];
        const bool f = bool(v & FZ_VALID_COVERAGE) & (cov[r] != 0.0) & (date[r] < kLimitSplit);
        const bool kept = f & ((total[r] != 0) | !(v & FZ_VALID_TOTAL));
        const bool null = kept & ((v & (FZ_VALID_COVERED | FZ_VALID_TOTAL)) != (FZ_VALID_COVERED | FZ_VALID_TOTAL));
        fetched += f;
        nulls += null;
    }
    fetched = block_sum(fetched, s_tmp);
    nulls = block_sum(nulls, s_tmp);
    if (threadIdx.x == 0 && (fetched | nulls)) {
        atomicAdd(reinterpret_cast<unsigned long long *>(counts + 1), (unsigned long long)fetched);
        atomicAdd(reinterpret_cast<unsigned long long *>(counts + 2), (unsigned long long)nulls);
    }
}

// kind FZ_PIECE_RQ2: GET_TOTAL_COVERAGE_EACH_PROJECT's rows (coverage NOT NULL AND coverage != 0 AND
// DATE(date) < LIMIT, queries1.py:120-129), trend value float(covered) / float(total) * 100 where
// total != 0 (rq2_coverage_count.py:300-303; a NULL line count counted and stored as NaN, as
// TrendEmit).  counts: [values, fetched rows, NULL-line rows].
// kind FZ_PIECE_RQ4B: get_full_coverage_trend's rows (coverage > 0, date < LIMIT, rq4b:315-326),
// value = coverage.  counts: [values, values, 0].
void piece_values(fz_ctx *c, int64_t project, int kind, double *out, int64_t *counts) {
    const Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_piece_values: call fz_store_build first");
    FZ_CHECK(project >= 0 && project < s.P, "fz_piece_values: project out of range");
    FZ_CHECK(kind == FZ_PIECE_RQ2 || kind == FZ_PIECE_RQ4B, "fz_piece_values: unknown kind");
    const fz_tables &t = s.t;
    const int64_t *offs = s.cov.offs;
    const int64_t p = project;
    int64_t *d_len = c->arena.get<int64_t>(1);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        *d_len = offs[p + 1] - offs[p];
        counts[1] = 0;
        counts[2] = 0;
    });
    const int64_t cap = s.cov.max_seg;
    const double *cov = t.c_coverage;
    const int64_t *date = t.c_date, *covered = t.c_covered, *total = t.c_total;
    const uint8_t *valid = t.c_valid;
    if (kind == FZ_PIECE_RQ2) {
        if (cap > 0) {
            const int64_t blocks = std::min<int64_t>((cap + kBlock * 16 - 1) / (kBlock * 16), 2048);
            k_piece_counts<<<unsigned(blocks), kBlock, 0, c->stream>>>(offs, p, valid, cov, date, total, counts);
            FZ_LAUNCH_CHECK();
        }
        compact_emit(c, cap, d_len,
                     [=] __device__(int64_t j) {
                         const int64_t r = offs[p] + j;
                         const uint8_t v = valid[r];
                         return bool(v & FZ_VALID_COVERAGE) & (cov[r] != 0.0) & (date[r] < kLimitSplit) &
                                ((total[r] != 0) | !(v & FZ_VALID_TOTAL));
                     },
                     [=] __device__(int64_t j, int64_t q) {
                         const int64_t r = offs[p] + j;
                         const uint8_t v = valid[r];
                         out[q] = (v & (FZ_VALID_COVERED | FZ_VALID_TOTAL)) != (FZ_VALID_COVERED | FZ_VALID_TOTAL)
                                      ? NAN
                                      : double(covered[r]) / double(total[r]) * 100.0;
                     },
                     counts);
    } else {
        compact_emit(c, cap, d_len,
                     [=] __device__(int64_t j) {
                         const int64_t r = offs[p] + j;
                         return bool(valid[r] & FZ_VALID_COVERAGE) & (cov[r] > 0.0) & (date[r] < kLimitSplit);
                     },
                     [=] __device__(int64_t j, int64_t q) { out[q] = cov[offs[p] + j]; }, counts);
        map_n(c, 1, nullptr, [=] __device__(int64_t) { counts[1] = counts[0]; });
    }
}

// ---- the project-major session exchange ------------------------------------------------------------
// Run r (desc[r]): len values at src (A or B) + src_off, covering sessions [base, base + len).  For
// destination d (sessions [cuts[d], cuts[d + 1])) the run's slice is written at table[d * (R + 1) + r]
// onward.  in_off[r] = exclusive prefix of the runs' lengths (one thread per value: its run by binary
// search over in_off, its destination by the <= 9-entry cut list).
__global__ __launch_bounds__(kBlock) void k_pack_runs(const double *__restrict__ a, const double *__restrict__ b,
                                                      const fz_run_desc *__restrict__ runs,
                                                      const int64_t *__restrict__ in_off, int64_t R,
                                                      const int64_t *__restrict__ cuts, int W,
                                                      const int64_t *__restrict__ table, int64_t n,
                                                      double *__restrict__ out) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        int64_t lo = 0, hi = R - 1;  // last run with in_off <= i
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (in_off[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const fz_run_desc rd = runs[lo];
        const int64_t j = i - in_off[lo];
        const int64_t sess = rd.base + j;
        int d = 0;
        while (d + 1 < W && cuts[d + 1] <= sess) ++d;
        const int64_t first = cuts[d] > rd.base ? cuts[d] : rd.base;
        const double v = rd.src == 0 ? a[rd.src_off + j] : b[rd.src_off + j];
        out[table[int64_t(d) * (R + 1) + lo] + (sess - first)] = v;
    }
}

void pack_runs(fz_ctx *c, const double *a, const double *b, const fz_run_desc *runs, const int64_t *in_off, int64_t R,
               const int64_t *cuts, int W, const int64_t *table, int64_t n, double *out) {
    if (n <= 0 || R <= 0) return;
    // algorithmic bytes: every value read and written once
    ProbeScope ps(c, "pack_runs", 16.0 * double(n));
    k_pack_runs<<<grid_for(n, kBlock, 8192), kBlock, 0, c->stream>>>(a, b, runs, in_off, R, cuts, W, table, n, out);
    FZ_LAUNCH_CHECK();
}

// The owner's transpose: R runs (run k = values [offs[k], offs[k + 1]) in project order, group
// grp[k] when G == 2) -> segment (session i, group) offsets [M * G + 1] and values
void transpose_runs(fz_ctx *c, const double *vals, const int64_t *offs, const uint8_t *grp, int64_t R, int G,
                    int64_t M, int64_t n, double *out, int64_t *out_offs) {
    FZ_CHECK(G == 1 || G == 2, "fz_transpose_runs: one or two groups");
    FZ_CHECK(ragged_transpose_ok(R > 0 ? R : 1, M > 0 ? M : 1, G), "fz_transpose_runs: shape out of range");
    const int64_t MM = M > 0 ? M : 1;
    if (R <= 0) {  // no runs: empty sessions
        map_n(c, MM * G + 1, nullptr, [=] __device__(int64_t i) { out_offs[i] = 0; });
        return;
    }
    auto in = [=] __device__(int64_t j) { return vals[j]; };
    if (G == 1)
        ragged_transpose<1>(c, offs, R, MM, n > 0 ? n : 1, in, RtOneGroup{}, out, out_offs);
    else
        ragged_transpose<2>(c, offs, R, MM, n > 0 ? n : 1, in, [=] __device__(int64_t k) { return int(grp[k]); }, out,
                            out_offs);
}

// ---- Spearman vs index / Shapiro-Wilk of one series spread over value buckets ------------------------
// A bucket: m values sorted ascending (ties never cross buckets) at global sorted positions
// [g0, g0 + m) of the n-value series; gidx[j] = the series (time-order) index of value j.
// Pass 0 -> part[14]: sum of m_k^2 (k <= n / 2), the Spearman sums (rx*ry, rx^2, ry^2, tie groups),
// each a double-double (hi, lo); then min, max, x0 (*x0_src when this bucket's rank holds series
// index n / 2, scipy's y -= x[N // 2]) and its flag.
// Pass 1 (params after combine 0) -> part[4]: sum of (y - x0) / range, sum of the signed
// coefficients.  Pass 2 -> part[6]: ssa, ssx, sax (seg_shapiro's pass C).
// params (device, kDistParams doubles): x0, range, a1, a2, fac, i1, sx / n, sa / n, n
constexpr int kDistParams = 10;
static_assert(kDistParams == FZ_DIST_PARAMS, "fz.h FZ_DIST_PARAMS");
constexpr int kDistPart[3] = {14, 4, 6};

void series_dist_partials(fz_ctx *c, int pass, const double *sorted, const int64_t *gidx, int64_t m, int64_t g0,
                          int64_t n, const double *params, const double *x0_src, double *part) {
    FZ_CHECK(pass >= 0 && pass <= 2 && n >= 0 && m >= 0 && g0 >= 0 && g0 + m <= n, "fz_series_dist_partials: bad arguments");
    int64_t *offs = c->arena.get<int64_t>(2);
    const int64_t h[2] = {0, m};
    set_i64(c, offs, h, 2);
    const int W = kDistPart[pass];
    if (m == 0) {  // an empty bucket: zero sums, +-inf extremes
        map_n(c, W, nullptr, [=] __device__(int64_t k) {
            double v = 0.0;
            if (pass == 0 && k == 10) v = INFINITY;
            if (pass == 0 && k == 11) v = -INFINITY;
            if (pass == 0 && k == 12) v = x0_src ? *x0_src : 0.0;
            if (pass == 0 && k == 13) v = x0_src ? 1.0 : 0.0;
            part[k] = v;
        });
        return;
    }
    Segs one{1, offs, m, m};
    ChunkedSegs cs = chunked(c, one);
    const double nn = double(n);
    if (pass == 0) {
        // (sums written as hi/lo pairs by a fold per quantity: seg_reduce returns hi + lo; keep the
        // pair by reducing twice would double the passes - the double-double result rounded to one
        // double is within 1 ulp of the exact sum, which the combine adds in bucket order)
        double *s = c->arena.get<double>(5);
        seg_reduce<1>(c, cs, [=] __device__(int64_t i, int32_t, double *x) {
            const int64_t k = g0 + i + 1;
            double mk = 0.0;
            if (n >= 3 && k <= n / 2) mk = stats::sw_m(k, n);
            x[0] = mk * mk;
        }, s, 0.0);
        int32_t *segid = segment_ids(c, one);
        TieRanks tr = seg_tie_ranks(c, cs, segid, sorted);
        const double mm = (nn + 1.0) / 2.0;
        const double *rank = tr.rank;
        const int64_t *flag = tr.flag;
        seg_reduce<4>(c, cs, [=] __device__(int64_t i, int32_t, double *x) {
            const double rx = double(gidx[i] + 1) - mm;
            const double ry = (double(g0) + rank[i]) - mm;
            x[0] = rx * ry;
            x[1] = rx * rx;
            x[2] = ry * ry;
            x[3] = flag[i] ? 1.0 : 0.0;
        }, s + 1, 12.0);
        map_n(c, 1, nullptr, [=] __device__(int64_t) {
            for (int k = 0; k < 5; ++k) {
                part[2 * k] = s[k];
                part[2 * k + 1] = 0.0;
            }
            part[10] = sorted[0];
            part[11] = sorted[m - 1];
            part[12] = x0_src ? *x0_src : 0.0;
            part[13] = x0_src ? 1.0 : 0.0;
        });
        return;
    }
    auto coef = [=] __device__(const double *pr) {
        stats::SwCoef cf;
        cf.n = n;
        cf.a1 = pr[2];
        cf.a2 = pr[3];
        cf.fac = pr[4];
        cf.i1 = int(pr[5]);
        return cf;
    };
    double *s = c->arena.get<double>(3);
    if (pass == 1) {
        seg_reduce<2>(c, cs, [=] __device__(int64_t i, int32_t, double *x) {
            x[0] = (sorted[i] - params[0]) / params[1];
            x[1] = stats::sw_coef_at(coef(params), g0 + i + 1);
        }, s, 8.0);
        map_n(c, 1, nullptr, [=] __device__(int64_t) {
            part[0] = s[0], part[1] = 0.0, part[2] = s[1], part[3] = 0.0;
        });
        return;
    }
    seg_reduce<3>(c, cs, [=] __device__(int64_t i, int32_t, double *x) {
        const double asa = stats::sw_coef_at(coef(params), g0 + i + 1) - params[7];
        const double xsx = (sorted[i] - params[0]) / params[1] - params[6];
        x[0] = asa * asa;
        x[1] = xsx * xsx;
        x[2] = asa * xsx;
    }, s, 8.0);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        for (int k = 0; k < 3; ++k) {
            part[2 * k] = s[k];
            part[2 * k + 1] = 0.0;
        }
    });
}

// Combine k buckets' partials (part[b * width + ...], bucket order) -> params / result (device):
// pass 0: params (x0, range, Shapiro-Wilk coefficients) and result[0..1] = Spearman rho, p
// (spearman_index_sorted's finishing); pass 1: params' sx / n, sa / n; pass 2: result[2..3] = W, p
// (seg_shapiro's finishing: NaN below 3 values, (1, 1) for a zero range).
__global__ void k_dist_combine(int pass, const double *__restrict__ part, int64_t k, int64_t n,
                               double *__restrict__ params, double *__restrict__ result) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int W = pass == 0 ? 14 : (pass == 1 ? 4 : 6);
    const int nd = pass == 0 ? 5 : (pass == 1 ? 2 : 3);
    DD acc[5] = {};
    for (int64_t b = 0; b < k; ++b)
        for (int q = 0; q < nd; ++q) acc[q] = dd_add(acc[q], DD{part[b * W + 2 * q], part[b * W + 2 * q + 1]});
    double sum[5];
    for (int q = 0; q < nd; ++q) sum[q] = acc[q].hi + acc[q].lo;
    if (pass == 0) {
        double mn = INFINITY, mx = -INFINITY, x0 = 0.0;
        for (int64_t b = 0; b < k; ++b) {
            const double *p = part + b * W;
            mn = p[10] < mn ? p[10] : mn;
            mx = p[11] > mx ? p[11] : mx;
            if (p[13] != 0.0) x0 = p[12];
        }
        params[0] = x0;
        params[1] = (mx - x0) - (mn - x0);
        params[8] = double(n);
        if (n >= 3) {
            const stats::SwCoef cf = stats::sw_coef(n, 2.0 * sum[0]);
            params[2] = cf.a1;
            params[3] = cf.a2;
            params[4] = cf.fac;
            params[5] = double(cf.i1);
        }
        double r = NAN, p = NAN;
        if (n >= 2 && sum[4] > 1.0) {
            const double f = 1.0 / double(n - 1);  // (np.cov: times the reciprocal)
            const double cxy = sum[1] * f, cxx = sum[2] * f, cyy = sum[3] * f;
            r = cxy / sqrt(cxx) / sqrt(cyy);
            if (r > 1.0) r = 1.0;
            if (r < -1.0) r = -1.0;
            const double dof = double(n - 2);
            double q = dof / ((r + 1.0) * (1.0 - r));
            if (q < 0.0) q = 0.0;
            const double t = r * sqrt(q);
            p = 2.0 * t_sf_once(fabs(t), dof);
        }
        result[0] = r;
        result[1] = p;
        return;
    }
    if (pass == 1) {
        params[6] = sum[0] / double(n);
        params[7] = sum[1] / double(n);
        return;
    }
    if (n < 3) {
        result[2] = NAN;
        result[3] = NAN;
        return;
    }
    if (params[1] < stats::kSwSmall) {  // zero range: scipy returns (1.0, 1.0)
        result[2] = 1.0;
        result[3] = 1.0;
        return;
    }
    const double ssa = sum[0], ssx = sum[1], sax = sum[2];
    const double ssassx = sqrt(ssa * ssx);
    const double w1 = (ssassx - sax) * (ssassx + sax) / (ssa * ssx);
    const double ww = 1.0 - w1;
    result[2] = ww;
    result[3] = sw_pvalue_once(n, ww, w1);
}

void series_dist_combine(fz_ctx *c, int pass, const double *part, int64_t k, int64_t n, double *params,
                         double *result) {
    FZ_CHECK(pass >= 0 && pass <= 2 && k >= 1 && n >= 0 && params && result, "fz_series_dist_combine: bad arguments");
    k_dist_combine<<<1, kWave, 0, c->stream>>>(pass, part, k, n, params, result);
    FZ_LAUNCH_CHECK();
}

}  // namespace fz
