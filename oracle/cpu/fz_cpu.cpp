// CPU BASELINE - test infrastructure only (see oracle/__init__.py): a multi-core C++ restatement of
// the six analyses of oracle/rq_oracle.py (itself citing the reference lines it follows) over the
// same host columns fz_store_build takes (include/fz.h: fz_tables, fz_rq4_groups - host pointers
// here).  bench.py's cpu_baseline leg times it with every host core (OpenMP); tests/test_cpu_baseline.py
// checks it against rq_oracle.py.  Never linked into, or called by, the product path.
//
// Layout: one per-project index per table (rows sorted by (project, key, row): the counting scatter
// is stable, then each project's rows sort by (key, row)), filtered views of it per query, and the
// analyses parallel over projects (RQ1-RQ4a) or sessions (RQ2 count / RQ4b), the statistics from
// csrc/fz_stats.h (the same AS R94 / incomplete-beta code the device uses, compiled for the host).
#include <omp.h>
#include <parallel/algorithm>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "fz.h"
#include "fz_stats.h"

namespace {

using std::vector;
namespace st = fz::stats;

constexpr int64_t TS_NULL = INT64_MAX;
constexpr int64_t US_DAY = 86400000000LL;
constexpr int64_t LIMIT_US = 20096 * US_DAY;      // '2025-01-08' (queries1.py:3)
constexpr int64_t RQ3_LIMIT_US = 20097 * US_DAY;  // '2025-01-09' (rq3:262-263)
constexpr uint8_t BT_FUZZING = 0, BT_COVERAGE = 1;
constexpr uint8_t R_FINISH = 0, R_HALFWAY_LOWER = 1, R_HALFWAY_UPPER = 2;
constexpr double NaN = std::numeric_limits<double>::quiet_NaN();

inline bool fixed_status(uint8_t s) { return s == 0 || s == 1; }  // 'Fixed', 'Fixed (Verified)'
inline int64_t day_of(int64_t us) { return us / US_DAY; }         // times are >= 1970

struct Result {
    std::map<std::string, vector<double>> f;
    std::map<std::string, vector<int64_t>> i;
};

// ------------------------------------------------------------------------------ per-project index
struct Index {
    vector<int64_t> off;  // [P + 1]
    vector<int32_t> rows;
};

template <class KeyF>
Index index_by_project(const uint32_t *proj, int64_t n, int64_t P, KeyF key) {
    const int T = omp_get_max_threads();
    vector<int64_t> hist(size_t(T) * P, 0);
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        int64_t *h = &hist[size_t(t) * P];
        for (int64_t i = n * t / T, e = n * (t + 1) / T; i < e; ++i) ++h[proj[i]];
    }
    Index ix;
    ix.off.assign(P + 1, 0);
    int64_t run = 0;
    for (int64_t p = 0; p < P; ++p) {
        ix.off[p] = run;
        for (int t = 0; t < T; ++t) {
            const int64_t c = hist[size_t(t) * P + p];
            hist[size_t(t) * P + p] = run;
            run += c;
        }
    }
    ix.off[P] = run;
    ix.rows.resize(n);
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        int64_t *pos = &hist[size_t(t) * P];
        for (int64_t i = n * t / T, e = n * (t + 1) / T; i < e; ++i) ix.rows[pos[proj[i]]++] = int32_t(i);
    }
    auto less = [&](int32_t a, int32_t b) {
        const int64_t ka = key(a), kb = key(b);
        return ka < kb || (ka == kb && a < b);
    };
    // giant projects (c5's Zipf head) sort with every thread, the rest one project per thread
    const int64_t big = std::max<int64_t>(1 << 16, n / (4 * T));
    vector<int64_t> small;
    for (int64_t p = 0; p < P; ++p) {
        if (ix.off[p + 1] - ix.off[p] > big)
            __gnu_parallel::sort(ix.rows.begin() + ix.off[p], ix.rows.begin() + ix.off[p + 1], less);
        else if (ix.off[p + 1] - ix.off[p] > 1)
            small.push_back(p);
    }
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t k = 0; k < int64_t(small.size()); ++k) {
        const int64_t p = small[k];
        std::sort(ix.rows.begin() + ix.off[p], ix.rows.begin() + ix.off[p + 1], less);
    }
    return ix;
}

// Rows of an index passing `pred`, same order (filter-then-sort == sort-then-filter: the sort is
// stable by row), with their keys.
struct View {
    vector<int64_t> off;
    vector<int32_t> rows;
    vector<int64_t> keys;
    int64_t len(int64_t p) const { return off[p + 1] - off[p]; }
    const int32_t *r(int64_t p) const { return rows.data() + off[p]; }
    const int64_t *k(int64_t p) const { return keys.data() + off[p]; }
};

template <class Pred>
View view_of(const Index &ix, const int64_t *key, Pred pred) {
    const int64_t P = int64_t(ix.off.size()) - 1;
    View v;
    v.off.assign(P + 1, 0);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t p = 0; p < P; ++p) {
        int64_t c = 0;
        for (int64_t j = ix.off[p]; j < ix.off[p + 1]; ++j) c += pred(ix.rows[j]) ? 1 : 0;
        v.off[p + 1] = c;
    }
    for (int64_t p = 0; p < P; ++p) v.off[p + 1] += v.off[p];
    v.rows.resize(v.off[P]);
    v.keys.resize(v.off[P]);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t p = 0; p < P; ++p) {
        int64_t o = v.off[p];
        for (int64_t j = ix.off[p]; j < ix.off[p + 1]; ++j) {
            const int32_t r = ix.rows[j];
            if (pred(r)) {
                v.rows[o] = r;
                v.keys[o++] = key[r];
            }
        }
    }
    return v;
}

inline int64_t lower(const int64_t *k, int64_t n, int64_t x) { return std::lower_bound(k, k + n, x) - k; }
inline int64_t upper(const int64_t *k, int64_t n, int64_t x) { return std::upper_bound(k, k + n, x) - k; }

// ---------------------------------------------------------------------------- numpy / scipy pieces
inline double np_lerp(double a, double b, double t) {  // numpy _lerp
    const double d = b - a;
    return t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
}
inline double pct_sorted(const double *s, int64_t n, double q) {  // np.percentile(linear), n >= 1
    const double vi = double(n - 1) * (q / 100.0);
    const double fl = std::floor(vi);
    int64_t a = int64_t(fl), b = a + 1;
    a = std::min(std::max<int64_t>(a, 0), n - 1);
    b = std::min(std::max<int64_t>(b, 0), n - 1);
    return np_lerp(s[a], s[b], vi - fl);
}
inline double median_sorted(const double *s, int64_t n) {
    return n <= 0 ? NaN : ((n & 1) ? s[n / 2] : (s[n / 2 - 1] + s[n / 2]) / 2.0);
}
inline double mean_of(const double *x, int64_t n) {
    long double s = 0;
    for (int64_t i = 0; i < n; ++i) s += x[i];
    return n > 0 ? double(s / n) : NaN;
}

// average ranks (1-based) of x: scipy.stats.rankdata(method='average')
vector<double> avg_ranks(const vector<double> &x) {
    const int64_t n = int64_t(x.size());
    vector<int64_t> o(n);
    for (int64_t i = 0; i < n; ++i) o[i] = i;
    std::stable_sort(o.begin(), o.end(), [&](int64_t a, int64_t b) { return x[a] < x[b]; });
    vector<double> r(n);
    for (int64_t a = 0; a < n;) {
        int64_t b = a + 1;
        while (b < n && x[o[b]] == x[o[a]]) ++b;
        const double v = double(a + b + 1) / 2.0;
        for (int64_t k = a; k < b; ++k) r[o[k]] = v;
        a = b;
    }
    return r;
}

// scipy.stats.spearmanr(range(n), x): (rho, p), NaN when n < 2 or x constant
void spearman_index(const vector<double> &x, double *rho, double *p) {
    const int64_t n = int64_t(x.size());
    *rho = *p = NaN;
    if (n < 2) return;
    bool constant = true;
    for (int64_t i = 1; i < n && constant; ++i) constant = x[i] == x[0];
    if (constant) return;
    const vector<double> ry = avg_ranks(x);
    const double m = double(n + 1) / 2.0;
    double sxy = 0, sxx = 0, syy = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double dx = double(i + 1) - m, dy = ry[i] - m;
        sxy += dx * dy;
        sxx += dx * dx;
        syy += dy * dy;
    }
    const double f = 1.0 / double(n - 1);  // (np.cov multiplies by the reciprocal of n - 1)
    double r = (sxy * f) / std::sqrt(sxx * f) / std::sqrt(syy * f);
    r = std::min(1.0, std::max(-1.0, r));
    const double dof = double(n - 2);
    double q = dof / ((r + 1.0) * (1.0 - r));
    if (q < 0.0) q = 0.0;
    *rho = r;
    *p = 2.0 * st::t_sf(std::fabs(r * std::sqrt(q)), dof);
}

// scipy.stats.shapiro(x): (W, p), NaN when n < 3
void shapiro(const vector<double> &x, double *w, double *p) {
    const int64_t n = int64_t(x.size());
    *w = *p = NaN;
    if (n < 3) return;
    vector<double> y(x);
    std::sort(y.begin(), y.end());
    const double x0 = x[n / 2];  // scipy: y = sort(x); y -= x[N // 2]
    for (auto &v : y) v -= x0;
    int ifault = 0;
    *w = st::swilk_sorted(y.data(), n, p, &ifault);
}

struct Desc {  // rq3:25-66 numbers (numpy describe)
    double count = 0, n_pos = 0, n_zero = 0, n_neg = 0, mean = NaN, median = NaN, std = NaN, min = NaN,
           max = NaN, q1 = NaN, q3 = NaN;
    vector<double> flat() const { return {count, n_pos, n_zero, n_neg, mean, median, std, min, max, q1, q3}; }
};
// describe of x given its ascending copy s
Desc describe(const vector<double> &x, const vector<double> &s) {
    Desc d;
    const int64_t n = int64_t(x.size());
    d.count = double(n);
    if (!n) return d;
    for (double v : x) {
        d.n_pos += v > 0;
        d.n_zero += v == 0;
        d.n_neg += v < 0;
    }
    d.mean = mean_of(x.data(), n);
    long double ss = 0;
    for (double v : x) ss += (long double)(v - d.mean) * (v - d.mean);
    d.std = std::sqrt(double(ss / n));
    d.median = median_sorted(s.data(), n);
    d.min = s[0];
    d.max = s[n - 1];
    d.q1 = pct_sorted(s.data(), n, 25);
    d.q3 = pct_sorted(s.data(), n, 75);
    return d;
}

vector<double> sorted_copy(const vector<double> &x) {
    vector<double> s(x);
    if (s.size() > (1u << 16))
        __gnu_parallel::sort(s.begin(), s.end());
    else
        std::sort(s.begin(), s.end());
    return s;
}

// scipy.stats.anderson(x, 'norm') from the ascending sample y: A2 and the 5 rounded critical values
vector<double> anderson(const vector<double> &y) {
    const int64_t n = int64_t(y.size());
    const double N = double(n), xbar = mean_of(y.data(), n);
    long double ss = 0;
    for (double v : y) ss += (long double)(v - xbar) * (v - xbar);
    const double s = std::sqrt(double(ss) / (N - 1.0));
    long double acc = 0;
#pragma omp parallel for reduction(+ : acc) schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const double wi = (y[i] - xbar) / s, wj = (y[n - 1 - i] - xbar) / s;
        acc += (2.0 * double(i + 1) - 1.0) / N * (st::log_ndtr(wi) + st::log_ndtr(-wj));
    }
    vector<double> out{-N - double(acc)};
    const double av[5] = {0.576, 0.656, 0.787, 0.918, 1.092};
    for (double a : av) out.push_back(std::rint(a / (1.0 + 4.0 / N - 25.0 / N / N) * 1000.0) / 1000.0);
    return out;
}

// scipy.stats.levene(x, y) (center='median') from the ascending samples: (W, p)
void levene(const vector<double> &x, const vector<double> &y, double *W, double *p) {
    const vector<double> *g[2] = {&x, &y};
    double zb[2], dv[2], nn[2];
    for (int k = 0; k < 2; ++k) {
        const vector<double> &s = *g[k];
        const int64_t n = int64_t(s.size());
        const double med = median_sorted(s.data(), n);
        long double a = 0;
        for (double v : s) a += std::fabs(v - med);
        zb[k] = double(a) / double(n);
        long double b = 0;
        for (double v : s) {
            const double d = std::fabs(v - med) - zb[k];
            b += (long double)d * d;
        }
        dv[k] = double(b);
        nn[k] = double(n);
    }
    const double N = nn[0] + nn[1];
    const double zbar = (zb[0] * nn[0] + zb[1] * nn[1]) / N;
    const double numer =
        (N - 2.0) * (nn[0] * (zb[0] - zbar) * (zb[0] - zbar) + nn[1] * (zb[1] - zbar) * (zb[1] - zbar));
    *W = numer / (dv[0] + dv[1]);
    *p = st::f1_sf(*W, N - 2.0);
}

// Brunner-Munzel (t, two-sided) and Mann-Whitney U (x vs y: two-sided p, U1) of two ascending
// samples: one merge visits every distinct value with its counts in x and y, which gives its
// average rank in the union and in each sample (scipy rankdata 'average') and the tie term.
struct TwoSample {
    double bm_stat, bm_p, mwu_p_two, u1;
};
TwoSample two_sample(const vector<double> &x, const vector<double> &y) {
    const int64_t nx = int64_t(x.size()), ny = int64_t(y.size());
    // visit(rc, rx, ry, cx, cy) once per distinct value, ascending
    auto merge = [&](auto visit) {
        for (int64_t i = 0, j = 0; i < nx || j < ny;) {
            const double v = j >= ny || (i < nx && x[i] <= y[j]) ? x[i] : y[j];
            int64_t cx = 0, cy = 0;
            while (i + cx < nx && x[i + cx] == v) ++cx;
            while (j + cy < ny && y[j + cy] == v) ++cy;
            visit(double(2 * (i + j) + cx + cy + 1) / 2.0, double(2 * i + cx + 1) / 2.0, double(2 * j + cy + 1) / 2.0,
                  cx, cy);
            i += cx;
            j += cy;
        }
    };
    double scx = 0, scy = 0, tie = 0;  // rank sums are exact in double (half-integers < 2^52)
    merge([&](double rc, double, double, int64_t cx, int64_t cy) {
        scx += double(cx) * rc;
        scy += double(cy) * rc;
        const double t = double(cx + cy);
        tie += t * t * t - t;
    });
    const double Nx = double(nx), Ny = double(ny);
    const double mcx = scx / Nx, mcy = scy / Ny;
    const double mx = (Nx + 1.0) / 2.0, my = (Ny + 1.0) / 2.0;
    double sx = 0, sy = 0;
    merge([&](double rc, double rx, double ry, int64_t cx, int64_t cy) {
        const double dx = ((rc - rx) - mcx) + mx, dy = ((rc - ry) - mcy) + my;
        sx += double(cx) * dx * dx;
        sy += double(cy) * dy * dy;
    });
    const double Sx = double(sx) / (Nx - 1.0), Sy = double(sy) / (Ny - 1.0);
    TwoSample r;
    r.bm_stat = Nx * Ny * (mcy - mcx) / ((Nx + Ny) * std::sqrt(Nx * Sx + Ny * Sy));
    const double num = (Nx * Sx + Ny * Sy) * (Nx * Sx + Ny * Sy);
    const double den = (Nx * Sx) * (Nx * Sx) / (Nx - 1.0) + (Ny * Sy) * (Ny * Sy) / (Ny - 1.0);
    r.bm_p = 2.0 * st::t_sf(std::fabs(r.bm_stat), num / den);
    // Mann-Whitney U: asymptotic with tie and continuity corrections, exact for small tie-free samples
    const double U1 = scx - Nx * (Nx + 1.0) / 2.0, U2 = Nx * Ny - U1, nn = Nx + Ny;
    const double U = std::max(U1, U2);
    double p;
    if (!(nx > 8 && ny > 8) && tie == 0.0) {
        const int64_t n1 = std::min(nx, ny), n2 = std::max(nx, ny), deg = n1 * n2;
        vector<double> c(deg + 1, 0.0);
        c[0] = 1.0;
        for (int64_t k = 1; k <= n1; ++k) {
            const int64_t m = n2 + k;
            for (int64_t v = deg; v >= m; --v) c[v] -= c[v - m];
            for (int64_t v = k; v <= deg; ++v) c[v] += c[v - k];
        }
        double total = 0;
        for (double v : c) total += v;
        const int64_t k = int64_t(U), kc = deg - k, lim = std::min(k, kc);
        double cdf = 0;
        for (int64_t v = 0; v <= lim; ++v) cdf += c[v] / total;
        p = k < kc ? 1.0 - cdf + c[k] / total : cdf;
    } else {
        const double sd = std::sqrt(Nx * Ny / 12.0 * ((nn + 1.0) - tie / (nn * (nn - 1.0))));
        p = st::norm_sf((U - Nx * Ny / 2.0 - 0.5) / sd);
    }
    r.mwu_p_two = std::min(1.0, std::max(0.0, 2.0 * p));
    r.u1 = U1;
    return r;
}

// ------------------------------------------------------------------------------------- the store
struct Store {
    const fz_tables *t;
    int64_t P;
    Index B, C, I;  // builds by (project, time), coverage by (project, date), issues by (project, rts)
    vector<uint8_t> elig;
};

void build_store(Store &s, const fz_tables *t) {
    s.t = t;
    s.P = t->n_projects;
    const int64_t *bt = t->b_time, *cd = t->c_date, *rts = t->i_rts;
    s.B = index_by_project(t->b_project, t->n_builds, s.P, [=](int32_t r) { return bt[r]; });
    s.C = index_by_project(t->c_project, t->n_cov, s.P, [=](int32_t r) { return cd[r]; });
    s.I = index_by_project(t->i_project, t->n_issues, s.P, [=](int32_t r) { return rts[r]; });
    // eligibility (rq1_detection_rate.py:144-152): >= 365 rows with coverage > 0 before the limit
    s.elig.assign(s.P, 0);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t p = 0; p < s.P; ++p) {
        int64_t c = 0;
        for (int64_t j = s.C.off[p]; j < s.C.off[p + 1]; ++j) {
            const int32_t r = s.C.rows[j];
            c += (t->c_valid[r] & FZ_VALID_COVERAGE) && t->c_coverage[r] > 0 && t->c_date[r] < LIMIT_US;
        }
        s.elig[p] = c >= 365;
    }
}

// -------------------------------------------------------------------------------------------- RQ1
void rq1(const Store &s, Result &R, int64_t threshold) {
    const fz_tables *t = s.t;
    const int64_t P = s.P;
    const View vb = view_of(s.B, t->b_time, [=](int32_t r) {
        return t->b_type[r] == BT_FUZZING && (t->b_result[r] == R_FINISH || t->b_result[r] == R_HALFWAY_LOWER) &&
               t->b_time[r] < LIMIT_US;
    });
    const View fz = view_of(s.B, t->b_time, [=](int32_t r) { return t->b_type[r] == BT_FUZZING; });
    vector<int64_t> c_lim(P), c_fix(P), c_tgt(P), c_without(P);
    vector<vector<int64_t>> m_issue(P), m_build(P);
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t p = 0; p < P; ++p) {
        const int64_t minv = vb.len(p) ? vb.k(p)[0] : TS_NULL;
        for (int64_t j = s.I.off[p]; j < s.I.off[p + 1]; ++j) {
            const int32_t i = s.I.rows[j];
            const int64_t rts = t->i_rts[i];
            const bool lim = rts < LIMIT_US, fx = fixed_status(t->i_status[i]);
            c_lim[p] += lim;
            c_fix[p] += lim && fx;
            c_tgt[p] += lim && fx && s.elig[p];
            if (!(fx && s.elig[p])) continue;
            if (!(rts != TS_NULL && rts > minv)) c_without[p] += t->pi_count[p];  // queries1.py:280-314
            if (rts == TS_NULL) continue;
            const int64_t k = lower(vb.k(p), vb.len(p), rts) - 1;                   // queries1.py:15-58
            if (k >= 0) {
                m_issue[p].push_back(i);
                m_build[p].push_back(vb.r(p)[k]);
            }
        }
    }
    // ROW_NUMBER() OVER (PARTITION BY number ORDER BY timecreated DESC): the latest build wins, a tie
    // goes to the first row in ORDER BY project, rts
    vector<int64_t> ci, mb;
    for (int64_t p = 0; p < P; ++p) {
        ci.insert(ci.end(), m_issue[p].begin(), m_issue[p].end());
        mb.insert(mb.end(), m_build[p].begin(), m_build[p].end());
    }
    std::unordered_map<int64_t, std::pair<int64_t, int64_t>> best;
    best.reserve(ci.size() * 2);
    for (int64_t k = 0; k < int64_t(ci.size()); ++k) {
        const int64_t num = t->i_number[ci[k]], tb = t->b_time[mb[k]];
        auto it = best.find(num);
        if (it == best.end() || tb > it->second.first) best[num] = {tb, k};
    }
    vector<uint8_t> keep(ci.size(), 0);
    for (auto &e : best) keep[e.second.second] = 1;
    vector<int64_t> kept_i, kept_b;
    for (size_t k = 0; k < ci.size(); ++k)
        if (keep[k]) {
            kept_i.push_back(ci[k]);
            kept_b.push_back(mb[k]);
        }
    // phase 1: projects alive per iteration; phase 2: distinct (iteration, project) detections
    int64_t max_iter = 0, total_fuzz = 0;
    for (int64_t p = 0; p < P; ++p)
        if (s.elig[p]) {
            max_iter = std::max(max_iter, fz.len(p));
            total_fuzz += fz.len(p);
        }
    vector<int64_t> iter_total(max_iter + 1, 0), iter_det(max_iter, 0);
    for (int64_t p = 0; p < P; ++p)
        if (s.elig[p]) ++iter_total[0], --iter_total[fz.len(p)];  // projects with >= i builds
    for (int64_t i = 1; i <= max_iter; ++i) iter_total[i] += iter_total[i - 1];
    iter_total.resize(max_iter);
    for (size_t a = 0; a < kept_i.size();) {
        const int64_t p = t->i_project[kept_i[a]];
        size_t b = a;
        vector<int64_t> its;
        for (; b < kept_i.size() && int64_t(t->i_project[kept_i[b]]) == p; ++b) {
            const int64_t it = lower(fz.k(p), fz.len(p), t->i_rts[kept_i[b]]);
            if (it > 0) its.push_back(it);
        }
        std::sort(its.begin(), its.end());
        its.erase(std::unique(its.begin(), its.end()), its.end());
        for (int64_t it : its) ++iter_det[it - 1];
        a = b;
    }
    auto nproj = [&](const vector<int64_t> &c) {
        int64_t n = 0;
        for (int64_t v : c) n += v > 0;
        return n;
    };
    auto sum = [](const vector<int64_t> &c) {
        int64_t n = 0;
        for (int64_t v : c) n += v;
        return n;
    };
    vector<int64_t> mp(P, 0);
    for (int64_t i : kept_i) mp[t->i_project[i]] = 1;
    int64_t n_elig = 0;
    for (uint8_t e : s.elig) n_elig += e;
    R.i["rq1_counts"] = {sum(c_lim), nproj(c_lim), sum(c_fix), nproj(c_fix), n_elig, sum(c_without), sum(c_tgt),
                         nproj(c_tgt), total_fuzz, int64_t(kept_i.size()), sum(mp)};
    R.i["rq1_iter_total"] = iter_total;
    R.i["rq1_iter_detected"] = iter_det;
    R.i["rq1_matched_issue"] = kept_i;
    R.i["rq1_matched_build"] = kept_b;
    // late stage (rq1_detection_rate.py:233-268): first_down is a key used as a list index
    vector<double> rates;
    int64_t first_down = -1;
    for (int64_t k = 1; k <= max_iter; ++k)
        if (iter_total[k - 1] >= threshold) {
            const double r = double(iter_det[k - 1]) / double(iter_total[k - 1]) * 100;
            if (r < 5 && first_down == -1) first_down = k;
            rates.push_back(r);
        }
    const int64_t nr = int64_t(rates.size());
    int64_t from = first_down < 0 ? std::max<int64_t>(0, nr + first_down) : first_down;
    vector<double> late;
    for (int64_t k = from; k < nr; ++k) late.push_back(rates[k]);
    vector<double> lo;
    if (!late.empty()) {
        vector<double> sl(late);
        std::sort(sl.begin(), sl.end());
        double nz = NaN, nzero = 0;
        for (double v : late) {
            nzero += v == 0;
            if (v != 0) nz = std::isnan(nz) ? v : std::min(nz, v);
        }
        const int64_t n = int64_t(sl.size());
        lo = {double(n), nzero, sl[0], sl[n - 1], pct_sorted(sl.data(), n, 25), pct_sorted(sl.data(), n, 75),
              median_sorted(sl.data(), n), mean_of(late.data(), n), nz};
    }
    R.f["rq1_late"] = lo;
}

// -------------------------------------------------------------------------------------- RQ2 count
void rq2_count(const Store &s, Result &R) {
    const fz_tables *t = s.t;
    const int64_t P = s.P;
    const View v = view_of(s.C, t->c_date, [=](int32_t r) {
        return (t->c_valid[r] & FZ_VALID_COVERAGE) && t->c_coverage[r] != 0 && t->c_date[r] < LIMIT_US;
    });
    vector<int64_t> ep;
    for (int64_t p = 0; p < P; ++p)
        if (s.elig[p]) ep.push_back(p);
    const int64_t E = int64_t(ep.size());
    vector<vector<double>> trend(E);
    vector<int64_t> raw_n(E), n_tr(E);
    vector<double> sw_w(E), sw_p(E), corr(E), corr_p(E);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t e = 0; e < E; ++e) {
        const int64_t p = ep[e];
        raw_n[e] = v.len(p);
        for (int64_t j = 0; j < v.len(p); ++j) {
            const int32_t r = v.r(p)[j];
            if (t->c_total[r] != 0) trend[e].push_back(double(t->c_covered[r]) / double(t->c_total[r]) * 100);
        }
        n_tr[e] = int64_t(trend[e].size());
        shapiro(trend[e], &sw_w[e], &sw_p[e]);         // rq2_coverage_count.py:305-314
        spearman_index(trend[e], &corr[e], &corr_p[e]);  // :316-322
    }
    int64_t ms = 1;
    for (int64_t e = 0; e < E; ++e) ms = std::max(ms, n_tr[e]);
    vector<vector<double>> sess(ms);  // :330-333: session i = the i-th value of every project
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < ms; ++i)
        for (int64_t e = 0; e < E; ++e)
            if (n_tr[e] > i) sess[i].push_back(trend[e][i]);
    vector<int64_t> offs(ms + 1, 0);
    for (int64_t i = 0; i < ms; ++i) offs[i + 1] = offs[i] + int64_t(sess[i].size());
    vector<double> vals(offs[ms]);
    int64_t ge = 0;
    while (ge < ms && int64_t(sess[ge].size()) >= 100) ++ge;  // :390 (lengths never increase)
    vector<double> avg(ge), med(ge), dmean(ge), pct(5 * ge);
    const double qs[5] = {5, 25, 50, 75, 95};
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t i = 0; i < ms; ++i) {
        std::copy(sess[i].begin(), sess[i].end(), vals.begin() + offs[i]);
        if (i >= ge) continue;
        vector<double> so(sess[i]);
        std::sort(so.begin(), so.end());
        const int64_t n = int64_t(so.size());
        avg[i] = dmean[i] = mean_of(sess[i].data(), n);
        med[i] = median_sorted(so.data(), n);
        for (int j = 0; j < 5; ++j) pct[j * ge + i] = pct_sorted(so.data(), n, qs[j]);
    }
    vector<double> valid;
    for (double c : corr)
        if (!std::isnan(c)) valid.push_back(c);
    vector<double> sv(valid);
    std::sort(sv.begin(), sv.end());
    double sp_r = NaN, sp_p = NaN, shw = NaN, shp = NaN;
    if (ge > 1) spearman_index(med, &sp_r, &sp_p);
    if (ge >= 3) shapiro(med, &shw, &shp);
    R.i["rq2c_raw_n"] = raw_n;
    R.i["rq2c_n_trend"] = n_tr;
    R.f["rq2c_sw_w"] = sw_w;
    R.f["rq2c_sw_p"] = sw_p;
    R.f["rq2c_corr"] = corr;
    R.i["rq2c_session_offsets"] = offs;
    R.f["rq2c_session_values"] = vals;
    R.f["rq2c_scalars"] = {mean_of(valid.data(), int64_t(valid.size())), median_sorted(sv.data(), int64_t(sv.size())),
                           sp_r, sp_p, shp};
    R.f["rq2c_average"] = avg;
    R.f["rq2c_median"] = med;
    R.f["rq2c_pct"] = pct;
    R.f["rq2c_dist_mean"] = dmean;
}

// ---------------------------------------------------------------------------------------- RQ2 add
void rq2_add(const Store &s, Result &R) {
    const fz_tables *t = s.t;
    const int64_t P = s.P;
    const View bm = view_of(s.B, t->b_time, [=](int32_t r) {
        return t->b_type[r] == BT_COVERAGE && (t->b_result[r] == R_HALFWAY_UPPER || t->b_result[r] == R_FINISH) &&
               t->b_time[r] < LIMIT_US;
    });
    const View cs = view_of(s.C, t->c_date, [=](int32_t r) { return t->c_date[r] < LIMIT_US; });
    vector<vector<int64_t>> rows(P);
    vector<vector<double>> dts(P), dcs(P);
    vector<int64_t> flags(2 * P, 0);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t p = 0; p < P; ++p) {
        if (!s.elig[p] || bm.len(p) == 0 || cs.len(p) == 0) continue;
        const int32_t *br = bm.r(p), *cr = cs.r(p);
        const int64_t nb = bm.len(p), nc = cs.len(p);
        vector<int64_t> cday(nc);
        for (int64_t j = 0; j < nc; ++j) {
            cday[j] = day_of(t->c_date[cr[j]]);
            if (!(t->c_valid[cr[j]] & FZ_VALID_COVERED)) flags[2 * p] = 1;
            if (!(t->c_valid[cr[j]] & FZ_VALID_TOTAL)) flags[2 * p + 1] = 1;
        }
        auto cov_on = [&](int32_t b) {  // coverage row on date(b), -1 none
            const int64_t d = day_of(t->b_time[b]);
            const int64_t j = lower(cday.data(), nc, d);
            return j < nc && cday[j] == d ? int64_t(cr[j]) : int64_t(-1);
        };
        auto val = [&](int64_t c, double &cv, double &tv) {
            cv = tv = NaN;
            if (c < 0) return;
            if (t->c_valid[c] & FZ_VALID_COVERED) cv = double(t->c_covered[c]);
            if (t->c_valid[c] & FZ_VALID_TOTAL) tv = double(t->c_total[c]);
        };
        int64_t run0 = 0;  // first build of the current (modules, revisions) run
        for (int64_t j = 1; j <= nb; ++j) {
            if (j < nb && t->b_group[br[j]] == t->b_group[br[j - 1]]) continue;
            if (j == nb) break;
            const int32_t f = br[run0], e = br[j - 1], st_ = br[j];
            const int64_t c0 = cov_on(e), c1 = cov_on(st_);
            double cv0, tv0, cv1, tv1;
            val(c0, cv0, tv0);
            val(c1, cv1, tv1);
            double dt = NaN, dc = NaN;  // rq2_coverage_and_added.py:189-200
            if (!std::isnan(tv0) && tv0 != 0 && !std::isnan(tv1) && tv1 != 0) {
                dt = tv1 - tv0;
                dc = (cv1 / tv1) * 100 - (cv0 / tv0) * 100;
            }
            for (int64_t x : {p, int64_t(f), int64_t(e), int64_t(st_), c0, c1}) rows[p].push_back(x);
            dts[p].push_back(dt);
            dcs[p].push_back(dc);
            run0 = j;
        }
    }
    vector<int64_t> ro;
    vector<double> dt, dc;
    for (int64_t p = 0; p < P; ++p) {
        ro.insert(ro.end(), rows[p].begin(), rows[p].end());
        dt.insert(dt.end(), dts[p].begin(), dts[p].end());
        dc.insert(dc.end(), dcs[p].begin(), dcs[p].end());
    }
    R.i["rq2a_rows"] = ro;
    R.f["rq2a_diff_total"] = dt;
    R.f["rq2a_diff_coverage"] = dc;
    R.i["rq2a_flags"] = flags;
}

// -------------------------------------------------------------------------------------------- RQ3
void rq3(const Store &s, Result &R) {
    const fz_tables *t = s.t;
    const int64_t P = s.P;
    const View fz = view_of(s.B, t->b_time, [=](int32_t r) {
        return t->b_type[r] == BT_FUZZING && (t->b_result[r] == R_HALFWAY_UPPER || t->b_result[r] == R_FINISH) &&
               t->b_time[r] < LIMIT_US;
    });
    const View cb =
        view_of(s.B, t->b_time, [=](int32_t r) { return t->b_type[r] == BT_COVERAGE && t->b_time[r] < RQ3_LIMIT_US; });
    const View tc = view_of(s.C, t->c_date,
                            [=](int32_t r) { return (t->c_valid[r] & FZ_VALID_COVERED) && t->c_date[r] < RQ3_LIMIT_US; });
    auto issue_ok = [&](int32_t i, int64_t p) {
        return fixed_status(t->i_status[i]) && s.elig[p] && t->i_rts[i] < LIMIT_US;
    };
    vector<int64_t> n_iss(P, 0);
    int64_t last = -1;  // the last issue-bearing project is never flushed (rq3:245-257)
    for (int64_t p = 0; p < P; ++p) {
        for (int64_t j = s.I.off[p]; j < s.I.off[p + 1]; ++j) n_iss[p] += issue_ok(s.I.rows[j], p);
        if (n_iss[p]) last = p;
    }
    struct Det {
        double pct;
        int64_t cov, tot, project, rts, issue;
    };
    struct Non {
        double pct;
        int64_t cov, tot;
    };
    vector<vector<Det>> det(P);
    vector<vector<Non>> non(P);
    auto frac = [&](int32_t r) { return double(t->c_covered[r]) / double(t->c_total[r]); };
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t p = 0; p < P; ++p) {
        if (!n_iss[p]) continue;
        const int64_t ntr = tc.len(p);
        const int32_t *tr = tc.r(p);
        vector<int64_t> days(ntr);
        for (int64_t k = 0; k < ntr; ++k) days[k] = day_of(tc.k(p)[k]);
        for (int64_t j = s.I.off[p]; j < s.I.off[p + 1]; ++j) {
            const int32_t i = s.I.rows[j];
            if (!issue_ok(i, p)) continue;
            if (fz.len(p) == 0 || cb.len(p) == 0 || ntr == 0) continue;
            const int64_t rts = t->i_rts[i];
            const int64_t a = lower(fz.k(p), fz.len(p), rts) - 1;  // :269 last Fuzzing build before
            if (a < 0) continue;
            const int32_t lf = fz.r(p)[a];
            const int64_t b = upper(cb.k(p), cb.len(p), rts);  // :273 first Coverage build after
            if (b >= cb.len(p)) continue;
            const int32_t fc = cb.r(p)[b];
            if (!(t->b_result[fc] == R_HALFWAY_UPPER || t->b_result[fc] == R_FINISH)) continue;
            if (t->b_time[fc] - t->b_time[lf] > US_DAY) continue;                                   // :277
            if (t->b_rev_canon[lf] < 0 || t->b_rev_canon[lf] != t->b_rev_canon[fc]) continue;      // :280
            const int64_t target = day_of(rts) + 1;                                                 // :286-292
            int64_t k = std::max<int64_t>(1, lower(days.data(), ntr, target));
            if (k >= ntr || days[k] != target) continue;
            if (t->c_covered[tr[k]] == 0) continue;
            const int32_t c0 = tr[k - 1], c1 = tr[k];
            if (t->c_total[c0] > 0 && t->c_total[c1] > 0)
                det[p].push_back({(frac(c1) - frac(c0)) * 100, t->c_covered[c1] - t->c_covered[c0],
                                  t->c_total[c1] - t->c_total[c0], p, rts, i});
        }
        if (p == last) continue;
        vector<int64_t> dd;
        for (const Det &d : det[p]) dd.push_back(day_of(d.rts));
        std::sort(dd.begin(), dd.end());
        for (int64_t k = 1; k < ntr; ++k) {
            const int32_t a = tr[k - 1], b = tr[k];
            if (std::binary_search(dd.begin(), dd.end(), days[k])) continue;
            if (t->c_total[a] > 0 && t->c_total[b] > 0)
                non[p].push_back({(frac(b) - frac(a)) * 100, t->c_covered[b] - t->c_covered[a],
                                  t->c_total[b] - t->c_total[a]});
        }
    }
    vector<double> dpct, npct, dtotf;
    vector<int64_t> dcols, ncols;
    int64_t n_all = 0;
    for (int64_t p = 0; p < P; ++p) {
        n_all += n_iss[p];
        for (const Det &d : det[p]) {
            dpct.push_back(d.pct);
            dtotf.push_back(double(d.tot));
            for (int64_t x : {d.cov, d.tot, d.project, d.issue}) dcols.push_back(x);
        }
        for (const Non &n : non[p]) {
            npct.push_back(n.pct);
            for (int64_t x : {n.cov, n.tot}) ncols.push_back(x);
        }
    }
    R.i["rq3_counts"] = {n_all, int64_t(dpct.size()), int64_t(npct.size())};
    R.f["rq3_det_pct"] = dpct;
    R.f["rq3_non_pct"] = npct;
    R.i["rq3_det_cols"] = dcols;
    R.i["rq3_non_cols"] = ncols;
    // statistics (:321-352)
    const vector<double> sd = sorted_copy(dpct), sn = sorted_copy(npct), stt = sorted_copy(dtotf);
    vector<double> desc;
    for (auto xs : {std::make_pair(&dpct, &sd), std::make_pair(&npct, &sn), std::make_pair(&dtotf, &stt)}) {
        const vector<double> d = describe(*xs.first, *xs.second).flat();
        desc.insert(desc.end(), d.begin(), d.end());
    }
    R.f["rq3_describe"] = desc;
    vector<double> tests;
    if (!dpct.empty() && !npct.empty()) {
        tests = anderson(sd);
        const vector<double> an = anderson(sn);
        tests.insert(tests.end(), an.begin(), an.end());
        double w, pw;
        levene(sd, sn, &w, &pw);
        const TwoSample bm = two_sample(sd, sn);
        for (double x : {w, pw, bm.bm_stat, bm.bm_p}) tests.push_back(x);
    }
    R.f["rq3_tests"] = tests;
}

// ------------------------------------------------------------------------------------------- RQ4a
void rq4a(const Store &s, const fz_rq4_groups *g, Result &R) {
    const fz_tables *t = s.t;
    const int64_t P = s.P;
    const View fb = view_of(s.B, t->b_time, [=](int32_t r) { return t->b_type[r] == BT_FUZZING && t->b_time[r] < LIMIT_US; });
    const View fi = view_of(s.I, t->i_rts, [=](int32_t r) { return fixed_status(t->i_status[r]) && t->i_rts[r] < LIMIT_US; });
    auto in_group = [&](int64_t p, int k) {  // rq4a_bug.py:94-121 (eligible projects without a CSV row -> G1)
        if (!s.elig[p]) return false;
        return ((g->member[p] >> k) & 1) || (k == 0 && ((g->member[p] >> 4) & 1));
    };
    int64_t mx = 0;
    for (int64_t p = 0; p < P; ++p)
        if (in_group(p, 0) || in_group(p, 1)) mx = std::max(mx, fb.len(p));
    vector<int64_t> tab[4];  // g1 total, g1 det, g2 total, g2 det (:302-346)
    for (auto &v : tab) v.assign(mx + 1, 0);
    vector<vector<int64_t>> dk(P);
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t p = 0; p < P; ++p) {
        if (!(in_group(p, 0) || in_group(p, 1)) || fb.len(p) == 0) continue;
        for (int64_t j = 0; j < fi.len(p); ++j) {
            const int64_t k = lower(fb.k(p), fb.len(p), fi.k(p)[j]);
            if (k > 0) dk[p].push_back(k);
        }
        std::sort(dk[p].begin(), dk[p].end());
        dk[p].erase(std::unique(dk[p].begin(), dk[p].end()), dk[p].end());
    }
    for (int64_t p = 0; p < P; ++p)
        for (int gi = 0; gi < 2; ++gi) {
            if (!in_group(p, gi) || fb.len(p) == 0) continue;
            ++tab[2 * gi][0];
            --tab[2 * gi][fb.len(p)];
            for (int64_t k : dk[p]) ++tab[2 * gi + 1][k - 1];
        }
    for (int gi = 0; gi < 2; ++gi)
        for (int64_t i = 1; i <= mx; ++i) tab[2 * gi][i] += tab[2 * gi][i - 1];
    for (auto &v : tab) v.resize(mx);
    // G4: introduction iteration (:246-299), pre/post windows of N = 7 builds (:350-412)
    const int N = 7;
    vector<int64_t> intro;
    int64_t steps[15][2] = {};
    int64_t trans[4] = {0, 0, 0, 0};
    int64_t any_window = 0;
    for (int64_t p = 0; p < P; ++p) {
        if (!in_group(p, 3)) continue;
        const int64_t ct = g->corpus_us[p];
        if (ct == TS_NULL) continue;
        const int64_t *bt = fb.k(p), nb = fb.len(p);
        const int64_t npre = lower(bt, nb, ct);
        intro.push_back(p);
        intro.push_back(nb == 0 ? 0 : npre);
        if (npre == 0) continue;
        const int64_t idx = npre - 1;
        if (idx - (N - 1) < 0 || idx + N >= nb - 1) continue;
        any_window = 1;
        const int64_t *it = fi.k(p), ni = fi.len(p);
        auto hit = [&](int64_t a, int64_t b) { return lower(it, ni, a) < lower(it, ni, b); };
        bool pre_any = false, post_any = false;
        for (int k = 1; k <= N; ++k) {
            const bool d0 = hit(bt[idx - (k - 1)], bt[idx - (k - 1) + 1]);
            steps[N - k][0] += 1;
            steps[N - k][1] += d0;
            pre_any |= d0;
            const bool d1 = hit(bt[idx + k], bt[idx + k + 1]);
            steps[N + k][0] += 1;
            steps[N + k][1] += d1;
            post_any |= d1;
        }
        trans[pre_any && post_any ? 0 : pre_any ? 1 : post_any ? 2 : 3] += 1;
    }
    // finishing (:156-207, :698-747, :277-285, :412-510)
    vector<double> sc;
    for (int gi = 0; gi < 2; ++gi) {
        vector<double> rates;
        for (int64_t i = 0; i < mx; ++i) {
            if (tab[0][i] >= 100 && tab[2][i] >= 100) {
                const int64_t tt = tab[2 * gi][i], dd = tab[2 * gi + 1][i];
                rates.push_back(tt > 0 ? double(dd) / double(tt) * 100 : 0.0);
            }
        }
        size_t f5 = 0;
        while (f5 < rates.size() && !(rates[f5] < 5)) ++f5;
        vector<double> ra(rates.begin() + f5, rates.end());
        std::sort(ra.begin(), ra.end());
        const int64_t n = int64_t(ra.size());
        sc.push_back(n ? median_sorted(ra.data(), n) : NaN);
        sc.push_back(n ? pct_sorted(ra.data(), n, 75) - pct_sorted(ra.data(), n, 25) : NaN);
    }
    vector<double> pos;
    for (size_t k = 1; k < intro.size(); k += 2)
        if (intro[k] > 0) pos.push_back(double(intro[k]));
    if (!pos.empty()) {
        vector<double> so(pos);
        std::sort(so.begin(), so.end());
        const int64_t n = int64_t(so.size());
        for (double x : {mean_of(pos.data(), n), median_sorted(so.data(), n), so[0], so[n - 1]}) sc.push_back(x);
    } else {
        for (int k = 0; k < 4; ++k) sc.push_back(NaN);
    }
    int64_t pre_n = 0, pre_d = 0, post_n = 0, post_d = 0;
    for (int k = 1; k <= N; ++k) {
        pre_n += steps[N - k][0];
        pre_d += steps[N - k][1];
        post_n += steps[N + k][0];
        post_d += steps[N + k][1];
    }
    sc.push_back(pre_n ? double(pre_d) / double(pre_n) * 100 : 0.0);
    sc.push_back(post_n ? double(post_d) / double(post_n) * 100 : 0.0);
    R.i["rq4a_g1_total"] = tab[0];
    R.i["rq4a_g1_det"] = tab[1];
    R.i["rq4a_g2_total"] = tab[2];
    R.i["rq4a_g2_det"] = tab[3];
    R.i["rq4a_intro"] = intro;
    vector<int64_t> sv;
    for (int k = 0; k < 15; ++k)
        if (k != N) sv.push_back(steps[k][0]), sv.push_back(steps[k][1]);
    R.i["rq4a_steps"] = sv;  // s = -7..-1, 1..7
    R.i["rq4a_transition"] = {trans[0], trans[1], trans[2], trans[3], any_window};
    R.f["rq4a_scalars"] = sc;
}

// ------------------------------------------------------------------------------------------- RQ4b
void rq4b(const Store &s, const fz_rq4_groups *g, Result &R) {
    const fz_tables *t = s.t;
    const int64_t P = s.P;
    auto in_group = [&](int64_t p, int k) { return s.elig[p] && ((g->member[p] >> k) & 1); };  // :193-219
    const View full = view_of(s.C, t->c_date, [=](int32_t r) {
        return (t->c_valid[r] & FZ_VALID_COVERAGE) && t->c_coverage[r] > 0 && t->c_date[r] < LIMIT_US;
    });
    const View pos_all =
        view_of(s.C, t->c_date, [=](int32_t r) { return (t->c_valid[r] & FZ_VALID_COVERAGE) && t->c_coverage[r] > 0; });
    vector<int64_t> gp[2];  // G2, G1 projects in id order
    int64_t ms = 0;
    for (int64_t p = 0; p < P; ++p)
        for (int gi = 0; gi < 2; ++gi)
            if (in_group(p, 1 - gi)) {
                gp[gi].push_back(p);
                ms = std::max(ms, full.len(p));
            }
    vector<int64_t> c2(ms), c1(ms);
    vector<double> q2(3 * ms, NaN), q1(3 * ms, NaN), pb(ms, NaN);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t i = 0; i < ms; ++i) {  // :910-1015
        vector<double> a[2];
        for (int gi = 0; gi < 2; ++gi)
            for (int64_t p : gp[gi])
                if (full.len(p) > i) a[gi].push_back(t->c_coverage[full.r(p)[i]]);
        c2[i] = int64_t(a[0].size());
        c1[i] = int64_t(a[1].size());
        for (int gi = 0; gi < 2; ++gi) {
            if (a[gi].empty()) continue;
            std::sort(a[gi].begin(), a[gi].end());
            double *q = gi == 0 ? &q2[3 * i] : &q1[3 * i];
            for (int j = 0; j < 3; ++j) q[j] = pct_sorted(a[gi].data(), int64_t(a[gi].size()), 25.0 * (j + 1));
        }
        if (a[0].size() >= 5 && a[1].size() >= 5) pb[i] = two_sample(a[0], a[1]).bm_p;
    }
    int64_t last = -1;  // :849-860
    for (int64_t i = 0; i < ms; ++i)
        if (c2[i] >= 100 && c1[i] >= 100) last = i;
    vector<double> sp6;
    if (last >= 0) {  // :879-899 over the sessions whose quartile triples are all non-NaN
        vector<double> seq[6];
        for (int64_t i = 0; i <= last; ++i) {
            bool ok = true;
            for (int j = 0; j < 3; ++j) ok = ok && !std::isnan(q2[3 * i + j]) && !std::isnan(q1[3 * i + j]);
            if (!ok) continue;
            for (int j = 0; j < 3; ++j) {
                seq[j].push_back(q1[3 * i + j]);
                seq[3 + j].push_back(q2[3 * i + j]);
            }
        }
        if (!seq[0].empty())
            for (auto &x : seq) {
                double r, pv;
                spearman_index(x, &r, &pv);
                sp6.push_back(r);
                sp6.push_back(pv);
            }
    }
    // coverage deltas around the corpus date, G3 u G4 in CSV order (:725-797)
    vector<double> pre[7], post[7];
    for (int64_t k = 0; k < g->n_order; ++k) {
        const int64_t p = g->order[k];
        if (!(in_group(p, 2) || in_group(p, 3)) || g->corpus_us[p] == TS_NULL) continue;
        const int64_t cd = (g->corpus_us[p] / US_DAY) * US_DAY;
        const int64_t n = pos_all.len(p), j = lower(pos_all.k(p), n, cd);
        if (j < 7 || j + 7 > n) continue;
        for (int i = 0; i < 7; ++i) {
            pre[i].push_back(t->c_coverage[pos_all.r(p)[j - 1 - i]]);
            post[i].push_back(t->c_coverage[pos_all.r(p)[j + i]]);
        }
    }
    vector<double> pre_flat, post_flat, med;
    for (int i = 0; i < 7; ++i) {
        pre_flat.insert(pre_flat.end(), pre[i].begin(), pre[i].end());
        post_flat.insert(post_flat.end(), post[i].begin(), post[i].end());
    }
    for (auto *side : {pre, post})
        for (int i = 0; i < 7; ++i) {
            vector<double> so(side[i]);
            std::sort(so.begin(), so.end());
            med.push_back(median_sorted(so.data(), int64_t(so.size())));
        }
    // initial coverage G2 vs G1 (:221-313)
    vector<double> init[2];
    for (int gi = 0; gi < 2; ++gi)
        for (int64_t p : gp[gi])
            if (full.len(p)) init[gi].push_back(t->c_coverage[full.r(p)[0]]);
    vector<double> tests;
    if (!init[0].empty() && !init[1].empty()) {
        const vector<double> s2 = sorted_copy(init[0]), s1 = sorted_copy(init[1]);
        const TwoSample ts = two_sample(s2, s1);
        double w, pw;
        levene(s2, s1, &w, &pw);
        tests = {ts.mwu_p_two, 2.0 * ts.u1 / (double(init[0].size()) * double(init[1].size())) - 1.0, ts.bm_stat,
                 ts.bm_p, w, pw};
    }
    R.i["rq4b_c2"] = c2;
    R.i["rq4b_c1"] = c1;
    R.f["rq4b_g2_q"] = q2;
    R.f["rq4b_g1_q"] = q1;
    R.f["rq4b_p_bm"] = pb;
    R.i["rq4b_last"] = {last};
    R.f["rq4b_spearman6"] = sp6;
    R.f["rq4b_pre"] = pre_flat;
    R.f["rq4b_post"] = post_flat;
    R.f["rq4b_medians"] = med;
    R.f["rq4b_init_g2"] = init[0];
    R.f["rq4b_init_g1"] = init[1];
    R.f["rq4b_tests"] = tests;
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
extern "C" {

enum { FZCPU_RQ1 = 1, FZCPU_RQ2_COUNT = 2, FZCPU_RQ2_ADD = 4, FZCPU_RQ3 = 8, FZCPU_RQ4A = 16, FZCPU_RQ4B = 32 };

// Index build + the analyses in `stages` (FZCPU_* bits) with `threads` OpenMP threads (0: all).
// seconds[7] (may be NULL): store, rq1, rq2_count, rq2_add, rq3, rq4a, rq4b wall times.  Returns a
// handle for fzcpu_get_* / fzcpu_free, NULL on a bad argument.
void *fzcpu_run(const fz_tables *t, const fz_rq4_groups *g, uint32_t stages, int threads, double *seconds) {
    if (!t || t->n_projects < 0 || ((stages & (FZCPU_RQ4A | FZCPU_RQ4B)) && !g)) return nullptr;
    if (threads > 0) omp_set_num_threads(threads);
    Result *R = new Result;
    double tm[7] = {0};
    double t0 = omp_get_wtime();
    Store s;
    build_store(s, t);
    double t1 = omp_get_wtime();
    tm[0] = t1 - t0;
    auto stage = [&](int bit, int slot, auto fn) {
        if (!(stages & bit)) return;
        const double a = omp_get_wtime();
        fn();
        tm[slot] = omp_get_wtime() - a;
    };
    stage(FZCPU_RQ1, 1, [&] { rq1(s, *R, 100); });
    stage(FZCPU_RQ2_COUNT, 2, [&] { rq2_count(s, *R); });
    stage(FZCPU_RQ2_ADD, 3, [&] { rq2_add(s, *R); });
    stage(FZCPU_RQ3, 4, [&] { rq3(s, *R); });
    stage(FZCPU_RQ4A, 5, [&] { rq4a(s, g, *R); });
    stage(FZCPU_RQ4B, 6, [&] { rq4b(s, g, *R); });
    if (seconds) std::memcpy(seconds, tm, sizeof tm);
    return R;
}

// Length of output `name` and *data its values (-1: no such output of that type).
int64_t fzcpu_get_f64(void *h, const char *name, const double **data) {
    auto &m = static_cast<Result *>(h)->f;
    auto it = m.find(name);
    if (it == m.end()) return -1;
    *data = it->second.data();
    return int64_t(it->second.size());
}

int64_t fzcpu_get_i64(void *h, const char *name, const int64_t **data) {
    auto &m = static_cast<Result *>(h)->i;
    auto it = m.find(name);
    if (it == m.end()) return -1;
    *data = it->second.data();
    return int64_t(it->second.size());
}

void fzcpu_free(void *h) { delete static_cast<Result *>(h); }

int fzcpu_max_threads(void) { return omp_get_max_threads(); }

int64_t fzcpu_limit_us(int which) { return which == 0 ? LIMIT_US : RQ3_LIMIT_US; }

}  // extern "C"
