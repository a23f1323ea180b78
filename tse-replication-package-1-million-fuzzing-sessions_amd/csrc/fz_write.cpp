// libfzwrite (include/fz_write.h): byte-exact csv.writer output of the RQ result tables, host code.
#include "fz_write.h"

#include <charconv>
#include <cmath>
#include <cstring>
#include <string>
#include <memory>
#include <thread>
#include <vector>

namespace {

// repr(float): CPython format_float_short(x, 'r', 0, Py_DTSF_ADD_DOT_0) over the shortest
// round-trip digits (std::to_chars scientific gives them as d[.ddd]e<exp>)
int repr_double(double v, char *out) {
    char *p = out;
    if (std::isnan(v)) {
        std::memcpy(p, "nan", 3);
        return 3;
    }
    if (std::signbit(v)) *p++ = '-';
    if (std::isinf(v)) {
        std::memcpy(p, "inf", 3);
        return int(p - out) + 3;
    }
    if (v == 0.0) {
        std::memcpy(p, "0.0", 3);
        return int(p - out) + 3;
    }
    char buf[48];
    const auto r = std::to_chars(buf, buf + sizeof(buf), std::fabs(v), std::chars_format::scientific);
    // buf: d[.ddd]e(+|-)XX
    char dig[32];
    int nd = 0;
    const char *q = buf;
    for (; q < r.ptr && *q != 'e'; ++q)
        if (*q != '.') dig[nd++] = *q;
    int exp10 = 0;
    std::from_chars(q + 1 + (q[1] == '+'), r.ptr, exp10);
    const int decpt = exp10 + 1;  // value = 0.d1d2...dn x 10^decpt
    if (decpt <= -4 || decpt > 16) {
        *p++ = dig[0];
        if (nd > 1) {
            *p++ = '.';
            std::memcpy(p, dig + 1, nd - 1);
            p += nd - 1;
        }
        *p++ = 'e';
        int e = decpt - 1;
        *p++ = e < 0 ? '-' : '+';
        if (e < 0) e = -e;
        if (e < 10) *p++ = '0';
        p = std::to_chars(p, p + 8, e).ptr;
        return int(p - out);
    }
    if (decpt <= 0) {
        *p++ = '0';
        *p++ = '.';
        for (int i = 0; i < -decpt; ++i) *p++ = '0';
        std::memcpy(p, dig, nd);
        p += nd;
    } else if (decpt >= nd) {
        std::memcpy(p, dig, nd);
        p += nd;
        for (int i = 0; i < decpt - nd; ++i) *p++ = '0';
        *p++ = '.';
        *p++ = '0';
    } else {
        std::memcpy(p, dig, decpt);
        p += decpt;
        *p++ = '.';
        std::memcpy(p, dig + decpt, nd - decpt);
        p += nd - decpt;
    }
    return int(p - out);
}

// str(datetime) of naive microseconds since 1970-01-01: 'YYYY-MM-DD HH:MM:SS[.ffffff]'
// (days -> civil date: H. Hinnant's days_from_civil inverse)
char *put_datetime(char *p, int64_t us) {
    constexpr int64_t kDay = 86400000000LL;
    int64_t days = us / kDay, rem = us % kDay;
    if (rem < 0) {
        rem += kDay;
        --days;
    }
    const int64_t z = days + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int64_t d = doy - (153 * mp + 2) / 5 + 1;
    const int64_t m = mp < 10 ? mp + 3 : mp - 9;
    if (m <= 2) ++y;
    auto two = [&](int64_t x) {
        *p++ = char('0' + x / 10);
        *p++ = char('0' + x % 10);
    };
    const int64_t yy = y;
    *p++ = char('0' + (yy / 1000) % 10);
    *p++ = char('0' + (yy / 100) % 10);
    *p++ = char('0' + (yy / 10) % 10);
    *p++ = char('0' + yy % 10);
    *p++ = '-';
    two(m);
    *p++ = '-';
    two(d);
    *p++ = ' ';
    const int64_t secs = rem / 1000000, frac = rem % 1000000;
    two(secs / 3600);
    *p++ = ':';
    two((secs / 60) % 60);
    *p++ = ':';
    two(secs % 60);
    if (frac) {
        *p++ = '.';
        int64_t f = frac;
        char t[6];
        for (int i = 5; i >= 0; --i) {
            t[i] = char('0' + f % 10);
            f /= 10;
        }
        std::memcpy(p, t, 6);
        p += 6;
    }
    return p;
}

// one csv.writer field (QUOTE_MINIMAL: quoted when it holds ',', '"', '\r' or '\n'; quotes doubled)
char *put_field(char *p, const char *s, int64_t n) {
    bool q = false;
    for (int64_t i = 0; i < n && !q; ++i) q = s[i] == ',' || s[i] == '"' || s[i] == '\r' || s[i] == '\n';
    if (!q) {
        std::memcpy(p, s, size_t(n));
        return p + n;
    }
    *p++ = '"';
    for (int64_t i = 0; i < n; ++i) {
        if (s[i] == '"') *p++ = '"';
        *p++ = s[i];
    }
    *p++ = '"';
    return p;
}

char *put_pool(char *p, const char *blob, const int64_t *off, int64_t id) {
    if (id < 0) return p;  // None -> ''
    return put_field(p, blob + off[id], off[id + 1] - off[id]);
}

char *put_i64(char *p, int64_t v) { return std::to_chars(p, p + 24, v).ptr; }

// rows [r0, r1) formatted by fmt(row, char *p) -> end.  Each worker formats its row range into a
// chain of 1 MiB blocks (a new block when the next row's bound does not fit), so its scratch is the
// exact output plus at most one row bound per block - not a worst-case-sized, zero-filled string -
// and the blocks are then copied to `out` at the workers' prefix-summed offsets
template <typename Bound, typename Fmt>
int64_t parallel_rows(int64_t n, int nthreads, char *out, int64_t cap, int64_t *row_end, Bound bound, Fmt fmt) {
    if (nthreads < 1) nthreads = 1;
    if (n < 4096) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    constexpr int64_t kBlock = int64_t(1) << 20;
    struct Block {
        std::unique_ptr<char[]> buf;
        int64_t used = 0, cap = 0;
    };
    std::vector<std::vector<Block>> parts(static_cast<size_t>(nthreads));
    std::vector<int64_t> sizes(static_cast<size_t>(nthreads), 0);
    std::vector<std::thread> th;
    auto work = [&](int w) {
        const int64_t r0 = n * w / nthreads, r1 = n * (w + 1) / nthreads;
        std::vector<Block> &bl = parts[size_t(w)];
        int64_t done = 0;  // bytes of the finished blocks
        for (int64_t r = r0; r < r1; ++r) {
            const int64_t b = bound(r);
            if (bl.empty() || bl.back().used + b > bl.back().cap) {
                if (!bl.empty()) done += bl.back().used;
                Block nb;
                nb.cap = b > kBlock ? b : kBlock;
                nb.buf.reset(new char[size_t(nb.cap)]);
                bl.push_back(std::move(nb));
            }
            Block &k = bl.back();
            char *p = fmt(r, k.buf.get() + k.used);
            k.used = int64_t(p - k.buf.get());
            if (row_end) row_end[r] = done + k.used;  // (local; shifted below)
        }
        sizes[size_t(w)] = done + (bl.empty() ? 0 : bl.back().used);
    };
    for (int w = 1; w < nthreads; ++w) th.emplace_back(work, w);
    work(0);
    for (auto &t : th) t.join();
    int64_t total = 0;
    for (int64_t v : sizes) total += v;
    if (total > cap) return -1;
    int64_t o = 0;
    for (int w = 0; w < nthreads; ++w) {
        int64_t q = o;
        for (const Block &k : parts[size_t(w)]) {
            std::memcpy(out + q, k.buf.get(), size_t(k.used));
            q += k.used;
        }
        if (row_end && o) {
            const int64_t r0 = n * w / nthreads, r1 = n * (w + 1) / nthreads;
            for (int64_t r = r0; r < r1; ++r) row_end[r] += o;
        }
        parts[size_t(w)].clear();
        o += sizes[size_t(w)];
    }
    return total;
}

constexpr int64_t kMaxRepr = 26;  // "-1.2345678901234567e-308," and the like

}  // namespace

extern "C" {

int fzw_repr(double v, char *out) { return repr_double(v, out); }

int64_t fzw_float_rows_cap(const int64_t *offs, int64_t nrows) {
    return nrows > 0 ? (offs[nrows] - offs[0]) * kMaxRepr + 2 * nrows : 0;
}

int64_t fzw_float_rows(const double *vals, const int64_t *offs, int64_t nrows, char *out, int64_t cap, int nthreads) {
    return parallel_rows(
        nrows, nthreads, out, cap, nullptr, [&](int64_t r) { return (offs[r + 1] - offs[r]) * kMaxRepr + 2; },
        [&](int64_t r, char *p) {
            for (int64_t i = offs[r]; i < offs[r + 1]; ++i) {
                if (i > offs[r]) *p++ = ',';
                p += repr_double(vals[i], p);
            }
            *p++ = '\r';
            *p++ = '\n';
            return p;
        });
}

static int64_t change_row_bound(const fzw_change_cols *c, int64_t r) {
    auto plen = [](const int64_t *off, int64_t id) { return id < 0 ? 0 : 2 * (off[id + 1] - off[id]) + 2; };
    return plen(c->proj_off, c->project[r]) + plen(c->mod_off, c->mod_f[r]) + plen(c->rev_off, c->rev_f[r]) +
           plen(c->mod_off, c->mod_s[r]) + plen(c->rev_off, c->rev_s[r]) + 2 * 27 + 8 * kMaxRepr + 16;
}

int64_t fzw_change_rows_cap(const fzw_change_cols *c, int64_t n) {
    int64_t b = 0;
    for (int64_t r = 0; r < n; ++r) b += change_row_bound(c, r);
    return b;
}

int64_t fzw_change_rows(const fzw_change_cols *c, int64_t n, char *out, int64_t cap, int64_t *row_end, int nthreads) {
    return parallel_rows(
        n, nthreads, out, cap, row_end, [&](int64_t r) { return change_row_bound(c, r); },
        [&](int64_t r, char *p) {
            const int64_t proj = c->project[r];
            // covered / total cell of coverage row cr: nan when absent or NULL; float or int by the
            // project's pandas dtype
            auto cell = [&](int64_t cr, const int64_t *col, const uint8_t *valid, const uint8_t *isf) {
                if (cr < 0 || !valid[cr]) {
                    std::memcpy(p, "nan", 3);
                    p += 3;
                } else if (isf[proj]) {
                    p += repr_double(double(col[cr]), p);
                } else {
                    p = put_i64(p, col[cr]);
                }
                *p++ = ',';
            };
            p = put_pool(p, c->proj_blob, c->proj_off, proj);
            *p++ = ',';
            p = put_datetime(p, c->t_end[r]);
            *p++ = ',';
            p = put_pool(p, c->mod_blob, c->mod_off, c->mod_f[r]);
            *p++ = ',';
            p = put_pool(p, c->rev_blob, c->rev_off, c->rev_f[r]);
            *p++ = ',';
            p = put_datetime(p, c->t_start[r]);
            *p++ = ',';
            p = put_pool(p, c->mod_blob, c->mod_off, c->mod_s[r]);
            *p++ = ',';
            p = put_pool(p, c->rev_blob, c->rev_off, c->rev_s[r]);
            *p++ = ',';
            cell(c->cov_i[r], c->c_covered, c->c_covered_valid, c->covered_is_float);
            cell(c->cov_i[r], c->c_total, c->c_total_valid, c->total_is_float);
            cell(c->cov_i1[r], c->c_covered, c->c_covered_valid, c->covered_is_float);
            cell(c->cov_i1[r], c->c_total, c->c_total_valid, c->total_is_float);
            const double dt = c->diff_total[r];
            if (std::isnan(dt)) {
                std::memcpy(p, "nan", 3);
                p += 3;
            } else if (c->total_is_float[proj]) {
                p += repr_double(dt, p);
            } else {
                p = put_i64(p, int64_t(dt));
            }
            *p++ = ',';
            p += repr_double(c->diff_coverage[r], p);
            *p++ = '\r';
            *p++ = '\n';
            return p;
        });
}

}  // extern "C"
