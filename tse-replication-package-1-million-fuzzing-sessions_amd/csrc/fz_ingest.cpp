// Native bulk ingest of the reference's plain-format dump: the
// `COPY <table> (<columns>) FROM stdin;` blocks of data/database/backup_clean.sql (README.md:14-15)
// parsed straight into typed columns - the replacement for restoring the dump into PostgreSQL and
// fetching rows through psycopg2 (program/__module/dbFile.py:16-24).
//
// One pass over the memory-mapped file finds the four tables' blocks; each block is cut into
// line-aligned slices parsed by worker threads (PostgreSQL text COPY format: tab-separated fields,
// \N = NULL, backslash escapes) into per-thread columns and first-occurrence dictionaries, which are
// then merged in slice order - so every dictionary (modules / revisions pools, build_type /
// result / status vocabularies) keeps the first-occurrence order of the whole column, exactly as
// the pandas path (store._from_frames) builds it, and project ids follow byte order.  Timestamps
// are parsed as the printed wall-clock time (a trailing UTC offset dropped, as store._ts does);
// any cell the native parser does not recognise is reported so the caller re-parses those cells.
//
// Host code only (g++, no GPU): libfzingest.so, C ABI in include/fz_ingest.h.
#include "fz_ingest.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr int64_t kTsNull = INT64_MAX;
constexpr uint8_t kCodeNull = 255;

thread_local std::string g_err;

// ---- field decoding ----------------------------------------------------------------------------
bool is_null(std::string_view f) { return f.size() == 2 && f[0] == '\\' && f[1] == 'N'; }

// PostgreSQL text COPY escapes (\b \f \n \r \t \v, octal \NNN, hex \xHH, anything else literal)
std::string unescape(std::string_view f) {
    std::string out;
    out.reserve(f.size());
    for (size_t i = 0; i < f.size(); ++i) {
        char c = f[i];
        if (c != '\\' || i + 1 >= f.size()) {
            out.push_back(c);
            continue;
        }
        char e = f[++i];
        switch (e) {
            case 'b': out.push_back('\b'); break;
            case 'f': out.push_back('\f'); break;
            case 'n': out.push_back('\n'); break;
            case 'r': out.push_back('\r'); break;
            case 't': out.push_back('\t'); break;
            case 'v': out.push_back('\v'); break;
            case 'x': {
                int v = 0, k = 0;
                while (k < 2 && i + 1 < f.size() && isxdigit((unsigned char)f[i + 1])) {
                    char h = f[++i];
                    v = v * 16 + (isdigit((unsigned char)h) ? h - '0' : (tolower(h) - 'a' + 10));
                    ++k;
                }
                if (k == 0) out.push_back('x');
                else out.push_back(char(v));
                break;
            }
            default:
                if (e >= '0' && e <= '7') {
                    int v = e - '0', k = 1;
                    while (k < 3 && i + 1 < f.size() && f[i + 1] >= '0' && f[i + 1] <= '7') {
                        v = v * 8 + (f[++i] - '0');
                        ++k;
                    }
                    out.push_back(char(v & 0xFF));
                } else {
                    out.push_back(e);
                }
        }
    }
    return out;
}

// days since 1970-01-01 of a proleptic Gregorian date
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = unsigned(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + int64_t(doe) - 719468;
}

bool digits(std::string_view s, size_t p, size_t n, int64_t &v) {
    if (p + n > s.size()) return false;
    v = 0;
    for (size_t k = 0; k < n; ++k) {
        const char c = s[p + k];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (c - '0');
    }
    return true;
}

// 'YYYY-MM-DD[( |T)HH:MM[:SS[.f{1,9}]]][(+|-)HH[[:]MM]]' -> microseconds of the printed time
bool parse_ts(std::string_view s, int64_t &us) {
    int64_t y, mo, d, h = 0, mi = 0, se = 0, frac = 0;
    if (!digits(s, 0, 4, y) || s.size() < 10 || s[4] != '-' || !digits(s, 5, 2, mo) || s[7] != '-' ||
        !digits(s, 8, 2, d))
        return false;
    if (mo < 1 || mo > 12 || d < 1 || d > 31) return false;
    size_t p = 10;
    if (p < s.size()) {
        if (s[p] != ' ' && s[p] != 'T') return false;
        ++p;
        if (!digits(s, p, 2, h) || p + 2 >= s.size() || s[p + 2] != ':' || !digits(s, p + 3, 2, mi)) return false;
        p += 5;
        if (p < s.size() && s[p] == ':') {
            if (!digits(s, p + 1, 2, se)) return false;
            p += 3;
            if (p < s.size() && s[p] == '.') {
                size_t q = p + 1;
                int n = 0;
                while (q < s.size() && s[q] >= '0' && s[q] <= '9') {
                    if (n < 6) frac = frac * 10 + (s[q] - '0');
                    ++n;
                    ++q;
                }
                if (n == 0 || n > 9) return false;
                for (int k = n; k < 6; ++k) frac *= 10;
                p = q;
            }
        }
        if (p < s.size()) {  // a UTC offset: dropped (the printed wall-clock time is kept)
            if (s[p] != '+' && s[p] != '-') return false;
            int64_t oh, om;
            if (!digits(s, p + 1, 2, oh)) return false;
            size_t q = p + 3;
            if (q < s.size()) {
                if (s[q] == ':') ++q;
                if (!digits(s, q, 2, om) || q + 2 != s.size()) return false;
            }
        }
        if (h > 23 || mi > 59 || se > 59) return false;
    }
    us = ((days_from_civil(y, unsigned(mo), unsigned(d)) * 86400 + h * 3600 + mi * 60 + se) * 1000000) + frac;
    return true;
}

bool parse_i64(std::string_view s, int64_t &v) {
    if (s.empty() || s.size() > 24) return false;
    char buf[32];
    memcpy(buf, s.data(), s.size());
    buf[s.size()] = 0;
    char *end = nullptr;
    errno = 0;
    const long long x = strtoll(buf, &end, 10);
    if (errno || end != buf + s.size()) return false;
    v = x;
    return true;
}

bool parse_f64(std::string_view s, double &v) {
    if (s.empty() || s.size() > 64) return false;
    for (char ch : s)  // hex floats: strtod reads them, Python's float() does not
        if (ch == 'x' || ch == 'X') return false;
    char buf[72];
    memcpy(buf, s.data(), s.size());
    buf[s.size()] = 0;
    char *end = nullptr;
    v = strtod(buf, &end);  // glibc: correctly rounded, like Python float()
    return end == buf + s.size();
}

// ---- dictionaries in first-occurrence order ---------------------------------------------------
// Keys are views into the mapped dump (or into `owned` for the rare escaped field), so a lookup
// allocates nothing; an entry's string is materialised once, on first occurrence.
struct Dict {
    std::vector<std::string> items;
    std::unordered_map<std::string_view, int32_t> index;
    std::deque<std::string> owned;
    int32_t id_view(std::string_view v) {
        auto it = index.find(v);
        if (it != index.end()) return it->second;
        const int32_t k = int32_t(items.size());
        items.emplace_back(v);
        index.emplace(v, k);
        return k;
    }
    int32_t id_field(std::string_view f) {  // a COPY field (escapes decoded)
        if (f.find('\\') == std::string_view::npos) return id_view(f);
        std::string s = unescape(f);  // looked up first: a repeated escaped value keeps no copy
        auto it = index.find(std::string_view(s));
        if (it != index.end()) return it->second;
        owned.push_back(std::move(s));
        return id_view(owned.back());
    }
    int32_t id(const std::string &s) {  // owned key (the merge step)
        auto it = index.find(std::string_view(s));
        if (it != index.end()) return it->second;
        owned.push_back(s);
        const int32_t k = int32_t(items.size());
        items.push_back(s);
        index.emplace(std::string_view(owned.back()), k);
        return k;
    }
};

struct Slice {  // one thread's rows of one block
    std::string_view text;
    int64_t rows = 0;
};

// ---- per-table column sets ------------------------------------------------------------------
struct Cols {
    // all tables: project (local dictionary ids, remapped after the merge)
    std::vector<int32_t> project;
    Dict projects;
    // buildlog_data
    std::vector<int32_t> b_type, b_result, b_modules, b_revisions;  // local dict ids / -1
    std::vector<int64_t> b_time;
    Dict d_type, d_result, d_modules, d_revisions;
    std::string names;                // name text back to back
    std::vector<int64_t> name_off;    // [rows + 1]
    std::vector<uint8_t> name_null;
    // total_coverage
    std::vector<int64_t> c_date, c_covered, c_total;
    std::vector<double> c_coverage;
    std::vector<uint8_t> c_cov_ok, c_covered_ok, c_total_ok;
    // issues
    std::vector<int64_t> i_number, i_rts, i_new_id;
    std::vector<int32_t> i_status;
    Dict d_status;
    // project_info
    std::vector<int64_t> pi_first;
    // cells the native parser did not recognise: (column code, row)
    std::vector<std::pair<int, int64_t>> bad;
    std::string error;
};

enum Table { T_BUILD = 0, T_COV, T_ISSUES, T_PI, T_N };
const char *kTableNames[T_N] = {"buildlog_data", "total_coverage", "issues", "project_info"};

struct Layout {  // field position of each needed column in a block's column list (-1: absent)
    int f[8];
    int nf;
};

enum BadCol { BAD_B_TIME = 0, BAD_C_DATE, BAD_C_COVERAGE, BAD_C_COVERED, BAD_C_TOTAL, BAD_I_NUMBER, BAD_I_RTS,
              BAD_I_NEW_ID, BAD_PI_FIRST };

void parse_slice(Table tab, const Layout &L, std::string_view text, Cols &c) {
    std::vector<std::string_view> fld(size_t(L.nf));
    int64_t row = 0;
    size_t p = 0;
    while (p < text.size()) {
        size_t e = text.find('\n', p);
        if (e == std::string_view::npos) e = text.size();
        std::string_view line = text.substr(p, e - p);
        p = e + 1;
        size_t q = 0;
        int k = 0;
        for (; k < L.nf; ++k) {
            size_t t = line.find('\t', q);
            if (t == std::string_view::npos) t = line.size();
            fld[size_t(k)] = line.substr(q, t - q);
            q = t + 1;
            if (t == line.size()) {
                ++k;
                break;
            }
        }
        if (k != L.nf || q <= line.size()) {
            c.error = std::string(kTableNames[tab]) + ": a row with " + std::to_string(k) + " fields, expected " +
                      std::to_string(L.nf);
            return;
        }
        auto F = [&](int which) { return fld[size_t(L.f[which])]; };
        const std::string_view pj = F(0);
        c.project.push_back(is_null(pj) ? -1 : c.projects.id_field(pj));
        int64_t v;
        double dv;
        switch (tab) {
            case T_BUILD: {
                auto code = [&](Dict &d, std::string_view s) { return is_null(s) ? -1 : d.id_field(s); };
                c.b_type.push_back(code(c.d_type, F(1)));
                c.b_result.push_back(code(c.d_result, F(2)));
                const std::string_view ts = F(3);
                if (is_null(ts)) c.b_time.push_back(kTsNull);
                else if (parse_ts(ts, v)) c.b_time.push_back(v);
                else {
                    c.b_time.push_back(kTsNull);
                    c.bad.push_back({BAD_B_TIME, row});
                }
                c.b_modules.push_back(code(c.d_modules, F(4)));
                c.b_revisions.push_back(code(c.d_revisions, F(5)));
                const std::string_view nm = F(6);
                if (c.name_off.empty()) c.name_off.push_back(0);
                if (is_null(nm)) {
                    c.name_null.push_back(1);
                } else {
                    c.name_null.push_back(0);
                    if (nm.find('\\') == std::string_view::npos) c.names.append(nm.data(), nm.size());
                    else c.names += unescape(nm);
                }
                c.name_off.push_back(int64_t(c.names.size()));
                break;
            }
            case T_COV: {
                const std::string_view ts = F(1);
                if (is_null(ts)) c.c_date.push_back(kTsNull);
                else if (parse_ts(ts, v)) c.c_date.push_back(v);
                else {
                    c.c_date.push_back(kTsNull);
                    c.bad.push_back({BAD_C_DATE, row});
                }
                const std::string_view cv = F(2);
                if (is_null(cv)) {
                    c.c_coverage.push_back(0.0);
                    c.c_cov_ok.push_back(0);
                } else if (parse_f64(cv, dv)) {
                    c.c_coverage.push_back(dv);
                    c.c_cov_ok.push_back(1);
                } else {
                    c.c_coverage.push_back(0.0);
                    c.c_cov_ok.push_back(0);
                    c.bad.push_back({BAD_C_COVERAGE, row});
                }
                for (int j = 0; j < 2; ++j) {
                    const std::string_view s = F(3 + j);
                    auto &col = j == 0 ? c.c_covered : c.c_total;
                    auto &ok = j == 0 ? c.c_covered_ok : c.c_total_ok;
                    if (is_null(s)) {
                        col.push_back(0);
                        ok.push_back(0);
                    } else if (parse_i64(s, v)) {
                        col.push_back(v);
                        ok.push_back(1);
                    } else {
                        col.push_back(0);
                        ok.push_back(0);
                        c.bad.push_back({j == 0 ? BAD_C_COVERED : BAD_C_TOTAL, row});
                    }
                }
                break;
            }
            case T_ISSUES: {
                const std::string_view num = F(1);
                if (!is_null(num) && parse_i64(num, v)) c.i_number.push_back(v);
                else {
                    c.i_number.push_back(0);
                    c.bad.push_back({BAD_I_NUMBER, row});
                }
                const std::string_view ts = F(2);
                if (is_null(ts)) c.i_rts.push_back(kTsNull);
                else if (parse_ts(ts, v)) c.i_rts.push_back(v);
                else {
                    c.i_rts.push_back(kTsNull);
                    c.bad.push_back({BAD_I_RTS, row});
                }
                c.i_status.push_back(is_null(F(3)) ? -1 : c.d_status.id_field(F(3)));
                if (L.f[4] >= 0) {
                    const std::string_view ni = F(4);
                    if (is_null(ni)) c.i_new_id.push_back(0);
                    else if (parse_i64(ni, v)) c.i_new_id.push_back(v);
                    else {
                        c.i_new_id.push_back(0);
                        c.bad.push_back({BAD_I_NEW_ID, row});
                    }
                } else {
                    c.i_new_id.push_back(0);
                }
                break;
            }
            case T_PI: {
                const std::string_view ts = F(1);
                if (is_null(ts)) c.pi_first.push_back(kTsNull);
                else if (parse_ts(ts, v)) c.pi_first.push_back(v);
                else {
                    c.pi_first.push_back(kTsNull);
                    c.bad.push_back({BAD_PI_FIRST, row});
                }
                break;
            }
            default: break;
        }
        ++row;
    }
}

}  // namespace

// ---- the result handle ------------------------------------------------------------------------
struct fz_ingest {
    std::vector<std::string> projects;          // byte order
    std::vector<std::string> vocab[5];          // build_type, result, modules, revisions, status
    int64_t n[T_N] = {0, 0, 0, 0};
    bool has[T_N] = {false, false, false, false};
    bool has_new_id = false;
    std::vector<uint32_t> proj[T_N];
    std::vector<uint8_t> b_type, b_result;
    std::vector<int32_t> b_modules, b_revisions;
    std::vector<int64_t> b_time;
    std::string names;
    std::vector<int64_t> name_off;
    std::vector<uint8_t> name_null;
    std::vector<int64_t> c_date, c_covered, c_total;
    std::vector<double> c_coverage;
    std::vector<uint8_t> c_cov_ok, c_covered_ok, c_total_ok;
    std::vector<int64_t> i_number, i_rts, i_new_id;
    std::vector<uint8_t> i_status;
    std::vector<int64_t> pi_first;
    std::vector<int64_t> bad;  // (column code, row) pairs, flattened
};

namespace {

// the COPY header: table name (schema-qualified or not, quoted or not) and its column list
bool parse_copy_header(std::string_view line, std::string &table, std::vector<std::string> &cols) {
    if (line.substr(0, 5) != "COPY ") return false;
    size_t p = 5;
    while (p < line.size() && line[p] == ' ') ++p;
    size_t open = line.find('(', p);
    if (open == std::string_view::npos) return false;
    std::string name(line.substr(p, open - p));
    while (!name.empty() && name.back() == ' ') name.pop_back();
    const size_t dot = name.rfind('.');
    if (dot != std::string::npos) name = name.substr(dot + 1);
    name.erase(std::remove(name.begin(), name.end(), '"'), name.end());
    const size_t close = line.find(')', open);
    if (close == std::string_view::npos) return false;
    std::string_view rest = line.substr(close + 1);
    if (rest.find("FROM stdin;") == std::string_view::npos) return false;
    cols.clear();
    std::string_view list = line.substr(open + 1, close - open - 1);
    size_t q = 0;
    while (q <= list.size()) {
        size_t c = list.find(',', q);
        if (c == std::string_view::npos) c = list.size();
        std::string col(list.substr(q, c - q));
        col.erase(std::remove(col.begin(), col.end(), '"'), col.end());
        col.erase(0, col.find_first_not_of(' '));
        col.erase(col.find_last_not_of(' ') + 1);
        cols.push_back(col);
        q = c + 1;
    }
    table = name;
    return true;
}

int col_index(const std::vector<std::string> &cols, const char *name) {
    for (size_t i = 0; i < cols.size(); ++i)
        if (cols[i] == name) return int(i);
    return -1;
}

void ingest(const char *data, size_t size, int threads, fz_ingest *out) {
    std::string_view all(data, size);
    struct Block {
        Table tab;
        Layout lay;
        std::string_view body;
    };
    std::vector<Block> blocks;
    size_t p = 0;
    for (;;) {  // the next line starting with "COPY " (memmem over the whole dump: no per-line loop)
        size_t at;
        if (p == 0 && all.substr(0, 5) == "COPY ") {
            at = 0;
        } else {
            const void *hit = memmem(all.data() + p, all.size() - p, "\nCOPY ", 6);
            if (!hit) break;
            at = size_t(static_cast<const char *>(hit) - all.data()) + 1;
        }
        size_t e = all.find('\n', at);
        if (e == std::string_view::npos) e = all.size();
        std::string_view line = all.substr(at, e - at);
        p = e;
        std::string table;
        std::vector<std::string> cols;
        if (!parse_copy_header(line, table, cols)) continue;
        // the block ends at a "\." line
        const size_t body_start = e + 1;
        size_t q;
        if (all.substr(body_start, 3) == "\\.\n" || all.substr(body_start) == "\\.") {
            q = body_start;
        } else {
            const void *hit = memmem(all.data() + body_start, all.size() - body_start, "\n\\.", 3);
            for (;;) {
                if (!hit) throw std::runtime_error("COPY " + table + " block not terminated by \\.");
                const size_t h = size_t(static_cast<const char *>(hit) - all.data());
                if (h + 3 == all.size() || all[h + 3] == '\n') {
                    q = h + 1;
                    break;
                }
                hit = memmem(all.data() + h + 1, all.size() - h - 1, "\n\\.", 3);
            }
        }
        p = q + 2 < all.size() ? q + 2 : all.size();
        int tab = -1;
        for (int t = 0; t < T_N; ++t)
            if (table == kTableNames[t]) tab = t;
        if (tab < 0) continue;
        Layout L{};
        for (int &x : L.f) x = -1;
        L.nf = int(cols.size());
        auto need = [&](int slot, const char *name, bool required) {
            L.f[slot] = col_index(cols, name);
            if (required && L.f[slot] < 0)
                throw std::runtime_error(std::string("COPY ") + kTableNames[tab] + ": no column " + name);
        };
        need(0, "project", true);
        if (tab == T_BUILD) {
            need(1, "build_type", true), need(2, "result", true), need(3, "timecreated", true);
            need(4, "modules", true), need(5, "revisions", true), need(6, "name", true);
        } else if (tab == T_COV) {
            need(1, "date", true), need(2, "coverage", true), need(3, "covered_line", true), need(4, "total_line", true);
        } else if (tab == T_ISSUES) {
            need(1, "number", true), need(2, "rts", true), need(3, "status", true), need(4, "new_id", false);
            out->has_new_id = L.f[4] >= 0;
        } else {
            need(1, "first_commit_datetime", true);
        }
        blocks.push_back({Table(tab), L, all.substr(body_start, q - body_start)});
        out->has[tab] = true;
    }
    for (int t = 0; t < 3; ++t)
        if (!out->has[t]) throw std::runtime_error(std::string("no COPY block for table '") + kTableNames[t] + "'");

    // parse: every block cut into line-aligned slices, one thread per slice
    struct Job {
        int block;
        std::string_view text;
        Cols cols;
    };
    std::vector<Job> jobs;
    for (size_t b = 0; b < blocks.size(); ++b) {
        const std::string_view body = blocks[b].body;
        const size_t per = std::max<size_t>(1 << 20, body.size() / size_t(threads) + 1);
        size_t s = 0;
        while (s < body.size()) {
            size_t e = std::min(body.size(), s + per);
            if (e < body.size()) {
                const size_t nl = body.find('\n', e);
                e = nl == std::string_view::npos ? body.size() : nl + 1;
            }
            jobs.push_back({int(b), body.substr(s, e - s), Cols()});
            s = e;
        }
    }
    {
        std::vector<std::thread> pool;
        std::atomic<size_t> next{0};
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([&] {
                for (size_t j; (j = next.fetch_add(1)) < jobs.size();) {
                    const Block &B = blocks[size_t(jobs[j].block)];
                    std::string_view text = jobs[j].text;
                    if (!text.empty() && text.back() == '\n') text.remove_suffix(1);
                    if (!text.empty()) parse_slice(B.tab, B.lay, text, jobs[j].cols);
                }
            });
        for (auto &th : pool) th.join();
    }
    for (auto &j : jobs)
        if (!j.cols.error.empty()) throw std::runtime_error(j.cols.error);

    // project ids: every name seen in any table, in byte order
    {
        std::unordered_map<std::string, int32_t> seen;
        for (auto &j : jobs)
            for (auto &s : j.cols.projects.items) seen.emplace(s, 0);
        out->projects.reserve(seen.size());
        for (auto &kv : seen) out->projects.push_back(kv.first);
        std::sort(out->projects.begin(), out->projects.end());  // std::string compares bytes (unsigned)
        for (size_t k = 0; k < out->projects.size(); ++k) seen[out->projects[k]] = int32_t(k);
        for (auto &j : jobs) {
            std::vector<int32_t> map(j.cols.projects.items.size());
            for (size_t k = 0; k < map.size(); ++k) map[k] = seen[j.cols.projects.items[k]];
            const Table tab = blocks[size_t(j.block)].tab;
            for (int32_t x : j.cols.project) {
                if (x < 0) throw std::runtime_error(std::string(kTableNames[tab]) + ": NULL project");
                out->proj[tab].push_back(uint32_t(map[size_t(x)]));
            }
        }
    }
    // vocabularies / pools in first-occurrence order of the whole column (slices in row order);
    // the code vocabularies start with the schema's fixed entries (schema.py)
    const std::vector<std::string> fixed[5] = {{"Fuzzing", "Coverage"}, {"Finish", "Halfway", "HalfWay", "Error"},
                                               {}, {}, {"Fixed", "Fixed (Verified)"}};
    Dict global[5];
    for (int d = 0; d < 5; ++d)
        for (auto &s : fixed[d]) global[d].id(s);
    auto remap = [&](int d, Dict &local, const std::vector<int32_t> &ids, auto push) {
        std::vector<int32_t> map(local.items.size());
        for (size_t k = 0; k < map.size(); ++k) map[k] = global[d].id(local.items[k]);
        for (int32_t x : ids) push(x < 0 ? -1 : map[size_t(x)]);
    };
    auto code8 = [](std::vector<uint8_t> &v) {
        return [&v](int32_t x) {
            if (x >= int32_t(kCodeNull)) throw std::runtime_error("more than 254 distinct codes");
            v.push_back(x < 0 ? kCodeNull : uint8_t(x));
        };
    };
    for (auto &j : jobs) {
        Cols &c = j.cols;
        const Table tab = blocks[size_t(j.block)].tab;
        const int64_t base = out->n[tab];
        for (auto &b : c.bad) {
            out->bad.push_back(b.first);
            out->bad.push_back(base + b.second);
        }
        const int64_t rows = int64_t(c.project.size());
        out->n[tab] += rows;
        if (tab == T_BUILD) {
            remap(0, c.d_type, c.b_type, code8(out->b_type));
            remap(1, c.d_result, c.b_result, code8(out->b_result));
            remap(2, c.d_modules, c.b_modules, [&](int32_t x) { out->b_modules.push_back(x); });
            remap(3, c.d_revisions, c.b_revisions, [&](int32_t x) { out->b_revisions.push_back(x); });
            out->b_time.insert(out->b_time.end(), c.b_time.begin(), c.b_time.end());
            const int64_t nb = int64_t(out->names.size());
            if (out->name_off.empty()) out->name_off.push_back(0);
            for (size_t k = 1; k < c.name_off.size(); ++k) out->name_off.push_back(nb + c.name_off[k]);
            out->names += c.names;
            out->name_null.insert(out->name_null.end(), c.name_null.begin(), c.name_null.end());
        } else if (tab == T_COV) {
            out->c_date.insert(out->c_date.end(), c.c_date.begin(), c.c_date.end());
            out->c_coverage.insert(out->c_coverage.end(), c.c_coverage.begin(), c.c_coverage.end());
            out->c_covered.insert(out->c_covered.end(), c.c_covered.begin(), c.c_covered.end());
            out->c_total.insert(out->c_total.end(), c.c_total.begin(), c.c_total.end());
            out->c_cov_ok.insert(out->c_cov_ok.end(), c.c_cov_ok.begin(), c.c_cov_ok.end());
            out->c_covered_ok.insert(out->c_covered_ok.end(), c.c_covered_ok.begin(), c.c_covered_ok.end());
            out->c_total_ok.insert(out->c_total_ok.end(), c.c_total_ok.begin(), c.c_total_ok.end());
        } else if (tab == T_ISSUES) {
            out->i_number.insert(out->i_number.end(), c.i_number.begin(), c.i_number.end());
            out->i_rts.insert(out->i_rts.end(), c.i_rts.begin(), c.i_rts.end());
            out->i_new_id.insert(out->i_new_id.end(), c.i_new_id.begin(), c.i_new_id.end());
            remap(4, c.d_status, c.i_status, code8(out->i_status));
        } else {
            out->pi_first.insert(out->pi_first.end(), c.pi_first.begin(), c.pi_first.end());
        }
        c = Cols();  // free the slice's columns as soon as they are merged
    }
    if (out->name_off.empty()) out->name_off.push_back(0);
    for (int d = 0; d < 5; ++d) out->vocab[d] = std::move(global[d].items);
}

}  // namespace

extern "C" {

const char *fz_ingest_last_error(void) { return g_err.c_str(); }

int fz_ingest_pg_dump(const char *path, int threads, fz_ingest **out) {
    try {
        *out = nullptr;
        const int fd = open(path, O_RDONLY);
        if (fd < 0) throw std::runtime_error(std::string("cannot open ") + path);
        struct stat st;
        fstat(fd, &st);
        const size_t size = size_t(st.st_size);
        void *m = size ? mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
        close(fd);
        if (size && m == MAP_FAILED) throw std::runtime_error("mmap failed");
        if (size) madvise(m, size, MADV_SEQUENTIAL);
        auto *h = new fz_ingest();
        try {
            ingest(static_cast<const char *>(m), size, threads > 0 ? threads : 1, h);
        } catch (...) {
            delete h;
            if (size) munmap(m, size);
            throw;
        }
        if (size) munmap(m, size);
        *out = h;
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

void fz_ingest_free(fz_ingest *h) { delete h; }

int64_t fz_ingest_rows(const fz_ingest *h, int table) { return table >= 0 && table < T_N ? h->n[table] : -1; }
int fz_ingest_has(const fz_ingest *h, int what) {
    if (what >= 0 && what < T_N) return h->has[what];
    return what == FZ_INGEST_HAS_NEW_ID ? h->has_new_id : 0;
}

// strings: a dictionary (projects = -1, vocabularies 0..4) or the build names (-2) as one blob
int64_t fz_ingest_strings(const fz_ingest *h, int which, char *blob, int64_t *offs) {
    if (which == -2) {
        if (blob) memcpy(blob, h->names.data(), h->names.size());
        if (offs) memcpy(offs, h->name_off.data(), h->name_off.size() * 8);
        return int64_t(h->names.size());
    }
    const std::vector<std::string> &v = which == -1 ? h->projects : h->vocab[which];
    int64_t total = 0;
    for (auto &s : v) {
        if (offs) offs[&s - v.data()] = total;
        if (blob) memcpy(blob + total, s.data(), s.size());
        total += int64_t(s.size());
    }
    if (offs) offs[v.size()] = total;
    return which == -1 || (which >= 0 && which < 5) ? total : -1;
}
int64_t fz_ingest_count(const fz_ingest *h, int which) {
    if (which == -1) return int64_t(h->projects.size());
    if (which >= 0 && which < 5) return int64_t(h->vocab[which].size());
    if (which == -3) return int64_t(h->bad.size() / 2);
    return -1;
}

int fz_ingest_column(const fz_ingest *h, int column, void *dst) {
    auto cp = [&](const auto &v) {
        memcpy(dst, v.data(), v.size() * sizeof(v[0]));
        return 0;
    };
    switch (column) {
        case FZ_COL_B_PROJECT: return cp(h->proj[T_BUILD]);
        case FZ_COL_B_TYPE: return cp(h->b_type);
        case FZ_COL_B_RESULT: return cp(h->b_result);
        case FZ_COL_B_TIME: return cp(h->b_time);
        case FZ_COL_B_MODULES: return cp(h->b_modules);
        case FZ_COL_B_REVISIONS: return cp(h->b_revisions);
        case FZ_COL_B_NAME_NULL: return cp(h->name_null);
        case FZ_COL_C_PROJECT: return cp(h->proj[T_COV]);
        case FZ_COL_C_DATE: return cp(h->c_date);
        case FZ_COL_C_COVERAGE: return cp(h->c_coverage);
        case FZ_COL_C_COVERAGE_OK: return cp(h->c_cov_ok);
        case FZ_COL_C_COVERED: return cp(h->c_covered);
        case FZ_COL_C_COVERED_OK: return cp(h->c_covered_ok);
        case FZ_COL_C_TOTAL: return cp(h->c_total);
        case FZ_COL_C_TOTAL_OK: return cp(h->c_total_ok);
        case FZ_COL_I_NUMBER: return cp(h->i_number);
        case FZ_COL_I_PROJECT: return cp(h->proj[T_ISSUES]);
        case FZ_COL_I_RTS: return cp(h->i_rts);
        case FZ_COL_I_STATUS: return cp(h->i_status);
        case FZ_COL_I_NEW_ID: return cp(h->i_new_id);
        case FZ_COL_PI_PROJECT: return cp(h->proj[T_PI]);
        case FZ_COL_PI_FIRST: return cp(h->pi_first);
        case FZ_COL_BAD: return cp(h->bad);
        default: return -1;
    }
}

}  // extern "C"
