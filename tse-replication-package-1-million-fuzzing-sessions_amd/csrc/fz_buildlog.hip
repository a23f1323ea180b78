// Build-log analysis: program/preparation/4_get_buildlog_analysis.py:14-246
// (buildlog_analysis) over a batch of Cloud Build logs held in HBM as UTF-8 text.
//
// Data-parallel restatement of the reference's per-log line loop (:82-214):
//   1. line starts  - str.splitlines() boundaries (\n \r \r\n \v \f \x1c \x1d \x1e U+0085 U+2028
//                     U+2029), per 4096-byte chunk of a log, written in order (chunk counts + scan);
//   2. classify     - one thread per line: the reference's patterns evaluated on the line alone ->
//                     a flag word (project capture, "Starting Step" skip / SET value, the PUSH DONE
//                     rule, jq / JSON-block markers, the tail tests of :228-237);
//   3. fold         - one wave per log: the first project capture, the last SET and the last PUSH
//                     DONE line give build_type (a SET line assigns; a PUSH DONE line maps every value
//                     but Coverage / Introspector to Fuzzing; both commute with nothing else), and
//                     the last 200 lines give result.
// The srcmap paths / revisions (jq_inplace lines and "Step #N: {" JSON blocks, :162-214) need a JSON
// parser: the lines that matter (skip, jq, open, close) are compacted for the host, which runs
// the block state machine on those lines only (tse_amd/buildlog.py).
// Regex semantics reproduced: '.' in gcr.io matches any one character, \s / strip() are Unicode
// whitespace, greedy groups of compile-(.*)-(.*)-x86_64; \d is taken as ASCII [0-9].
#include "fz_device.h"
#include "fz_internal.h"
#include "fz_views.h"

namespace fz {

enum : uint32_t {
    BL_IMAGE = 1u << 0,      // a project capture (image, or GCS when no image on the line)
    BL_SKIP = 1u << 2,       // "Starting Step" line that ends the line's processing (:104-105)
    BL_PUSHDONE = 1u << 3,   // PUSH\s*DONE (:150-152)
    BL_JQ = 1u << 8,         // jq_inplace [^ ]+ '...' (:163)
    BL_OPEN = 1u << 9,       // "Step #N: {" (a JSON block may start, :183-186)
    BL_CLOSE = 1u << 10,     // strip() ends with '}' (a JSON block ends, :196)
    BL_EQ_ERROR = 1u << 11,  // strip() == "ERROR"
    BL_EQ_PUSH = 1u << 12,
    BL_EQ_DONE = 1u << 13,
    BL_EQ_DEADLINE = 1u << 14,
    BL_HAS_ERROR = 1u << 15,  // "ERROR" in line
};
constexpr int kSetShift = 4;  // bits 4..7: the value the line SETs (0: none)
enum { BT_NONE = 0, BT_cov = 1, BT_intro = 2, BT_FUZZ = 3, BT_UNKNOWN = 4, BT_INTRO = 5, BT_COV = 6 };
enum { BR_NONE = 0, BR_ERROR = 1, BR_SUCCESS = 2, BR_UNKNOWN = 3 };

// ---- one line as bytes ------------------------------------------------------------------------
struct Line {
    const uint8_t *p;
    int n;
    __device__ int at(int k) const { return k < n ? int(p[k]) : -1; }
};

__device__ inline int utf8_len(int b) {
    return b < 0x80 ? 1 : (b & 0xE0) == 0xC0 ? 2 : (b & 0xF0) == 0xE0 ? 3 : (b & 0xF8) == 0xF0 ? 4 : 1;
}

// length of the Unicode whitespace character (str.isspace) starting at k, 0 if none
__device__ inline int ws_at(const Line &L, int k) {
    const int b = L.at(k);
    if (b < 0) return 0;
    if ((b >= 0x09 && b <= 0x0D) || (b >= 0x1C && b <= 0x20)) return 1;
    const int b1 = L.at(k + 1), b2 = L.at(k + 2);
    if (b == 0xC2 && (b1 == 0x85 || b1 == 0xA0)) return 2;
    if (b == 0xE1 && b1 == 0x9A && b2 == 0x80) return 3;
    if (b == 0xE2 && b1 == 0x80 && ((b2 >= 0x80 && b2 <= 0x8A) || b2 == 0xA8 || b2 == 0xA9 || b2 == 0xAF)) return 3;
    if (b == 0xE2 && b1 == 0x81 && b2 == 0x9F) return 3;
    if (b == 0xE3 && b1 == 0x80 && b2 == 0x80) return 3;
    return 0;
}
// length of the whitespace character ending at e (exclusive), 0 if none
__device__ inline int ws_before(const Line &L, int e) {
    if (e >= 1 && ws_at(L, e - 1) == 1) return 1;
    if (e >= 2 && ws_at(L, e - 2) == 2) return 2;
    if (e >= 3 && ws_at(L, e - 3) == 3) return 3;
    return 0;
}
// str.strip() of [b, e)
__device__ inline void strip(const Line &L, int &b, int &e) {
    int w;
    while (b < e && (w = ws_at(L, b)) > 0) b += w;
    while (e > b && (w = ws_before(L, e)) > 0) e -= w;
}

// Pattern bytes at position k: the end position, or -1.  '\x01' in pat = any one character.
__device__ inline int match_at(const Line &L, int k, const char *pat) {
    for (int j = 0; pat[j]; ++j) {
        const int b = L.at(k);
        if (b < 0) return -1;
        if (pat[j] == '\x01') {
            k += utf8_len(b);
            if (k > L.n) return -1;
        } else {
            if (b != (unsigned char)pat[j]) return -1;
            ++k;
        }
    }
    return k;
}
// first k >= from where pat matches (pat starts with an ASCII byte), -1 if none
__device__ inline int find(const Line &L, int from, const char *pat, int lim = -1) {
    const int end = lim < 0 ? L.n : lim;
    const int c0 = (unsigned char)pat[0];
    for (int k = from; k < end; ++k)
        if (L.p[k] == c0 && match_at(L, k, pat) >= 0) return k;
    return -1;
}
// the same on [b, e) with '"' bytes of the text ignored (text.replace('"', '') at :103)
__device__ inline bool contains_noquote(const Line &L, int b, int e, const char *pat) {
    for (int k = b; k < e; ++k) {
        if (L.p[k] == '"') continue;
        int q = k, j = 0;
        for (; pat[j]; ++j) {
            while (q < e && L.p[q] == '"') ++q;
            if (q >= e || L.p[q] != (unsigned char)pat[j]) break;
            ++q;
        }
        if (!pat[j]) return true;
    }
    return false;
}
__device__ inline bool equals(const Line &L, int b, int e, const char *pat) {
    int j = 0;
    for (; pat[j]; ++j)
        if (b + j >= e || L.p[b + j] != (unsigned char)pat[j]) return false;
    return b + j == e;
}
__device__ inline bool is_digit(int b) { return b >= '0' && b <= '9'; }
__device__ inline int digits(const Line &L, int k) {
    int n = 0;
    while (is_digit(L.at(k + n))) ++n;
    return n;
}

template <int N>
constexpr int plen(const char (&)[N]) {
    return N - 1;
}
constexpr char kImage[] = "Already have image: gcr.io/oss-fuzz/";
constexpr char kGcs[] = "No URLs matched: gs://oss-fuzz-coverage/";

// group(1) of IMAGE / GCS (:62-63, 84-98): the first occurrence that matches; cap = (off, len)
__device__ inline bool image_capture(const Line &L, int &off, int &len) {
    for (int k = find(L, 0, kImage); k >= 0; k = find(L, k + 1, kImage)) {
        const int s = k + plen(kImage);
        int e = s, w;
        while (e < L.n && L.p[e] != ':' && (w = ws_at(L, e)) == 0) e += utf8_len(L.p[e]);
        if (e > s) {
            off = s;
            len = e - s;
            return true;
        }
    }
    return false;
}
__device__ inline bool gcs_capture(const Line &L, int &off, int &len) {
    for (int k = find(L, 0, kGcs); k >= 0; k = find(L, k + 1, kGcs)) {
        const int s = k + plen(kGcs);
        int e = s;
        while (e < L.n && L.p[e] != '/') ++e;
        if (e > s && match_at(L, e, "/textcov_reports") >= 0) {
            off = s;
            len = e - s;
            return true;
        }
    }
    return false;
}

// value of group(2) of compile-(.*)-(.*)-x86_64 (:72, 140-149), -1 when no match
__device__ inline int compile_value(const Line &L) {
    const int s = find(L, 0, "compile-");
    if (s < 0) return -1;
    int qL = -1;  // last "-x86_64" at or after s + 9
    for (int q = find(L, s + 9, "-x86_64"); q >= 0; q = find(L, q + 1, "-x86_64")) qL = q;
    if (qL < 0) return -1;
    int p = -1;  // last '-' in [s + 8, qL - 1]
    for (int k = qL - 1; k >= s + 8; --k)
        if (L.p[k] == '-') {
            p = k;
            break;
        }
    if (p < 0) return -1;
    const int b = p + 1, e = qL;
    if (equals(L, b, e, "address") || equals(L, b, e, "memory") || equals(L, b, e, "undefined") ||
        equals(L, b, e, "none"))
        return BT_FUZZ;
    if (equals(L, b, e, "coverage")) return BT_COV;
    if (equals(L, b, e, "introspector")) return BT_INTRO;
    return BT_UNKNOWN;
}

__device__ inline uint32_t classify(const Line &L, int &cap_off, int &cap_len) {
    uint32_t f = 0;
    cap_off = -1;
    cap_len = 0;
    {
        int o, n;
        if (image_capture(L, o, n) || gcs_capture(L, o, n)) {
            f |= BL_IMAGE;
            cap_off = o;
            cap_len = n;
        }
    }
    int sb = 0, se = L.n;
    strip(L, sb, se);
    if (equals(L, sb, se, "ERROR")) f |= BL_EQ_ERROR;
    if (equals(L, sb, se, "PUSH")) f |= BL_EQ_PUSH;
    if (equals(L, sb, se, "DONE")) f |= BL_EQ_DONE;
    if (equals(L, sb, se, "ERROR: context deadline exceeded")) f |= BL_EQ_DEADLINE;
    if (find(L, 0, "ERROR") >= 0) f |= BL_HAS_ERROR;
    uint32_t set = BT_NONE;
    const int nd = match_at(L, 0, "Starting Step #") >= 0 ? digits(L, 15) : 0;
    if (nd > 0) {  // re.match(r"Starting Step #\d+\s*(.*)") (:101-118)
        int b = 15 + nd, e = L.n;
        strip(L, b, e);
        bool only_quotes = true;
        for (int k = b; k < e; ++k) only_quotes &= L.p[k] == '"';
        if (only_quotes || contains_noquote(L, b, e, "srcmap") || contains_noquote(L, b, e, "build"))
            return f | BL_SKIP;
        if (contains_noquote(L, b, e, "coverage"))
            set = BT_cov;
        else if (contains_noquote(L, b, e, "introspector"))
            set = BT_intro;
        else if (contains_noquote(L, b, e, "address-x86_64") || contains_noquote(L, b, e, "undefined-x86_64") ||
                 contains_noquote(L, b, e, "memory-x86_64") || contains_noquote(L, b, e, "none-x86_64") ||
                 contains_noquote(L, b, e, "address-i386"))
            set = BT_FUZZ;
        else
            set = BT_UNKNOWN;
    } else {  // :120-152 (the ERROR pattern '\nERROR.*' never matches a line)
        for (int k = find(L, 0, "Step #"); k >= 0; k = find(L, k + 1, "Step #")) {
            const int d = digits(L, k + 6);
            if (d > 0 && match_at(L, k + 6 + d, ": Pulling image: gcr\x01io/oss-fuzz-base/base-runner") >= 0) {
                set = (d == 1 && L.p[k + 6] == '0') ? BT_INTRO
                      : (d == 1 && L.p[k + 6] == '4') ? BT_COV
                      : (d == 1 && L.p[k + 6] == '5') ? BT_FUZZ
                                                       : BT_UNKNOWN;
                break;
            }
        }
        const int r = find(L, 0, "/report/");
        if (r >= 0 && find(L, r + 8, ".html") >= 0) set = BT_COV;
        if (find(L, 0, "Unable to find image 'gcr\x01io/oss-fuzz-base/base-runner:latest' locally") >= 0) set = BT_FUZZ;
        const int cv = compile_value(L);
        if (cv >= 0) set = uint32_t(cv);
        for (int k = find(L, 0, "PUSH"); k >= 0; k = find(L, k + 1, "PUSH")) {
            int q = k + 4, w;
            while ((w = ws_at(L, q)) > 0) q += w;
            if (match_at(L, q, "DONE") >= 0) {
                f |= BL_PUSHDONE;
                break;
            }
        }
    }
    f |= set << kSetShift;
    // jq_inplace [^ ]+ '(.*?)' (:64, 163)
    for (int k = find(L, 0, "jq_inplace "); k >= 0; k = find(L, k + 1, "jq_inplace ")) {
        const int x = k + 11;
        int y = x;
        while (y < L.n && L.p[y] != ' ') ++y;
        if (y > x && L.at(y + 1) == '\'' && find(L, y + 2, "'") >= 0) {
            f |= BL_JQ;
            break;
        }
    }
    // JSON block markers (:183-197): "Step #\d+:" then the rest stripped == "{"; strip() ends with '}'
    if (se > sb && L.p[se - 1] == '}') f |= BL_CLOSE;
    if (se > sb && L.p[se - 1] == '{') {
        for (int k = find(L, 0, "Step #"); k >= 0; k = find(L, k + 1, "Step #")) {
            const int d = digits(L, k + 6);
            if (d > 0 && L.at(k + 6 + d) == ':') {
                int b = k + 7 + d, e = L.n;
                strip(L, b, e);
                if (e == b + 1 && L.p[b] == '{') f |= BL_OPEN;
                break;
            }
        }
    }
    return f;
}

// The same classification in ONE scan of the line (the "Starting Step #N" lines - a few per log -
// keep the pattern-by-pattern code above): every pattern of :120-214 starts with one of eleven
// bytes, so a byte that is none of them (a constant 256-bit set, no memory) costs one test; at a
// trigger byte only that byte's patterns are matched, and what the reference's searches depend on
// is recorded as positions - the first image / GCS occurrence with a non-empty capture, the first
// "Step #N: Pulling image" and the first "Step #N:", the first "compile-" and the last "-x86_64",
// the first "/report/" and the last ".html", the earliest quote a jq_inplace candidate needs and
// the last quote - and folded after the scan exactly as the searches would (pattern-by-pattern:
// ~12 scans of every line).
__device__ inline bool trigger_byte(int b) {
    // 'A' 'N' 'E' 'S' '/' 'U' 'c' '-' 'P' 'j' '.' '\''
    constexpr uint64_t lo = (1ull << '/') | (1ull << '-') | (1ull << '.') | (1ull << '\'');
    constexpr uint64_t hi = (1ull << ('A' - 64)) | (1ull << ('N' - 64)) | (1ull << ('E' - 64)) | (1ull << ('S' - 64)) |
                            (1ull << ('U' - 64)) | (1ull << ('c' - 64)) | (1ull << ('P' - 64)) | (1ull << ('j' - 64));
    return b < 64 ? ((lo >> b) & 1ull) != 0 : (b < 128 && ((hi >> (b - 64)) & 1ull) != 0);
}

__device__ inline uint32_t classify1(const Line &L, int &cap_off, int &cap_len) {
    if (match_at(L, 0, "Starting Step #") >= 0 && digits(L, 15) > 0) return classify(L, cap_off, cap_len);
    const int n = L.n;
    int img_off = -1, img_len = 0, gcs_off = -1, gcs_len = 0;
    bool has_error = false, unable = false, pushdone = false;
    int pull_set = -1;         // set value of the first "Step #N: Pulling image: ...base-runner"
    int step_colon = -1;       // end of the first "Step #N:" (the JSON-open test)
    int first_compile = -1, last_x86 = -1, first_report = -1, last_html = -1;
    int jq_need = INT_MAX, last_quote = -1;  // a jq_inplace candidate needs a quote at >= jq_need
    for (int k = 0; k < n; ++k) {
        const int b = L.p[k];
        if (!trigger_byte(b)) continue;
        switch (b) {
        case 'A':
            if (img_off < 0 && match_at(L, k, kImage) >= 0) {
                const int st = k + plen(kImage);
                int e = st, w;
                while (e < n && L.p[e] != ':' && (w = ws_at(L, e)) == 0) e += utf8_len(L.p[e]);
                if (e > st) img_off = st, img_len = e - st;
            }
            break;
        case 'N':
            if (gcs_off < 0 && match_at(L, k, kGcs) >= 0) {
                const int st = k + plen(kGcs);
                int e = st;
                while (e < n && L.p[e] != '/') ++e;
                if (e > st && match_at(L, e, "/textcov_reports") >= 0) gcs_off = st, gcs_len = e - st;
            }
            break;
        case 'E':
            if (!has_error && match_at(L, k, "ERROR") >= 0) has_error = true;
            break;
        case 'S':
            if ((pull_set < 0 || step_colon < 0) && match_at(L, k, "Step #") >= 0) {
                const int d = digits(L, k + 6);
                if (d > 0) {
                    if (pull_set < 0 && match_at(L, k + 6 + d, ": Pulling image: gcr\x01io/oss-fuzz-base/base-runner") >= 0)
                        pull_set = (d == 1 && L.p[k + 6] == '0')   ? BT_INTRO
                                   : (d == 1 && L.p[k + 6] == '4') ? BT_COV
                                   : (d == 1 && L.p[k + 6] == '5') ? BT_FUZZ
                                                                    : BT_UNKNOWN;
                    if (step_colon < 0 && L.at(k + 6 + d) == ':') step_colon = k + 7 + d;
                }
            }
            break;
        case '/':
            if (first_report < 0 && match_at(L, k, "/report/") >= 0) first_report = k;
            break;
        case '.':
            if (match_at(L, k, ".html") >= 0) last_html = k;
            break;
        case 'U':
            if (!unable && match_at(L, k, "Unable to find image 'gcr\x01io/oss-fuzz-base/base-runner:latest' locally") >= 0)
                unable = true;
            break;
        case 'c':
            if (first_compile < 0 && match_at(L, k, "compile-") >= 0) first_compile = k;
            break;
        case '-':
            if (match_at(L, k, "-x86_64") >= 0) last_x86 = k;
            break;
        case 'P':
            if (!pushdone && match_at(L, k, "PUSH") >= 0) {
                int q = k + 4, w;
                while ((w = ws_at(L, q)) > 0) q += w;
                if (match_at(L, q, "DONE") >= 0) pushdone = true;
            }
            break;
        case 'j':
            if (match_at(L, k, "jq_inplace ") >= 0) {
                const int x = k + 11;
                int y = x;
                while (y < n && L.p[y] != ' ') ++y;
                if (y > x && L.at(y + 1) == '\'') jq_need = y + 2 < jq_need ? y + 2 : jq_need;
            }
            break;
        default:  // '\''
            last_quote = k;
            break;
        }
    }
    uint32_t f = 0;
    cap_off = -1;
    cap_len = 0;
    if (img_off >= 0) {
        f |= BL_IMAGE, cap_off = img_off, cap_len = img_len;
    } else if (gcs_off >= 0) {
        f |= BL_IMAGE, cap_off = gcs_off, cap_len = gcs_len;
    }
    int sb = 0, se = n;
    strip(L, sb, se);
    if (equals(L, sb, se, "ERROR")) f |= BL_EQ_ERROR;
    if (equals(L, sb, se, "PUSH")) f |= BL_EQ_PUSH;
    if (equals(L, sb, se, "DONE")) f |= BL_EQ_DONE;
    if (equals(L, sb, se, "ERROR: context deadline exceeded")) f |= BL_EQ_DEADLINE;
    if (has_error) f |= BL_HAS_ERROR;
    // :120-152 in the reference's order: each later test overrides the value
    uint32_t set = pull_set >= 0 ? uint32_t(pull_set) : BT_NONE;
    if (first_report >= 0 && last_html >= first_report + 8) set = BT_COV;
    if (unable) set = BT_FUZZ;
    if (first_compile >= 0 && last_x86 >= first_compile + 9) {  // compile_value: group(2) of the greedy match
        int p = -1;
        for (int k = last_x86 - 1; k >= first_compile + 8; --k)
            if (L.p[k] == '-') {
                p = k;
                break;
            }
        if (p >= 0) {
            const int b = p + 1, e = last_x86;
            set = (equals(L, b, e, "address") || equals(L, b, e, "memory") || equals(L, b, e, "undefined") ||
                   equals(L, b, e, "none"))
                      ? BT_FUZZ
                  : equals(L, b, e, "coverage")     ? BT_COV
                  : equals(L, b, e, "introspector") ? BT_INTRO
                                                    : BT_UNKNOWN;
        }
    }
    if (pushdone) f |= BL_PUSHDONE;
    f |= set << kSetShift;
    if (last_quote >= jq_need) f |= BL_JQ;
    if (se > sb && L.p[se - 1] == '}') f |= BL_CLOSE;
    if (se > sb && L.p[se - 1] == '{' && step_colon >= 0) {
        int b = step_colon, e = n;
        strip(L, b, e);
        if (e == b + 1 && L.p[b] == '{') f |= BL_OPEN;
    }
    return f;
}

// ---- 1. line starts -------------------------------------------------------------------------
// A byte chunk of one log (host-built list: every chunk lies inside one log).
struct LogChunks {
    const int32_t *log;
    const int64_t *begin, *end;
};
constexpr int kLineChunk = 4096;
constexpr int kLineItems = kLineChunk / kBlock;

__device__ inline bool is_break1(int b) { return b == 0x0A || b == 0x0B || b == 0x0C || b == 0x0D || (b >= 0x1C && b <= 0x1E); }
// does a line start at i (ls <= i < le)?
__device__ inline bool line_starts(const uint8_t *t, int64_t ls, int64_t i) {
    if (i == ls) return true;
    const int b1 = t[i - 1];
    if (b1 == 0x0A || b1 == 0x0B || b1 == 0x0C || (b1 >= 0x1C && b1 <= 0x1E)) return true;
    if (b1 == 0x0D) return t[i] != 0x0A;  // "\r\n" is one break
    if (i - 2 >= ls && t[i - 2] == 0xC2 && b1 == 0x85) return true;
    if (i - 3 >= ls && t[i - 3] == 0xE2 && t[i - 2] == 0x80 && (b1 == 0xA8 || b1 == 0xA9)) return true;
    return false;
}

__global__ __launch_bounds__(kBlock) void k_line_count(const uint8_t *__restrict__ t, const int64_t *__restrict__ log_offs,
                                                       LogChunks ch, int64_t nch, int64_t *__restrict__ cnt) {
    for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const int64_t ls = log_offs[ch.log[c]], b = ch.begin[c], e = ch.end[c];
        int64_t n = 0;
        for (int64_t i = b + threadIdx.x; i < e; i += kBlock) n += line_starts(t, ls, i);
        __shared__ int64_t s_tmp[4];
        n = block_sum(n, s_tmp);
        if (threadIdx.x == 0) cnt[c] = n;
    }
}

__global__ __launch_bounds__(kBlock) void k_line_write(const uint8_t *__restrict__ t, const int64_t *__restrict__ log_offs,
                                                       LogChunks ch, int64_t nch, const int64_t *__restrict__ off,
                                                       int64_t *__restrict__ line_start) {
    __shared__ int64_t s_tmp[4];
    for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const int64_t ls = log_offs[ch.log[c]], b = ch.begin[c], e = ch.end[c];
        // thread j owns the bytes [b + j * kLineItems, ...): order within the chunk by block scan
        const int64_t mb = b + int64_t(threadIdx.x) * kLineItems;
        int64_t n = 0;
        for (int k = 0; k < kLineItems; ++k) n += (mb + k < e) && line_starts(t, ls, mb + k);
        int64_t o = off[c] + block_excl_scan<int64_t>(n, s_tmp, (int64_t *)nullptr);
        for (int k = 0; k < kLineItems; ++k)
            if (mb + k < e && line_starts(t, ls, mb + k)) line_start[o++] = mb + k;
    }
}

// ---- 2. classify ------------------------------------------------------------------------------
__device__ inline bool break_at(const uint8_t *t, int64_t i, int64_t le) {
    const int b = t[i];
    if (is_break1(b)) return true;
    if (b == 0xC2 && i + 1 < le && t[i + 1] == 0x85) return true;
    if (b == 0xE2 && i + 2 < le && t[i + 1] == 0x80 && (t[i + 2] == 0xA8 || t[i + 2] == 0xA9)) return true;
    return false;
}

// One wave per 64 consecutive lines: their bytes (one contiguous span) are staged in LDS with
// coalesced 16-byte loads, then every lane scans its own line there; a span longer than the wave's
// buffer (very long lines) is read from global memory instead.
constexpr int kWaveBuf = 8192;
#ifndef FZ_BL_ONEPASS
#define FZ_BL_ONEPASS 1  // (0: the pattern-by-pattern classification, for A/B)
#endif
__global__ __launch_bounds__(kBlock) void k_line_classify(const uint8_t *__restrict__ t, int64_t n_bytes,
                                                          const int64_t *__restrict__ log_offs, int64_t n_logs,
                                                          const int64_t *__restrict__ line_start,
                                                          const int64_t *__restrict__ d_nl, int32_t *__restrict__ line_len,
                                                          uint32_t *__restrict__ line_flags, int64_t *__restrict__ line_cap) {
    __shared__ uint4 s_buf[kBlock / kWave][kWaveBuf / 16];
    const int64_t nl = *d_nl;
    const int w = wave_id(), lane = lane_id();
    uint8_t *buf = reinterpret_cast<uint8_t *>(s_buf[w]);
    for (int64_t lw = (int64_t(blockIdx.x) * (kBlock / kWave) + w) * kWave; lw < nl;
         lw += int64_t(gridDim.x) * kBlock) {
        const int64_t l = lw + lane;
        const int64_t sb = line_start[lw];
        const int64_t se = lw + kWave < nl ? line_start[lw + kWave] : n_bytes;
        const int64_t base = sb & ~int64_t(15);
        const bool staged = se - base <= kWaveBuf;
        if (staged) {
            const uint4 *src = reinterpret_cast<const uint4 *>(t + base);
            const int64_t nfull = (se - base) / 16;  // whole words, then the tail byte by byte
            for (int64_t k = lane; k < nfull; k += kWave) s_buf[w][k] = src[k];
            for (int64_t k = base + nfull * 16 + lane; k < se; k += kWave) buf[k - base] = t[k];
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
        if (l < nl) {
            const int64_t s = line_start[l];
            const int64_t lg = upper_bound_i64(log_offs, 0, n_logs + 1, s) - 1;  // the log holding byte s
            const int64_t le = log_offs[lg + 1];
            // the line's bytes (a line's break lies before the next line's start <= se)
            const uint8_t *lp = staged ? buf + (s - base) : t + s;
            const int64_t lim = le - s;
            int64_t e = 0;
            while (e < lim && !break_at(lp, e, lim)) ++e;
            const Line L{lp, int(e)};
            e += s;
            int co, cl;
            line_flags[l] = FZ_BL_ONEPASS ? classify1(L, co, cl) : classify(L, co, cl);
            line_len[l] = int32_t(e - s);
            line_cap[l] = co < 0 ? -1 : ((int64_t(co) << 32) | int64_t(cl));
        }
        __builtin_amdgcn_wave_barrier();  // the buffer is refilled for the next 64 lines
    }
}

// ---- 3. fold per log ----------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_log_fold(const int64_t *__restrict__ log_offs, int64_t n_logs,
                                                     const int64_t *__restrict__ line_start, const int64_t *__restrict__ d_nl,
                                                     const uint32_t *__restrict__ line_flags,
                                                     const int64_t *__restrict__ line_cap, fz_buildlog_out o) {
    const int lane = lane_id();
    const int64_t nl = *d_nl;
    for (int64_t g = int64_t(blockIdx.x) * 4 + wave_id(); g < n_logs; g += int64_t(gridDim.x) * 4) {
        const int64_t l0 = lower_bound_i64(line_start, 0, nl, log_offs[g]);
        const int64_t l1 = lower_bound_i64(line_start, 0, nl, log_offs[g + 1]);
        const int64_t n = l1 - l0;
        int64_t first_cap = INT64_MAX, last_set = -1, last_pd = -1;
        uint32_t tail = 0;
        for (int64_t l = l0 + lane; l < l1; l += kWave) {
            const uint32_t f = line_flags[l];
            if ((f & BL_IMAGE) && l < first_cap) first_cap = l;
            if ((f >> kSetShift) & 0xFu) last_set = l;
            if (f & BL_PUSHDONE) last_pd = l;
            if (l >= l1 - 200) tail |= f;
        }
        first_cap = wave_min(first_cap);
        last_set = wave_max(last_set);
        last_pd = wave_max(last_pd);
        tail |= __shfl_xor(tail, 1, 64);
        tail |= __shfl_xor(tail, 2, 64);
        tail |= __shfl_xor(tail, 4, 64);
        tail |= __shfl_xor(tail, 8, 64);
        tail |= __shfl_xor(tail, 16, 64);
        tail |= __shfl_xor(tail, 32, 64);
        if (lane != 0) continue;
        if (n == 0) {  // empty text: the reference returns before the analysis (:54-55)
            o.log_status[g] = 1;
            o.log_type[g] = BT_NONE;
            o.log_result[g] = BR_NONE;
            o.log_proj_off[g] = -1;
            o.log_proj_len[g] = 0;
            o.log_line0[g] = l0;
            continue;
        }
        o.log_line0[g] = l0;
        int bt = BT_NONE;
        if (last_set >= 0) {
            bt = int((line_flags[last_set] >> kSetShift) & 0xFu);
            if (last_pd >= last_set && bt != BT_COV && bt != BT_INTRO) bt = BT_FUZZ;
        } else if (last_pd >= 0) {
            bt = BT_FUZZ;
        }
        o.log_type[g] = bt;
        if (first_cap != INT64_MAX) {
            const int64_t cp = line_cap[first_cap];
            o.log_proj_off[g] = line_start[first_cap] + (cp >> 32);
            o.log_proj_len[g] = int32_t(cp & 0xffffffff);
        } else {
            o.log_proj_off[g] = -1;
            o.log_proj_len[g] = 0;
        }
        if (n == 1) {  // lines[-2] raises IndexError (:230)
            o.log_status[g] = 2;
            o.log_result[g] = BR_NONE;
            continue;
        }
        o.log_status[g] = 0;
        const bool err2 = (line_flags[l1 - 2] & BL_HAS_ERROR) != 0;
        o.log_result[g] = (err2 || (tail & BL_EQ_ERROR))              ? BR_ERROR
                          : ((tail & BL_EQ_PUSH) && (tail & BL_EQ_DONE)) ? BR_SUCCESS
                          : (tail & BL_EQ_DEADLINE)                      ? BR_ERROR
                                                                         : BR_UNKNOWN;
    }
}

// lines the host's srcmap extraction needs (skip / jq / JSON open / close), unordered
__global__ __launch_bounds__(kBlock) void k_line_events(const int64_t *__restrict__ line_start,
                                                        const int32_t *__restrict__ line_len,
                                                        const uint32_t *__restrict__ line_flags,
                                                        const int64_t *__restrict__ d_nl, fz_buildlog_out o) {
    const int64_t nl = *d_nl;
    constexpr uint32_t kEvent = BL_SKIP | BL_JQ | BL_OPEN | BL_CLOSE;
    for (int64_t l = int64_t(blockIdx.x) * kBlock + threadIdx.x; l < nl; l += int64_t(gridDim.x) * kBlock) {
        const uint32_t f = line_flags[l];
        if (!(f & kEvent)) continue;
        const unsigned long long k = atomicAdd(reinterpret_cast<unsigned long long *>(o.n_events), 1ull);
        if (int64_t(k) < o.event_cap) {
            o.ev_line[k] = l;
            o.ev_start[k] = line_start[l];
            o.ev_len[k] = line_len[l];
            o.ev_flags[k] = f & kEvent;
        }
    }
}

void buildlog(fz_ctx *c, const uint8_t *text, int64_t n_bytes, const int64_t *log_offs_host, const int64_t *log_offs,
              int64_t n_logs, const fz_buildlog_out *o) {
    FZ_CHECK(n_logs >= 0 && n_bytes >= 0, "fz_buildlog: negative size");
    FZ_CHECK(o != nullptr && o->n_lines && o->n_events, "fz_buildlog: outputs");
    if (n_logs == 0) {
        FZ_HIP(hipMemsetAsync(o->n_lines, 0, 8, c->stream));
        FZ_HIP(hipMemsetAsync(o->n_events, 0, 8, c->stream));
        return;
    }
    // chunk list (host): every log cut into kLineChunk-byte pieces
    std::vector<int32_t> clog;
    std::vector<int64_t> cb, ce;
    for (int64_t g = 0; g < n_logs; ++g) {
        const int64_t a = log_offs_host[g], b = log_offs_host[g + 1];
        FZ_CHECK(a <= b && b <= n_bytes, "fz_buildlog: log offsets");
        for (int64_t x = a; x < b; x += kLineChunk) {
            clog.push_back(int32_t(g));
            cb.push_back(x);
            ce.push_back(x + kLineChunk < b ? x + kLineChunk : b);
        }
    }
    const int64_t nch = int64_t(clog.size());
    int64_t *d_nl = o->n_lines;
    if (nch == 0) {
        FZ_HIP(hipMemsetAsync(d_nl, 0, 8, c->stream));
    }
    int32_t *d_clog = c->arena.get<int32_t>(nch);
    int64_t *d_cb = c->arena.get<int64_t>(nch), *d_ce = c->arena.get<int64_t>(nch);
    int64_t *cnt = c->arena.get<int64_t>(nch + 1), *off = c->arena.get<int64_t>(nch + 1);
    if (nch > 0) {
        FZ_HIP(hipMemcpyAsync(d_clog, clog.data(), size_t(nch) * 4, hipMemcpyHostToDevice, c->stream));
        FZ_HIP(hipMemcpyAsync(d_cb, cb.data(), size_t(nch) * 8, hipMemcpyHostToDevice, c->stream));
        FZ_HIP(hipMemcpyAsync(d_ce, ce.data(), size_t(nch) * 8, hipMemcpyHostToDevice, c->stream));
        const LogChunks ch{d_clog, d_cb, d_ce};
        const unsigned g = unsigned(nch < 16384 ? nch : 16384);
        {
            ProbeScope ps(c, "buildlog_lines", 2.0 * double(n_bytes));
            k_line_count<<<g, kBlock, 0, c->stream>>>(text, log_offs, ch, nch, cnt);
            FZ_LAUNCH_CHECK();
        }
        scan_exclusive_i64(c, cnt, off, nch, d_nl);
    }
    // the line arrays are sized by the count (one read-back per batch)
    FZ_HIP(hipMemcpyAsync(c->h_pinned, d_nl, 8, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    const int64_t cap = c->h_pinned[0] > 0 ? c->h_pinned[0] : 1;
    int64_t *line_start = c->arena.get<int64_t>(cap);
    if (nch > 0) {
        const LogChunks ch{d_clog, d_cb, d_ce};
        k_line_write<<<unsigned(nch < 16384 ? nch : 16384), kBlock, 0, c->stream>>>(text, log_offs, ch, nch, off,
                                                                                    line_start);
        FZ_LAUNCH_CHECK();
    }
    int32_t *line_len = c->arena.get<int32_t>(cap);
    uint32_t *line_flags = c->arena.get<uint32_t>(cap);
    int64_t *line_cap = c->arena.get<int64_t>(cap);
    {
        // algorithmic bytes: every byte of text read once + 16 B per line written (about 1 line per
        // 60 bytes of log: counted as bytes / 4)
        ProbeScope ps(c, "buildlog_classify", double(n_bytes) * 1.25);
        k_line_classify<<<grid_for(cap, kBlock, 16384), kBlock, 0, c->stream>>>(text, n_bytes, log_offs, n_logs,
                                                                              line_start, d_nl, line_len, line_flags,
                                                                              line_cap);
        FZ_LAUNCH_CHECK();
    }
    k_log_fold<<<grid_for((n_logs + 3) / 4, 1, 8192), kBlock, 0, c->stream>>>(log_offs, n_logs, line_start, d_nl,
                                                                              line_flags, line_cap, *o);
    FZ_LAUNCH_CHECK();
    FZ_HIP(hipMemsetAsync(o->n_events, 0, 8, c->stream));
    k_line_events<<<grid_for(cap, kBlock, 8192), kBlock, 0, c->stream>>>(line_start, line_len, line_flags, d_nl, *o);
    FZ_LAUNCH_CHECK();
}

}  // namespace fz
