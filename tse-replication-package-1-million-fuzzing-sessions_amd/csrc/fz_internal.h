// Internal declarations shared by the libfz translation units.
//
// Design: one fz_ctx per GPU.  It owns
//   * a scratch arena (grow-only device blocks, bump-allocated, reset at the start of every
//     public call) so steady-state calls never hipMalloc;
//   * the sorted store (fz_store.hip) - the replacement for PostgreSQL's tables + indexes.
// Kernels are plain HIP for gfx950: 256-thread workgroups (4 waves of 64), wave-level
// ballot/popcount for ranking and counting, LDS for block-level staging.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <initializer_list>
#include <stdexcept>
#include <string>
#include <vector>

#include "fz.h"

namespace fz {

constexpr int kBlock = 256;   // threads per workgroup (4 wave64)
constexpr int kWave = 64;
constexpr int kSortBlock = 1024;  // LDS bitonic sorts: 16 waves share one 4096-entry network

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define FZ_HIP(expr)                                                                           \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            throw ::fz::Error(FZ_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define FZ_CHECK(cond, msg)                                              \
    do {                                                                 \
        if (!(cond)) throw ::fz::Error(FZ_E_INVALID, std::string(msg)); \
    } while (0)

// a call out of order (FZ_E_STATE), e.g. a graph replay over a changed store
#define FZ_STATE(cond, msg)                                              \
    do {                                                                 \
        if (!(cond)) throw ::fz::Error(FZ_E_STATE, std::string(msg));   \
    } while (0)

#define FZ_LAUNCH_CHECK() FZ_HIP(hipGetLastError())

// Grow-only bump allocator over device blocks.
class Arena {
   public:
    ~Arena() { release(); }
    void *alloc(size_t bytes) {
        bytes = (bytes + 255) & ~size_t(255);
        if (bytes == 0) bytes = 256;
        for (; cur_ < blocks_.size(); ++cur_) {
            Block &b = blocks_[cur_];
            if (b.used + bytes <= b.size) {
                void *p = static_cast<char *>(b.ptr) + b.used;
                b.used += bytes;
                return p;
            }
        }
        size_t sz = bytes < (size_t(64) << 20) ? (size_t(64) << 20) : bytes;
        void *p = nullptr;
        FZ_HIP(hipMalloc(&p, sz));
        blocks_.push_back({p, sz, bytes});
        cur_ = blocks_.size() - 1;
        return p;
    }
    template <typename T>
    T *get(int64_t n) {
        return static_cast<T *>(alloc(size_t(n < 1 ? 1 : n) * sizeof(T)));
    }
    void reset() {
        for (auto &b : blocks_) b.used = 0;
        cur_ = 0;
    }
    void release() {
        for (auto &b : blocks_) (void)hipFree(b.ptr);
        blocks_.clear();
        cur_ = 0;
    }

   private:
    struct Block {
        void *ptr;
        size_t size;
        size_t used;
    };
    std::vector<Block> blocks_;
    size_t cur_ = 0;
};

// Persistent device buffer (re-allocated only when it must grow).
struct DevBuf {
    void *ptr = nullptr;
    size_t cap = 0;
    uint64_t gen = 0;  // bumped by every (re)allocation: a recorded graph holding ptr checks it
    ~DevBuf() {
        if (ptr) (void)hipFree(ptr);
    }
    template <typename T>
    T *ensure(int64_t n) {
        size_t bytes = size_t(n < 1 ? 1 : n) * sizeof(T);
        if (bytes > cap) {
            if (ptr) FZ_HIP(hipFree(ptr));
            ptr = nullptr;
            FZ_HIP(hipMalloc(&ptr, bytes));
            cap = bytes;
            ++gen;
        }
        return static_cast<T *>(ptr);
    }
    template <typename T>
    T *as() const {
        return static_cast<T *>(ptr);
    }
};

// A sorted view of one table (non-owning): rows in (project, time) order, their original row ids,
// sort times, projects, and per-project [offs[p], offs[p+1]) segments (n_projects + 1 entries).
struct View {
    int64_t n = 0;
    int64_t max_seg = 0;
    // (coverage view) the most rows of one project dated before the analyses' limit (2025-01-08,
    // queries1.py:3): every RQ2-count / RQ4b session axis is at most this long - their per-session
    // arrays, transposes and statistics are sized by it, not by the longest segment (config 5: a
    // 20.8 M-row project of which 2,960 rows precede the limit)
    int64_t lim_seg = 0;
    // view position q is store row row0 + q: the store's columns are gathered into view order, so
    // a view's row ids are implicit (the filters read no row array)
    int64_t row0 = 0;
    const int64_t *time = nullptr;
    const uint32_t *proj = nullptr;
    const int64_t *offs = nullptr;
};

// The replacement for the PostgreSQL tables + indexes: every table sorted once per load.
struct Store {
    bool built = false;
    fz_tables t{};
    int64_t P = 0;
    DevBuf b_time, b_proj, c_time, c_proj, i_time, i_proj;
    DevBuf off_fuzz, off_covb, off_cov, off_iss;
    View fuzz;    // buildlog_data, build_type = Fuzzing, by (project, timecreated)   queries1.py:267-278
    View covb;    // buildlog_data, build_type = Coverage, by (project, timecreated)
    View cov;     // total_coverage by (project, date)                              queries1.py:120-129
    View issues;  // issues by (project, rts), ties in row order                    rq3:219-232
    int64_t num_min = 0, num_max = 0;                   // issues.number range
    // eligible projects (the GROUP BY/HAVING every script starts from), computed once per load
    DevBuf elig;     // uint8 [P]
    DevBuf n_elig;   // int64 [2]: eligible projects, the most rows of one project before the limit
    DevBuf elig_cnt; // int32 [P]: each project's qualifying rows (a project cut across ranks sums them)
    // The tables themselves in sorted order: after the build `t` points at these sorted copies and
    // every view's row id IS the position in its sorted table, so filters and joins read columns
    // sequentially instead of gathering through the sort permutation.  perm maps a sorted
    // position back to the caller's row id (for row-id outputs: matched issues / builds, change
    // rows, detected issues).
    DevBuf sb_type, sb_result, sb_group, sb_canon, sc_coverage, sc_covered, sc_total, sc_valid, si_number, si_status;
    DevBuf b_perm, c_perm, i_perm;
    const int32_t *bperm = nullptr, *cperm = nullptr, *iperm = nullptr;

    // What a recorded analysis graph bakes in from the store: the sorted tables' pointers and sizes
    // and the buffers behind them.  Equal signatures = a replay reads what the recording read
    // (a rebuild over a table of the same shape keeps it; a reallocation or another table does not).
    uint64_t signature() const {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
        mix(built);
        mix(uint64_t(P));
        const unsigned char *tb = reinterpret_cast<const unsigned char *>(&t);
        for (size_t i = 0; i < sizeof(t); ++i) mix(tb[i]);
        for (const DevBuf *d : {&b_time, &b_proj, &c_time, &c_proj, &i_time, &i_proj,
                                &off_fuzz, &off_covb, &off_cov, &off_iss, &elig, &n_elig, &elig_cnt, &sb_type, &sb_result,
                                &sb_group, &sb_canon, &sc_coverage, &sc_covered, &sc_total, &sc_valid, &si_number,
                                &si_status, &b_perm, &c_perm, &i_perm}) {
            mix(reinterpret_cast<uintptr_t>(d->ptr));
            mix(d->gen);
        }
        for (const View *v : {&fuzz, &covb, &cov, &issues}) {
            mix(uint64_t(v->n));
            mix(uint64_t(v->max_seg));
            mix(uint64_t(v->lim_seg));
        }
        return h;
    }
};

// Per-kernel timing probe (fz_probe_begin/end/get): brackets every launch of the named kernels
// with HIP events on the context stream and accumulates their algorithmic bytes, so bench.py can
// report achieved GB/s per kernel.
struct Probe {
    std::vector<std::string> names;     // probed kernels (empty: probe off)
    std::vector<hipEvent_t> pool;       // pairs (start, stop)
    std::vector<int> owner;             // name index of each used pair
    size_t used = 0;
    std::vector<int64_t> launches;
    std::vector<double> bytes, ms;      // ms: filled by fz_probe_end
    std::vector<std::string> results;   // names of the last finished probe window (fz_probe_get)
    // algorithmic bytes that depend on a device count (e.g. rows kept by a filter): each probed
    // launch's count is copied (async, on the stream) into counts[slot] and added at fz_probe_end
    // as counts[slot] * per_count to the owner's bytes
    static constexpr int64_t kMaxCounts = 1 << 16;
    DevBuf counts;
    struct Deferred {
        int owner;
        int64_t slot;
        double per_count;
    };
    std::vector<Deferred> deferred;
    bool active() const { return !names.empty(); }
    int index(const char *n) const {
        for (size_t i = 0; i < names.size(); ++i)
            if (names[i] == n) return int(i);
        return -1;
    }
};

}  // namespace fz

struct fz_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // a child context (fz_ctx_create_child) runs analyses on its own stream over its parent's
    // store; everything else (arena, probe, look-back state, pinned staging) is its own
    fz_ctx *parent = nullptr;
    int64_t sort_passes = 0;       // radix passes run by this context (store statistics)
    fz::Arena arena;
    fz::Store store;
    fz::Probe probe;
    int64_t *h_pinned = nullptr;   // small pinned host staging area (32 KiB)
    int64_t *d_pinned = nullptr;   // the same area's device address (kernels write read-backs straight to it)
    // decoupled look-back state (fz_lookback.h; single-pass scan, compaction, radix passes): status
    // words tagged with a per-launch epoch, and a tile ticket counter each launch resets itself
    fz::DevBuf os_status;          // uint64 [max words of one launch]
    fz::DevBuf os_ticket;          // uint32 [4] self-resetting tile counters
    bool lb_pending = false;       // a look-back reset is owed (the next fill batch or look-back use runs it)
    unsigned int os_epoch = 0;
    // radix digit totals, two buffers used by alternate sorts: each sort's passes zero the other
    // one, so the next sort's histogram starts from zero without a memset launch
    fz::DevBuf os_hist;            // uint64 [2][kOsMaxPasses * 256]
    // per-segment arrival tickets of the chunked reductions whose last chunk folds its segment
    // (fz_seg.h seg_reduce): zero between launches - each segment's last arriver resets its word
    fz::DevBuf seg_tickets;        // uint32 [segments]
    int os_hist_cur = -1;          // buffer of the next sort (-1: not allocated / not known zero)
    // HIP graph recording (fz_capture_begin/end): a context on the null stream records on a
    // private stream; the context's own stream is restored when the recording ends
    bool capturing = false;
    hipStream_t capture_stream = nullptr;
    hipStream_t capture_saved = nullptr;
    // the store build's counter read-back (fz_store.hip): the host waits for this event, not for
    // the stream, so the gather launched after the copies overlaps the round trip
    hipEvent_t ev_readback = nullptr;
    // store-build helpers (fz_store_set_helpers: children of this context, idle while the store is
    // built): the build forks the tables' independent sorts onto their streams / contexts
    std::vector<fz_ctx *> helpers;
    hipEvent_t ev_fork = nullptr, ev_join[4] = {};
    // set while a public libfz call runs on this context (fz_api.hip guarded()): the store build
    // refuses helpers that are inside a call of their own (FZ_E_STATE) instead of racing on their
    // arena and look-back state
    std::atomic<int> in_call{0};
};

namespace fz {
// The store an analysis reads: the context's own, or its parent's for a child context.
inline Store &store_of(fz_ctx *c) { return c->parent ? c->parent->store : c->store; }

// RAII bracket around one launch of kernel `name` moving `bytes` algorithmic bytes, plus
// per_count bytes for every unit of the device count *d_count (read when the scope closes, i.e.
// after the launch, so it may be the launch's own output count).
struct ProbeScope {
    fz_ctx *c;
    bool on;
    int owner = -1;
    const int64_t *d_count = nullptr;
    double per_count = 0.0;
    const int64_t *d_count2 = nullptr;  // (a second device count, add_count)
    double per_count2 = 0.0;
    size_t pair = 0;  // index of this scope's (start, stop) events in the pool
    // per bytes more for every unit of another device count (read when the scope closes)
    void add_count(const int64_t *count, double per) {
        d_count2 = count;
        per_count2 = per;
    }
    ProbeScope(fz_ctx *ctx, const char *name, double bytes, const int64_t *count = nullptr, double per = 0.0)
        : c(ctx), on(false), d_count(count), per_count(per) {
        Probe &p = c->probe;
        if (!p.active()) return;
        const int k = p.index(name);
        if (k < 0) return;
        owner = k;
        if (p.used + 2 > p.pool.size()) {
            for (int i = 0; i < 64; ++i) {
                hipEvent_t e;
                FZ_HIP(hipEventCreate(&e));
                p.pool.push_back(e);
            }
        }
        // the scope's event pair is reserved now, so a scope opened inside this one (a scan inside
        // a merge sort) takes the next pair instead of this one's stop event
        pair = p.used;
        p.used += 2;
        FZ_HIP(hipEventRecord(p.pool[pair], c->stream));
        p.owner.push_back(k);
        p.bytes[k] += bytes;
        p.launches[k] += 1;
        on = true;
    }
    // more algorithmic bytes for this scope's kernel, known only after its launch (host side)
    static void add_bytes(fz_ctx *ctx, const char *name, double bytes) {
        Probe &p = ctx->probe;
        if (!p.active()) return;
        const int k = p.index(name);
        if (k >= 0) p.bytes[k] += bytes;
    }
    ~ProbeScope() {
        if (!on) return;
        Probe &p = c->probe;
        (void)hipEventRecord(p.pool[pair + 1], c->stream);
        const int64_t *dc[2] = {d_count, d_count2};
        const double pc[2] = {per_count, per_count2};
        for (int i = 0; i < 2; ++i) {
            if (!on || !dc[i] || int64_t(p.deferred.size()) >= Probe::kMaxCounts) continue;
            const int64_t slot = int64_t(p.deferred.size());
            (void)hipMemcpyAsync(p.counts.as<int64_t>() + slot, dc[i], 8, hipMemcpyDeviceToDevice, c->stream);
            p.deferred.push_back({owner, slot, pc[i]});
        }
    }
};
}  // namespace fz

namespace fz {

// ---- primitives (fz_prims.hip) --------------------------------------------------------------
// Device-wide exclusive scan of int64 (in != out allowed). Returns nothing; total written to
// out_total (device) if non-null.
void scan_exclusive_i64(fz_ctx *c, const int64_t *in, int64_t *out, int64_t n, int64_t *out_total);
// The same over the first *d_live elements of a capacity n_cap (device count): elements past them are
// neither read nor written, except out[live] = the total when live < n_cap.
void scan_exclusive_i64_dn(fz_ctx *c, const int64_t *in, int64_t *out, int64_t n_cap, const int64_t *d_live,
                           int64_t *out_total);
// Stable LSD radix sort of (uint64 key, uint32 value) over bits [0, bits).  Uses arena scratch;
// the result is written back to keys/vals.
void radix_sort_pairs(fz_ctx *c, uint64_t *keys, uint32_t *vals, int64_t n, int bits);
// The same without the copy back: on return keys / vals point at the sorted data (the inputs or
// arena scratch of the current call).
void radix_sort_pairs_swap(fz_ctx *c, uint64_t *&keys, uint32_t *&vals, int64_t n, int bits);
// The same over the first *d_live of n_cap keys (device count): the passes' tiles past them leave at
// once; on return keys / vals [0, *d_live) are sorted, the entries past them undefined.
void radix_sort_pairs_swap_live(fz_ctx *c, uint64_t *&keys, uint32_t *&vals, int64_t n_cap, const int64_t *d_live,
                                int bits);
// Columns that travel with the keys through every pass (each pass records every input position's
// destination and moves the columns there): on return out[j] holds column j in sorted order.
constexpr int kMaxPayload = 6;
struct RadixPayload {
    int n = 0;
    const void *in[kMaxPayload] = {};
    void *out[kMaxPayload] = {};
    int size[kMaxPayload] = {};  // bytes per element: 1, 4 or 8
    // (host-side option) no constant-digit read-back for this sort: the store's project-prefix
    // sorts, enqueued ahead of the build's own read-back, whose digits all vary in practice
    bool no_digit_probe = false;
    double bytes() const {
        double b = 0.0;
        for (int j = 0; j < n; ++j) b += size[j];
        return b;
    }
};
void radix_sort_pairs_payload(fz_ctx *c, uint64_t *&keys, uint32_t *&vals, int64_t n, int bits, RadixPayload &pl);
// the same for keys of at most 32 bits held as uint32 (4 bytes less per key and pass)
void radix_sort_pairs_payload32(fz_ctx *c, uint32_t *&keys, uint32_t *&vals, int64_t n, int bits, RadixPayload &pl);
// The same sort of (key_src[i], i): the keys read from a read-only column, the values the rows'
// positions - nothing copied beforehand.  keys / vals: two caller scratch buffers of n entries (the
// passes ping-pong through them and one arena pair); on return they point at the sorted result.
// Stable sort of one segment [0, offs[1]) of doubles by (value, position) - splitter buckets from
// a sorted sample, one onesweep scatter pass, an LDS sort per bucket (fz_prims.hip).  offs[0] must
// be 0; val / pos are written on [0, offs[1]) only.  n_cap: host bound of offs[1], < 2^31.
void sample_sort_f64_seg1(fz_ctx *c, const double *src, const int64_t *offs, int64_t n_cap, double *val,
                          int32_t *pos);
bool sample_sort_on();  // FZ_SAMPLE_SORT=0: the LSD radix path instead (A/B builds of one library)
// Reductions whose last-arriving block folds the partials (one launch fewer each) when
// FZ_FUSED_FOLD=1 - off by default (measured slower at config 2, fz_series.hip).  seg_tickets: the context's zeroed per-segment ticket
// words (each fold resets its own), or null while a graph is recorded and they would have to grow.
bool fused_fold_on();
unsigned *seg_tickets(fz_ctx *c, int64_t S);
void radix_sort_rows_payload32(fz_ctx *c, const uint32_t *key_src, uint32_t *&keys, uint32_t *&vals, int64_t n,
                               int bits, RadixPayload &pl);
// radix_sort_pairs_payload32 over the first *d_live of n_cap entries (device count)
void radix_sort_pairs_payload32_live(fz_ctx *c, uint32_t *&keys, uint32_t *&vals, int64_t n_cap, const int64_t *d_live,
                                     int bits, RadixPayload &pl);
// Up to three such sorts (32-bit keys, values, payload columns) in shared launches: one histogram
// launch for all, then one launch per digit pass over every table that has that digit.  Per table:
// key_src (optional, as radix_sort_rows_payload32: the first pass reads the keys there and takes the
// positions as values) or keys + vals (caller buffers of n entries, overwritten); on return keys /
// vals / pl.out point at the sorted data.  hist0: [3][8][256] u64 digit totals, zeroed by the caller.
struct RadixTab {
    const uint32_t *key_src = nullptr;
    const uint8_t *type_src = nullptr;  // (with key_src) key = key_src | min(type, 2) << type_shift
    int type_shift = 0;
    uint32_t *keys = nullptr;
    uint32_t *vals = nullptr;
    int64_t n = 0;
    int bits = 0;
    RadixPayload pl;
    int npass = 0;  // (set by the sort)
};
constexpr int64_t kRadixTabHistWords = 3 * 8 * 256;
// side: (optional) a min / max of an int64 column (FZ_TS_NULL skipped) in the histogram launch's
// extra workgroups - partials part[4 * b + {2, 3}] for b < blocks
struct RadixSideMinMax {
    const int64_t *src = nullptr;
    int64_t n = 0;
    int64_t *part = nullptr;
    unsigned blocks = 0;
};
void radix_sort_tables_payload32(fz_ctx *c, RadixTab *tabs, int nt, unsigned long long *hist0,
                                 const RadixSideMinMax *side = nullptr);
// min/max over int64 values skipping FZ_TS_NULL: writes {min, max} to host array.
void minmax_i64_to_host(fz_ctx *c, const int64_t *const *cols, const int64_t *ns, int ncols,
                        int64_t *host_minmax);
// Per-project [start,end) offsets of a project-sorted uint32 array.
void segment_offsets(fz_ctx *c, const uint32_t *sorted_proj, int64_t n, int64_t P, int64_t *offsets);
// numpy-compatible describe of a device double vector (n may be 0).
void describe_f64(fz_ctx *c, const double *x, int64_t n, fz_describe *dev_out);
// Order-preserving uint64 image of a double (for radix sorting doubles; NaN sorts last).
__host__ __device__ inline uint64_t f64_key(double d) {
    uint64_t u = __builtin_bit_cast(uint64_t, d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__host__ __device__ inline double f64_from_key(uint64_t k) {
    uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __builtin_bit_cast(double, u);
}

inline int bits_for(uint64_t maxval) {
    int b = 0;
    while (b < 64 && (maxval >> b) != 0) ++b;
    return b;
}

inline unsigned grid_for(int64_t n, int per_block = kBlock, unsigned cap = 8192) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return unsigned(g);
}

void sync(fz_ctx *c);
// d[0..n) = v[0..n) (host values passed by value through a kernel argument; n <= 4)
void set_i64(fz_ctx *c, int64_t *d, const int64_t *v, int n);
// Byte fills of up to 16 device regions in ONE launch (instead of one hipMemsetAsync each).
struct Fill {
    void *ptr;
    int64_t bytes;
    unsigned char value;
};
void fill_batch(fz_ctx *c, std::initializer_list<Fill> regions);
// The same plus, in the same launch, a byte copy and one int64 word (*word_src -> *word_dst; a word
// inside a filled region is written in place of its fill)
void fill_copy_batch(fz_ctx *c, std::initializer_list<Fill> regions, const void *copy_src, void *copy_dst,
                     int64_t copy_bytes, const int64_t *word_src = nullptr, int64_t *word_dst = nullptr);
// Device-side byte fill / copy kernels on the context stream.  Used instead of hipMemsetAsync /
// hipMemcpyAsync(D2D) on every path an fz_capture recording may contain: a recorded sequence is
// then kernels only, replayed in stream order.
void dev_fill(fz_ctx *c, void *p, unsigned char value, int64_t bytes);
void dev_copy(fz_ctx *c, void *dst, const void *src, int64_t bytes);

}  // namespace fz
