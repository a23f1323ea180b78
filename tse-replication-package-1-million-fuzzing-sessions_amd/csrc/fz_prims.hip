// Device-wide primitives: exclusive scan, stable LSD radix sort, min/max, segment offsets,
// numpy-compatible describe.  All launches go to the context stream; scratch comes from the arena.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "fz_device.h"
#include "fz_internal.h"
#include "fz_lookback.h"
#include "fz_views.h"

namespace fz {

void sync(fz_ctx *c) { FZ_HIP(hipStreamSynchronize(c->stream)); }

constexpr int kMaxFills = 18;
struct FillList {
    int n;
    unsigned char *ptr[kMaxFills];
    int64_t bytes[kMaxFills];
    unsigned char value[kMaxFills];
    // optional, in the same launch: a byte copy (copy_n bytes copy_src -> copy_dst) and one int64
    // word (*word_src -> *word_dst); a word that lies inside a filled region takes the place of its
    // fill there (no ordering between the fill and the word)
    const unsigned char *copy_src;
    unsigned char *copy_dst;
    int64_t copy_n;
    const int64_t *word_src;
    int64_t *word_dst;
    int word_in_fill;
};
__global__ __launch_bounds__(kBlock) void k_fill_batch(FillList f) {
    const int64_t *wdst = f.word_in_fill ? f.word_dst : nullptr;
    for (int r = 0; r < f.n; ++r) {
        unsigned char *p = f.ptr[r];
        const int64_t nb = f.bytes[r];
        const unsigned char v = f.value[r];
        if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {  // 8-byte stores, byte tail
            const uint64_t w = 0x0101010101010101ull * v;
            const int64_t n8 = nb >> 3;
            for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n8; i += int64_t(gridDim.x) * kBlock) {
                uint64_t *q = reinterpret_cast<uint64_t *>(p) + i;
                *q = (reinterpret_cast<const int64_t *>(q) == wdst) ? uint64_t(*f.word_src) : w;
            }
            for (int64_t i = (n8 << 3) + int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nb;
                 i += int64_t(gridDim.x) * kBlock)
                p[i] = v;
        } else {
            for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nb; i += int64_t(gridDim.x) * kBlock)
                p[i] = v;
        }
    }
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < f.copy_n; i += int64_t(gridDim.x) * kBlock)
        f.copy_dst[i] = f.copy_src[i];
    if (f.word_dst && !f.word_in_fill && blockIdx.x == 0 && threadIdx.x == 0) *f.word_dst = *f.word_src;
}
void fill_batch(fz_ctx *c, std::initializer_list<Fill> regions) { fill_copy_batch(c, regions, nullptr, nullptr, 0); }

void fill_copy_batch(fz_ctx *c, std::initializer_list<Fill> regions, const void *copy_src, void *copy_dst,
                     int64_t copy_bytes, const int64_t *word_src, int64_t *word_dst) {
    FillList f{};
    f.copy_src = static_cast<const unsigned char *>(copy_src);
    f.copy_dst = static_cast<unsigned char *>(copy_dst);
    f.copy_n = copy_src ? copy_bytes : 0;
    f.word_src = word_src;
    f.word_dst = word_dst;
    int64_t most = f.copy_n;
    for (const Fill &r : regions) {
        FZ_CHECK(f.n < kMaxFills, "fill_batch: too many regions");
        if (r.bytes <= 0) continue;
        f.ptr[f.n] = static_cast<unsigned char *>(r.ptr);
        f.bytes[f.n] = r.bytes;
        f.value[f.n] = r.value;
        most = r.bytes > most ? r.bytes : most;
        const char *lo = static_cast<const char *>(r.ptr), *wp = reinterpret_cast<const char *>(word_dst);
        if (word_dst && wp >= lo && wp < lo + r.bytes) {  // the word replaces its fill (8-byte path only)
            FZ_CHECK((reinterpret_cast<uintptr_t>(r.ptr) & 7) == 0 && (wp - lo) % 8 == 0 && wp + 8 <= lo + r.bytes,
                     "fill_copy_batch: the word must be an aligned word of an aligned region");
            f.word_in_fill = 1;
        }
        ++f.n;
    }
    if (c->lb_pending && f.n + 2 <= kMaxFills) {
        // an owed look-back reset (lookback_reset) rides along: the tickets and status words are two
        // more zero regions
        c->lb_pending = false;
        const Fill owed[2] = {{c->os_ticket.ptr, int64_t(c->os_ticket.cap), 0}, {c->os_status.ptr, int64_t(c->os_status.cap), 0}};
        for (const Fill &r : owed) {
            if (!r.ptr || r.bytes <= 0) continue;
            f.ptr[f.n] = static_cast<unsigned char *>(r.ptr);
            f.bytes[f.n] = r.bytes;
            f.value[f.n] = 0;
            most = r.bytes > most ? r.bytes : most;
            ++f.n;
        }
    }
    if (f.n == 0 && f.copy_n == 0 && !word_dst) return;
    k_fill_batch<<<grid_for((most + 7) / 8, kBlock, 1024), kBlock, 0, c->stream>>>(f);
    FZ_LAUNCH_CHECK();
}

__global__ __launch_bounds__(kBlock) void k_copy_bytes(unsigned char *__restrict__ dst,
                                                       const unsigned char *__restrict__ src, int64_t nb) {
    if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 7) == 0) {
        const int64_t n8 = nb >> 3;
        for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n8; i += int64_t(gridDim.x) * kBlock)
            reinterpret_cast<uint64_t *>(dst)[i] = reinterpret_cast<const uint64_t *>(src)[i];
        for (int64_t i = (n8 << 3) + int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nb; i += int64_t(gridDim.x) * kBlock)
            dst[i] = src[i];
    } else {
        for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nb; i += int64_t(gridDim.x) * kBlock)
            dst[i] = src[i];
    }
}
void dev_fill(fz_ctx *c, void *p, unsigned char value, int64_t bytes) { fill_batch(c, {{p, bytes, value}}); }
void dev_copy(fz_ctx *c, void *dst, const void *src, int64_t bytes) {
    if (bytes <= 0) return;
    k_copy_bytes<<<grid_for((bytes + 7) / 8, kBlock, 4096), kBlock, 0, c->stream>>>(
        static_cast<unsigned char *>(dst), static_cast<const unsigned char *>(src), bytes);
    FZ_LAUNCH_CHECK();
}

struct I64x4 {
    int64_t v[4];
};
__global__ void k_set_i64(int64_t *d, I64x4 v, int n) {
    if (threadIdx.x < n) d[threadIdx.x] = v.v[threadIdx.x];
}
void set_i64(fz_ctx *c, int64_t *d, const int64_t *v, int n) {
    FZ_CHECK(n >= 1 && n <= 4, "set_i64: 1..4 values");
    I64x4 a{};
    for (int i = 0; i < n; ++i) a.v[i] = v[i];
    k_set_i64<<<1, 64, 0, c->stream>>>(d, a, n);
    FZ_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------ scan (int64)
constexpr int kScanItems = 8;
constexpr int kScanChunk = kBlock * kScanItems;  // 2048 elements per workgroup

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const int64_t *__restrict__ in, int64_t n,
                                                        int64_t *__restrict__ sums) {
    __shared__ int64_t s_tmp[4];
    const int64_t base = int64_t(blockIdx.x) * kScanChunk;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        int64_t idx = base + i * kBlock + threadIdx.x;
        if (idx < n) acc += in[idx];
    }
    int64_t tot = block_sum(acc, s_tmp);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// Exclusive scan of one chunk per workgroup, plus a per-chunk carry (may be null).
__global__ __launch_bounds__(kBlock) void k_scan_chunk(const int64_t *__restrict__ in, int64_t *__restrict__ out,
                                                       int64_t n, const int64_t *__restrict__ carry,
                                                       int64_t *__restrict__ total) {
    __shared__ int64_t s_val[kScanChunk];
    __shared__ int64_t s_tmp[4];
    const int64_t base = int64_t(blockIdx.x) * kScanChunk;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        int64_t idx = base + i * kBlock + threadIdx.x;
        s_val[i * kBlock + threadIdx.x] = idx < n ? in[idx] : 0;
    }
    __syncthreads();
    int64_t loc[kScanItems];
    int64_t run = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        loc[i] = run;
        run += s_val[threadIdx.x * kScanItems + i];
    }
    int64_t btot;
    int64_t off = block_excl_scan(run, s_tmp, &btot);
    off += carry ? carry[blockIdx.x] : 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) s_val[threadIdx.x * kScanItems + i] = loc[i] + off;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        int64_t idx = base + i * kBlock + threadIdx.x;
        if (idx < n) out[idx] = s_val[i * kBlock + threadIdx.x];
    }
    if (total && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *total = off + btot;
}

// One 1024-thread workgroup scans up to 8192 elements (64 KiB of LDS): a single launch for the
// mid-sized scans (radix digit counts of <= 32 tiles, per-project offsets, compactions).
constexpr int kScan1Threads = 1024;
constexpr int kScan1Items = 8;
constexpr int kScan1Max = kScan1Threads * kScan1Items;

__global__ __launch_bounds__(kScan1Threads) void k_scan_single(const int64_t *__restrict__ in,
                                                               int64_t *__restrict__ out, int64_t n,
                                                               int64_t *__restrict__ total) {
    __shared__ int64_t s_val[kScan1Max];
    __shared__ int64_t s_w[kScan1Threads / 64];
    const int tid = threadIdx.x;
    for (int i = 0; i < kScan1Items; ++i) {
        const int idx = i * kScan1Threads + tid;
        s_val[idx] = idx < n ? in[idx] : 0;
    }
    __syncthreads();
    int64_t loc[kScan1Items];
    int64_t run = 0;
    for (int i = 0; i < kScan1Items; ++i) {
        loc[i] = run;
        run += s_val[tid * kScan1Items + i];
    }
    const int64_t inc = wave_incl_scan(run);
    if (lane_id() == 63) s_w[wave_id()] = inc;
    __syncthreads();
    int64_t woff = 0, tot = 0;
    for (int w = 0; w < kScan1Threads / 64; ++w) {
        const int64_t v = s_w[w];
        if (w < wave_id()) woff += v;
        tot += v;
    }
    const int64_t off = woff + inc - run;
    for (int i = 0; i < kScan1Items; ++i) s_val[tid * kScan1Items + i] = loc[i] + off;
    __syncthreads();
    for (int i = 0; i < kScan1Items; ++i) {
        const int idx = i * kScan1Threads + tid;
        if (idx < n) out[idx] = s_val[idx];
    }
    if (total && tid == 0) *total = tot;
}

// FZ_TRACE=1: host-side trace of the look-back / radix bookkeeping (graph-recording diagnostics)
static bool trace_on() {
    static const bool on = std::getenv("FZ_TRACE") != nullptr;
    return on;
}

Lookback lookback_begin(fz_ctx *c, int64_t words) {
    if (c->lb_pending) lookback_flush(c);
    if (c->os_status.cap < size_t(words < 1 ? 1 : words) * 8) {
        uint64_t *st = c->os_status.ensure<uint64_t>(words);
        dev_fill(c, st, 0, int64_t(c->os_status.cap));
        c->os_epoch = 0;
    }
    if (c->os_ticket.cap == 0) {  // (four counters: up to four look-back launches fused in one kernel)
        dev_fill(c, c->os_ticket.ensure<unsigned int>(4), 0, 16);
    }
    if (++c->os_epoch == (1u << 14)) {  // epoch wrap: clear the status words once
        dev_fill(c, c->os_status.ptr, 0, int64_t(c->os_status.cap));
        c->os_epoch = 1;
    }
    if (trace_on())
        std::fprintf(stderr, "[fz] ctx %p lookback words %lld epoch %u status %p cap %zu\n", (void *)c,
                     (long long)words, c->os_epoch, c->os_status.ptr, c->os_status.cap);
    return Lookback{c->os_status.as<uint64_t>(), c->os_ticket.as<unsigned int>(), uint64_t(c->os_epoch) << 48};
}

Lookback lookback_begin_n(fz_ctx *c, const int64_t *words, int k, Lookback *out) {
    FZ_CHECK(k >= 1 && k <= 4, "lookback_begin_n: 1..4 launches");
    int64_t tot = 0;
    for (int j = 0; j < k; ++j) tot += words[j] > 0 ? words[j] : 1;
    const Lookback lb = lookback_begin(c, tot);
    int64_t o = 0;
    for (int j = 0; j < k; ++j) {
        out[j] = Lookback{lb.status + o, lb.ticket + j, lb.epoch};
        o += words[j] > 0 ? words[j] : 1;
    }
    return lb;
}

// Zero the tile tickets and every status word of the context (one kernel: a graph recording starts
// with it, so each replay finds no status word carrying one of its recorded epochs).
__global__ __launch_bounds__(kBlock) void k_lb_reset(unsigned int *__restrict__ ticket, uint64_t *__restrict__ status,
                                                     int64_t words) {
    if (blockIdx.x == 0 && threadIdx.x < 4 && ticket) ticket[threadIdx.x] = 0u;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < words; i += int64_t(gridDim.x) * kBlock)
        status[i] = 0ull;
}

// The reset is owed rather than launched: the context's next fill batch carries it (two more zero
// regions, one launch fewer at the head of a recording), else the next look-back use launches it.
void lookback_reset(fz_ctx *c) {
    c->lb_pending = true;
    c->os_epoch = 0;
}
void lookback_flush(fz_ctx *c) {
    c->lb_pending = false;
    const int64_t words = int64_t(c->os_status.cap / 8);
    if (!c->os_ticket.cap && !words) return;
    k_lb_reset<<<grid_for(words, kBlock, 2048), kBlock, 0, c->stream>>>(
        c->os_ticket.cap ? c->os_ticket.as<unsigned int>() : nullptr, c->os_status.as<uint64_t>(), words);
    FZ_LAUNCH_CHECK();
}

// Single-pass exclusive scan: 4096-element tiles, tile prefixes by decoupled look-back
// (fz_lookback.h).
constexpr int kLbItems = 16;
constexpr int kLbTile = kBlock * kLbItems;  // 4096

// d_live (optional): only the first *d_live (<= n) elements are scanned - tiles past them exit after
// drawing their ticket (a capacity-sized launch over a short live prefix costs little), and out[live]
// receives the total when live < n.
__global__ __launch_bounds__(kBlock) void k_scan_lookback(const int64_t *__restrict__ in, int64_t *__restrict__ out,
                                                          int64_t n_cap, int64_t ntiles_cap, Lookback lb,
                                                          int64_t *__restrict__ total,
                                                          const int64_t *__restrict__ d_live) {
    __shared__ int64_t s_val[kLbTile];
    __shared__ int64_t s_tmp[4];
    __shared__ int64_t s_prefix;
    __shared__ unsigned int s_tile;
    const int tid = threadIdx.x;
    const int64_t live = d_live ? (*d_live < n_cap ? *d_live : n_cap) : n_cap;
    const int64_t n = live;
    const int64_t ntiles = live > 0 ? (live + kLbTile - 1) / kLbTile : 1;
    (void)ntiles_cap;
    // workgroups past the live tiles leave before drawing a ticket (no contention on the counter);
    // the live ones draw tickets 0 .. ntiles - 1 and the last drawer resets the counter
    if (int64_t(blockIdx.x) >= ntiles) return;
    if (tid == 0) s_tile = lb_take_tile(lb.ticket, unsigned(ntiles));
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t base = tile * kLbTile;
    int64_t x[kLbItems];
#pragma unroll
    for (int i = 0; i < kLbItems; ++i) {
        const int64_t idx = base + i * kBlock + tid;
        x[i] = idx < n ? in[idx] : 0;
    }
#pragma unroll
    for (int i = 0; i < kLbItems; ++i) s_val[i * kBlock + tid] = x[i];
    __syncthreads();
    int64_t loc[kLbItems];
    int64_t run = 0;
#pragma unroll
    for (int i = 0; i < kLbItems; ++i) {
        loc[i] = run;
        run += s_val[tid * kLbItems + i];
    }
    int64_t agg;
    const int64_t off = block_excl_scan(run, s_tmp, &agg);
    if (tid < kWave) {
        const int64_t prefix = lb_exclusive_prefix(lb, tile, agg);
        if (tid == 0) {
            s_prefix = prefix;
            if (tile == ntiles - 1) {
                if (total) *total = prefix + agg;
                if (live < n_cap) out[live] = prefix + agg;
            }
        }
    }
    __syncthreads();
    const int64_t pre = s_prefix;
    for (int i = 0; i < kLbItems; ++i) s_val[tid * kLbItems + i] = loc[i] + off + pre;
    __syncthreads();
    for (int i = 0; i < kLbItems; ++i) {
        const int64_t idx = base + i * kBlock + tid;
        if (idx < n) out[idx] = s_val[i * kBlock + tid];
    }
}

static void scan_exclusive_impl(fz_ctx *c, const int64_t *in, int64_t *out, int64_t n, int64_t *out_total) {
    if (n <= 0) {
        if (out_total) dev_fill(c, out_total, 0, sizeof(int64_t));
        return;
    }
    if (n > kScanChunk && n <= kScan1Max) {
        k_scan_single<<<1, kScan1Threads, 0, c->stream>>>(in, out, n, out_total);
        FZ_LAUNCH_CHECK();
        return;
    }
    if (n > kScan1Max) {
        const int64_t ntiles = (n + kLbTile - 1) / kLbTile;
        const Lookback lb = lookback_begin(c, ntiles);
        // algorithmic bytes: the int64 input read, the int64 output written (the long scans only:
        // shorter ones are one- or few-workgroup launches)
        ProbeScope ps(c, "scan_i64", 16.0 * double(n));
        k_scan_lookback<<<unsigned(ntiles), kBlock, 0, c->stream>>>(in, out, n, ntiles, lb, out_total, nullptr);
        FZ_LAUNCH_CHECK();
        lookback_end(c, ntiles);
        return;
    }
    const int64_t nb = (n + kScanChunk - 1) / kScanChunk;
    if (nb == 1) {
        k_scan_chunk<<<1, kBlock, 0, c->stream>>>(in, out, n, nullptr, out_total);
        FZ_LAUNCH_CHECK();
        return;
    }
    int64_t *sums = c->arena.get<int64_t>(nb);
    k_scan_reduce<<<unsigned(nb), kBlock, 0, c->stream>>>(in, n, sums);
    FZ_LAUNCH_CHECK();
    scan_exclusive_impl(c, sums, sums, nb, nullptr);  // recursion depth log_2048(n)
    k_scan_chunk<<<unsigned(nb), kBlock, 0, c->stream>>>(in, out, n, sums, out_total);
    FZ_LAUNCH_CHECK();
}

void scan_exclusive_i64(fz_ctx *c, const int64_t *in, int64_t *out, int64_t n, int64_t *out_total) {
    scan_exclusive_impl(c, in, out, n, out_total);
}

// (the short path of scan_exclusive_i64_dn: the scan ran over the capacity; the live total from it)
__global__ void k_scan_live_end(const int64_t *__restrict__ in, int64_t *__restrict__ out, int64_t n_cap,
                                const int64_t *__restrict__ d_live, int64_t *__restrict__ total) {
    const int64_t live = *d_live < n_cap ? *d_live : n_cap;
    const int64_t t = live > 0 ? out[live - 1] + in[live - 1] : 0;
    if (live < n_cap) out[live] = t;
    if (total) *total = t;
}

void scan_exclusive_i64_dn(fz_ctx *c, const int64_t *in, int64_t *out, int64_t n_cap, const int64_t *d_live,
                           int64_t *out_total) {
    if (n_cap <= kScan1Max || d_live == nullptr) {  // (short: one or few workgroups anyway)
        scan_exclusive_impl(c, in, out, n_cap, d_live ? nullptr : out_total);
        if (d_live && n_cap > 0) {
            k_scan_live_end<<<1, 1, 0, c->stream>>>(in, out, n_cap, d_live, out_total);
            FZ_LAUNCH_CHECK();
        } else if (d_live && out_total) {
            dev_fill(c, out_total, 0, sizeof(int64_t));
        }
        return;
    }
    const int64_t ntiles = (n_cap + kLbTile - 1) / kLbTile;
    const Lookback lb = lookback_begin(c, ntiles);
    ProbeScope ps(c, "scan_i64", 0.0, d_live, 16.0);
    k_scan_lookback<<<unsigned(ntiles), kBlock, 0, c->stream>>>(in, out, n_cap, ntiles, lb, out_total, d_live);
    FZ_LAUNCH_CHECK();
    lookback_end(c, ntiles);
}

// ------------------------------------------------------------------------- LSD radix sort
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
#ifndef FZ_OS_BLOCK
#define FZ_OS_BLOCK 512
#endif
#ifndef FZ_OS_TILE
#define FZ_OS_TILE 4096
#endif
#ifndef FZ_OS_WINDOW
#define FZ_OS_WINDOW 8
#endif
// the first payload column loaded with the keys (same-box A/B, scripts/bench_ab.sh: c3 20.73 ->
// 20.62 ms, c5 30.75 -> 30.66, c2 unchanged; 88 -> 105 VGPRs, occupancy 5 -> 4 waves per SIMD)
#ifndef FZ_OS_PREFETCH
#define FZ_OS_PREFETCH 1
#endif
constexpr int kOsBlock = FZ_OS_BLOCK;        // threads per radix-pass workgroup
constexpr int kSortTile = FZ_OS_TILE;        // keys per workgroup
static_assert(kOsBlock >= kRadix && kSortTile % kOsBlock == 0, "radix pass shape");
constexpr int kSortTileBig = 8192, kOsBlockBig = 1024;  // the large sorts' tile shape
#ifndef FZ_OS_TILE_NP
#define FZ_OS_TILE_NP FZ_OS_TILE
#endif
#ifndef FZ_OS_BLOCK_NP
#define FZ_OS_BLOCK_NP FZ_OS_BLOCK
#endif
// sorts without payload columns below kOsBigN keys (RQ3's union: ~790 k 64-bit keys at config 2)
constexpr int kSortTileNp = FZ_OS_TILE_NP, kOsBlockNp = FZ_OS_BLOCK_NP;
constexpr int64_t kOsBigN = int64_t(1) << 22;            // keys from which a sort takes it

// ---- single-sweep LSD passes (one launch per digit pass) -----------------------------------
// One histogram kernel counts every pass's digits up front (the global digit bases of every
// pass, from one read of the keys).  Each pass is then ONE kernel: a tile
// ranks its 4096 keys (stable: round, wave, lane order), publishes its per-digit counts, and gets
// its global base per digit by decoupled look-back over the preceding tiles' status words
// {flag:2, epoch:14, count:48} (tiles in ticket order; 8 predecessors per poll) - no per-tile
// histogram pass, no device-wide scan of the tile x digit counts.  Epoch tags make stale words
// from earlier passes invisible, so the status array is never cleared between passes.
// Grouped look-back: every tile also adds its counts into a {tiles:16, sum:48} word of its group
// of 8 tiles; a tile walks its own group's earlier tiles one by one, then whole groups (a group's
// last inclusive word or its completed sum) - O(tiles / 8) status reads instead of O(tiles), which
// matters because every tile polls through the coherent (uncached) path: 20.1 -> 17.8 us per
// 650 k-key pass, 154 -> 140 us per 16 M-key pass.
// Shape (scripts/radix_micro.py, MI355X): 512 threads (8 waves x 8 rounds) per 4096-key tile -
// two waves per SIMD hide the ranking loop's LDS round trips (17.8 vs 20.8 us per 650 k-key pass
// with 4 waves); 8-predecessor polls beat 16/32 (look-back traffic is bandwidth-limited).
constexpr int kOsMaxPasses = 8;
constexpr int kOsWindow = FZ_OS_WINDOW;
#ifndef FZ_HIST_KPB
#define FZ_HIST_KPB 2048
#endif
constexpr int kHistKeysPerBlock = FZ_HIST_KPB;  // keys per histogram workgroup (its flush is npass x 256 atomics;
// 8192 keys per workgroup made the small sorts' loops latency-bound: 6 -> 20 us for 65 k keys)
#ifndef FZ_HIST_MAXB
#define FZ_HIST_MAXB 256
#endif
constexpr int kHistMaxBlocks = FZ_HIST_MAXB;
#ifndef FZ_HIST_BIGB
#define FZ_HIST_BIGB 2048
#endif
constexpr unsigned kHistBigBlocks = FZ_HIST_BIGB;  // (sorts of >= 4 M keys)
constexpr int kOsGroup = 8;  // tiles per look-back group (one {tiles, sum} word per group and digit)

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void k_onesweep_hist(const KeyT *__restrict__ keys, int64_t n_cap, int npass,
                                                          unsigned long long *__restrict__ ghist,
                                                          unsigned long long *__restrict__ gsum, int64_t gsum_words,
                                                          const int64_t *__restrict__ d_live) {
    __shared__ uint32_t s_h[kOsMaxPasses][kRadix];
    const int64_t n = d_live && *d_live < n_cap ? *d_live : n_cap;  // (live-bounded sorts: the first *d_live keys)
    // the passes' look-back group sums start from zero (this launch precedes every pass)
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < gsum_words; i += int64_t(gridDim.x) * kBlock)
        gsum[i] = 0ull;
    for (int i = threadIdx.x; i < kOsMaxPasses * kRadix; i += kBlock) (&s_h[0][0])[i] = 0u;
    __syncthreads();
    // (kHistUnroll keys per thread loaded before any is counted: one memory round trip per group
    // of keys - with one key per iteration the loop waited on every load, 0.8 TB/s at 12.5 M keys)
    constexpr int kHistUnroll = 8;
    const int64_t stride = int64_t(gridDim.x) * kBlock;
    for (int64_t i0 = int64_t(blockIdx.x) * kBlock + threadIdx.x; i0 - threadIdx.x < n; i0 += stride * kHistUnroll) {
      uint64_t kk[kHistUnroll];
#pragma unroll
      for (int u = 0; u < kHistUnroll; ++u) {
          const int64_t i = i0 + u * stride;
          kk[u] = i < n ? uint64_t(keys[i]) : 0ull;
      }
#pragma unroll
      for (int u = 0; u < kHistUnroll; ++u) {
        const int64_t i = i0 + u * stride;
        if (i - threadIdx.x >= n) break;  // (wave-uniform: whole waves past the end stop together)
        const bool valid = i < n;
        const uint64_t k = kk[u];
        for (int p = 0; p < npass; ++p) {
            const uint32_t d = uint32_t(k >> (p * kRadixBits)) & (kRadix - 1);
            // wave-uniform digit (typical for the high digits): one add instead of 64 conflicting
            const uint32_t d0 = __shfl(d, 0, 64);
            const uint64_t act = __ballot(valid);
            if (__ballot(valid && d == d0) == act) {
                if (lane_id() == 0 && act) atomicAdd(&s_h[p][d0], uint32_t(__popcll(act)));
            } else if (p == npass - 1 && npass > 1) {
                // the top digit of a narrow key (a project prefix of 11-14 bits: a few values per
                // wave) - one add per distinct digit; per-lane adds to the same few counters
                // serialised (config 3's eighth: 63 us for 12.5 M keys)
                const uint64_t peers = match_digit<kRadixBits>(d, valid);
                if (valid && (__ffsll((long long)peers) - 1) == lane_id()) atomicAdd(&s_h[p][d], uint32_t(__popcll(peers)));
            } else if (valid) {
                atomicAdd(&s_h[p][d], 1u);
            }
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * kRadix; i += kBlock) {
        const uint32_t v = (&s_h[0][0])[i];
        if (v) atomicAdd(&ghist[i], (unsigned long long)v);
    }
}

#ifdef FZ_OS_TIMING
// experiment builds only: wall-clock (100 MHz) phase stamps of three tiles of the last launch
__device__ unsigned long long g_os_t[3][8];
__device__ unsigned long long g_os_first;
#define OS_STAMP(ph)                                                                        \
    do {                                                                                    \
        if (tid == 0) {                                                                     \
            const int sl = tile == 0 ? 0 : (tile == int64_t(gridDim.x) / 2 ? 1 : (tile == int64_t(gridDim.x) - 1 ? 2 : -1)); \
            if (sl >= 0) g_os_t[sl][ph] = wall_clock64();                                   \
        }                                                                                   \
    } while (0)
extern "C" int fz_debug_os_timing(unsigned long long *out) {
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_os_t), sizeof(g_os_t));
    hipMemcpyFromSymbol(out + 24, HIP_SYMBOL(g_os_first), sizeof(g_os_first));
    unsigned long long big = ~0ull;
    hipMemcpyToSymbol(HIP_SYMBOL(g_os_first), &big, sizeof(big));
    return 0;
}
#else
#define OS_STAMP(ph) do {} while (0)
#endif

// One payload column of a radix pass (HAS_PL): the tile's values staged in LDS at their keys'
// digit-sorted slots, then written out in the same per-digit runs as the keys (coalesced).
// (pre: column 0's values, loaded with the keys before the ranking - its load latency hides
// behind the ranking and the look-back - or null: loaded here)
template <typename T, int ITEMS, int BLOCK>
__device__ inline void onesweep_move(const T *__restrict__ in, T *__restrict__ out, T *s, const uint16_t *lpos,
                                     const int32_t *gp, int64_t wbase, int lane, int64_t n, int64_t valid_n, int tid,
                                     const uint64_t *pre = nullptr) {
    T x[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const int64_t idx = wbase + r * kWave + lane;
        x[r] = pre ? T(pre[r]) : (idx < n ? in[idx] : T(0));
    }
    __syncthreads();  // the previous column (or the keys) has left the LDS
#pragma unroll
    for (int r = 0; r < ITEMS; ++r)
        if (wbase + r * kWave + lane < n) s[lpos[r]] = x[r];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < ITEMS; ++m) {
        const int i = tid + m * BLOCK;
        if (i < valid_n) out[gp[m]] = s[i];
    }
}

// One tile of a radix pass (k_onesweep: one sort; k_onesweep_tabs: a tile of one of up to three
// tables' sorts in a shared launch).  The LDS arrays are the caller's (static __shared__ in the
// kernels: one set per workgroup).
template <typename KeyT, bool HAS_VALS, int TILE, int BLOCK>
struct OsShared {
    static constexpr int WAVES = BLOCK / kWave;
    uint64_t stage[TILE];  // the keys, then 8-byte payload columns
    uint32_t vals[HAS_VALS ? TILE : 1];
    uint32_t run[kRadix];
    uint32_t wcnt[WAVES][kRadix];
    uint32_t start[kRadix];
    int64_t goff[kRadix];
    uint32_t tmp[WAVES];
    int64_t tmp64[WAVES];
};

template <typename KeyT, bool HAS_VALS, bool HAS_PL, int TILE, int BLOCK>
__device__ __forceinline__ void onesweep_tile(OsShared<KeyT, HAS_VALS, TILE, BLOCK> &sh, const int64_t tile,
                                              const KeyT *__restrict__ keys_in, const uint32_t *__restrict__ vals_in,
                                              KeyT *__restrict__ keys_out, uint32_t *__restrict__ vals_out, int64_t n,
                                              int shift, const int64_t gcount, uint64_t *__restrict__ status,
                                              uint64_t epoch, unsigned long long *__restrict__ gsum,
                                              const RadixPayload &pl, const uint8_t *__restrict__ type_src = nullptr,
                                              int type_shift = 0) {
    constexpr int ITEMS = TILE / BLOCK, WAVES = BLOCK / kWave;
    KeyT *const s_keys = reinterpret_cast<KeyT *>(sh.stage);
    uint64_t *const s_stage = sh.stage;
    uint32_t *const s_vals = sh.vals;
    uint32_t *const s_run = sh.run;
    uint32_t(*const s_wcnt)[kRadix] = sh.wcnt;
    uint32_t *const s_start = sh.start;
    int64_t *const s_goff = sh.goff;
    uint32_t *const s_tmp = sh.tmp;
    int64_t *const s_tmp64 = sh.tmp64;
    const int tid = threadIdx.x;
    const int w = wave_id(), lane = lane_id();
    const bool dig = tid < kRadix;  // threads [0, 256) own one digit each after the ranking
    const int64_t base = tile * TILE;
#ifdef FZ_OS_TIMING
    if (tid == 0) atomicMin(&g_os_first, (unsigned long long)wall_clock64());
#endif
    OS_STAMP(0);
    // wave w owns the contiguous slice [w * T/W, (w + 1) * T/W) of the tile; round r covers
    // its keys r * 64 + lane, so (wave, round, lane) is position order and ranking is stable with
    // wave-private digit counters - no workgroup barrier inside the ranking loop
    const int64_t wbase = base + int64_t(w) * (TILE / WAVES);

    KeyT k[ITEMS];
    uint32_t v[ITEMS];
    uint32_t rank[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const int64_t idx = wbase + r * kWave + lane;
        const bool valid = idx < n;
        k[r] = valid ? keys_in[idx] : KeyT(0);
        // (type_src: the key is [type |] project, made here from the two columns - the builds'
        // (Fuzzing 0, Coverage 1, any other type 2) << pbits | project of the store's prefix sort)
        if (type_src && valid) {
            const uint32_t ty = type_src[idx];
            k[r] |= KeyT(ty > 1u ? 2u : ty) << type_shift;
        }
        // (no vals_in: the values are the keys' positions - a sort's first pass over row ids)
        v[r] = (HAS_VALS && valid) ? (vals_in ? vals_in[idx] : uint32_t(idx)) : 0u;
    }
#if FZ_OS_PREFETCH
    // the first payload column in flight with the keys
    constexpr bool kPre = HAS_PL;
    uint64_t p0[kPre ? ITEMS : 1];
    if constexpr (kPre) {
        const int sz0 = pl.n > 0 ? pl.size[0] : 0;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const int64_t idx = wbase + r * kWave + lane;
            p0[r] = 0ull;
            if (idx < n) {
                if (sz0 == 8) p0[r] = static_cast<const uint64_t *>(pl.in[0])[idx];
                else if (sz0 == 4) p0[r] = static_cast<const uint32_t *>(pl.in[0])[idx];
                else if (sz0 == 1) p0[r] = static_cast<const uint8_t *>(pl.in[0])[idx];
            }
        }
    }
#else
    constexpr bool kPre = false;
    const uint64_t *p0 = nullptr;
#endif
    uint32_t *cnt_w = s_wcnt[w];
#ifdef FZ_OS_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    OS_STAMP(6);
#endif
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const bool valid = wbase + r * kWave + lane < n;
        const uint32_t d = uint32_t(k[r] >> shift) & (kRadix - 1);
        const uint64_t peers = match_digit<kRadixBits>(d, valid);
        const uint32_t before = valid ? cnt_w[d] : 0u;  // all lanes read before the leader writes
        rank[r] = before + uint32_t(__popcll(peers & lanemask_lt()));
        if (valid && (__ffsll((long long)peers) - 1) == lane) cnt_w[d] = before + uint32_t(__popcll(peers));
    }
    __syncthreads();
    OS_STAMP(1);
    // digit tid: tile count and per-wave exclusive offsets (stored back into s_wcnt)
    uint32_t cnt = 0;
    uint64_t *my = &status[tile * kRadix + (dig ? tid : 0)];
    if (dig) {
        for (int i = 0; i < WAVES; ++i) {
            const uint32_t x = s_wcnt[i][tid];
            s_wcnt[i][tid] = cnt;
            cnt += x;
        }
        s_run[tid] = cnt;
        // publish this tile's count of digit tid (own word + its group's {tiles:16, sum:48} word),
        // then look back for the counts of all earlier tiles
        __hip_atomic_store(my, (tile == 0 ? kLbInc : kLbAgg) | epoch | uint64_t(cnt), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&gsum[(tile / kOsGroup) * kRadix + tid], (1ull << 48) | (unsigned long long)cnt,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t tstart = block_excl_scan<uint32_t, WAVES>(cnt, s_tmp, (uint32_t *)nullptr);
    if (dig) s_start[tid] = tstart;  // visible to the scatter after the next scan's barriers
    const int64_t gstart = block_excl_scan<int64_t, WAVES>(gcount, s_tmp64, (int64_t *)nullptr);
    OS_STAMP(2);
    int64_t prefix = 0;
    // (1) the earlier tiles of this tile's group one by one, nearest first, up to an inclusive word
    const int64_t g0 = (tile / kOsGroup) * kOsGroup;
    bool found = tile == 0;
    for (int64_t q = tile - 1; dig && !found && q >= g0;) {
        uint64_t sw[kOsGroup - 1];
#pragma unroll
        for (int j = 0; j < kOsGroup - 1; ++j)
            sw[j] = q - j >= g0 ? __hip_atomic_load(&status[(q - j) * kRadix + tid], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : 0ull;
        int j = 0;
        for (; j < kOsGroup - 1 && q - j >= g0; ++j) {
            const uint64_t x = sw[j];
            if ((x & kLbEpochMask) != epoch || !(x & kLbFlags)) break;  // not published yet
            prefix += int64_t(x & kLbVal);
            if ((x & kLbFlags) == kLbInc) {
                found = true;
                break;
            }
        }
        if (found) break;
        q -= j;
        if (q >= g0) __builtin_amdgcn_s_sleep(1);
    }
    // (2) whole earlier groups, nearest first: a group's last tile's inclusive word ends the walk,
    // else its sum word once all of its tiles have added (traffic O(tiles / group))
    for (int64_t G = g0 / kOsGroup - 1; dig && !found && G >= 0;) {
        uint64_t lw[kOsWindow], gw[kOsWindow];
#pragma unroll
        for (int j = 0; j < kOsWindow; ++j) {
            const bool ok = G - j >= 0;
            lw[j] = ok ? __hip_atomic_load(&status[((G - j) * kOsGroup + kOsGroup - 1) * kRadix + tid],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0ull;
            gw[j] = ok ? __hip_atomic_load(&gsum[(G - j) * kRadix + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0ull;
        }
        int j = 0;
        for (; j < kOsWindow && G - j >= 0; ++j) {
            const uint64_t x = lw[j];
            if ((x & kLbEpochMask) == epoch && (x & kLbFlags) == kLbInc) {
                prefix += int64_t(x & kLbVal);
                found = true;
                break;
            }
            if ((gw[j] >> 48) != uint64_t(kOsGroup)) break;  // a tile of the group has not added yet
            prefix += int64_t(gw[j] & kLbVal);
        }
        if (found) break;
        G -= j;
        if (G >= 0 && j < kOsWindow) __builtin_amdgcn_s_sleep(1);
    }
    if (dig) {
        if (tile > 0)
            __hip_atomic_store(my, kLbInc | epoch | uint64_t(prefix + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_goff[tid] = gstart + prefix - int64_t(tstart);
    }
    OS_STAMP(3);
    // stage the tile digit-sorted in LDS, then write it out in per-digit runs
    uint16_t lpos[HAS_PL ? ITEMS : 1];  // HAS_PL: LDS slot of item r
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const int64_t idx = wbase + r * kWave + lane;
        if (idx < n) {
            const uint32_t d = uint32_t(k[r] >> shift) & (kRadix - 1);
            const uint32_t pos = s_start[d] + cnt_w[d] + rank[r];
            s_keys[pos] = k[r];
            if (HAS_VALS) s_vals[pos] = v[r];
            if (HAS_PL) lpos[r] = uint16_t(pos);
        }
    }
    __syncthreads();
    OS_STAMP(4);
    const int64_t valid_n = (n - base) < TILE ? (n - base) : TILE;
    int32_t gp[HAS_PL ? ITEMS : 1];  // HAS_PL: output position of LDS slot tid + m * BLOCK
#pragma unroll
    for (int m = 0; m < ITEMS; ++m) {
        const int i = tid + m * BLOCK;
        if (i < valid_n) {
            const KeyT kk = s_keys[i];
            const uint32_t d = uint32_t(kk >> shift) & (kRadix - 1);
            const int64_t gpos = s_goff[d] + i;
#ifdef FZ_OS_EXPERIMENT_NOWRITE
            if (gpos < 0)
#endif
            {
                keys_out[gpos] = kk;
                if (HAS_VALS) vals_out[gpos] = s_vals[i];
            }
            if (HAS_PL) gp[m] = int32_t(gpos);
        }
    }
    if (HAS_PL) {
        // the payload columns follow their keys through the same LDS slots and per-digit runs
        for (int j = 0; j < pl.n; ++j) {
            const uint64_t *pre = kPre && j == 0 ? p0 : nullptr;
            if (pl.size[j] == 8)
                onesweep_move<uint64_t, ITEMS, BLOCK>(static_cast<const uint64_t *>(pl.in[j]), static_cast<uint64_t *>(pl.out[j]),
                                        s_stage, lpos, gp, wbase, lane, n, valid_n, tid, pre);
            else if (pl.size[j] == 4)
                onesweep_move<uint32_t, ITEMS, BLOCK>(static_cast<const uint32_t *>(pl.in[j]), static_cast<uint32_t *>(pl.out[j]),
                                        reinterpret_cast<uint32_t *>(s_stage), lpos, gp, wbase, lane, n, valid_n, tid,
                                        pre);
            else
                onesweep_move<uint8_t, ITEMS, BLOCK>(static_cast<const uint8_t *>(pl.in[j]), static_cast<uint8_t *>(pl.out[j]),
                                       reinterpret_cast<uint8_t *>(s_stage), lpos, gp, wbase, lane, n, valid_n, tid,
                                       pre);
        }
    }
#ifdef FZ_OS_TIMING
    __syncthreads();
    OS_STAMP(5);
#endif
}

// KeyT: uint64_t, or uint32_t for keys of at most 32 bits (the prefix / session-index transposes:
// 4 bytes per key less to read and write in every pass)
template <typename KeyT, bool HAS_VALS, bool HAS_PL, int TILE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_onesweep(const KeyT *__restrict__ keys_in,
                                                     const uint32_t *__restrict__ vals_in,
                                                     KeyT *__restrict__ keys_out, uint32_t *__restrict__ vals_out,
                                                     int64_t n, int shift, const unsigned long long *__restrict__ ghist,
                                                     uint64_t *__restrict__ status, unsigned int *__restrict__ ticket,
                                                     uint64_t epoch,
                                                     unsigned long long *__restrict__ gsum,
                                                     unsigned long long *__restrict__ next_hist,
                                                     RadixPayload pl, const int64_t *__restrict__ d_live) {
    static_assert(BLOCK >= kRadix && TILE % BLOCK == 0 && TILE <= 65536, "radix pass shape");
    __shared__ OsShared<KeyT, HAS_VALS, TILE, BLOCK> sh;
    __shared__ unsigned int s_tile;
    const int tid = threadIdx.x;
    if (tid == 0) s_tile = lb_take_tile(ticket, gridDim.x);
    const bool dig = tid < kRadix;
    if (next_hist && blockIdx.x == 0)  // the next sort's digit totals start from zero
        for (int i = tid; i < kOsMaxPasses * kRadix; i += BLOCK) next_hist[i] = 0ull;
    for (int i = tid; i < OsShared<KeyT, HAS_VALS, TILE, BLOCK>::WAVES * kRadix; i += BLOCK) (&sh.wcnt[0][0])[i] = 0;
    const int64_t gcount = dig ? int64_t(ghist[tid]) : 0;  // issued early: consumed after the ranking
    // live-bounded sorts (d_live): only the first *d_live keys are sorted; the tiles past them leave
    // after drawing their ticket (no later tile looks back at them), the entries past them untouched
    if (d_live && *d_live < n) n = *d_live > 0 ? *d_live : 0;
    __syncthreads();
    const int64_t tile = s_tile;
    if (tile * TILE >= n) return;
    onesweep_tile<KeyT, HAS_VALS, HAS_PL, TILE, BLOCK>(sh, tile, keys_in, vals_in, keys_out, vals_out, n, shift, gcount,
                                                       status, epoch, gsum, pl);
}

// ---- up to three tables' sorts in shared launches (the store's prefix sorts) ----------------
// One histogram launch counts every table's digits (table k's workgroups [hb[k], hb[k + 1])), then
// each pass is ONE launch over all tables that have that digit: tile t of the launch (ticket order)
// is tile t - tile0[k] of table k, which looks back only over its own table's tiles (their own
// status words and group sums) - three sorts' launch latencies and look-back tails become one.
constexpr int kOsMaxTabs = 3;
static_assert(kRadixTabHistWords == kOsMaxTabs * kOsMaxPasses * kRadix, "fz_internal.h kRadixTabHistWords");
struct OsTab {
    const uint32_t *keys_in = nullptr;
    const uint32_t *vals_in = nullptr;  // null: the keys' positions (a first pass over row ids)
    uint32_t *keys_out = nullptr;
    uint32_t *vals_out = nullptr;
    int64_t n = 0;
    int npass = 0;
    const unsigned long long *ghist = nullptr;  // [npass][kRadix] digit totals (zeroed before the histogram)
    unsigned long long *gsum = nullptr;         // [npass][groups][kRadix] look-back group sums
    int64_t gwords = 0;                         // groups * kRadix
    uint64_t *status = nullptr;                 // this table's (tile, digit) status words
    const uint8_t *type_src = nullptr;          // (first pass / histogram) key |= min(type, 2) << type_shift
    int type_shift = 0;
    RadixPayload pl;
};
struct OsTabs {
    OsTab t[kOsMaxTabs];
    RadixSideMinMax side;  // (histogram launch) blocks [hb[nt], hb[nt] + side.blocks): its partials
    int nt = 0;
    int64_t tile0[kOsMaxTabs + 1] = {0, 0, 0, 0};  // (pass launches) global tile range of table k
    unsigned hb[kOsMaxTabs + 1] = {0, 0, 0, 0};    // (histogram launch) workgroup range of table k
};

__global__ __launch_bounds__(kBlock) void k_onesweep_hist_tabs(const OsTabs T) {
    __shared__ uint32_t s_h[kOsMaxPasses][kRadix];
    if (blockIdx.x >= T.hb[T.nt]) {
        // the side job: min / max of an int64 column skipping FZ_TS_NULL, per-workgroup partials
        // part[4 * b + {2, 3}] (the store's issue-number range; one launch fewer than its own)
        __shared__ int64_t s_lo[kBlock / kWave], s_hi[kBlock / kWave];
        const RadixSideMinMax &sd = T.side;
        const unsigned b = blockIdx.x - T.hb[T.nt];
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int64_t i = int64_t(b) * kBlock + threadIdx.x; i < sd.n; i += int64_t(sd.blocks) * kBlock) {
            const int64_t v = sd.src[i];
            if (v == FZ_TS_NULL) continue;
            lo = v < lo ? v : lo;
            hi = v > hi ? v : hi;
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane_id() == 0) {
            s_lo[wave_id()] = lo;
            s_hi[wave_id()] = hi;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < kBlock / kWave; ++w) {
                lo = s_lo[w] < lo ? s_lo[w] : lo;
                hi = s_hi[w] > hi ? s_hi[w] : hi;
            }
            sd.part[4 * b + 2] = lo;
            sd.part[4 * b + 3] = hi;
        }
        return;
    }
    int k = 0;
    while (k + 1 < T.nt && blockIdx.x >= T.hb[k + 1]) ++k;
    const OsTab &tb = T.t[k];
    const unsigned blk = blockIdx.x - T.hb[k], nblk = T.hb[k + 1] - T.hb[k];
    const int npass = tb.npass;
    const int64_t n = tb.n;
    const uint32_t *keys = tb.keys_in;
    unsigned long long *gh = const_cast<unsigned long long *>(tb.ghist);
    // (this launch precedes every pass: the passes' group sums start from zero)
    for (int64_t i = int64_t(blk) * kBlock + threadIdx.x; i < tb.gwords * npass; i += int64_t(nblk) * kBlock)
        tb.gsum[i] = 0ull;
    for (int i = threadIdx.x; i < kOsMaxPasses * kRadix; i += kBlock) (&s_h[0][0])[i] = 0u;
    __syncthreads();
    constexpr int kHistUnroll = 8;
    const int64_t stride = int64_t(nblk) * kBlock;
    for (int64_t i0 = int64_t(blk) * kBlock + threadIdx.x; i0 - threadIdx.x < n; i0 += stride * kHistUnroll) {
        uint32_t kk[kHistUnroll];
#pragma unroll
        for (int u = 0; u < kHistUnroll; ++u) {
            const int64_t i = i0 + u * stride;
            kk[u] = i < n ? keys[i] : 0u;
            if (tb.type_src && i < n) {
                const uint32_t ty = tb.type_src[i];
                kk[u] |= (ty > 1u ? 2u : ty) << tb.type_shift;
            }
        }
#pragma unroll
        for (int u = 0; u < kHistUnroll; ++u) {
            const int64_t i = i0 + u * stride;
            if (i - threadIdx.x >= n) break;  // (wave-uniform)
            const bool valid = i < n;
            for (int p = 0; p < npass; ++p) {
                const uint32_t d = (kk[u] >> (p * kRadixBits)) & (kRadix - 1);
                const uint32_t d0 = __shfl(d, 0, 64);
                const uint64_t act = __ballot(valid);
                if (__ballot(valid && d == d0) == act) {
                    if (lane_id() == 0 && act) atomicAdd(&s_h[p][d0], uint32_t(__popcll(act)));
                } else if (p == npass - 1 && npass > 1) {
                    const uint64_t peers = match_digit<kRadixBits>(d, valid);
                    if (valid && (__ffsll((long long)peers) - 1) == lane_id())
                        atomicAdd(&s_h[p][d], uint32_t(__popcll(peers)));
                } else if (valid) {
                    atomicAdd(&s_h[p][d], 1u);
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * kRadix; i += kBlock) {
        const uint32_t v = (&s_h[0][0])[i];
        if (v) atomicAdd(&gh[i], (unsigned long long)v);
    }
}

template <bool HAS_PL, int TILE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_onesweep_tabs(const OsTabs T, int pass, unsigned int *__restrict__ ticket,
                                                         uint64_t epoch) {
    __shared__ OsShared<uint32_t, true, TILE, BLOCK> sh;
    __shared__ unsigned int s_tile;
    const int tid = threadIdx.x;
    if (tid == 0) s_tile = lb_take_tile(ticket, gridDim.x);
    for (int i = tid; i < OsShared<uint32_t, true, TILE, BLOCK>::WAVES * kRadix; i += BLOCK) (&sh.wcnt[0][0])[i] = 0;
    __syncthreads();
    const int64_t g = s_tile;
    int k = 0;
    while (k + 1 < T.nt && g >= T.tile0[k + 1]) ++k;
    const OsTab &tb = T.t[k];
    const int64_t tile = g - T.tile0[k];
    if (tile * TILE >= tb.n) return;
    const int64_t gcount = tid < kRadix ? int64_t(tb.ghist[pass * kRadix + tid]) : 0;
    onesweep_tile<uint32_t, true, HAS_PL, TILE, BLOCK>(sh, tile, tb.keys_in, tb.vals_in, tb.keys_out, tb.vals_out,
                                                       tb.n, pass * kRadixBits, gcount, tb.status, epoch,
                                                       tb.gsum + pass * tb.gwords, tb.pl,
                                                       pass == 0 ? tb.type_src : nullptr, tb.type_shift);
}

void radix_sort_tables_payload32(fz_ctx *c, RadixTab *tabs, int nt, unsigned long long *hist0,
                                 const RadixSideMinMax *side) {
    FZ_CHECK(nt >= 1 && nt <= kOsMaxTabs, "radix_sort_tables: 1..3 tables");
    int64_t nmax = 0, ntot = 0;
    int npass_max = 0;
    for (int k = 0; k < nt; ++k) {
        RadixTab &r = tabs[k];
        FZ_CHECK(r.bits >= 0 && r.bits <= 32 && r.n >= 0 && r.n < (int64_t(1) << 31) && (r.n == 0 || r.vals) &&
                     (!r.type_src || r.key_src),
                 "radix_sort_tables: bad table");
        r.npass = (r.n > 1 && r.bits > 0) ? (r.bits + kRadixBits - 1) / kRadixBits : 0;
        if (r.npass == 0) {  // unmoved (at most one key or a 0-bit key)
            FZ_CHECK(!r.key_src, "radix sort from a read-only key source needs a pass");
            for (int j = 0; j < r.pl.n; ++j) r.pl.out[j] = const_cast<void *>(r.pl.in[j]);
        }
        nmax = r.n > nmax ? r.n : nmax;
        ntot += r.npass ? r.n : 0;
        npass_max = r.npass > npass_max ? r.npass : npass_max;
    }
    if (npass_max == 0) {
        FZ_CHECK(!side || side->blocks == 0, "radix_sort_tables: a side job needs a sort");
        return;
    }
    const bool big = nmax >= kOsBigN;
    const int64_t tile = big ? kSortTileBig : kSortTile;
    // per table: tiles, look-back groups, the digit totals (hist0: zeroed [nt][kOsMaxPasses][kRadix]),
    // group sums; ping-pong scratch for keys, values and payload columns
    OsTabs T;
    T.nt = nt;
    int64_t nb[kOsMaxTabs] = {}, gw[kOsMaxTabs] = {};
    void *pbuf[kOsMaxTabs][2][kMaxPayload] = {};
    uint32_t *k2[kOsMaxTabs] = {}, *v2[kOsMaxTabs] = {};
    for (int k = 0; k < nt; ++k) {
        RadixTab &r = tabs[k];
        OsTab &o = T.t[k];
        nb[k] = r.npass ? (r.n + tile - 1) / tile : 0;
        gw[k] = ((nb[k] + kOsGroup - 1) / kOsGroup) * kRadix;
        o.n = r.npass ? r.n : 0;
        o.npass = r.npass;
        o.ghist = hist0 + int64_t(k) * kOsMaxPasses * kRadix;
        o.gwords = gw[k];
        o.gsum = r.npass ? c->arena.get<unsigned long long>(gw[k] * r.npass) : nullptr;
        o.keys_in = r.key_src ? r.key_src : r.keys;
        o.type_src = r.type_src;
        o.type_shift = r.type_shift;
        if (!r.npass) continue;
        k2[k] = c->arena.get<uint32_t>(r.n);
        v2[k] = c->arena.get<uint32_t>(r.n);
        for (int j = 0; j < r.pl.n; ++j)
            for (int b = 0; b < 2; ++b) pbuf[k][b][j] = c->arena.alloc(size_t(r.n) * size_t(r.pl.size[j]));
    }
    // histogram: workgroups in proportion to each table's keys
    {
        double hbytes = 0.0;
        unsigned at = 0;
        const unsigned hblocks_all = ntot >= (int64_t(1) << 22) ? kHistBigBlocks : unsigned(kHistMaxBlocks);
        for (int k = 0; k < nt; ++k) {
            T.hb[k] = at;
            if (T.t[k].n > 0) {
                unsigned b = unsigned(double(hblocks_all) * double(T.t[k].n) / double(ntot > 0 ? ntot : 1));
                const unsigned need = unsigned((T.t[k].n + kHistKeysPerBlock - 1) / kHistKeysPerBlock);
                b = b < 1 ? 1 : (b > need ? need : b);
                at += b;
                hbytes += 4.0 * double(T.t[k].n);
            }
        }
        T.hb[nt] = at;
        for (int k = nt + 1; k <= kOsMaxTabs; ++k) T.hb[k] = at;
        if (side) T.side = *side;
        ProbeScope ps(c, "radix_hist", hbytes);
        k_onesweep_hist_tabs<<<at + T.side.blocks, kBlock, 0, c->stream>>>(T);
        FZ_LAUNCH_CHECK();
    }
    // the passes: table k's current keys / values / columns
    const uint32_t *ka[kOsMaxTabs], *va[kOsMaxTabs];
    uint32_t *kb[kOsMaxTabs], *vb[kOsMaxTabs];
    for (int k = 0; k < nt; ++k) {
        RadixTab &r = tabs[k];
        ka[k] = r.key_src ? r.key_src : r.keys;
        va[k] = r.key_src ? nullptr : r.vals;
        kb[k] = k2[k];
        vb[k] = v2[k];
    }
    int passes = 0;
    for (int p = 0; p < npass_max; ++p) {
        OsTabs P = T;
        int64_t tiles = 0;
        double bytes = 0.0;
        bool any_pl = false;
        for (int k = 0; k < nt; ++k) {
            RadixTab &r = tabs[k];
            OsTab &o = P.t[k];
            P.tile0[k] = tiles;
            if (p >= r.npass) {  // (this table's sort has no such digit: no tiles in this launch)
                o.n = 0;
                continue;
            }
            o.keys_in = ka[k];
            o.vals_in = va[k];
            o.keys_out = kb[k];
            o.vals_out = vb[k];
            o.pl = r.pl;
            for (int j = 0; j < r.pl.n; ++j) {
                o.pl.in[j] = p == 0 ? r.pl.in[j] : pbuf[k][(p - 1) & 1][j];
                o.pl.out[j] = pbuf[k][p & 1][j];
            }
            any_pl = any_pl || r.pl.n > 0;
            tiles += nb[k];
            bytes += (16.0 + 2.0 * r.pl.bytes()) * double(r.n);
        }
        for (int k = nt; k <= kOsMaxTabs; ++k) P.tile0[k] = tiles;
        P.tile0[nt] = tiles;
        const Lookback lb = lookback_begin(c, tiles * kRadix);
        for (int k = 0; k < nt; ++k) P.t[k].status = lb.status + P.tile0[k] * kRadix;
        {
            ProbeScope ps(c, "radix_scatter", bytes);
            if (big) {
                if (any_pl) k_onesweep_tabs<true, kSortTileBig, kOsBlockBig><<<unsigned(tiles), kOsBlockBig, 0, c->stream>>>(P, p, lb.ticket, lb.epoch);
                else k_onesweep_tabs<false, kSortTileBig, kOsBlockBig><<<unsigned(tiles), kOsBlockBig, 0, c->stream>>>(P, p, lb.ticket, lb.epoch);
            } else {
                if (any_pl) k_onesweep_tabs<true, kSortTile, kOsBlock><<<unsigned(tiles), kOsBlock, 0, c->stream>>>(P, p, lb.ticket, lb.epoch);
                else k_onesweep_tabs<false, kSortTile, kOsBlock><<<unsigned(tiles), kOsBlock, 0, c->stream>>>(P, p, lb.ticket, lb.epoch);
            }
            FZ_LAUNCH_CHECK();
        }
        lookback_end(c, tiles);
        ++passes;
        for (int k = 0; k < nt; ++k) {
            RadixTab &r = tabs[k];
            if (p >= r.npass) continue;
            if (p == 0 && r.key_src) {  // (the source is never written: the caller's buffers take its place)
                ka[k] = kb[k];
                va[k] = vb[k];
                kb[k] = r.keys;
                vb[k] = r.vals;
            } else {
                const uint32_t *tk = ka[k], *tv = va[k];
                ka[k] = kb[k];
                va[k] = vb[k];
                kb[k] = const_cast<uint32_t *>(tk);
                vb[k] = const_cast<uint32_t *>(tv);
            }
        }
    }
    for (int k = 0; k < nt; ++k) {
        RadixTab &r = tabs[k];
        if (!r.npass) continue;
        r.keys = const_cast<uint32_t *>(ka[k]);
        r.vals = const_cast<uint32_t *>(va[k]);
        for (int j = 0; j < r.pl.n; ++j) r.pl.out[j] = pbuf[k][(r.npass - 1) & 1][j];
    }
    c->sort_passes += passes;
}

void radix_sort_pairs(fz_ctx *c, uint64_t *keys, uint32_t *vals, int64_t n, int bits) {
    uint64_t *k = keys;
    uint32_t *v = vals;
    radix_sort_pairs_swap(c, k, v, n, bits);
    if (k != keys) {
        dev_copy(c, keys, k, n * int64_t(sizeof(uint64_t)));
        if (vals) dev_copy(c, vals, v, n * int64_t(sizeof(uint32_t)));
    }
}

void radix_sort_pairs_swap(fz_ctx *c, uint64_t *&keys, uint32_t *&vals, int64_t n, int bits) {
    RadixPayload none;
    radix_sort_pairs_payload(c, keys, vals, n, bits, none);
}


// key_src (optional): the first pass reads the keys from this read-only array (never written; the
// passes ping-pong between two scratch buffers) and takes the values as the keys' positions (vals
// must be non-null: set to the result buffer) - no key / row-id copy made beforehand.
template <typename KeyT>
static void radix_payload_impl(fz_ctx *c, KeyT *&keys, uint32_t *&vals, int64_t n, int bits, RadixPayload &pl,
                               const int64_t *d_live = nullptr, const KeyT *key_src = nullptr) {
    if (n <= 1 || bits <= 0) {  // nothing to sort (one key, or a 0-bit key: one project): unmoved
        FZ_CHECK(!key_src, "radix sort from a read-only key source needs a pass");
        for (int j = 0; j < pl.n; ++j) pl.out[j] = const_cast<void *>(pl.in[j]);
        return;
    }
    const int npass = (bits + kRadixBits - 1) / kRadixBits;
    // large sorts (the 100 M-row tables) take 8192-key tiles of 1024 threads: per-digit runs twice
    // as long per tile (fewer partial-line writes) and half the look-back work (same-box A/B: c3
    // 20.5 -> 20.0 ms, c5 30.7 -> 30.0); the small sorts of config 2 keep 4096 x 512
    const bool big = n >= kOsBigN;
    const bool np = !big && pl.n == 0 && kSortTileNp != kSortTile;  // (the no-payload tile shape)
    const int64_t tile = big ? kSortTileBig : (np ? kSortTileNp : kSortTile);
    const int64_t nb = (n + tile - 1) / tile;
    FZ_CHECK(n < (int64_t(1) << 47), "radix_sort_pairs: too many keys");
    // digit totals of every pass (one read of the keys)
    constexpr int64_t kHistWords = kOsMaxPasses * kRadix;
    if (c->os_hist_cur < 0) {  // first sort of the context (or after a sort that ran no pass)
        unsigned long long *h2 = c->os_hist.ensure<unsigned long long>(2 * kHistWords);
        dev_fill(c, h2, 0, int64_t(sizeof(unsigned long long)) * 2 * kHistWords);
        c->os_hist_cur = 0;
    }
    if (trace_on())
        std::fprintf(stderr, "[fz] ctx %p radix n %lld bits %d hist_cur %d hist %p\n", (void *)c, (long long)n, bits,
                     c->os_hist_cur, c->os_hist.ptr);
    unsigned long long *ghist = c->os_hist.as<unsigned long long>() + c->os_hist_cur * kHistWords;
    unsigned long long *next_hist = c->os_hist.as<unsigned long long>() + (1 - c->os_hist_cur) * kHistWords;
    const int64_t ngroups = (nb + kOsGroup - 1) / kOsGroup;
    const int64_t gwords = ngroups * kRadix;  // per pass
    unsigned long long *gsum = c->arena.get<unsigned long long>(gwords * npass);
    {
        ProbeScope ps(c, "radix_hist", 8.0 * double(n));
        // (sorts of up to 4 M keys: at most 256 workgroups - each adds its npass x 256 digit counts
        // with global atomics, and more workgroups' adds serialised on those words; larger sorts
        // keep 2,048, the occupancy their streaming needs: capped at 256, configs 3 / 5 took 13.9 /
        // 19.4 ms instead of 13.1 / 17.8, same box)
        const unsigned hblocks = n >= (int64_t(1) << 22) ? kHistBigBlocks : unsigned(kHistMaxBlocks);
        k_onesweep_hist<KeyT><<<grid_for(n, kHistKeysPerBlock, hblocks), kBlock, 0, c->stream>>>(
            key_src ? key_src : keys, n, npass, ghist, gsum, gwords * npass, d_live);
        FZ_LAUNCH_CHECK();
    }
    // Constant-digit passes are identity permutations.  Finding them needs a host round trip, which
    // stalls the stream for longer than a pass over a few million keys takes: only large sorts
    // (>= 4 M keys, where one pass costs ~0.1 ms or more) skip them - not while a graph is being
    // recorded (no host round trip can happen then: every pass is recorded) - and not when the
    // caller says the digits all vary (pl.no_digit_probe: the store's project-prefix sorts, where
    // the round trip would stall the stream for a pass it never saves).
    bool need[kOsMaxPasses];
    for (int p = 0; p < npass; ++p) need[p] = true;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    FZ_HIP(hipStreamIsCapturing(c->stream, &cap));
    if (n >= (int64_t(1) << 22) && !pl.no_digit_probe && !key_src && cap == hipStreamCaptureStatusNone) {
        unsigned long long *hh = reinterpret_cast<unsigned long long *>(c->h_pinned);
        FZ_HIP(hipMemcpyAsync(hh, ghist, sizeof(unsigned long long) * npass * kRadix, hipMemcpyDeviceToHost,
                              c->stream));
        sync(c);
        for (int p = 0; p < npass; ++p) {
            int nz = 0;
            for (int d = 0; d < kRadix; ++d) nz += hh[p * kRadix + d] != 0;
            need[p] = nz > 1;
        }
    }
    KeyT *k2 = c->arena.get<KeyT>(n);
    uint32_t *v2 = vals ? c->arena.get<uint32_t>(n) : nullptr;
    KeyT *ka = keys, *kb = k2;
    uint32_t *va = vals, *vb = v2;
    if (key_src) {  // first pass: the source keys and implicit positions -> k2 / v2; then k2 <-> keys
        FZ_CHECK(vals != nullptr, "radix sort from a key source: a value buffer is required");
        ka = const_cast<KeyT *>(key_src);
        va = nullptr;
    }
    bool first = true;
    FZ_CHECK(pl.n == 0 || n < (int64_t(1) << 31), "radix_sort_pairs_payload: payload sorts are limited to 2^31 keys");
    void *pbuf[2][kMaxPayload] = {};
    for (int j = 0; j < pl.n; ++j)  // two scratch copies per column: the passes ping-pong them
        for (int b = 0; b < 2; ++b) pbuf[b][j] = c->arena.alloc(size_t(n) * size_t(pl.size[j]));
    int ppass = 0;  // payload passes run: the current columns are pl.in (0) or pbuf[(ppass - 1) & 1]
    int passes = 0;
    for (int p = 0; p < npass; ++p) {
        if (!need[p]) continue;
        const Lookback lb = lookback_begin(c, nb * kRadix);  // (tile, digit) status words
        RadixPayload step = pl;
        for (int j = 0; j < pl.n; ++j) {
            step.in[j] = ppass == 0 ? pl.in[j] : pbuf[(ppass - 1) & 1][j];
            step.out[j] = pbuf[ppass & 1][j];
        }
        {
            // algorithmic traffic of one pass: read + write every key (8 B), value (4 B) and payload
            ProbeScope ps(c, "radix_scatter", (2.0 * sizeof(KeyT) + (vals ? 8.0 : 0.0) + 2.0 * pl.bytes()) * double(n));
#define FZ_OS_LAUNCH(V, PL)                                                                                   \
    do {                                                                                                      \
        if (big)                                                                                              \
            k_onesweep<KeyT, V, PL, kSortTileBig, kOsBlockBig><<<unsigned(nb), kOsBlockBig, 0, c->stream>>>(   \
                ka, va, kb, vb, n, p * kRadixBits, ghist + p * kRadix, lb.status, lb.ticket, lb.epoch,          \
                gsum + p * gwords, next_hist, step, d_live);                                                  \
        else if (!PL && np)                                                                                   \
            k_onesweep<KeyT, V, false, kSortTileNp, kOsBlockNp><<<unsigned(nb), kOsBlockNp, 0, c->stream>>>(   \
                ka, va, kb, vb, n, p * kRadixBits, ghist + p * kRadix, lb.status, lb.ticket, lb.epoch,          \
                gsum + p * gwords, next_hist, step, d_live);                                                  \
        else                                                                                                  \
            k_onesweep<KeyT, V, PL, kSortTile, kOsBlock><<<unsigned(nb), kOsBlock, 0, c->stream>>>(            \
                ka, va, kb, vb, n, p * kRadixBits, ghist + p * kRadix, lb.status, lb.ticket, lb.epoch,          \
                gsum + p * gwords, next_hist, step, d_live);                                                  \
    } while (0)
            if (pl.n > 0) {
                if (vals)
                    FZ_OS_LAUNCH(true, true);
                else
                    FZ_OS_LAUNCH(false, true);
            } else if (vals) {
                FZ_OS_LAUNCH(true, false);
            } else {
                FZ_OS_LAUNCH(false, false);
            }
#undef FZ_OS_LAUNCH
            FZ_LAUNCH_CHECK();
        }
        lookback_end(c, nb);
        if (pl.n > 0) ++ppass;
        if (key_src && first) {  // (the source is never written: the caller's buffers take its place)
            ka = kb;
            va = vb;
            kb = keys;
            vb = vals;
        } else {
            std::swap(ka, kb);
            std::swap(va, vb);
        }
        first = false;
        ++passes;
    }
    FZ_CHECK(!key_src || passes > 0, "radix sort from a read-only key source ran no pass");
    keys = ka;  // the buffers holding the result (the inputs or arena scratch)
    vals = va;
    for (int j = 0; j < pl.n; ++j)  // where each payload column ended (unmoved: the input itself)
        pl.out[j] = ppass == 0 ? const_cast<void *>(pl.in[j]) : pbuf[(ppass - 1) & 1][j];
    c->sort_passes += passes;
    // the passes zeroed the other buffer: it serves the next sort; with no pass nothing was zeroed
    c->os_hist_cur = passes > 0 ? 1 - c->os_hist_cur : -1;
}

void radix_sort_pairs_payload(fz_ctx *c, uint64_t *&keys, uint32_t *&vals, int64_t n, int bits, RadixPayload &pl) {
    radix_payload_impl<uint64_t>(c, keys, vals, n, bits, pl);
}
void radix_sort_pairs_swap_live(fz_ctx *c, uint64_t *&keys, uint32_t *&vals, int64_t n_cap, const int64_t *d_live,
                                int bits) {
    RadixPayload none;
    radix_payload_impl<uint64_t>(c, keys, vals, n_cap, bits, none, d_live);
}
void radix_sort_pairs_payload32(fz_ctx *c, uint32_t *&keys, uint32_t *&vals, int64_t n, int bits, RadixPayload &pl) {
    FZ_CHECK(bits <= 32, "radix_sort_pairs_payload32: keys of more than 32 bits");
    radix_payload_impl<uint32_t>(c, keys, vals, n, bits, pl);
}
void radix_sort_pairs_payload32_live(fz_ctx *c, uint32_t *&keys, uint32_t *&vals, int64_t n_cap, const int64_t *d_live,
                                     int bits, RadixPayload &pl) {
    FZ_CHECK(bits <= 32, "radix_sort_pairs_payload32_live: keys of more than 32 bits");
    radix_payload_impl<uint32_t>(c, keys, vals, n_cap, bits, pl, d_live);
}
void radix_sort_rows_payload32(fz_ctx *c, const uint32_t *key_src, uint32_t *&keys, uint32_t *&vals, int64_t n,
                               int bits, RadixPayload &pl) {
    FZ_CHECK(bits <= 32 && bits > 0 && n > 1, "radix_sort_rows_payload32: bad key width or size");
    radix_payload_impl<uint32_t>(c, keys, vals, n, bits, pl, nullptr, key_src);
}

// ----------------------------------------------------------- sample sort of one segment (fp64)
// One segment [0, offs[1]) of up to ~1.3 M doubles (RQ3's detected u non-detected union: ~0.8 M
// values at config 2) sorted stably by (value, position) in five launches instead of the LSD radix
// sort's eleven (keys, histogram, eight 8-bit passes, values) - each of those passes a
// latency-bound look-back over ~200 tiles, ~15 us apart from ~10 us of launch gap:
//  1. one workgroup sorts 2048 strided samples (a bitonic network in registers and shuffles, LDS
//     only for the 10 stages that cross waves) and takes every 16th as a splitter (127);
//  2. every value gets its bucket: 2i for keys strictly between splitters i-1 and i, 2i+1 for
//     keys equal to splitter i (a heavy tie - the zeros - lands whole in an equality bucket, which
//     needs no sort), and the bucket counts (one LDS add per run of equal buckets in a wave);
//  3. one stable onesweep pass over the 8-bit bucket ids (positions implicit, the values as the
//     payload) writes the segment in bucket order straight into val / pos - position order kept
//     inside each bucket, so an equality bucket is already final;
//  4. one workgroup per range bucket sorts it in place in LDS by an LSD radix sort over the key
//     bytes that differ inside the bucket (stable: ties keep position order); a bucket past the
//     LDS capacity (12 K values: sampling noise, or clustered values) is sorted by k_ss_runs as
//     LDS-sorted runs merged by its workgroup in global memory.
// The output is the stable sort's, element for element.
constexpr int kSsSamples = 2048;
constexpr int kSsSplit = 127;
constexpr int kSsBuckets = 2 * kSsSplit + 1;  // 255: bucket ids fit an 8-bit digit
constexpr int kSsBlock = 1024;
constexpr int kSsWaves = kSsBlock / kWave;
constexpr int kSsIpt = 12;
constexpr int kSsMax = kSsBlock * kSsIpt;  // values one workgroup sorts in LDS
static_assert(kSsMax <= 65536, "bucket-local indices are 16-bit");
static_assert(kSsSamples == 2 * kSsBlock, "two samples per thread");

__global__ __launch_bounds__(kSsBlock) void k_ss_splitters(const double *__restrict__ src,
                                                            const int64_t *__restrict__ offs, int64_t n_cap,
                                                            uint64_t *__restrict__ spl,
                                                            unsigned long long *__restrict__ counts,
                                                            unsigned long long *__restrict__ gsum, int64_t gsum_words,
                                                            int64_t *__restrict__ d_hi) {
    chain_prio();
    __shared__ uint64_t s[kSsSamples];
    const int tid = threadIdx.x, lane = lane_id();
    const int64_t hi = offs[1] < n_cap ? (offs[1] > 0 ? offs[1] : 0) : n_cap;
    // (the scatter pass's digit totals and look-back group sums start from zero)
    for (int i = tid; i < 256; i += kSsBlock) counts[i] = 0ull;
    for (int64_t i = tid; i < gsum_words; i += kSsBlock) gsum[i] = 0ull;
    // thread t holds samples 2t, 2t + 1 (strided positions of the segment)
    uint64_t x[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = 2 * tid + h;
        x[h] = hi > 0 ? f64_key(src[(int64_t(j) * hi) / kSsSamples]) : ~0ull;
    }
    // bitonic network: element e = 2t + h; stage (k, j) pairs e with e ^ j, ascending where e & k == 0
    // (unrolled: each stage's kind - in-thread, shuffle or LDS - is resolved at compile time)
#pragma unroll
    for (int k = 2; k <= kSsSamples; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            uint64_t y[2];
            if (j == 1) {
                y[0] = x[1];
                y[1] = x[0];
            } else if ((j >> 1) < kWave) {  // partner thread t ^ (j / 2): same wave
#pragma unroll
                for (int h = 0; h < 2; ++h) y[h] = __shfl_xor(x[h], j >> 1, 64);
            } else {  // across waves: through LDS
                s[2 * tid] = x[0];
                s[2 * tid + 1] = x[1];
                __syncthreads();
#pragma unroll
                for (int h = 0; h < 2; ++h) y[h] = s[(2 * tid + h) ^ j];
                __syncthreads();
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = 2 * tid + h;
                const bool up = (e & k) == 0, low = (e & j) == 0;
                const uint64_t mn = x[h] < y[h] ? x[h] : y[h], mx = x[h] < y[h] ? y[h] : x[h];
                x[h] = (low == up) ? mn : mx;
            }
        }
    }
    s[2 * tid] = x[0];
    s[2 * tid + 1] = x[1];
    __syncthreads();
    if (tid < kSsSplit) spl[tid] = s[(tid + 1) * (kSsSamples / (kSsSplit + 1))];
    if (tid == 0) *d_hi = hi;
    (void)lane;
}

// bucket of key k: 2p + 1 when k equals splitter p, else 2p (p = splitters below k)
__device__ inline uint32_t ss_bucket(const uint64_t *s_spl, uint64_t k) {
    int p = 0;
#pragma unroll
    for (int step = 64; step > 0; step >>= 1)
        if (p + step <= kSsSplit && s_spl[p + step - 1] < k) p += step;
    return (p < kSsSplit && s_spl[p] == k) ? uint32_t(2 * p + 1) : uint32_t(2 * p);
}

__global__ __launch_bounds__(kSsBlock) void k_ss_ids(const double *__restrict__ src, const int64_t *__restrict__ d_hi,
                                                    const uint64_t *__restrict__ spl, uint32_t *__restrict__ ids,
                                                    unsigned long long *__restrict__ counts) {
    __shared__ uint64_t s_spl[kSsSplit];
    __shared__ uint32_t s_h[256];
    for (int i = threadIdx.x; i < kSsSplit; i += kSsBlock) s_spl[i] = spl[i];
    for (int i = threadIdx.x; i < 256; i += kSsBlock) s_h[i] = 0u;
    __syncthreads();
    const int64_t hi = *d_hi;
    constexpr int U = 4;  // values per thread loaded before any is bucketed (loads in flight together)
    const int64_t stride = int64_t(gridDim.x) * kSsBlock;
    for (int64_t i0 = int64_t(blockIdx.x) * kSsBlock + threadIdx.x; i0 - threadIdx.x < hi; i0 += stride * U) {
        double x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = i0 + u * stride < hi ? src[i0 + u * stride] : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i - threadIdx.x >= hi) break;  // (uniform: the workgroup's base)
            const bool valid = i < hi;
            const uint32_t b = valid ? ss_bucket(s_spl, f64_key(x[u])) : 0u;
            if (valid) ids[i] = b;
            // one LDS add per distinct bucket of the wave (the zeros' bucket is a third of the
            // non-detected sample: per-lane adds to it serialised)
            const uint64_t peers = match_digit<8>(b, valid);
            if (valid && (__ffsll((long long)peers) - 1) == lane_id()) atomicAdd(&s_h[b], uint32_t(__popcll(peers)));
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kSsBuckets; i += kSsBlock)
        if (s_h[i]) atomicAdd(&counts[i], (unsigned long long)s_h[i]);
}

// LDS workspace of one bucket sort: keys exchanged as two 32-bit halves
struct SsShared {
    uint32_t x[kSsMax];
    uint16_t ix[kSsMax];
    uint32_t wcnt[kSsWaves][256];
    uint32_t start[256];
    uint32_t tmp[kSsWaves];
    uint64_t orw[kSsWaves];
};

// Stable LSD radix sort of n <= kSsMax (key, index) pairs held in registers, element
// q = ss_q(R, round) = wave * R * 64 + round * 64 + lane for rounds < R = ss_rounds(n): every wave
// holds a run of R * 64 elements, so a bucket of a few thousand keeps all 16 waves busy and the
// rounds past R (no element) are skipped; only the key bytes that differ among the pairs are passes.
__device__ inline int ss_rounds(int n) { return (n + kSsBlock - 1) / kSsBlock; }
__device__ inline int ss_q(int R, int r) { return wave_id() * R * kWave + r * kWave + lane_id(); }
__device__ inline void ss_lds_sort(uint64_t (&k)[kSsIpt], uint16_t (&ix)[kSsIpt], int n, uint64_t kref, SsShared &sh) {
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    const int R = ss_rounds(n);
    const int wbase = w * R * kWave;
    // the bytes that vary: OR of (key ^ kref), kref = one of the keys (the first)
    uint64_t dif = 0;
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r)
        if (r < R && wbase + r * kWave + lane < n) dif |= k[r] ^ kref;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dif |= __shfl_xor(dif, off, 64);
    if (lane == 0) sh.orw[w] = dif;
    __syncthreads();
    dif = 0;
#pragma unroll
    for (int i = 0; i < kSsWaves; ++i) dif |= sh.orw[i];
    for (int byte = 0; byte < 8; ++byte) {
        if (!((dif >> (8 * byte)) & 0xffull)) continue;
        const int shift = 8 * byte;
        for (int i = tid; i < kSsWaves * 256; i += kSsBlock) (&sh.wcnt[0][0])[i] = 0u;
        __syncthreads();
        uint32_t *cnt_w = sh.wcnt[w];
        uint32_t dst[kSsIpt];
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            dst[r] = 0u;
            if (r < R) {  // (uniform: the rounds past R hold no element)
                const bool valid = wbase + r * kWave + lane < n;
                const uint32_t d = uint32_t(k[r] >> shift) & 255u;
                const uint64_t peers = match_digit<8>(d, valid);
                const uint32_t before = valid ? cnt_w[d] : 0u;  // all lanes read before the leader writes
                dst[r] = before + uint32_t(__popcll(peers & lanemask_lt()));
                if (valid && (__ffsll((long long)peers) - 1) == lane) cnt_w[d] = before + uint32_t(__popcll(peers));
            }
        }
        __syncthreads();
        uint32_t tot = 0;
        if (tid < 256)
            for (int i = 0; i < kSsWaves; ++i) {
                const uint32_t x = sh.wcnt[i][tid];
                sh.wcnt[i][tid] = tot;
                tot += x;
            }
        const uint32_t st = block_excl_scan<uint32_t, kSsWaves>(tot, sh.tmp, (uint32_t *)nullptr);
        if (tid < 256) sh.start[tid] = st;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            if (r < R && wbase + r * kWave + lane < n) {
                const uint32_t d = uint32_t(k[r] >> shift) & 255u;
                dst[r] += sh.start[d] + cnt_w[d];
                sh.x[dst[r]] = uint32_t(k[r] >> 32);
                sh.ix[dst[r]] = ix[r];
            }
        }
        __syncthreads();
        // (the high words land in k's high halves at once: the low halves still go out from k)
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            const int q = wbase + r * kWave + lane;
            if (r < R && q < n) {
                k[r] = (uint64_t(sh.x[q]) << 32) | (k[r] & 0xffffffffull);
                ix[r] = sh.ix[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r)
            if (r < R && wbase + r * kWave + lane < n) sh.x[dst[r]] = uint32_t(k[r]);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            const int q = wbase + r * kWave + lane;
            if (r < R && q < n) k[r] = (k[r] & 0xffffffff00000000ull) | sh.x[q];
        }
        __syncthreads();
    }
    __syncthreads();  // (no pass: sh.orw is read; the next call writes it)
}

// Bucket b's start in bucket order and its length (every thread; wave-uniform values).
__device__ inline void ss_bucket_range(const unsigned long long *__restrict__ counts, int b, int64_t &base,
                                       int64_t &len) {
    __shared__ int64_t s_t64[kSsWaves];
    __shared__ int64_t s_base, s_len;
    const int tid = threadIdx.x;
    const int64_t cnt = tid < kSsBuckets ? int64_t(counts[tid]) : 0;
    const int64_t st = block_excl_scan<int64_t, kSsWaves>(cnt, s_t64, (int64_t *)nullptr);
    if (tid == b) {
        s_base = st;
        s_len = cnt;
    }
    __syncthreads();
    auto uni = [](int64_t x) {  // (scalar registers for the bounds and the pointers made from them)
        const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(x)),
                       h = __builtin_amdgcn_readfirstlane(uint32_t(uint64_t(x) >> 32));
        return int64_t((uint64_t(h) << 32) | l);
    };
    base = uni(s_base);
    len = uni(s_len);
}

// One workgroup per range bucket of <= kSsMax values, sorted in place in val / pos (bucket order
// on entry; the bucket's positions are read before any is written).  Equality buckets are final;
// longer range buckets are k_ss_runs'.  A range bucket lies between two sample quantiles, so its
// values are spread: a counting sort into n value sub-buckets (linear in value when the range is
// finite, else in key), each value's rank inside its sub-bucket by comparison (key, then position:
// stable) - O(n) work and five barriers.  A sub-bucket of more than kSsSkew values, or sub-buckets
// whose squared sizes sum past kSsWork (long runs of repeated values that no sample hit), send the
// bucket to the LSD radix sort in LDS instead.
// (measured at config 2, same box: thresholds of 2,048 values / 4 M squared values ranked RQ3's
// union's tie runs by comparison - k_ss_buckets 454 us, the step 1.48 ms - against 90 us / 1.16 ms
// with the LDS radix sort taking every bucket with a sub-bucket of more than 128 values)
#ifndef FZ_SS_SKEW
#define FZ_SS_SKEW 128
#endif
#ifndef FZ_SS_TAIL_KEY
#define FZ_SS_TAIL_KEY 1  // the two tail buckets' sub-buckets linear in key, not in value
#endif
#ifndef FZ_SS_WORK
#define FZ_SS_WORK 0x7fffffff
#endif
constexpr int kSsSkew = FZ_SS_SKEW;  // largest sub-bucket ranked by comparison
constexpr int kSsWork = FZ_SS_WORK;  // sum of squared sub-bucket sizes ranked by comparison
#ifndef FZ_SS_STRIDED
#define FZ_SS_STRIDED 1  // (0: wave-contiguous items, the A/B baseline)
#endif
struct SsVbShared {  // the value-bucket sort's LDS (aliases SsShared: one or the other per bucket)
    uint64_t key[kSsMax];
    uint16_t pos[kSsMax];                   // values in sub-bucket order (bucket-local index)
    uint32_t cnt[(kSsMax + 2 + 1) / 2];     // 16-bit sub-bucket counters, then starts (+ sentinel)
};
union SsLds {
    SsShared lsd;
    SsVbShared vb;
};
__global__ __launch_bounds__(kSsBlock) void k_ss_buckets(const unsigned long long *__restrict__ counts,
                                                          double *__restrict__ val, int32_t *__restrict__ pos) {
    __shared__ SsLds L;
    __shared__ uint64_t s_lo[kSsWaves], s_hi[kSsWaves];
    __shared__ uint32_t s_tmp[kSsWaves], s_max[kSsWaves], s_sq[kSsWaves];
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    const int b = blockIdx.x;
    if (b & 1) return;  // (an equality bucket: one key, already in position order)
    int64_t base, len;
    ss_bucket_range(counts, b, base, len);
    if (len <= 1 || len > kSsMax) return;
    double *v = val + base;
    int32_t *ps = pos + base;
    const int wbase = w * (kSsMax / kSsWaves);
    const int n = int(len);
    uint16_t *const cnt16 = reinterpret_cast<uint16_t *>(L.vb.cnt);
    uint64_t k[kSsIpt];
    uint64_t lo = ~0ull, hi = 0ull;
    // value q of the bucket is thread q % kSsBlock's item q / kSsBlock (block-strided: a bucket of a
    // few thousand values keeps every wave busy - with wave-contiguous items, config 2's ~4 K-value
    // buckets ran on 5 of the 16 waves, 12 dependent items each); the LDS radix fallback below
    // re-reads its wave-contiguous layout
    auto qof = [&](int r) { return FZ_SS_STRIDED ? r * kSsBlock + tid : wbase + r * kWave + lane; };
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r) {
        const int q = qof(r);
        k[r] = q < n ? f64_key(v[q]) : 0ull;
        if (q < n) {
            lo = k[r] < lo ? k[r] : lo;
            hi = k[r] > hi ? k[r] : hi;
        }
    }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (lane == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
    }
    for (int j = tid; j < (n + 2) / 2; j += kSsBlock) L.vb.cnt[j] = 0u;
    __syncthreads();
    lo = ~0ull;
    hi = 0ull;
#pragma unroll
    for (int q = 0; q < kSsWaves; ++q) {
        lo = s_lo[q] < lo ? s_lo[q] : lo;
        hi = s_hi[q] > hi ? s_hi[q] : hi;
    }
    // sub-bucket of a key: linear in value over a finite range (spread values stay spread), else in
    // key.  The two tail buckets (below the first splitter, above the last) are bucketed in key
    // always: unbounded on one side, they are dense near their inner end - config 2's union: -50 ..
    // -0.5 and 0.5 .. 50 put 515 / 545 values into one value-linear sub-bucket (the LDS radix sort,
    // ~88 us for the launch), while the key - the float's exponent and mantissa - spreads them about
    // logarithmically (largest sub-bucket 47 / 42)
    const bool tail = FZ_SS_TAIL_KEY && (b == 0 || b == 2 * kSsSplit);
    const double vlo = f64_from_key(lo), vhi = f64_from_key(hi);
    const bool vlin = !tail && isfinite(vlo) && isfinite(vhi) && isfinite(vhi - vlo) && vhi > vlo;
    const double vsc = vlin ? double(n) / (vhi - vlo) : 0.0, ksc = double(n) / (double(hi - lo) + 1.0);
    auto sub = [&](uint64_t key) -> uint32_t {
        const double qd = vlin ? (f64_from_key(key) - vlo) * vsc : double(key - lo) * ksc;
        return qd < double(n - 1) ? (qd > 0.0 ? uint32_t(qd) : 0u) : uint32_t(n - 1);
    };
    uint32_t bs[kSsIpt];  // sub-bucket << 16 | slot in it
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r) {
        const int q = qof(r);
        bs[r] = 0u;
        if (q < n) {
            const uint32_t sb = sub(k[r]);
            const uint32_t sh = (sb & 1u) * 16u;
            bs[r] = (sb << 16) | ((atomicAdd(&L.vb.cnt[sb >> 1], 1u << sh) >> sh) & 0xffffu);
        }
    }
    __syncthreads();
    // sub-bucket starts: thread t scans EPT consecutive counters; the largest decides the fallback
    constexpr int EPT = (kSsMax + 1 + kSsBlock - 1) / kSsBlock;
    uint32_t sum = 0, mx = 0, sq = 0;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int j = tid * EPT + e;
        const uint32_t ce = j < n ? cnt16[j] : 0u;
        sum += ce;
        sq += ce > 1u ? ce * ce : 0u;  // (<= n^2 < 2^28)
        mx = ce > mx ? ce : mx;
    }
    mx = wave_max(mx);
    sq = wave_sum(sq);
    if (lane == 0) {
        s_max[w] = mx;
        s_sq[w] = sq;
    }
    uint32_t run = block_excl_scan<uint32_t, kSsWaves>(sum, s_tmp, (uint32_t *)nullptr);
#pragma unroll
    for (int e = 0; e < EPT; ++e) {  // (block_excl_scan's barriers ordered every read above)
        const int j = tid * EPT + e;
        if (j < n) {
            const uint32_t ce = cnt16[j];
            cnt16[j] = uint16_t(run);
            run += ce;
        }
    }
    if (tid == 0) cnt16[n] = uint16_t(n);
    __syncthreads();
    uint32_t gmax = 0, gsq = 0;
#pragma unroll
    for (int q = 0; q < kSsWaves; ++q) {
        gmax = s_max[q] > gmax ? s_max[q] : gmax;
        gsq += s_sq[q];
    }
    int32_t dq[kSsIpt];
    // the in-sub-bucket ranking costs sum(m^2) comparisons over the block (m values in a
    // sub-bucket) and about m LDS round trips per item of the longest sub-bucket: past a few hundred
    // tied values the LDS radix sort below is cheaper (FZ_SS_SKEW / FZ_SS_WORK)
    if (gmax > uint32_t(kSsSkew) || gsq > uint32_t(kSsWork)) {
        // (a long run of one value: the radix sort, whose cost does not depend on the spread)
        __syncthreads();
        uint16_t ix[kSsIpt];
        const int R = ss_rounds(n);  // (ss_lds_sort's layout: a run of R * 64 values per wave)
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {  // (nothing written yet: v holds the bucket as on entry)
            const int q = ss_q(R, r);
            ix[r] = uint16_t(q);
            k[r] = r < R && q < n ? f64_key(v[q]) : 0ull;
        }
        ss_lds_sort(k, ix, n, lo, L.lsd);
        int32_t pp[kSsIpt];
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            const int q = ss_q(R, r);
            pp[r] = r < R && q < n ? ps[ix[r]] : 0;
        }
        __syncthreads();  // every position read before any is overwritten
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            const int q = ss_q(R, r);
            if (r < R && q < n) {
                v[q] = f64_from_key(k[r]);
                ps[q] = pp[r];
            }
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r) {
        const int q = qof(r);
        if (q < n) {
            const uint32_t slot = cnt16[bs[r] >> 16] + (bs[r] & 0xffffu);
            L.vb.pos[slot] = uint16_t(q);
            L.vb.key[slot] = k[r];  // (slot order: the ranking reads key and position at x together)
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r) {
        const int q = qof(r);
        dq[r] = -1;
        if (q >= n) continue;
        const uint32_t st = cnt16[bs[r] >> 16], en = cnt16[(bs[r] >> 16) + 1];
        uint32_t rank = 0;
        if (en - st > 1) {  // (alone in its sub-bucket: rank 0)
            // four slots' key / position reads in flight together (the lanes of a wave walk
            // sub-buckets of different lengths: one LDS round trip per slot was ~240 cycles)
            auto before = [&](uint64_t kx, int ox) { return uint32_t((kx < k[r]) || (kx == k[r] && ox < q)); };
            uint32_t x = st;
            for (; x + 4 <= en; x += 4) {
                const int o0 = L.vb.pos[x], o1 = L.vb.pos[x + 1], o2 = L.vb.pos[x + 2], o3 = L.vb.pos[x + 3];
                const uint64_t k0 = L.vb.key[x], k1 = L.vb.key[x + 1], k2 = L.vb.key[x + 2], k3 = L.vb.key[x + 3];
                rank += before(k0, o0) + before(k1, o1) + before(k2, o2) + before(k3, o3);
            }
            for (; x < en; ++x) rank += before(L.vb.key[x], L.vb.pos[x]);
        }
        dq[r] = int32_t(st + rank);
    }
    // (the values were read into registers at the start; the positions are read only now - not
    // live through the counting and ranking: 48 VGPRs spilled with them - and all before any write)
    int32_t np[kSsIpt];
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r) np[r] = dq[r] >= 0 ? ps[qof(r)] : 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSsIpt; ++r) {
        if (dq[r] >= 0) {
            v[dq[r]] = f64_from_key(k[r]);
            ps[dq[r]] = np[r];
        }
    }
}

// A range bucket past the LDS capacity: runs of kSsMax values sorted in LDS into (ka, ia) - keys
// and original positions - then merged pairwise by the workgroup (a merge path per thread, ties
// from the left run first: stable), the result written back over the bucket.  Every other
// bucket's workgroup leaves at once.
__global__ __launch_bounds__(kSsBlock) void k_ss_runs(const unsigned long long *__restrict__ counts,
                                                       uint64_t *__restrict__ ka, uint32_t *__restrict__ ia,
                                                       uint64_t *__restrict__ kb, uint32_t *__restrict__ ib,
                                                       double *__restrict__ val, int32_t *__restrict__ pos) {
    __shared__ SsShared sh;
    const int tid = threadIdx.x;
    const int b = blockIdx.x;
    if (b & 1) return;
    int64_t base, len;
    ss_bucket_range(counts, b, base, len);
    if (len <= kSsMax) return;
    double *v = val + base;
    int32_t *ps = pos + base;
    uint64_t *ks = ka + base, *kd = kb + base;
    uint32_t *is = ia + base, *id = ib + base;
    for (int64_t c0 = 0; c0 < len; c0 += kSsMax) {
        const int n = int(len - c0 < kSsMax ? len - c0 : kSsMax);
        const int R = ss_rounds(n);
        uint64_t k[kSsIpt];
        uint16_t ix[kSsIpt];
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            const int q = ss_q(R, r);
            k[r] = r < R && q < n ? f64_key(v[c0 + q]) : 0ull;
            ix[r] = uint16_t(q);
        }
        ss_lds_sort(k, ix, n, f64_key(v[c0]), sh);
#pragma unroll
        for (int r = 0; r < kSsIpt; ++r) {
            const int q = ss_q(R, r);
            if (r < R && q < n) {
                ks[c0 + q] = k[r];
                is[c0 + q] = uint32_t(ps[c0 + ix[r]]);
            }
        }
    }
    __syncthreads();
    for (int64_t width = kSsMax; width < len; width <<= 1) {
        for (int64_t s0 = 0; s0 < len; s0 += 2 * width) {
            const int64_t a1 = s0 + width < len ? s0 + width : len, b1 = s0 + 2 * width < len ? s0 + 2 * width : len;
            const int64_t na = a1 - s0, nb = b1 - a1, tot = na + nb;
            const uint64_t *A = ks + s0, *B = ks + a1;
            const int64_t per = (tot + kSsBlock - 1) / kSsBlock;
            const int64_t d0 = int64_t(tid) * per;
            if (d0 >= tot) continue;
            const int64_t d1 = d0 + per < tot ? d0 + per : tot;
            int64_t l = d0 - nb > 0 ? d0 - nb : 0, h = d0 < na ? d0 : na;
            while (l < h) {  // A elements among the first d0 outputs
                const int64_t mid = (l + h) >> 1;
                if (A[mid] <= B[d0 - mid - 1]) l = mid + 1;
                else h = mid;
            }
            int64_t i = l, j = d0 - l;
            for (int64_t d = d0; d < d1; ++d) {
                const bool ta = j >= nb || (i < na && A[i] <= B[j]);
                kd[s0 + d] = ta ? A[i] : B[j];
                id[s0 + d] = ta ? is[s0 + i] : is[a1 + j];
                if (ta) ++i;
                else ++j;
            }
        }
        __syncthreads();
        uint64_t *tk = ks;
        ks = kd;
        kd = tk;
        uint32_t *ti = is;
        is = id;
        id = ti;
    }
    for (int64_t q = tid; q < len; q += kSsBlock) {
        v[q] = f64_from_key(ks[q]);
        ps[q] = int32_t(is[q]);
    }
}

bool sample_sort_on() {
    static const bool on = [] {
        const char *e = std::getenv("FZ_SAMPLE_SORT");
        return !e || std::atoi(e) != 0;
    }();
    return on;
}

void sample_sort_f64_seg1(fz_ctx *c, const double *src, const int64_t *offs, int64_t n_cap, double *val,
                          int32_t *pos) {
    FZ_CHECK(n_cap > 0 && n_cap < (int64_t(1) << 31), "sample_sort_f64_seg1: 1 .. 2^31 - 1 positions");
    uint64_t *spl = c->arena.get<uint64_t>(kSsSplit + 1);
    unsigned long long *counts = c->arena.get<unsigned long long>(256);
    int64_t *d_hi = c->arena.get<int64_t>(1);
    uint32_t *ids = c->arena.get<uint32_t>(n_cap);
    uint32_t *kout = c->arena.get<uint32_t>(n_cap);
    uint64_t *ka = c->arena.get<uint64_t>(n_cap), *kb = c->arena.get<uint64_t>(n_cap);
    uint32_t *ia = c->arena.get<uint32_t>(n_cap), *ib = c->arena.get<uint32_t>(n_cap);
    const int64_t nb = (n_cap + kSortTile - 1) / kSortTile;
    const int64_t gwords = ((nb + kOsGroup - 1) / kOsGroup) * kRadix;
    unsigned long long *gsum = c->arena.get<unsigned long long>(gwords);
    k_ss_splitters<<<1, kSsBlock, 0, c->stream>>>(src, offs, n_cap, spl, counts, gsum, gwords, d_hi);
    // (256 workgroups: each adds its 255 bucket counts to the totals with global atomics - 2,048
    // workgroups' adds serialised on the 255 words, 47 us at config 2)
    k_ss_ids<<<grid_for(n_cap, kSsBlock, 256), kSsBlock, 0, c->stream>>>(src, d_hi, spl, ids, counts);
    FZ_LAUNCH_CHECK();
    const Lookback lb = lookback_begin(c, nb * kRadix);
    RadixPayload pl;
    pl.n = 1;
    pl.in[0] = src;
    pl.size[0] = 8;
    pl.out[0] = val;
    {
        // algorithmic traffic: bucket id 4 + value 8 read, bucket id 4 + position 4 + value 8 written
        ProbeScope ps(c, "radix_scatter", 0.0, d_hi, 28.0);
        k_onesweep<uint32_t, true, true, kSortTile, kOsBlock><<<unsigned(nb), kOsBlock, 0, c->stream>>>(
            ids, nullptr, kout, reinterpret_cast<uint32_t *>(pos), n_cap, 0, counts, lb.status, lb.ticket, lb.epoch,
            gsum, nullptr, pl, d_hi);
        FZ_LAUNCH_CHECK();
    }
    lookback_end(c, nb);
    {
        // algorithmic traffic per value: value 8 + position 4 read and written (range buckets)
        ProbeScope ps(c, "seg_sample_sort", 0.0, d_hi, 24.0);
        k_ss_buckets<<<kSsBuckets, kSsBlock, 0, c->stream>>>(counts, val, pos);
        k_ss_runs<<<kSsBuckets, kSsBlock, 0, c->stream>>>(counts, ka, ia, kb, ib, val, pos);
        FZ_LAUNCH_CHECK();
    }
}

// ------------------------------------------------------------------------------- min / max
// min / max over non-NULL values of up to kMinMaxCols columns in one launch (blockIdx.y = column)
constexpr int kMinMaxCols = 8;
struct MinMaxCols {
    const int64_t *x[kMinMaxCols];
    int64_t n[kMinMaxCols];
};
__global__ __launch_bounds__(kBlock) void k_minmax(MinMaxCols cols, unsigned long long *__restrict__ mm) {
    const int col = blockIdx.y;
    const int64_t *__restrict__ x = cols.x[col];
    const int64_t n = cols.n[col];
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const int64_t v = x[i];
        if (v == FZ_TS_NULL) continue;
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    __shared__ int64_t s_lo[4], s_hi[4];
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (lane_id() == 0) {
        s_lo[wave_id()] = lo;
        s_hi[wave_id()] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; ++i) {
            lo = s_lo[i] < lo ? s_lo[i] : lo;
            hi = s_hi[i] > hi ? s_hi[i] : hi;
        }
        lo = s_lo[0] < lo ? s_lo[0] : lo;
        hi = s_hi[0] > hi ? s_hi[0] : hi;
        // order-preserving unsigned images so one unsigned atomic min/max covers negatives too
        atomicMin(&mm[2 * col], (unsigned long long)(lo) ^ 0x8000000000000000ull);
        atomicMax(&mm[2 * col + 1], (unsigned long long)(hi) ^ 0x8000000000000000ull);
    }
}

void minmax_i64_to_host(fz_ctx *c, const int64_t *const *cols, const int64_t *ns, int ncols, int64_t *host_minmax) {
    FZ_CHECK(ncols >= 1 && ncols <= kMinMaxCols, "minmax: 1..8 columns");
    unsigned long long *mm = c->arena.get<unsigned long long>(2 * ncols);
    MinMaxCols mc{};
    int64_t nmax = 0;
    for (int i = 0; i < ncols; ++i) {
        mc.x[i] = cols[i];
        mc.n[i] = ns[i] > 0 ? ns[i] : 0;
        nmax = mc.n[i] > nmax ? mc.n[i] : nmax;
    }
    // {min, max} start values through a kernel argument (no pageable host-to-device copy)
    for (int i = 0; i < ncols; i += 2) {
        const int64_t init[4] = {-1, 0, -1, 0};
        set_i64(c, reinterpret_cast<int64_t *>(mm) + 2 * i, init, ncols - i >= 2 ? 4 : 2);
    }
    if (nmax > 0) {  // one launch for every column
        const dim3 g(grid_for(nmax, kBlock * 8, 512), unsigned(ncols));
        k_minmax<<<g, kBlock, 0, c->stream>>>(mc, mm);
        FZ_LAUNCH_CHECK();
    }
    FZ_HIP(hipMemcpyAsync(c->h_pinned, mm, 2 * ncols * 8, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    for (int i = 0; i < 2 * ncols; ++i)
        host_minmax[i] = int64_t(uint64_t(c->h_pinned[i]) ^ 0x8000000000000000ull);
}

// ------------------------------------------------------------------------ segment offsets
void segment_offsets(fz_ctx *c, const uint32_t *sorted_proj, int64_t n, int64_t P, int64_t *offsets) {
    segment_offsets_dn(c, sorted_proj, nullptr, n < 0 ? 0 : n, P, offsets);  // row-parallel, host length
}

// -------------------------------------------------------------------------------- describe
__global__ void k_set_i64(int64_t *p, int64_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *p = v;
}

// keys of x[0..n) as order-preserving images; entries past n sort last.
__global__ __launch_bounds__(kBlock) void k_f64_keys(const double *__restrict__ x, int64_t nmax,
                                                     const int64_t *__restrict__ d_n, uint64_t *__restrict__ k) {
    const int64_t n = *d_n;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nmax; i += int64_t(gridDim.x) * kBlock)
        k[i] = i < n ? f64_key(x[i]) : ~0ull;
}

// Double-double partial sums of x (pass 1) or of (x - mean)^2 (pass 2, mean read from device);
// blockIdx.y = job, partials of job j at part[2 * gridDim.x * j ...].
// Job j's partial sums -> ms[2 * j + mode] (mode 0: mean; mode 1: sqrt(sum / n) = std, ddof 0):
// the per-block partials summed by one block, in block order - by k_dd_final, or (tickets) by the
// block that arrives last, stores write-through + one agent-scope ticket add per block.
__device__ inline void dd_final_block(const double *pj, int nparts, int64_t n, int mode, double *ms_slot) {
    __shared__ double s_hi[4], s_lo[4];
    DD acc{0.0, 0.0};
    for (int i = threadIdx.x; i < nparts; i += kBlock) acc = dd_add(acc, DD{pj[2 * i], pj[2 * i + 1]});
    acc = wave_dd_sum(acc);
    if (lane_id() == 0) {
        s_hi[wave_id()] = acc.hi;
        s_lo[wave_id()] = acc.lo;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        DD t{s_hi[0], s_lo[0]};
        for (int i = 1; i < 4; ++i) t = dd_add(t, DD{s_hi[i], s_lo[i]});
        const double s = t.hi + t.lo;
        const double q = n > 0 ? s / double(n) : NAN;
        *ms_slot = mode == 0 ? q : sqrt(q);
    }
}

__global__ __launch_bounds__(kBlock) void k_dd_partial(SortedDescArgs a, const double *__restrict__ ms,
                                                       double *__restrict__ part, unsigned *tickets = nullptr,
                                                       int mode = 0, double *ms_out = nullptr) {
    __shared__ double s_hi[4], s_lo[4];
    __shared__ int s_last;
    const int j = blockIdx.y;
    const double *__restrict__ x = a.x[j];
    const int64_t n = *a.d_n[j];
    DD acc{0.0, 0.0};
    const double m = ms ? ms[2 * j] : 0.0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        double v = x[i];
        if (ms) {
            v = v - m;
            v = v * v;
        }
        acc = dd_add_d(acc, v);
    }
    acc = wave_dd_sum(acc);
    if (lane_id() == 0) {
        s_hi[wave_id()] = acc.hi;
        s_lo[wave_id()] = acc.lo;
    }
    __syncthreads();
    double *pj = part + 2 * int64_t(gridDim.x) * j;
    if (threadIdx.x == 0) {
        DD t{s_hi[0], s_lo[0]};
        for (int i = 1; i < 4; ++i) t = dd_add(t, DD{s_hi[i], s_lo[i]});
        if (tickets) {
            store_wt(&pj[2 * blockIdx.x], t.hi);
            store_wt(&pj[2 * blockIdx.x + 1], t.lo);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned old = __hip_atomic_fetch_add(&tickets[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == gridDim.x - 1;
            if (s_last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&tickets[j], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            pj[2 * blockIdx.x] = t.hi;
            pj[2 * blockIdx.x + 1] = t.lo;
        }
    }
    if (!tickets) return;
    __syncthreads();
    if (s_last) dd_final_block(pj, int(gridDim.x), n, mode, ms_out + 2 * j + mode);
}

// Reduce job blockIdx.x's partials into ms[2 * job + mode].
__global__ __launch_bounds__(kBlock) void k_dd_final(const double *__restrict__ part, int nparts, SortedDescArgs a,
                                                     int mode, double *__restrict__ ms) {
    const int j = blockIdx.x;
    dd_final_block(part + 2 * int64_t(nparts) * j, nparts, *a.d_n[j], mode, ms + 2 * j + mode);
}

__device__ inline int64_t lower_bound_u64(const uint64_t *a, int64_t n, uint64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ inline int64_t upper_bound_u64(const uint64_t *a, int64_t n, uint64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// fz_describe of n ascending keys sk (global or LDS) with the given mean / std
// (bounds, optional: the sample's {lower_bound(-0.0), upper_bound(+0.0), upper_bound(+inf)} found
// by the caller - three lanes' searches at once instead of three one after another)
__device__ void describe_from_sorted(const uint64_t *sk, int64_t n, double mean, double std,
                                     fz_describe *__restrict__ out, const int64_t *bounds = nullptr) {
    fz_describe d;
    d.count = n;
    if (n <= 0) {
        d.n_pos = d.n_zero = d.n_neg = 0;
        d.mean = d.median = d.std = d.min = d.max = d.q1 = d.q3 = d.min_nonzero = NAN;
        d.has_nonzero = 0;
        *out = d;
        return;
    }
    d.mean = mean;
    d.std = std;
    const uint64_t kneg0 = f64_key(-0.0), kpos0 = f64_key(0.0), kinf = f64_key(INFINITY);
    const int64_t lt0 = bounds ? bounds[0] : lower_bound_u64(sk, n, kneg0);
    const int64_t le0 = bounds ? bounds[1] : upper_bound_u64(sk, n, kpos0);
    const int64_t leinf = bounds ? bounds[2] : upper_bound_u64(sk, n, kinf);
    d.n_neg = lt0;
    d.n_zero = le0 - lt0;
    d.n_pos = leinf - le0;
    auto get = [&](int64_t i) { return f64_from_key(sk[i]); };
    d.min = get(0);
    d.max = get(n - 1);
    // np.median: middle element, or mean of the two middle ones ((a + b) / 2)
    d.median = (n & 1) ? get(n / 2) : (get(n / 2 - 1) + get(n / 2)) / 2.0;
    d.q1 = np_percentile_sorted(get, n, 25.0);
    d.q3 = np_percentile_sorted(get, n, 75.0);
    // min over values != 0 (rq1_detection_rate.py:264)
    if (lt0 > 0) {
        d.min_nonzero = get(0);
        d.has_nonzero = 1;
    } else if (le0 < n) {
        d.min_nonzero = get(le0);
        d.has_nonzero = 1;
    } else {
        d.min_nonzero = NAN;
        d.has_nonzero = 0;
    }
    *out = d;
}

__global__ void k_describe_finish(SortedDescArgs a, const double *__restrict__ ms) {
    chain_prio();
    const int j = blockIdx.x, lane = threadIdx.x;
    const uint64_t *sk = a.k[j];
    const int64_t n = *a.d_n[j];
    // lanes 0 / 1 / 2: the sign-class bounds, one binary search each
    int64_t b = 0;
    if (lane < 3 && n > 0) {
        const uint64_t kv = lane == 0 ? f64_key(-0.0) : (lane == 1 ? f64_key(0.0) : f64_key(INFINITY));
        b = lane == 0 ? lower_bound_u64(sk, n, kv) : upper_bound_u64(sk, n, kv);
    }
    const int64_t bounds[3] = {__shfl(b, 0, 64), __shfl(b, 1, 64), __shfl(b, 2, 64)};
    if (lane == 0) describe_from_sorted(sk, n, ms[2 * j], ms[2 * j + 1], a.out[j], bounds);
}

// samples of a capacity up to this are described by selection (k_describe_sel: one workgroup,
// passes over the sample); larger ones sort their keys (radix) first
constexpr int64_t kDescSelMax = 65536;
struct DescSmallArgs {
    const double *x[kDescBatch];
    const int64_t *d_n[kDescBatch];
    fz_describe *out[kDescBatch];
    int64_t stage_cap;  // keys staged in the dynamic LDS (its size / 8): samples of up to this many
};
// ---- describe by selection (one workgroup per sample, no sorted copy) ------------------------
// The order statistics a describe needs (median, the quartiles' interpolation neighbours, the
// smallest non-zero value) are selected by value-bucket histograms over the sample's key range:
// the sample is re-read from global memory (L2-resident for the samples this serves) in each pass -
// statistics (min / max / sum / sign counts), squared deviations, one histogram, one gather of the
// wanted buckets - and a wanted bucket of more than 64 values is narrowed by re-histogramming its
// key interval.  One launch for any live length (rounds 1-3: an LDS bitonic network up to 4096
// values, a 64-bit radix sort + five launches beyond).
constexpr int kSelNB = 4096;
constexpr int kSelMaxT = 8;
constexpr int kSelBlock = 512;  // (8 waves: room for 256 VGPRs, no spills)
struct SelShared {
    uint32_t cnt[kSelNB + 1];
    uint8_t map[kSelNB];
    uint64_t list[kSelMaxT][64];
    uint32_t fill[kSelMaxT];
    uint64_t lo[kSelBlock / kWave], hi[kSelBlock / kWave];
    uint32_t tmp[kSelBlock / kWave];
    int64_t rank[kSelMaxT], tb[kSelMaxT], toff[kSelMaxT], tsz[kSelMaxT];
    int tslot[kSelMaxT];
    int twide[kSelMaxT];                      // wide target t: its wide-bucket slot
    unsigned long long wlo[kSelMaxT], whi[kSelMaxT];  // key range of each distinct wide bucket
    int nwide;
    // wide target t's state while narrowing: key interval [wl, wh], rank in it, count, sub-bucket
    unsigned long long wl[kSelMaxT], wh[kSelMaxT];
    int64_t wr[kSelMaxT], wc[kSelMaxT];
    uint32_t wsb[kSelMaxT];
    int wact[kSelMaxT];
    uint64_t res[kSelMaxT];
    int64_t r, rc;
    uint32_t sb;
};

__device__ inline void sel_minmax(uint64_t &lo, uint64_t &hi, SelShared &sh) {
    constexpr int NW = kSelBlock / kWave;
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (lane_id() == 0) {
        sh.lo[wave_id()] = lo;
        sh.hi[wave_id()] = hi;
    }
    __syncthreads();
    lo = sh.lo[0];
    hi = sh.hi[0];
    for (int q = 1; q < NW; ++q) {
        lo = sh.lo[q] < lo ? sh.lo[q] : lo;
        hi = sh.hi[q] > hi ? sh.hi[q] : hi;
    }
    __syncthreads();
}

__device__ inline uint32_t sel_bucket(uint64_t k, uint64_t lo, double sc, int nb) {
    const uint32_t q = uint32_t(double(k - lo) * sc);
    return q < uint32_t(nb) ? q : uint32_t(nb - 1);
}

// for every i < n of this thread (i = tid, tid + BS, ...; that order): body(i, load(i)), the loads
// of kSelU consecutive items issued before their bodies (one memory latency per kSelU items, not
// one per item)
constexpr int kSelU = 8;
template <int U = kSelU, typename Load, typename Body>
__device__ inline void sel_for(int64_t n, const Load &load, const Body &body) {
    using T = decltype(load(int64_t(0)));
    for (int64_t i0 = threadIdx.x; i0 < n; i0 += int64_t(kSelBlock) * U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + int64_t(u) * kSelBlock;
            v[u] = i < n ? load(i) : T{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + int64_t(u) * kSelBlock;
            if (i < n) body(i, v[u]);
        }
    }
}

#ifdef FZ_DESC_TIMING
// experiment builds only: wall-clock (100 MHz) phase stamps of the last k_describe_sel workgroup 0
__device__ unsigned long long g_desc_t[32];
#define DESC_STAMP(ph)                                                       \
    do {                                                                     \
        __syncthreads();                                                     \
        if (threadIdx.x == 0 && blockIdx.x == 0) g_desc_t[ph] = wall_clock64();     \
    } while (0)
extern "C" int fz_debug_desc_timing(unsigned long long *out) {
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_desc_t), sizeof(g_desc_t));
    return 0;
}
#else
#define DESC_STAMP(ph) \
    do {               \
    } while (0)
#endif

// sh.res[t] = the key of rank sh.rank[t] (t < nt) among the n keys key(i), whose min / max are lo / hi
template <typename KeyF>
__device__ void wg_select_global(const KeyF &key, int64_t n, uint64_t lo, uint64_t hi, int nt, SelShared &sh) {
    constexpr int BS = kSelBlock, NW = BS / kWave;
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    if (lo == hi) {
        if (tid < nt) sh.res[tid] = lo;
        __syncthreads();
        return;
    }
    const int nb = n < kSelNB ? int(n) : kSelNB;
    const double sc = double(nb) / (double(hi - lo) + 1.0);
    // first level linear in VALUE when the range is finite (then a bucket rarely holds more than a
    // few distinct values: integer data - ties - gets one value per bucket, dense centres spread),
    // else linear in key; either is monotone in the key order, so a bucket is a key interval
    const double vlo = f64_from_key(lo), vhi = f64_from_key(hi);
    const bool vlin = isfinite(vlo) && isfinite(vhi) && isfinite(vhi - vlo) && vhi > vlo;
    const double vsc = vlin ? double(nb) / (vhi - vlo) : 0.0;
    auto bucket1 = [&](uint64_t k) -> uint32_t {
        if (!vlin) return sel_bucket(k, lo, sc, nb);
        const double q = (f64_from_key(k) - vlo) * vsc;  // (>= 0; NaN keys lie above hi: not here)
        return q < double(nb - 1) ? uint32_t(q) : uint32_t(nb - 1);
    };
    for (int j = tid; j <= nb; j += BS) sh.cnt[j] = 0u;
    for (int j = tid; j < nb; j += BS) sh.map[j] = 0xff;
    __syncthreads();
    DESC_STAMP(3);
    sel_for(n, key, [&](int64_t, uint64_t k) { atomicAdd(&sh.cnt[bucket1(k)], 1u); });
    __syncthreads();
    DESC_STAMP(4);
    {  // exclusive scan of the bucket counts: thread t takes buckets [t * 4, t * 4 + 4)
        constexpr int BPT = kSelNB / BS;
        uint32_t sum = 0;
        for (int e = 0; e < BPT; ++e) sum += tid * BPT + e < nb ? sh.cnt[tid * BPT + e] : 0u;
        uint32_t run = block_excl_scan<uint32_t, NW>(sum, sh.tmp, (uint32_t *)nullptr);
        for (int e = 0; e < BPT; ++e) {
            if (tid * BPT + e < nb) {
                const uint32_t ce = sh.cnt[tid * BPT + e];
                sh.cnt[tid * BPT + e] = run;
                run += ce;
            }
        }
        if (tid == 0) sh.cnt[nb] = uint32_t(n);
    }
    __syncthreads();
    DESC_STAMP(10);
    if (tid < nt) {
        const uint32_t r = uint32_t(sh.rank[tid]);
        int l0 = 0, h0 = nb - 1;
        while (l0 < h0) {
            const int mid = (l0 + h0 + 1) >> 1;
            if (sh.cnt[mid] <= r) l0 = mid;
            else h0 = mid - 1;
        }
        sh.tb[tid] = l0;
        sh.toff[tid] = int64_t(r) - int64_t(sh.cnt[l0]);
        sh.tsz[tid] = int64_t(sh.cnt[l0 + 1]) - int64_t(sh.cnt[l0]);
    }
    __syncthreads();
    DESC_STAMP(11);
    if (tid == 0) {  // list slots of the narrow buckets (map 0..), slots of the distinct wide ones (0x80 | w)
        int used = 0, wide = 0;
        for (int t = 0; t < nt; ++t) {
            int slot = -1, ws = -1;
            for (int u = 0; u < t; ++u)
                if (sh.tb[u] == sh.tb[t]) {
                    slot = sh.tslot[u];
                    ws = sh.twide[u];
                }
            if (slot < 0 && ws < 0) {
                if (sh.tsz[t] <= 64) {
                    slot = used++;
                    sh.fill[slot] = 0u;
                    sh.map[sh.tb[t]] = uint8_t(slot);
                } else {
                    ws = wide++;
                    sh.wlo[ws] = ~0ull;
                    sh.whi[ws] = 0ull;
                    sh.map[sh.tb[t]] = uint8_t(0x80 | ws);
                }
            }
            sh.tslot[t] = slot;
            sh.twide[t] = ws;
        }
        sh.nwide = wide;
    }
    __syncthreads();
    DESC_STAMP(12);
    // one pass: the narrow buckets' keys gathered, the wide buckets' key ranges (a wide bucket of
    // one key - ties - needs nothing more)
    const int nwide = sh.nwide;
    uint64_t wlo[kSelMaxT], whi[kSelMaxT];
#pragma unroll
    for (int q = 0; q < kSelMaxT; ++q) {
        wlo[q] = ~0ull;
        whi[q] = 0ull;
    }
    sel_for<4>(n, key, [&](int64_t, uint64_t k) {
        const uint8_t slot = sh.map[bucket1(k)];
        if (slot < 0x80) {
            sh.list[slot][atomicAdd(&sh.fill[slot], 1u)] = k;
        } else if (slot != 0xff) {
#pragma unroll
            for (int q = 0; q < kSelMaxT; ++q)
                if ((slot & 0x7f) == q) {
                    wlo[q] = k < wlo[q] ? k : wlo[q];
                    whi[q] = k > whi[q] ? k : whi[q];
                }
        }
    });
    DESC_STAMP(13);
    // (the slots' wave reductions two at a time, interleaved: independent shuffle chains)
#pragma unroll
    for (int q0 = 0; q0 < kSelMaxT; q0 += 2) {
        if (q0 < nwide) {  // (uniform)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t a0 = __shfl_xor(wlo[q0], off, 64), b0 = __shfl_xor(whi[q0], off, 64);
                const uint64_t a1 = __shfl_xor(wlo[q0 + 1], off, 64), b1 = __shfl_xor(whi[q0 + 1], off, 64);
                wlo[q0] = a0 < wlo[q0] ? a0 : wlo[q0];
                whi[q0] = b0 > whi[q0] ? b0 : whi[q0];
                wlo[q0 + 1] = a1 < wlo[q0 + 1] ? a1 : wlo[q0 + 1];
                whi[q0 + 1] = b1 > whi[q0 + 1] ? b1 : whi[q0 + 1];
            }
            if (lane == 0) {
                atomicMin(&sh.wlo[q0], (unsigned long long)wlo[q0]);
                atomicMax(&sh.whi[q0], (unsigned long long)whi[q0]);
                if (q0 + 1 < nwide) {
                    atomicMin(&sh.wlo[q0 + 1], (unsigned long long)wlo[q0 + 1]);
                    atomicMax(&sh.whi[q0 + 1], (unsigned long long)whi[q0 + 1]);
                }
            }
        }
    }
    __syncthreads();
    DESC_STAMP(5);
    auto rank_list = [&](int slot, int sz, int64_t want, int t) {  // one wave
        const uint64_t e = lane < sz ? sh.list[slot][lane] : ~0ull;
        int rr = 0;
        for (int j = 0; j < sz; ++j) {
            const uint64_t o = sh.list[slot][j];
            rr += (o < e) || (o == e && j < lane);
        }
        if (lane < sz && rr == int(want)) sh.res[t] = e;
    };
    for (int t = w; t < nt; t += NW)
        if (sh.tslot[t] >= 0) rank_list(sh.tslot[t], int(sh.tsz[t]), sh.toff[t], t);
    __syncthreads();
    // wide buckets: every wide target's key interval narrowed in the same passes - per round one
    // histogram pass (target t's sub-buckets in its own slice of sh.cnt) and one min / max pass over
    // the sub-bucket holding its rank - until it holds one key or <= 64 values; then one gather of
    // all the narrow intervals (uniform control flow: the target state is in LDS)
    DESC_STAMP(6);
    constexpr int kSlice = kSelNB / kSelMaxT;
    if (tid < nt) {
        const bool wide = sh.tslot[tid] < 0;
        sh.wr[tid] = sh.toff[tid];
        sh.wc[tid] = wide ? sh.tsz[tid] : 0;
        sh.wl[tid] = wide ? sh.wlo[sh.twide[tid]] : 1ull;
        sh.wh[tid] = wide ? sh.whi[sh.twide[tid]] : 0ull;  // (lo > hi: no key matches)
    }
    __syncthreads();
    auto uni64 = [](uint64_t x) {  // (wave-uniform value -> scalar registers)
        const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(x)), h = __builtin_amdgcn_readfirstlane(uint32_t(x >> 32));
        return (uint64_t(h) << 32) | l;
    };
#ifdef FZ_DESC_TIMING
    int round = 0;
#endif
    for (;;) {
#ifdef FZ_DESC_TIMING
        const int rs = round < 2 ? 16 + 6 * round : -1;
        ++round;
#define RSTAMP(k) \
    do {          \
        if (rs >= 0) DESC_STAMP(rs + (k)); \
    } while (0)
#else
#define RSTAMP(k) \
    do {          \
    } while (0)
#endif
        uint64_t al[kSelMaxT], ah[kSelMaxT];
        double asc[kSelMaxT];
        int anb[kSelMaxT];
        bool any = false;
#pragma unroll
        for (int t = 0; t < kSelMaxT; ++t) {
            const bool act = __builtin_amdgcn_readfirstlane(t < nt && sh.wl[t] != sh.wh[t] && sh.wc[t] > 64);
            any |= act;
            al[t] = act ? uni64(sh.wl[t]) : 1ull;
            ah[t] = act ? uni64(sh.wh[t]) : 0ull;
            anb[t] = act ? __builtin_amdgcn_readfirstlane(sh.wc[t] < kSlice ? int(sh.wc[t]) : kSlice) : 1;
            asc[t] = act ? __builtin_bit_cast(double, uni64(__builtin_bit_cast(uint64_t, double(anb[t]) / (double(ah[t] - al[t]) + 1.0)))) : 0.0;
        }
        if (!any) break;  // (uniform)
        RSTAMP(0);
        if (tid < kSelMaxT) sh.wact[tid] = tid < nt && sh.wl[tid] != sh.wh[tid] && sh.wc[tid] > 64;
        for (int j = tid; j < kSelNB; j += BS) sh.cnt[j] = 0u;
        __syncthreads();
        RSTAMP(1);
        sel_for<4>(n, key, [&](int64_t, uint64_t k) {
#pragma unroll
            for (int t = 0; t < kSelMaxT; ++t)
                if (k >= al[t] && k <= ah[t]) atomicAdd(&sh.cnt[t * kSlice + sel_bucket(k, al[t], asc[t], anb[t])], 1u);
        });
        __syncthreads();
        RSTAMP(2);
        static_assert(kSlice == kWave * (kSlice / kWave), "a slice is a whole number of lanes' runs");
        if (w < kSelMaxT && sh.wact[w]) {  // wave w: the sub-bucket holding target w's rank
            // lane l sums its run of kSlice / 64 sub-buckets, ONE 32-bit wave scan over the runs,
            // the lane whose run holds the rank walks it (instead of a dependent scan per 64)
            constexpr int RUN = kSlice / kWave;
            const uint32_t r = uint32_t(sh.wr[w]);
            const int nb2 = sh.wc[w] < kSlice ? int(sh.wc[w]) : kSlice;
            uint32_t cnt[RUN], sum = 0;
#pragma unroll
            for (int e = 0; e < RUN; ++e) {
                const int j = lane * RUN + e;
                cnt[e] = j < nb2 ? sh.cnt[w * kSlice + j] : 0u;
                sum += cnt[e];
            }
            const uint32_t incl = wave_incl_scan(sum);
            const uint64_t hit = __ballot(incl > r);
            const int l = __ffsll((unsigned long long)hit) - 1;  // (the rank is below the total)
            if (lane == l) {
                uint32_t before = incl - sum;
#pragma unroll
                for (int e = 0; e < RUN; ++e) {
                    if (before + cnt[e] > r) {
                        sh.wr[w] = int64_t(r - before);
                        sh.wc[w] = int64_t(cnt[e]);
                        sh.wsb[w] = uint32_t(lane * RUN + e);
                        sh.wlo[w] = ~0ull;
                        sh.whi[w] = 0ull;
                        break;
                    }
                    before += cnt[e];
                }
            }
        }
        __syncthreads();
        RSTAMP(3);
        uint32_t asb[kSelMaxT];
#pragma unroll
        for (int t = 0; t < kSelMaxT; ++t) asb[t] = al[t] <= ah[t] ? __builtin_amdgcn_readfirstlane(sh.wsb[t]) : 0u;
        // (a sub-bucket holds few keys - about wc / kSlice: LDS atomics on its bounds, no registers)
        sel_for<4>(n, key, [&](int64_t, uint64_t k) {
#pragma unroll
            for (int t = 0; t < kSelMaxT; ++t)
                if (k >= al[t] && k <= ah[t] && sel_bucket(k, al[t], asc[t], anb[t]) == asb[t]) {
                    // (ties: once a bound holds the key, its copies only read - no serialised
                    // atomics on one word)
                    if (k < sh.wlo[t]) atomicMin(&sh.wlo[t], (unsigned long long)k);
                    if (k > sh.whi[t]) atomicMax(&sh.whi[t], (unsigned long long)k);
                }
        });
        __syncthreads();
        RSTAMP(4);
        if (tid < kSelMaxT && sh.wact[tid]) {
            sh.wl[tid] = sh.wlo[tid];
            sh.wh[tid] = sh.whi[tid];
        }
        __syncthreads();
        RSTAMP(5);
    }
#undef RSTAMP
    DESC_STAMP(7);
    // one key left (ties): the result; else <= 64 values in [wl, wh]: one gather for all, ranked
    bool gather = false;
    uint64_t gl[kSelMaxT], gh[kSelMaxT];
#pragma unroll
    for (int t = 0; t < kSelMaxT; ++t) {
        const bool wide = t < nt && sh.tslot[t] < 0;
        const bool g = __builtin_amdgcn_readfirstlane(wide && sh.wl[t] != sh.wh[t]);
        gather |= g;
        gl[t] = g ? uni64(sh.wl[t]) : 1ull;
        gh[t] = g ? uni64(sh.wh[t]) : 0ull;
    }
    if (tid < nt && sh.tslot[tid] < 0) {
        if (sh.wl[tid] == sh.wh[tid]) sh.res[tid] = sh.wl[tid];
        sh.fill[tid] = 0u;
    }
    if (!gather) {  // (uniform)
        __syncthreads();
        return;
    }
    __syncthreads();
    sel_for<4>(n, key, [&](int64_t, uint64_t k) {
#pragma unroll
        for (int t = 0; t < kSelMaxT; ++t)
            if (k >= gl[t] && k <= gh[t]) sh.list[t][atomicAdd(&sh.fill[t], 1u)] = k;
    });
    __syncthreads();
    if (w < nt && sh.tslot[w] < 0 && sh.wl[w] != sh.wh[w]) rank_list(w, int(sh.wc[w]), sh.wr[w], w);
    __syncthreads();
}

// fz_describe of each job's sample (blockIdx.x = job), any live length
__device__ inline DD block_dd_sum_sel(DD acc, double *s_hi, double *s_lo) {
    acc = wave_dd_sum(acc);
    if (lane_id() == 0) {
        s_hi[wave_id()] = acc.hi;
        s_lo[wave_id()] = acc.lo;
    }
    __syncthreads();
    DD t{s_hi[0], s_lo[0]};
    for (int i = 1; i < kSelBlock / kWave; ++i) t = dd_add(t, DD{s_hi[i], s_lo[i]});
    __syncthreads();
    return t;
}
constexpr int64_t kSelLds = 12288;  // samples of up to this many values are staged in LDS (96 KiB of keys)
#ifndef FZ_DESC_NET_MAX
#define FZ_DESC_NET_MAX 1024  // samples of up to this many values sorted by a register network (512 .. 8,192)
#endif
static_assert(FZ_DESC_NET_MAX >= 512 && FZ_DESC_NET_MAX <= 8192 && (FZ_DESC_NET_MAX & (FZ_DESC_NET_MAX - 1)) == 0,
              "FZ_DESC_NET_MAX: a network size of 512 .. 8,192 keys");
#ifndef FZ_DESC_LDS_FIT
#define FZ_DESC_LDS_FIT 1  // (0: every describe workgroup stages kSelLds keys' worth of LDS; A/B builds)
#endif

// Sort the staged keys s[0, kSelBlock * E) ascending (entries at >= n read as ~0) by a bitonic
// network held in registers: E keys per thread, stages of distance < E inside a thread, < 64 E by
// shuffles inside a wave, only the 6 longest through LDS.  (Samples of <= 8,192 values: their
// order statistics straight off the sorted keys - the selection's histogram and narrowing rounds
// took 18-33 us per describe at config 2, four describes on the analyses' chains.)
template <int E>
__device__ inline void wg_bitonic_keys(uint64_t *s, int64_t n) {
    const int tid = threadIdx.x;
    uint64_t k[E];
#pragma unroll
    for (int h = 0; h < E; ++h) {
        const int e = E * tid + h;
        k[h] = e < n ? s[e] : ~0ull;
    }
    __syncthreads();
    // (unrolled: constant distances, direct register indexing in the in-thread stages)
#pragma unroll
    for (int kk = 2; kk <= kSelBlock * E; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j < E) {
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    if (h & j) continue;
                    const bool up = ((E * tid + h) & kk) == 0;
                    const uint64_t a = k[h], b = k[h | j];
                    if ((a > b) == up) {
                        k[h] = b;
                        k[h | j] = a;
                    }
                }
                continue;
            }
            uint64_t y[E];
            if (j / E < kWave) {
#pragma unroll
                for (int h = 0; h < E; ++h) y[h] = __shfl_xor(k[h], j / E, 64);
            } else {
#pragma unroll
                for (int h = 0; h < E; ++h) s[E * tid + h] = k[h];
                __syncthreads();
#pragma unroll
                for (int h = 0; h < E; ++h) y[h] = s[(E * tid + h) ^ j];
                __syncthreads();
            }
#pragma unroll
            for (int h = 0; h < E; ++h) {
                const int e = E * tid + h;
                const bool up = (e & kk) == 0, low = (e & j) == 0;
                const uint64_t mn = k[h] < y[h] ? k[h] : y[h], mx = k[h] < y[h] ? y[h] : k[h];
                k[h] = (low == up) ? mn : mx;
            }
        }
    }
#pragma unroll
    for (int h = 0; h < E; ++h) s[E * tid + h] = k[h];
    __syncthreads();
}
__global__ __launch_bounds__(kSelBlock) void k_describe_sel(DescSmallArgs a) {
    chain_prio();
    constexpr int NW = kSelBlock / kWave;
    __shared__ SelShared sh;
    // (sized by the launch to the batch's capacity: a 1,000-value sample's workgroup holds 33 KB of
    // LDS, not 121 KB, and is placed beside the other chains' workgroups instead of waiting for an
    // idle CU)
    extern __shared__ uint64_t s_keys[];
    __shared__ double s_hi[NW], s_lo[NW];
    __shared__ unsigned long long s_c[3];
    const int tid = threadIdx.x;
    const double *__restrict__ x = a.x[blockIdx.x];
    fz_describe *__restrict__ out = a.out[blockIdx.x];
    const int64_t n = *a.d_n[blockIdx.x];
    if (n <= 0) {
        if (tid == 0) describe_from_sorted(nullptr, 0, 0.0, 0.0, out);
        return;
    }
    DESC_STAMP(0);
    const uint64_t kneg0 = f64_key(-0.0), kpos0 = f64_key(0.0), kinf = f64_key(INFINITY);
    if (tid < 3) s_c[tid] = 0ull;
    uint64_t lo = ~0ull, hi = 0ull;
    DD acc{0.0, 0.0};
    unsigned long long lt0 = 0, le0 = 0, leinf = 0;
    // (a sample that fits is staged in LDS by this first pass: the later passes read LDS)
    const bool staged = n <= a.stage_cap;
    auto ld = [=](int64_t i) { return x[i]; };
    sel_for(n, ld, [&](int64_t i, double v) {
        const uint64_t k = f64_key(v);
        if (staged) s_keys[i] = k;
        acc = dd_add_d(acc, v);
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
        lt0 += k < kneg0;
        le0 += k <= kpos0;
        leinf += k <= kinf;
    });
    sel_minmax(lo, hi, sh);
    lt0 = wave_sum(lt0);
    le0 = wave_sum(le0);
    leinf = wave_sum(leinf);
    if (lane_id() == 0) {
        atomicAdd(&s_c[0], lt0);
        atomicAdd(&s_c[1], le0);
        atomicAdd(&s_c[2], leinf);
    }
    DD t = block_dd_sum_sel(acc, s_hi, s_lo);  // (its barriers order the counters too)
    DESC_STAMP(1);
    const double mean = (t.hi + t.lo) / double(n);
    acc = DD{0.0, 0.0};
    auto sq = [&](int64_t, double v) {
        v = v - mean;
        v = v * v;
        acc = dd_add_d(acc, v);
    };
    if (staged) sel_for(n, [&](int64_t i) { return f64_from_key(s_keys[i]); }, sq);
    else sel_for(n, ld, sq);
    t = block_dd_sum_sel(acc, s_hi, s_lo);
    DESC_STAMP(2);
    const double std = sqrt((t.hi + t.lo) / double(n));
    const int64_t c_lt0 = int64_t(s_c[0]), c_le0 = int64_t(s_c[1]), c_leinf = int64_t(s_c[2]);
    // ranks: median (n / 2, and n / 2 - 1), np.percentile 25 / 75 neighbours, the smallest non-zero
    if (tid == 0) {
        auto nb = [&](double q, int up) {
            const double vi = double(n - 1) * (q / 100.0);
            int64_t r = int64_t(floor(vi)) + up;
            return r > n - 1 ? n - 1 : (r < 0 ? 0 : r);
        };
        sh.rank[0] = n / 2;
        sh.rank[1] = (n & 1) ? n / 2 : n / 2 - 1;
        sh.rank[2] = nb(25.0, 0);
        sh.rank[3] = nb(25.0, 1);
        sh.rank[4] = nb(75.0, 0);
        sh.rank[5] = nb(75.0, 1);
        sh.rank[6] = c_lt0 > 0 ? 0 : (c_le0 < n ? c_le0 : 0);
    }
    __syncthreads();
    if (n <= int64_t(FZ_DESC_NET_MAX)) {  // (the keys are staged: stage_cap >= the network >= n)
        // the network sized to the sample (kSelBlock * E keys): a 1,000-value sample takes the
        // 1,024-key network (55 stages of 2 keys a thread).  Only the small networks: the work of a
        // network is stages x keys a thread on one CU's four SIMDs (78 x 8 / 91 x 16 at 4,096 /
        // 8,192 keys: phase stamps 31 / 88 us, against 6 us for 1,024 keys and ~15 us for the
        // selection's passes)
        if (n <= int64_t(kSelBlock)) wg_bitonic_keys<1>(s_keys, n);
#if FZ_DESC_NET_MAX > 512
        else if (n <= int64_t(kSelBlock) * 2) wg_bitonic_keys<2>(s_keys, n);
#endif
#if FZ_DESC_NET_MAX > 1024
        else if (n <= int64_t(kSelBlock) * 4) wg_bitonic_keys<4>(s_keys, n);
#endif
#if FZ_DESC_NET_MAX > 2048
        else if (n <= int64_t(kSelBlock) * 8) wg_bitonic_keys<8>(s_keys, n);
#endif
#if FZ_DESC_NET_MAX > 4096
        else wg_bitonic_keys<16>(s_keys, n);
#endif
        if (tid < 7) sh.res[tid] = s_keys[sh.rank[tid]];
        __syncthreads();
    } else if (staged) {
        wg_select_global([&](int64_t i) { return s_keys[i]; }, n, lo, hi, 7, sh);
    } else {
        wg_select_global([=](int64_t i) { return f64_key(x[i]); }, n, lo, hi, 7, sh);
    }
    DESC_STAMP(8);
    if (tid != 0) return;
    auto get = [&](int64_t j) {
        uint64_t r = 0;
        for (int q = 0; q < 7; ++q)
            if (sh.rank[q] == j) r = sh.res[q];
        return f64_from_key(r);
    };
    fz_describe d;
    d.count = n;
    d.mean = mean;
    d.std = std;
    d.n_neg = c_lt0;
    d.n_zero = c_le0 - c_lt0;
    d.n_pos = c_leinf - c_le0;
    d.min = f64_from_key(lo);
    d.max = f64_from_key(hi);
    d.median = (n & 1) ? get(n / 2) : (get(n / 2 - 1) + get(n / 2)) / 2.0;
    d.q1 = np_percentile_sorted(get, n, 25.0);
    d.q3 = np_percentile_sorted(get, n, 75.0);
    if (c_lt0 > 0 || c_le0 < n) {
        d.min_nonzero = f64_from_key(sh.res[6]);
        d.has_nonzero = 1;
    } else {
        d.min_nonzero = NAN;
        d.has_nonzero = 0;
    }
    *out = d;
#ifdef FZ_DESC_TIMING
    if (blockIdx.x == 0) g_desc_t[9] = wall_clock64();
#endif
}

uint64_t *sorted_keys_dn(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n) {
    if (nmax <= 4096) return sort_small_keys(c, x, nmax < 1 ? 1 : nmax, d_n);  // one workgroup, LDS
    const int64_t nn = nmax < 1 ? 1 : nmax;
    uint64_t *k = c->arena.get<uint64_t>(nn);
    k_f64_keys<<<grid_for(nn, kBlock, 1024), kBlock, 0, c->stream>>>(x, nmax, d_n, k);
    FZ_LAUNCH_CHECK();
    uint32_t *none = nullptr;
    radix_sort_pairs_swap(c, k, none, nmax, 64);
    return k;
}

void describe_f64_dn(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n, fz_describe *dev_out) {
    const DescJob j{x, nmax, d_n, dev_out};
    describe_f64_dn_batch(c, &j, 1);
}

void describe_f64_dn_batch(fz_ctx *c, const DescJob *jobs, int njobs) {
    FZ_CHECK(njobs <= kDescBatch, "describe batch larger than kDescBatch");
    DescSmallArgs a{};
    SortedDescJob big[kDescBatch];
    int ns = 0, nb = 0;
    for (int i = 0; i < njobs; ++i) {
        const DescJob &j = jobs[i];
        if (j.nmax <= kDescSelMax) {  // by selection in one workgroup (any live length; re-reads)
            a.x[ns] = j.x;
            a.d_n[ns] = j.d_n;
            a.out[ns] = j.out;
            ++ns;
        } else {
            big[nb++] = SortedDescJob{sorted_keys_dn(c, j.x, j.nmax, j.d_n), j.x, j.nmax, j.d_n, j.out};
        }
    }
    if (ns > 0) {  // every such job in one launch
        // the staged keys' LDS: the bitonic network of the largest capacity (every live length fits
        // it), kSelLds beyond the networks
        int64_t cap = 1;
        for (int i = 0; i < njobs; ++i)
            if (jobs[i].nmax <= kDescSelMax) cap = jobs[i].nmax > cap ? jobs[i].nmax : cap;
        int64_t net = kSelBlock;
        while (net < cap && net < FZ_DESC_NET_MAX) net *= 2;
        a.stage_cap = cap > net || !FZ_DESC_LDS_FIT ? kSelLds : net;
        const size_t lds = size_t(a.stage_cap) * 8;
        if (lds > 65536)  // (per device: set on every such launch, never cached)
            FZ_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_describe_sel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(kSelLds * 8)));
        // (algorithmic bytes: one read of the first job's live values)
        ProbeScope ps(c, "describe_select", 0.0, a.d_n[0], 8.0);
        k_describe_sel<<<ns, kSelBlock, lds, c->stream>>>(a);
        FZ_LAUNCH_CHECK();
    }
    if (nb > 0) describe_sorted_dn_batch(c, big, nb);
}

void describe_sorted_dn_finish(fz_ctx *c, const SortedDescJob *jobs, int njobs, const double *ms) {
    FZ_CHECK(njobs >= 1 && njobs <= kDescBatch, "sorted describe batch size");
    SortedDescArgs a{};
    for (int i = 0; i < njobs; ++i) {
        a.k[i] = jobs[i].k;
        a.x[i] = jobs[i].x;
        a.d_n[i] = jobs[i].d_n;
        a.out[i] = jobs[i].out;
    }
    k_describe_finish<<<njobs, 64, 0, c->stream>>>(a, ms);
    FZ_LAUNCH_CHECK();
}

void describe_sorted_dn(fz_ctx *c, const uint64_t *k, const double *x, int64_t nmax, const int64_t *d_n,
                        fz_describe *dev_out) {
    const SortedDescJob j{k, x, nmax, d_n, dev_out};
    describe_sorted_dn_batch(c, &j, 1);
}

// The describes of up to kDescBatch sorted samples: five launches in all (two double-double passes
// of partial + final, one finish), each covering every job (blockIdx.y / blockIdx.x = job).
void describe_sorted_dn_batch(fz_ctx *c, const SortedDescJob *jobs, int njobs) {
    FZ_CHECK(njobs >= 1 && njobs <= kDescBatch, "sorted describe batch size");
    SortedDescArgs a{};
    int64_t nn = 1;
    for (int i = 0; i < njobs; ++i) {
        a.k[i] = jobs[i].k;
        a.x[i] = jobs[i].x;
        a.d_n[i] = jobs[i].d_n;
        a.out[i] = jobs[i].out;
        nn = jobs[i].nmax > nn ? jobs[i].nmax : nn;
    }
    const unsigned g = grid_for(nn, kBlock, 1024);
    double *part = c->arena.get<double>(2 * int64_t(g) * njobs);
    double *ms = c->arena.get<double>(2 * njobs);
    const dim3 gp(g, unsigned(njobs));
    // (the last block of each job folds its partials: no k_dd_final launches)
    unsigned *tk = fused_fold_on() && g <= 1024 ? seg_tickets(c, njobs) : nullptr;
    if (tk) {
        k_dd_partial<<<gp, kBlock, 0, c->stream>>>(a, nullptr, part, tk, 0, ms);
        k_dd_partial<<<gp, kBlock, 0, c->stream>>>(a, ms, part, tk, 1, ms);
    } else {
        k_dd_partial<<<gp, kBlock, 0, c->stream>>>(a, nullptr, part);
        k_dd_final<<<njobs, kBlock, 0, c->stream>>>(part, int(g), a, 0, ms);
        k_dd_partial<<<gp, kBlock, 0, c->stream>>>(a, ms, part);
        k_dd_final<<<njobs, kBlock, 0, c->stream>>>(part, int(g), a, 1, ms);
    }
    k_describe_finish<<<njobs, 64, 0, c->stream>>>(a, ms);
    FZ_LAUNCH_CHECK();
}

void describe_f64(fz_ctx *c, const double *x, int64_t n, fz_describe *dev_out) {
    int64_t *d_n = c->arena.get<int64_t>(1);
    k_set_i64<<<1, 64, 0, c->stream>>>(d_n, n < 0 ? 0 : n);
    FZ_LAUNCH_CHECK();
    describe_f64_dn(c, x, n < 0 ? 0 : n, d_n, dev_out);
}

// ----------------------------------------------------------------------- views / compaction

// Offsets of a project-sorted array of device length: row i starts the segments (proj[i-1], proj[i]]; the ids
// below the first row's and above the last row's are filled by id.  One coalesced read of proj
// instead of a ~20-step dependent binary search per id.
__global__ __launch_bounds__(kBlock) void k_segment_offsets_rows(const uint32_t *__restrict__ proj,
                                                                 const int64_t *__restrict__ d_n, int64_t n_cap,
                                                                 int64_t P, int64_t *__restrict__ offsets) {
    const int64_t n = d_n ? *d_n : n_cap;  // d_n null: the length is the host-known n_cap
    const int64_t first = n > 0 ? int64_t(proj[0]) : P + 1, last = n > 0 ? int64_t(proj[n - 1]) : -1;
    const int64_t span = n_cap > P + 1 ? n_cap : P + 1;
    // (wave-uniform trip count: the waves fill the gaps between consecutive rows' ids together)
    for (int64_t i0 = int64_t(blockIdx.x) * kBlock + (threadIdx.x & ~(kWave - 1)); i0 < span;
         i0 += int64_t(gridDim.x) * kBlock) {
        const int64_t i = i0 + lane_id();
        if (i <= P && i < span) {  // ids before the first row's and after the last row's
            if (i <= first) offsets[i] = 0;  // lower_bound of the first row's id is 0 too
            else if (i > last) offsets[i] = n;
        }
        int64_t a = 1, e = 0;
        if (i > 0 && i < n && i < span) {
            const int64_t pp = int64_t(proj[i - 1]), pc = int64_t(proj[i]);
            a = pp + 1;
            e = pc < P ? pc : P;  // ids stay in [0, P]
        }
        wave_fill_ranges(offsets, a, e, i);
    }
}

void segment_offsets_dn(fz_ctx *c, const uint32_t *sorted_proj, const int64_t *d_n, int64_t n_cap, int64_t P,
                        int64_t *offsets) {
    const int64_t span = n_cap > P + 1 ? n_cap : P + 1;
    k_segment_offsets_rows<<<grid_for(span, kBlock, 4096), kBlock, 0, c->stream>>>(sorted_proj, d_n, n_cap, P, offsets);
    FZ_LAUNCH_CHECK();
}

__global__ __launch_bounds__(kBlock) void k_count_flags(const uint8_t *__restrict__ f, int64_t n, int64_t *out) {
    __shared__ int64_t s_tmp[4];
    int64_t acc = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        acc += f[i] != 0;
    acc = block_sum(acc, s_tmp);
    if (threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long *>(out), (unsigned long long)acc);
}

struct FlagSets {
    const uint8_t *f[4];
    int64_t *out[4];
};
__global__ __launch_bounds__(kBlock) void k_count_flags_n(FlagSets fs, int64_t n) {  // blockIdx.y = set
    __shared__ int64_t s_tmp[4];
    const uint8_t *f = fs.f[blockIdx.y];
    int64_t acc = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        acc += f[i] != 0;
    acc = block_sum(acc, s_tmp);
    if (threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long *>(fs.out[blockIdx.y]), (unsigned long long)acc);
}

void count_flags_n(fz_ctx *c, const uint8_t *const *flags, int64_t *const *outs, int k, int64_t P) {
    FZ_CHECK(k >= 1 && k <= 4, "count_flags_n: 1..4 flag arrays");
    FlagSets fs{};
    for (int j = 0; j < k; ++j) {
        fs.f[j] = flags[j];
        fs.out[j] = outs[j];
    }
    k_count_flags_n<<<dim3(grid_for(P, kBlock, 256), unsigned(k)), kBlock, 0, c->stream>>>(fs, P);
    FZ_LAUNCH_CHECK();
}

void count_flags(fz_ctx *c, const uint8_t *flags, int64_t P, int64_t *out) {
    k_count_flags<<<grid_for(P, kBlock, 256), kBlock, 0, c->stream>>>(flags, P, out);
    FZ_LAUNCH_CHECK();
}

}  // namespace fz
