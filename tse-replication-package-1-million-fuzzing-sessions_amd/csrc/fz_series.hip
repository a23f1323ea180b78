// Segmented series operations (fz_seg.h): chunk maps, segmented sort, tie ranks, Spearman vs
// index, Shapiro-Wilk, percentiles, means, medians.
#include "fz_seg.h"
#include "fz_segsort.h"
#include "fz_stats.h"

namespace fz {

// ------------------------------------------------------------------------------ chunk maps
// chunks per segment; segments of <= min_len values get none (they are reduced elsewhere)
__global__ __launch_bounds__(kBlock) void k_chunk_count(const int64_t *__restrict__ offs, int64_t S, int64_t min_len,
                                                        int64_t *__restrict__ cnt) {
    for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < S; s += int64_t(gridDim.x) * kBlock) {
        const int64_t len = offs[s + 1] - offs[s];
        cnt[s] = len > min_len ? (len + kChunk - 1) / kChunk : 0;
    }
}

// Size-class lists (fz_seg.h SegLists).  Each workgroup owns a contiguous range of segments: it
// counts its classes (pass 1), reserves its slice of every list with one atomic per class, then
// writes the ids in order (pass 2) - a few thousand atomics in all instead of one per wave.
__device__ inline int seg_class(int64_t len) {
    return len <= kMicroSeg ? -1
           : len <= kTinySeg ? kClassTiny
           : len <= 1024 ? kClassMid
           : len <= kLdsSortMax ? kClassWide : kClassBig;
}
__device__ inline bool in_class(int cls, int k) { return k == kClassNonTiny ? cls > kClassTiny : cls == k; }

__global__ __launch_bounds__(kBlock) void k_seg_classes(const int64_t *__restrict__ offs, int64_t S, SegLists L) {
    __shared__ unsigned long long s_run[kNumClasses];
    __shared__ unsigned s_wave[4][kNumClasses];
    const int tid = threadIdx.x, w = wave_id();
    const int64_t per = (S + gridDim.x - 1) / gridDim.x;
    const int64_t s0 = int64_t(blockIdx.x) * per, s1 = s0 + per < S ? s0 + per : S;
    if (tid < kNumClasses) s_run[tid] = 0;
    __syncthreads();
    unsigned cnt[kNumClasses] = {};
    for (int64_t s = s0 + tid; s < s1; s += kBlock) {
        const int cls = seg_class(offs[s + 1] - offs[s]);
#pragma unroll
        for (int k = 0; k < kNumClasses; ++k) cnt[k] += in_class(cls, k);
    }
#pragma unroll
    for (int k = 0; k < kNumClasses; ++k) {
        const unsigned v = wave_sum(cnt[k]);
        if (lane_id() == 0 && v) atomicAdd(&s_run[k], (unsigned long long)v);
    }
    __syncthreads();
    if (tid < kNumClasses && s_run[tid])
        s_run[tid] = atomicAdd(reinterpret_cast<unsigned long long *>(L.d_n + tid), s_run[tid]);
    __syncthreads();
    for (int64_t base = s0; base < s1; base += kBlock) {
        const int64_t s = base + tid;
        const int cls = s < s1 ? seg_class(offs[s + 1] - offs[s]) : -1;
        uint64_t m[kNumClasses];
#pragma unroll
        for (int k = 0; k < kNumClasses; ++k) {
            m[k] = __ballot(in_class(cls, k));
            if (lane_id() == 0) s_wave[w][k] = unsigned(__popcll(m[k]));
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kNumClasses; ++k) {
            if (!in_class(cls, k)) continue;
            unsigned before = 0;
            for (int v = 0; v < w; ++v) before += s_wave[v][k];
            L.ids[k][s_run[k] + before + unsigned(__popcll(m[k] & lanemask_lt()))] = int32_t(s);
        }
        __syncthreads();
        if (tid < kNumClasses) s_run[tid] += s_wave[0][tid] + s_wave[1][tid] + s_wave[2][tid] + s_wave[3][tid];
        __syncthreads();
    }
}

SegLists seg_lists(fz_ctx *c, const Segs &sg) {
    SegLists L;
    L.on = true;
    const int64_t S = sg.S, n = sg.n_cap;
    auto bound = [&](int64_t minlen) { return (S < n / (minlen + 1) + 1 ? S : n / (minlen + 1) + 1); };
    L.cap[kClassTiny] = bound(kMicroSeg);
    L.cap[kClassMid] = bound(kTinySeg);
    L.cap[kClassWide] = bound(1024);
    L.cap[kClassBig] = bound(kLdsSortMax);
    L.cap[kClassNonTiny] = bound(kTinySeg);
    L.d_n = c->arena.get<int64_t>(kNumClasses);
    for (int k = 0; k < kNumClasses; ++k) L.ids[k] = c->arena.get<int32_t>(L.cap[k]);
    dev_fill(c, L.d_n, 0, kNumClasses * 8);
    if (S > 0) {
        k_seg_classes<<<grid_for(S, kBlock, 2048), kBlock, 0, c->stream>>>(sg.offs, S, L);
        FZ_LAUNCH_CHECK();
    }
    return L;
}

__global__ __launch_bounds__(kBlock) void k_chunk_fill(const int64_t *__restrict__ offs, int64_t S,
                                                       const int64_t *__restrict__ coff, ChunkMap cm) {
    const int64_t n = *cm.d_n;
    for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < n; k += int64_t(gridDim.x) * kBlock) {
        const int64_t s = upper_bound_i64(coff, 0, S + 1, k) - 1;
        const int64_t b = offs[s] + (k - coff[s]) * kChunk;
        const int64_t e = b + kChunk < offs[s + 1] ? b + kChunk : offs[s + 1];
        cm.seg[k] = int32_t(s);
        cm.begin[k] = b;
        cm.end[k] = e;
    }
}

ChunkedSegs chunked(fz_ctx *c, const Segs &sg) {
    ChunkedSegs cs;
    cs.sg = sg;
    // Short segments: implicit chunks (no map kernels) while the grid stays near the explicit
    // one - an empty chunk's workgroup exits after two offset loads.
    // (Very many segments: tiny ones are reduced one per thread, an explicit map covers the others.)
    const bool many = sg.S > kManySegs;
    const int64_t cps = sg.len_bound() > kChunk ? (sg.len_bound() + kChunk - 1) / kChunk : 1;
    const int64_t explicit_cap = sg.S + sg.n_cap / kChunk + 1;
    if (sg.S > 0 && !many && (cps == 1 || sg.S * cps <= 2 * explicit_cap + 4096) && sg.S * cps < (int64_t(1) << 31)) {
        cs.cps = cps;
        return cs;
    }
    ChunkMap &cm = cs.cm;
    if (many) cs.lists = seg_lists(c, sg);
    const int64_t nontiny = sg.S < sg.n_cap / (kTinySeg + 1) + 1 ? sg.S : sg.n_cap / (kTinySeg + 1) + 1;
    cm.cap = (many ? nontiny : sg.S) + sg.n_cap / kChunk + 1;
    cm.d_n = c->arena.get<int64_t>(1);
    cm.seg = c->arena.get<int32_t>(cm.cap);
    cm.begin = c->arena.get<int64_t>(cm.cap);
    cm.end = c->arena.get<int64_t>(cm.cap);
    cs.chunk_off = c->arena.get<int64_t>(sg.S + 1);
    int64_t *cnt = c->arena.get<int64_t>(sg.S + 1);
    dev_fill(c, cnt, 0, (sg.S + 1) * 8);
    if (sg.S > 0) {
        k_chunk_count<<<grid_for(sg.S), kBlock, 0, c->stream>>>(sg.offs, sg.S, many ? kTinySeg : -1, cnt);
        FZ_LAUNCH_CHECK();
    }
    scan_exclusive_i64(c, cnt, cs.chunk_off, sg.S + 1, cm.d_n);
    k_chunk_fill<<<grid_for(cm.cap, kBlock, 4096), kBlock, 0, c->stream>>>(sg.offs, sg.S, cs.chunk_off, cm);
    FZ_LAUNCH_CHECK();
    return cs;
}

ChunkMap make_chunks(fz_ctx *c, const Segs &sg) { return chunked(c, sg).cm; }

// (off by default: same-box A/B at config 2, 1.239 ms/step with the separate fold launches against
// 1.274 with the last-arriver folds - the write-through stores and the ticket round trip in every
// workgroup cost more than the launches they save; FZ_FUSED_FOLD=1 turns them on)
bool fused_fold_on() {
    static const bool on = [] {
        const char *e = std::getenv("FZ_FUSED_FOLD");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

unsigned *seg_tickets(fz_ctx *c, int64_t S) {
    // (grown rarely - the first sizes already cover the analyses' reductions - and zeroed once: a
    // recording made after a growth stays valid, one made before it is refused at replay)
    if (c->seg_tickets.cap < size_t(S) * sizeof(unsigned)) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        FZ_HIP(hipStreamIsCapturing(c->stream, &cap));
        if (cap != hipStreamCaptureStatusNone) return nullptr;  // (no allocation while recording: unfused)
        const int64_t n = S > 16384 ? S : 16384;
        unsigned *t = c->seg_tickets.ensure<unsigned>(n);
        dev_fill(c, t, 0, n * int64_t(sizeof(unsigned)));
    }
    return c->seg_tickets.as<unsigned>();
}

// Segment id of every position (positions past offs[S] get S).  A workgroup takes a chunk of
// kIdChunk positions: one search finds the segments of its first and last position, and a position
// searches only between those (none at all when one segment covers the chunk - long sessions);
// a per-position search over all S + 1 offsets cost ~log2(S) dependent loads per value.
constexpr int kIdChunk = 4096;
__global__ __launch_bounds__(kBlock) void k_segment_ids(const int64_t *__restrict__ offs, int64_t S, int64_t n,
                                                        int32_t *__restrict__ id) {
    __shared__ int64_t s_rng[2];
    for (int64_t c0 = int64_t(blockIdx.x) * kIdChunk; c0 < n; c0 += int64_t(gridDim.x) * kIdChunk) {
        const int64_t c1 = c0 + kIdChunk < n ? c0 + kIdChunk : n;
        if (threadIdx.x == 0) {
            const int64_t lo = upper_bound_i64(offs, 0, S + 1, c0) - 1;
            s_rng[0] = lo;
            s_rng[1] = upper_bound_i64(offs, lo > 0 ? lo : 0, S + 1, c1 - 1) - 1;
        }
        __syncthreads();
        const int64_t lo = s_rng[0], hi = s_rng[1];
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock) {
            const int64_t s = lo == hi ? lo : upper_bound_i64(offs, lo > 0 ? lo : 0, hi + 1, i) - 1;
            id[i] = int32_t(s > S ? S : (s < 0 ? 0 : s));
        }
        __syncthreads();  // s_rng is rewritten for the next chunk
    }
}

int32_t *segment_ids(fz_ctx *c, const Segs &sg) {
    int32_t *id = c->arena.get<int32_t>(sg.n_cap);
    if (sg.n_cap <= 0) return id;
    const int64_t chunks = (sg.n_cap + kIdChunk - 1) / kIdChunk;
    k_segment_ids<<<unsigned(chunks < 8192 ? chunks : 8192), kBlock, 0, c->stream>>>(sg.offs, sg.S, sg.n_cap, id);
    FZ_LAUNCH_CHECK();
    return id;
}

const int64_t *single_segment(fz_ctx *c, const int64_t *d_n) {
    int64_t *o = c->arena.get<int64_t>(2);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        o[0] = 0;
        o[1] = *d_n;
    });
    return o;
}

// -------------------------------------------------------------------------- segmented sort
// One workgroup per segment of <= kLdsSortMax values: bitonic network over (key, position) pairs
// in LDS (48 KiB), padded to a power of two with +inf keys.  Ties may come out in any order -
// every consumer (ranks, percentiles, rank tests) is invariant to the order inside a tie group.
// Two instantiations: BS = 256 threads for segments of <= 1024 values (small LDS footprint, many
// workgroups per CU) and BS = 1024 for 1025..4096; each skips the other's segments.
#ifndef FZ_SL_BLOCK
#define FZ_SL_BLOCK 1024
#endif
constexpr int kLdsSortBlock = FZ_SL_BLOCK;  // threads of the 1025..4096-value class
template <int BS, int MAXN>
__global__ __launch_bounds__(BS) void k_seg_sort_lds(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                     int64_t S, double *__restrict__ out_val,
                                                     int32_t *__restrict__ out_pos, uint64_t *__restrict__ out_key,
                                                     const int32_t *__restrict__ list, const int64_t *__restrict__ d_ln) {
    __shared__ uint64_t sk[MAXN];
    __shared__ int32_t sp[MAXN];
    constexpr int kMinN = MAXN / 4;
    const int tid = threadIdx.x;
    const int64_t ns = list ? *d_ln : S;
    for (int64_t w = blockIdx.x; w < ns; w += gridDim.x) {
        const int64_t s = list ? list[w] : w;
        const int64_t b = offs[s];
        const int n = int(offs[s + 1] - b);
        if (n <= 0 || n > MAXN || (MAXN == kLdsSortMax && n <= kMinN)) continue;
        int np2 = 1;
        while (np2 < n) np2 <<= 1;
        for (int i = tid; i < np2; i += BS) {
            sk[i] = i < n ? f64_key(src[b + i]) : ~0ull;
            sp[i] = i;
        }
        __syncthreads();
        for (int k = 2; k <= np2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = tid; t < (np2 >> 1); t += BS) {  // every thread owns a pair
                    const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ixj = i + j;  // j = 2^m
                    {
                        const uint64_t a = sk[i], d = sk[ixj];
                        const bool up = (i & k) == 0;
                        if ((a > d) == up) {
                            sk[i] = d;
                            sk[ixj] = a;
                            const int32_t t = sp[i];
                            sp[i] = sp[ixj];
                            sp[ixj] = t;
                        }
                    }
                }
                bitonic_stage_sync(k, j, np2);
            }
        }
        for (int i = tid; i < n; i += BS) {
            if (out_val) out_val[b + i] = f64_from_key(sk[i]);
            if (out_pos) out_pos[b + i] = int32_t(b + sp[i]);
            if (out_key) out_key[b + i] = sk[i];
        }
        __syncthreads();
    }
}

// Every segment of <= kMicroSeg values: one thread each, Batcher's 19-comparator network on
// (key, position) pairs in registers.
__device__ inline void ce_kv(uint64_t &ka, uint32_t &pa, uint64_t &kb, uint32_t &pb) {
    if (kb < ka || (kb == ka && pb < pa)) {
        const uint64_t tk = ka;
        const uint32_t tp = pa;
        ka = kb;
        pa = pb;
        kb = tk;
        pb = tp;
    }
}
__global__ __launch_bounds__(kBlock) void k_seg_sort_micro(const double *__restrict__ src,
                                                           const int64_t *__restrict__ offs, int64_t S,
                                                           double *__restrict__ out_val, int32_t *__restrict__ out_pos) {
    for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < S; s += int64_t(gridDim.x) * kBlock) {
        const int64_t b = offs[s];
        const int n = int(offs[s + 1] - b);
        if (n > kMicroSeg || n <= 0) continue;
        uint64_t k[kMicroSeg];
        uint32_t p[kMicroSeg];
#pragma unroll
        for (int q = 0; q < kMicroSeg; ++q) {
            k[q] = q < n ? f64_key(src[b + q]) : ~0ull;
            p[q] = uint32_t(q);
        }
        constexpr int net[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
                                    {0, 4}, {1, 5}, {2, 6}, {3, 7}, {2, 4}, {3, 5}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
        for (int c = 0; c < 19; ++c) ce_kv(k[net[c][0]], p[net[c][0]], k[net[c][1]], p[net[c][1]]);
#pragma unroll
        for (int q = 0; q < kMicroSeg; ++q) {
            if (q < n) {
                if (out_val) out_val[b + q] = f64_from_key(k[q]);
                if (out_pos) out_pos[b + q] = int32_t(b + p[q]);
            }
        }
    }
}

// Segments of kMicroSeg < len <= kTinySeg values from a list: one wave each, a 64-lane bitonic
// network on (key, position) in registers (ties by position: deterministic).
__global__ __launch_bounds__(kBlock) void k_seg_sort_wave(const double *__restrict__ src,
                                                          const int64_t *__restrict__ offs,
                                                          const int32_t *__restrict__ list,
                                                          const int64_t *__restrict__ d_ln, double *__restrict__ out_val,
                                                          int32_t *__restrict__ out_pos) {
    const int64_t ns = *d_ln;
    const int lane = lane_id();
    for (int64_t w = int64_t(blockIdx.x) * 4 + wave_id(); w < ns; w += int64_t(gridDim.x) * 4) {
        const int64_t s = list[w], b = offs[s];
        const int n = int(offs[s + 1] - b);
        unsigned long long k = lane < n ? f64_key(src[b + lane]) : ~0ull;
        unsigned p = unsigned(lane);
#pragma unroll
        for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
            for (int j = kk >> 1; j > 0; j >>= 1) {
                const unsigned long long ok = __shfl_xor(k, j, 64);
                const unsigned op = __shfl_xor(p, j, 64);
                const bool other_less = ok < k || (ok == k && op < p);
                const bool want_min = ((lane & j) == 0) == ((lane & kk) == 0);
                if (want_min == other_less) {
                    k = ok;
                    p = op;
                }
            }
        }
        if (lane < n) {
            if (out_val) out_val[b + lane] = f64_from_key(k);
            if (out_pos) out_pos[b + lane] = int32_t(b + p);
        }
    }
}

// Value bucket sort, one workgroup per segment of min_len < n <= MAXN values (the store's time
// sort, fz_store.hip k_seg_time_bucket, over f64 values): n buckets over the segment's range
// [lo, hi] of the order-preserving image f64_key - the bucket of key k is
// floor((k - lo) * n / (hi - lo + 1)), monotone in k - counted with LDS atomics (the returned count
// is the value's slot in its bucket), bucket starts by one block scan, and a value's output slot is
// its bucket start plus the number of values of its bucket ordered before it by (key, position):
// a total order, so equal values keep their input order (stable, like the merge sort).  O(n) work
// for values spread over their range - coverage series and sessions - against the bitonic
// network's O(n log^2 n) compare-exchanges with a barrier per stage.  A segment whose largest
// bucket holds more than kValSkew values (ties, clusters) is sorted by the LDS bitonic network on
// (key, position) inside the same workgroup (MAXN <= 4096: keys in LDS), or flagged for the
// segmented merge sort (the 16384 class, which re-reads keys from the cache-resident column).
constexpr int kValSkew = 32;
#ifndef FZ_VB4_BLOCK
#define FZ_VB4_BLOCK 1024
#endif
#ifndef FZ_VB_C16
#define FZ_VB_C16 1  // 16-bit counters in the 16,384 class (0: 32-bit, the A/B baseline)
#endif
#ifndef FZ_VB_WPE
#define FZ_VB_WPE 8  // its waves per SIMD: two 1,024-thread workgroups per CU (64 VGPRs)
#endif
#ifndef FZ_VB_SMALL_WPE
#define FZ_VB_SMALL_WPE 8  // the 256- / 512-thread classes (102 / 104 -> 64 registers): config 5L 34.00 -> 33.84 ms
                           // (profiles/r06_filter_items_vb_small_ab.txt)
#endif
#ifndef FZ_VB4_WPE
#define FZ_VB4_WPE 8  // the same for the 4,096 class: 98 -> 63 registers, two workgroups per CU, the kernel
                      // 296 -> 191 us and config 3L 19.54 -> 18.72 ms (profiles/r06_occupancy_ab.txt); the
                      // 256- and 512-thread classes keep the compiler's choice (config 2 a hair slower capped)
#endif
constexpr int kVb4Block = FZ_VB4_BLOCK;                 // threads per workgroup of the 2049..4096 class
constexpr int kVb4Grid = 2048 * (1024 / FZ_VB4_BLOCK);  // its persistent grid (same threads in all)
template <int BS, int MAXN>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(MAXN > kLdsSortMax ? (FZ_VB_C16 ? FZ_VB_WPE : 1) : (BS == 1024 ? FZ_VB4_WPE : FZ_VB_SMALL_WPE))))
void k_seg_val_bucket(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                       int64_t S, int64_t min_len, double *__restrict__ out_val,
                                                       int32_t *__restrict__ out_pos, const int32_t *__restrict__ list,
                                                       const int64_t *__restrict__ d_ln, uint8_t *__restrict__ bigflag,
                                                       bool flag_longer) {
    constexpr int IPT = MAXN / BS;  // values (and buckets in the scan) per thread
    constexpr int NW = BS / kWave;
    constexpr bool KEYS_LDS = MAXN <= kLdsSortMax;
    // the class without its keys in LDS counts in 16-bit halves of the counter words (counts, starts
    // and staged positions are < 65,536): 66 KB of LDS instead of 99 KB, two workgroups per CU
    constexpr bool C16 = !KEYS_LDS && FZ_VB_C16;
    constexpr int CNT_WORDS = C16 ? (MAXN + 2) / 2 + 1 : MAXN + 1;
    static_assert(MAXN <= 16384 && MAXN % BS == 0 && (MAXN & (MAXN - 1)) == 0, "value bucket sort shape");
    static_assert(KEYS_LDS || CNT_WORDS + MAXN / 2 >= MAXN, "value staging: MAXN / 2 u64 slots");
    // bucket counts, then starts (+ sentinel), then staging; positions in bucket order (u16, bitonic
    // fallback: pair positions) right after them
    __shared__ alignas(8) uint32_t s_mem[CNT_WORDS + MAXN / 2];
    uint32_t *const s_cnt = s_mem;
    uint16_t *const c16 = reinterpret_cast<uint16_t *>(s_mem);
    uint16_t *const s_pos = reinterpret_cast<uint16_t *>(s_mem + CNT_WORDS);
    auto cnt_get = [&](uint32_t q) -> uint32_t {
        if constexpr (C16) return c16[q];
        else return s_cnt[q];
    };
    auto cnt_set = [&](uint32_t q, uint32_t v) {
        if constexpr (C16) c16[q] = uint16_t(v);
        else s_cnt[q] = v;
    };
    __shared__ uint64_t s_key[KEYS_LDS ? MAXN : 1];
    __shared__ uint64_t s_lo[NW], s_hi[NW];
    __shared__ uint32_t s_tmp[NW], s_max[NW];
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    const int64_t ns = list ? *d_ln : S;
    for (int64_t it = blockIdx.x; it < ns; it += gridDim.x) {
        const int64_t s = list ? list[it] : it;
        const int64_t b = offs[s];
        const int64_t len = offs[s + 1] - b;
        if (len <= min_len) continue;
        if (len > MAXN) {
            if (flag_longer && tid == 0) bigflag[s] = 1;
            continue;
        }
        const int n = int(len);
        uint64_t k[IPT];
        uint64_t lo = ~0ull, hi = 0ull;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            k[m] = i < n ? f64_key(src[b + i]) : 0ull;
            if (i < n) {
                lo = k[m] < lo ? k[m] : lo;
                hi = k[m] > hi ? k[m] : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane == 0) {
            s_lo[w] = lo;
            s_hi[w] = hi;
        }
        for (int j = tid; j < CNT_WORDS; j += BS) s_cnt[j] = 0u;
        __syncthreads();
        lo = ~0ull;
        hi = 0ull;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            lo = s_lo[q] < lo ? s_lo[q] : lo;
            hi = s_hi[q] > hi ? s_hi[q] : hi;
        }
        const double scale = double(n) / (double(hi - lo) + 1.0);
        uint32_t bs[IPT];  // bucket << 16 | slot in the bucket
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            bs[m] = 0u;
            if (i < n) {
                // (C16: re-read, coalesced, from the cache-resident segment - no key held across
                // the barrier)
                const uint64_t km = C16 ? f64_key(src[b + i]) : k[m];
                uint32_t q = uint32_t(double(km - lo) * scale);
                q = q < uint32_t(n) ? q : uint32_t(n - 1);
                uint32_t slot;
                if constexpr (C16) {  // (a half never exceeds n <= 16,384: no carry into its neighbour)
                    const uint32_t sh = (q & 1u) << 4;
                    slot = (atomicAdd(&s_cnt[q >> 1], 1u << sh) >> sh) & 0xffffu;
                } else {
                    slot = atomicAdd(&s_cnt[q], 1u);
                }
                bs[m] = (q << 16) | slot;
                if (KEYS_LDS) s_key[i] = k[m];
            }
        }
        __syncthreads();
        // bucket starts: each thread scans IPT consecutive buckets; the largest bucket decides skew
        uint32_t sum = 0, mx = 0;
#pragma unroll
        for (int e = 0; e < IPT; ++e) {
            const uint32_t ce = cnt_get(tid * IPT + e);
            sum += ce;
            mx = ce > mx ? ce : mx;
        }
        mx = wave_max(mx);
        if (lane == 0) s_max[w] = mx;
        uint32_t run = block_excl_scan<uint32_t, NW>(sum, s_tmp, (uint32_t *)nullptr);
#pragma unroll
        for (int e = 0; e < IPT; ++e) {  // (block_excl_scan's barriers ordered every read above)
            const uint32_t ce = cnt_get(tid * IPT + e);
            cnt_set(tid * IPT + e, run);
            run += ce;
        }
        if (tid == 0) cnt_set(MAXN, uint32_t(n));
        __syncthreads();
        uint32_t gmax = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) gmax = s_max[q] > gmax ? s_max[q] : gmax;
        if (gmax > uint32_t(kValSkew)) {
            if constexpr (KEYS_LDS) {
                // ties / clusters: bitonic network on (key, position), keys already in LDS
                int np2 = 1;
                while (np2 < n) np2 <<= 1;
                for (int i = tid; i < np2; i += BS) {
                    if (i >= n) s_key[i] = ~0ull;
                    s_pos[i] = uint16_t(i);
                }
                __syncthreads();
                for (int kk = 2; kk <= np2; kk <<= 1) {
                    for (int j = kk >> 1; j > 0; j >>= 1) {
                        for (int t = tid; t < (np2 >> 1); t += BS) {
                            const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ixj = i + j;
                            const uint64_t ka = s_key[i], kb = s_key[ixj];
                            const uint16_t pa = s_pos[i], pb = s_pos[ixj];
                            if ((kb < ka || (kb == ka && pb < pa)) == ((i & kk) == 0)) {
                                s_key[i] = kb;
                                s_key[ixj] = ka;
                                s_pos[i] = pb;
                                s_pos[ixj] = pa;
                            }
                        }
                        bitonic_stage_sync(kk, j, np2);
                    }
                }
                for (int i = tid; i < n; i += BS) {
                    out_val[b + i] = f64_from_key(s_key[i]);
                    out_pos[b + i] = int32_t(b + s_pos[i]);
                }
            } else {
                if (tid == 0) bigflag[s] = 1;
            }
            __syncthreads();  // LDS is reused by the next segment
            continue;
        }
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            if (i < n) s_pos[cnt_get(bs[m] >> 16) + (bs[m] & 0xffffu)] = uint16_t(i);
        }
        __syncthreads();
        int32_t dq[IPT];  // sorted position of value i inside the segment
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * BS;
            dq[m] = -1;
            if (i >= n) continue;
            const uint32_t st = cnt_get(bs[m] >> 16), en = cnt_get((bs[m] >> 16) + 1);
            uint32_t rank = 0;
            if (en - st > 1) {  // (alone in its bucket: rank 0)
                // (C16: the key re-read from the cache-resident segment - k[] is dead past the
                // bucketing, which keeps the class at 64 registers, two workgroups per CU)
                const uint64_t km = C16 ? f64_key(src[b + i]) : k[m];
                for (uint32_t x = st; x < en; ++x) {
                    const int ox = s_pos[x];
                    if (ox == i) continue;
                    const uint64_t kx = KEYS_LDS ? s_key[ox] : f64_key(src[b + ox]);
                    rank += (kx < km) || (kx == km && ox < i);
                }
            }
            dq[m] = int32_t(st + rank);
        }
        __syncthreads();  // the rank loops' LDS reads are done: LDS is staging now
        // coalesced output: positions, then values, staged in sorted order (u32 slots for the whole
        // segment in the bucket counts; u64 slots in the key array, or half a segment per round in
        // the bucket counts when the keys are not in LDS)
        // (C16: the segment-local position, b added on the way out)
#pragma unroll
        for (int m = 0; m < IPT; ++m)
            if (dq[m] >= 0) cnt_set(dq[m], C16 ? uint32_t(tid + m * BS) : uint32_t(b + tid + m * BS));
        __syncthreads();
        if constexpr (C16) {
            // the values gathered by the staged positions from the cache-resident segment (the
            // value is the key's bijective image: the same bits as a staged key)
            for (int q = tid; q < n; q += BS) {
                const uint32_t lp = cnt_get(q);
                out_pos[b + q] = int32_t(uint32_t(b) + lp);
                out_val[b + q] = src[b + lp];
            }
            __syncthreads();  // LDS is reused by the next segment
            continue;
        }
        for (int q = tid; q < n; q += BS) out_pos[b + q] = int32_t(cnt_get(q));
        __syncthreads();
        uint64_t *stg = KEYS_LDS ? s_key : reinterpret_cast<uint64_t *>(s_mem);
        constexpr int CAP = KEYS_LDS ? MAXN : MAXN / 2;
        for (int h = 0; h < n; h += CAP) {
#pragma unroll
            for (int m = 0; m < IPT; ++m)
                if (dq[m] >= h && dq[m] < h + CAP) stg[dq[m] - h] = k[m];
            __syncthreads();
            const int e = n - h < CAP ? n - h : CAP;
            for (int q = tid; q < e; q += BS) out_val[b + h + q] = f64_from_key(stg[q]);
            __syncthreads();
        }
        __syncthreads();  // LDS is reused by the next segment
    }
}

// Every segment of <= kLdsSortMax values (len_bound: a host bound of the longest one); with lists,
// each kernel walks its own size class only.
static void launch_seg_sort_lds(fz_ctx *c, unsigned g, const double *src, const int64_t *offs, int64_t S,
                                int64_t len_bound, double *val, int32_t *pos, uint64_t *key,
                                const SegLists *L = nullptr) {
    if (L && L->on) {
        auto grid = [](int64_t cap, int64_t lim) { return unsigned(cap < 1 ? 1 : (cap < lim ? cap : lim)); };
        k_seg_sort_micro<<<grid_for(S, kBlock, 8192), kBlock, 0, c->stream>>>(src, offs, S, val, pos);
        k_seg_sort_wave<<<grid((L->cap[kClassTiny] + 3) / 4, 8192), kBlock, 0, c->stream>>>(
            src, offs, L->ids[kClassTiny], L->d_n + kClassTiny, val, pos);
        k_seg_sort_lds<256, 1024><<<grid(L->cap[kClassMid], 8192), 256, 0, c->stream>>>(
            src, offs, S, val, pos, key, L->ids[kClassMid], L->d_n + kClassMid);
        if (len_bound > 1024)
            k_seg_sort_lds<kLdsSortBlock, kLdsSortMax><<<grid(L->cap[kClassWide], 8192), kLdsSortBlock, 0, c->stream>>>(
                src, offs, S, val, pos, key, L->ids[kClassWide], L->d_n + kClassWide);
        FZ_LAUNCH_CHECK();
        return;
    }
    k_seg_sort_lds<256, 1024><<<g, 256, 0, c->stream>>>(src, offs, S, val, pos, key, nullptr, nullptr);
    if (len_bound > 1024)
        k_seg_sort_lds<kLdsSortBlock, kLdsSortMax><<<g, kLdsSortBlock, 0, c->stream>>>(src, offs, S, val, pos, key,
                                                                                        nullptr, nullptr);
    FZ_LAUNCH_CHECK();
}

uint64_t *sort_small_keys(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n) {
    uint64_t *k = c->arena.get<uint64_t>(nmax);
    const int64_t *offs = single_segment(c, d_n);
    map_n(c, nmax, nullptr, [=] __device__(int64_t i) { k[i] = ~0ull; });  // entries past *d_n
    launch_seg_sort_lds(c, 1, x, offs, 1, nmax, nullptr, nullptr, k);
    return k;
}

#ifndef FZ_TILE_BUCKETS
// 1: the merge sort's tile phase tries a bucket sort first (fz_segsort.h) - measured slower and
// kept off (same box: c5L 35.06 vs 34.82 ms, c4 3.01 vs 2.90; profiles/r06_tile_buckets_ab.txt):
// tied tiles pay the attempt and the network
#define FZ_TILE_BUCKETS 0
#endif
struct F64Key {
    static constexpr bool kBuckets = FZ_TILE_BUCKETS;
    const double *src;
    __device__ uint64_t operator()(int64_t i) const { return f64_key(src[i]); }
};
struct F64Sink {
    double *val;
    int32_t *pos;
    __device__ void operator()(int32_t, int64_t q, uint64_t k, uint32_t v) const {
        val[q] = f64_from_key(k);
        pos[q] = int32_t(v);
    }
};

// One segment [offs[0], offs[1]) of a value array as radix keys: positions before it key 0, after
// it ~0, so a stable sort of the whole array leaves them where they are and the segment's values
// sorted in between; payload = the position.
// (only the positions before hi are keyed and sorted: the sort is bounded by offs[1], the
// positions past it are left undefined)
__global__ __launch_bounds__(kBlock) void k_f64_seg1_keys(const double *__restrict__ x, int64_t n,
                                                          const int64_t *__restrict__ offs, uint64_t *__restrict__ k,
                                                          uint32_t *__restrict__ v) {
    const int64_t lo = offs[0], hi = offs[1] < n ? offs[1] : n;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < hi; i += int64_t(gridDim.x) * kBlock) {
        k[i] = i < lo ? 0ull : f64_key(x[i]);
        v[i] = uint32_t(i);
    }
}

__global__ __launch_bounds__(kBlock) void k_f64_from_keys(const uint64_t *__restrict__ k, const uint32_t *__restrict__ v,
                                                          int64_t n_cap, const int64_t *__restrict__ offs,
                                                          double *__restrict__ val, int32_t *__restrict__ pos) {
    const int64_t n = offs[1] < n_cap ? offs[1] : n_cap;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        val[i] = f64_from_key(k[i]);
        pos[i] = int32_t(v[i]);
    }
}

// (the sample sort's work follows the live length - config 3 / 5's empty RQ3 union of 1e8 capacity
// costs five short launches, where the merge sort's tile and merge rounds were ~25 - and its range
// buckets average 1/128 of the live values: 6 K at config 2's 0.8 M, against an LDS capacity of
// 12 K; a longer bucket - a live union of several million - takes the slower in-workgroup merge)
constexpr int64_t kSampleSortMax = (int64_t(1) << 31) - 1;
// The segments the bucket sorts flagged (longer than 16,384 values, or skewed) by LSD radix passes
// instead of the merge rounds: their values copied back to back in position order (64-bit keys,
// positions), 8 stable passes on the value key over the live rows, then stable passes on the
// segment index (positions ride as values, the value keys as payload) - the result is each
// segment's (value, position) order, the merge sort's own order.
// Measured slower and kept off: config 5L 37.28 vs 36.46 ms with the merge rounds (same box,
// profiles/r06_big_radix_ab.txt) - a recorded graph runs all eight value passes over ~75 M keys,
// and the segment passes carry the 8-byte keys; the merge rounds' late rounds touch only the
// longest segments.
#ifndef FZ_BIG_RADIX
#define FZ_BIG_RADIX 0
#endif
#ifndef FZ_BIG_RADIX_MIN
#define FZ_BIG_RADIX_MIN (1 << 20)  // longest flagged segment from which the radix path pays (merge rounds)
#endif
constexpr int64_t kBigRadixMin = FZ_BIG_RADIX_MIN;
__global__ __launch_bounds__(kBlock) void k_big_len(const int64_t *__restrict__ offs, int64_t S,
                                                    const uint8_t *__restrict__ flag, int64_t *__restrict__ len) {
    for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s <= S; s += int64_t(gridDim.x) * kBlock)
        len[s] = s < S && flag[s] ? offs[s + 1] - offs[s] : 0;
}
// tile k of the map: its rows at cofs[s] + (row - offs[s]) of the packed arrays
__global__ __launch_bounds__(kBlock) void k_big_pack(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                     const int64_t *__restrict__ cofs, TileMap tm,
                                                     uint64_t *__restrict__ key, uint32_t *__restrict__ pos) {
    const int64_t nt = *tm.d_n;
    for (int64_t k = blockIdx.x; k < nt; k += gridDim.x) {
        const int32_t s = tm.seg[k];
        const int64_t b = tm.begin[k], e = b + kTile < offs[s + 1] ? b + kTile : offs[s + 1];
        const int64_t base = cofs[s] - offs[s];
        for (int64_t r = b + threadIdx.x; r < e; r += kBlock) {
            key[base + r] = f64_key(src[r]);
            pos[base + r] = uint32_t(r);
        }
    }
}
// after the value passes: each packed row's segment index (dead rows past the live count: S)
__global__ __launch_bounds__(kBlock) void k_big_segkey(const int64_t *__restrict__ offs, int64_t S,
                                                       const uint32_t *__restrict__ pos, const int64_t *__restrict__ d_live,
                                                       int64_t n_cap, uint32_t *__restrict__ seg) {
    const int64_t live = *d_live;
    for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < n_cap; j += int64_t(gridDim.x) * kBlock)
        seg[j] = j < live ? uint32_t(upper_bound_i64(offs, 0, S + 1, int64_t(pos[j])) - 1) : uint32_t(S);
}
__global__ __launch_bounds__(kBlock) void k_big_unpack(const int64_t *__restrict__ offs,
                                                       const int64_t *__restrict__ cofs, const uint32_t *__restrict__ seg,
                                                       const uint64_t *__restrict__ key,
                                                       const uint32_t *__restrict__ pos, const int64_t *__restrict__ d_live,
                                                       double *__restrict__ out_val, int32_t *__restrict__ out_pos) {
    const int64_t live = *d_live;
    for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < live; j += int64_t(gridDim.x) * kBlock) {
        const uint32_t s = seg[j];
        const int64_t q = offs[s] + (j - cofs[s]);
        out_val[q] = f64_from_key(key[j]);
        out_pos[q] = int32_t(pos[j]);
    }
}
static void radix_big_segments(fz_ctx *c, const int64_t *offs, int64_t S, int64_t n_cap, const uint8_t *flag,
                               const double *src, double *out_val, int32_t *out_pos) {
    const TileMap tm = big_tiles(c, offs, S, n_cap, flag);
    if (tm.cap <= 0) return;
    int64_t *len = c->arena.get<int64_t>(S + 1);
    int64_t *cofs = c->arena.get<int64_t>(S + 1);
    int64_t *d_live = c->arena.get<int64_t>(1);
    k_big_len<<<grid_for(S + 1), kBlock, 0, c->stream>>>(offs, S, flag, len);
    FZ_LAUNCH_CHECK();
    scan_exclusive_i64(c, len, cofs, S + 1, d_live);
    uint64_t *key = c->arena.get<uint64_t>(n_cap);
    uint32_t *pos = c->arena.get<uint32_t>(n_cap);
    k_big_pack<<<unsigned(tm.cap < 4096 ? tm.cap : 4096), kBlock, 0, c->stream>>>(src, offs, cofs, tm, key, pos);
    FZ_LAUNCH_CHECK();
    radix_sort_pairs_swap_live(c, key, pos, n_cap, d_live, 64);
    uint32_t *seg = c->arena.get<uint32_t>(n_cap);
    k_big_segkey<<<grid_for(n_cap, kBlock, 4096), kBlock, 0, c->stream>>>(offs, S, pos, d_live, n_cap, seg);
    FZ_LAUNCH_CHECK();
    RadixPayload pl;
    pl.n = 1;
    pl.in[0] = key;
    pl.size[0] = 8;
    radix_sort_pairs_payload32_live(c, seg, pos, n_cap, d_live, bits_for(uint64_t(S)), pl);
    k_big_unpack<<<grid_for(n_cap, kBlock, 4096), kBlock, 0, c->stream>>>(
        offs, cofs, seg, static_cast<const uint64_t *>(pl.out[0]), pos, d_live, out_val, out_pos);
    FZ_LAUNCH_CHECK();
}

SortedSegs seg_sort_f64(fz_ctx *c, const double *src, const Segs &sg, const int32_t *) {
    const int64_t n = sg.n_cap;
    SortedSegs out;
    out.val = c->arena.get<double>(n);
    out.pos = c->arena.get<int32_t>(n);
    if (n <= 0 || sg.S <= 0) return out;
    if (sg.S == 1 && sg.len_bound() > 16384 && n < kSampleSortMax && sample_sort_on()) {
        // one long segment (RQ3's union, a long series): splitter buckets, one scatter pass
        // and an LDS sort per bucket - five launches (fz_prims.hip sample_sort_f64_seg1; every
        // single-segment caller's segment starts at 0: single_segment, RQ3's union, fz_sort_f64)
        sample_sort_f64_seg1(c, src, sg.offs, n, out.val, out.pos);
        return out;
    }
    if (sg.S == 1 && sg.len_bound() > 16384 && n < (int64_t(1) << 22)) {
        // one long segment (RQ3's detected u non-detected union, a long series): the LSD radix sort
        // (8 passes at HBM rate, stable: ties keep position order, as the merge sort keeps them)
        // instead of the merge sort's tile sort and log2(n / 4096) merge rounds.  It sorts the whole
        // capacity, so only below 4 M entries: the merge sort's work follows the live length (a
        // 100 M-row table's empty RQ3 union), and larger radix sorts would skip constant-digit
        // passes after a host round trip that a recorded graph cannot make.
        uint64_t *k = c->arena.get<uint64_t>(n);
        uint32_t *v = c->arena.get<uint32_t>(n);
        // (live-bounded: the passes cover the segment's end offs[1], not the capacity - RQ3's union
        // fills ~80 % of its capacity at config 2)
        k_f64_seg1_keys<<<grid_for(n, kBlock, 4096), kBlock, 0, c->stream>>>(src, n, sg.offs, k, v);
        FZ_LAUNCH_CHECK();
        radix_sort_pairs_swap_live(c, k, v, n, sg.offs + 1, 64);
        k_f64_from_keys<<<grid_for(n, kBlock, 4096), kBlock, 0, c->stream>>>(k, v, n, sg.offs, out.val, out.pos);
        FZ_LAUNCH_CHECK();
        return out;
    }
    // segments of <= 16384 values: one workgroup each, value bucket sort by length class (each
    // launch skips the other classes' segments; one wave / one thread for the tiny ones when there
    // are very many segments); longer or skewed segments of the 16384 class: the segmented merge
    // sort (fz_segsort.h), which touches only the flagged segments' rows
    const int64_t S = sg.S, lb = sg.len_bound();
    const int64_t *offs = sg.offs;
    // algorithmic bytes per live value (offs[S]): value 8 read; value 8 + position 4 written
    ProbeScope ps(c, "seg_value_sort", 0.0, offs + S, 20.0);
    SegLists L;
    if (S > kManySegs) L = seg_lists(c, sg);
    uint8_t *flag = nullptr;
    if (lb > kLdsSortMax) {
        flag = c->arena.get<uint8_t>(S);
        dev_fill(c, flag, 0, S);
    }
    auto grid = [](int64_t cap, int64_t lim) { return unsigned(cap < 1 ? 1 : (cap < lim ? cap : lim)); };
    const bool lists = L.on;
    const int64_t *dn = L.d_n;
    auto class_list = [&](int k) { return lists ? L.ids[k] : nullptr; };
    auto class_n = [&](int k) { return lists ? dn + k : nullptr; };
    auto class_cap = [&](int k) { return lists ? L.cap[k] : S; };
    if (lists) {
        k_seg_sort_micro<<<grid_for(S, kBlock, 8192), kBlock, 0, c->stream>>>(src, offs, S, out.val, out.pos);
        k_seg_sort_wave<<<grid((L.cap[kClassTiny] + 3) / 4, 8192), kBlock, 0, c->stream>>>(
            src, offs, L.ids[kClassTiny], dn + kClassTiny, out.val, out.pos);
        FZ_LAUNCH_CHECK();
    }
    k_seg_val_bucket<256, 1024><<<grid(class_cap(kClassMid), 16384), 256, 0, c->stream>>>(
        src, offs, S, lists ? kTinySeg : 0, out.val, out.pos, class_list(kClassMid), class_n(kClassMid), flag, false);
    FZ_LAUNCH_CHECK();
    if (lb > 1024) {
        k_seg_val_bucket<512, 2048><<<grid(class_cap(kClassWide), 4096), 512, 0, c->stream>>>(
            src, offs, S, 1024, out.val, out.pos, class_list(kClassWide), class_n(kClassWide), flag, false);
        k_seg_val_bucket<kVb4Block, kLdsSortMax><<<grid(class_cap(kClassWide), kVb4Grid), kVb4Block, 0, c->stream>>>(
            src, offs, S, 2048, out.val, out.pos, class_list(kClassWide), class_n(kClassWide), flag, false);
        FZ_LAUNCH_CHECK();
    }
    if (lb > kLdsSortMax) {
        k_seg_val_bucket<1024, 16384><<<grid(class_cap(kClassBig), 512), 1024, 0, c->stream>>>(
            src, offs, S, kLdsSortMax, out.val, out.pos, class_list(kClassBig), class_n(kClassBig), flag, true);
        FZ_LAUNCH_CHECK();
        if (FZ_BIG_RADIX && lb > kBigRadixMin)
            radix_big_segments(c, offs, S, n, flag, src, out.val, out.pos);
        else
            sort_big_segments(c, offs, S, n, lb, flag, F64Key{src}, F64Sink{out.val, out.pos});
    }
    return out;
}

// Brunner-Munzel and Mann-Whitney U of segment s from its sums: s1 = {sum of x's union ranks, of
// y's, nx, ny, tie term t^3 - t (two exact halves)}, s2 = {sum of x's squared rank deviations, y's}
// (scipy _stats_py.py brunnermunzel; _mannwhitneyu.py, exact null distribution when allowed)
__device__ inline void rank_tests_finish(const double *s1, const double *s2, bool single, const RankTestOut &o,
                                         int64_t s) {
    const double nx = s1[2], ny = s1[3];
    const double rcx = s1[0] / nx, rcy = s1[1] / ny;
    const double Sx = s2[0] / (nx - 1.0), Sy = s2[1] / (ny - 1.0);
    double w = nx * ny * (rcy - rcx);
    w /= (nx + ny) * sqrt(nx * Sx + ny * Sy);
    const double num = (nx * Sx + ny * Sy) * (nx * Sx + ny * Sy);
    const double den = (nx * Sx) * (nx * Sx) / (nx - 1.0) + (ny * Sy) * (ny * Sy) / (ny - 1.0);
    const double df = num / den;
    if (o.bm_stat) o.bm_stat[s] = w;
    if (o.bm_p) o.bm_p[s] = 2.0 * t_sf_once(fabs(w), df);
    if (o.nx) o.nx[s] = nx;
    if (o.ny) o.ny[s] = ny;
    // Mann-Whitney U (x vs y)
    const double R1 = s1[0];
    const double U1 = R1 - nx * (nx + 1.0) / 2.0;
    const double U2 = nx * ny - U1;
    const double nn = nx + ny;
    const double tie = s1[4] + s1[5];
    const double mu = nx * ny / 2.0;
    const double sd = sqrt(nx * ny / 12.0 * ((nn + 1.0) - tie / (nn * (nn - 1.0))));
    if (o.u1) o.u1[s] = U1;
    // exact null distribution (scipy _mannwhitneyu._MWU): counts of U = coefficients of the
    // Gaussian binomial [n1+n2 choose n1]_q, built as prod_k (1 - q^(n2+k)) / (1 - q^k)
    const bool exact = o.exact_scratch && single && !(nx > 8.0 && ny > 8.0) && !(tie > 0.0);
    double *conf = o.exact_scratch;
    int64_t n1 = int64_t(nx < ny ? nx : ny), n2 = int64_t(nx < ny ? ny : nx);
    double total = 1.0;
    if (exact) {
        const int64_t deg = n1 * n2;
        for (int64_t u = 0; u <= deg; ++u) conf[u] = u == 0 ? 1.0 : 0.0;
        for (int64_t k = 1; k <= n1; ++k) {
            const int64_t m = n2 + k;
            for (int64_t u = deg; u >= m; --u) conf[u] -= conf[u - m];
            for (int64_t u = k; u <= deg; ++u) conf[u] += conf[u - k];
        }
        total = 0.0;
        for (int64_t u = 0; u <= deg; ++u) total += conf[u];
    }
    auto pv = [&](double U, double f) {
        double p;
        if (exact) {  // _MWU.sf(U): 1 - cdf(U) + pmf(U) when U < n1*n2 - U, else cdf(n1*n2 - U)
            const int64_t k = int64_t(U);
            const int64_t kc = n1 * n2 - k;
            const int64_t lim = k < kc ? k : kc;
            double cdf = 0.0;
            for (int64_t u = 0; u <= lim; ++u) cdf += conf[u] / total;
            p = k < kc ? 1.0 - cdf + conf[k] / total : cdf;
        } else {
            const double z = (U - mu - 0.5) / sd;
            p = stats::norm_sf(z);
        }
        p *= f;
        return p < 0.0 ? 0.0 : (p > 1.0 ? 1.0 : p);
    };
    if (o.mwu_p_two) o.mwu_p_two[s] = pv(U1 > U2 ? U1 : U2, 2.0);
    if (o.mwu_p_greater) o.mwu_p_greater[s] = pv(U1, 1.0);
    if (o.ties) o.ties[s] = tie;
}

// ------------------------------------------------------------------------------ tie ranks
TieRanks seg_tie_ranks(fz_ctx *c, const ChunkedSegs &cs, const int32_t *segid, const double *sorted) {
    const Segs &sg = cs.sg;
    const int64_t n = sg.n_cap;
    const int64_t *offs = sg.offs;
    const int64_t S = sg.S;
    TieRanks tr;
    tr.rank = c->arena.get<double>(n);
    tr.ngroups = c->arena.get<double>(S);
    int64_t *flag = c->arena.get<int64_t>(n);
    int64_t *gid = c->arena.get<int64_t>(n);
    int64_t *gstart = c->arena.get<int64_t>(n + 1);
    // (every pass over the live elements offs[S] only: the arrays past them are never read)
    const int64_t *d_live = offs + S;
    map_n(c, n, d_live, [=] __device__(int64_t i) {
        const int64_t s = segid[i];
        flag[i] = (i == offs[s] || sorted[i] != sorted[i - 1]) ? 1 : 0;
    });
    int64_t *d_g = c->arena.get<int64_t>(1);
    scan_exclusive_i64_dn(c, flag, gid, n, d_live, d_g);
    map_n(c, n, d_live, [=] __device__(int64_t i) {
        if (flag[i]) gstart[gid[i]] = i;
        if (i == offs[S] - 1) gstart[*d_g] = offs[S];  // the sentinel, by the last live element
    });
    double *rank = tr.rank;
    map_n(c, n, d_live, [=] __device__(int64_t i) {
        const int64_t g = gid[i] + (flag[i] ? 0 : -1);  // exclusive scan: group index of element i
        const int64_t s = segid[i];
        const int64_t a = gstart[g], b = gstart[g + 1];
        rank[i] = double(a + b + 1) / 2.0 - double(offs[s]);
    });
    seg_reduce<1>(c, cs, [=] __device__(int64_t i, int32_t, double *x) { x[0] = double(flag[i]); }, tr.ngroups);
    tr.flag = flag;
    tr.gid = gid;
    tr.gstart = gstart;
    return tr;
}

// ------------------------------------------------------------ two-sample rank tests per segment
// Each segment holds the x sample (grp 0) and the y sample (grp 1) in any order.
//   Brunner-Munzel (scipy _stats_py.py brunnermunzel, t distribution, two-sided)
//   Mann-Whitney U asymptotic (scipy _mannwhitneyu.py: tie term, continuity) two-sided + greater
void seg_rank_tests(fz_ctx *c, const double *vals, const uint8_t *grp, const Segs &sg, const int32_t *segid,
                    const RankTestOut &o) {
    ChunkedSegs cs = chunked(c, sg);
    SortedSegs ss = seg_sort_f64(c, vals, sg, segid);
    seg_rank_tests_sorted(c, ss, grp, cs, segid, o);
}

void seg_rank_tests_sorted(fz_ctx *c, const SortedSegs &ss, const uint8_t *grp, const ChunkedSegs &cs,
                           const int32_t *segid, const RankTestOut &o) {
    const Segs &sg = cs.sg;
    const int64_t n = sg.n_cap, S = sg.S;
    const int64_t *offs = sg.offs;
    TieRanks tr = seg_tie_ranks(c, cs, segid, ss.val);
    // cx[i] = number of x elements before sorted position i (cx[n] = total)
    int64_t *isx = c->arena.get<int64_t>(n);
    int64_t *cx = c->arena.get<int64_t>(n + 1);
    const int32_t *pos = ss.pos;
    map_n(c, n, offs + S, [=] __device__(int64_t i) { isx[i] = grp[pos[i]] == 0 ? 1 : 0; });
    scan_exclusive_i64_dn(c, isx, cx, n, offs + S, cx + n);  // (cx[live] = the total too)
    // within-sample average rank of every element
    double *rw = c->arena.get<double>(n);
    const int64_t *flag = tr.flag, *gid = tr.gid, *gstart = tr.gstart;
    map_n(c, n, offs + S, [=] __device__(int64_t i) {
        const int64_t s = segid[i], s0 = offs[s];
        const int64_t g = gid[i] - 1 + flag[i];
        const int64_t a = gstart[g], b = gstart[g + 1];
        const int64_t xb = cx[a] - cx[s0], xg = cx[b] - cx[a];
        const int64_t yb = (a - s0) - xb, yg = (b - a) - xg;
        rw[i] = isx[i] ? double(xb) + double(xg + 1) / 2.0 : double(yb) + double(yg + 1) / 2.0;
    });
    const double *rc = tr.rank;
    double *s1 = c->arena.get<double>(S * 6);
    seg_reduce<6>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const bool xs = isx[i];
        x[0] = xs ? rc[i] : 0.0;
        x[1] = xs ? 0.0 : rc[i];
        x[2] = xs ? 1.0 : 0.0;
        x[3] = xs ? 0.0 : 1.0;
        // tie term t^3 - t (int64-exact), split into two exactly representable halves
        int64_t tt = 0;
        if (flag[i]) {
            const int64_t g = gid[i];
            const int64_t t = gstart[g + 1] - gstart[g];
            tt = t * t * t - t;
        }
        x[4] = double(tt & ~int64_t((1 << 26) - 1));
        x[5] = double(tt & int64_t((1 << 26) - 1));
    }, s1, 25.0);  // isx 1 + rank 8 + flag 8 (+ group bounds of tied elements)
    double *s2 = c->arena.get<double>(S * 2);
    seg_reduce<2>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const double nx = s1[6 * s + 2], ny = s1[6 * s + 3];
        const bool xs = isx[i];
        const double cm = xs ? s1[6 * s] / nx : s1[6 * s + 1] / ny;  // np.mean(rankcx) / (rankcy)
        const double wm = xs ? (nx + 1.0) / 2.0 : (ny + 1.0) / 2.0;  // np.mean(rankx) (exact)
        const double d = ((rc[i] - rw[i]) - cm) + wm;
        x[0] = xs ? d * d : 0.0;
        x[1] = xs ? 0.0 : d * d;
    }, s2, 17.0);  // isx 1 + both ranks 16
    per_seg(c, S, [=] __device__(int64_t s) { rank_tests_finish(s1 + 6 * s, s2 + 2 * s, S == 1, o, s); });
}

// (Used while one half holds at most kBmHalvesMax values - a few per thread: at config 3's 4,000-value
// halves the per-thread walks are long dependent chains and the device-wide rank passes win.)
// Brunner-Munzel p of M sessions whose two samples are already sorted: x = sv[offs2[2i],
// offs2[2i + 1]), y = sv[offs2[2i + 1], offs2[2i + 2]), both ascending.  One workgroup per session,
// each thread walking a contiguous run of one half in order (a merge): a value's average rank in
// the union is its count below in both halves plus the middle of its tie group across both, its
// within-sample rank the same in its own half - the pointers into the other half only move
// forward, a new tie group finds its end by binary search.  Then the two sums scipy's
// brunnermunzel forms (t distribution, two-sided): no union sort, no device-wide rank passes.
// p = NaN unless both samples hold >= min_n values.
// visit(rc, rw) for this thread's run of a (na values) against the other half b (nb values)
template <typename F>
__device__ inline void bm_walk_run(const double *a, int64_t na, const double *b, int64_t nb, int64_t k0, int64_t k1,
                                   F visit) {
    if (k0 >= k1) return;
    double v = a[k0];
    int64_t la = lower_bound_d(a, 0, k0 + 1, v), ua = upper_bound_d(a, k0, na, v);
    int64_t lb = lower_bound_d(b, 0, nb, v), ub = upper_bound_d(b, lb, nb, v);
    for (int64_t k = k0; k < k1; ++k) {
        if (k > k0 && a[k] != v) {  // a new tie group starts at k
            v = a[k];
            la = k;
            ua = upper_bound_d(a, k, na, v);
            while (lb < nb && b[lb] < v) ++lb;
            if (ub < lb) ub = lb;
            while (ub < nb && b[ub] <= v) ++ub;
        }
        const double rc = double(la + lb) + double((ua - la) + (ub - lb) + 1) / 2.0;
        const double rw = double(la) + double(ua - la + 1) / 2.0;
        visit(rc, rw);
    }
}
// this thread's share of a (one contiguous run per thread of the workgroup)
template <typename F>
__device__ inline void bm_walk(const double *a, int64_t na, const double *b, int64_t nb, F visit) {
    const int64_t per = (na + kBlock - 1) / kBlock;
    const int64_t k0 = int64_t(threadIdx.x) * per;
    bm_walk_run(a, na, b, nb, k0, k0 + per < na ? k0 + per : na, visit);
}
__global__ __launch_bounds__(kBlock) void k_bm_sorted_halves(const double *__restrict__ sv,
                                                             const int64_t *__restrict__ offs2, int64_t M,
                                                             int64_t min_n, double *__restrict__ pbm) {
    __shared__ double s_tmp[4];
    for (int64_t i = blockIdx.x; i < M; i += gridDim.x) {
        const int64_t x0 = offs2[2 * i], x1 = offs2[2 * i + 1], y1 = offs2[2 * i + 2];
        const int64_t nx = x1 - x0, ny = y1 - x1;
        if (nx < min_n || ny < min_n) {
            if (threadIdx.x == 0) pbm[i] = NAN;
            continue;
        }
        const double *x = sv + x0, *y = sv + x1;
        double ax = 0.0, ay = 0.0;
        bm_walk(x, nx, y, ny, [&](double rc, double) { ax += rc; });
        bm_walk(y, ny, x, nx, [&](double rc, double) { ay += rc; });
        const double Nx = double(nx), Ny = double(ny);
        const double rcx = block_sum(ax, s_tmp) / Nx, rcy = block_sum(ay, s_tmp) / Ny;
        const double wmx = (Nx + 1.0) / 2.0, wmy = (Ny + 1.0) / 2.0;  // mean within-sample rank
        double bx = 0.0, by = 0.0;
        bm_walk(x, nx, y, ny, [&](double rc, double rw) {
            const double d = ((rc - rw) - rcx) + wmx;
            bx += d * d;
        });
        bm_walk(y, ny, x, nx, [&](double rc, double rw) {
            const double d = ((rc - rw) - rcy) + wmy;
            by += d * d;
        });
        const double Sx = block_sum(bx, s_tmp) / (Nx - 1.0), Sy = block_sum(by, s_tmp) / (Ny - 1.0);
        if (threadIdx.x == 0) {
            double w = Nx * Ny * (rcy - rcx);
            w /= (Nx + Ny) * sqrt(Nx * Sx + Ny * Sy);
            const double num = (Nx * Sx + Ny * Sy) * (Nx * Sx + Ny * Sy);
            const double den = (Nx * Sx) * (Nx * Sx) / (Nx - 1.0) + (Ny * Sy) * (Ny * Sy) / (Ny - 1.0);
            pbm[i] = 2.0 * t_sf_once(fabs(w), num / den);
        }
    }
}

void bm_sorted_halves(fz_ctx *c, const double *sorted, const int64_t *offs2, int64_t M, int64_t min_n, double *pbm) {
    if (M <= 0) return;
    k_bm_sorted_halves<<<unsigned(M < 16384 ? M : 16384), kBlock, 0, c->stream>>>(sorted, offs2, M, min_n, pbm);
    FZ_LAUNCH_CHECK();
}

// Sum over the NW waves of a workgroup (s_tmp: NW slots).
template <int NW>
__device__ inline double block_sum_nw(double x, double *s_tmp) {
    x = wave_sum(x);
    if (lane_id() == 0) s_tmp[wave_id()] = x;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += s_tmp[w];
    __syncthreads();
    return t;
}

// The Brunner-Munzel p of one session from its union ranks rc and within-sample ranks rw:
// d = rc - rw per value, sums as scipy's brunnermunzel forms them (t distribution, two-sided).
__device__ inline double bm_pvalue(double Nx, double Ny, double rcx, double rcy, double Sx, double Sy) {
    double w = Nx * Ny * (rcy - rcx);
    w /= (Nx + Ny) * sqrt(Nx * Sx + Ny * Sy);
    const double num = (Nx * Sx + Ny * Sy) * (Nx * Sx + Ny * Sy);
    const double den = (Nx * Sx) * (Nx * Sx) / (Nx - 1.0) + (Ny * Sy) * (Ny * Sy) / (Ny - 1.0);
    return 2.0 * t_sf_once(fabs(w), num / den);
}

// Brunner-Munzel of sessions whose sorted halves hold up to MAXN values together (config 3: ~10^4
// values per session, too long for the per-thread merge walks of k_bm_sorted_halves): one
// workgroup per session stages both halves in LDS (one coalesced read), then every value finds its
// tie range in its own half and in the other by four binary searches in LDS - independent per
// value, so a thread's values overlap their searches instead of walking a dependent chain - giving
// its union rank rc and within-sample rank rw at once; the two sums of scipy's brunnermunzel follow
// from rc - rw kept in registers.  Sessions come from a size-class list (or all M, list null).
template <int BS, int MAXN>
__global__ __launch_bounds__(BS) void k_bm_halves_lds(const double *__restrict__ sv, const int64_t *__restrict__ offs2,
                                                     int64_t M, const int32_t *__restrict__ list,
                                                     const int64_t *__restrict__ d_ln, int64_t min_n,
                                                     double *__restrict__ pbm) {
    constexpr int NW = BS / kWave;
    constexpr int IPT = MAXN / BS;
    static_assert(MAXN % BS == 0, "shape");
    __shared__ double s_v[MAXN];
    __shared__ double s_tmp[NW];
    const int tid = threadIdx.x;
    const int64_t ns = list ? *d_ln : M;
    for (int64_t it = blockIdx.x; it < ns; it += gridDim.x) {
        const int64_t i = list ? list[it] : it;
        const int64_t x0 = offs2[2 * i], x1 = offs2[2 * i + 1], y1 = offs2[2 * i + 2];
        const int nx = int(x1 - x0), ny = int(y1 - x1), n = nx + ny;
        if (nx < min_n || ny < min_n || n > MAXN) {
            if (tid == 0) pbm[i] = NAN;
            continue;
        }
        for (int j = tid; j < n; j += BS) s_v[j] = sv[x0 + j];
        __syncthreads();
        const double *X = s_v, *Y = s_v + nx;
        double d[IPT];
        double ax = 0.0, ay = 0.0;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int j = tid + m * BS;
            d[m] = 0.0;
            if (j >= n) continue;
            const bool inx = j < nx;
            const double *own = inx ? X : Y, *oth = inx ? Y : X;
            const int no = inx ? nx : ny, nt = inx ? ny : nx, k = inx ? j : j - nx;
            const double v = own[k];
            // (each search's predicate holds on a prefix of its range - NaNs sort last and compare
            // false - so one probe at the range's near end settles the untied case: a value without
            // ties costs the one search in the other half, not four)
            int la = 0, hi = k;  // first index of v in own (own[k] == v)
            if (k == 0 || own[k - 1] < v) la = k;
            while (la < hi) {
                const int md = (la + hi) >> 1;
                if (own[md] < v) la = md + 1;
                else hi = md;
            }
            int ua = k + 1;  // one past the last index of v in own
            hi = (ua < no && own[ua] <= v) ? no : ua;
            while (ua < hi) {
                const int md = (ua + hi) >> 1;
                if (own[md] <= v) ua = md + 1;
                else hi = md;
            }
            int lb = 0;
            hi = nt;
            while (lb < hi) {
                const int md = (lb + hi) >> 1;
                if (oth[md] < v) lb = md + 1;
                else hi = md;
            }
            int ub = lb;
            hi = (ub < nt && oth[ub] <= v) ? nt : ub;
            while (ub < hi) {
                const int md = (ub + hi) >> 1;
                if (oth[md] <= v) ub = md + 1;
                else hi = md;
            }
            const double rc = double(la + lb) + double((ua - la) + (ub - lb) + 1) / 2.0;
            const double rw = double(la) + double(ua - la + 1) / 2.0;
            d[m] = rc - rw;
            if (inx) ax += rc;
            else ay += rc;
        }
        const double Nx = double(nx), Ny = double(ny);
        const double rcx = block_sum_nw<NW>(ax, s_tmp) / Nx, rcy = block_sum_nw<NW>(ay, s_tmp) / Ny;
        const double wmx = (Nx + 1.0) / 2.0, wmy = (Ny + 1.0) / 2.0;  // mean within-sample rank
        double bx = 0.0, by = 0.0;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int j = tid + m * BS;
            if (j >= n) continue;
            if (j < nx) {
                const double e = (d[m] - rcx) + wmx;
                bx += e * e;
            } else {
                const double e = (d[m] - rcy) + wmy;
                by += e * e;
            }
        }
        const double Sx = block_sum_nw<NW>(bx, s_tmp) / (Nx - 1.0), Sy = block_sum_nw<NW>(by, s_tmp) / (Ny - 1.0);
        if (tid == 0) pbm[i] = bm_pvalue(Nx, Ny, rcx, rcy, Sx, Sy);
        // (block_sum_nw's trailing barrier: every read of s_v is done before the next session's loads)
    }
}

// The same for sessions of at most 64 values (a size-class list): one wave each, a value per lane;
// its tie ranges are counted against the other lanes' values (64 shuffles, no memory traffic).
__global__ __launch_bounds__(kBlock) void k_bm_wave(const double *__restrict__ sv, const int64_t *__restrict__ offs2,
                                                    const int32_t *__restrict__ list, const int64_t *__restrict__ d_ln,
                                                    int64_t min_n, double *__restrict__ pbm) {
    const int64_t ns = *d_ln;
    const int lane = lane_id();
    for (int64_t it = int64_t(blockIdx.x) * 4 + wave_id(); it < ns; it += int64_t(gridDim.x) * 4) {
        const int64_t i = list[it];
        const int64_t x0 = offs2[2 * i], x1 = offs2[2 * i + 1], y1 = offs2[2 * i + 2];
        const int nx = int(x1 - x0), ny = int(y1 - x1), n = nx + ny;
        if (nx < min_n || ny < min_n || n > kWave) {
            if (lane == 0) pbm[i] = NAN;
            continue;
        }
        const bool valid = lane < n, inx = lane < nx;
        const double v = valid ? sv[x0 + lane] : 0.0;
        int la = 0, ua = 0, lb = 0, ub = 0;
        for (int t = 0; t < n; ++t) {
            const double u = __shfl(v, t, kWave);
            const bool same = (t < nx) == inx;
            const int lt = u < v, le = u <= v;
            la += same ? lt : 0;
            ua += same ? le : 0;
            lb += same ? 0 : lt;
            ub += same ? 0 : le;
        }
        const double rc = double(la + lb) + double((ua - la) + (ub - lb) + 1) / 2.0;
        const double rw = double(la) + double(ua - la + 1) / 2.0;
        const double d = rc - rw;
        const double Nx = double(nx), Ny = double(ny);
        const double rcx = wave_sum(valid && inx ? rc : 0.0) / Nx, rcy = wave_sum(valid && !inx ? rc : 0.0) / Ny;
        const double e = inx ? (d - rcx) + (Nx + 1.0) / 2.0 : (d - rcy) + (Ny + 1.0) / 2.0;
        const double Sx = wave_sum(valid && inx ? e * e : 0.0) / (Nx - 1.0);
        const double Sy = wave_sum(valid && !inx ? e * e : 0.0) / (Ny - 1.0);
        if (lane == 0) pbm[i] = bm_pvalue(Nx, Ny, rcx, rcy, Sx, Sy);
    }
}

// Brunner-Munzel p of M sessions from their sorted halves (offs2 as bm_sorted_halves; soffs[M + 1]:
// session offsets, soffs[k] = offs2[2k]; n_cap: values in all sessions; every session holds at
// most kBmLdsMax values).  Few sessions (configs 2 / 3): one workgroup each over all of them.  Very
// many (config 5's Zipf tail: one session per index of the longest project, ~10^7, nearly all
// holding a handful of values): size-class lists - sessions of <= 8 values are never tested (both
// halves need min_n >= 5), <= 64 one wave each, <= 4096 a 256-thread workgroup, longer 1024 threads.
// (FZ_BM_FEW: up to this many sessions one 1024-thread workgroup each; more take the size classes -
// a 1024-thread workgroup stages 96 KiB of LDS, one per CU: config 3L's eighth, 10,000 sessions of
// ~1,000 values, queued 40 rounds deep behind it)
#ifndef FZ_BM_FEW
#define FZ_BM_FEW 2048
#endif
void bm_halves(fz_ctx *c, const double *sorted, const int64_t *offs2, const int64_t *soffs, int64_t M, int64_t n_cap,
               int64_t min_n, double *pbm) {
    if (M <= 0) return;
    if (M <= FZ_BM_FEW) {
        k_bm_halves_lds<1024, kBmLdsMax><<<unsigned(M < 4096 ? M : 4096), 1024, 0, c->stream>>>(
            sorted, offs2, M, nullptr, nullptr, min_n, pbm);
        FZ_LAUNCH_CHECK();
        return;
    }
    static_assert(kMicroSeg < 10, "sessions of <= kMicroSeg values have a half below min_n = 5");
    map_n(c, M, nullptr, [=] __device__(int64_t i) { pbm[i] = NAN; });
    const SegLists L = seg_lists(c, Segs{M, soffs, n_cap});
    auto grid = [](int64_t cap, int64_t lim) { return unsigned(cap < 1 ? 1 : (cap < lim ? cap : lim)); };
    k_bm_wave<<<grid((L.cap[kClassTiny] + 3) / 4, 8192), kBlock, 0, c->stream>>>(
        sorted, offs2, L.ids[kClassTiny], L.d_n + kClassTiny, min_n, pbm);
    k_bm_halves_lds<256, 4096><<<grid(L.cap[kClassMid], 8192), 256, 0, c->stream>>>(
        sorted, offs2, M, L.ids[kClassMid], L.d_n + kClassMid, min_n, pbm);
    k_bm_halves_lds<256, 4096><<<grid(L.cap[kClassWide], 4096), 256, 0, c->stream>>>(
        sorted, offs2, M, L.ids[kClassWide], L.d_n + kClassWide, min_n, pbm);
    k_bm_halves_lds<1024, kBmLdsMax><<<grid(L.cap[kClassBig], 2048), 1024, 0, c->stream>>>(
        sorted, offs2, M, L.ids[kClassBig], L.d_n + kClassBig, min_n, pbm);
    FZ_LAUNCH_CHECK();
}

// --------------------------------------------------------------------- Spearman vs index
void seg_spearman_index(fz_ctx *c, const ChunkedSegs &cs, const SortedSegs &ss, const TieRanks &tr, double *rho,
                        double *pval) {
    const int64_t *offs = cs.sg.offs;
    const int64_t S = cs.sg.S;
    const int32_t *pos = ss.pos;
    const double *rank = tr.rank;
    double *sums = c->arena.get<double>(S * 3);
    // deviations from the common mean rank (n+1)/2 are half-integers: the products are exact
    seg_reduce<3>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const int64_t b = offs[s];
        const double m = double(offs[s + 1] - b + 1) / 2.0;
        const double rx = double(pos[i] - b + 1) - m;
        const double ry = rank[i] - m;
        x[0] = rx * ry;
        x[1] = rx * rx;
        x[2] = ry * ry;
    }, sums, 12.0);  // position 4 + rank 8
    const double *ng = tr.ngroups;
    per_seg(c, S, [=] __device__(int64_t s) {
        const int64_t n = offs[s + 1] - offs[s];
        double r = NAN, p = NAN;
        if (n >= 2 && ng[s] > 1.0) {
            // np.corrcoef: c01 / std0 / std1 with c = dot(dev, dev.T) * (1 / (n - 1)) (np.cov
            // multiplies by the reciprocal)
            const double f = 1.0 / double(n - 1);
            const double cxy = sums[3 * s] * f, cxx = sums[3 * s + 1] * f, cyy = sums[3 * s + 2] * f;
            r = cxy / sqrt(cxx) / sqrt(cyy);
            if (r > 1.0) r = 1.0;
            if (r < -1.0) r = -1.0;
            const double dof = double(n - 2);
            double q = dof / ((r + 1.0) * (1.0 - r));
            if (q < 0.0) q = 0.0;  // numpy clip(0); NaN stays NaN
            const double t = r * sqrt(q);
            p = 2.0 * t_sf_once(fabs(t), dof);
        }
        rho[s] = r;
        if (pval) pval[s] = p;
    });
}

// scipy.stats.spearmanr(range(n), x) per segment from the sorted segments alone, one workgroup per
// segment (segments of at most kSpearmanSmall values): each thread walks a run of the sorted values,
// a tie group's bounds come from one binary search when it starts, and the rank products are summed
// directly - the same exact half-integer sums as seg_spearman_index, without the device-wide tie
// rank passes.
#ifndef FZ_SERIES_DEFER
#define FZ_SERIES_DEFER 1
#endif
constexpr bool kSeriesDefer = FZ_SERIES_DEFER;
constexpr int64_t kSpearmanSmall = 4096;  // <= 16 values per thread: longer runs are latency chains

// Double-double sums of NV per-thread partials over the workgroup (NW waves), the rounded results
// in every thread.
template <int NV, int NW = 4>
__device__ inline void block_dd_sums(const DD (&acc)[NV], double (&s_hi)[NW][NV], double (&s_lo)[NW][NV],
                                     double (&out)[NV]) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const DD r = wave_dd_sum(acc[v]);
        if (lane_id() == 0) {
            s_hi[wave_id()][v] = r.hi;
            s_lo[wave_id()][v] = r.lo;
        }
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        DD t{s_hi[0][v], s_lo[0][v]};
        for (int w = 1; w < NW; ++w) t = dd_add(t, DD{s_hi[w][v], s_lo[w][v]});
        out[v] = t.hi + t.lo;
    }
    __syncthreads();
}

#ifdef FZ_SERIES_TIMING
// experiment builds only: wall-clock (100 MHz) phase stamps of the last k_series_small launch
__device__ unsigned long long g_series_t[8];
#define SERIES_STAMP(ph)                                        \
    do {                                                        \
        __syncthreads();                                        \
        if (threadIdx.x == 0) g_series_t[ph] = wall_clock64(); \
    } while (0)
extern "C" int fz_debug_series_timing(unsigned long long *out) {
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_series_t), sizeof(g_series_t));
    return 0;
}
#else
#define SERIES_STAMP(ph) \
    do {                 \
    } while (0)
#endif
// (experiment builds: stamps 4-7 inside the one-workgroup Shapiro-Wilk pass of a single-workgroup
// launch - after the normal scores' sum, the first and second sums, thread 0's p-value)
#ifdef FZ_SERIES_TIMING
#define SW_STAMP(ph)                                                                    \
    do {                                                                                \
        __syncthreads();                                                                \
        if (gridDim.x == 1 && threadIdx.x == 0) g_series_t[4 + (ph)] = wall_clock64(); \
    } while (0)
#else
#define SW_STAMP(ph) \
    do {             \
    } while (0)
#endif
// scipy.stats.shapiro (swilk.c) of one sorted segment v[b, b + n) (src: the same values in input
// order, for y -= x[N // 2]) by the workgroup, each thread over its run [k0, k1) of <= kSmallPer
// values: the passes of seg_shapiro (sum of m_i^2, then sx / sa, then ssa / ssx / sax), every sum
// double-double as there; a thread's coefficients stay in registers between the last two passes.
// s_m (LDS, kSpearmanSmall / 2 doubles): the normal scores m_k (k <= n / 2) of the first pass,
// reused by the coefficients of the second - one ppnd per score instead of one per score and pass
template <int BS = kBlock>
__device__ inline void shapiro_block(const double *__restrict__ v, const double *__restrict__ src, int64_t b,
                                     int64_t n, int64_t k0, int64_t k1, double (&s_hi)[BS / kWave][3],
                                     double (&s_lo)[BS / kWave][3], double *s_m, double *w_out, double *p_out) {
    constexpr int NW = BS / kWave, PER = int(kSpearmanSmall / BS);
    DD a0[1] = {{0.0, 0.0}};
    if (n >= 3)
        for (int64_t k = 1 + threadIdx.x; k <= n / 2; k += BS) {
            const double m = stats::sw_m(k, n);
            s_m[k - 1] = m;
            a0[0] = dd_add_d(a0[0], m * m);
        }
    double summ2[1];
    block_dd_sums<1, NW>(a0, reinterpret_cast<double(&)[NW][1]>(s_hi), reinterpret_cast<double(&)[NW][1]>(s_lo), summ2);
    SW_STAMP(0);
    if (n < 3) {
        if (threadIdx.x == 0) {
            *w_out = NAN;
            *p_out = NAN;
        }
        return;
    }
    const stats::SwCoef cf = stats::sw_coef(n, 2.0 * summ2[0]);
    const double x0 = src[b + n / 2];
    const double range = (v[b + n - 1] - x0) - (v[b] - x0);
    // value j's scaled deviation and signed coefficient (stats::sw_coef_at with the pass-A score of
    // the mirrored index), computed again in the last pass instead of held: two PER-double arrays
    // per thread took the kernel to 235 VGPRs (two workgroups per CU)
    auto yc = [&](int64_t j, double &y, double &co) {
        y = (v[j] - x0) / range;
        const int64_t i = j - b + 1, jm = n + 1 - i, k = i < jm ? i : jm;
        const double a = i == jm ? 0.0 : stats::sw_a_m(cf, k, s_m[k - 1]);
        co = i == jm ? 0.0 : (i > jm ? a : -a);
    };
    DD a1[2] = {{0.0, 0.0}, {0.0, 0.0}};
#pragma unroll 4
    for (int u = 0; u < PER; ++u) {
        const int64_t j = k0 + u;
        if (j < k1) {
            double y, co;
            yc(j, y, co);
            a1[0] = dd_add_d(a1[0], y);
            a1[1] = dd_add_d(a1[1], co);
        }
    }
    double s1[2];
    block_dd_sums<2, NW>(a1, reinterpret_cast<double(&)[NW][2]>(s_hi), reinterpret_cast<double(&)[NW][2]>(s_lo), s1);
    SW_STAMP(1);
    const double sx = s1[0] / double(n), sa = s1[1] / double(n);
    DD a2[3] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
#pragma unroll 4
    for (int u = 0; u < PER; ++u) {
        const int64_t j = k0 + u;
        if (j < k1) {
            double y, co;
            yc(j, y, co);
            const double asa = co - sa, xsx = y - sx;
            a2[0] = dd_add_d(a2[0], asa * asa);
            a2[1] = dd_add_d(a2[1], xsx * xsx);
            a2[2] = dd_add_d(a2[2], asa * xsx);
        }
    }
    double s2[3];
    block_dd_sums<3, NW>(a2, s_hi, s_lo, s2);
    SW_STAMP(2);
    if (threadIdx.x == 0) {
        if (range < stats::kSwSmall) {  // zero range: scipy returns (1.0, 1.0)
            *w_out = 1.0;
            *p_out = 1.0;
            return;
        }
        const double ssa = s2[0], ssx = s2[1], sax = s2[2];
        const double ssassx = sqrt(ssa * ssx);
        const double w1 = (ssassx - sax) * (ssassx + sax) / (ssa * ssx);
        const double ww = 1.0 - w1;
        *w_out = ww;
        *p_out = sw_pvalue_once(n, ww, w1);
#ifdef FZ_SERIES_TIMING
        if (gridDim.x == 1) g_series_t[7] = wall_clock64();
#endif
    }
}

// (sw_w non-null: Shapiro-Wilk of every segment too, from the same workgroup's pass; rho null:
// Shapiro-Wilk only)
__global__ __launch_bounds__(kBlock) void k_spearman_index_small(const double *__restrict__ sv,
                                                                 const int32_t *__restrict__ pos,
                                                                 const int64_t *__restrict__ offs, int64_t S,
                                                                 double *__restrict__ rho, double *__restrict__ pval,
                                                                 const double *__restrict__ src = nullptr,
                                                                 double *__restrict__ sw_w = nullptr,
                                                                 double *__restrict__ sw_p = nullptr) {
    __shared__ double s_tmp[4];
    __shared__ double s_hi[4][3], s_lo[4][3];
    __shared__ double s_m[kSpearmanSmall / 2];
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t b = offs[s], n = offs[s + 1] - b;
        const int64_t per = (n + kBlock - 1) / kBlock;
        const int64_t k0 = b + int64_t(threadIdx.x) * per, k1 = k0 + per < b + n ? k0 + per : b + n;
        if (!kSeriesDefer || !sw_w || !rho) {
            if (sw_w) shapiro_block(sv, src, b, n, k0, k1, s_hi, s_lo, s_m, sw_w + s, sw_p + s);
            if (rho) spearman_block<kBlock>(sv, pos, b, n, s_tmp, rho + s, pval ? pval + s : nullptr);
            continue;
        }
        // both: the Spearman sums first, then Shapiro-Wilk, the two p-values on different waves
        // (thread 0: Shapiro-Wilk's, the last thread: Spearman's)
        const SpearmanT st = spearman_block<kBlock>(sv, pos, b, n, s_tmp, rho + s, pval ? pval + s : nullptr, true);
        shapiro_block(sv, src, b, n, k0, k1, s_hi, s_lo, s_m, sw_w + s, sw_p + s);
        if (pval && threadIdx.x == kBlock - 1) pval[s] = spearman_p(st);
    }
}

// spearmanr(range(n), x) sums of long sorted segments, chunk by chunk (the chunked-reduction map,
// kChunk values per workgroup): the chunk's values and positions are staged in LDS (coalesced),
// each thread takes kRedItems consecutive ones, and a value's tie group [gs, ge) comes from the
// tie-start flags - inside the thread, else from a block max-scan of the preceding threads' last
// start / a reverse min-scan of the following threads' first start, else (a group crossing the
// chunk's edge) from one binary search at each edge.  Every value's rank is then known in its
// chunk alone: the double-double partials (sum rx*ry, rx^2, ry^2, tie groups) of each chunk go to
// the segmented fold.  One launch instead of the device-wide tie-rank passes (flag, scan, group
// starts, ranks, group count) and the reduction over their arrays.
constexpr int kSpNV = 4;
__global__ __launch_bounds__(kBlock) void k_spearman_chunks(ChunkMap cm, const int64_t *__restrict__ offs, int64_t cps,
                                                            int64_t nk_host, const double *__restrict__ sv,
                                                            const int32_t *__restrict__ pos, double *__restrict__ part) {
    constexpr int IPT = kRedItems;
    __shared__ double s_v[kChunk];
    __shared__ int32_t s_p[kChunk];
    __shared__ int64_t s_w[2][4];
    __shared__ int64_t s_edge[2];
    __shared__ double s_hi[4][kSpNV], s_lo[4][kSpNV];
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
    const int64_t nk = cm.d_n ? *cm.d_n : nk_host;
    for (int64_t k = blockIdx.x; k < nk; k += gridDim.x) {
        int32_t seg;
        int64_t b, e;
        if (cm.d_n) {
            seg = cm.seg[k];
            b = cm.begin[k];
            e = cm.end[k];
        } else {
            seg = int32_t(k / cps);
            b = offs[seg] + (k % cps) * kChunk;
            e = b + kChunk < offs[seg + 1] ? b + kChunk : offs[seg + 1];
        }
        const int64_t sb = offs[seg], se = offs[seg + 1];
        const int len = e > b ? int(e - b) : 0;
        if (len == 0) {  // an empty chunk: zero partials, no barriers
            if (tid < kSpNV) {
                part[(k * kSpNV + tid) * 2] = 0.0;
                part[(k * kSpNV + tid) * 2 + 1] = 0.0;
            }
            continue;
        }
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int j = tid + m * kBlock;
            if (j < len) {
                s_v[j] = sv[b + j];
                s_p[j] = pos[b + j];
            }
        }
        // the tie groups crossing the chunk's edges (two lanes of different waves search at once)
        if (tid == 0) {
            int64_t gs = b;
            if (len > 0 && b > sb && sv[b - 1] == sv[b]) gs = lower_bound_d(sv, sb, b, sv[b]);
            s_edge[0] = gs;
        } else if (tid == kWave) {
            int64_t ge = e;
            if (len > 0 && e < se && sv[e] == sv[e - 1]) ge = upper_bound_d(sv, e, se, sv[e - 1]);
            s_edge[1] = ge;
        }
        __syncthreads();
        const int64_t head = s_edge[0], tail = s_edge[1];
        // this thread's run q0 .. q0 + IPT - 1: tie-start flags, first / last start in the run
        const int q0 = tid * IPT;
        bool f[IPT];
        int64_t first = INT64_MAX, last = -1;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int q = q0 + m;
            f[m] = q < len && (q == 0 ? head == b : s_v[q] != s_v[q - 1]);
            if (f[m]) {
                first = first < b + q ? first : b + q;
                last = b + q;
            }
        }
        // exclusive max-scan of `last` over the preceding threads, reverse min-scan of `first` over
        // the following ones (wave shuffles, then the four waves' totals)
        int64_t incl_max = last, incl_min = first;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int64_t a = __shfl_up(incl_max, off, kWave);
            const int64_t d = __shfl_down(incl_min, off, kWave);
            if (lane >= off) incl_max = a > incl_max ? a : incl_max;
            if (lane + off < kWave) incl_min = d < incl_min ? d : incl_min;
        }
        if (lane == kWave - 1) s_w[0][w] = incl_max;
        if (lane == 0) s_w[1][w] = incl_min;
        int64_t before = __shfl_up(incl_max, 1, kWave), after = __shfl_down(incl_min, 1, kWave);
        if (lane == 0) before = -1;
        if (lane == kWave - 1) after = INT64_MAX;
        __syncthreads();
        for (int q = 0; q < 4; ++q) {
            if (q < w) before = s_w[0][q] > before ? s_w[0][q] : before;
            if (q > w) after = s_w[1][q] < after ? s_w[1][q] : after;
        }
        if (before < 0) before = head;        // the group continues from before the chunk
        if (after == INT64_MAX) after = tail;  // ... or past its end
        // next start after each element of the run (right to left), group start (left to right)
        int64_t ge[IPT];
        int64_t nxt = after;
#pragma unroll
        for (int m = IPT - 1; m >= 0; --m) {
            ge[m] = nxt;
            if (f[m]) nxt = b + q0 + m;
        }
        const double mm = double(se - sb + 1) / 2.0;
        DD acc[kSpNV];
#pragma unroll
        for (int v = 0; v < kSpNV; ++v) acc[v] = DD{0.0, 0.0};
        int64_t gs = before;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int q = q0 + m;
            if (q >= len) continue;
            if (f[m]) gs = b + q;
            const double rx = double(s_p[q] - sb + 1) - mm;
            const double ry = double((gs - sb) + (ge[m] - sb) + 1) / 2.0 - mm;
            acc[0] = dd_add_d(acc[0], rx * ry);
            acc[1] = dd_add_d(acc[1], rx * rx);
            acc[2] = dd_add_d(acc[2], ry * ry);
            acc[3] = dd_add_d(acc[3], f[m] ? 1.0 : 0.0);
        }
#pragma unroll
        for (int v = 0; v < kSpNV; ++v) {
            const DD r = wave_dd_sum(acc[v]);
            if (lane == 0) {
                s_hi[w][v] = r.hi;
                s_lo[w][v] = r.lo;
            }
        }
        __syncthreads();
        if (tid < kSpNV) {
            DD t{s_hi[0][tid], s_lo[0][tid]};
            for (int q = 1; q < 4; ++q) t = dd_add(t, DD{s_hi[q][tid], s_lo[q][tid]});
            part[(k * kSpNV + tid) * 2] = t.hi;
            part[(k * kSpNV + tid) * 2 + 1] = t.lo;
        }
        __syncthreads();  // LDS is reused by the next chunk
    }
}

// Brunner-Munzel of two samples from their sorted union (one segment [0, *d_live)): x = the values
// whose source position pos[i] < *d_nx, y the others; before[i] = the x values before union
// position i (an exclusive scan, before[live] = their total).  Chunk by chunk as k_spearman_chunks:
// a value's union tie group [gs, ge) from the tie-start flags (edge binary searches), its union
// rank rc = (gs + ge + 1) / 2, its within-sample rank rw from the x counts at the group's bounds
// (before[gs], before[ge]).  PASS 0 sums rc per sample; PASS 1 the squared deviations
// ((rc - rw) - mean rc) + mean rw per sample (means from PASS 0's sums) - the two reductions of
// scipy's brunnermunzel, each one launch + the fold, instead of the tie-rank passes, the x-count
// scan, the within-sample rank map and three segmented reductions.
constexpr int kBmNV = 2;
// brunnermunzel(x, y) from the union-rank sums s0 = {sum rank_c(x), sum rank_c(y)} and the squared
// deviation sums s1 (scipy _stats_py.py brunnermunzel, alternative two-sided, t distribution)
__device__ inline void bm_finish(int64_t nx_, int64_t ny_, const double *s0, const double *s1, double *bm_stat,
                                 double *bm_p) {
    const double nx = double(nx_), ny = double(ny_);
    const double rcx = s0[0] / nx, rcy = s0[1] / ny;
    const double Sx = s1[0] / (nx - 1.0), Sy = s1[1] / (ny - 1.0);
    double w = nx * ny * (rcy - rcx);
    w /= (nx + ny) * sqrt(nx * Sx + ny * Sy);
    const double num = (nx * Sx + ny * Sy) * (nx * Sx + ny * Sy);
    const double den = (nx * Sx) * (nx * Sx) / (nx - 1.0) + (ny * Sy) * (ny * Sy) / (ny - 1.0);
    if (bm_stat) *bm_stat = w;
    if (bm_p) *bm_p = 2.0 * t_sf_once(fabs(w), num / den);
}

template <int PASS>
__global__ __launch_bounds__(kBlock) void k_bm_union_chunks(int64_t cps, const int64_t *__restrict__ offs,
                                                            const double *__restrict__ sv,
                                                            const int32_t *__restrict__ pos,
                                                            const int64_t *__restrict__ before,
                                                            const int64_t *__restrict__ d_nx,
                                                            const double *__restrict__ sums0,
                                                            double *__restrict__ part, unsigned *tickets,
                                                            double *fold_out, double *bm_stat, double *bm_p) {
    constexpr int IPT = kRedItems;
    const bool fold = tickets != nullptr;
    __shared__ double s_v[kChunk];
    __shared__ int64_t s_w[2][4];
    __shared__ int64_t s_edge[2];
    __shared__ double s_hi[4][kBmNV], s_lo[4][kBmNV];
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
    const int64_t sb = offs[0], se = offs[1];
    const int64_t nx = *d_nx, ny = (se - sb) - nx;
    for (int64_t k = blockIdx.x; k < cps; k += gridDim.x) {
        const int64_t b = sb + k * kChunk;
        const int64_t e = b + kChunk < se ? b + kChunk : se;
        const int len = e > b ? int(e - b) : 0;
        if (len == 0) {  // past the union's live end: zero partials, no barriers
            if (tid < kBmNV) {
                store_wt(&part[(k * kBmNV + tid) * 2], 0.0);
                store_wt(&part[(k * kBmNV + tid) * 2 + 1], 0.0);
            }
            if (fold && chunk_arrive<kBmNV>(tickets, part, fold_out, 0, cps) && PASS == 1 && tid == 0)
                bm_finish(nx, ny, sums0, fold_out, bm_stat, bm_p);
            continue;
        }
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int j = tid + m * kBlock;
            if (j < len) s_v[j] = sv[b + j];
        }
        if (tid == 0) {
            int64_t gs = b;
            if (len > 0 && b > sb && sv[b - 1] == sv[b]) gs = lower_bound_d(sv, sb, b, sv[b]);
            s_edge[0] = gs;
        } else if (tid == kWave) {
            int64_t ge = e;
            if (len > 0 && e < se && sv[e] == sv[e - 1]) ge = upper_bound_d(sv, e, se, sv[e - 1]);
            s_edge[1] = ge;
        }
        __syncthreads();
        const int64_t head = s_edge[0], tail = s_edge[1];
        const int q0 = tid * IPT;
        bool f[IPT];
        int64_t first = INT64_MAX, last = -1;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int q = q0 + m;
            f[m] = q < len && (q == 0 ? head == b : s_v[q] != s_v[q - 1]);
            if (f[m]) {
                first = first < b + q ? first : b + q;
                last = b + q;
            }
        }
        int64_t incl_max = last, incl_min = first;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int64_t a = __shfl_up(incl_max, off, kWave);
            const int64_t d = __shfl_down(incl_min, off, kWave);
            if (lane >= off) incl_max = a > incl_max ? a : incl_max;
            if (lane + off < kWave) incl_min = d < incl_min ? d : incl_min;
        }
        if (lane == kWave - 1) s_w[0][w] = incl_max;
        if (lane == 0) s_w[1][w] = incl_min;
        int64_t bef = __shfl_up(incl_max, 1, kWave), aft = __shfl_down(incl_min, 1, kWave);
        if (lane == 0) bef = -1;
        if (lane == kWave - 1) aft = INT64_MAX;
        __syncthreads();
        for (int q = 0; q < 4; ++q) {
            if (q < w) bef = s_w[0][q] > bef ? s_w[0][q] : bef;
            if (q > w) aft = s_w[1][q] < aft ? s_w[1][q] : aft;
        }
        if (bef < 0) bef = head;
        if (aft == INT64_MAX) aft = tail;
        int64_t ge[IPT];
        int64_t nxt = aft;
#pragma unroll
        for (int m = IPT - 1; m >= 0; --m) {
            ge[m] = nxt;
            if (f[m]) nxt = b + q0 + m;
        }
        const double Nx = double(nx), Ny = double(ny);
        DD acc[kBmNV] = {DD{0.0, 0.0}, DD{0.0, 0.0}};
        int64_t gs = bef;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int q = q0 + m;
            if (q >= len) continue;
            if (f[m]) gs = b + q;
            const bool isx = pos[b + q] < nx;
            const double rc = double((gs - sb) + (ge[m] - sb) + 1) / 2.0;
            if constexpr (PASS == 0) {
                acc[isx ? 0 : 1] = dd_add_d(acc[isx ? 0 : 1], rc);
            } else {
                const int64_t xb = before[gs] - before[sb], xg = before[ge[m]] - before[gs];
                const int64_t yb = (gs - sb) - xb, yg = (ge[m] - gs) - xg;
                const double rw = isx ? double(xb) + double(xg + 1) / 2.0 : double(yb) + double(yg + 1) / 2.0;
                const double cm = isx ? sums0[0] / Nx : sums0[1] / Ny;        // np.mean(rankcx / rankcy)
                const double wm = isx ? (Nx + 1.0) / 2.0 : (Ny + 1.0) / 2.0;  // np.mean(rankx) (exact)
                const double d = ((rc - rw) - cm) + wm;
                acc[isx ? 0 : 1] = dd_add_d(acc[isx ? 0 : 1], d * d);
            }
        }
#pragma unroll
        for (int v = 0; v < kBmNV; ++v) {
            const DD r = wave_dd_sum(acc[v]);
            if (lane == 0) {
                s_hi[w][v] = r.hi;
                s_lo[w][v] = r.lo;
            }
        }
        __syncthreads();
        if (tid < kBmNV) {
            DD t{s_hi[0][tid], s_lo[0][tid]};
            for (int q = 1; q < 4; ++q) t = dd_add(t, DD{s_hi[q][tid], s_lo[q][tid]});
            store_wt(&part[(k * kBmNV + tid) * 2], t.hi);
            store_wt(&part[(k * kBmNV + tid) * 2 + 1], t.lo);
        }
        if (fold && chunk_arrive<kBmNV>(tickets, part, fold_out, 0, cps) && PASS == 1 && tid == 0)
            bm_finish(nx, ny, sums0, fold_out, bm_stat, bm_p);
        __syncthreads();
    }
}

void bm_union_sorted(fz_ctx *c, const Segs &one, const double *sorted, const int32_t *pos, const int64_t *before,
                     const int64_t *d_nx, double *bm_stat, double *bm_p) {
    const int64_t cap = one.n_cap;
    if (cap <= 0) return;
    const int64_t cps = (cap + kChunk - 1) / kChunk;  // (a capacity-sized map: chunks past the live end are empty)
    ChunkedSegs cs;
    cs.sg = one;
    cs.cps = cps;
    double *part = c->arena.get<double>(cps * kBmNV * 2);
    double *s0 = c->arena.get<double>(kBmNV), *s1 = c->arena.get<double>(kBmNV);
    const unsigned g = unsigned(cps < 8192 ? cps : 8192);
    const int64_t *offs = one.offs;
    // (a few hundred chunks: the last chunk of each pass folds the sums - and, in the second pass,
    // finishes the test - in place of k_seg_sum and the finishing launch)
    unsigned *tickets = fused_fold_on() && cps <= kFoldChunks ? seg_tickets(c, 1) : nullptr;
    {
        ProbeScope ps(c, "seg_rank_union", 0.0, offs + 1, 24.0);  // value 8 + position 4 + x count 8 (+ 4) per value
        k_bm_union_chunks<0><<<g, kBlock, 0, c->stream>>>(cps, offs, sorted, pos, before, d_nx, nullptr, part,
                                                          tickets, s0, nullptr, nullptr);
        FZ_LAUNCH_CHECK();
        if (!tickets) seg_fold_parts<kBmNV>(c, cs, part, s0);
        k_bm_union_chunks<1><<<g, kBlock, 0, c->stream>>>(cps, offs, sorted, pos, before, d_nx, s0, part,
                                                          tickets, s1, bm_stat, bm_p);
        FZ_LAUNCH_CHECK();
        if (!tickets) seg_fold_parts<kBmNV>(c, cs, part, s1);
    }
    if (!tickets)
        map_n(c, 1, nullptr, [=] __device__(int64_t) {  // as seg_rank_tests_sorted's finishing
            bm_finish(*d_nx, (offs[1] - offs[0]) - *d_nx, s0, s1, bm_stat, bm_p);
        });
}

// spearmanr(range(n), x) and shapiro(x) of one series x[0, *d_n) of at most kSpearmanSmall values
// in one workgroup: the keys sorted with their positions by a bitonic network held in registers
// (eight elements per thread: stages of distance 1-4 inside a thread, 8-256 by shuffles inside a
// wave, only the 6 of distance >= 512 through LDS with barriers - the whole network in LDS took
// 78 barrier stages, ~30 us of RQ2 count's chain), then the Spearman and Shapiro-Wilk passes over
// the sorted values in LDS.  (Equal keys keep either order: the tie groups are ranked as groups.)
constexpr int kSeriesBlock = 512;  // (1,024 threads spilled 120 VGPRs: the statistics' code)
static_assert(int(kSpearmanSmall) == kSeriesBlock * 8, "series network shape");
#ifndef FZ_SERIES_NET_CLASSES
#define FZ_SERIES_NET_CLASSES 1  // (0: every series through the 4,096-pair network; A/B builds)
#endif
// The series x[0, n) sorted by (key, position) with a bitonic network of kSeriesBlock * E pairs held
// in registers (E per thread: stages of distance < E inside a thread, < 64 E by shuffles inside a
// wave, the rest through LDS with barriers); the sorted values and positions left in sv / spos.
template <int E>
__device__ inline void series_net(const double *__restrict__ x, int n, uint64_t *sk, int32_t *spos) {
    constexpr int BS = kSeriesBlock;
    const int tid = threadIdx.x;
    uint64_t k[E];
    int32_t ps[E];
    {  // (all E loads in flight at once: a guarded load per element waited on each in turn)
        double v[E];
#pragma unroll
        for (int h = 0; h < E; ++h) {
            const int e = E * tid + h;
            v[h] = n > 0 ? x[e < n ? e : 0] : 0.0;
        }
#pragma unroll
        for (int h = 0; h < E; ++h) {
            const int e = E * tid + h;
            k[h] = e < n ? f64_key(v[h]) : ~0ull;
            ps[h] = e;
        }
    }
    // element e = E * tid + h; stage (kk, j) pairs e with e ^ j, ascending where e & kk == 0: the
    // lower element keeps the smaller key, the upper the larger (equal keys: each keeps its own)
    auto settle = [&](int h, uint64_t y, int32_t yp, int kk, int j) {
        const int e = E * tid + h;
        const bool up = (e & kk) == 0, low = (e & j) == 0;
        const bool take = (low == up) ? (y < k[h]) : (y > k[h]);
        if (take) {
            k[h] = y;
            ps[h] = yp;
        }
    };
    // (both loops unrolled: every stage's distance is a constant - the in-thread stages index
    // registers directly instead of through indirect register moves)
#pragma unroll
    for (int kk = 2; kk <= BS * E; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j < E) {
                uint64_t y[E];
                int32_t yp[E];
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    y[h] = k[h ^ j];
                    yp[h] = ps[h ^ j];
                }
#pragma unroll
                for (int h = 0; h < E; ++h) settle(h, y[h], yp[h], kk, j);
            } else if (j / E < kWave) {
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    const uint64_t y = __shfl_xor(k[h], j / E, 64);
                    const int32_t yp = __shfl_xor(ps[h], j / E, 64);
                    settle(h, y, yp, kk, j);
                }
            } else {
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    sk[E * tid + h] = k[h];
                    spos[E * tid + h] = ps[h];
                }
                __syncthreads();
                uint64_t y[E];
                int32_t yp[E];
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    y[h] = sk[(E * tid + h) ^ j];
                    yp[h] = spos[(E * tid + h) ^ j];
                }
                __syncthreads();
#pragma unroll
                for (int h = 0; h < E; ++h) settle(h, y[h], yp[h], kk, j);
            }
        }
    }
    double *sv = reinterpret_cast<double *>(sk);
#pragma unroll
    for (int h = 0; h < E; ++h) {
        sv[E * tid + h] = f64_from_key(k[h]);
        spos[E * tid + h] = ps[h];
    }
}
__global__ __launch_bounds__(kSeriesBlock) void k_series_small(const double *__restrict__ x,
                                                               const int64_t *__restrict__ d_n, double *rho,
                                                               double *pv, double *w, double *wp) {
    chain_prio();
    constexpr int BS = kSeriesBlock, NW = BS / kWave;
    __shared__ uint64_t sk[kSpearmanSmall];
    __shared__ int32_t spos[kSpearmanSmall];
    __shared__ double s_tmp[NW];
    __shared__ double s_hi[NW][3], s_lo[NW][3];
    __shared__ double s_m[kSpearmanSmall / 2];
    const int tid = threadIdx.x;
    SERIES_STAMP(0);
    const int n = int(*d_n);
    // the network sized to the series (the work is stages x pairs a thread on one CU: 78 x 8 for
    // 4,096 pairs, 45 x 1 for 512)
#if FZ_SERIES_NET_CLASSES
    if (n <= BS) series_net<1>(x, n, sk, spos);
    else if (n <= 2 * BS) series_net<2>(x, n, sk, spos);
    else if (n <= 4 * BS) series_net<4>(x, n, sk, spos);
    else
#endif
        series_net<8>(x, n, sk, spos);
    double *sv = reinterpret_cast<double *>(sk);
    __syncthreads();
    SERIES_STAMP(1);
    const SpearmanT st = spearman_block<BS>(sv, spos, 0, n, s_tmp, rho, pv, kSeriesDefer);
    SERIES_STAMP(2);
    const int64_t per = (int64_t(n) + BS - 1) / BS;
    const int64_t k0 = int64_t(tid) * per, k1 = k0 + per < n ? k0 + per : n;
    shapiro_block<BS>(sv, x, 0, n, k0, k1, s_hi, s_lo, s_m, w, wp);
    // (the Spearman p-value on the last wave while thread 0 finishes the Shapiro-Wilk one)
    if (kSeriesDefer && pv && tid == BS - 1) *pv = spearman_p(st);
    SERIES_STAMP(3);
}

bool series_small_ok(int64_t n_cap) { return n_cap <= kSpearmanSmall; }
void series_small(fz_ctx *c, const double *x, const int64_t *d_n, double *rho, double *pv, double *w, double *wp) {
    k_series_small<<<1, kSeriesBlock, 0, c->stream>>>(x, d_n, rho, pv, w, wp);
    FZ_LAUNCH_CHECK();
}

void spearman_shapiro_sorted(fz_ctx *c, const ChunkedSegs &cs, const int32_t *segid, const SortedSegs &ss,
                             const double *src, double *rho, double *pval, double *w, double *p) {
    const Segs &sg = cs.sg;
    if (sg.S <= 0) return;
    if (sg.len_bound() <= kSpearmanSmall) {  // both in one launch, one workgroup per segment
        // algorithmic bytes per live value: sorted value 8 + position 4 + input value 8 read
        ProbeScope ps(c, "spearman_shapiro", 0.0, sg.offs + sg.S, 20.0);
        k_spearman_index_small<<<unsigned(sg.S < 16384 ? sg.S : 16384), kBlock, 0, c->stream>>>(
            ss.val, ss.pos, sg.offs, sg.S, rho, pval, src, w, p);
        FZ_LAUNCH_CHECK();
        return;
    }
    if (rho) spearman_index_sorted(c, cs, segid, ss, rho, pval);
    seg_shapiro(c, cs, src, ss, w, p);
}

void spearman_index_sorted(fz_ctx *c, const ChunkedSegs &cs, const int32_t *segid, const SortedSegs &ss, double *rho,
                           double *pval) {
    const Segs &sg = cs.sg;
    if (sg.S <= 0) return;
    if (sg.len_bound() <= kSpearmanSmall) {
        k_spearman_index_small<<<unsigned(sg.S < 16384 ? sg.S : 16384), kBlock, 0, c->stream>>>(ss.val, ss.pos, sg.offs,
                                                                                              sg.S, rho, pval);
        FZ_LAUNCH_CHECK();
        return;
    }
    if (cs.lists.on) {  // (very many segments: the size-class lists, device-wide tie ranks)
        TieRanks tr = seg_tie_ranks(c, cs, segid, ss.val);
        seg_spearman_index(c, cs, ss, tr, rho, pval);
        return;
    }
    const int64_t S = sg.S;
    const int64_t *offs = sg.offs;
    const int64_t blocks = cs.cps > 0 ? S * cs.cps : cs.cm.cap;
    double *part = c->arena.get<double>(blocks * kSpNV * 2);
    {
        // algorithmic bytes per live value: value 8 + position 4 read
        ProbeScope ps(c, "seg_spearman", 8.0 * kSpNV * double(S), offs + S, 12.0);
        k_spearman_chunks<<<unsigned(blocks < 8192 ? blocks : 8192), kBlock, 0, c->stream>>>(cs.cm, offs, cs.cps, blocks,
                                                                                             ss.val, ss.pos, part);
        FZ_LAUNCH_CHECK();
        double *sums = c->arena.get<double>(S * kSpNV);
        seg_fold_parts<kSpNV>(c, cs, part, sums);
        per_seg(c, S, [=] __device__(int64_t s) {  // as seg_spearman_index
            const int64_t n = offs[s + 1] - offs[s];
            double r = NAN, p = NAN;
            if (n >= 2 && sums[kSpNV * s + 3] > 1.0) {
                const double f = 1.0 / double(n - 1);  // (np.cov: times the reciprocal)
                const double cxy = sums[kSpNV * s] * f, cxx = sums[kSpNV * s + 1] * f, cyy = sums[kSpNV * s + 2] * f;
                r = cxy / sqrt(cxx) / sqrt(cyy);
                if (r > 1.0) r = 1.0;
                if (r < -1.0) r = -1.0;
                const double dof = double(n - 2);
                double q = dof / ((r + 1.0) * (1.0 - r));
                if (q < 0.0) q = 0.0;
                const double t = r * sqrt(q);
                p = 2.0 * t_sf_once(fabs(t), dof);
            }
            rho[s] = r;
            if (pval) pval[s] = p;
        });
    }
}

// ------------------------------------------------------------------------- Shapiro-Wilk
void seg_shapiro(fz_ctx *c, const ChunkedSegs &cs, const double *src, const SortedSegs &ss, double *w, double *p) {
    const int64_t *offs = cs.sg.offs;
    const int64_t S = cs.sg.S;
    const double *v = ss.val;
    double *summ2 = c->arena.get<double>(S);
    double *coef = c->arena.get<double>(S * 4);   // a1, a2, fac, i1
    double *shift = c->arena.get<double>(S * 2);  // x0 (= x[n//2]), range
    double *s1 = c->arena.get<double>(S * 2);     // sx, sa
    double *s2 = c->arena.get<double>(S * 3);     // ssa, ssx, sax
    // pass A: summ2 = 2 * sum_{i <= n/2} m_i^2
    seg_reduce<1>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const int64_t b = offs[s], n = offs[s + 1] - b, k = i - b + 1;
        double m = 0.0;
        if (n >= 3 && k <= n / 2) m = stats::sw_m(k, n);
        x[0] = m * m;
    }, summ2, 0.0);  // (normal scores computed, nothing read per element)
    per_seg(c, S, [=] __device__(int64_t s) {
        const int64_t b = offs[s], n = offs[s + 1] - b;
        if (n < 3) return;
        const stats::SwCoef cf = stats::sw_coef(n, 2.0 * summ2[s]);
        coef[4 * s] = cf.a1;
        coef[4 * s + 1] = cf.a2;
        coef[4 * s + 2] = cf.fac;
        coef[4 * s + 3] = double(cf.i1);
        const double x0 = src[b + n / 2];  // scipy: y = sort(x); y -= x[N//2]
        shift[2 * s] = x0;
        shift[2 * s + 1] = (v[b + n - 1] - x0) - (v[b] - x0);
    });
    auto coef_of = [=] __device__(int32_t s, int64_t n) {
        stats::SwCoef cf;
        cf.n = n;
        cf.a1 = coef[4 * s];
        cf.a2 = coef[4 * s + 1];
        cf.fac = coef[4 * s + 2];
        cf.i1 = int(coef[4 * s + 3]);
        return cf;
    };
    // pass B: sx = sum y/range, sa = sum of signed coefficients
    seg_reduce<2>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const int64_t b = offs[s], n = offs[s + 1] - b;
        x[0] = x[1] = 0.0;
        if (n < 3) return;
        const double range = shift[2 * s + 1];
        x[0] = (v[i] - shift[2 * s]) / range;
        x[1] = stats::sw_coef_at(coef_of(s, n), i - b + 1);
    }, s1, 8.0);
    // pass C: ssa, ssx, sax
    seg_reduce<3>(c, cs, [=] __device__(int64_t i, int32_t s, double *x) {
        const int64_t b = offs[s], n = offs[s + 1] - b;
        x[0] = x[1] = x[2] = 0.0;
        if (n < 3) return;
        const double range = shift[2 * s + 1];
        const double sa = s1[2 * s + 1] / double(n), sx = s1[2 * s] / double(n);
        const double asa = stats::sw_coef_at(coef_of(s, n), i - b + 1) - sa;
        const double xsx = (v[i] - shift[2 * s]) / range - sx;
        x[0] = asa * asa;
        x[1] = xsx * xsx;
        x[2] = asa * xsx;
    }, s2, 8.0);
    per_seg(c, S, [=] __device__(int64_t s) {
        const int64_t n = offs[s + 1] - offs[s];
        if (n < 3) {
            w[s] = NAN;
            p[s] = NAN;
            return;
        }
        if (shift[2 * s + 1] < stats::kSwSmall) {  // zero range: scipy returns (1.0, 1.0)
            w[s] = 1.0;
            p[s] = 1.0;
            return;
        }
        const double ssa = s2[3 * s], ssx = s2[3 * s + 1], sax = s2[3 * s + 2];
        const double ssassx = sqrt(ssa * ssx);
        const double w1 = (ssassx - sax) * (ssassx + sax) / (ssa * ssx);
        const double ww = 1.0 - w1;
        w[s] = ww;
        p[s] = sw_pvalue_once(n, ww, w1);
    });
}

// ------------------------------------------------------------- percentiles, means, medians
void seg_percentiles(fz_ctx *c, const Segs &sg, const double *sorted, const double *q_host, int nq, double *out,
                     double *median, double *out2) {
    double q[8];
    for (int j = 0; j < nq && j < 8; ++j) q[j] = q_host[j];
    const int64_t *offs = sg.offs;
    per_seg(c, sg.S, [=] __device__(int64_t s) {
        const int64_t b = offs[s], n = offs[s + 1] - b;
        if (median)  // (seg_median's value, from the same thread's reads)
            median[s] = n <= 0 ? NAN : ((n & 1) ? sorted[b + n / 2] : (sorted[b + n / 2 - 1] + sorted[b + n / 2]) / 2.0);
        double *o = out2 ? ((s & 1) ? out2 : out) + (s >> 1) * nq : out + s * nq;
        for (int j = 0; j < nq; ++j) {
            if (n <= 0) {
                o[j] = NAN;
                continue;
            }
            o[j] = np_percentile_sorted([&](int64_t k) { return sorted[b + k]; }, n, q[j]);
        }
    });
}

void seg_mean(fz_ctx *c, const ChunkedSegs &cs, const double *vals, double *out) {
    double *sum = c->arena.get<double>(cs.sg.S);
    seg_reduce<1>(c, cs, [=] __device__(int64_t i, int32_t, double *x) { x[0] = vals[i]; }, sum);
    const int64_t *offs = cs.sg.offs;
    per_seg(c, cs.sg.S, [=] __device__(int64_t s) {
        const int64_t n = offs[s + 1] - offs[s];
        out[s] = n > 0 ? sum[s] / double(n) : NAN;
    });
}

void seg_median(fz_ctx *c, const Segs &sg, const double *sorted, double *out) {
    const int64_t *offs = sg.offs;
    per_seg(c, sg.S, [=] __device__(int64_t s) {
        const int64_t b = offs[s], n = offs[s + 1] - b;
        if (n <= 0) {
            out[s] = NAN;
            return;
        }
        out[s] = (n & 1) ? sorted[b + n / 2] : (sorted[b + n / 2 - 1] + sorted[b + n / 2]) / 2.0;
    });
}

// ------------------------------------------------- order statistics without sorting (seg_qstats)
// RQ2's per-session statistics (rq2_coverage_count.py:139-152, :439-440) need the mean, the
// median and five percentiles of each session - at most 12 order statistics, not the whole sorted
// session.  Each segment's order statistics are SELECTED: one read of its values (the mean's
// double-double sum on the way), a value-bucket histogram over the segment's key range in LDS (the
// bucket of key k is floor((k - lo) * nb / (hi - lo + 1)), monotone in k, so a bucket holds exactly
// the values of a key interval), one block scan, and each wanted rank's bucket ranked in one wave.
// A bucket of more than 64 values (clusters) is refined by re-histogramming its key interval until
// it holds <= 64 values or one key.  Nothing is written but the statistics.
struct QsArgs {
    double q[8];
    int nq;
    double *mean, *median, *pcts;  // [S], [S], [S * nq]
    double *mean2;                 // [S] a second copy of the means (optional)
    int64_t *d_ge100;              // += segments of >= 100 values
};
constexpr int kQsMaxT = 2 * 8 + 2;  // ranks wanted per segment (two per percentile, two for the median)
#ifndef FZ_QS_KEYS_GLOBAL
#define FZ_QS_KEYS_GLOBAL 1
#endif
constexpr bool kQsKeysGlobal = FZ_QS_KEYS_GLOBAL;

// rank t of the nt = 2 + 2 * nq order statistics a segment of n >= 1 values needs: statistics.median
// reads ranks 0, 1; np_percentile_sorted(q[j]) reads ranks 2 + 2j, 3 + 2j (its prev / next index)
__device__ inline int64_t qs_rank(int64_t n, const QsArgs &a, int t) {
    if (t == 0) return n / 2;
    if (t == 1) return (n & 1) ? n / 2 : n / 2 - 1;
    const int j = (t - 2) >> 1;
    const double vi = double(n - 1) * (a.q[j] / 100.0);
    int64_t r = int64_t(floor(vi)) + ((t - 2) & 1);
    return r > n - 1 ? n - 1 : (r < 0 ? 0 : r);
}

// the statistics of one segment from its order statistics get(rank) (ranks from qs_ranks)
template <typename Get>
__device__ inline void qs_write(const QsArgs &a, int64_t s, int64_t n, double sum, Get get) {
    if (n <= 0) {
        a.mean[s] = NAN;
        if (a.mean2) a.mean2[s] = NAN;
        a.median[s] = NAN;
        for (int j = 0; j < a.nq; ++j) a.pcts[s * a.nq + j] = NAN;
        return;
    }
    a.mean[s] = sum / double(n);
    if (a.mean2) a.mean2[s] = sum / double(n);
    a.median[s] = (n & 1) ? get(n / 2) : (get(n / 2 - 1) + get(n / 2)) / 2.0;
    for (int j = 0; j < a.nq; ++j) a.pcts[s * a.nq + j] = np_percentile_sorted(get, n, a.q[j]);
}

// Size classes of the selection: lists of the segments too long for one lane (filled by
// k_qs_micro), one list per class - tiny (33-64 values: one wave each; 9-16 / 17-32 values: a
// quarter / half of a wave each), mid and big (one workgroup each).
enum { kQsTiny = 0, kQsMid = 1, kQsBig = 2, kQsBlock = 3, kQsTiny16 = 4, kQsTiny32 = 5, kQsLists = 6 };
struct QsLists {
    int32_t *ids[kQsLists];
    int64_t *d_n;  // [kQsLists] (zero on entry)
};

// append segment s to list cls of L when `want` (wave-aggregated: one atomic per wave and class)
__device__ inline void qs_append(const QsLists &L, int cls, bool want, int64_t s) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lane = lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(reinterpret_cast<unsigned long long *>(L.d_n + cls),
                                         (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    if (want) L.ids[cls][base + __popcll(m & lanemask_lt())] = int32_t(s);
}

// One lane per segment (wave v: segments 64v .. 64v + 63, coalesced offset reads): a segment of
// <= kMicroSeg values is finished by its lane (register sorting network); longer ones go to their
// class list - tiny (<= kTinySeg), mid (<= 1024), block (<= 2048), big.
__global__ __launch_bounds__(kBlock) void k_qs_micro(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                     int64_t S, QsArgs a, QsLists L) {
    const int lane = lane_id();
    const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
    for (int64_t v = int64_t(blockIdx.x) * (kBlock / kWave) + wave_id(); v * 64 < S; v += nwaves) {
        const int64_t s = v * 64 + lane;
        const int64_t b = s < S ? offs[s] : 0;
        const int64_t n = s < S ? offs[s + 1] - b : -1;
        qs_append(L, kQsTiny16, n > kMicroSeg && n <= 16, s);
        qs_append(L, kQsTiny32, n > 16 && n <= 32, s);
        qs_append(L, kQsTiny, n > 32 && n <= kTinySeg, s);
        qs_append(L, 1, n > kTinySeg && n <= 1024, s);
        qs_append(L, 2, n > 2048, s);
        qs_append(L, 3, n > 1024 && n <= 2048, s);
        if (n < 0 || n > kMicroSeg) continue;
        uint64_t k[kMicroSeg];
        DD acc{0.0, 0.0};
#pragma unroll
        for (int q = 0; q < kMicroSeg; ++q) {
            const double x = q < n ? src[b + q] : 0.0;
            if (q < n) acc = dd_add_d(acc, x);
            k[q] = q < n ? f64_key(x) : ~0ull;
        }
        constexpr int net[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
                                    {0, 4}, {1, 5}, {2, 6}, {3, 7}, {2, 4}, {3, 5}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
        for (int c = 0; c < 19; ++c) {
            const uint64_t x = k[net[c][0]], y = k[net[c][1]];
            k[net[c][0]] = x < y ? x : y;
            k[net[c][1]] = x < y ? y : x;
        }
        auto get = [&](int64_t j) {
            uint64_t r = k[0];
#pragma unroll
            for (int q = 1; q < kMicroSeg; ++q) r = j == q ? k[q] : r;
            return f64_from_key(r);
        };
        qs_write(a, s, n, acc.hi + acc.lo, get);
    }
}

// The tiny lists: GW lanes per segment, 64 / GW segments per wave (GW-lane bitonic network on the
// keys, order statistics gathered by shuffles).  Sessions of 9-16 values - most of the tall
// session layouts' tail (config 5L: ~1.3 M sessions of 9-64 values) - take a quarter of a wave
// each: a quarter of the waves and 10 network stages instead of 21.
template <int GW>
__global__ __launch_bounds__(kBlock) void k_qs_tiny(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                    const int32_t *__restrict__ list, const int64_t *__restrict__ d_ln,
                                                    QsArgs a) {
    static_assert(GW == 16 || GW == 32 || GW == 64, "group width");
    constexpr int PER = kWave / GW;
    const int lane = lane_id();
    const int sub = lane & (GW - 1), grp = lane / GW;
    const int64_t ns = *d_ln;
    const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
    for (int64_t w = int64_t(blockIdx.x) * (kBlock / kWave) + wave_id(); w * PER < ns; w += nwaves) {
        const int64_t idx = w * PER + grp;
        const bool have = idx < ns;
        const int64_t st = have ? list[idx] : 0;
        const int64_t sb = have ? offs[st] : 0;
        const int sn = have ? int(offs[st + 1] - sb) : 0;
        const double x = sub < sn ? src[sb + sub] : 0.0;
        DD acc{sub < sn ? x : 0.0, 0.0};
#pragma unroll
        for (int off = GW / 2; off > 0; off >>= 1) {
            DD y{__shfl_xor(acc.hi, off, 64), __shfl_xor(acc.lo, off, 64)};
            acc = dd_add(acc, y);
        }
        unsigned long long key = sub < sn ? f64_key(x) : ~0ull;
#pragma unroll
        for (int kk = 2; kk <= GW; kk <<= 1) {
#pragma unroll
            for (int j = kk >> 1; j > 0; j >>= 1) {
                const unsigned long long ok = __shfl_xor(key, j, 64);
                const bool want_min = ((sub & j) == 0) == ((sub & kk) == 0);
                if (want_min == (ok < key)) key = ok;
            }
        }
        // every rank any statistic reads, gathered by shuffles (all lanes take part)
        const int nt = 2 + 2 * a.nq;
        int rk[kQsMaxT];
        double rv[kQsMaxT];
#pragma unroll
        for (int t = 0; t < kQsMaxT; ++t) {
            rk[t] = t < nt && sn > 0 ? int(qs_rank(sn, a, t)) : -1;
            rv[t] = f64_from_key(__shfl(key, grp * GW + (rk[t] < 0 ? 0 : rk[t]), 64));
        }
        if (sub == 0 && have) {
            auto get = [&](int64_t j) {
                double r = 0.0;
#pragma unroll
                for (int t = 0; t < kQsMaxT; ++t) r = rk[t] == j ? rv[t] : r;
                return r;
            };
            qs_write(a, st, sn, acc.hi + acc.lo, get);
        }
    }
}

// The segments of one class list (at most MAXN values each), one workgroup each.
template <int BS, int MAXN>
#ifndef FZ_QS_BIG_WPE
#define FZ_QS_BIG_WPE 6  // the keys-from-global class at 6 waves per SIMD (80 registers, a 60-byte spill): three
                         // 512-thread workgroups per CU; config 3L 19.13 -> 18.81 ms (profiles/r06_qs_big_wpe_ab.txt)
#endif
struct QsBlockWpe {  // (the keys-from-global big class: its waves per SIMD)
    static constexpr int v = (MAXN > 2048 && kQsKeysGlobal) ? FZ_QS_BIG_WPE : 1;
};
template <int BS, int MAXN>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(QsBlockWpe<BS, MAXN>::v))) void k_qs_block(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                 const int32_t *__restrict__ list, const int64_t *__restrict__ d_ln,
                                                 QsArgs a) {
    constexpr int NW = BS / kWave;
    constexpr int IPT = MAXN / BS;                // values per thread
    constexpr int NB = MAXN < 4096 ? MAXN : 4096;  // buckets
    constexpr int BPT = NB / BS > 0 ? NB / BS : 1;
    // (the 16384 class keeps the keys in LDS: 16 per thread in registers spilled - 31 VGPRs of
    // scratch per lane, 2.6x the algorithmic bytes in HBM traffic at config 3; FZ_QS_KEYS_GLOBAL:
    // it re-reads them from the (L2-resident) session instead - no 128 KiB key array, several
    // workgroups per CU instead of one)
    constexpr bool KEYS_GLOBAL = MAXN > 2048 && kQsKeysGlobal;
    constexpr bool KEYS_LDS = MAXN > 2048 && !KEYS_GLOBAL;
    constexpr int UF = KEYS_GLOBAL ? 4 : IPT;  // (keys re-read: a few loads in flight per thread, not 32)
    static_assert(MAXN % BS == 0 && NB % BS == 0, "qstats shape");
    __shared__ uint64_t s_keys[KEYS_LDS ? MAXN : 1];
    __shared__ uint32_t s_cnt[NB + 1];
    __shared__ uint8_t s_map[NB];
    __shared__ uint64_t s_list[kQsMaxT][64];
    __shared__ uint32_t s_fill[kQsMaxT];
    __shared__ uint64_t s_lo[NW], s_hi[NW];
    __shared__ double s_dhi[NW], s_dlo[NW];
    __shared__ uint32_t s_tmp[NW];
    __shared__ int64_t s_tb[kQsMaxT], s_toff[kQsMaxT], s_tsz[kQsMaxT];
    __shared__ int s_tslot[kQsMaxT];
    __shared__ uint64_t s_res[kQsMaxT];
    __shared__ int64_t s_r, s_rc;
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    int64_t ge100 = 0;
    const int64_t ln = *d_ln;
    for (int64_t it = blockIdx.x; it < ln; it += gridDim.x) {
        const int64_t s = list[it];
        const int64_t b = offs[s];
        const int64_t n = offs[s + 1] - b;
        uint64_t kr[KEYS_LDS || KEYS_GLOBAL ? 1 : IPT];
        auto K = [&](int m) -> uint64_t {
            if constexpr (KEYS_GLOBAL) {
                const int64_t i = tid + int64_t(m) * BS;
                return i < n ? f64_key(src[b + i]) : 0ull;
            } else {
                return KEYS_LDS ? s_keys[tid + m * BS] : kr[m];
            }
        };
        auto K_set = [&](int m, uint64_t v) {
            if constexpr (KEYS_LDS) s_keys[tid + m * BS] = v;
            else if constexpr (!KEYS_GLOBAL) kr[m] = v;
        };
        uint64_t lo = ~0ull, hi = 0ull;
        DD acc{0.0, 0.0};
#pragma unroll UF
        for (int m = 0; m < IPT; ++m) {
            const int64_t i = tid + int64_t(m) * BS;
            const double x = i < n ? src[b + i] : 0.0;
            const uint64_t km = i < n ? f64_key(x) : 0ull;
            K_set(m, km);
            if (i < n) {
                acc = dd_add_d(acc, x);
                lo = km < lo ? km : lo;
                hi = km > hi ? km : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        acc = wave_dd_sum(acc);
        if (lane == 0) {
            s_lo[w] = lo;
            s_hi[w] = hi;
            s_dhi[w] = acc.hi;
            s_dlo[w] = acc.lo;
        }
        const int nb = n < NB ? int(n) : NB;
        for (int j = tid; j <= nb; j += BS) s_cnt[j] = 0u;
        for (int j = tid; j < nb; j += BS) s_map[j] = 0xff;
        __syncthreads();
        lo = s_lo[0];
        hi = s_hi[0];
#pragma unroll
        for (int q = 1; q < NW; ++q) {
            lo = s_lo[q] < lo ? s_lo[q] : lo;
            hi = s_hi[q] > hi ? s_hi[q] : hi;
        }
        const int nt = 2 + 2 * a.nq;
        const double scale = double(nb) / (double(hi - lo) + 1.0);
        auto bucket = [&](uint64_t key, uint64_t klo, double sc, int nbk) {
            uint32_t q = uint32_t(double(key - klo) * sc);
            return q < uint32_t(nbk) ? q : uint32_t(nbk - 1);
        };
        // the first level linear in VALUE when the range is finite (coverage percentages: dense
        // centres spread, repeated values one per bucket), else in key - monotone either way
        const double vlo = f64_from_key(lo), vhi = f64_from_key(hi);
        const bool vlin = isfinite(vlo) && isfinite(vhi) && isfinite(vhi - vlo) && vhi > vlo;
        const double vsc = vlin ? double(nb) / (vhi - vlo) : 0.0;
        auto bucket1 = [&](uint64_t key) -> uint32_t {
            if (!vlin) return bucket(key, lo, scale, nb);
            const double q = (f64_from_key(key) - vlo) * vsc;
            return q < double(nb - 1) ? uint32_t(q) : uint32_t(nb - 1);
        };
        if (lo != hi) {
#pragma unroll UF
            for (int m = 0; m < IPT; ++m)
                if (tid + int64_t(m) * BS < n) atomicAdd(&s_cnt[bucket1(K(m))], 1u);
            __syncthreads();
            // bucket starts: thread t scans buckets [t * BPT, t * BPT + BPT)
            uint32_t sum = 0;
#pragma unroll
            for (int e = 0; e < BPT; ++e) sum += tid * BPT + e < nb ? s_cnt[tid * BPT + e] : 0u;
            uint32_t run = block_excl_scan<uint32_t, NW>(sum, s_tmp, (uint32_t *)nullptr);
#pragma unroll
            for (int e = 0; e < BPT; ++e) {
                if (tid * BPT + e < nb) {
                    const uint32_t ce = s_cnt[tid * BPT + e];
                    s_cnt[tid * BPT + e] = run;
                    run += ce;
                }
            }
            if (tid == 0) s_cnt[nb] = uint32_t(n);
            __syncthreads();
            if (tid < nt) {  // the bucket holding rank rk[tid]: the last start <= rank
                const uint32_t r = uint32_t(qs_rank(n, a, tid));
                int l0 = 0, h0 = nb - 1;
                while (l0 < h0) {
                    const int mid = (l0 + h0 + 1) >> 1;
                    if (s_cnt[mid] <= r) l0 = mid;
                    else h0 = mid - 1;
                }
                s_tb[tid] = l0;
                s_toff[tid] = int64_t(r) - int64_t(s_cnt[l0]);
                s_tsz[tid] = int64_t(s_cnt[l0 + 1]) - int64_t(s_cnt[l0]);
            }
            __syncthreads();
            if (tid == 0) {  // one list slot per distinct small target bucket
                int used = 0;
                for (int t = 0; t < nt; ++t) {
                    int slot = -1;
                    if (s_tsz[t] <= 64) {
                        for (int u = 0; u < t; ++u)
                            if (s_tslot[u] >= 0 && s_tb[u] == s_tb[t]) slot = s_tslot[u];
                        if (slot < 0) {
                            slot = used++;
                            s_fill[slot] = 0u;
                            s_map[s_tb[t]] = uint8_t(slot);
                        }
                    }
                    s_tslot[t] = slot;
                }
            }
            __syncthreads();
#pragma unroll UF
            for (int m = 0; m < IPT; ++m) {
                if (tid + int64_t(m) * BS < n) {
                    const uint8_t slot = s_map[bucket1(K(m))];
                    if (slot != 0xff) s_list[slot][atomicAdd(&s_fill[slot], 1u)] = K(m);
                }
            }
            __syncthreads();
            for (int t = w; t < nt; t += NW) {  // rank inside the bucket (ties: any of them)
                const int slot = s_tslot[t];
                if (slot < 0) continue;
                const int sz = int(s_tsz[t]);
                const uint64_t e = lane < sz ? s_list[slot][lane] : ~0ull;
                int r = 0;
                for (int j = 0; j < sz; ++j) {
                    const uint64_t o = s_list[slot][j];
                    r += (o < e) || (o == e && j < lane);
                }
                if (lane < sz && r == int(s_toff[t])) s_res[t] = e;
            }
            __syncthreads();
            // a target bucket of more than 64 values: narrow its key interval until it holds <= 64
            // values or one key (uniform control flow: every thread runs the same rounds)
            for (int t = 0; t < nt; ++t) {
                if (s_tslot[t] >= 0) continue;
                // the bucket's key interval [rlo, rhi] (a bucket = the values of one key interval)
                const uint32_t tb = uint32_t(s_tb[t]);
                uint64_t rlo = ~0ull, rhi = 0ull;
#pragma unroll UF
                for (int m = 0; m < IPT; ++m)
                    if (tid + int64_t(m) * BS < n && bucket1(K(m)) == tb) {
                        rlo = K(m) < rlo ? K(m) : rlo;
                        rhi = K(m) > rhi ? K(m) : rhi;
                    }
                rlo = wave_min(rlo);
                rhi = wave_max(rhi);
                if (lane == 0) {
                    s_lo[w] = rlo;
                    s_hi[w] = rhi;
                }
                __syncthreads();
                rlo = s_lo[0];
                rhi = s_hi[0];
                for (int q = 1; q < NW; ++q) {
                    rlo = s_lo[q] < rlo ? s_lo[q] : rlo;
                    rhi = s_hi[q] > rhi ? s_hi[q] : rhi;
                }
                int64_t r = s_toff[t], cnt = s_tsz[t];
                __syncthreads();
                while (rlo != rhi && cnt > 64) {
                    const int nb2 = cnt < NB ? int(cnt) : NB;
                    const double sc2 = double(nb2) / (double(rhi - rlo) + 1.0);
                    for (int j = tid; j <= nb2; j += BS) s_cnt[j] = 0u;
                    __syncthreads();
#pragma unroll UF
                    for (int m = 0; m < IPT; ++m)
                        if (tid + int64_t(m) * BS < n && K(m) >= rlo && K(m) <= rhi)
                            atomicAdd(&s_cnt[bucket(K(m), rlo, sc2, nb2)], 1u);
                    __syncthreads();
                    {  // the sub-bucket holding rank r: thread t sums buckets [t * BPT, t * BPT + BPT),
                       // one block scan, the thread whose run holds r walks it (not a dependent wave
                       // scan per 64 buckets)
                        uint32_t cb[BPT], sum = 0;
#pragma unroll
                        for (int e = 0; e < BPT; ++e) {
                            const int j = tid * BPT + e;
                            cb[e] = j < nb2 ? s_cnt[j] : 0u;
                            sum += cb[e];
                        }
                        const uint32_t run = block_excl_scan<uint32_t, NW>(sum, s_tmp, (uint32_t *)nullptr);
                        const uint32_t rr = uint32_t(r);
                        if (rr >= run && rr < run + sum) {
                            uint32_t before = run;
#pragma unroll
                            for (int e = 0; e < BPT; ++e) {
                                if (rr >= before && rr < before + cb[e]) {
                                    s_r = int64_t(rr - before);
                                    s_rc = int64_t(cb[e]);
                                    s_cnt[NB] = uint32_t(tid * BPT + e);
                                }
                                before += cb[e];
                            }
                        }
                    }
                    __syncthreads();
                    const uint32_t sb = s_cnt[NB];
                    uint64_t nlo = ~0ull, nhi = 0ull;
#pragma unroll UF
                    for (int m = 0; m < IPT; ++m)
                        if (tid + int64_t(m) * BS < n && K(m) >= rlo && K(m) <= rhi && bucket(K(m), rlo, sc2, nb2) == sb) {
                            nlo = K(m) < nlo ? K(m) : nlo;
                            nhi = K(m) > nhi ? K(m) : nhi;
                        }
                    nlo = wave_min(nlo);
                    nhi = wave_max(nhi);
                    if (lane == 0) {
                        s_lo[w] = nlo;
                        s_hi[w] = nhi;
                    }
                    __syncthreads();
                    nlo = s_lo[0];
                    nhi = s_hi[0];
                    for (int q = 1; q < NW; ++q) {
                        nlo = s_lo[q] < nlo ? s_lo[q] : nlo;
                        nhi = s_hi[q] > nhi ? s_hi[q] : nhi;
                    }
                    r = s_r;
                    cnt = s_rc;
                    rlo = nlo;
                    rhi = nhi;
                    __syncthreads();
                }
                if (rlo == rhi) {
                    if (tid == 0) s_res[t] = rlo;
                } else {  // <= 64 values in [rlo, rhi]: list them, one wave ranks them
                    if (tid == 0) s_fill[0] = 0u;
                    __syncthreads();
#pragma unroll UF
                    for (int m = 0; m < IPT; ++m)
                        if (tid + int64_t(m) * BS < n && K(m) >= rlo && K(m) <= rhi)
                            s_list[0][atomicAdd(&s_fill[0], 1u)] = K(m);
                    __syncthreads();
                    if (w == 0) {
                        const int sz = int(cnt);
                        const uint64_t e = lane < sz ? s_list[0][lane] : ~0ull;
                        int rr = 0;
                        for (int j = 0; j < sz; ++j) {
                            const uint64_t o = s_list[0][j];
                            rr += (o < e) || (o == e && j < lane);
                        }
                        if (lane < sz && rr == int(r)) s_res[t] = e;
                    }
                }
                __syncthreads();
            }
        } else if (tid < nt) {
            s_res[tid] = lo;  // one distinct key
        }
        __syncthreads();
        if (tid == 0) {
            DD tot{s_dhi[0], s_dlo[0]};
            for (int q = 1; q < NW; ++q) tot = dd_add(tot, DD{s_dhi[q], s_dlo[q]});
            auto get = [&](int64_t j) {
                uint64_t r = 0;
                for (int t = 0; t < nt; ++t)
                    if (qs_rank(n, a, t) == j) r = s_res[t];
                return f64_from_key(r);
            };
            qs_write(a, s, n, tot.hi + tot.lo, get);
            if (n >= 100) ++ge100;
        }
        __syncthreads();  // LDS is reused by the next segment
    }
    if (tid == 0 && ge100) atomic_add_i64(a.d_ge100, ge100);
}

// The mid list (kTinySeg < n <= 1024 values): one 256-thread workgroup per segment sorts the keys
// in LDS (bitonic network, +inf padding; only its stages of distance >= 128 need a workgroup
// barrier) and reads the order statistics off the sorted keys - at these lengths a few dozen LDS
// stages beat the histogram selection's barrier rounds and per-target list ranking (config 2:
// ~3,000 sessions of <= 1,000 values).
__global__ __launch_bounds__(256) void k_qs_sort_mid(const double *__restrict__ src, const int64_t *__restrict__ offs,
                                                     const int32_t *__restrict__ list,
                                                     const int64_t *__restrict__ d_ln, QsArgs a) {
    constexpr int BS = 256, MAXN = 1024, NW = BS / kWave;
    __shared__ uint64_t sk[MAXN];
    __shared__ double s_dhi[NW], s_dlo[NW];
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
    int64_t ge100 = 0;
    const int64_t ln = *d_ln;
    for (int64_t it = blockIdx.x; it < ln; it += gridDim.x) {
        const int64_t s = list[it];
        const int64_t b = offs[s];
        const int n = int(offs[s + 1] - b);
        int np2 = 64;
        while (np2 < n) np2 <<= 1;
        DD acc{0.0, 0.0};
        for (int i = tid; i < np2; i += BS) {
            const double x = i < n ? src[b + i] : 0.0;
            if (i < n) acc = dd_add_d(acc, x);
            sk[i] = i < n ? f64_key(x) : ~0ull;
        }
        acc = wave_dd_sum(acc);
        if (lane == 0) {
            s_dhi[w] = acc.hi;
            s_dlo[w] = acc.lo;
        }
        __syncthreads();
        for (int k = 2; k <= np2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = tid; t < (np2 >> 1); t += BS) {
                    const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ixj = i + j;
                    const uint64_t u = sk[i], d = sk[ixj];
                    if ((u > d) == ((i & k) == 0)) {
                        sk[i] = d;
                        sk[ixj] = u;
                    }
                }
                bitonic_stage_sync(k, j, np2);
            }
        }
        if (tid == 0) {
            DD tot{s_dhi[0], s_dlo[0]};
            for (int q = 1; q < NW; ++q) tot = dd_add(tot, DD{s_dhi[q], s_dlo[q]});
            qs_write(a, s, n, tot.hi + tot.lo, [&](int64_t j) { return f64_from_key(sk[j]); });
            if (n >= 100) ++ge100;
        }
        __syncthreads();  // LDS is reused by the next segment
    }
    if (tid == 0 && ge100) atomic_add_i64(a.d_ge100, ge100);
}

// The mid and 1025-2048 lists by ONE WAVE per segment, no workgroup barrier: the segment's keys
// in registers (32 per lane), a value-bucket histogram in the wave's own LDS slice, the bucket starts
// by one wave scan, each wanted rank's bucket found by a binary search (one lane per rank) and
// ranked by the wave - a bucket of more than 64 values is narrowed by re-histogramming its key
// interval (as k_qs_block).  Eight independent waves per workgroup, up to four workgroups per CU:
// sessions overlap their latencies instead of queueing behind each other's barriers (k_qs_block
// held a 256-thread workgroup through ~10 barrier rounds per session).
constexpr int kQsWaveBlock = 512, kQsWaveNB = 1024;
// waves per SIMD the register budget allows: 2 (a 4-wave budget of 128 VGPRs spilled 100 / 316 B
// per lane in the 1024- / 2048-value classes)
template <int MAXN>
struct QsWaveWpe {
    static constexpr int v = 2;
};
__device__ __forceinline__ void qs_wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
template <int MAXN>
__global__ __launch_bounds__(kQsWaveBlock) __attribute__((amdgpu_waves_per_eu(QsWaveWpe<MAXN>::v, QsWaveWpe<MAXN>::v))) void k_qs_wave(const double *__restrict__ src,
                                                          const int64_t *__restrict__ offs,
                                                          const int32_t *__restrict__ list_a,
                                                          const int64_t *__restrict__ d_na,
                                                          const int32_t *__restrict__ list_b,
                                                          const int64_t *__restrict__ d_nb, QsArgs a) {
    constexpr int IPT = MAXN / kWave, WPB = kQsWaveBlock / kWave, NBW = kQsWaveNB, BPL = NBW / kWave;
    static_assert(MAXN % kWave == 0 && NBW % kWave == 0, "qs wave shape");
    __shared__ uint32_t s_cnt[WPB][NBW + 1];
    __shared__ uint64_t s_list[WPB][64];
    __shared__ uint32_t s_fill[WPB];
    const int w = wave_id(), lane = lane_id();
    uint32_t *const cnt = s_cnt[w];
    uint64_t *const lst = s_list[w];
    const int64_t na = *d_na, ntot = na + (d_nb ? *d_nb : 0);
    const int nt = 2 + 2 * a.nq;
    int64_t ge100 = 0;
    for (int64_t it = int64_t(blockIdx.x) * WPB + w; it < ntot; it += int64_t(gridDim.x) * WPB) {
        const int64_t s = it < na ? list_a[it] : list_b[it - na];
        const int64_t b = offs[s];
        const int n = int(offs[s + 1] - b);
        uint64_t K[IPT];
        DD acc{0.0, 0.0};
        uint64_t lo = ~0ull, hi = 0ull;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = lane + m * kWave;
            const double x = i < n ? src[b + i] : 0.0;
            K[m] = i < n ? f64_key(x) : ~0ull;
            if (i < n) {
                acc = dd_add_d(acc, x);
                lo = K[m] < lo ? K[m] : lo;
                hi = K[m] > hi ? K[m] : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        acc = wave_dd_sum(acc);
        uint64_t mine = lo;  // lane t < nt: the key of target t
        if (lo != hi) {
            const int nbk = n < NBW ? n : NBW;
            const double vlo = f64_from_key(lo), vhi = f64_from_key(hi);
            const bool vlin = isfinite(vlo) && isfinite(vhi) && isfinite(vhi - vlo) && vhi > vlo;
            const double vsc = vlin ? double(nbk) / (vhi - vlo) : 0.0;
            const double ksc = double(nbk) / (double(hi - lo) + 1.0);
            auto kbucket = [](uint64_t key, uint64_t klo, double sc, int nb) -> uint32_t {
                const uint32_t q = uint32_t(double(key - klo) * sc);
                return q < uint32_t(nb) ? q : uint32_t(nb - 1);
            };
            // the first level linear in VALUE when the range is finite, else in key (as k_qs_block)
            auto bucket1 = [&](uint64_t key) -> uint32_t {
                if (!vlin) return kbucket(key, lo, ksc, nbk);
                const double q = (f64_from_key(key) - vlo) * vsc;
                return q < double(nbk - 1) ? uint32_t(q) : uint32_t(nbk - 1);
            };
            for (int j = lane; j <= nbk; j += kWave) cnt[j] = 0u;
            qs_wave_sync();
#pragma unroll
            for (int m = 0; m < IPT; ++m)
                if (lane + m * kWave < n) atomicAdd(&cnt[bucket1(K[m])], 1u);
            qs_wave_sync();
            // bucket starts: lane l owns buckets [l * BPL, l * BPL + BPL)
            auto wave_starts = [&](int nb) {
                uint32_t cb[BPL], sum = 0;
#pragma unroll
                for (int e = 0; e < BPL; ++e) {
                    const int j = lane * BPL + e;
                    cb[e] = j < nb ? cnt[j] : 0u;
                    sum += cb[e];
                }
                uint32_t run = wave_incl_scan(sum) - sum;
                qs_wave_sync();
#pragma unroll
                for (int e = 0; e < BPL; ++e) {
                    const int j = lane * BPL + e;
                    if (j < nb) cnt[j] = run;
                    run += cb[e];
                }
            };
            wave_starts(nbk);
            if (lane == 0) cnt[nbk] = uint32_t(n);
            qs_wave_sync();
            int tb = 0;
            uint32_t toff = 0, tsz = 0;
            if (lane < nt) {  // target `lane`'s bucket: the last start <= its rank
                const uint32_t r = uint32_t(qs_rank(n, a, lane));
                int l0 = 0, h0 = nbk - 1;
                while (l0 < h0) {
                    const int mid = (l0 + h0 + 1) >> 1;
                    if (cnt[mid] <= r) l0 = mid;
                    else h0 = mid - 1;
                }
                tb = l0;
                toff = r - cnt[l0];
                tsz = cnt[l0 + 1] - cnt[l0];
            }
            // rank `off` among the (<= 64) keys of the list: the wave's answer
            auto rank_in_list = [&](int sz, uint32_t off) -> uint64_t {
                const uint64_t e = lane < sz ? lst[lane] : ~0ull;
                int rk = 0;
                for (int j = 0; j < sz; ++j) {
                    const uint64_t o = lst[j];
                    rk += (o < e) || (o == e && j < lane);
                }
                const uint64_t hit = __ballot(lane < sz && rk == int(off));
                return __shfl(e, hit ? __ffsll((long long)hit) - 1 : 0, 64);
            };
            int listed = -1;  // the first-level bucket the list holds
            for (int t = 0; t < nt; ++t) {
                const int bt = __shfl(tb, t, 64);
                const uint32_t off = __shfl(toff, t, 64), sz = __shfl(tsz, t, 64);
                uint64_t val;
                if (sz <= 64) {
                    if (bt != listed) {
                        if (lane == 0) s_fill[w] = 0u;
                        qs_wave_sync();
#pragma unroll
                        for (int m = 0; m < IPT; ++m)
                            if (lane + m * kWave < n && bucket1(K[m]) == uint32_t(bt))
                                lst[atomicAdd(&s_fill[w], 1u)] = K[m];
                        qs_wave_sync();
                        listed = bt;
                    }
                    val = rank_in_list(int(sz), off);
                } else {
                    // narrow the bucket's key interval until it holds <= 64 keys or one key
                    listed = -1;
                    uint64_t rlo = ~0ull, rhi = 0ull;
#pragma unroll
                    for (int m = 0; m < IPT; ++m)
                        if (lane + m * kWave < n && bucket1(K[m]) == uint32_t(bt)) {
                            rlo = K[m] < rlo ? K[m] : rlo;
                            rhi = K[m] > rhi ? K[m] : rhi;
                        }
                    rlo = wave_min(rlo);
                    rhi = wave_max(rhi);
                    uint32_t r = off, cntv = sz;
                    while (rlo != rhi && cntv > 64u) {
                        const int nb2 = cntv < uint32_t(NBW) ? int(cntv) : NBW;
                        const double sc2 = double(nb2) / (double(rhi - rlo) + 1.0);
                        qs_wave_sync();
                        for (int j = lane; j <= nb2; j += kWave) cnt[j] = 0u;
                        qs_wave_sync();
#pragma unroll
                        for (int m = 0; m < IPT; ++m)
                            if (lane + m * kWave < n && K[m] >= rlo && K[m] <= rhi)
                                atomicAdd(&cnt[kbucket(K[m], rlo, sc2, nb2)], 1u);
                        qs_wave_sync();
                        // the sub-bucket holding rank r: the lane whose run covers r walks it
                        uint32_t cb[BPL], sum = 0;
#pragma unroll
                        for (int e = 0; e < BPL; ++e) {
                            const int j = lane * BPL + e;
                            cb[e] = j < nb2 ? cnt[j] : 0u;
                            sum += cb[e];
                        }
                        const uint32_t run = wave_incl_scan(sum) - sum;
                        int sb = -1;
                        uint32_t nr = 0, nc = 0;
                        if (r >= run && r < run + sum) {
                            uint32_t before = run;
#pragma unroll
                            for (int e = 0; e < BPL; ++e) {
                                if (sb < 0 && r >= before && r < before + cb[e]) {
                                    sb = lane * BPL + e;
                                    nr = r - before;
                                    nc = cb[e];
                                }
                                before += cb[e];
                            }
                        }
                        const uint64_t who = __ballot(sb >= 0);
                        const int src_lane = __ffsll((long long)who) - 1;
                        sb = __shfl(sb, src_lane, 64);
                        r = __shfl(nr, src_lane, 64);
                        cntv = __shfl(nc, src_lane, 64);
                        uint64_t nlo = ~0ull, nhi = 0ull;
#pragma unroll
                        for (int m = 0; m < IPT; ++m)
                            if (lane + m * kWave < n && K[m] >= rlo && K[m] <= rhi &&
                                kbucket(K[m], rlo, sc2, nb2) == uint32_t(sb)) {
                                nlo = K[m] < nlo ? K[m] : nlo;
                                nhi = K[m] > nhi ? K[m] : nhi;
                            }
                        rlo = wave_min(nlo);
                        rhi = wave_max(nhi);
                    }
                    if (rlo == rhi) {
                        val = rlo;
                    } else {  // <= 64 keys in [rlo, rhi]
                        qs_wave_sync();
                        if (lane == 0) s_fill[w] = 0u;
                        qs_wave_sync();
#pragma unroll
                        for (int m = 0; m < IPT; ++m)
                            if (lane + m * kWave < n && K[m] >= rlo && K[m] <= rhi)
                                lst[atomicAdd(&s_fill[w], 1u)] = K[m];
                        qs_wave_sync();
                        val = rank_in_list(int(cntv), r);
                    }
                }
                if (lane == t) mine = val;
            }
            qs_wave_sync();  // (the next segment reuses the LDS slice)
        }
        // the targets' keys through the wave's list slice (lane t -> slot t), lane 0 writes
        qs_wave_sync();
        if (lane < nt) lst[lane] = mine;
        qs_wave_sync();
        if (lane == 0) {
            auto get = [&](int64_t j) {
                uint64_t r = lst[0];
                for (int t = 0; t < nt; ++t)
                    if (qs_rank(n, a, t) == j) r = lst[t];
                return f64_from_key(r);
            };
            qs_write(a, s, n, acc.hi + acc.lo, get);
            if (n >= 100) ++ge100;
        }
        qs_wave_sync();
    }
    if (lane == 0 && ge100) atomic_add_i64(a.d_ge100, ge100);
}

bool seg_qstats_ok(const Segs &sg) { return sg.len_bound() <= kQsMax; }
#ifndef FZ_QS_BIG_BLOCK
#define FZ_QS_BIG_BLOCK 512
#endif
constexpr int kQsBigBlock = FZ_QS_BIG_BLOCK;  // threads of the 2049 .. kQsMax class
#ifndef FZ_QS_WAVE
#define FZ_QS_WAVE 1  // the 65-2048 classes one wave per segment (0: k_qs_sort_mid / k_qs_block<256, 2048>)
#endif
constexpr bool kQsWave = FZ_QS_WAVE;

void seg_qstats(fz_ctx *c, const double *vals, const Segs &sg, const double *q_host, int nq, double *mean,
                double *median, double *pcts, int64_t *d_ge100, double *mean2) {
    FZ_CHECK(nq >= 0 && nq <= 8, "seg_qstats: at most 8 percentiles");
    FZ_CHECK(seg_qstats_ok(sg), "seg_qstats: segment longer than kQsMax");
    QsArgs a{};
    for (int j = 0; j < nq; ++j) a.q[j] = q_host[j];
    a.nq = nq;
    a.mean = mean;
    a.mean2 = mean2;
    a.median = median;
    a.pcts = pcts;
    a.d_ge100 = d_ge100;
    const int64_t S = sg.S, lb = sg.len_bound();
    if (S <= 0) return;
    // algorithmic bytes: the values once (8 B each) + the offsets + the statistics written
    ProbeScope ps(c, "seg_qstats", double(S) * (8.0 + 8.0 * (2 + nq)), sg.offs + S, 8.0);
    // class lists (capacities: a segment of the class holds more than the class below allows)
    auto cap = [&](int64_t minlen) { return S < sg.n_cap / (minlen + 1) + 1 ? S : sg.n_cap / (minlen + 1) + 1; };
    const int64_t caps[kQsLists] = {lb > 32 ? cap(32) : 0, lb > kTinySeg ? cap(kTinySeg) : 0,
                                    lb > 2048 ? cap(2048) : 0, lb > 1024 ? cap(1024) : 0, cap(kMicroSeg),
                                    lb > 16 ? cap(16) : 0};
    QsLists L;
    L.d_n = c->arena.get<int64_t>(kQsLists);
    for (int k = 0; k < kQsLists; ++k) L.ids[k] = c->arena.get<int32_t>(caps[k]);
    dev_fill(c, L.d_n, 0, kQsLists * 8);
    const int64_t groups = (S + 63) / 64;
    k_qs_micro<<<grid_for(groups, kBlock / kWave, 8192), kBlock, 0, c->stream>>>(vals, sg.offs, S, a, L);
    FZ_LAUNCH_CHECK();
    auto grid = [](int64_t n, int64_t lim) { return unsigned(n < 1 ? 1 : (n < lim ? n : lim)); };
    if (lb > kMicroSeg) {
        k_qs_tiny<16><<<grid((caps[kQsTiny16] + 15) / 16, 8192), kBlock, 0, c->stream>>>(
            vals, sg.offs, L.ids[kQsTiny16], L.d_n + kQsTiny16, a);
        FZ_LAUNCH_CHECK();
    }
    if (lb > 16) {
        k_qs_tiny<32><<<grid((caps[kQsTiny32] + 7) / 8, 8192), kBlock, 0, c->stream>>>(
            vals, sg.offs, L.ids[kQsTiny32], L.d_n + kQsTiny32, a);
        FZ_LAUNCH_CHECK();
    }
    if (lb > 32) {
        k_qs_tiny<64><<<grid((caps[kQsTiny] + 3) / 4, 8192), kBlock, 0, c->stream>>>(vals, sg.offs, L.ids[kQsTiny],
                                                                                      L.d_n + kQsTiny, a);
        FZ_LAUNCH_CHECK();
    }
    if (lb > kTinySeg) {
        // (the mid list stays with the LDS bitonic sort: one wave per session measured 141 vs 67 us
        // per step at config 2's ~3,000 sessions of <= 1,000 values, serial probe)
        k_qs_sort_mid<<<grid(caps[1], 8192), 256, 0, c->stream>>>(vals, sg.offs, L.ids[1], L.d_n + 1, a);
        FZ_LAUNCH_CHECK();
    }
    if (kQsWave && lb > 1024) {
        // the 1025-2048 list one wave per segment (32 keys per lane)
        constexpr int wpb = kQsWaveBlock / kWave;
        k_qs_wave<2048><<<grid((caps[3] + wpb - 1) / wpb, 4096), kQsWaveBlock, 0, c->stream>>>(
            vals, sg.offs, L.ids[3], L.d_n + 3, nullptr, nullptr, a);
        FZ_LAUNCH_CHECK();
    }
    if (!kQsWave && lb > 1024) {
        // 1025 - 2048 values (a session of config 3's one-per-project values: 1,250 at an eighth of
        // the table): 256-thread workgroups with 8 values per thread - several per CU in flight, where
        // the 1024-thread class held one workgroup per CU with 15 of its 16 value slots per thread idle
        k_qs_block<256, 2048><<<grid(caps[3], 8192), 256, 0, c->stream>>>(vals, sg.offs, L.ids[3], L.d_n + 3, a);
        FZ_LAUNCH_CHECK();
    }
    if (lb > 2048) {
        // (512 threads, keys in LDS: 203 VGPRs and no scratch; at 1024 threads the kernel spilled 17-31
        // VGPRs per lane, keys in registers or in LDS)
        k_qs_block<kQsBigBlock, kQsMax><<<grid(caps[2], 1024), kQsBigBlock, 0, c->stream>>>(vals, sg.offs, L.ids[2],
                                                                                           L.d_n + 2, a);
        FZ_LAUNCH_CHECK();
    }
}

// levene([x, y], center='median') (scipy _morestats.py levene), the two medians given on the
// device (medx / medy: e.g. fields of fz_describe results)
// levene([x, y], center='median') (scipy _morestats.py levene) from zb = the mean absolute
// deviations from each median, dv = the sums of their squared deviations from zb -> out = W, p
__device__ inline void levene_finish(const double *zb, const double *dv, double nx, double ny, double *out) {
    const double N = nx + ny;
    double zbar = 0.0;
    zbar += zb[0] * nx;
    zbar += zb[1] * ny;
    zbar /= N;
    const double numer = (N - 2.0) * (nx * (zb[0] - zbar) * (zb[0] - zbar) + ny * (zb[1] - zbar) * (zb[1] - zbar));
    double dvar = 0.0;
    dvar += dv[0];
    dvar += dv[1];
    const double W = numer / (1.0 * dvar);
    out[0] = W;
    out[1] = stats::f1_sf(W, N - 2.0);
}

void levene_two_med(fz_ctx *c, const double *medx, const double *x, int64_t nxm, const int64_t *d_nx,
                    const double *medy, const double *y, int64_t nym, const int64_t *d_ny, double *out) {
    double *med = c->arena.get<double>(2);
    int64_t *ox = c->arena.get<int64_t>(2), *oy = c->arena.get<int64_t>(2);  // each sample's one segment
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        ox[0] = 0;
        ox[1] = *d_nx;
        oy[0] = 0;
        oy[1] = *d_ny;
        med[0] = *medx;
        med[1] = *medy;
    });
    double *zb = c->arena.get<double>(2), *dv = c->arena.get<double>(2);
    Segs sx{1, ox, nxm}, sy{1, oy, nym};
    ChunkedSegs cx = chunked(c, sx), cy = chunked(c, sy);
    seg_reduce<1>(c, cx, [=] __device__(int64_t i, int32_t, double *v) { v[0] = fabs(x[i] - med[0]); }, zb);
    seg_reduce<1>(c, cy, [=] __device__(int64_t i, int32_t, double *v) { v[0] = fabs(y[i] - med[1]); }, zb + 1);
    map_n(c, 1, nullptr, [=] __device__(int64_t) {
        zb[0] /= double(*d_nx);
        zb[1] /= double(*d_ny);
    });
    seg_reduce<1>(c, cx, [=] __device__(int64_t i, int32_t, double *v) {
        const double d = fabs(x[i] - med[0]) - zb[0];
        v[0] = d * d;
    }, dv);
    seg_reduce<1>(c, cy, [=] __device__(int64_t i, int32_t, double *v) {
        const double d = fabs(y[i] - med[1]) - zb[1];
        v[0] = d * d;
    }, dv + 1);
    map_n(c, 1, nullptr, [=] __device__(int64_t) { levene_finish(zb, dv, double(*d_nx), double(*d_ny), out); });
}

// ------------------------------------------------- two small samples: every test in one workgroup
// mannwhitneyu, brunnermunzel (union ranks), Cliff's delta and levene(center='median') of x[0, *d_nx)
// and y[0, *d_ny), each of at most kTwoSmall values: both samples sorted in LDS (one bitonic network
// over the two halves), a value's union rank / within-sample rank / tie group from binary searches in
// the two sorted halves, the medians read off them, every sum double-double as on the multi-launch
// path (seg_rank_tests_sorted, levene_two_med), the same finishing formulas.  One launch instead of
// about 25.
constexpr int kTwoSmall = 4096;
constexpr int kTwoBlock = 512;
template <int NV>
__device__ inline void block_dd_sums16(const DD (&acc)[NV], double (*s_hi)[NV], double (*s_lo)[NV], double (&out)[NV]) {
    constexpr int NW = kTwoBlock / kWave;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const DD r = wave_dd_sum(acc[v]);
        if (lane_id() == 0) {
            s_hi[wave_id()][v] = r.hi;
            s_lo[wave_id()][v] = r.lo;
        }
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        DD t{s_hi[0][v], s_lo[0][v]};
        for (int w = 1; w < NW; ++w) t = dd_add(t, DD{s_hi[w][v], s_lo[w][v]});
        out[v] = t.hi + t.lo;
    }
    __syncthreads();
}
__device__ inline int lb_lds(const double *a, int lo, int hi, double v) {
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}
__device__ inline int ub_lds(const double *a, int lo, int hi, double v) {
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (a[m] <= v) lo = m + 1;
        else hi = m;
    }
    return lo;
}
struct TwoSmallOut {
    double *mwu_p_two, *bm_stat, *bm_p, *cliff, *levene;  // levene: W, p
    double *exact_scratch;                              // 8 * kTwoSmall + 1 doubles
};
__global__ __launch_bounds__(kTwoBlock) void k_two_sample_small(const double *__restrict__ xin,
                                                               const int64_t *__restrict__ d_nx,
                                                               const double *__restrict__ yin,
                                                               const int64_t *__restrict__ d_ny, TwoSmallOut o) {
    chain_prio();
    constexpr int NW = kTwoBlock / kWave;
    __shared__ uint64_t sk[2 * kTwoSmall];  // x's keys in [0, np2), y's in [np2, 2 np2); then the values
    __shared__ double s_hi[NW][6], s_lo[NW][6];
    const int tid = threadIdx.x;
    const int nx = int(*d_nx), ny = int(*d_ny);
    int np2 = 1;
    while (np2 < (nx > ny ? nx : ny)) np2 <<= 1;
    for (int i = tid; i < np2; i += kTwoBlock) {
        sk[i] = i < nx ? f64_key(xin[i]) : ~0ull;
        sk[np2 + i] = i < ny ? f64_key(yin[i]) : ~0ull;
    }
    __syncthreads();
    // one bitonic network of np2 entries on both halves at once (pair q of half q / (np2 / 2))
    const int hp = np2 >> 1;
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < np2; t += kTwoBlock) {
                const int h = t >= hp ? 1 : 0, q = t - h * hp;
                const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), ixj = i + j;
                uint64_t *a = sk + h * np2;
                const uint64_t u = a[i], d = a[ixj];
                if ((u > d) == ((i & k) == 0)) {
                    a[i] = d;
                    a[ixj] = u;
                }
            }
            __syncthreads();
        }
    }
    // keys -> values in place (as doubles)
    double *xs = reinterpret_cast<double *>(sk), *ys = reinterpret_cast<double *>(sk + np2);
    for (int i = tid; i < np2; i += kTwoBlock) {
        xs[i] = f64_from_key(sk[i]);
        ys[i] = f64_from_key(sk[np2 + i]);
    }
    __syncthreads();
    const double Nx = double(nx), Ny = double(ny);
    // pass 1: union rank sums, tie term (each union tie group once: at its first x value, or at its
    // first y value when it holds no x)
    DD a1[6] = {};
    auto group = [&](const double *a, int na, const double *b, int nb, int i, int &la, int &ua, int &lb, int &ub) {
        const double v = a[i];
        la = lb_lds(a, 0, i + 1, v);
        ua = ub_lds(a, i, na, v);
        lb = lb_lds(b, 0, nb, v);
        ub = ub_lds(b, lb, nb, v);
    };
    for (int i = tid; i < nx + ny; i += kTwoBlock) {
        const bool isx = i < nx;
        const int k = isx ? i : i - nx;
        int la, ua, lb, ub;
        if (isx) group(xs, nx, ys, ny, k, la, ua, lb, ub);
        else group(ys, ny, xs, nx, k, la, ua, lb, ub);
        const double rc = double(la + lb + ua + ub + 1) / 2.0;
        if (isx) a1[0] = dd_add_d(a1[0], rc);
        else a1[1] = dd_add_d(a1[1], rc);
        if (k == la && (isx || ub == lb)) {  // t^3 - t, int64-exact, in two exactly representable halves
            const int64_t t = int64_t(ua - la) + int64_t(ub - lb), tt = t * t * t - t;
            a1[4] = dd_add_d(a1[4], double(tt & ~int64_t((1 << 26) - 1)));
            a1[5] = dd_add_d(a1[5], double(tt & int64_t((1 << 26) - 1)));
        }
    }
    double s1[6];
    block_dd_sums16<6>(a1, s_hi, s_lo, s1);
    s1[2] = Nx;
    s1[3] = Ny;
    // pass 2: squared deviations of (union rank - within-sample rank) from their means
    DD a2[2] = {};
    const double cmx = s1[0] / Nx, cmy = s1[1] / Ny, wmx = (Nx + 1.0) / 2.0, wmy = (Ny + 1.0) / 2.0;
    for (int i = tid; i < nx + ny; i += kTwoBlock) {
        const bool isx = i < nx;
        const int k = isx ? i : i - nx;
        int la, ua, lb, ub;
        if (isx) group(xs, nx, ys, ny, k, la, ua, lb, ub);
        else group(ys, ny, xs, nx, k, la, ua, lb, ub);
        const double rc = double(la + lb + ua + ub + 1) / 2.0;
        const double rw = double(la) + double(ua - la + 1) / 2.0;
        const double d = ((rc - rw) - (isx ? cmx : cmy)) + (isx ? wmx : wmy);
        if (isx) a2[0] = dd_add_d(a2[0], d * d);
        else a2[1] = dd_add_d(a2[1], d * d);
    }
    double s2[2];
    block_dd_sums16<2>(a2, reinterpret_cast<double(*)[2]>(s_hi), reinterpret_cast<double(*)[2]>(s_lo), s2);
    // levene: medians, mean absolute deviations, their squared deviations
    const double medx = nx <= 0 ? NAN : ((nx & 1) ? xs[nx / 2] : (xs[nx / 2 - 1] + xs[nx / 2]) / 2.0);
    const double medy = ny <= 0 ? NAN : ((ny & 1) ? ys[ny / 2] : (ys[ny / 2 - 1] + ys[ny / 2]) / 2.0);
    DD a3[2] = {};
    for (int i = tid; i < nx; i += kTwoBlock) a3[0] = dd_add_d(a3[0], fabs(xs[i] - medx));
    for (int i = tid; i < ny; i += kTwoBlock) a3[1] = dd_add_d(a3[1], fabs(ys[i] - medy));
    double zb[2];
    block_dd_sums16<2>(a3, reinterpret_cast<double(*)[2]>(s_hi), reinterpret_cast<double(*)[2]>(s_lo), zb);
    zb[0] /= Nx;
    zb[1] /= Ny;
    DD a4[2] = {};
    for (int i = tid; i < nx; i += kTwoBlock) {
        const double d = fabs(xs[i] - medx) - zb[0];
        a4[0] = dd_add_d(a4[0], d * d);
    }
    for (int i = tid; i < ny; i += kTwoBlock) {
        const double d = fabs(ys[i] - medy) - zb[1];
        a4[1] = dd_add_d(a4[1], d * d);
    }
    double dv[2];
    block_dd_sums16<2>(a4, reinterpret_cast<double(*)[2]>(s_hi), reinterpret_cast<double(*)[2]>(s_lo), dv);
    if (tid != 0) return;
    double u1 = 0.0;
    RankTestOut ro;
    ro.mwu_p_two = o.mwu_p_two;
    ro.u1 = &u1;
    ro.bm_stat = o.bm_stat;
    ro.bm_p = o.bm_p;
    ro.exact_scratch = o.exact_scratch;
    rank_tests_finish(s1, s2, true, ro, 0);
    *o.cliff = (2.0 * u1) / (Nx * Ny) - 1.0;
    levene_finish(zb, dv, Nx, Ny, o.levene);
}

bool two_sample_small_ok(int64_t nx_cap, int64_t ny_cap) { return nx_cap <= kTwoSmall && ny_cap <= kTwoSmall; }

void two_sample_small(fz_ctx *c, const double *x, const int64_t *d_nx, const double *y, const int64_t *d_ny,
                      double *mwu_p_two, double *bm_stat, double *bm_p, double *cliff, double *levene) {
    TwoSmallOut o{mwu_p_two, bm_stat, bm_p, cliff, levene, c->arena.get<double>(8 * kTwoSmall + 1)};
    k_two_sample_small<<<1, kTwoBlock, 0, c->stream>>>(x, d_nx, y, d_ny, o);
    FZ_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------ session exchange
// A session owner receives, from each of R shards, that shard's values of its sessions grouped by
// segment (session, or session x group) - R runs one after another.  The merge interleaves them
// segment by segment: segment s holds run 0's values of s, then run 1's, ... (= global project
// order, the order the single-table path's stable sort gives).  One wave per (run, segment) copies
// its contiguous values: coalesced reads and writes, no sort.
__global__ void k_runs_merge(const double *__restrict__ in, const int64_t *__restrict__ sizes,
                             const int64_t *__restrict__ in_start, const int64_t *__restrict__ out_offs, int64_t R,
                             int64_t S, double *__restrict__ out) {
    const int64_t nw = int64_t(gridDim.x) * (blockDim.x / kWave);
    const int lane = lane_id();
    for (int64_t q = int64_t(blockIdx.x) * (blockDim.x / kWave) + wave_id(); q < R * S; q += nw) {
        const int64_t n = sizes[q];
        if (n == 0) continue;
        const int64_t r = q / S, s = q - r * S;
        int64_t dst = out_offs[s];
        for (int64_t k = 0; k < r; ++k) dst += sizes[k * S + s];
        const int64_t src = in_start[q];
        for (int64_t j = lane; j < n; j += kWave) out[dst + j] = in[src + j];
    }
}

void runs_merge(fz_ctx *c, const double *values, const int64_t *sizes, int64_t R, int64_t S, double *out,
                int64_t *out_offs) {
    int64_t *in_start = c->arena.get<int64_t>(R * S > 0 ? R * S : 1);
    int64_t *tot = c->arena.get<int64_t>(S + 1);
    if (R * S > 0) scan_exclusive_i64(c, sizes, in_start, R * S, nullptr);
    map_n(c, S + 1, nullptr, [=] __device__(int64_t s) {
        int64_t t = 0;
        if (s < S)
            for (int64_t r = 0; r < R; ++r) t += sizes[r * S + s];
        tot[s] = t;
    });
    scan_exclusive_i64(c, tot, out_offs, S + 1, nullptr);
    if (R * S == 0) return;
    const int64_t waves = R * S;
    const int64_t blocks = (waves + kBlock / kWave - 1) / (kBlock / kWave);
    k_runs_merge<<<unsigned(blocks < 16384 ? blocks : 16384), kBlock, 0, c->stream>>>(values, sizes, in_start,
                                                                                     out_offs, R, S, out);
    FZ_LAUNCH_CHECK();
}

}  // namespace fz
