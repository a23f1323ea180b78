// Segmented merge sort for segments longer than one LDS tile (10k-row
// projects and sessions, Zipf giants of ~20M rows).
//
// Segments of <= kTile rows are sorted inside one workgroup by the callers' own LDS kernels.  The
// long ("big") ones go through this engine, which touches only their rows:
//   1. tile map      - every big segment is cut into kTile-row tiles (device-built list);
//   2. tile sort     - one workgroup per tile sorts (key, val) pairs in LDS (bitonic network);
//   3. merge rounds  - round r merges pairs of sorted runs of kTile << r rows inside each segment;
//                      one workgroup per kTile-row OUTPUT chunk finds its two input spans by a
//                      merge-path search, merges them in LDS and writes the chunk coalesced.  A
//                      segment leaves the engine in round ceil(log2(tiles)) - 1 through the caller's
//                      sink (its final layout), earlier rounds ping-pong two scratch buffers.
// Order: lexicographic on (key, val) with val = the row's input position, so the result is a
// total order and STABLE (equal keys keep input order) - what the store's ORDER BY time needs.
// Traffic per big row: 12 B read + 12 B written per round plus the key generation and the sink,
// against 16-24 B x 8-10 full-table passes of the LSD radix sort it replaces.
#pragma once

#include "fz_device.h"
#include "fz_internal.h"

namespace fz {

constexpr int kTile = 4096;            // rows per tile (= the LDS sort limit of the small kernels)
constexpr int kTileSortBlock = 1024;   // threads of the tile sort (4 pairs per thread per stage)

struct TileMap {
    int64_t cap = 0;           // host bound of the number of tiles
    int64_t *d_n = nullptr;    // device count
    int32_t *seg = nullptr;    // tile -> segment
    int64_t *begin = nullptr;  // tile -> first row
};

// Tiles of the segments with len > kTile, or, when flag is given, of exactly the segments with
// flag[s] != 0 (the ones the callers' bucket sorts left: too long, skewed, or a time span that does
// not fit their key).  n_cap: host bound of offs[S].
TileMap big_tiles(fz_ctx *c, const int64_t *offs, int64_t S, int64_t n_cap, const uint8_t *flag);

__device__ inline bool kv_less(uint64_t ka, uint32_t va, uint64_t kb, uint32_t vb) {
    return ka < kb || (ka == kb && va < vb);
}

// Number of rounds a segment of len rows goes through (0: one tile, the tile sort is final).
__host__ __device__ inline int merge_rounds(int64_t len) {
    int r = 0;
    while ((int64_t(kTile) << r) < len) ++r;
    return r;
}

// Phase 2: sort each tile by (key(i), i).  Single-tile segments go straight to sink(s, q, key, val);
// the others to (ok, ov).
// KeyGen::kBuckets (value keys): a tile is first tried as a BUCKET sort - n + 1 buckets linear in
// the key over the tile's key range, counted with LDS atomics, a row's rank = its bucket's start +
// the rows of its bucket with a smaller (key, position), staged in LDS in sorted order and written
// coalesced; a tile whose largest bucket holds more than kTileSkew rows (ties, clusters) takes the
// bitonic network below.  O(n) instead of the network's 78 stages per 4,096-row tile (config 5L's
// Zipf head: ~18 k tiles per value sort, 2.2 ms of bitonic stages per step).
template <class K>
struct TileBuckets {
    template <class T>
    static constexpr bool has(decltype(T::kBuckets) *) { return T::kBuckets; }
    template <class T>
    static constexpr bool has(...) { return false; }
    static constexpr bool value = has<K>(nullptr);
};
constexpr int kTileSkew = 32;
template <class KeyGen, class Sink>
__global__ __launch_bounds__(kTileSortBlock) void k_tile_sort(TileMap tm, const int64_t *__restrict__ offs, KeyGen key,
                                                              uint64_t *__restrict__ ok, uint32_t *__restrict__ ov,
                                                              Sink sink) {
    constexpr bool BUCKETS = TileBuckets<KeyGen>::value;
    constexpr int IPT = kTile / kTileSortBlock;
    constexpr int NW = kTileSortBlock / kWave;
    __shared__ uint64_t sk[kTile];
    __shared__ uint32_t sv[kTile];
    __shared__ uint32_t s_cnt[BUCKETS ? kTile + 1 : 1];
    __shared__ uint64_t s_lo[NW], s_hi[NW];
    __shared__ uint32_t s_tmp[NW], s_max[NW];
    const int64_t ntiles = *tm.d_n;
    for (int64_t k = blockIdx.x; k < ntiles; k += gridDim.x) {  // persistent grid over the tiles
    const int32_t s = tm.seg[k];
    const int64_t b = tm.begin[k], se = offs[s + 1];
    const int n = int((se - b) < kTile ? (se - b) : kTile);
    const bool single = (offs[s] == b) && (se - b <= kTile);
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    const int tid = threadIdx.x;
    if constexpr (BUCKETS) {
        const int w = wave_id(), lane = lane_id();
        uint64_t kr[IPT];
        uint64_t lo = ~0ull, hi = 0ull;
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * kTileSortBlock;
            kr[m] = i < n ? key(b + i) : ~0ull;
            if (i < n) {
                sk[i] = kr[m];
                lo = kr[m] < lo ? kr[m] : lo;
                hi = kr[m] > hi ? kr[m] : hi;
            }
        }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane == 0) {
            s_lo[w] = lo;
            s_hi[w] = hi;
        }
        for (int j = tid; j <= kTile; j += kTileSortBlock) s_cnt[j] = 0u;
        __syncthreads();
        lo = s_lo[0];
        hi = s_hi[0];
#pragma unroll
        for (int q = 1; q < NW; ++q) {
            lo = s_lo[q] < lo ? s_lo[q] : lo;
            hi = s_hi[q] > hi ? s_hi[q] : hi;
        }
        const double scale = double(n) / (double(hi - lo) + 1.0);
        uint32_t bs[IPT];  // bucket << 16 | slot in the bucket
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const int i = tid + m * kTileSortBlock;
            bs[m] = 0u;
            if (i < n) {
                uint32_t q = uint32_t(double(kr[m] - lo) * scale);
                q = q < uint32_t(n) ? q : uint32_t(n - 1);
                bs[m] = (q << 16) | atomicAdd(&s_cnt[q], 1u);
            }
        }
        __syncthreads();
        // bucket starts: thread t scans buckets [t * IPT, t * IPT + IPT)
        uint32_t sum = 0, mx = 0;
#pragma unroll
        for (int e = 0; e < IPT; ++e) {
            const uint32_t ce = s_cnt[tid * IPT + e];
            sum += ce;
            mx = ce > mx ? ce : mx;
        }
        mx = wave_max(mx);
        if (lane == 0) s_max[w] = mx;
        uint32_t run = block_excl_scan<uint32_t, NW>(sum, s_tmp, (uint32_t *)nullptr);
#pragma unroll
        for (int e = 0; e < IPT; ++e) {
            const uint32_t ce = s_cnt[tid * IPT + e];
            s_cnt[tid * IPT + e] = run;
            run += ce;
        }
        if (tid == 0) s_cnt[kTile] = uint32_t(n);
        __syncthreads();
        uint32_t gmax = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) gmax = s_max[q] > gmax ? s_max[q] : gmax;
        if (gmax <= uint32_t(kTileSkew)) {
            // rows in bucket order (positions), then each row's rank inside its bucket
#pragma unroll
            for (int m = 0; m < IPT; ++m) {
                const int i = tid + m * kTileSortBlock;
                if (i < n) sv[s_cnt[bs[m] >> 16] + (bs[m] & 0xffffu)] = uint32_t(i);
            }
            __syncthreads();
            int dq[IPT];
#pragma unroll
            for (int m = 0; m < IPT; ++m) {
                const int i = tid + m * kTileSortBlock;
                dq[m] = -1;
                if (i >= n) continue;
                const uint32_t st = s_cnt[bs[m] >> 16], en = s_cnt[(bs[m] >> 16) + 1];
                uint32_t rank = 0;
                for (uint32_t x = st; en - st > 1 && x < en; ++x) {
                    const int ox = int(sv[x]);
                    if (ox == i) continue;
                    const uint64_t kx = sk[ox];
                    rank += (kx < kr[m]) || (kx == kr[m] && ox < i);
                }
                dq[m] = int(st + rank);
            }
            __syncthreads();  // the ranking's reads of sk / sv are done: stage in sorted order
#pragma unroll
            for (int m = 0; m < IPT; ++m) {
                if (dq[m] < 0) continue;
                sk[dq[m]] = kr[m];
                sv[dq[m]] = uint32_t(b + tid + m * kTileSortBlock);
            }
            __syncthreads();
            for (int i = tid; i < n; i += kTileSortBlock) {
                if (single) {
                    sink(s, b + i, sk[i], sv[i]);
                } else {
                    ok[b + i] = sk[i];
                    ov[b + i] = sv[i];
                }
            }
            __syncthreads();
            continue;
        }
        // (skewed: the network, from the keys already in LDS)
    }
    for (int i = tid; i < np2; i += kTileSortBlock) {
        if (i < n) {
            sk[i] = key(b + i);
            sv[i] = uint32_t(b + i);
        } else {
            sk[i] = ~0ull;
            sv[i] = ~0u;
        }
    }
    __syncthreads();
    for (int kk = 2; kk <= np2; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < (np2 >> 1); t += kTileSortBlock) {
                const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ixj = i + j;
                const uint64_t ka = sk[i], kb = sk[ixj];
                const uint32_t va = sv[i], vb = sv[ixj];
                if (kv_less(kb, vb, ka, va) == ((i & kk) == 0)) {
                    sk[i] = kb;
                    sk[ixj] = ka;
                    sv[i] = vb;
                    sv[ixj] = va;
                }
            }
            bitonic_stage_sync(kk, j, np2);
        }
    }
    for (int i = tid; i < n; i += kTileSortBlock) {
        if (single) {
            sink(s, b + i, sk[i], sv[i]);
        } else {
            ok[b + i] = sk[i];
            ov[b + i] = sv[i];
        }
    }
    __syncthreads();
    }
}

// Phase 3, round r: output chunk = tile k's row range; runs of L = kTile << r rows.
struct MergeChunk {
    bool active, final;
    int64_t b, e, a0, a1, b1, d0, d1;  // output [b, e); pair A = [a0, a1), B = [a1, b1); diagonals
};
__device__ inline MergeChunk merge_chunk(const TileMap &tm, const int64_t *offs, int r, int64_t k, int32_t &s) {
    MergeChunk m;
    s = tm.seg[k];
    const int64_t sb = offs[s], se = offs[s + 1], len = se - sb;
    const int64_t L = int64_t(kTile) << r;
    m.active = L < len;  // else the segment finished in an earlier round
    m.final = 2 * L >= len;
    m.b = tm.begin[k];
    m.e = (m.b + kTile < se) ? m.b + kTile : se;
    const int64_t ps = sb + ((m.b - sb) / (2 * L)) * (2 * L);
    m.a0 = ps;
    m.a1 = ps + L < se ? ps + L : se;
    m.b1 = ps + 2 * L < se ? ps + 2 * L : se;
    m.d0 = m.b - ps;
    m.d1 = m.e - ps;
    return m;
}

// Merge-path split of every chunk's start diagonal for round r (fz_segsort.hip).
void merge_splits(fz_ctx *c, const TileMap &tm, const int64_t *offs, int r, const uint64_t *ik, const uint32_t *iv,
                  int64_t *split);

constexpr int kMergeThreads = 512;
constexpr int kMergeIt = kTile / kMergeThreads;  // outputs per thread

template <class Sink>
__global__ __launch_bounds__(kMergeThreads) void k_merge_round(TileMap tm, const int64_t *__restrict__ offs, int r,
                                                               const int64_t *__restrict__ split,
                                                               const uint64_t *__restrict__ ik,
                                                               const uint32_t *__restrict__ iv, uint64_t *__restrict__ ok,
                                                               uint32_t *__restrict__ ov, Sink sink) {
    __shared__ uint64_t sk[kTile];
    __shared__ uint32_t sv[kTile];
    const int64_t ntiles = *tm.d_n;
    const int tid = threadIdx.x;
    for (int64_t k = blockIdx.x; k < ntiles; k += gridDim.x) {  // persistent grid over the chunks
        int32_t s;
        const MergeChunk m = merge_chunk(tm, offs, r, k, s);
        if (!m.active) continue;
        // the chunk's A rows are [ia0, ia1) of A, its B rows [d0 - ia0, d1 - ia1) of B; the end split
        // is the next chunk's start split, or all of A at the end of the pair
        const int64_t ia0 = split[k], ia1 = m.e == m.b1 ? m.a1 - m.a0 : split[k + 1];
        const int64_t ib0 = m.d0 - ia0, ib1 = m.d1 - ia1;
        const int nal = int(ia1 - ia0), cnt = nal + int(ib1 - ib0);
        for (int i = tid; i < cnt; i += kMergeThreads) {
            const int64_t src = i < nal ? m.a0 + ia0 + i : m.a1 + ib0 + (i - nal);
            sk[i] = ik[src];
            sv[i] = iv[src];
        }
        __syncthreads();
        // each thread merges kMergeIt consecutive outputs from its own split (binary search in LDS);
        // the two candidate heads stay in registers, (~0, ~0) marks an exhausted side
        uint64_t rk[kMergeIt];
        uint32_t rv[kMergeIt];
        const int d = tid * kMergeIt;
        if (d < cnt) {
            const int nbl = cnt - nal;
            int lo = d - nbl > 0 ? d - nbl : 0, hi = d < nal ? d : nal;
            while (lo < hi) {
                const int q = (lo + hi) >> 1;
                const int jb = nal + (d - 1 - q);
                if (kv_less(sk[q], sv[q], sk[jb], sv[jb]))
                    lo = q + 1;
                else
                    hi = q;
            }
            int ia = lo, ib = nal + (d - lo);
            uint64_t ka = ia < nal ? sk[ia] : ~0ull, kb = ib < cnt ? sk[ib] : ~0ull;
            uint32_t va = ia < nal ? sv[ia] : ~0u, vb = ib < cnt ? sv[ib] : ~0u;
#pragma unroll
            for (int q = 0; q < kMergeIt; ++q) {
                const bool ta = kv_less(ka, va, kb, vb);
                rk[q] = ta ? ka : kb;
                rv[q] = ta ? va : vb;
                if (ta) {
                    ++ia;
                    ka = ia < nal ? sk[ia] : ~0ull;
                    va = ia < nal ? sv[ia] : ~0u;
                } else {
                    ++ib;
                    kb = ib < cnt ? sk[ib] : ~0ull;
                    vb = ib < cnt ? sv[ib] : ~0u;
                }
            }
        }
        __syncthreads();
        if (d < cnt) {
#pragma unroll
            for (int q = 0; q < kMergeIt; ++q) {
                if (d + q < cnt) {
                    sk[d + q] = rk[q];
                    sv[d + q] = rv[q];
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < cnt; i += kMergeThreads) {
            if (m.final) {
                sink(s, m.b + i, sk[i], sv[i]);
            } else {
                ok[m.b + i] = sk[i];
                ov[m.b + i] = sv[i];
            }
        }
        __syncthreads();
    }
}

// Sort the big segments of [offs, S): key(i) for input row i, result delivered to sink(s, q, key, i)
// for every output row q of every big segment.  max_len: host bound of the longest big segment
// (sets the number of merge rounds).  n_cap: host bound of offs[S].
template <class KeyGen, class Sink>
void sort_big_segments(fz_ctx *c, const int64_t *offs, int64_t S, int64_t n_cap, int64_t max_len, const uint8_t *flag,
                       KeyGen key, Sink sink) {
    if (S <= 0 || n_cap <= 0) return;
    const TileMap tm = big_tiles(c, offs, S, n_cap, flag);
    if (tm.cap <= 0) return;
    uint64_t *k0 = c->arena.get<uint64_t>(n_cap);
    uint32_t *v0 = c->arena.get<uint32_t>(n_cap);
    const int R = merge_rounds(max_len);
    uint64_t *k1 = R > 1 ? c->arena.get<uint64_t>(n_cap) : nullptr;
    uint32_t *v1 = R > 1 ? c->arena.get<uint32_t>(n_cap) : nullptr;
    // persistent grids: a few resident workgroups per CU walk the tile list (most tiles of a late
    // round belong to segments that are already done and cost two loads)
    const unsigned gt = unsigned(tm.cap < 1024 ? tm.cap : 1024);
    const unsigned gm = unsigned(tm.cap < 1536 ? tm.cap : 1536);
    int64_t *split = c->arena.get<int64_t>(tm.cap);
    k_tile_sort<KeyGen, Sink><<<gt, kTileSortBlock, 0, c->stream>>>(tm, offs, key, k0, v0, sink);
    FZ_LAUNCH_CHECK();
    for (int r = 0; r < R; ++r) {
        const bool even = (r & 1) == 0;
        const uint64_t *ik = even ? k0 : k1;
        const uint32_t *iv = even ? v0 : v1;
        merge_splits(c, tm, offs, r, ik, iv, split);
        k_merge_round<Sink><<<gm, kMergeThreads, 0, c->stream>>>(tm, offs, r, split, ik, iv, even ? k1 : k0,
                                                                 even ? v1 : v0, sink);
        FZ_LAUNCH_CHECK();
    }
}

}  // namespace fz
