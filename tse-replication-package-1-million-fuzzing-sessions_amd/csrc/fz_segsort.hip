// Tile map of the segmented merge sort (fz_segsort.h).
#include "fz_segsort.h"
#include "fz_views.h"

namespace fz {

__global__ __launch_bounds__(kBlock) void k_tile_count(const int64_t *__restrict__ offs, int64_t S,
                                                       const uint8_t *__restrict__ flag, int64_t *__restrict__ cnt) {
    for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < S; s += int64_t(gridDim.x) * kBlock) {
        const int64_t len = offs[s + 1] - offs[s];
        // with flags, exactly the flagged segments (the caller's bucket sorts took the others)
        const bool big = flag != nullptr ? (flag[s] != 0 && len > 0) : len > kTile;
        cnt[s] = big ? (len + kTile - 1) / kTile : 0;
    }
}

__global__ __launch_bounds__(kBlock) void k_tile_fill(const int64_t *__restrict__ offs, int64_t S,
                                                      const int64_t *__restrict__ toff, TileMap tm) {
    const int64_t n = *tm.d_n;
    for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < n; k += int64_t(gridDim.x) * kBlock) {
        const int64_t s = upper_bound_i64(toff, 0, S + 1, k) - 1;
        tm.seg[k] = int32_t(s);
        tm.begin[k] = offs[s] + (k - toff[s]) * kTile;
    }
}

// Merge-path splits of every chunk's start diagonal, one wave per chunk: i = number of A rows
// among the first d merged rows = the first m in [lo, hi) with !(A[m] < B[d-1-m]) (hi if none),
// found by a 64-ary search (the lanes probe 64 evenly spaced m at once: one global-memory round
// trip per step instead of one per bisection).  All chunks search in parallel, before the merge.
__global__ __launch_bounds__(kBlock) void k_merge_splits(TileMap tm, const int64_t *__restrict__ offs, int r,
                                                         const uint64_t *__restrict__ ik,
                                                         const uint32_t *__restrict__ iv, int64_t *__restrict__ split) {
    const int64_t ntiles = *tm.d_n;
    const int lane = lane_id();
    for (int64_t k = int64_t(blockIdx.x) * 4 + wave_id(); k < ntiles; k += int64_t(gridDim.x) * 4) {
        int32_t s;
        const MergeChunk m = merge_chunk(tm, offs, r, k, s);
        if (!m.active) continue;
        const int64_t na = m.a1 - m.a0, nb = m.b1 - m.a1, d = m.d0;
        int64_t lo = d - nb > 0 ? d - nb : 0, hi = d < na ? d : na;
        while (lo < hi) {
            const int64_t step = (hi - lo + kWave - 1) / kWave;
            const int64_t q = lo + int64_t(lane) * step;
            bool p = false;
            if (q < hi) {
                const int64_t jb = m.a1 + (d - 1 - q);
                p = kv_less(ik[m.a0 + q], iv[m.a0 + q], ik[jb], iv[jb]);
            }
            const int t = __popcll(__ballot(p));  // P holds on a prefix of the probes
            if (t == 0) {
                hi = lo;
            } else {
                const int64_t nhi = lo + int64_t(t) * step;
                lo = lo + int64_t(t - 1) * step + 1;
                hi = nhi < hi ? nhi : hi;
            }
        }
        if (lane == 0) split[k] = lo;
    }
}

void merge_splits(fz_ctx *c, const TileMap &tm, const int64_t *offs, int r, const uint64_t *ik, const uint32_t *iv,
                  int64_t *split) {
    const unsigned gs = unsigned((tm.cap + 3) / 4 < 4096 ? (tm.cap + 3) / 4 : 4096);
    k_merge_splits<<<gs, kBlock, 0, c->stream>>>(tm, offs, r, ik, iv, split);
    FZ_LAUNCH_CHECK();
}

TileMap big_tiles(fz_ctx *c, const int64_t *offs, int64_t S, int64_t n_cap, const uint8_t *flag) {
    TileMap tm;
    // sum over big segments of ceil(len / kTile) <= n_cap / kTile + (number of big segments)
    tm.cap = n_cap / kTile + (flag ? S : n_cap / (kTile + 1)) + 1;
    tm.d_n = c->arena.get<int64_t>(1);
    tm.seg = c->arena.get<int32_t>(tm.cap);
    tm.begin = c->arena.get<int64_t>(tm.cap);
    int64_t *cnt = c->arena.get<int64_t>(S + 1);
    int64_t *toff = c->arena.get<int64_t>(S + 1);
    k_tile_count<<<grid_for(S), kBlock, 0, c->stream>>>(offs, S, flag, cnt);
    FZ_LAUNCH_CHECK();
    dev_fill(c, cnt + S, 0, 8);
    scan_exclusive_i64(c, cnt, toff, S + 1, tm.d_n);
    k_tile_fill<<<grid_for(tm.cap, kBlock, 4096), kBlock, 0, c->stream>>>(offs, S, toff, tm);
    FZ_LAUNCH_CHECK();
    return tm;
}

}  // namespace fz
