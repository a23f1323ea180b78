// Ragged transpose: runs (a project's trend values, in project order) -> session-major segments.
//
// rq2_coverage_count.py:329-333 appends value i of every project to coverage_by_session_index[i]
// in project order; rq4b_coverage.py:917-931 does the same per group (G2, G1).  With run k holding
// len_k values and group g_k, value i of run k goes to segment (i, g_k) at
//
//     offs[i * G + g_k] + #{q < k : g_q = g_k, len_q > i}
//
// - a permutation known from the lengths alone, so no sort of the values is needed (rounds 1-3
// radix-sorted every value by its session index, 2-4 payload passes over the whole table).
//
//   1. rank the runs by (group, length): one counting launch for <= kRtRankMax runs, else the
//      stable LSD radix sort of R 32-bit keys (R = projects, ~1e4: microseconds);
//   2. tables (one launch): per block b of 64 runs, pre[b][j] = #{sorted position j' < j whose run
//      lies before the block} - so the runs before block b that are longer than i are counted by
//      two lookups; the sorted lengths' prefix sums; each block's tile count (its longest run / 64);
//   3. segment offsets: offs[i * G + g] = sum over runs of min(len, i) (+ the earlier group's count
//      of segment i) from one binary search of i in the sorted lengths - no scan over sessions;
//   4. the move: one workgroup per tile of 64 runs x 64 sessions stages the tile in LDS (reads:
//      each run's 64 consecutive values, 512 B per wave load), then each wave writes one session at
//      a time: the block's live runs of a group are consecutive in their segment (ballot + popcount
//      gives a lane's slot), so the writes are runs of up to 512 B as well;
//   5. a block's single-run tail: past its second-longest run only its longest run is live, and a
//      64 x 64 tile would move 64 values (one live lane per session, a binary search and 128
//      offset loads per tile - config 5L's 20.8M-value giant: 325 k such tiles, 4.7 ms).  Those
//      sessions go kRtTail at a time, one value per thread: its value read and its slot written
//      coalesced (dest = the segment's offset + the earlier blocks' live runs of its group).
//
// Algorithmic traffic (probe "ragged_transpose"): 8 B read + 8 B written per value, plus 8 B per
// segment offset.
#pragma once

#include "fz_seg.h"

namespace fz {

constexpr int kRtRuns = 64;        // runs per tile (one per lane)
constexpr int kRtSess = 64;        // sessions per tile
constexpr int kRtRankMax = 2048;   // runs ranked by counting in one launch; more: the radix sort
constexpr int64_t kRtTableMax = int64_t(1) << 26;  // pre[] entries (4 B each) before the fallback
constexpr int kRtTail = 4096;      // sessions per single-run tail tile (kBlock threads x 16)

// the transpose applies when its tables stay small (R runs, M sessions, G groups)
inline bool ragged_transpose_ok(int64_t R, int64_t M, int G) {
    const int64_t nB = (R + kRtRuns - 1) / kRtRuns;
    return R > 0 && R < (int64_t(1) << 31) && M * G < (int64_t(1) << 31) && (nB + 1) * (R + 1) <= kRtTableMax;
}

template <typename Grp>
__global__ __launch_bounds__(kBlock) void k_rt_keys(const int64_t *__restrict__ offs, int64_t R, int lb, Grp grp,
                                                    uint32_t *__restrict__ key, uint32_t *__restrict__ id) {
    for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < R; k += int64_t(gridDim.x) * kBlock) {
        key[k] = (uint32_t(grp(k)) << lb) | uint32_t(offs[k + 1] - offs[k]);
        id[k] = uint32_t(k);
    }
}

// stable rank of every key by counting (R <= kRtRankMax): rank = #smaller + #equal before.  One
// wave per key: the lanes compare 64 keys at a time (LDS broadcast-free, one key per lane) and the
// wave sums - a thread walking all R keys alone was latency-bound (42 us at R = 1000)
template <typename Grp>
__global__ __launch_bounds__(kBlock) void k_rt_rank(const int64_t *__restrict__ offs, int64_t R, int lb, Grp grp,
                                                    uint32_t *__restrict__ skey, uint32_t *__restrict__ sid) {
    __shared__ uint32_t s_key[kRtRankMax];
    for (int64_t j = threadIdx.x; j < R; j += kBlock)
        s_key[j] = (uint32_t(grp(j)) << lb) | uint32_t(offs[j + 1] - offs[j]);
    __syncthreads();
    const int lane = lane_id();
    const int64_t nw = int64_t(gridDim.x) * (kBlock / kWave);
    for (int64_t k = int64_t(blockIdx.x) * (kBlock / kWave) + wave_id(); k < R; k += nw) {
        const uint32_t mine = s_key[k];
        uint32_t rank = 0;
        for (int64_t j = lane; j < R; j += kWave) {
            const uint32_t o = s_key[j];
            rank += (o < mine) || (o == mine && j < k);
        }
        rank = wave_sum(rank);
        if (lane == 0) {
            skey[rank] = mine;
            sid[rank] = uint32_t(k);
        }
    }
}

// pre[b][j] (b in [0, nB], j in [0, R]) = #{j' < j : sid[j'] < 64 b}  (workgroups 0..nB);
// workgroup nB + 1: plen[j] = sum of the j smallest lengths per group range (exclusive prefix of
// the masked keys), gs[0..2] the group boundaries in sorted order;
// workgroup nB + 2: tile counts per block (longest run / kRtSess, rounded up) -> tpre[nB + 1]
constexpr int kRtTabBlock = 1024;
static __global__ __launch_bounds__(kRtTabBlock) void k_rt_tables(const uint32_t *__restrict__ skey,
                                                           const uint32_t *__restrict__ sid,
                                                           const int64_t *__restrict__ offs, int64_t R, int lb,
                                                           int64_t nB, uint32_t *__restrict__ pre,
                                                           int64_t *__restrict__ plen, int64_t *__restrict__ gs,
                                                           int64_t *__restrict__ tpre, int64_t *__restrict__ tdense,
                                                           int32_t *__restrict__ trun) {
    constexpr int NW = kRtTabBlock / kWave;
    __shared__ int64_t s_tmp[NW];
    const int64_t b = blockIdx.x;
    const uint32_t mask = (1u << lb) - 1u;
    int64_t run = 0;
    if (b <= nB) {
        const uint32_t lim = uint32_t(b * kRtRuns);
        uint32_t *row = pre + b * (R + 1);
        for (int64_t j0 = 0; j0 <= R; j0 += kRtTabBlock) {
            const int64_t j = j0 + threadIdx.x;
            const int64_t f = (j < R && sid[j] < lim) ? 1 : 0;
            int64_t tot;
            const int64_t ex = block_excl_scan<int64_t, NW>(f, s_tmp, &tot);
            if (j <= R) row[j] = uint32_t(run + ex);
            run += tot;
        }
        return;
    }
    if (b == nB + 1) {
        for (int64_t j0 = 0; j0 <= R; j0 += kRtTabBlock) {
            const int64_t j = j0 + threadIdx.x;
            const int64_t len = j < R ? int64_t(skey[j] & mask) : 0;
            int64_t tot;
            const int64_t ex = block_excl_scan<int64_t, NW>(len, s_tmp, &tot);
            if (j <= R) plen[j] = run + ex;
            run += tot;
        }
        if (threadIdx.x == 0) {  // group 0's keys (< 2^lb) come first: the first key of group 1
            int64_t lo = 0, hi = R;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((skey[mid] >> lb) == 0u) lo = mid + 1;
                else hi = mid;
            }
            gs[0] = 0;
            gs[1] = lo;
            gs[2] = R;
        }
        return;
    }
    // tile counts: thread bb takes block bb; the block scan folds them in order.  A block's dense
    // tiles cover the sessions below its second-longest run (rounded up to whole tiles), its tail
    // tiles the rest of its longest run (kRtTail sessions each)
    for (int64_t b0 = 0; b0 < nB; b0 += kRtTabBlock) {
        const int64_t bb = b0 + threadIdx.x;
        int64_t tiles = 0;
        if (bb < nB) {
            int64_t mx = 0, mx2 = 0, arg = bb * kRtRuns;
            const int64_t k1 = (bb + 1) * kRtRuns < R ? (bb + 1) * kRtRuns : R;
            for (int64_t k = bb * kRtRuns; k < k1; ++k) {
                const int64_t len = offs[k + 1] - offs[k];
                if (len > mx) {
                    mx2 = mx;
                    mx = len;
                    arg = k;
                } else if (len > mx2) {
                    mx2 = len;
                }
            }
            const int64_t dense = (mx2 + kRtSess - 1) / kRtSess;
            const int64_t rest = mx - dense * kRtSess;
            tiles = dense + (rest > 0 ? (rest + kRtTail - 1) / kRtTail : 0);
            tdense[bb] = dense;
            trun[bb] = int32_t(arg);
        }
        int64_t tot;
        const int64_t ex = block_excl_scan<int64_t, NW>(tiles, s_tmp, &tot);
        if (bb < nB) tpre[bb] = run + ex;
        run += tot;
    }
    if (threadIdx.x == 0) tpre[nB] = run;
}

// Segment offsets: out[i * G + g] for i in [0, M), out[M * G] = total; cidx[i * G + g] = the
// sorted position where group g's runs longer than i start
static __global__ __launch_bounds__(kBlock) void k_rt_offsets(const uint32_t *__restrict__ skey,
                                                       const int64_t *__restrict__ plen,
                                                       const int64_t *__restrict__ gs, int lb, int G, int64_t M,
                                                       int64_t *__restrict__ out, int32_t *__restrict__ cidx) {
    const uint32_t mask = (1u << lb) - 1u;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i <= M; i += int64_t(gridDim.x) * kBlock) {
        int64_t before = 0, cnt[2] = {0, 0};
        for (int g = 0; g < G; ++g) {
            // first sorted position of group g with length > i
            int64_t lo = gs[g], hi = gs[g + 1];
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (int64_t(skey[mid] & mask) <= i) lo = mid + 1;
                else hi = mid;
            }
            cnt[g] = gs[g + 1] - lo;
            before += plen[lo] - plen[gs[g]] + i * cnt[g];  // sum of min(len, i) over the group
            if (i < M) cidx[i * G + g] = int32_t(lo);
        }
        if (i == M) {
            out[M * G] = before;
            continue;
        }
        out[i * G] = before;
        if (G == 2) out[i * G + 1] = before + cnt[0];
    }
}

// The move: tile t = (block b, session chunk) of kRtRuns x kRtSess values, staged in LDS.
// In: value j of the input (run k's values are j in [offs[k], offs[k + 1])).
template <int G, typename In, typename Grp>
__global__ __launch_bounds__(kBlock) void k_rt_move(const int64_t *__restrict__ offs, int64_t R, int64_t M, In in,
                                                    Grp grp, const uint32_t *__restrict__ pre,
                                                    const int64_t *__restrict__ gs, const int64_t *__restrict__ tpre,
                                                    int64_t nB, const int64_t *__restrict__ tdense,
                                                    const int32_t *__restrict__ trun, const int64_t *__restrict__ soffs,
                                                    const int32_t *__restrict__ cidx, double *__restrict__ out) {
    __shared__ double s_v[kRtRuns][kRtSess + 1];
    __shared__ int64_t s_base[G][kRtSess];
    const int lane = lane_id(), w = wave_id();
    constexpr int NW = kBlock / kWave;
    const int64_t ntiles = tpre[nB];
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        // block of tile t: last b with tpre[b] <= t (blocks without tiles are skipped by the search)
        int64_t lo = 0, hi = nB - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (tpre[mid] <= t) lo = mid;
            else hi = mid - 1;
        }
        const int64_t b = lo;
        const int64_t tb = t - tpre[b], nd = tdense[b];
        if (tb >= nd) {  // the block's single-run tail: one session per thread, no LDS
            const int64_t k = trun[b];
            const int64_t st = offs[k], len = offs[k + 1] - st;
            const int g = G == 2 ? grp(k) : 0;
            const uint32_t *prow = pre + b * (R + 1);
            const uint32_t before_end = prow[gs[g + 1]];
            const int64_t ib = nd * kRtSess + (tb - nd) * int64_t(kRtTail);
            for (int64_t i = ib + threadIdx.x; i < ib + kRtTail && i < len; i += kBlock)
                out[soffs[i * G + g] + int64_t(before_end) - int64_t(prow[cidx[i * G + g]])] = in(st + i);
            continue;  // (no LDS used: no barrier owed)
        }
        const int64_t i0 = tb * kRtSess;
        const int64_t k0 = b * kRtRuns;
        // stage: wave w loads runs w, w + NW, ...: 64 consecutive values each
        for (int r = w; r < kRtRuns; r += NW) {
            const int64_t k = k0 + r;
            if (k >= R) break;
            const int64_t st = offs[k], len = offs[k + 1] - st;
            const int64_t i = i0 + lane;
            if (i < len) s_v[r][lane] = in(st + i);
        }
        // segment bases of the block's runs: offs + (runs of the group before the block, longer than i)
        const uint32_t *prow = pre + b * (R + 1);
        for (int q = threadIdx.x; q < G * kRtSess; q += kBlock) {
            const int g = q / kRtSess, l = q % kRtSess;
            const int64_t i = i0 + l;
            if (i < M) s_base[g][l] = soffs[i * G + g] + int64_t(prow[gs[g + 1]]) - int64_t(prow[cidx[i * G + g]]);
        }
        __syncthreads();
        // write: wave w takes sessions w, w + NW, ...; lane = run
        const int64_t k = k0 + lane;
        const int64_t len = k < R ? offs[k + 1] - offs[k] : 0;
        const int g = (G == 2 && k < R) ? grp(k) : 0;
        for (int l = w; l < kRtSess; l += NW) {
            const int64_t i = i0 + l;
            const bool alive = i < len;
            const uint64_t m0 = __ballot(alive && g == 0);
            const uint64_t m1 = G == 2 ? __ballot(alive && g == 1) : 0ull;
            if ((m0 | m1) == 0ull) break;  // (runs only end: no later session of the tile is live)
            if (alive) {
                const uint64_t m = g == 0 ? m0 : m1;
                out[s_base[g][l] + __popcll(m & lanemask_lt())] = s_v[lane][l];
            }
        }
        __syncthreads();  // LDS is restaged by the next tile
    }
}

struct RtOneGroup {
    __device__ int operator()(int64_t) const { return 0; }
};

// Scratch of one transpose (arena) and its launches.  out_offs: [M * G + 1]; out: offs[R] values.
template <int G, typename In, typename Grp>
void ragged_transpose(fz_ctx *c, const int64_t *offs, int64_t R, int64_t M, int64_t n_cap, In in, Grp grp,
                      double *out, int64_t *out_offs) {
    static_assert(G == 1 || G == 2, "ragged_transpose: one or two groups");
    FZ_CHECK(ragged_transpose_ok(R, M, G), "ragged_transpose: shape out of range");
    hipStream_t st = c->stream;
    const int lb = bits_for(uint64_t(M));  // lengths <= M
    FZ_CHECK(lb + (G == 2 ? 1 : 0) <= 32, "ragged_transpose: run lengths past 32 bits");
    const int kbits = lb + (G == 2 ? 1 : 0);
    const int64_t nB = (R + kRtRuns - 1) / kRtRuns;
    uint32_t *skey, *sid;
    if (R <= kRtRankMax) {
        skey = c->arena.get<uint32_t>(R);
        sid = c->arena.get<uint32_t>(R);
        const int64_t wg = (R + kBlock / kWave - 1) / (kBlock / kWave);  // one wave per key
        k_rt_rank<Grp><<<unsigned(wg < 128 ? wg : 128), kBlock, 0, st>>>(offs, R, lb, grp, skey, sid);
        FZ_LAUNCH_CHECK();
    } else {
        skey = c->arena.get<uint32_t>(R);
        sid = c->arena.get<uint32_t>(R);
        k_rt_keys<Grp><<<grid_for(R), kBlock, 0, st>>>(offs, R, lb, grp, skey, sid);
        FZ_LAUNCH_CHECK();
        RadixPayload none;
        radix_sort_pairs_payload32(c, skey, sid, R, kbits, none);
    }
    uint32_t *pre = c->arena.get<uint32_t>((nB + 1) * (R + 1));
    int64_t *plen = c->arena.get<int64_t>(R + 1);
    int64_t *gs = c->arena.get<int64_t>(3);
    int64_t *tpre = c->arena.get<int64_t>(nB + 1);
    int64_t *tdense = c->arena.get<int64_t>(nB);
    int32_t *trun = c->arena.get<int32_t>(nB);
    k_rt_tables<<<unsigned(nB + 3), kRtTabBlock, 0, st>>>(skey, sid, offs, R, lb, nB, pre, plen, gs, tpre, tdense,
                                                          trun);
    FZ_LAUNCH_CHECK();
    int32_t *cidx = c->arena.get<int32_t>(M * G);
    k_rt_offsets<<<grid_for(M + 1, kBlock, 16384), kBlock, 0, st>>>(skey, plen, gs, lb, G, M, out_offs, cidx);
    FZ_LAUNCH_CHECK();
    // tiles: at most one per block plus one per kRtSess values
    const int64_t tiles_cap = nB + n_cap / kRtSess + 1;
    ProbeScope ps(c, "ragged_transpose", 8.0 * double(M * G + 1), offs + R, 16.0);
    k_rt_move<G, In, Grp><<<unsigned(tiles_cap < 4096 ? tiles_cap : 4096), kBlock, 0, st>>>(
        offs, R, M, in, grp, pre, gs, tpre, nB, tdense, trun, out_offs, cidx, out);
    FZ_LAUNCH_CHECK();
}

}  // namespace fz
