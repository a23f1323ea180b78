// RQ1 - bug-detection rate per fuzzing iteration (rq1_detection_rate.py:101-269).
//
// Reference flow and its replacement here:
//   eligibility GROUP BY/HAVING (:144-152)            -> k_elig_hist (LDS-privatised histogram)
//   878 x ALL_FUZZING_BUILD (:189-203)                -> segment lengths of store.fuzz, histogram,
//                                                        reverse scan (projects alive at iteration i)
//   SAME_DATE_BUILD_ISSUE as-of join (queries1.py:15-58) -> per-issue lower_bound in the filtered
//                                                        (Finish|Halfway, < LIMIT) Fuzzing view
//   ROW_NUMBER() OVER (PARTITION BY number ...)        -> two stable radix sorts (build time desc,
//                                                        then number); segment heads survive
//   43k x O(B) iteration scans (:213-230)             -> per-issue lower_bound in store.fuzz;
//                                                        distinct (iteration, project) by adjacency
//   finalize + late-stage stats (:233-268)            -> rate kernel + describe_f64_dn
#include "fz_device.h"
#include "fz_internal.h"
#include "fz_views.h"

namespace fz {

constexpr int64_t kLimitUs = 1736294400000000LL;  // '2025-01-08 00:00:00' (queries1.py:3)
constexpr int64_t kEligMin = 365;                 // HAVING COUNT(*) >= 365

__global__ __launch_bounds__(kBlock) void k_copy_elig(const uint8_t *__restrict__ src, const int64_t *__restrict__ n,
                                                      int64_t P, uint8_t *__restrict__ dst, int64_t *__restrict__ d_count) {
    for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < P; p += int64_t(gridDim.x) * kBlock)
        dst[p] = src[p];
    if (blockIdx.x == 0 && threadIdx.x == 0 && d_count) *d_count = *n;
}

// total_coverage rows: coverage IS NOT NULL AND coverage > 0 AND date < LIMIT, per project.
// One 1024-thread workgroup per CU (16 waves: enough loads in flight to stream HBM) takes a
// contiguous slice into an LDS histogram and writes it as one row of a [blocks][P] partial table
// (no global atomics, deterministic); k_elig_sum adds the columns.  Each thread handles two rows
// per iteration, their four column loads issued before either predicate.
constexpr int kEligBlocks = 256;
constexpr int kEligThreads = 1024;
constexpr int64_t kEligLdsMax = 16384;  // 64 KiB of int32 bins

// (part2 != null: a second histogram of every row before the limit, any validity - the store's
// bound on the analyses' session axes, View::lim_seg - in the second half of the LDS)
__global__ __launch_bounds__(kEligThreads) void k_elig_hist(const uint32_t *__restrict__ proj,
                                                            const int64_t *__restrict__ date,
                                                            const double *__restrict__ cov,
                                                            const uint8_t *__restrict__ valid, int64_t n, int64_t P,
                                                            int64_t limit, int32_t *__restrict__ part,
                                                            int32_t *__restrict__ part2) {
    extern __shared__ int32_t s_hist[];
    int32_t *const s_h2 = s_hist + P;
    for (int64_t p = threadIdx.x; p < (part2 ? 2 * P : P); p += kEligThreads) s_hist[p] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = int64_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
    int64_t i = lo + threadIdx.x;
    for (; i + kEligThreads < hi; i += 2 * kEligThreads) {
        const int64_t j = i + kEligThreads;
        const uint8_t va = valid[i], vb = valid[j];
        const double ca = cov[i], cb = cov[j];
        const int64_t da = date[i], db = date[j];
        const uint32_t pa = proj[i], pb = proj[j];
        if ((va & FZ_VALID_COVERAGE) && ca > 0.0 && da < limit) atomicAdd(&s_hist[pa], 1);
        if ((vb & FZ_VALID_COVERAGE) && cb > 0.0 && db < limit) atomicAdd(&s_hist[pb], 1);
        if (part2) {
            if (da < limit) atomicAdd(&s_h2[pa], 1);
            if (db < limit) atomicAdd(&s_h2[pb], 1);
        }
    }
    if (i < hi) {
        if ((valid[i] & FZ_VALID_COVERAGE) && cov[i] > 0.0 && date[i] < limit) atomicAdd(&s_hist[proj[i]], 1);
        if (part2 && date[i] < limit) atomicAdd(&s_h2[proj[i]], 1);
    }
    __syncthreads();
    for (int64_t p = threadIdx.x; p < P; p += kEligThreads) part[int64_t(blockIdx.x) * P + p] = s_hist[p];
    if (part2)
        for (int64_t p = threadIdx.x; p < P; p += kEligThreads) part2[int64_t(blockIdx.x) * P + p] = s_h2[p];
}

// fallback for very many projects: global atomics straight into counts
__global__ __launch_bounds__(kBlock) void k_elig_atomic(const uint32_t *__restrict__ proj,
                                                        const int64_t *__restrict__ date,
                                                        const double *__restrict__ cov,
                                                        const uint8_t *__restrict__ valid, int64_t n, int64_t limit,
                                                        int32_t *__restrict__ counts, int32_t *__restrict__ counts2) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        if ((valid[i] & FZ_VALID_COVERAGE) && cov[i] > 0.0 && date[i] < limit) atomicAdd(&counts[proj[i]], 1);
        if (counts2 && date[i] < limit) atomicAdd(&counts2[proj[i]], 1);
    }
}

// Column sums of the [nb][P] partial table: a workgroup owns 64 projects (one per lane, coalesced
// rows), its 4 waves split the nb partial rows, LDS adds the 4 wave sums.  part == null: counts
// are already final (atomic fallback), only the flags are derived.
// (part2 / counts2 != null: the before-limit histogram's column sums too, their maximum atomically
// into *lim_max - zero on entry)
__global__ __launch_bounds__(kBlock) void k_elig_sum(const int32_t *__restrict__ part, int nb, int64_t P,
                                                     int32_t *__restrict__ counts, uint8_t *__restrict__ elig,
                                                     int64_t *__restrict__ n_elig, const int32_t *__restrict__ part2,
                                                     const int32_t *__restrict__ counts2,
                                                     int64_t *__restrict__ lim_max) {
    __shared__ int32_t s_sum[4][kWave];
    __shared__ int32_t s_sum2[4][kWave];
    const int64_t p = int64_t(blockIdx.x) * kWave + lane_id();
    const int w = wave_id();
    int32_t s = 0, s2 = 0;
    if (part && p < P) {
#pragma unroll 8
        for (int b = w; b < nb; b += 4) s += part[int64_t(b) * P + p];
        if (part2)
#pragma unroll 8
            for (int b = w; b < nb; b += 4) s2 += part2[int64_t(b) * P + p];
    }
    s_sum[w][lane_id()] = s;
    s_sum2[w][lane_id()] = s2;
    __syncthreads();
    if (w != 0) return;
    if (lim_max) {
        int64_t m = 0;
        if (p < P)
            m = part ? int64_t(s_sum2[0][lane_id()] + s_sum2[1][lane_id()] + s_sum2[2][lane_id()] + s_sum2[3][lane_id()])
                     : int64_t(counts2[p]);
        m = wave_max(m);
        if (lane_id() == 0 && m > 0)
            atomicMax(reinterpret_cast<unsigned long long *>(lim_max), (unsigned long long)m);
    }
    if (p >= P) return;
    if (part) {
        s = s_sum[0][lane_id()] + s_sum[1][lane_id()] + s_sum[2][lane_id()] + s_sum[3][lane_id()];
        if (counts) counts[p] = s;
    } else {
        s = counts[p];
    }
    if (elig) {
        const bool e = s >= kEligMin;
        elig[p] = e;
        if (e) atomic_add_i64(n_elig, 1);
    }
}

// counts[p] (and, if elig != null, elig[p] = counts >= 365 with *n_elig += #eligible; if lim_max !=
// null, *lim_max (zero on entry) = the most rows of one project dated before the limit)
static void eligibility(fz_ctx *c, const fz_tables *t, int64_t limit, int32_t *counts, uint8_t *elig,
                        int64_t *n_elig, int64_t *lim_max = nullptr) {
    const int64_t P = t->n_projects;
    if (P <= 0) return;
    // algorithmic bytes: project 4 + date 8 + coverage 8 + validity 1 per row
    ProbeScope ps(c, "elig_hist", 21.0 * double(t->n_cov));
    if (P <= kEligLdsMax) {
        const int nb = t->n_cov > 0 ? kEligBlocks : 1;
        int32_t *part = c->arena.get<int32_t>(int64_t(nb) * P);
        int32_t *part2 = lim_max ? c->arena.get<int32_t>(int64_t(nb) * P) : nullptr;
        const size_t lds = size_t(P) * 4 * (lim_max ? 2 : 1);
        if (lds > 65536)  // (both histograms of up to 16384 bins: up to 128 KiB of the CU's 160)
            // function attributes are per device: set on every such launch (cheap), never cached
            // in a process-wide flag that a second device or a concurrent build would race on
            FZ_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_elig_hist),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(2 * kEligLdsMax * 4)));
        k_elig_hist<<<nb, kEligThreads, lds, c->stream>>>(
            t->c_project, t->c_date, t->c_coverage, t->c_valid, t->n_cov, P, limit, part, part2);
        k_elig_sum<<<unsigned((P + kWave - 1) / kWave), kBlock, 0, c->stream>>>(part, nb, P, counts, elig, n_elig,
                                                                               part2, nullptr, lim_max);
    } else {
        if (!counts) counts = c->arena.get<int32_t>(P);
        int32_t *counts2 = lim_max ? c->arena.get<int32_t>(P) : nullptr;
        dev_fill(c, counts, 0, P * 4);
        if (counts2) dev_fill(c, counts2, 0, P * 4);
        k_elig_atomic<<<grid_for(t->n_cov, kBlock, 2048), kBlock, 0, c->stream>>>(
            t->c_project, t->c_date, t->c_coverage, t->c_valid, t->n_cov, limit, counts, counts2);
        k_elig_sum<<<unsigned((P + kWave - 1) / kWave), kBlock, 0, c->stream>>>(nullptr, 0, P, counts, elig, n_elig,
                                                                               nullptr, counts2, lim_max);
    }
    FZ_LAUNCH_CHECK();
}

void eligibility_counts(fz_ctx *c, const fz_tables *t, int64_t limit, int32_t *counts) {
    eligibility(c, t, limit, counts, nullptr, nullptr);
}

// Computed once per fz_store_build (store.elig / store.n_elig).
// zeroed: the caller's fill already cleared the two counters (s.n_elig, allocated beforehand)
void store_eligibility(fz_ctx *c, bool zeroed) {
    Store &s = store_of(c);
    const int64_t P = s.P;
    uint8_t *elig = s.elig.ensure<uint8_t>(P);
    int64_t *n = s.n_elig.ensure<int64_t>(2);
    int32_t *cnt = s.elig_cnt.ensure<int32_t>(P);  // (kept: fz_store_elig_counts reads them)
    if (!zeroed) dev_fill(c, n, 0, 16);
    eligibility(c, &s.t, kLimitUs, cnt, elig, n, n + 1);
}

// elig[p] = project has >= 365 qualifying coverage rows; *d_count = number eligible.
// Every RQ script starts from this set (rq1:144-152, rq2_count:272-280, rq2_add:20-27, rq3:222-226,
// rq4a:68-80, rq4b:164-181 - the same GROUP BY/HAVING), so the store computes it once per load.
void eligible_projects(fz_ctx *c, uint8_t *elig, int64_t *d_count, std::initializer_list<Fill> fills) {
    const Store &s = store_of(c);
    const int64_t P = s.P;
    const uint8_t *src = s.elig.as<uint8_t>();
    const int64_t *n = s.n_elig.as<int64_t>();
    if (fills.size() == 0) {
        k_copy_elig<<<grid_for(P > 0 ? P : 1), kBlock, 0, c->stream>>>(src, n, P, elig, d_count);
        FZ_LAUNCH_CHECK();
        return;
    }
    // the analysis' output / scratch fills, the flags copy and the count in one launch
    fill_copy_batch(c, fills, src, elig, P, n, d_count);
}

// Histogram of Fuzzing-build counts over eligible projects; total and max.
__global__ __launch_bounds__(kBlock) void k_iter_hist(const int64_t *__restrict__ offs, const uint8_t *__restrict__ elig,
                                                      int64_t P, int64_t *__restrict__ hist,
                                                      int64_t *__restrict__ counts) {
    for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < P; p += int64_t(gridDim.x) * kBlock) {
        if (!elig[p]) continue;
        const int64_t nf = offs[p + 1] - offs[p];
        atomic_add_i64(&hist[nf], 1);
        atomic_add_i64(&counts[FZ_RQ1_TOTAL_FUZZ], nf);
        atomicMax(reinterpret_cast<unsigned long long *>(&counts[FZ_RQ1_MAX_ITER]), (unsigned long long)nf);
    }
}

__global__ __launch_bounds__(kBlock) void k_reverse_tail(const int64_t *__restrict__ hist, int64_t M,
                                                         int64_t *__restrict__ rev) {
    for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < M; j += int64_t(gridDim.x) * kBlock)
        rev[j] = hist[M - j];
}

// iter_total[i-1] = sum_{k >= i} hist[k]
__global__ __launch_bounds__(kBlock) void k_iter_total(const int64_t *__restrict__ rev_excl,
                                                       const int64_t *__restrict__ rev, int64_t M,
                                                       int64_t *__restrict__ iter_total) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x + 1; i <= M; i += int64_t(gridDim.x) * kBlock) {
        const int64_t j = M - i;
        iter_total[i - 1] = rev_excl[j] + rev[j];
    }
}

struct ValidFuzzRq1 {  // result IN ('Finish', 'Halfway') AND DATE(timecreated) < LIMIT  (queries1.py:39-43)
    static constexpr int kBytes = 9;  // column bytes read per row (filter_compact probe)
    const uint8_t *result;
    const int64_t *time;
    __device__ bool operator()(int32_t r) const {
        const uint8_t x = result[r];
        return (x <= 1) & (time[r] < kLimitUs);
    }
};

// One pass over the (project, rts)-sorted issues: counts, per-project flags, as-of join.
// *ctr += the active lanes of this wave with pred (one atomic per wave, by its first active lane)
__device__ inline void wave_count_add(int64_t *ctr, bool pred) {
    const uint64_t m = __ballot(pred);
    if (!m) return;
    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
    if (lane_id() == leader) atomicAdd(reinterpret_cast<unsigned long long *>(ctr), (unsigned long long)__popcll(m));
}

__global__ __launch_bounds__(kBlock) void k_issue_pass(View iss, const uint8_t *__restrict__ status,
                                                       const uint8_t *__restrict__ elig,
                                                       const int32_t *__restrict__ pi_count,
                                                       const int32_t *__restrict__ vrow,
                                                       const int64_t *__restrict__ vtime,
                                                       const int64_t *__restrict__ voffs, int64_t *__restrict__ counts,
                                                       uint8_t *__restrict__ f_lim, uint8_t *__restrict__ f_fixlim,
                                                       uint8_t *__restrict__ f_tgt, int64_t *__restrict__ mbuild,
                                                       int64_t *__restrict__ mbtime) {
    for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < iss.n; j += int64_t(gridDim.x) * kBlock) {
        const int32_t r = int32_t(iss.row0 + j);
        const uint32_t p = iss.proj[j];
        const int64_t rts = iss.time[j];
        const bool lim = rts < kLimitUs;
        const bool fixed = status[r] <= 1;
        const bool el = elig[p];
        // (the three counters: one atomic per wave each - per-issue atomics on three words serialise)
        wave_count_add(&counts[FZ_RQ1_ISSUES_LIM], lim);
        wave_count_add(&counts[FZ_RQ1_FIXED_LIM], lim && fixed);
        wave_count_add(&counts[FZ_RQ1_TARGET], lim && fixed && el);
        if (lim) {
            f_lim[p] = 1;
            if (fixed) {
                f_fixlim[p] = 1;
                if (el) f_tgt[p] = 1;
            }
        }
        int64_t mb = -1, bt = 0;
        if (fixed && el) {
            if (rts != FZ_TS_NULL) {
                const int64_t lo = voffs[p], hi = voffs[p + 1];
                const int64_t k = lower_bound_i64(vtime, lo, hi, rts);
                if (k > lo) {
                    mb = vrow[k - 1];
                    bt = vtime[k - 1];
                }
            }
            if (mb < 0 && pi_count) atomic_add_i64(&counts[FZ_RQ1_WITHOUT_MATCHING], pi_count[p]);
        }
        mbuild[j] = mb;
        mbtime[j] = bt;
    }
}

// ROW_NUMBER() OVER (PARTITION BY number ORDER BY timecreated DESC) = 1 (queries1.py:29-32):
// sort the matched rows by issue number (range-compressed key, stable in output order); in each
// number group the row with the latest build time survives, the earliest in output order on ties.
__global__ __launch_bounds__(kBlock) void k_dedup_keys(const int64_t *__restrict__ mbuild, View iss,
                                                       const int64_t *__restrict__ number, int64_t n, int64_t nmin,
                                                       uint64_t pad, uint64_t *__restrict__ keys,
                                                       uint32_t *__restrict__ vals) {
    for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < n; j += int64_t(gridDim.x) * kBlock) {
        keys[j] = mbuild[j] >= 0 ? uint64_t(number[iss.row0 + j] - nmin) : pad;
        vals[j] = uint32_t(j);
    }
}

// Entries [0, n_loc) are this shard's matches; entries from n_loc on are other shards' (ext):
// they compete for their number but are never kept.  Tie order = ORDER BY project, rts across
// shards: an ext entry from a preceding shard sorts before every local row, one from a following
// shard after.
__global__ __launch_bounds__(kBlock) void k_dedup_pick(const uint32_t *__restrict__ vals,
                                                       const uint64_t *__restrict__ keys,
                                                       const int64_t *__restrict__ mbuild,
                                                       const int64_t *__restrict__ mbtime, int64_t n_loc,
                                                       fz_rq1_ext ext, int64_t n, int64_t *__restrict__ keep) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const uint32_t j = vals[i];
        if (j >= n_loc) continue;
        if (mbuild[j] < 0) {
            keep[j] = 0;
            continue;
        }
        const uint64_t k = keys[i];
        int64_t a = i, b = i + 1;  // the number group [a, b) (tiny: duplicates are rare)
        while (a > 0 && keys[a - 1] == k) --a;
        while (b < n && keys[b] == k) ++b;
        const int64_t tj = mbtime[j];
        bool win = true;
        for (int64_t q = a; q < b && win; ++q) {
            const uint32_t v = vals[q];
            if (v == j) continue;
            if (v < n_loc) {
                if (mbuild[v] < 0) continue;
                win = tj > mbtime[v] || (tj == mbtime[v] && j < v);
            } else {
                const int64_t e = v - n_loc, te = ext.build_time[e];
                win = tj > te || (tj == te && !ext.before[e]);
            }
        }
        keep[j] = win ? 1 : 0;
    }
}

__global__ __launch_bounds__(kBlock) void k_dedup_ext_keys(fz_rq1_ext ext, int64_t nmin, uint64_t pad, int64_t n_loc,
                                                           uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (int64_t e = int64_t(blockIdx.x) * kBlock + threadIdx.x; e < ext.n; e += int64_t(gridDim.x) * kBlock) {
        const int64_t d = ext.number[e] - nmin;
        keys[n_loc + e] = d >= 0 && uint64_t(d) < pad ? uint64_t(d) : pad;
        vals[n_loc + e] = uint32_t(n_loc + e);
    }
}

// Compact kept matches in (project, rts) order; iteration = #Fuzzing builds with time < rts.
__global__ __launch_bounds__(kBlock) void k_matched_out(View iss, const int64_t *__restrict__ keep,
                                                        const int64_t *__restrict__ pos,
                                                        const int64_t *__restrict__ mbuild, View fuzz,
                                                        int64_t *__restrict__ out_issue,
                                                        int64_t *__restrict__ out_build, int64_t *__restrict__ it_arr,
                                                        uint32_t *__restrict__ p_arr, uint8_t *__restrict__ f_match,
                                                        const int32_t *__restrict__ iperm,
                                                        const int32_t *__restrict__ bperm) {
    for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < iss.n; j += int64_t(gridDim.x) * kBlock) {
        if (!keep[j]) continue;
        const int64_t q = pos[j];
        const uint32_t p = iss.proj[j];
        out_issue[q] = iperm[iss.row0 + j];
        out_build[q] = bperm[mbuild[j]];
        const int64_t lo = fuzz.offs[p], hi = fuzz.offs[p + 1];
        it_arr[q] = lower_bound_i64(fuzz.time, lo, hi, iss.time[j]) - lo;
        p_arr[q] = p;
        f_match[p] = 1;
    }
}

__global__ __launch_bounds__(kBlock) void k_distinct_iter(const int64_t *__restrict__ it_arr,
                                                          const uint32_t *__restrict__ p_arr,
                                                          const int64_t *__restrict__ d_n,
                                                          int64_t *__restrict__ iter_det) {
    const int64_t n = *d_n;
    for (int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x; q < n; q += int64_t(gridDim.x) * kBlock) {
        const int64_t it = it_arr[q];
        if (it <= 0) continue;
        if (q > 0 && p_arr[q - 1] == p_arr[q] && it_arr[q - 1] == it) continue;
        atomic_add_i64(&iter_det[it - 1], 1);
    }
}

// Kept iterations are the prefix 1..K (iter_total is non-increasing); first key with rate < 5.
__global__ __launch_bounds__(kBlock) void k_rates(const int64_t *__restrict__ iter_total,
                                                  const int64_t *__restrict__ iter_det, int64_t M, int64_t threshold,
                                                  int64_t *__restrict__ counts, double *__restrict__ rates) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < M; i += int64_t(gridDim.x) * kBlock) {
        const int64_t tot = iter_total[i];
        if (tot < threshold || tot <= 0) continue;
        atomic_add_i64(&counts[FZ_RQ1_KEPT_ITERS], 1);
        const double r = double(iter_det[i]) / double(tot) * 100.0;  // :245 (Python float ops)
        rates[i] = r;
        if (r < 5.0) atomicMin(reinterpret_cast<unsigned long long *>(&counts[FZ_RQ1_FIRST_DOWN]),
                                (unsigned long long)(i + 1));
    }
}

// late = rates[first_down:] (first_down is a KEY used as a list index; -1 -> the last rate).
__global__ void k_late_bounds(int64_t *__restrict__ counts, int64_t *__restrict__ late_lo) {
    if (threadIdx.x || blockIdx.x) return;
    const int64_t K = counts[FZ_RQ1_KEPT_ITERS];
    int64_t fd = counts[FZ_RQ1_FIRST_DOWN];
    if (uint64_t(fd) == ~0ull) fd = -1;
    counts[FZ_RQ1_FIRST_DOWN] = fd;
    int64_t lo = fd >= 0 ? fd : K - 1;
    if (lo < 0) lo = 0;
    const int64_t n = K > lo ? K - lo : 0;
    counts[FZ_RQ1_LATE] = n;
    late_lo[0] = lo;
    late_lo[1] = n;
}

__global__ __launch_bounds__(kBlock) void k_late_copy(const double *__restrict__ rates,
                                                      const int64_t *__restrict__ late_lo, double *__restrict__ late) {
    const int64_t lo = late_lo[0], n = late_lo[1];
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        late[i] = rates[lo + i];
}

void rq1_finish(fz_ctx *c, int64_t threshold, const int64_t *iter_total, const int64_t *iter_det, int64_t M,
                int64_t *counts, fz_describe *late_out) {
    hipStream_t st = c->stream;
    fill_batch(c, {{counts + FZ_RQ1_KEPT_ITERS, 8, 0}, {counts + FZ_RQ1_FIRST_DOWN, 8, 0xff}});
    double *rates = c->arena.get<double>(M);
    double *late = c->arena.get<double>(M);
    int64_t *late_lo = c->arena.get<int64_t>(2);
    if (M > 0) {
        k_rates<<<grid_for(M), kBlock, 0, st>>>(iter_total, iter_det, M, threshold, counts, rates);
        FZ_LAUNCH_CHECK();
    }
    k_late_bounds<<<1, 64, 0, st>>>(counts, late_lo);
    k_late_copy<<<grid_for(M > 0 ? M : 1), kBlock, 0, st>>>(rates, late_lo, late);
    FZ_LAUNCH_CHECK();
    describe_f64_dn(c, late, M, late_lo + 1, late_out);
}

void rq1(fz_ctx *c, int64_t threshold, const fz_rq1_ext *ext_in, const fz_rq1_out *o) {
    Store &s = store_of(c);
    FZ_CHECK(s.built, "fz_rq1: call fz_store_build first");
    FZ_CHECK(o && o->counts && o->eligible && o->iter_total && o->iter_detected && o->matched_issue &&
                 o->matched_build && o->late,
             "fz_rq1: null output buffer");
    const fz_rq1_ext ext = ext_in ? *ext_in : fz_rq1_ext{0, nullptr, nullptr, nullptr};
    FZ_CHECK(ext.n >= 0 && (ext.n == 0 || (ext.number && ext.build_time && ext.before)),
             "fz_rq1_ex: bad competitor arrays");
    FZ_CHECK(s.issues.n + ext.n < (int64_t(1) << 32), "fz_rq1_ex: too many competitors");
    const fz_tables &t = s.t;
    const int64_t P = s.P;
    const int64_t M = s.fuzz.max_seg;
    hipStream_t st = c->stream;
    int64_t *hist = c->arena.get<int64_t>(M + 1);
    uint8_t *flags = c->arena.get<uint8_t>(4 * P);
    // eligibility (:144-152), with the output / scratch fills in the same launch
    eligible_projects(c, o->eligible, o->counts + FZ_RQ1_ELIGIBLE,
                      {{o->counts, FZ_RQ1_FIRST_DOWN * 8, 0},
                       {o->counts + FZ_RQ1_FIRST_DOWN, 8, 0xff},
                       {o->counts + FZ_RQ1_FIRST_DOWN + 1, (FZ_RQ1_NCOUNTS - FZ_RQ1_FIRST_DOWN - 1) * 8, 0},
                       {o->iter_total, (M > 0 ? M : 1) * 8, 0},
                       {o->iter_detected, (M > 0 ? M : 1) * 8, 0},
                       {hist, (M + 1) * 8, 0},
                       {flags, 4 * (P > 0 ? P : 1), 0}});

    // phase 1: projects alive at each iteration (:189-203)
    if (P > 0) {
        k_iter_hist<<<grid_for(P), kBlock, 0, st>>>(s.fuzz.offs, o->eligible, P, hist, o->counts);
        FZ_LAUNCH_CHECK();
    }
    if (M > 0) {
        int64_t *rev = c->arena.get<int64_t>(M);
        int64_t *rex = c->arena.get<int64_t>(M);
        k_reverse_tail<<<grid_for(M), kBlock, 0, st>>>(hist, M, rev);
        scan_exclusive_i64(c, rev, rex, M, nullptr);
        k_iter_total<<<grid_for(M), kBlock, 0, st>>>(rex, rev, M, o->iter_total);
        FZ_LAUNCH_CHECK();
    }

    // SAME_DATE_BUILD_ISSUE partner view
    TmpView v1;
    filter_view(c, s.fuzz, s.fuzz.n, P, ValidFuzzRq1{t.b_result, t.b_time}, v1);

    // issues pass
    const int64_t NI = s.issues.n;
    uint8_t *f_lim = flags, *f_fixlim = flags + P, *f_tgt = flags + 2 * P, *f_match = flags + 3 * P;
    int64_t *mbuild = c->arena.get<int64_t>(NI);
    int64_t *mbtime = c->arena.get<int64_t>(NI);
    if (NI > 0) {
        k_issue_pass<<<grid_for(NI, kBlock, 2048), kBlock, 0, st>>>(s.issues, t.i_status, o->eligible, t.pi_count,
                                                                    v1.row, v1.time, v1.offs, o->counts, f_lim,
                                                                    f_fixlim, f_tgt, mbuild, mbtime);
        FZ_LAUNCH_CHECK();
    }

    // ROW_NUMBER dedup by issue number
    int64_t *keep = c->arena.get<int64_t>(NI);
    int64_t *pos = c->arena.get<int64_t>(NI);
    int64_t *d_nm = o->counts + FZ_RQ1_MATCHED;
    if (NI > 0) {
        const int64_t NA = NI + ext.n;
        uint64_t *keys = c->arena.get<uint64_t>(NA);
        uint32_t *vals = c->arena.get<uint32_t>(NA);
        const unsigned g = grid_for(NA, kBlock, 2048);
        const uint64_t pad = uint64_t(s.num_max >= s.num_min ? s.num_max - s.num_min : 0) + 1;
        k_dedup_keys<<<grid_for(NI, kBlock, 2048), kBlock, 0, st>>>(mbuild, s.issues, t.i_number, NI, s.num_min, pad,
                                                                    keys, vals);
        FZ_LAUNCH_CHECK();
        if (ext.n > 0) {
            k_dedup_ext_keys<<<grid_for(ext.n, kBlock, 2048), kBlock, 0, st>>>(ext, s.num_min, pad, NI, keys, vals);
            FZ_LAUNCH_CHECK();
        }
        radix_sort_pairs_swap(c, keys, vals, NA, bits_for(pad));
        k_dedup_pick<<<g, kBlock, 0, st>>>(vals, keys, mbuild, mbtime, NI, ext, NA, keep);
        FZ_LAUNCH_CHECK();
    }
    scan_exclusive_i64(c, keep, pos, NI, d_nm);

    // phase 2: iteration of each kept match; distinct (iteration, project) (:213-230)
    int64_t *it_arr = c->arena.get<int64_t>(NI);
    uint32_t *p_arr = c->arena.get<uint32_t>(NI);
    if (NI > 0) {
        const unsigned g = grid_for(NI, kBlock, 2048);
        k_matched_out<<<g, kBlock, 0, st>>>(s.issues, keep, pos, mbuild, s.fuzz, o->matched_issue, o->matched_build,
                                            it_arr, p_arr, f_match, s.iperm, s.bperm);
        k_distinct_iter<<<g, kBlock, 0, st>>>(it_arr, p_arr, d_nm, o->iter_detected);
        FZ_LAUNCH_CHECK();
    }
    if (P > 0) {  // the four project flag counts in one launch
        const uint8_t *fl[4] = {f_lim, f_fixlim, f_tgt, f_match};
        int64_t *outs[4] = {o->counts + FZ_RQ1_ISSUES_LIM_PROJECTS, o->counts + FZ_RQ1_FIXED_LIM_PROJECTS,
                            o->counts + FZ_RQ1_TARGET_PROJECTS, o->counts + FZ_RQ1_MATCHED_PROJECTS};
        count_flags_n(c, fl, outs, 4, P);
    }

    // finalize (:233-268)
    rq1_finish(c, threshold, o->iter_total, o->iter_detected, M, o->counts, o->late);
}

}  // namespace fz
