// Sorted views and stream compaction (templated on the row predicate, so the RQ translation
// units instantiate their own filters).
//
// A view is the replacement for one "WHERE project = X AND <filter> ORDER BY time" query issued
// per project by the reference (e.g. queries1.py:267-278, rq4a_bug.py:124-137): all projects at
// once, rows in (project, time) order, with per-project [offs[p], offs[p+1]) segments.
#pragma once

#include "fz_device.h"
#include "fz_internal.h"

namespace fz {

// A view whose buffers live in the arena (valid for one public call).
struct TmpView {
    int64_t cap = 0;          // upper bound of n (host-known)
    int64_t *d_n = nullptr;   // device count
    int32_t *row = nullptr;   // original row ids
    int64_t *time = nullptr;  // sort time
    uint32_t *proj = nullptr;
    int64_t *offs = nullptr;  // [P + 1]
};

template <typename Pred>
__global__ __launch_bounds__(kBlock) void k_flag_rows(const int32_t *__restrict__ rows, int64_t n,
                                                      const int64_t *__restrict__ d_live, Pred pred,
                                                      int64_t *__restrict__ flags) {
    const int64_t live = d_live ? *d_live : n;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        flags[i] = (i < live && pred(rows[i])) ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void k_compact_view(const int32_t *__restrict__ rows,
                                                         const int64_t *__restrict__ times,
                                                         const uint32_t *__restrict__ proj, int64_t n,
                                                         const int64_t *__restrict__ flags,
                                                         const int64_t *__restrict__ pos, int32_t *__restrict__ orow,
                                                         int64_t *__restrict__ otime, uint32_t *__restrict__ oproj);

// Offsets of a project-sorted array whose length is only known on the device.
__global__ __launch_bounds__(kBlock) void k_segment_offsets_dn(const uint32_t *__restrict__ proj,
                                                               const int64_t *__restrict__ d_n, int64_t P,
                                                               int64_t *__restrict__ offsets);

// Rows of src (n rows, in view order; only the first *src_live when given) satisfying pred(row)
// -> dst (same order).
template <typename Pred>
void filter_view(fz_ctx *c, const int32_t *rows, const int64_t *times, const uint32_t *proj, int64_t n, int64_t P,
                 Pred pred, TmpView &dst, const int64_t *src_live = nullptr) {
    dst.cap = n;
    dst.d_n = c->arena.get<int64_t>(1);
    dst.row = c->arena.get<int32_t>(n);
    dst.time = c->arena.get<int64_t>(n);
    dst.proj = c->arena.get<uint32_t>(n);
    dst.offs = c->arena.get<int64_t>(P + 1);
    int64_t *flags = c->arena.get<int64_t>(n);
    int64_t *pos = c->arena.get<int64_t>(n);
    if (n > 0) {
        k_flag_rows<<<grid_for(n, kBlock, 4096), kBlock, 0, c->stream>>>(rows, n, src_live, pred, flags);
        FZ_LAUNCH_CHECK();
    }
    scan_exclusive_i64(c, flags, pos, n, dst.d_n);
    if (n > 0) {
        k_compact_view<<<grid_for(n, kBlock, 4096), kBlock, 0, c->stream>>>(rows, times, proj, n, flags, pos,
                                                                           dst.row, dst.time, dst.proj);
        FZ_LAUNCH_CHECK();
    }
    k_segment_offsets_dn<<<grid_for(P + 1, kBlock, 1u << 30), kBlock, 0, c->stream>>>(dst.proj, dst.d_n, P, dst.offs);
    FZ_LAUNCH_CHECK();
}

// lower_bound of v in a[lo, hi)
__device__ inline int64_t lower_bound_i64(const int64_t *a, int64_t lo, int64_t hi, int64_t v) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ inline int64_t upper_bound_i64(const int64_t *a, int64_t lo, int64_t hi, int64_t v) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ inline void atomic_add_i64(int64_t *p, int64_t v) {
    atomicAdd(reinterpret_cast<unsigned long long *>(p), static_cast<unsigned long long>(v));
}

// Count nonzero bytes of flags[0..P) into *out (adds).
void count_flags(fz_ctx *c, const uint8_t *flags, int64_t P, int64_t *out);
// describe of x[0..*d_n) with nmax a host upper bound (fz_prims.hip).
void describe_f64_dn(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n, fz_describe *dev_out);
// ascending order-preserving keys (f64_key) of x[0..*d_n); entries past *d_n are ~0.
uint64_t *sorted_keys_dn(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n);
// the same for nmax <= 4096 in one workgroup (LDS bitonic network, fz_series.hip)
uint64_t *sort_small_keys(fz_ctx *c, const double *x, int64_t nmax, const int64_t *d_n);
void describe_sorted_dn(fz_ctx *c, const uint64_t *sorted_keys, const double *x, int64_t nmax, const int64_t *d_n,
                        fz_describe *dev_out);

}  // namespace fz
