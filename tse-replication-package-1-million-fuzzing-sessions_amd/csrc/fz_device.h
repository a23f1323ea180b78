// Device-side building blocks shared by the kernels (wave64 scans/reductions, digit matching,
// double-double accumulation, numpy-compatible percentile interpolation).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace fz {

__device__ inline int lane_id() { return threadIdx.x & 63; }
__device__ inline int wave_id() { return threadIdx.x >> 6; }
__device__ inline uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Bitonic networks in LDS map pair q to the elements i = ((q & ~(j-1)) << 1) | (q & (j-1)) and
// i + j, with pairs q = tid + m * blockDim (blockDim a multiple of 64).  A stage with j <= 64 only
// touches the 128 elements of one wave's 64 consecutive pairs, so between two such stages the
// wave's own (in-order) LDS traffic is the only dependency: wait for it, skip the workgroup
// barrier (63 of the 78 stages of a 4096-entry network).  Call after stage (k, j) of a network of
// np2 entries; the last stage always ends with the barrier.
__device__ inline void bitonic_stage_sync(int k, int j, int np2) {
    const int nj = j > 1 ? (j >> 1) : k;  // the next stage's distance (stage k << 1 starts at k)
    if (j <= 64 && nj <= 64 && !(j == 1 && k == np2))
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else
        __syncthreads();
}

// A write-through (sc1) 8-byte store: another workgroup may read it after a ticket / flag hand-off
// (the storing wave drains its stores before the ticket add, the reader acquires after it).
__device__ inline void store_wt(double *p, double x) {
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __builtin_bit_cast(unsigned long long, x),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave priority of the one-workgroup kernels that finish an analysis chain (describes, the
// small-series tests, the finishing tables): their waves share CUs with the other streams' bulk
// kernels; FZ_CHAIN_PRIO=1 raises their issue priority (s_setprio 3).
#ifndef FZ_CHAIN_PRIO
#define FZ_CHAIN_PRIO 0
#endif
__device__ inline void chain_prio() {
    if constexpr (FZ_CHAIN_PRIO != 0) __builtin_amdgcn_s_setprio(3);
}

// offs[q] = v for q in [a, e] of every lane's range (a > e: none), each range stored by the whole
// wave 64 entries a round (all 64 lanes must call it): a lane whose range spans thousands of ids -
// the ids before a shard's first project, the gap between a table's two prefix types - no longer
// stores them one by one on its own
__device__ inline void wave_fill_ranges(int64_t *offs, int64_t a, int64_t e, int64_t v) {
    uint64_t m = __ballot(a <= e);
    while (m) {
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int64_t A = __shfl(a, l, 64), E = __shfl(e, l, 64), V = __shfl(v, l, 64);
        for (int64_t q = A + lane_id(); q <= E; q += 64) offs[q] = V;
    }
}

template <typename T>
__device__ inline T wave_incl_scan(T x) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        T y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

template <typename T>
__device__ inline T wave_sum(T x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

template <typename T>
__device__ inline T wave_max(T x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T y = __shfl_xor(x, off, 64);
        x = y > x ? y : x;
    }
    return x;
}

template <typename T>
__device__ inline T wave_min(T x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T y = __shfl_xor(x, off, 64);
        x = y < x ? y : x;
    }
    return x;
}

// Exclusive scan over a 256-thread block; s_tmp must hold 4 T.  *total receives the block sum.
template <typename T, int NW = 4>  // NW waves per workgroup
__device__ inline T block_excl_scan(T x, T *s_tmp, T *total) {
    T inc = wave_incl_scan(x);
    const int w = wave_id();
    if (lane_id() == 63) s_tmp[w] = inc;
    __syncthreads();
    T woff = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {  // s_tmp holds one slot per wave
        T v = s_tmp[i];
        if (i < w) woff += v;
        tot += v;
    }
    __syncthreads();
    if (total) *total = tot;
    return woff + inc - x;
}

template <typename T>
__device__ inline T block_sum(T x, T *s_tmp) {
    x = wave_sum(x);
    if (lane_id() == 0) s_tmp[wave_id()] = x;
    __syncthreads();
    T tot = s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
    __syncthreads();
    return tot;
}

// Lanes of this wave whose `bits`-bit digit equals mine (all 64 lanes must execute this).
template <int BITS>
__device__ inline uint64_t match_digit(uint32_t d, bool valid) {
    // per bit: one compare for the ballot, then the lane keeps the ballot (bit set) or its
    // complement (bit clear) by xor with (bit - 1) - 32-bit halves, no 64-bit selects
    const uint64_t v = __ballot(valid);
    uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const uint32_t bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit != 0u);
        const uint32_t flip = bit - 1u;  // 0 when set, all ones when clear
        lo &= uint32_t(bal) ^ flip;
        hi &= uint32_t(bal >> 32) ^ flip;
    }
    return (uint64_t(hi) << 32) | lo;
}

// ---- double-double (error-free) accumulation -----------------------------------------------
struct DD {
    double hi, lo;
};
__host__ __device__ inline DD two_sum(double a, double b) {
    double s = a + b;
    double bb = s - a;
    double e = (a - (s - bb)) + (b - bb);
    return {s, e};
}
__host__ __device__ inline DD dd_add(DD a, DD b) {
    DD s = two_sum(a.hi, b.hi);
    double lo = s.lo + a.lo + b.lo;
    return two_sum(s.hi, lo);
}
__host__ __device__ inline DD dd_add_d(DD a, double b) {
    DD s = two_sum(a.hi, b);
    return two_sum(s.hi, s.lo + a.lo);
}
__device__ inline DD wave_dd_sum(DD x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        DD y{__shfl_xor(x.hi, off, 64), __shfl_xor(x.lo, off, 64)};
        x = dd_add(x, y);
    }
    return x;
}

// numpy.lib._function_base_impl._lerp (numpy 2.2): a + (b-a)*t, or b - (b-a)*(1-t) when t >= 0.5
__host__ __device__ inline double np_lerp(double a, double b, double t) {
    double diff = b - a;
    if (t >= 0.5) return b - diff * (1.0 - t);
    return a + diff * t;
}

// numpy.percentile(sorted x, q, method='linear') on an ascending array of n >= 1 values:
// virtual index (n-1)*q/100 (numpy: `(n - 1) * quantiles`, quantiles = q/100 as float64).
template <typename Get>
__host__ __device__ inline double np_percentile_sorted(Get get, int64_t n, double q) {
    double quant = q / 100.0;
    double vi = double(n - 1) * quant;
    double fl = floor(vi);
    int64_t prev = int64_t(fl);
    int64_t next = prev + 1;
    if (prev > n - 1) prev = n - 1;
    if (prev < 0) prev = 0;
    if (next > n - 1) next = n - 1;
    if (next < 0) next = 0;
    double gamma = vi - fl;
    return np_lerp(get(prev), get(next), gamma);
}

}  // namespace fz
