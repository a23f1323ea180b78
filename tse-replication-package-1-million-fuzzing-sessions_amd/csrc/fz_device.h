// Device-side building blocks shared by the kernels (wave64 scans/reductions, digit matching,
// double-double accumulation, numpy-compatible percentile interpolation).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace fz {

__device__ inline int lane_id() { return threadIdx.x & 63; }
__device__ inline int wave_id() { return threadIdx.x >> 6; }
__device__ inline uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

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
template <typename T>
__device__ inline T block_excl_scan(T x, T *s_tmp, T *total) {
    T inc = wave_incl_scan(x);
    const int w = wave_id();
    if (lane_id() == 63) s_tmp[w] = inc;
    __syncthreads();
    T woff = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
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
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
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
