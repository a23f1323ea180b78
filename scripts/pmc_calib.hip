// Calibration of the gfx950 PMC byte counters (FETCH_SIZE / WRITE_SIZE) for the access widths the
// engine's kernels use.  MI355X_MICROARCH.md's HBM section calibrates only 16-B-per-lane streaming
// reads (FETCH_SIZE = 1/2 of the bytes) and 16-B streaming stores (exact) and says other widths are
// uncalibrated; the store's time sort, gather and filters read 1-, 4- and 8-byte columns.  Each
// kernel below moves a known byte count (1 GiB: past the 256 MiB Infinity Cache) at one width;
// scripts/pmc_calib.py divides the counter by it.
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/build/pmc_calib scripts/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- scripts/build/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

template <int W> struct Vec;
template <> struct Vec<1> { using T = uint8_t; };
template <> struct Vec<2> { using T = uint16_t; };
template <> struct Vec<4> { using T = uint32_t; };
template <> struct Vec<8> { using T = uint64_t; };
template <> struct Vec<16> { using T = uint4; };

__device__ inline uint32_t fold(uint8_t v) { return v; }
__device__ inline uint32_t fold(uint16_t v) { return v; }
__device__ inline uint32_t fold(uint32_t v) { return v; }
__device__ inline uint32_t fold(uint64_t v) { return uint32_t(v) ^ uint32_t(v >> 32); }
__device__ inline uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// coalesced streaming read, W bytes per lane, grid-stride; the sink is written only when the fold
// equals a run-time value the buffer never produces (no write traffic; a compile-time constant let
// the compiler drop the 1- and 2-byte loops: their fold cannot reach it)
template <int W>
__global__ __launch_bounds__(256) void k_read_w(const typename Vec<W>::T *__restrict__ src, int64_t n, uint32_t *sink, uint32_t magic) {
    uint32_t acc = 0;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) acc += fold(src[i]);
    if (acc == magic) sink[0] = acc;
}

template <int W>
__global__ __launch_bounds__(256) void k_write_w(typename Vec<W>::T *__restrict__ dst, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        typename Vec<W>::T v{};
        dst[i] = v;
    }
}

// the Infinity-Cache eviction between measured kernels (its own name: not booked to k_write_w<16>)
__global__ __launch_bounds__(256) void k_flush(uint4 *__restrict__ dst, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) dst[i] = uint4{};
}

// segmented 8-byte read like the time sort's: one workgroup per segment of L rows starting at an
// arbitrary (8-byte aligned, not line aligned) offset, rows tid + m * 1024
__global__ __launch_bounds__(1024) void k_read_seg8(const uint64_t *__restrict__ src, int64_t L, int64_t nseg, uint32_t *sink) {
    uint32_t acc = 0;
    for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x)
        for (int64_t i = threadIdx.x; i < L; i += 1024) acc ^= fold(src[s * L + i]);
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// segmented 1-byte write (a byte column written segment by segment)
__global__ __launch_bounds__(1024) void k_write_seg1(uint8_t *__restrict__ dst, int64_t L, int64_t nseg) {
    for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x)
        for (int64_t i = threadIdx.x; i < L; i += 1024) dst[s * L + i] = 0;
}

// random 8-byte gather (a permutation's reads)
__global__ __launch_bounds__(256) void k_gather8(const uint64_t *__restrict__ src, int64_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const uint64_t j = (uint64_t(i) * 0x9E3779B97F4A7C15ull) % uint64_t(n);
        acc ^= fold(src[j]);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                 \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

int main() {
    const int64_t bytes = int64_t(1) << 30;
    void *a = nullptr, *b = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 1, bytes));
    CK(hipDeviceSynchronize());
    const unsigned grid = 8192;
    // between kernels, a 1 GiB write of the other buffer evicts the first from the Infinity Cache
    auto flush = [&] {
        k_flush<<<grid, 256>>>(static_cast<uint4 *>(b), bytes / 16);
        CK(hipDeviceSynchronize());
    };
#define READ(W)                                                                                     \
    flush();                                                                                        \
    k_read_w<W><<<grid, 256>>>(static_cast<const Vec<W>::T *>(a), bytes / W, sink, 0xffffffffu);                 \
    CK(hipDeviceSynchronize());                                                                     \
    printf("k_read_w<%d> %lld\n", W, (long long)bytes);
#define WRITE(W)                                                                                    \
    flush();                                                                                        \
    k_write_w<W><<<grid, 256>>>(static_cast<Vec<W>::T *>(a), bytes / W);                            \
    CK(hipDeviceSynchronize());                                                                     \
    printf("k_write_w<%d> %lld\n", W, (long long)bytes);
    READ(1) READ(2) READ(4) READ(8) READ(16)
    WRITE(1) WRITE(2) WRITE(4) WRITE(8) WRITE(16)
    const int64_t L = 10003, nseg = (bytes / 8) / L;
    flush();
    k_read_seg8<<<2048, 1024>>>(static_cast<const uint64_t *>(a), L, nseg, sink);
    CK(hipDeviceSynchronize());
    printf("k_read_seg8 %lld\n", (long long)(nseg * L * 8));
    const int64_t L1 = 10003, nseg1 = bytes / L1;
    flush();
    k_write_seg1<<<2048, 1024>>>(static_cast<uint8_t *>(a), L1, nseg1);
    CK(hipDeviceSynchronize());
    printf("k_write_seg1 %lld\n", (long long)(nseg1 * L1));
    flush();
    k_gather8<<<grid, 256>>>(static_cast<const uint64_t *>(a), bytes / 8, sink);
    CK(hipDeviceSynchronize());
    printf("k_gather8 %lld\n", (long long)bytes);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
