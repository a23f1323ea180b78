// Decoupled look-back shared by the single-pass kernels (scan, stream compaction, radix passes).
//
// A launch takes tiles in the order its workgroups start (a ticket counter), so every tile a
// workgroup waits for is already running.  Each tile publishes a status word
// {flag:2, epoch:14, value:48} - AGG (its own aggregate) first, INC (inclusive prefix) once known -
// with agent-scope atomics: the payload travels inside the flag word, so no separate fence /
// acquire is needed.  Every launch bumps a 14-bit epoch; a word from an earlier launch has another
// epoch and reads as "not published", so the status array is never cleared between launches (only
// when it grows, the epoch wraps, or a graph recording starts).  The ticket counter resets itself:
// the workgroup that draws the launch's last ticket sets it back to 0 (every other workgroup of the
// launch has drawn by then), so each launch starts from 0 with no host-side bookkeeping - which is
// also what makes a recorded (HIP graph) sequence of look-back launches replayable.
#pragma once

#include "fz_device.h"
#include "fz_internal.h"

namespace fz {

struct Lookback {
    uint64_t *status;      // [words] status words of this launch
    unsigned int *ticket;  // self-resetting tile counter (0 between launches)
    uint64_t epoch;        // epoch << 48
};

constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbFlags = 3ull << 62;
constexpr uint64_t kLbVal = (1ull << 48) - 1ull, kLbEpochMask = ((1ull << 14) - 1ull) << 48;

// Host: prepare `words` status words for one launch (call lookback_end(c, tiles) after it).
Lookback lookback_begin(fz_ctx *c, int64_t words);
inline void lookback_end(fz_ctx *, int64_t) {}
// The same for k <= 4 look-back passes run side by side in ONE launch: out[j] gets its own status
// words (words[j]) and its own ticket counter.
Lookback lookback_begin_n(fz_ctx *c, const int64_t *words, int k, Lookback *out);
// Reset the host epoch now and owe the device reset of the ticket and the status words: the
// context's next fill_batch zeroes them with its own regions, else the next lookback_begin launches
// the reset first (lookback_flush).
void lookback_reset(fz_ctx *c);
void lookback_flush(fz_ctx *c);

// Thread 0 of a workgroup: this workgroup's tile index (in start order); the last tile of the
// launch (ntiles workgroups) resets the counter for the next launch.
__device__ inline unsigned int lb_take_tile(unsigned int *ticket, unsigned int ntiles) {
    const unsigned int t = atomicAdd(ticket, 1u);
    if (t == ntiles - 1u) atomicExch(ticket, 0u);
    return t;
}

__device__ inline bool lb_ready(uint64_t w, uint64_t epoch) { return (w & kLbEpochMask) == epoch && (w & kLbFlags); }

// Wave-wide (all 64 lanes of ONE wave): publish `agg` for `tile` (status word `slot`, tiles are
// `stride` words apart), look back over the predecessors 64 at a time and return the exclusive
// prefix (the same value on every lane); publishes the inclusive prefix before returning.
__device__ inline int64_t lb_exclusive_prefix(const Lookback &lb, int64_t tile, int64_t agg) {
    const int lane = lane_id();
    if (lane == 0)
        __hip_atomic_store(&lb.status[tile], (tile == 0 ? kLbInc : kLbAgg) | lb.epoch | (uint64_t(agg) & kLbVal),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t prefix = 0;
    for (int64_t end = tile; end > 0;) {
        const int64_t p = end - kWave + lane;  // lane 63 = nearest predecessor
        const uint64_t w = p >= 0 ? __hip_atomic_load(&lb.status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : (kLbInc | lb.epoch);  // before tile 0: an inclusive prefix of 0
        const bool ready = lb_ready(w, lb.epoch);
        const uint64_t inc = __ballot(ready && (w & kLbFlags) == kLbInc);
        const uint64_t wait = __ballot(!ready);
        const int hi = inc ? 63 - __clzll((long long)inc) : -1;  // nearest inclusive lane
        const uint64_t need = hi >= 0 ? (hi == 63 ? 0ull : ~0ull << (hi + 1)) : ~0ull;
        if (wait & need) {  // a tile between the inclusive prefix and this one has not published
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        prefix += wave_sum<int64_t>(lane >= (hi < 0 ? 0 : hi) && p >= 0 ? int64_t(w & kLbVal) : 0);
        if (hi >= 0) break;
        end -= kWave;
    }
    if (lane == 0 && tile > 0)
        __hip_atomic_store(&lb.status[tile], kLbInc | lb.epoch | (uint64_t(prefix + agg) & kLbVal), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

}  // namespace fz
