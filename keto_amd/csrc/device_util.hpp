// device_util.hpp — wave-level building blocks shared by the traversal kernels
// (device_engine.hip, partition.hip).  64-lane wavefronts (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kdev {

constexpr int kCntShift = 36;  // packed append counter: count << 36 | row-length prefix
constexpr uint64_t kPreMask = (1ull << kCntShift) - 1;
// Frontier lists appended through the packed counter must hold fewer than 2^28 entries:
// the count field is 28 bits, and a list capacity at or above that lets the count wrap
// before any append sees idx >= cap (an overflow nobody flags).  With capacity below it,
// the first append past the end raises the overflow flag and the round is retried.
constexpr uint64_t kMaxListEntries = (1ull << (64 - kCntShift)) - (1ull << 20);

// 64-lane inclusive scan of a uint64 value
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// 64-lane inclusive scans of a u32 / i32 held one per lane, without LDS: DPP row shifts
// (1, 2, 4, 8) scan each 16-lane row, then the three lower row totals are read with
// v_readlane and added.  Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
    const int row = (int)(__lane_id() >> 4);
    return x + (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
}

// inclusive prefix maximum over lanes (values >= -1; -1 = none)
__device__ __forceinline__ int wave_incl_max_i32(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xf, 0xf, false));
    const int r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31);
    const int r2 = __builtin_amdgcn_readlane(x, 47);
    const int row = (int)(__lane_id() >> 4);
    const int c = row == 0 ? -1 : row == 1 ? r0 : row == 2 ? max(r0, r1) : max(max(r0, r1), r2);
    return max(x, c);
}

// Append (key, row length) to a frontier list with one atomic per wave.  Every lane of
// the wave must call this (inactive lanes pass want = false).
__device__ __forceinline__ void wave_append(bool want, uint64_t key, uint64_t deg, int lane, unsigned long long *ctr,
                                            uint64_t base, uint64_t cap, uint64_t *out_key, uint64_t *out_pre,
                                            uint64_t *out_mask, uint64_t mask, unsigned int *overflow) {
    uint64_t val = want ? ((1ull << kCntShift) | deg) : 0ull;
    uint64_t incl = wave_incl_scan(val, lane);
    uint64_t total = __shfl(incl, 63, 64);
    if (!total) return;
    unsigned long long start = 0;
    if (lane == 63) {
        start = atomicAdd(ctr, (unsigned long long)total);
        // a row-length prefix that carries into the count field corrupts both: flag it
        if ((start & kPreMask) + (total & kPreMask) > kPreMask) atomicOr(overflow, 1u);
    }
    start = __shfl(start, 63, 64);
    if (want) {
        uint64_t pos = start + incl - val;
        uint64_t idx = base + (pos >> kCntShift);
        if (idx < cap) {
            out_key[idx] = key;
            out_pre[idx] = pos & kPreMask;
            if (out_mask) out_mask[idx] = mask;
        } else {
            atomicOr(overflow, 1u);
        }
    }
}

// Append key to a list with one atomic per wave (all lanes call)
__device__ __forceinline__ void wave_touch(bool want, uint64_t key, int lane, unsigned long long *ctr,
                                           uint64_t *touch, uint64_t cap, unsigned int *overflow) {
    uint64_t bal = __ballot(want);
    if (!bal) return;
    int leader = __ffsll((unsigned long long)bal) - 1;
    unsigned long long start = 0;
    if (lane == leader) start = atomicAdd(ctr, (unsigned long long)__popcll(bal));
    start = __shfl(start, leader, 64);
    if (want) {
        uint64_t idx = start + __popcll(bal & ((1ull << lane) - 1));
        if (idx < cap)
            touch[idx] = key;
        else
            atomicOr(overflow, 1u);
    }
}

// first index in a[0, n) with a[i] > key, computed by one full wave (64-ary search)
__device__ __forceinline__ uint64_t wave_upper_bound(const uint64_t *a, uint64_t n, uint64_t key, int lane) {
    uint64_t lo = 0, hi = n;
    while (hi - lo > 64) {
        uint64_t step = (hi - lo + 63) / 64;
        uint64_t idx = lo + (uint64_t)lane * step;
        bool le = idx < hi && a[idx] <= key;
        int cnt = __popcll(__ballot(le));
        if (cnt == 0) return lo;  // a[lo] > key
        uint64_t nlo = lo + (uint64_t)(cnt - 1) * step + 1;
        uint64_t nhi = lo + (uint64_t)cnt * step;
        lo = nlo;
        hi = nhi < hi ? nhi : hi;
    }
    uint64_t idx = lo + lane;
    bool le = idx < hi && a[idx] <= key;
    return lo + __popcll(__ballot(le));
}

}  // namespace kdev
